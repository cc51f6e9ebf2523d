# read-ahead v3 (kernel stores rows into pinned memory, parallel CPU copy): attach tests, per-call walks;
# D2H by destination page size (ubench); batched kernel A/B with nontemporal query-tile loads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for kind in masks shares; do
  n=2000000; [ $kind = shares ] && n=200000
  for ra in 1 0; do
    IRIS_READAHEAD=$ra timeout -k 10 120 python tools/ra_diag.py $kind $n 3 > $O/diag_${kind}_$ra.log 2>&1 || { echo "diag rc=$?"; tail -3 $O/diag_${kind}_$ra.log; exit 1; }
    echo "$kind ra=$ra"; cat $O/diag_${kind}_$ra.log
  done
done
timeout -k 10 180 ./tools/ubench_launch > $O/launch.log 2>&1 || { echo "ubench rc=$?"; tail -5 $O/launch.log; exit 1; }
grep -E "d2h|kpin|reg" $O/launch.log
timeout -k 10 600 ./tools/gpu_r03x.sh
