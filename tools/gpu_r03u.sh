# same-box: read-ahead on/off in tools/ra_diag.py and in the bench's host-masks line; D2H micro-benchmark;
# small-range shares kernel A/B (LDS K-split T=2 shipped, T=1, round-2 workspace form)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 120 ./tools/ubench_launch > $O/launch.log 2>&1 || { echo "ubench rc=$?"; tail -5 $O/launch.log; exit 1; }
grep -E "d2h|kern\+d2h|xwait" $O/launch.log
for ra in 0 1; do
  IRIS_READAHEAD=$ra timeout -k 10 120 python tools/ra_diag.py masks 2000000 3 > $O/diag_masks_$ra.log 2>&1 || { echo "diag rc=$?"; tail -3 $O/diag_masks_$ra.log; exit 1; }
  echo "ra=$ra"; cat $O/diag_masks_$ra.log
  IRIS_READAHEAD=$ra timeout -k 10 300 python bench.py --workload host-masks --attached --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_masks_$ra.log 2>&1 || { echo "bench rc=$?"; tail -3 $O/bench_masks_$ra.log; exit 1; }
  grep '^{' $O/bench_masks_$ra.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench host-masks ra=$ra ms/step', round(d['ms_per_step'],3), d['resident_same_chunks'])"
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_attach.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for lib in hip sharesT1 sharesold; do
  IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$lib.so timeout -k 10 120 python tools/chunk_latency.py 20000 1000 > $O/lat_${lib}_$r.log 2>&1 || { echo "lat $lib rc=$?"; tail -3 $O/lat_${lib}_$r.log; exit 1; }
  echo "$lib r=$r"; grep -E "^shares-dev " $O/lat_${lib}_$r.log | cut -c1-150
done
done
