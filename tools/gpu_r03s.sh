# read-ahead diagnosis: per-call time of attached host-slice calls, read-ahead off / on / variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03s; mkdir -p $O
for kind in masks shares; do
  n=2000000; [ $kind = shares ] && n=200000
  for v in "IRIS_READAHEAD=0" "IRIS_READAHEAD=1" "IRIS_RA_DIAG=1" "IRIS_RA_DIAG=2"; do
    echo "== $kind $v"
    env $v timeout -k 10 120 python tools/ra_diag.py $kind $n 3 > $O/${kind}_$v.log 2>&1 || { echo "rc=$?"; tail -3 $O/${kind}_$v.log; exit 1; }
    cat $O/${kind}_$v.log
  done
done
