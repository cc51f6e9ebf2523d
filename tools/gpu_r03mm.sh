#!/bin/bash
# read-ahead copy-out: helper threads 0/1/3/5/7 (IRIS_COPY_HELPERS), masks and shares chunk walks
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03mm; mkdir -p $O
for kind in masks shares; do
  n=2000000; [ $kind = shares ] && n=200000
  for h in 3 0 1 5 7 3; do
    IRIS_COPY_HELPERS=$h timeout -k 10 120 python tools/ra_diag.py $kind $n 3 > $O/diag_${kind}_$h.log 2>&1 || { echo "diag rc=$?"; tail -3 $O/diag_${kind}_$h.log; exit 1; }
    echo "$kind helpers=$h"; grep -v 4-KB $O/diag_${kind}_$h.log
  done
done
