#!/bin/bash
# DistanceEngine on participant-sized chunks: load-ring depth of shares_split_kernel (IRIS_SHARES_SPLIT_STAGES 3 shipped, 4, 5, 6 first;
# then IRIS_SHARES_SPLIT_ROT=1 with 3 and 6 stages): parity of each variant, then interleaved 20k-share call / kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ss; rm -rf $O; mkdir -p $O
for lib in shrot shrot6; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_attach.py -m gpu -x -q -k "share or distance or u16" --timeout 120 --timeout-method thread > $O/${lib}_tests.log 2>&1 || { echo "$lib tests rc=$?"; tail -20 $O/${lib}_tests.log; exit 1; }
  echo "$lib $(tail -1 $O/${lib}_tests.log)"
done
for r in 1 2; do
for lib in hip shrot shrot6; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -k 10 200 python tools/chunk_latency.py 20000 1000 > $O/lat_${lib}_$r.log 2>&1 || { echo "lat $lib rc=$?"; tail -5 $O/lat_${lib}_$r.log; exit 1; }
  echo "$lib r$r $(grep '^shares-dev' $O/lat_${lib}_$r.log)"
done
done
