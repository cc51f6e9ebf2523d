# fused last-workgroup search reduce: parity + participant-sized latency
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_group.py tests/test_gpu_trits.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/chunk_latency.py 20000 3000 > $O/lat.log 2>&1 || { echo "lat rc=$?"; tail -5 $O/lat.log; exit 1; }
grep -v '^{' $O/lat.log
timeout -k 10 200 python tools/chunk_latency.py 10000 3000 > $O/lat10k.log 2>&1 || { echo "lat rc=$?"; tail -5 $O/lat10k.log; exit 1; }
grep -v '^{' $O/lat10k.log
