# round 4: device-output rows visible to an unordered reader as soon as the call returns -- the shipped
# library (rows written through L2) and a build that stores them like the other kernels (IRIS_ROWS_WT=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py -v --timeout 120 --timeout-method thread -k "unordered_reader or completion_word" > $O/ship.log 2>&1 || { echo "ship rc=$?"; tail -30 $O/ship.log; exit 1; }
tail -2 $O/ship.log
IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_nowt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py -v --timeout 120 --timeout-method thread -k "unordered_reader" > $O/nowt.log 2>&1
echo "nowt rc=$?"; grep -E "PASSED|FAILED|assert" $O/nowt.log | head -10
