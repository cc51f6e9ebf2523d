set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 ./tools/call_overhead > $O/overhead.log 2>&1 || { echo "overhead rc=$?"; tail -5 $O/overhead.log; exit 1; }
cat $O/overhead.log
