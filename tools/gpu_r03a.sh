set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03a/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r03a/tests.log; exit 1; }
tail -3 gpurun_out/r03a/tests.log
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/r03a/bench.log; exit 1; }
grep '^{' gpurun_out/r03a/bench.log
