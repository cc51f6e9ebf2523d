# Round-2 GPU pass: the whole -m gpu suite, smoke, the default bench line and its rocprof summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/gpu_tests.log | tail -20; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_n1.log 2>&1 || { echo bench failed; tail $O/bench_n1.log; exit 1; }
grep '^{' $O/bench_n1.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo prof failed; exit 1; }
echo done
