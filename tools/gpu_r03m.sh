# restored tree + small-range kernels (deep-ring K-split search, K-split masks): GPU suite,
# smoke, default bench line, launch-latency micro-benchmark, participant-sized calls
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 60 ./tools/ubench_launch > $O/launch.log 2>&1 || { echo "ubench rc=$?"; tail -5 $O/launch.log; exit 1; }
cat $O/launch.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 ./tools/call_overhead > $O/overhead.log 2>&1 || { echo "overhead rc=$?"; tail -5 $O/overhead.log; exit 1; }
cat $O/overhead.log
for w in search masks; do
  timeout -k 10 200 python bench.py --workload $w --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline --reuse-engine > $O/chunk_$w.log 2>&1 || { echo "chunk $w rc=$?"; tail -3 $O/chunk_$w.log; exit 1; }
  grep '^{' $O/chunk_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunk20k $w', 'step_us', round(d['ms_per_step']*1e3,2), 'kernel_us', round(d['kernel']['avg_ms']*1e3,2), 'ok', d['check'])"
done
timeout -k 10 300 python bench.py > $O/bench.log 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.log
