# round 4: the whole GPU suite and smoke on the current tree, the default bench line with its rocprofv3 kernel
# stats, the reference's 20 000-record calls (engine reused), and PMC traffic of every HBM-bound kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/default.log 2>&1 || { echo "default bench rc=$?"; tail -5 $O/default.log; exit 1; }
grep '^{' $O/default.log > $O/default.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 120 tools/call_overhead > $O/call_overhead.txt 2>&1 || { echo "call_overhead rc=$?"; exit 1; }
cat $O/call_overhead.txt
for w in search masks shares; do
  timeout -k 10 200 python bench.py --workload $w --n-per-gpu 20000 --steps 400 --warmup 20 --no-cpu-baseline --reuse-engine > $O/chunk20k_${w}_reuse.log 2>&1 || { echo "chunk $w rc=$?"; exit 1; }
  grep '^{' $O/chunk20k_${w}_reuse.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel']['avg_ms']; print('chunk20k_$w', 'step_us', round(d['ms_per_step']*1e3,1), 'unprofiled_us', round(d['ms_per_step_unprofiled']*1e3,1), 'kernel_us', round(k*1e3,1), 'ratio', round(d['ms_per_step_unprofiled']/k,3), d['check']['ok'])"
done
WORKLOADS="search masks shares resolver resolve-masks" NO_LANES=1 timeout -k 10 700 bash tools/pmc_traffic.sh > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
echo all ok
