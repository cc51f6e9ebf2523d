# full GPU suite on the round-3 library + batch PMC (SQ passes, FETCH/WRITE) of the new default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
Q=1024 EXTRA='--prewarm-s 0' OUT=$O/pmc_sq timeout -k 10 400 bash tools/pmc_batch.sh > /dev/null 2>&1 || { echo "pmc_batch failed"; exit 1; }
cat $O/pmc_sq/summary.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 bench.py --no-cpu-baseline --workload batch --queries 1024 --steps 1 --warmup 0 --prewarm-s 0 > $O/pmc_$c.log 2>&1 || { echo "pmc $c rc=$?"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > $O/batch_stats.log 2>&1 || { echo "stats rc=$?"; tail -5 $O/batch_stats.log; exit 1; }
grep '^{' $O/batch_stats.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch', round(d['ms_per_step'],1), round(d['roofline']['frac'],4), d['check']['ok'])"
