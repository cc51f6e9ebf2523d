# round 4: configs[2] evidence on ONE box -- package power while the 1024-query batch runs and
# while the fp4 MFMA runs alone (energy per MFMA), rocprofv3 kernel stats, and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ) of the same launch shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04e; rm -rf $O; mkdir -p $O
timeout 30 amd-smi metric -g 0 -p -c > $O/idle.txt 2>&1 || { echo "amd-smi failed"; tail -5 $O/idle.txt; exit 1; }
poll() {  # poll package power + clocks while PID runs
    local pid=$1 f=$2
    while kill -0 $pid 2>/dev/null; do
        echo "T $(date +%s.%N)" >> $f
        timeout 5 amd-smi metric -g 0 -p -c >> $f 2>&1
        sleep 0.2
    done
}
timeout -k 10 300 python bench.py --workload batch --queries 1024 --steps 4 --warmup 1 --prewarm-s 0.5 --no-cpu-baseline > $O/batch.log 2>&1 &
pid=$!; poll $pid $O/batch.pwr; wait $pid || { echo "batch rc=$?"; tail -3 $O/batch.log; exit 1; }
grep '^{' $O/batch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch kernel_ms', round(d['kernel']['avg_ms'],2), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
timeout -k 10 60 tools/ubench_mfma_power 12 > $O/mfma_alone.txt 2>&1 &
pid=$!; poll $pid $O/mfma_alone.pwr; wait $pid || { echo "ubench rc=$?"; cat $O/mfma_alone.txt; exit 1; }
cat $O/mfma_alone.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --workload batch --queries 1024 --steps 3 --warmup 1 --prewarm-s 0 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -3 $O/prof.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 bench.py --no-cpu-baseline --workload batch --queries 1024 --steps 1 --warmup 0 --prewarm-s 0 > $O/pmc_$c.log 2>&1 || { echo "pmc $c rc=$?"; tail -3 $O/pmc_$c.log; exit 1; }
done
OUT=$O/sq Q=1024 EXTRA='--prewarm-s 0' timeout -k 10 500 bash tools/pmc_batch.sh > $O/sq.log 2>&1 || { echo "sq rc=$?"; tail -5 $O/sq.log; exit 1; }
echo all ok
