# round 4: configs[2] energy per MFMA on ONE box -- package power while the 1024-query batch runs and while
# tools/ubench_mfma_power runs its modes (0 the MFMA alone; 1 the batched kernel's MFMA sequence fed from LDS;
# 2 the same with the template operands expanded by VALU; 3 the template operands held constant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04g_power; rm -rf $O; mkdir -p $O
timeout 30 amd-smi metric -g 0 -p -c > $O/idle.txt 2>&1 || { echo "amd-smi failed"; tail -5 $O/idle.txt; exit 1; }
poll() {  # poll package power + clocks while PID runs
    local pid=$1 f=$2
    while kill -0 $pid 2>/dev/null; do
        echo "T $(date +%s.%N)" >> $f
        timeout 5 amd-smi metric -g 0 -p -c >> $f 2>&1
        sleep 0.2
    done
}
if [ -z "$NO_BATCH" ]; then
  timeout -k 10 300 python bench.py --workload batch --queries 1024 --steps 4 --warmup 1 --prewarm-s 0.5 --no-cpu-baseline > $O/batch.log 2>&1 &
  pid=$!; poll $pid $O/batch.pwr; wait $pid || { echo "batch rc=$?"; tail -3 $O/batch.log; exit 1; }
  grep '^{' $O/batch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch kernel_ms', round(d['kernel']['avg_ms'],2), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
fi
for m in ${MODES:-0 1 2 3}; do
  timeout -k 10 60 tools/ubench_mfma_power 10 $m > $O/mode$m.txt 2>&1 &
  pid=$!; poll $pid $O/mode$m.pwr; wait $pid || { echo "ubench mode $m rc=$?"; cat $O/mode$m.txt; exit 1; }
  cat $O/mode$m.txt
done
echo all ok
