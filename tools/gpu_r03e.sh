# batch kernel: 2 queries x 2 tiles per wave (IRIS_BATCH_KERNEL=3) vs the shipped 4 x 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -k "batch_1024_queries or many_groups" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 2 3 2 3; do
  IRIS_BATCH_KERNEL=$k timeout -k 10 300 python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > $O/batch_k$k.log 2>&1 || { echo "bench k=$k failed"; tail -5 $O/batch_k$k.log; exit 1; }
  grep '^{' $O/batch_k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k=$k', round(d['ms_per_step'],1), round(d['kernel']['avg_ms'],1), round(d['roofline']['frac'],4), d['check']['ok'])"
  grep '^{' $O/batch_k$k.log >> $O/batch_all.jsonl
done
