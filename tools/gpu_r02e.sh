set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "batch_1024_queries or many_groups" > $O/t.log 2>&1 || { echo "tests k2 failed"; tail -30 $O/t.log; exit 1; }
IRIS_BATCH_KERNEL=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k "batch_1024_queries or many_groups" > $O/t3.log 2>&1 || { echo "tests k3 failed"; tail -30 $O/t3.log; exit 1; }
tail -1 $O/t.log; tail -1 $O/t3.log
for k in 2 3 1 2 3; do
  IRIS_BATCH_KERNEL=$k timeout -k 10 300 python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > $O/batch_k$k.log 2>&1 || { echo "bench k=$k failed"; tail -5 $O/batch_k$k.log; exit 1; }
  grep '^{' $O/batch_k$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel", '$k', d["kernel"]["avg_ms"], d["roofline"]["frac"], d["check"]["ok"])'
done
