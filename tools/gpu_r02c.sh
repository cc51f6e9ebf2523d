set -o pipefail
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py -k batch tests/test_gpu_parity.py::test_batch_search_matches_single > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
for k in 2 1 2 1; do
  IRIS_BATCH_KERNEL=$k timeout -k 10 300 python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > $O/batch_k$k.log 2>&1 || { echo "bench k=$k failed"; tail -5 $O/batch_k$k.log; exit 1; }
  grep '^{' $O/batch_k$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel", '$k', d["kernel"]["avg_ms"], d["roofline"]["frac"], d["check"]["ok"])'
done
