set -o pipefail
O=gpurun_out/r02a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bench_dist.py > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
timeout -k 10 200 python bench.py > $O/search.log 2>&1 || { echo search failed; tail $O/search.log; exit 1; }
timeout -k 10 200 python bench.py --workload shares --steps 5 --warmup 1 > $O/shares.log 2>&1 || { echo shares failed; exit 1; }
timeout -k 10 200 python bench.py --workload criterion --steps 20 > $O/crit.log 2>&1 || { echo crit failed; exit 1; }
timeout -k 10 300 python bench.py --workload batch --steps 2 --warmup 1 > $O/batch.log 2>&1 || { echo batch failed; exit 1; }
tail -2 $O/t.log; for f in search shares crit batch; do grep '^{' $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["check"]["ok"], (d.get("cpu_baseline") or {}).get("value"), (d.get("cpu_baseline") or {}).get("cores"))'; done
