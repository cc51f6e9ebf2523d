#!/bin/bash
# search kernel time per template at 10M / 40M / 80M: how much does the grid's drain cost at 10M?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03dd; mkdir -p $O
for n in 10000000 40000000 80000000 10000000; do
  timeout -k 10 300 python bench.py --n-per-gpu $n --steps 10 --warmup 2 --no-cpu-baseline --prewarm-s 2 > $O/search_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -3 $O/search_$n.log; exit 1; }
  grep '^{' $O/search_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel']['avg_ms']; print('$n', 'kernel_ms', round(k,4), 'ns/template', round(k*1e6/$n,4), 'TB/s', round(3200*$n/k/1e9,1), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
done
