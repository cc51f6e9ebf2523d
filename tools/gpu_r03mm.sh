#!/bin/bash
# search tail split: parity (tail vs one-shape, oracle), then 10M / 12.5M A/B interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03mm; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_group.py -x -q -k "not batch" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 10000000 12500000; do
for r in 1 2; do
for t in 1 0; do
  IRIS_SEARCH_TAIL=$t timeout -k 10 200 python bench.py --n-per-gpu $n --steps 30 --warmup 3 --no-cpu-baseline --prewarm-s 2 > $O/s_${n}_${t}_$r.log 2>&1 || { echo "bench rc=$?"; tail -3 $O/s_${n}_${t}_$r.log; exit 1; }
  grep '^{' $O/s_${n}_${t}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n $n tail $t r$r kernel_ms', round(d['kernel']['avg_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
done
done
done
