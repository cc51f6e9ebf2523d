#!/bin/bash
# Small-range template search A/B: the search parity + fuzz tests, then bench.py on configs[0]
# (criterion: 1 x 31 x 10k) and a 20k-template search with the shipped library and the variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/small_ab; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for v in hip "$@"; do
    for w in criterion search20k; do
      args="--workload criterion --steps 200 --warmup 10"
      [ $w = search20k ] && args="--n-per-gpu 20000 --steps 200 --warmup 10 --prewarm-s 0.5"
      IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -k 10 120 python bench.py $args --no-cpu-baseline \
          > $out/$w-$v$r.json 2>> $out/err.log || { echo "bench $w $v failed"; tail $out/err.log; exit 1; }
      python3 -c "import json; j=json.load(open('$out/$w-$v$r.json')); print('%-10s %-8s'%('$w','$v'), 'step_ms', round(j['ms_per_step'],4), 'kernel', round(j['kernel']['avg_ms'],4), 'value %.3e'%j['value'], j['check'].get('ok'))"
    done
  done
done
