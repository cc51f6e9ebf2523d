#!/bin/bash
# Batched-query A/B: the GPU tests that cover the batch kernels (oracle parity up to 1024 queries,
# 1024 x 10M planted), then bench.py --workload batch with the shipped library and the variant
# libraries named (mpc-iris-code_amd/libiris_<v>.so), interleaved on one box.  Q=${Q:-256} queries.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/batch_ab
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -k "batch" -x -q --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for v in hip "$@"; do
    IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --workload batch --queries ${Q:-256} \
        --steps 3 --warmup 1 --prewarm-s 0 --no-cpu-baseline > $out/$v$r.json 2>> $out/err.log || { echo "bench $v failed"; tail $out/err.log; exit 1; }
    python3 -c "import json; j=json.load(open('$out/$v$r.json')); print('%-9s'%'$v', round(j['ms_per_step'],2), 'kernel', round(j['kernel']['avg_ms'],2), 'value %.3e'%j['value'], 'frac', round(j['roofline']['frac'],3), j['check'].get('ok'))"
  done
done
