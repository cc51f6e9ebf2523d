#!/bin/bash
# Resolver A/B: the resolver GPU tests, then bench.py --workload resolver (3 parties, 10M entries) with the
# shipped library and the variant libraries named, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/res_ab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "resolv" -x -q --timeout 200 --timeout-method thread \
    > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for v in hip "$@"; do
    IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -k 10 120 python bench.py --workload resolver --steps 200 \
        --warmup 10 --prewarm-s 1 --no-cpu-baseline > $out/$v$r.json 2>> $out/err.log || { echo "bench $v failed"; tail $out/err.log; exit 1; }
    python3 -c "import json; j=json.load(open('$out/$v$r.json')); print('%-8s'%'$v', round(j['ms_per_step'],4), 'kernel', round(j['kernel']['avg_ms'],4), j['check'].get('ok'))"
  done
done
