#!/bin/bash
# search: 8 tiles per wave, one wave per SIMD (256 accumulators in AGPRs; half the query-fragment L2 reads per
# template) vs the shipped 4 tiles x 2 waves per SIMD; parity of the variant, then interleaved bench runs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03rr; rm -rf $O; mkdir -p $O
IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_t8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "search or template or mfma" --timeout 120 --timeout-method thread > $O/t8_tests.log 2>&1 || { echo "t8 tests rc=$?"; tail -20 $O/t8_tests.log; exit 1; }
tail -1 $O/t8_tests.log
for r in 1 2; do
for lib in hip t8; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/${lib}_$r.log 2>&1 || { echo "$lib bench rc=$?"; tail -3 $O/${lib}_$r.log; exit 1; }
  grep '^{' $O/${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib r$r', 'kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
done
done
