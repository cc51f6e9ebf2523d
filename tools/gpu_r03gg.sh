#!/bin/bash
# batched kernel: bit-field-insert selects in the N-group epilogue (shipped) vs compare + v_cndmask (libiris_nobfi)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03gg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q -k "batch" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for lib in hip nobfi; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -k 10 200 python bench.py --workload batch --queries 1024 --steps 2 --warmup 1 --no-cpu-baseline --prewarm-s 0.5 > $O/${lib}_$r.log 2>&1 || { echo "$lib bench rc=$?"; tail -3 $O/${lib}_$r.log; exit 1; }
  grep '^{' $O/${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib r$r', 'kernel_ms', round(d['kernel']['avg_ms'],1), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
done
done
