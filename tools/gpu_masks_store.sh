#!/bin/bash
# MasksEngine write-stream decomposition: bench.py --workload masks (10M masks, [u16;31] rows out)
# with the shipped library and the diagnostic builds that store half / none of the row bytes
# (tools/build_variant.sh storehalf -DIRIS_STORE_DIAG=1, storenone -DIRIS_STORE_DIAG=2; their
# result checks fail by design).  Two interleaved rounds on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/masks_store
mkdir -p $out
for r in 1 2; do
  for v in hip storeplain storehalf storenone; do
    IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -k 10 120 python bench.py --workload masks --steps 200 \
        --warmup 10 --prewarm-s 1 --no-cpu-baseline > $out/$v$r.json 2>> $out/err.log
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "bench $v failed rc=$rc"; tail $out/err.log; exit 1; fi
    python3 -c "import json; j=json.load(open('$out/$v$r.json')); print('%-10s'%'$v', round(j['ms_per_step'],3), 'kernel', round(j['kernel']['avg_ms'],3), j['check'].get('ok'))"
  done
done
