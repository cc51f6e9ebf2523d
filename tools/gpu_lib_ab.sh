#!/bin/bash
# Same-box A/B of whole libraries on several workloads: bash tools/gpu_lib_ab.sh VARIANT [workloads...]
# (default: search, trits search, masks, resolve-masks); two interleaved rounds, kernel ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
v=$1; shift
out=gpurun_out/lib_ab; mkdir -p $out
wls=${*:-"search trits masks resolve-masks"}
for r in 1 2; do
  for w in $wls; do
    for lib in hip $v; do
      args="--workload $w"; [ "$w" = trits ] && args="--layout trits"
      IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$lib.so timeout -k 10 120 python bench.py $args --steps 100 --warmup 5 \
          --prewarm-s 1 --no-cpu-baseline > $out/$w-$lib$r.json 2>> $out/err.log || { echo "bench $w $lib failed"; tail $out/err.log; exit 1; }
      python3 -c "import json; j=json.load(open('$out/$w-$lib$r.json')); print('%-14s %-8s'%('$w','$lib'), 'kernel', round(j['kernel']['avg_ms'],4), j['check'].get('ok'))"
    done
  done
done
