#!/bin/bash
# Times bench.py for several in-tree library builds (IRIS_HIP_LIB) on the GPU box.
# usage: tools/run_variants.sh WORKLOAD lib1.so lib2.so ...   (stops at the first fault/timeout)
w=$1; shift
mkdir -p gpurun_out
i=0
for lib in "$@"; do
    i=$((i + 1))
    name=$(basename "$lib" .so)
    log="gpurun_out/var_${w}_${i}_${name}.log"
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -k 10 150 python bench.py --workload "$w" --no-cpu-baseline $BENCH_ARGS \
        > "$log" 2>&1
    rc=$?
    kms=$(grep '^{' "$log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel']['avg_ms'],4), d['check']['ok'])" 2>/dev/null)
    echo "$w $i $name rc=$rc kernel_ms,ok=$kms"
    # 3 = parity spot-check failed (expected for timing-only variants); anything else non-zero stops
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
