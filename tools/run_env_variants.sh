#!/bin/bash
# Times one bench workload under several values of an environment knob (same library).
# usage: tools/run_env_variants.sh WORKLOAD VAR v1 v2 ...   ("-" = unset); BENCH_ARGS passed through
w=$1; var=$2; shift 2
mkdir -p gpurun_out
for v in "$@"; do
    log="gpurun_out/envvar_${w}_${var}_${v}.log"
    if [ "$v" = "-" ]; then
        env -u "$var" timeout -k 10 200 python bench.py --workload "$w" --no-cpu-baseline $BENCH_ARGS > "$log" 2>&1
    else
        env "$var=$v" timeout -k 10 200 python bench.py --workload "$w" --no-cpu-baseline $BENCH_ARGS > "$log" 2>&1
    fi
    rc=$?
    kms=$(grep '^{' "$log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel']['avg_ms'],4), d['check']['ok'])" 2>/dev/null)
    echo "$w $var=$v rc=$rc kernel_ms,ok=$kms"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
