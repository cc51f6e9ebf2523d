#!/bin/bash
# Batched-kernel variants on one box: kernel time (bench.py) + clock / MFMA busy / waits (one PMC pass).
# usage: tools/batch_variants.sh Q "label:lib.so:KERNEL" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
Q=$1; shift
O=gpurun_out/batch_variants; mkdir -p $O
for spec in "$@"; do
    IFS=: read label lib k <<< "$spec"
    export IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib IRIS_BATCH_KERNEL=$k IRIS_TEST_HOOKS=1
    timeout -k 10 200 python bench.py --workload batch --queries $Q --steps 3 --warmup 1 --no-cpu-baseline --prewarm-s 0.5 > $O/$label.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "$label bench rc=$rc"; tail -3 $O/$label.log; exit 1; fi
    ms=$(grep '^{' $O/$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel']['avg_ms'],1), d['check']['ok'])")
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA --output-format csv -d $O/pmc_$label -o run -- \
        python3 bench.py --workload batch --queries $Q --steps 1 --warmup 0 --no-cpu-baseline --prewarm-s 0 > $O/pmc_$label.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "$label pmc rc=$rc"; exit 1; fi
    pm=$(python3 - $O/pmc_$label <<'PY'
import csv, collections, glob, sys
by = collections.defaultdict(dict); ts = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "batch" in r["Kernel_Name"] and "reduce" not in r["Kernel_Name"]:
            by[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            ts[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
d = max(by, key=lambda k: ts[k]); v = by[d]; t = ts[d]
clk = v["GRBM_GUI_ACTIVE"] / 8 / t
print(f"pmc_ms {t*1e3:.1f} clock {clk/1e9:.3f} GHz mfma_busy {v['SQ_VALU_MFMA_BUSY_CYCLES']/1024/(clk*t):.3f} "
      f"wait_any {v['SQ_WAIT_ANY']/v['SQ_WAVE_CYCLES']:.3f} wait_inst {v['SQ_WAIT_INST_ANY']/v['SQ_WAVE_CYCLES']:.3f} "
      f"Mcycles {clk*t/1e6:.1f} busyxclk {v['SQ_VALU_MFMA_BUSY_CYCLES']/1024/t/1e9:.3f}")
PY
)
    echo "$label kernel_ms,ok= $ms | $pm"
done
