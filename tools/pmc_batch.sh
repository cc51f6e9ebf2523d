#!/bin/bash
# SQ counters of the batched kernel (configs[2] shape at --queries Q), two passes:
# issue/wait breakdown and LDS; summarised into gpurun_out/pmc_batch/summary.txt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=${OUT:-gpurun_out/pmc_batch}
mkdir -p $out
Q=${Q:-64}
p1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
p2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
p3="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_COUNT"
i=0
for p in "$p1" "$p2" "$p3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- \
        python3 bench.py --no-cpu-baseline --workload batch --queries $Q --steps 1 --warmup 0 ${EXTRA} > "$out/p$i.log" 2>&1 \
        || { echo "pass $i failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
done
python3 - "$out" <<'PY' > $out/summary.txt
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(float)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "batch_kernel" not in row["Kernel_Name"] and "batch_lds_kernel" not in row["Kernel_Name"]:
            continue
        acc[row["Counter_Name"]] += float(row["Counter_Value"])
for k in sorted(acc):
    print(f"{k:32s} {acc[k]:.6g}")
PY
cat $out/summary.txt
