#!/bin/bash
# TRITS vs TILES search on one box (interleaved), then SQ counters of the TRITS kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/trits_perf
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trits.py -x -q --timeout 200 --timeout-method thread \
    > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for lay in tiles trits tiles trits; do
  timeout -k 10 120 python bench.py --layout $lay --steps 50 --warmup 5 --prewarm-s 1 --no-cpu-baseline \
      >> $out/bench.jsonl 2>> $out/bench.err || { echo "bench $lay failed"; tail $out/bench.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/trits_perf/bench.jsonl"):
    j = json.loads(l)
    print(j["config"]["layout"], round(j["ms_per_step"], 3), "kernel", round(j["kernel"]["avg_ms"], 3),
          "value %.3e" % j["value"], "frac", round(j["roofline"]["frac"], 3), j["check"]["ok"])
PY
[ -n "$NOPMC" ] && exit 0
p1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
p2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_COUNT"
p3="SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
i=0
for p in "$p1" "$p2" "$p3"; do
    i=$((i+1))
    for lay in trits tiles; do
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$out/p${i}_$lay" -o run -- \
        python3 bench.py --no-cpu-baseline --layout $lay --steps 3 --warmup 1 --prewarm-s 0 > "$out/p${i}_$lay.log" 2>&1 \
        || { echo "pass $i $lay failed rc=$?"; tail -5 "$out/p${i}_$lay.log"; exit 1; }
    done
done
python3 - "$out" <<'PY' > $out/summary.txt
import csv, glob, sys, collections
out = sys.argv[1]
for lay, kern in (("trits", "trits_mfma_kernel<1"), ("tiles", "template_mfma_kernel<1")):
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for f in glob.glob(f"{out}/p*_{lay}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kern not in row["Kernel_Name"]:
                continue
            acc[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row.get("Dispatch_Id"))
    print("==", lay, kern)
    for k in sorted(acc):
        print(f"{k:32s} {acc[k] / max(1, len(disp[k])):.6g}  (per dispatch, {len(disp[k])} dispatches)")
PY
cat $out/summary.txt
