#!/bin/bash
# TILES search kernel: what bounds it.  bench.py (configs[1], 10M) with the shipped library and
# diagnostic builds of chunk_step (csrc/iris_mfma.hip, IRIS_MFMA_DIAG = 1 no den MFMA, 2 no
# MFMAs, 3 no operand expansion; tools/build_variant.sh mdiagN -DIRIS_MFMA_DIAG=N; their result
# checks fail by design), two interleaved rounds, then GRBM/SQ counters per variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/tiles_diag
mkdir -p $out
for r in 1 2; do
  for v in hip "$@"; do
    IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -k 10 120 python bench.py --layout ${LAYOUT:-tiles} --steps 100 --warmup 5 \
        --prewarm-s 1 --no-cpu-baseline > $out/$v$r.json 2>> $out/err.log
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "bench $v failed rc=$rc"; tail $out/err.log; exit 1; fi
    python3 -c "import json; j=json.load(open('$out/$v$r.json')); print('%-8s'%'$v', round(j['ms_per_step'],3), 'kernel', round(j['kernel']['avg_ms'],3), j['check'].get('ok'))"
  done
done
[ -n "$NOPMC" ] && exit 0
for v in hip "$@"; do
  IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
      --output-format csv -d "$out/pmc_$v" -o run -- python3 bench.py --layout ${LAYOUT:-tiles} --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 \
      > "$out/pmc_$v.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "pmc $v failed rc=$rc"; tail -5 "$out/pmc_$v.log"; exit 1; fi
done
python3 - "$out" "$@" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in ["hip"] + sys.argv[2:]:
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for f in glob.glob(f"{out}/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if not any(k in row["Kernel_Name"] for k in ("template_mfma_kernel<1", "trits_mfma_kernel<1")):
                continue
            acc[row["Counter_Name"]] += float(row["Counter_Value"])
            disp[row["Counter_Name"]].add(row.get("Dispatch_Id"))
    print(v, " ".join(f"{k}={acc[k] / max(1, len(disp[k])):.4g}" for k in sorted(acc)))
PY
