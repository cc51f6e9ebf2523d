# share preparation decomposition: shipped vs no-stores vs no-ChaCha diagnostic builds + PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03i; mkdir -p $O
for spec in ship:libiris_hip.so nostore:libiris_prepnost.so nochacha:libiris_prepnocc.so ship2:libiris_hip.so; do
  IFS=: read label lib <<< "$spec"
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -k 10 200 python bench.py --workload prepare --steps 10 --warmup 1 --prewarm-s 1 --no-cpu-baseline > $O/$label.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "$label rc=$rc"; tail -3 $O/$label.log; exit 1; fi
  grep '^{' $O/$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['kernel']['avg_ms'],3), d['check']['ok'])"
done
for c in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM" WRITE_SIZE FETCH_SIZE; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$tag -o run -- python3 bench.py --workload prepare --steps 1 --warmup 0 --prewarm-s 0 --no-cpu-baseline > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag rc=$?"; tail -3 $O/pmc_$tag.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(float); t = {}
for f in glob.glob(f"{out}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "prepare_direct_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            t[r["Counter_Name"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
for k, v in sorted(acc.items()):
    print(f"{k:28s} {v:.5g}")
PY
