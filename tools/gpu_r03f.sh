# batch kernels: shipped 4q x 8t (k=2) vs 2q x 16t groups (k=4) vs 2x2 waves (k=3): parity, time, PMC
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -k "batch_1024_queries or many_groups" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 2 4 3 2 4; do
  IRIS_BATCH_KERNEL=$k timeout -k 10 300 python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline > $O/batch_k$k.log 2>&1 || { echo "bench k=$k failed"; tail -5 $O/batch_k$k.log; exit 1; }
  grep '^{' $O/batch_k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k=$k', round(d['ms_per_step'],1), round(d['kernel']['avg_ms'],1), round(d['roofline']['frac'],4), d['check']['ok'])"
  grep '^{' $O/batch_k$k.log >> $O/batch_all.jsonl
done
for k in 2 4; do
  for c in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU"; do
    tag=$(echo $c | cut -d' ' -f1)
    IRIS_BATCH_KERNEL=$k timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_k${k}_$tag -o run -- python3 bench.py --no-cpu-baseline --workload batch --queries 1024 --steps 1 --warmup 0 --prewarm-s 0 > $O/pmc_k${k}_$tag.log 2>&1 || { echo "pmc k=$k $tag rc=$?"; tail -3 $O/pmc_k${k}_$tag.log; exit 1; }
  done
done
python3 - $O <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for k in (2, 4):
    acc = collections.defaultdict(float)
    for f in glob.glob(f"{out}/pmc_k{k}_*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "batch_lds_kernel" in row["Kernel_Name"]:
                acc[row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"k={k}", {c: f"{v:.4g}" for c, v in sorted(acc.items())})
    print(f"k={k} beyond-L2 bytes (FETCH*1024*2 + WRITE*1024): {acc['FETCH_SIZE']*2048 + acc['WRITE_SIZE']*1024:.4g}")
PY
