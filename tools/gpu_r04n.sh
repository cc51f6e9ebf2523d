# round 4: (1) the per-workgroup timeline of a 10M search launch (diagnostic build -DIRIS_MFMA_DIAG=4);
# (2) the batched launch's FETCH_SIZE three times on one box (is the 2.9-4.5 TB spread run-to-run or box-to-box?)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04n; mkdir -p $O
IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_tl.so timeout -k 10 300 python3 tools/search_timeline.py > $O/timeline.txt 2>&1 || { echo "timeline rc=$?"; tail -5 $O/timeline.txt; exit 1; }
cat $O/timeline.txt
for i in 1 2 3; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$i -o run -- python3 bench.py --no-cpu-baseline --workload batch --queries 1024 --steps 1 --warmup 0 --prewarm-s 0 > $O/fetch$i.log 2>&1 || { echo "pmc $i rc=$?"; tail -3 $O/fetch$i.log; exit 1; }
  python3 - $O/fetch$i <<'PY'
import csv, glob, sys
by = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "batch_lds_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            by[r["Dispatch_Id"]] = by.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
big = max(by.values())
print("batch FETCH_SIZE beyond L2 per launch: %.3f TB" % (big * 1024 * 2 / 1e12))
PY
done
