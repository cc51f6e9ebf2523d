#!/bin/bash
# batched kernel: nontemporal query-tile loads (libiris_ant) vs shipped; time + FETCH_SIZE per launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03x; mkdir -p $O
for r in 1 2; do
for lib in hip ant; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -k 10 200 python bench.py --workload batch --queries 1024 --steps 2 --warmup 1 --no-cpu-baseline --prewarm-s 0.5 > $O/${lib}_$r.log 2>&1 || { echo "$lib bench rc=$?"; tail -3 $O/${lib}_$r.log; exit 1; }
  grep '^{' $O/${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib r$r', 'kernel_ms', round(d['kernel']['avg_ms'],1), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
done
done
for lib in hip ant; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$lib -o run -- python3 bench.py --workload batch --queries 1024 --steps 1 --warmup 0 --no-cpu-baseline --prewarm-s 0 > $O/pmc_$lib.log 2>&1 || { echo "pmc $lib rc=$?"; tail -3 $O/pmc_$lib.log; exit 1; }
  python3 - $O/pmc_$lib $lib <<'PY'
import csv, glob, sys
tot = 0.0; t = 0
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "batch_lds_kernel" in r["Kernel_Name"] and r["Counter_Name"].startswith("FETCH_SIZE"):
            tot += float(r["Counter_Value"]); t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print(sys.argv[2], "FETCH_SIZE", tot, "kB -> x1024x2 =", round(tot * 2048 / 1e12, 3), "TB beyond L2 per launch;", round(t, 1), "ms")
PY
done
