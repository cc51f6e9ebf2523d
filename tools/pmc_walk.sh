#!/bin/bash
# PMC traffic of a masks walk's read-ahead windows (the packed-row kernels): FETCH_SIZE and
# WRITE_SIZE, each in its own rocprofv3 pass, over tools/walk_host masks 3M x 3 walks; every walk
# computes each record once, so bytes per record = the masks kernels' counters / (3 x 3M).
# Output: gpurun_out/$1/pmc_walk.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip -Wl,-rpath,$PWD/mpc-iris-code_amd \
    -Wl,-rpath-link,/opt/rocm/lib -o tools/walk_host || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_walk_$c -o run -- tools/walk_host masks 3000000 3 \
        > $O/pmc_walk_$c.log 2>&1 || { echo "pass $c failed"; tail -5 $O/pmc_walk_$c.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys
o = sys.argv[1]
tot = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    s, k = 0.0, set()
    for f in glob.glob(f"{o}/pmc_walk_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c and ("masks_mfma_kernel" in r["Kernel_Name"] or "masks_split_kernel" in r["Kernel_Name"]):
                s += float(r["Counter_Value"])
                k.add(r["Kernel_Name"].split("(")[0])
    tot[c] = (s, sorted(k))
recs = 3 * 3_000_000
fetch = tot["FETCH_SIZE"][0] * 1024 * 2 / recs  # MI355X_MICROARCH.md: FETCH_SIZE kB, half of wide streaming reads
write = tot["WRITE_SIZE"][0] * 1024 / recs
with open(f"{o}/pmc_walk.txt", "w") as f:
    print(f"masks walk, 3 walks x 3M records, kernels {tot['FETCH_SIZE'][1]}", file=f)
    print(f"FETCH_SIZE x 1024 x 2 / record = {fetch:.1f} B (algorithmic read 1600 B)", file=f)
    print(f"WRITE_SIZE x 1024 / record = {write:.2f} B (algorithmic 32 B packed rows to pinned host memory)", file=f)
print(open(f"{o}/pmc_walk.txt").read())
PY
