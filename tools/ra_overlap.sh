#!/bin/bash
# Do consecutive read-ahead windows overlap on the two side streams?  rocprofv3 kernel trace of a
# 1M-share walk from C++ (tools/walk_host), then begin/end of each shares kernel and the gap to
# the one before it (negative = overlap).  Output under gpurun_out/$1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip -Wl,-rpath,$PWD/mpc-iris-code_amd \
    -Wl,-rpath-link,/opt/rocm/lib -o tools/walk_host || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/ra_trace -o run -- tools/walk_host shares 1000000 4 \
    > $O/ra_overlap_walk.txt 2>&1 || exit 1
python3 - "$O" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/ra_trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "shares" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]))
rows.sort()
out = open(sys.argv[1] + "/ra_overlap.txt", "w")
prev_end = None
for s, e, k in rows[-30:]:
    gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:9.1f}"
    print(f"{s / 1e3:14.1f} {e / 1e3:14.1f} {(e - s) / 1e3:9.1f} us gap {gap} {k}", file=out)
    prev_end = e if prev_end is None else max(prev_end, e)
out.close()
print(open(sys.argv[1] + "/ra_overlap.txt").read())
PY
