#!/bin/bash
# Where a walk's first call spends its time: HIP API + kernel trace (no counters) of
# tools/walk_host masks 200000 8; per-call API durations summarised by rocprofv3 --stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip -Wl,-rpath,$PWD/mpc-iris-code_amd \
    -Wl,-rpath-link,/opt/rocm/lib -o $TMPDIR/walk_host || exit 1
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/fc -o run -- $TMPDIR/walk_host masks 200000 8 \
    > $O/fc_walk.txt 2>&1 || { tail -5 $O/fc_walk.txt; exit 1; }
cat $O/fc_walk.txt | grep -E "^walk|calls"
head -25 $O/fc/run_hip_stats.csv
