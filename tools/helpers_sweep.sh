#!/bin/bash
# Per-call times of the 3M-mask walk from C++ (tools/walk_host.cpp) against the number of copy-out
# helper threads (IRIS_COPY_HELPERS): is the call's host side (the expansion into the caller's
# array) what bounds the walk?  Output: gpurun_out/$1/helpers_sweep.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip \
    -Wl,-rpath,$PWD/mpc-iris-code_amd -Wl,-rpath-link,/opt/rocm/lib -o /tmp/walk_host || exit 1
for H in ${HELPERS:-0 1 3 7}; do
    echo "== IRIS_COPY_HELPERS=$H" >> $O/helpers_sweep.txt
    IRIS_COPY_HELPERS=$H timeout -k 10 180 /tmp/walk_host masks 3000000 6 >> $O/helpers_sweep.txt 2>&1 || { echo "rc=$?"; exit 1; }
done
grep -E "==|calls after|walk 5" $O/helpers_sweep.txt
