#!/bin/bash
# Per-phase times of the 3M-mask walk's calls from C++, against a build of the library with phase
# timers (tools/diag/libiris_hip_timers.so, built outside the tree's sources).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L tools/diag -l:libiris_hip_timers.so \
    -Wl,-rpath,$PWD/tools/diag -Wl,-rpath,/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -o /tmp/walk_host_t || exit 1
for H in ${HELPERS:-3 7}; do
    echo "== ${KIND:-masks} IRIS_COPY_HELPERS=$H $MODE ${IRIS_DIAG_PLAIN:+plain-stores} ${IRIS_DIAG_SPREAD:+spread} $PIN ${IRIS_DIAG_HELPER_CPUS:+helpers on $IRIS_DIAG_HELPER_CPUS} ${IRIS_DIAG_NODE:+helpers on the creator node}" >> $O/call_timers.txt
    IRIS_COPY_HELPERS=$H timeout -k 10 180 $PIN /tmp/walk_host_t ${KIND:-masks} ${RECORDS:-3000000} 6 - $MODE >> $O/call_timers.txt 2>&1 || { echo "rc=$?"; exit 1; }
done
grep -E "==|calls after|walk [1-5]|call timers|diag:|first call of" $O/call_timers.txt
