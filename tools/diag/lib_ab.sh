#!/bin/bash
# A/B of two library builds on one box: the C++ walk (tools/walk_host.cpp) linked against the tree's
# libiris_hip.so and against tools/diag/$LIB (a variant built from a patched copy), alternating.
#   tools/diag/lib_ab.sh TAG LIB KIND RECORDS ROUNDS
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
LIB=$2; KIND=${3:-shares}; N=${4:-1000000}; R=${5:-2}
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip \
    -Wl,-rpath,$PWD/mpc-iris-code_amd -Wl,-rpath-link,/opt/rocm/lib -o /tmp/wh_a || exit 1
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L tools/diag -l:$LIB \
    -Wl,-rpath,$PWD/tools/diag -Wl,-rpath,/opt/rocm/lib -Wl,-rpath-link,/opt/rocm/lib -o /tmp/wh_b || exit 1
for r in $(seq $R); do
    for v in a b; do
        echo "== $v ($([ $v = a ] && echo libiris_hip.so || echo $LIB)) round $r" >> $O/lib_ab.txt
        timeout -k 10 240 /tmp/wh_$v $KIND $N 6 /tmp/lib_ab_$KIND.rec >> $O/lib_ab.txt 2>&1 || { echo "rc=$?"; tail -3 $O/lib_ab.txt; exit 1; }
    done
done
rm -f /tmp/lib_ab_$KIND.rec
grep -E "==|walk [1-5]:|calls after" $O/lib_ab.txt
