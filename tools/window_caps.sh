#!/bin/bash
# Read-ahead window cap sweep of the chunk walks from C++ (tools/walk_host): masks 3M and shares 1M
# records in 20 000-record calls, window caps of 4..54 chunks (IRIS_READAHEAD_WINDOW_MAX test hook)
# and the default.  Output: gpurun_out/$1/window_caps.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
g++ -O2 -std=c++17 -I include tools/walk_host.cpp -L mpc-iris-code_amd -liris_hip -Wl,-rpath,$PWD/mpc-iris-code_amd \
    -Wl,-rpath-link,/opt/rocm/lib -o tools/walk_host || exit 1
for kind in masks shares; do
    n=$([ $kind = masks ] && echo 3000000 || echo 1000000)
    for cap in default 4 8 16 54; do
        if [ $cap = default ]; then env=""; else env="IRIS_TEST_HOOKS=1 IRIS_READAHEAD_WINDOW_MAX=$cap"; fi
        echo "== $kind n=$n cap=$cap" >> $O/window_caps.txt
        env $env timeout -k 10 200 tools/walk_host $kind $n 6 >> $O/window_caps.txt 2>&1 || exit 1
    done
done
grep -E "^==|walk 5|calls after" $O/window_caps.txt
