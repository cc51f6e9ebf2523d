#!/bin/bash
# rocprofv3 kernel-trace summaries of every bench workload (run on the GPU box from the repo root).
# Each run is bounded by its own timeout; the script stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prof
mkdir -p $out
run() {  # name, timeout, bench args...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o run -- \
        python3 bench.py --no-cpu-baseline "$@" > "$out/$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -5 "$out/$name.log"; exit 1; }
    echo "$name ok: $(grep '^{' "$out/$name.log" | cut -c1-160)"
}
run search 300 --steps 20 --warmup 3
run masks 300 --workload masks --steps 20 --warmup 3
run shares 300 --workload shares --steps 5 --warmup 1
run batch 300 --workload batch --queries 1024 --steps 1 --warmup 1
run resolver 300 --workload resolver --steps 20 --warmup 3
run resolve-masks 300 --workload resolve-masks --steps 20 --warmup 3
run prepare 300 --workload prepare --steps 2 --warmup 1
run load 300 --workload load --steps 2 --warmup 1
