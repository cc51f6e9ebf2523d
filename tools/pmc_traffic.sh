#!/bin/bash
# HBM traffic per launch from PMC counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE and
# WRITE_SIZE each in their own rocprofv3 pass (--pmc only with --kernel-trace-free runs),
# for each bench workload; summarised by tools/pmc_summarize.py into gpurun_out/pmc/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmc
mkdir -p $out
pass() {  # workload counter tag args...
    local w=$1 c=$2 tag=$3; shift 3
    timeout -k 10 300 rocprofv3 --pmc "$c" --output-format csv -d "$out/${w}_$c$tag" -o run -- \
        python3 bench.py --no-cpu-baseline --workload "$w" "$@" > "$out/${w}_$c$tag.log" 2>&1 \
        || { echo "$w $c$tag failed rc=$?"; tail -5 "$out/${w}_$c$tag.log"; exit 1; }
    echo "$w $c$tag ok"
}
ws=${WORKLOADS:-search masks shares resolver}
for w in $ws; do
    a="--steps 3 --warmup 1"
    [ $w = batch ] && a="--queries 1024 --steps 1 --warmup 0"
    pass $w FETCH_SIZE "" $a || exit 1
    pass $w WRITE_SIZE "" $a || exit 1
done
if [ -z "$NO_LANES" ]; then
    pass search FETCH_SIZE _lanes --steps 3 --warmup 1 --layout lanes || exit 1
    pass search WRITE_SIZE _lanes --steps 3 --warmup 1 --layout lanes || exit 1
fi
