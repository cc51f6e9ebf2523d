# Every bench.py workload once on one box (round 4), each line kept in gpurun_out only if its
# check passed (tools/keep_bench.py), then rocprofv3 kernel stats of the headline search.
# usage: bash tools/bench_all_r04.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r04}; O=gpurun_out/bench_$T; mkdir -p $O
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -3 $O/$name.log; exit 1; }
    python3 tools/keep_bench.py $O/kept_$name.jsonl $O/$name.log > /dev/null || { echo "$name check failed"; exit 1; }
    grep '^{' $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline') or {}; print('$name', '%.4g'%d['value'], d['unit'], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],3), 'cpu', c.get('value'), c.get('cores'))"
}
run search 300 --steps 20 --warmup 3
run search_single 300 --gpus 1 --single-process --steps 20 --warmup 3 --no-cpu-baseline
run masks 300 --workload masks --steps 20 --warmup 3
run shares 300 --workload shares --steps 5 --warmup 1
run batch 300 --workload batch --queries 1024 --steps 3 --warmup 1
run criterion 300 --workload criterion --steps 20 --warmup 3
run resolver 300 --workload resolver --steps 20 --warmup 3
run resolve-masks 300 --workload resolve-masks --steps 20 --warmup 3
run prepare 300 --workload prepare --steps 5 --warmup 1
run load 300 --workload load --steps 2 --warmup 1 --no-cpu-baseline
run host-masks 300 --workload host-masks --steps 3 --warmup 1
run host-shares 300 --workload host-shares --steps 3 --warmup 1
run host-masks_attached 300 --workload host-masks --attached --steps 3 --warmup 1
run host-shares_attached 300 --workload host-shares --attached --steps 3 --warmup 1
run search_lanes 300 --steps 10 --warmup 2 --layout lanes --no-cpu-baseline
for w in search masks shares resolve-masks; do
  run chunk20k_$w 200 --workload $w --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline
done
run chunk20k_search_reuse 200 --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline --reuse-engine
run chunk20k_masks_reuse 200 --workload masks --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline --reuse-engine
run chunk20k_shares_reuse 200 --workload shares --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline --reuse-engine
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo "prof rc=$?"; exit 1; }
[ -n "$SKIP_PMC" ] && { echo "all ok (pmc skipped)"; exit 0; }
# HBM traffic of every HBM-bound kernel on this tree (FETCH_SIZE / WRITE_SIZE in separate passes)
WORKLOADS="search masks shares resolver resolve-masks" timeout -k 10 900 bash tools/pmc_traffic.sh > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
echo all ok
