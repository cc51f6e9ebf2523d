# round 4, the final tree: the whole -m gpu suite and smoke(); the default bench line with its rocprof kernel stats; the
# host-slice lines (whole-array and participant-sized uploads, attached walk) and the load line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -3 $O/$name.log; exit 1; }
    python3 tools/keep_bench.py $O/kept_$name.jsonl $O/$name.log > /dev/null || { echo "$name check failed"; exit 1; }
    grep '^{' $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline') or {}; print('$name', '%.4g'%d['value'], d['unit'], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],3), 'cpu', c.get('value'), c.get('cores'))"
}
run default 300
run host-masks 300 --workload host-masks --steps 3 --warmup 1
run host-shares 300 --workload host-shares --steps 3 --warmup 1
run host-masks_chunk20k 300 --workload host-masks --chunk 20000 --steps 3 --warmup 1
run host-masks_attached 300 --workload host-masks --attached --steps 3 --warmup 1
run load 300 --workload load --steps 3 --warmup 1 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo all ok
