# Every bench.py workload once on one box, each line kept in profiles/ only if its check passed
# (tools/keep_bench.py).  usage: bash tools/bench_all_r02.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r02}; O=gpurun_out/bench_$T; mkdir -p $O
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -3 $O/$name.log; exit 1; }
    python3 tools/keep_bench.py $O/kept_$name.jsonl $O/$name.log > /dev/null || { echo "$name check failed"; exit 1; }
    grep '^{' $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline') or {}; print('$name', '%.4g'%d['value'], d['unit'], 'kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],3), 'cpu', c.get('value'), c.get('cores'))"
}
run search 300 --steps 20 --warmup 3
run masks 300 --workload masks --steps 20 --warmup 3
run shares 300 --workload shares --steps 5 --warmup 1
run batch 300 --workload batch --queries 1024 --steps 2 --warmup 1
run criterion 300 --workload criterion --steps 20 --warmup 3
run resolver 300 --workload resolver --steps 20 --warmup 3
run resolve-masks 300 --workload resolve-masks --steps 20 --warmup 3
run prepare 300 --workload prepare --steps 3 --warmup 1
run load 300 --workload load --steps 2 --warmup 1 --no-cpu-baseline
run host-shares 300 --workload host-shares --steps 3 --warmup 1
run host-masks 300 --workload host-masks --steps 3 --warmup 1
run search_lanes 300 --steps 10 --warmup 2 --layout lanes --no-cpu-baseline
run search_trits 300 --steps 20 --warmup 3 --layout trits --no-cpu-baseline
for w in search masks shares resolve-masks; do
  run chunk20k_$w 200 --workload $w --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline
done
echo all ok
