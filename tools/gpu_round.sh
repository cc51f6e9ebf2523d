#!/bin/bash
# One GPU-box session: tools/gpu_round.sh TAG STEP...  (run from the repo root by gpurun)
#   tests   the whole -m gpu suite          smoke   __graft_entry__.smoke()
#   prof    rocprofv3 kernel stats of the default bench line
#   pmc     HBM counters of the default bench line (tools/pmc_traffic.sh's passes, into gpurun_out/pmc)
#   walks:KIND  tools/walk_calls.py KIND (per-call times of chunk walks, mapped file and attached)
#   mpc:N   tools/mpc_request.py N (one MPC request end to end over N templates)
#   any other STEP is a bench line named in the table below
# Output under gpurun_out/TAG; every GPU step has its own time limit and the script stops at
# the first failure (no retries).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
bench_args() {
    case $1 in
    default) echo "" ;;
    masks) echo "--workload masks --steps 20 --warmup 3" ;;
    shares) echo "--workload shares --steps 5 --warmup 1" ;;
    batch) echo "--workload batch --queries 1024 --steps 1 --warmup 1 --no-cpu-baseline" ;;
    resolver) echo "--workload resolver --steps 20 --warmup 3" ;;
    resolve-masks) echo "--workload resolve-masks --steps 20 --warmup 3" ;;
    host-resolver) echo "--workload host-resolver --steps 5 --warmup 1" ;;
    host-resolve-masks) echo "--workload host-resolve-masks --steps 10 --warmup 2" ;;
    prepare) echo "--workload prepare --steps 2 --warmup 1" ;;
    load) echo "--workload load --steps 3 --warmup 1 --no-cpu-baseline" ;;
    host-masks) echo "--workload host-masks --steps 3 --warmup 1" ;;
    host-shares) echo "--workload host-shares --steps 3 --warmup 1" ;;
    host-masks_chunk20k) echo "--workload host-masks --chunk 20000 --steps 3 --warmup 1" ;;
    host-shares_chunk20k) echo "--workload host-shares --chunk 20000 --steps 3 --warmup 1" ;;
    host-masks_attached) echo "--workload host-masks --attached --steps 3 --warmup 1" ;;
    host-shares_attached) echo "--workload host-shares --attached --steps 3 --warmup 1" ;;
    host-masks_mmap) echo "--workload host-masks --mmap --steps 10 --warmup 2" ;;
    host-shares_mmap) echo "--workload host-shares --mmap --steps 10 --warmup 2" ;;
    host-shares_mmap2m) echo "--workload host-shares --mmap --n-per-gpu 2000000 --steps 10 --warmup 2" ;;
    host-masks_mmap_off) echo "--workload host-masks --mmap --steps 3 --warmup 1 --no-auto-resident" ;;
    *) return 1 ;;
    esac
}
for S in "$@"; do
    case $S in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 ||
            { echo "tests rc=$?"; grep -E "FAILED|Error|error" $O/tests.log | tail -20; tail -5 $O/tests.log; exit 1; }
        tail -1 $O/tests.log ;;
    tests:*)  # tests:file1,file2 -- those GPU test files only
        F=$(echo ${S#tests:} | tr ',' ' ' | sed 's#\([^ ]*\)#tests/\1#g')
        timeout -k 10 900 python -u -m pytest $F -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_part.log 2>&1 ||
            { echo "tests rc=$?"; grep -E "FAILED|Error|error|assert" $O/tests_part.log | tail -20; tail -5 $O/tests_part.log; exit 1; }
        tail -1 $O/tests_part.log ;;
    mpc:*)  # mpc:N -- one MPC request end to end over N templates (tools/mpc_request.py)
        timeout -k 10 700 python tools/mpc_request.py ${S#mpc:} 3 > $O/mpc_request_${S#mpc:}.log 2>&1 ||
            { echo "mpc rc=$?"; tail -5 $O/mpc_request_${S#mpc:}.log; exit 1; }
        tail -1 $O/mpc_request_${S#mpc:}.log ;;
    diag)
        timeout -k 10 300 python tools/resident_diag.py > $O/resident_diag.log 2>&1 || { echo "diag rc=$?"; tail -5 $O/resident_diag.log; exit 1; }
        cat $O/resident_diag.log ;;
    walks:*)  # walks:shares / walks:masks -- per-call times of chunk walks (tools/walk_calls.py)
        timeout -k 10 300 python tools/walk_calls.py ${S#walks:} 8 > $O/walks_${S#walks:}.log 2>&1 ||
            { echo "walks rc=$?"; tail -5 $O/walks_${S#walks:}.log; exit 1; }
        grep -E "walk 7:" $O/walks_${S#walks:}.log ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
        tail -1 $O/smoke.log ;;
    prof)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- \
            python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof_search.log; exit 1; }
        echo "prof ok" ;;
    pmc)
        WORKLOADS=search NO_LANES=1 bash tools/pmc_traffic.sh > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
        tail -3 $O/pmc.log ;;
    *)
        A=$(bench_args $S) || { echo "unknown step $S"; exit 2; }
        timeout -k 10 300 python bench.py $A > $O/$S.log 2>&1 || { echo "$S rc=$?"; tail -3 $O/$S.log; exit 1; }
        grep '^{' $O/$S.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('cpu_baseline') or {}; k=d.get('kernel') or {}; print('$S', '%.4g'%d['value'], d['unit'], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(k.get('avg_ms') or 0,4), 'frac', round(d['roofline']['frac'],3), 'cpu', c.get('value'), c.get('cores'))" ;;
    esac
done
echo "all ok"
