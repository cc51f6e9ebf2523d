# round 4: completion-word device-output calls (tests + participant-sized chunk lines), the
# masks read/write ceiling (ubench_rw at 8 and 12 waves per CU) and masks kernel variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -3 $O/$name.log; exit 1; }
    grep '^{' $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'ms', round(d['ms_per_step'],4), 'unprof', d.get('ms_per_step_unprofiled'), 'kernel_ms', round(d['kernel']['avg_ms'],4), 'ok', d['check']['ok'])"
}
for w in masks shares search; do
  run chunk20k_${w}_reuse 200 --workload $w --n-per-gpu 20000 --steps 300 --warmup 20 --no-cpu-baseline --reuse-engine --prewarm-s 1
done
run chunk20k_shares 200 --workload shares --n-per-gpu 20000 --steps 300 --warmup 20 --no-cpu-baseline --prewarm-s 1
timeout -k 10 120 tools/ubench_rw > $O/ubench_rw.txt 2>&1 || { echo "ubench rc=$?"; exit 1; }
cat $O/ubench_rw.txt
BENCH_ARGS="--steps 200 --warmup 5" timeout -k 10 900 bash tools/run_variants.sh masks libiris_hip.so libiris_t8q0.so libiris_t4b3q0.so libiris_t4b2q1.so libiris_t2b4q0.so libiris_hip.so libiris_t4b3q0.so > $O/variants.txt 2>&1 || { echo "variants rc=$?"; cat $O/variants.txt; exit 1; }
cat $O/variants.txt
