# readahead of attached host-slice calls: GPU suite, then the reference-loop bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03r; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_attach.py -x -q --timeout 120 --timeout-method thread > $O/attach.log 2>&1 || { echo "attach tests rc=$?"; tail -30 $O/attach.log; exit 1; }
tail -1 $O/attach.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -3 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log > $O/$name.jsonl
  python3 -c "
import json; d=json.loads(open('$O/$name.jsonl').read())
print('$name', 'value %.4g'%d['value'], 'ms', round(d['ms_per_step'],4), 'unprof', d.get('ms_per_step_unprofiled'), 'kernel_ms', round(d['kernel']['avg_ms'],5), 'ok', d['check']['ok'], {k: v for k, v in d.items() if k in ('attached', 'resident_same_chunks')})
"
}
run host-masks_attached --workload host-masks --attached --steps 3 --warmup 1 --no-cpu-baseline
run host-shares_attached --workload host-shares --attached --steps 3 --warmup 1 --no-cpu-baseline
IRIS_READAHEAD=0 run host-masks_attached_nora --workload host-masks --attached --steps 3 --warmup 1 --no-cpu-baseline
IRIS_READAHEAD=0 run host-shares_attached_nora --workload host-shares --attached --steps 3 --warmup 1 --no-cpu-baseline
run chunk20k_masks --workload masks --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline --reuse-engine
run chunk20k_search --n-per-gpu 20000 --steps 200 --warmup 10 --no-cpu-baseline --reuse-engine
