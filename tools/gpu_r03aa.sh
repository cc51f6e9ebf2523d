#!/bin/bash
# read-ahead v3: GPU suite, host-slice bench lines; then the batched-kernel A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -3 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log > $O/$name.jsonl
  python3 -c "
import json; d=json.loads(open('$O/$name.jsonl').read())
print('$name', 'value %.4g'%d['value'], 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['kernel']['avg_ms'],5), 'ok', d['check']['ok'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), {k: v for k, v in d.items() if k in ('resident_same_chunks',)})
"
}
run host-masks_attached --workload host-masks --attached --steps 3 --warmup 1
run host-shares_attached --workload host-shares --attached --steps 3 --warmup 1
timeout -k 10 120 python tools/ra_diag.py masks 2000000 3 > $O/diag_masks.log 2>&1 && cat $O/diag_masks.log
timeout -k 10 600 ./tools/gpu_r03x.sh
