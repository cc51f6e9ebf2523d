#!/bin/bash
# read-ahead after the ordering fix: per-call walks and the host-slice bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03jj; mkdir -p $O
for kind in masks shares; do
  n=2000000; [ $kind = shares ] && n=200000
  for ra in 1 0; do
    IRIS_READAHEAD=$ra timeout -k 10 120 python tools/ra_diag.py $kind $n 3 > $O/diag_${kind}_$ra.log 2>&1 || { echo "diag rc=$?"; tail -3 $O/diag_${kind}_$ra.log; exit 1; }
    echo "$kind ra=$ra"; cat $O/diag_${kind}_$ra.log
  done
done
for w in host-masks host-shares; do
  timeout -k 10 300 python bench.py --workload $w --attached --steps 3 --warmup 1 > $O/$w.log 2>&1 || { echo "$w rc=$?"; tail -3 $O/$w.log; exit 1; }
  grep '^{' $O/$w.log > $O/${w}_attached.jsonl
  python3 -c "import json; d=json.loads(open('$O/${w}_attached.jsonl').read()); print('$w attached', 'value %.4g'%d['value'], 'ms', round(d['ms_per_step'],4), d['check']['ok'], d['resident_same_chunks'], 'cpu', d['cpu_baseline']['value'])"
done
