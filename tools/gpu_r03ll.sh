#!/bin/bash
# search at 10M: 4 tiles per wave (shipped) vs 1 tile per wave (IRIS_TILES_PER_WAVE=1: 4x the waves, a 4x shorter drain)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ll; mkdir -p $O
for r in 1 2; do
for tpw in 4 1; do
  IRIS_TILES_PER_WAVE=$tpw timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --prewarm-s 2 > $O/s_${tpw}_$r.log 2>&1 || { echo "bench rc=$?"; tail -3 $O/s_${tpw}_$r.log; exit 1; }
  grep '^{' $O/s_${tpw}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tpw $tpw r$r kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
done
done
