#!/bin/bash
# package power and clocks (amd-smi metric, polled) while the batched, share-preparation and search kernels run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03qq; rm -rf $O; mkdir -p $O
timeout 30 amd-smi metric -g 0 -p -c > $O/idle.txt 2>&1 || { echo "amd-smi failed"; tail -5 $O/idle.txt; exit 1; }
cat $O/idle.txt
for w in batch prepare search; do
  args="--steps 4 --warmup 1 --prewarm-s 3"
  [ $w = batch ] && args="--queries 1024 --steps 4 --warmup 1 --prewarm-s 0.5"
  [ $w = prepare ] && args="--steps 200 --warmup 1 --prewarm-s 3"
  [ $w = search ] && args="--steps 400 --warmup 1 --prewarm-s 6"
  timeout -k 10 200 python bench.py --workload $w $args --no-cpu-baseline > $O/$w.log 2>&1 &
  pid=$!
  while kill -0 $pid 2>/dev/null; do
    echo "T $(date +%s.%N)" >> $O/$w.pwr
    timeout 5 amd-smi metric -g 0 -p -c >> $O/$w.pwr 2>&1
    sleep 0.2
  done
  wait $pid || { echo "$w rc=$?"; tail -3 $O/$w.log; exit 1; }
  echo "$w done"; grep '^{' $O/$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w kernel_ms', round(d['kernel']['avg_ms'],3), d['check']['ok'])"
done
