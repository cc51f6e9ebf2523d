# round 3: device groups (RCCL), host attachment, bench modes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_attach.py -x -v --timeout 120 --timeout-method thread > $O/tests_new.log 2>&1 || { echo "new tests rc=$?"; tail -40 $O/tests_new.log; exit 1; }
tail -3 $O/tests_new.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_dist.py -x -v --timeout 200 --timeout-method thread > $O/tests_dist.log 2>&1 || { echo "dist tests rc=$?"; tail -40 $O/tests_dist.log; exit 1; }
tail -3 $O/tests_dist.log
for m in masks shares; do
  timeout -k 10 300 python bench.py --workload host-$m --attached --steps 3 --warmup 1 --no-cpu-baseline --prewarm-s 1 > $O/host_${m}_att.log 2>&1 || { echo "host-$m rc=$?"; tail -5 $O/host_${m}_att.log; exit 1; }
  grep '^{' $O/host_${m}_att.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d['kernel']['avg_ms'], d.get('resident_same_chunks'), d['check'])"
done
timeout -k 10 300 python bench.py --gpus 1 --single-process --no-cpu-baseline > $O/single.log 2>&1 || { echo "single rc=$?"; tail -5 $O/single.log; exit 1; }
grep '^{' $O/single.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('single', d['value'], d['ms_per_step'], d['kernel']['avg_ms'], d['roofline']['frac'], d['check']['ok'])"
