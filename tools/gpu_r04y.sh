# round 4: file loads through two pinned slots the helper threads fill from the mapping (shipped now) against the
# DMA from registered page-cache windows (libiris_regload.so), interleaved; the load / io / group / attach tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_io.py tests/test_gpu_group.py tests/test_gpu_attach.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in hip regload; do
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --workload load --steps 3 --warmup 1 --no-cpu-baseline > $O/load_${v}_$i.log 2>&1 || { echo "load $v rc=$?"; tail -5 $O/load_${v}_$i.log; exit 1; }
    grep '^{' $O/load_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('load $v', 'ms_per_step', round(d['ms_per_step'],2), 'value', '%.4g'%d['value'], 'file_GBps', d.get('file_GBps'), d['check']['ok'])"
  done
done
python3 tools/keep_bench.py $O/kept_load.jsonl $O/load_hip_2.log > /dev/null || { echo "load check failed"; exit 1; }
echo all ok
