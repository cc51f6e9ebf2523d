# round 4: persistent search kernel -- parity (new test + the whole -m gpu suite), then interleaved search timing:
# shipped (persistent, static units) vs one workgroup per 16 tiles (IRIS_SEARCH_DYN=0) vs dynamic units (=2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "persistent or large_search or async" > $O/new.log 2>&1 || { echo "new tests rc=$?"; tail -30 $O/new.log; exit 1; }
tail -2 $O/new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in hip nodyn dyn2; do
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline > $O/search_${v}_$i.log 2>&1 || { echo "bench $v rc=$?"; tail -3 $O/search_${v}_$i.log; exit 1; }
    grep '^{' $O/search_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('search $v', 'kernel_ms', round(d['kernel']['avg_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
  done
done
