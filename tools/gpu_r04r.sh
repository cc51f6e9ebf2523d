# round 4: persistent search with workgroup units kept in step (IRIS_SEARCH_DYN=4) and one 8-wave workgroup per CU
# (IRIS_SEARCH_WG_WAVES=8): oracle tests, then timing
# the large-range oracle tests on every variant, then interleaved timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04r; mkdir -p $O
for v in wg w8; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "persistent or large_search" > $O/tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -20 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
for i in 1 2; do
  for v in hip wg w8; do
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline > $O/search_${v}_$i.log 2>&1 || { echo "bench $v rc=$?"; tail -3 $O/search_${v}_$i.log; exit 1; }
    grep '^{' $O/search_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('search $v', 'kernel_ms', round(d['kernel']['avg_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
  done
done
