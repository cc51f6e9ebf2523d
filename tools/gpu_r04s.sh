# round 4: the final tree -- the whole -m gpu suite and smoke(); the large-range oracle tests on the two last
# search variants (workgroup units kept in step, IRIS_SEARCH_DYN=4; one 8-wave workgroup per CU,
# IRIS_SEARCH_WG_WAVES=8) and their timing against the shipped grid; the default bench line with rocprof stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
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
timeout -k 10 300 python bench.py > $O/default.log 2>&1 || { echo "default bench rc=$?"; tail -5 $O/default.log; exit 1; }
grep '^{' $O/default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], 'kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],4), 'cpu', d['cpu_baseline']['value'], d['check']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo all ok
