#!/bin/bash
# Whole -m gpu suite, smoke, the default bench line, the 1024-query batch line (+ A/B against a variant
# library when named) and rocprof stats of the default line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r02final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/gpu_tests.log | tail -20; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_n1.log 2>&1 || { echo bench failed; tail $O/bench_n1.log; exit 1; }
grep '^{' $O/bench_n1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('search', d['ms_per_step'], d['value'], d['roofline']['frac'])"
for v in hip "$@"; do
  IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$v.so timeout -k 10 300 python bench.py --workload batch --queries 1024 --steps 2 --warmup 1 > $O/batch_$v.log 2>&1 || { echo "batch $v failed"; tail $O/batch_$v.log; exit 1; }
  grep '^{' $O/batch_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch1024 $v', round(d['ms_per_step'],1), '%.4g' % d['value'], round(d['roofline']['frac'],3), d['check']['ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_search -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_search.log 2>&1 || { echo prof failed; exit 1; }
echo done
