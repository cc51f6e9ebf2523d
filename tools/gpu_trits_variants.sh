#!/bin/bash
# TRITS parity tests, then interleaved search benches: TILES, TRITS (shipped) and the
# variant libraries named on the command line (mpc-iris-code_amd/libiris_<name>.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/trits_var
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trits.py -x -q --timeout 200 --timeout-method thread \
    > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
run() {  # label layout [lib]
  local lib=${3:+mpc-iris-code_amd/libiris_$3.so}
  IRIS_HIP_LIB=${lib:-mpc-iris-code_amd/libiris_hip.so} timeout -k 10 120 python bench.py --layout $2 --steps 100 \
      --warmup 5 --prewarm-s 1 --no-cpu-baseline > $out/$1.json 2>> $out/bench.err \
      || { echo "bench $1 failed"; tail $out/bench.err; exit 1; }
  python3 -c "import json,sys; j=json.load(open('$out/$1.json')); print('%-10s'%'$1', round(j['ms_per_step'],3), 'kernel', round(j['kernel']['avg_ms'],3), 'value %.3e'%j['value'], j['check']['ok'])"
}
for r in 1 2; do
  run tiles$r tiles || exit 1
  run trits$r trits || exit 1
  for v in "$@"; do run ${v}$r trits $v || exit 1; done
done
