# round 4: the host-slice calls' transient database kept per device (shipped) against a hipMalloc + hipFree per call
# (libiris_notc.so), participant-sized uploads and whole arrays, interleaved; parity / attach / io tests on the shipped build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_attach.py tests/test_gpu_io.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in hip notc; do
    for spec in "host-masks 20000" "host-shares 2000" "host-masks 0"; do
      set -- $spec; wl=$1; ch=$2; c=""; [ $ch != 0 ] && c="--chunk $ch"
      IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --workload $wl $c --steps 3 --warmup 1 --no-cpu-baseline > $O/${wl}_${ch}_${v}_$i.log 2>&1 || { echo "bench $wl $v rc=$?"; tail -5 $O/${wl}_${ch}_${v}_$i.log; exit 1; }
      grep '^{' $O/${wl}_${ch}_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl chunk $ch $v', 'ms_per_step', round(d['ms_per_step'],2), 'value', '%.4g'%d['value'], d['check']['ok'])"
    done
  done
done
echo all ok
