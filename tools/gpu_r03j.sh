set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for spec in agent:libiris_hip.so system:libiris_fusedsys.so agent2:libiris_hip.so; do
  IFS=: read label lib <<< "$spec"
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -k 10 200 python tools/chunk_latency.py 20000 3000 > $O/lat_$label.log 2>&1 || { echo "lat $label rc=$?"; tail -5 $O/lat_$label.log; exit 1; }
  echo "== $label"; grep '^search' $O/lat_$label.log
done
