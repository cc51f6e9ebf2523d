# round 4: large database reads through the pinned slots (shipped) against the runtime's copy into the pageable array
# (libiris_rtread.so), interleaved; the parity / io / attach tests (which read back everything) on the shipped build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04af; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_io.py tests/test_gpu_attach.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in hip rtread; do
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python tools/read_paths.py $v >> $O/read_paths.txt 2>&1 || { echo "read $v rc=$?"; tail -5 $O/read_paths.txt; exit 1; }
  done
done
cat $O/read_paths.txt
echo all ok
