# round 4: row-packed batch kernel (IRIS_BATCH_KERNEL 5) -- parity tests, then interleaved kernel time + PMC
# clock/MFMA busy against the shipped kernel 4, then the MFMA power micro-benchmark modes (tools/gpu_r04g.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -k "batch_rows or row_packing" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 900 bash tools/batch_variants.sh 1024 ship4:libiris_hip.so:4 rows5:libiris_hip.so:5 ship4b:libiris_hip.so:4 rows5b:libiris_hip.so:5 || exit 1
timeout -k 10 300 bash tools/gpu_r04g.sh || exit 1
