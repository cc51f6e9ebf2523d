#!/bin/bash
# read-ahead ordering only when the device stream is busy: correctness first, then the walks and bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_prepare.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/kk_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/kk_tests.log; exit 1; }
tail -1 gpurun_out/kk_tests.log
./tools/gpu_r03jj.sh
