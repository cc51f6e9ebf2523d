#!/bin/bash
# robustness: the whole GPU suite with the opt-in TRITS tests, then the attach / read-ahead tests once more
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ii; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_prepare.py -x -q --timeout 200 --timeout-method thread > $O/first.log 2>&1 || { echo "first rc=$?"; tail -30 $O/first.log; exit 1; }
tail -1 $O/first.log
IRIS_TEST_TRITS=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py -x -q --timeout 200 --timeout-method thread > $O/attach.log 2>&1 || { echo "attach rc=$?"; tail -30 $O/attach.log; exit 1; }
tail -1 $O/attach.log
