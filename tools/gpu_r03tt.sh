#!/bin/bash
# the device-restoring entry points: the new test, then the whole GPU suite, smoke and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k keep_the_callers --timeout 60 --timeout-method thread 2>&1 | tail -3 || exit 1
./tools/gpu_r03ff.sh
