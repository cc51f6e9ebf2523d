#!/bin/bash
# the opt-in TRITS layout tests on the final tree (IRIS_TEST_TRITS=1), and the extended-size GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03uu; rm -rf $O; mkdir -p $O
IRIS_TEST_TRITS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "trits" --timeout 300 --timeout-method thread > $O/trits.log 2>&1 || { echo "trits rc=$?"; tail -20 $O/trits.log; exit 1; }
tail -1 $O/trits.log
