#!/bin/bash
# pooled read-ahead row buffers: attach + parity tests, walk timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03cc; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/ra_diag.py masks 2000000 3 > $O/diag_masks.log 2>&1 && cat $O/diag_masks.log
timeout -k 10 120 python tools/ra_diag.py shares 200000 3 > $O/diag_shares.log 2>&1 && cat $O/diag_shares.log
