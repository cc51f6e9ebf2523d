#!/bin/bash
# end-of-session tree: attach tests (incl. concurrent walks), then every bench line (tools/bench_all_r03.sh r03b)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03bb; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_attach.py -x -q --timeout 200 --timeout-method thread > $O/attach.log 2>&1 || { echo "attach tests rc=$?"; tail -30 $O/attach.log; exit 1; }
tail -1 $O/attach.log
bash tools/bench_all_r03.sh r03b
