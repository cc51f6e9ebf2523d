#!/bin/bash
# rocprofv3 kernel stats of the batch (1024 queries) and TRITS search lines on the final library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_r02; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/batch -o run -- python3 bench.py --workload batch --queries 1024 --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline > $O/batch.log 2>&1 || { echo "batch prof failed"; tail $O/batch.log; exit 1; }
grep '^{' $O/batch.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch', d['kernel']['avg_ms'], d['check']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trits -o run -- python3 bench.py --layout trits --steps 20 --warmup 3 --no-cpu-baseline > $O/trits.log 2>&1 || { echo "trits prof failed"; tail $O/trits.log; exit 1; }
grep '^{' $O/trits.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('trits', d['kernel']['avg_ms'], d['check']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prepare -o run -- python3 bench.py --workload prepare --steps 5 --warmup 1 --no-cpu-baseline > $O/prepare.log 2>&1 || { echo "prepare prof failed"; tail $O/prepare.log; exit 1; }
grep '^{' $O/prepare.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prepare', d['kernel']['avg_ms'], d['check']['ok'])"
