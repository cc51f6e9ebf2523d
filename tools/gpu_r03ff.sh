#!/bin/bash
# the committed tree as the driver runs it: GPU suite, smoke, default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ff; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.log').read().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['check']['ok'], (d['cpu_baseline'] or {}).get('value'))"
