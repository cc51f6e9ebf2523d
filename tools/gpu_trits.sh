#!/bin/bash
# TRITS layout: GPU parity tests, then search bench in both layouts (same box), then kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/trits
timeout -k 10 400 python -u -m pytest tests/test_gpu_trits.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/trits/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/trits/tests.log; exit 1; }
tail -3 gpurun_out/trits/tests.log
for lay in tiles trits tiles trits; do
  timeout -k 10 120 python bench.py --layout $lay --steps 50 --warmup 5 --no-cpu-baseline \
      >> gpurun_out/trits/bench.jsonl 2>> gpurun_out/trits/bench.err || { echo "bench $lay failed"; tail gpurun_out/trits/bench.err; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/trits/bench.jsonl"):
    j = json.loads(l)
    print(j["config"]["layout"], round(j["ms_per_step"], 3), "kernel", round(j["kernel"]["avg_ms"], 3),
          "value %.3e" % j["value"], "frac", round(j["roofline"]["frac"], 3), j["check"]["ok"])
PY
