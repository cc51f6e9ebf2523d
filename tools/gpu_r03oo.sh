#!/bin/bash
# share preparation: clock and busy cycles of the shipped kernel vs its no-store / no-ChaCha diagnostic builds,
# and the SDWA rot16 variant (IRIS_PREP_SDWA=1) interleaved with the shipped one
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03oo; rm -rf $O; mkdir -p $O
for spec in ship:libiris_hip.so nostore:libiris_prepnost.so nochacha:libiris_prepnocc.so sdwa:libiris_prepsdwa.so; do
  IFS=: read label lib <<< "$spec"
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -k 10 200 python bench.py --workload prepare --steps 10 --warmup 1 --prewarm-s 1 --no-cpu-baseline > $O/$label.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "$label rc=$rc"; tail -3 $O/$label.log; exit 1; fi
  grep '^{' $O/$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['kernel']['avg_ms'],3), d['check']['ok'])"
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $O/pmc_$label -o run -- python3 bench.py --workload prepare --steps 3 --warmup 1 --prewarm-s 1 --no-cpu-baseline > $O/pmc_$label.log 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "pmc $label rc=$rc"; tail -3 $O/pmc_$label.log; exit 1; fi
done
for spec in ship2:libiris_hip.so sdwa2:libiris_prepsdwa.so ship3:libiris_hip.so sdwa3:libiris_prepsdwa.so; do
  IFS=: read label lib <<< "$spec"
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -k 10 200 python bench.py --workload prepare --steps 10 --warmup 1 --prewarm-s 1 --no-cpu-baseline > $O/$label.log 2>&1 || { echo "$label rc=$?"; tail -3 $O/$label.log; exit 1; }
  grep '^{' $O/$label.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', round(d['kernel']['avg_ms'],3), d['check']['ok'])"
done
python3 - $O <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for label in ("ship", "nostore", "nochacha", "sdwa"):
    by = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
    for f in glob.glob(f"{out}/pmc_{label}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "prepare_direct_kernel" in r["Kernel_Name"]:
                d = r["Dispatch_Id"]
                by[d][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
    for d in sorted(by, key=int)[-2:]:
        c = by[d]; t = dur[d]
        print(f"{label:9s} dispatch {d}: {t*1e3:.2f} ms  clock {c['GRBM_GUI_ACTIVE']/8/t/1e9:.3f} GHz  "
              f"SQ_BUSY/GRBM {c['SQ_BUSY_CYCLES']/c['GRBM_GUI_ACTIVE']:.3f}  VALU {c['SQ_INSTS_VALU']:.4g}  "
              + "  ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
PY
IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_prepsdwa.so timeout -k 10 300 python -u -m pytest tests/test_gpu_prepare.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/sdwa_tests.log 2>&1 || { echo "sdwa tests rc=$?"; tail -5 $O/sdwa_tests.log; exit 1; }
tail -1 $O/sdwa_tests.log
