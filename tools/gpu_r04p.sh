# round 4: search kernel forms, interleaved on one box: one workgroup per 16 tiles (shipped) vs persistent grids with
# units from a work counter of 1 / 2 / 4 / 8 sub-units of 4 tiles (IRIS_SEARCH_DYN=2, IRIS_SEARCH_UNIT=H)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04p; mkdir -p $O
for i in 1 2; do
  for v in ${VARIANTS:-hip dyn2 d2h2 d2h4 d2h8}; do
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline > $O/search_${v}_$i.log 2>&1 || { echo "bench $v rc=$?"; tail -3 $O/search_${v}_$i.log; exit 1; }
    grep '^{' $O/search_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('search $v', 'kernel_ms', round(d['kernel']['avg_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
  done
done
