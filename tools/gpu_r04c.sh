# round 4: interleaved A/B on one box -- masks 10M (shipped vs T=4 / 3 workgroups per CU / query
# from L2), fused resolve-masks for both, and 20k-record device-output calls with and without the
# completion word
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04c; mkdir -p $O
BENCH_ARGS="--steps 200 --warmup 5" timeout -k 10 600 bash tools/run_variants.sh masks libiris_hip.so libiris_t4b3q0.so libiris_hip.so libiris_t4b3q0.so libiris_hip.so libiris_t4b3q0.so > $O/masks.txt 2>&1 || { echo "variants rc=$?"; cat $O/masks.txt; exit 1; }
cat $O/masks.txt
BENCH_ARGS="--steps 200 --warmup 5" timeout -k 10 600 bash tools/run_variants.sh resolve-masks libiris_hip.so libiris_t4b3q0.so libiris_hip.so libiris_t4b3q0.so > $O/resolve.txt 2>&1 || { echo "variants rc=$?"; cat $O/resolve.txt; exit 1; }
cat $O/resolve.txt
for lib in libiris_hip.so libiris_nodone.so libiris_hip.so libiris_nodone.so; do
  for w in masks shares; do
    IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/$lib timeout -k 10 200 python bench.py --workload $w --n-per-gpu 20000 --steps 500 --warmup 20 --no-cpu-baseline --reuse-engine --prewarm-s 1 > $O/c_${w}_$lib.log 2>&1 || { echo "chunk rc=$?"; tail -3 $O/c_${w}_$lib.log; exit 1; }
    grep '^{' $O/c_${w}_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w $lib', 'ms', round(d['ms_per_step']*1e3,2), 'unprof_us', round(d['ms_per_step_unprofiled']*1e3,2), 'kernel_us', round(d['kernel']['avg_ms']*1e3,2), 'ok', d['check']['ok'])"
  done
done
