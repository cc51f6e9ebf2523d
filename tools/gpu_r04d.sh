# round 4: MasksEngine 10M, tiles per wave 8 (shipped: 29 VGPRs spilled) vs 5 / 6 / 7 (no spills), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04d; mkdir -p $O
BENCH_ARGS="--steps 200 --warmup 5" timeout -k 10 900 bash tools/run_variants.sh masks libiris_hip.so libiris_mt6.so libiris_mt7.so libiris_mt5.so libiris_hip.so libiris_mt6.so libiris_mt7.so libiris_mt5.so libiris_hip.so libiris_mt6.so libiris_mt7.so > $O/masks.txt 2>&1 || { echo "variants rc=$?"; cat $O/masks.txt; exit 1; }
cat $O/masks.txt
BENCH_ARGS="--steps 200 --warmup 5" timeout -k 10 300 bash tools/run_variants.sh resolve-masks libiris_hip.so libiris_hip.so > $O/resolve.txt 2>&1 || { echo "variants rc=$?"; cat $O/resolve.txt; exit 1; }
cat $O/resolve.txt
