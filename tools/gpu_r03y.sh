# host-row paths by destination page size, then the batched-kernel A/B (tools/gpu_r03x.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 180 ./tools/ubench_launch > $O/launch.log 2>&1 || { echo "ubench rc=$?"; tail -5 $O/launch.log; exit 1; }
grep -E "d2h|kpin|reg" $O/launch.log
timeout -k 10 600 ./tools/gpu_r03x.sh
