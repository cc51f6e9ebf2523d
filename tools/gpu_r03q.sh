# host-row output paths for participant-sized calls (1.24 MB of [20000][31] u16)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 120 ./tools/ubench_launch > $O/launch.log 2>&1 || { echo "ubench rc=$?"; tail -5 $O/launch.log; exit 1; }
cat $O/launch.log
