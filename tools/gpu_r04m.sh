# round 4: tools/ubench_rw with chip-wide time-slotted writes (mode 5) against burst / trickle / read-only
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 tools/ubench_rw > $O/rw.txt 2>&1 || { echo "ubench rc=$?"; tail -5 $O/rw.txt; exit 1; }
cat $O/rw.txt
