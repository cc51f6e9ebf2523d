# participant-sized call latency: default scheduling vs spin / yield
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03c; mkdir -p $O
for s in auto spin; do
  IRIS_SCHEDULE=$s timeout -k 10 200 python tools/chunk_latency.py 20000 3000 > $O/lat_$s.log 2>&1 || { echo "lat $s rc=$?"; tail -5 $O/lat_$s.log; exit 1; }
  echo "== $s"; grep -v '^{' $O/lat_$s.log
done
