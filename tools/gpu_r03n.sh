# small-range search: K-split with 2 tiles per workgroup + two-level ticket (shipped) vs 1 tile
# per workgroup, vs a 3-deep ring; masks K-split; unprofiled call time vs kernel time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for lib in hip splitT1 splitS3; do
  for n in 10000 20000; do
    IRIS_HIP_LIB=mpc-iris-code_amd/libiris_$lib.so timeout -k 10 120 python tools/chunk_latency.py $n 2000 > $O/lat_${lib}_${n}_$r.log 2>&1 || { echo "lat $lib rc=$?"; tail -3 $O/lat_${lib}_${n}_$r.log; exit 1; }
    echo "$lib n=$n r=$r"; grep -E "^(search|masks-dev) " $O/lat_${lib}_${n}_$r.log | cut -c1-160
  done
done
done
timeout -k 10 120 ./tools/call_overhead > $O/overhead.log 2>&1 || { echo "overhead rc=$?"; tail -5 $O/overhead.log; exit 1; }
cat $O/overhead.log
