# round 4: why the non-attached host-slice masks call moves 29 GB/s while the shares call moves 53 GB/s --
# kernel + memory-copy traces of both bench workloads, the box's host memcpy rate, and the host-output
# rows stored straight into pinned buffers (shipped now) against the copy-engine D2H (libiris_d2h.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_io.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in hip d2h; do
    for wl in host-masks host-shares; do
      IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || { echo "bench $wl $v rc=$?"; tail -5 $O/${wl}_${v}_$i.log; exit 1; }
      grep '^{' $O/${wl}_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $v', 'ms_per_step', round(d['ms_per_step'],2), 'GBps', round(d['host_input_GBps'],1), d['check']['ok'])"
    done
  done
done
for v in hip d2h; do
  IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --workload host-masks --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { echo "prof $v rc=$?"; tail -5 $O/prof_$v.log; exit 1; }
done
timeout -k 10 120 python3 - > $O/memcpy.log 2>&1 <<'EOF' || { echo "memcpy rc=$?"; exit 1; }
import numpy as np, time
for shape, dt in (((2_000_000, 200), np.uint64), ((200_000, 12800), np.uint16)):
    a = np.random.default_rng(1).integers(0, 2**16, shape).astype(dt)
    b = np.empty_like(a)
    for i in range(3):
        t = time.perf_counter(); np.copyto(b, a); dt_ = time.perf_counter() - t
        print(shape, 'numpy copy (1 thread)', round(a.nbytes / dt_ / 1e9, 1), 'GB/s')
EOF
cat $O/memcpy.log
find $O -name "*memory_copy_stats.csv" -o -name "*kernel_stats.csv" | sort | while read f; do echo "== $f"; head -12 "$f"; done
echo all ok
