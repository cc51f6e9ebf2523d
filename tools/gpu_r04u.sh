# round 4 (r04u, then r04v with the page-node choice): non-attached host-slice calls -- large database writes through two pinned slots filled by
# the helper threads (shipped now) against the runtime's staging of pageable copies (libiris_rt.so:
# pinned rows only; libiris_d2h.so: neither), host-masks and host-shares interleaved, and with 7
# copy helpers; NUMA layout of the box for the record
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04v; mkdir -p $O
{ for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus $(cat $n/cpulist)"; done
  for c in /sys/class/drm/card*/device/numa_node; do echo "$c $(cat $c)"; done
  grep -E "Cpus_allowed_list" /proc/self/status; nproc; } > $O/numa.txt 2>&1
cat $O/numa.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_attach.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_io.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in auto pinned runtime d2h; do
    lib=hip; hk=""; [ $v = d2h ] && lib=d2h; [ $v = pinned ] && hk="IRIS_TEST_HOOKS=1 IRIS_UPLOAD=pinned"; [ $v = runtime ] && hk="IRIS_TEST_HOOKS=1 IRIS_UPLOAD=runtime"
    for wl in host-masks host-shares; do
      env $hk IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$lib.so timeout -k 10 200 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || { echo "bench $wl $v rc=$?"; tail -5 $O/${wl}_${v}_$i.log; exit 1; }
      grep '^{' $O/${wl}_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $v', 'ms_per_step', round(d['ms_per_step'],2), 'GBps', round(d['host_input_GBps'],1), d['check']['ok'], d['host_pages_numa'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_hip -o run -- python3 bench.py --workload host-masks --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_hip.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof_hip.log; exit 1; }
echo all ok
