# round 4: the pinned upload slots' size and count (64 MB x 2 shipped; 128 x 2, 64 x 3, 32 x 4 variants), host-masks
# and load, interleaved on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04aa; mkdir -p $O
for i in 1 2; do
  for v in hip s128 s3 s32x4; do
    for wl in host-masks load; do
      IRIS_HIP_LIB=$PWD/mpc-iris-code_amd/libiris_$v.so timeout -k 10 200 python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || { echo "bench $wl $v rc=$?"; tail -5 $O/${wl}_${v}_$i.log; exit 1; }
      grep '^{' $O/${wl}_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $v', 'ms_per_step', round(d['ms_per_step'],2), d['check']['ok'])"
    done
  done
done
echo all ok
