# round 4: upload path by record source (tools/upload_sources.py), and the attached 20k-record masks walk with the
# upload pinned either way (the attach uploads through it once; the walk itself uploads nothing)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 400 python tools/upload_sources.py /tmp/r04x > $O/upload_sources.txt 2>&1 || { echo "sources rc=$?"; tail -5 $O/upload_sources.txt; exit 1; }
cat $O/upload_sources.txt
for i in 1 2; do
  for v in auto runtime; do
    hk=""; [ $v = runtime ] && hk="IRIS_TEST_HOOKS=1 IRIS_UPLOAD=runtime"
    env $hk timeout -k 10 200 python bench.py --workload host-masks --attached --steps 3 --warmup 1 --no-cpu-baseline > $O/att_${v}_$i.log 2>&1 || { echo "att $v rc=$?"; tail -5 $O/att_${v}_$i.log; exit 1; }
    grep '^{' $O/att_${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['resident_same_chunks']; print('attached $v', 'ms_per_step', round(d['ms_per_step'],3), 'vs host_out', round(r['attached_vs_host_out'],3), 'vs device_out', round(r['attached_vs_device_out'],3), d['check']['ok'], d['host_pages_numa'])"
  done
done
echo all ok
