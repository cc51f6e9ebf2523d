set -o pipefail
for w in search masks shares batch resolver resolve-masks prepare load host-shares host-masks; do
  extra="--steps 3 --warmup 1"
  [ $w = batch ] && extra="--steps 1 --warmup 1 --queries 64"
  timeout -k 10 300 python bench.py --workload $w $extra --no-cpu-baseline > gpurun_out/allw_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc $(grep '^{' gpurun_out/allw_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["check"])')"
  [ $rc -ne 0 ] && [ $rc -ne 3 ] && exit $rc
done
exit 0
