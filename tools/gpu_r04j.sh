# round 4: same-box A/B of the round-3 library + bench (ab_r03/, built from bb10ef5) against the current tree,
# interleaved, for the resident HBM-bound workloads (kernel ms from the bench's HIP events)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04j; mkdir -p $O
run() {  # tag dir workload steps
    local tag=$1 dir=$2 w=$3 st=$4
    (cd $dir && timeout -k 10 200 python bench.py --workload $w --steps $st --warmup 5 --no-cpu-baseline) > $O/${w}_$tag.log 2>&1 || { echo "$w $tag rc=$?"; tail -3 $O/${w}_$tag.log; exit 1; }
    grep '^{' $O/${w}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w $tag kernel_ms', round(d['kernel']['avg_ms'],4), 'frac', round(d['roofline']['frac'],4), d['check']['ok'])"
}
for i in 1 2; do
  for w in masks search resolve-masks; do
    run cur . $w 200 || exit 1
    run r03 ab_r03 $w 200 || exit 1
  done
  run cur . shares 20 || exit 1
  run r03 ab_r03 shares 20 || exit 1
done
echo all ok
