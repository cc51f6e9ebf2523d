# rocprofv3 kernel durations of participant-sized calls (GPU begin -> end, no HIP-event bracket):
# search 10k / 20k with the fused tail and with the separate reduce, masks 10k / 20k
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03o; mkdir -p $O
for n in 10000 20000; do
  for mode in fused sep; do
    f=1; [ $mode = sep ] && f=0
    IRIS_FUSED_REDUCE=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${mode}_$n -o run -- python3 tools/chunk_latency.py $n 500 > $O/${mode}_$n.log 2>&1 || { echo "prof $mode $n rc=$?"; tail -5 $O/${mode}_$n.log; exit 1; }
    s=$(find /tmp/prof_${mode}_$n -name "*kernel_stats.csv" | head -1)
    cp "$s" $O/${mode}_${n}_kernel_stats.csv
    python3 -c "
import csv,sys
for r in csv.DictReader(open('$s')):
    print('$mode $n', r['Name'][:70].ljust(70), r['Calls'], r['AverageNs'], r['MinNs'])
"
  done
done
