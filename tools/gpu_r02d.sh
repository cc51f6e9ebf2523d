set -o pipefail
for k in 2 1; do
  IRIS_BATCH_KERNEL=$k OUT=gpurun_out/r02d/pmc_k$k Q=256 bash tools/pmc_batch.sh > /dev/null 2>&1 || { echo "pmc k=$k failed"; exit 1; }
  echo "== kernel $k"; cat gpurun_out/r02d/pmc_k$k/summary.txt
done
