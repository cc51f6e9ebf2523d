#!/bin/bash
# round-3 PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of every bench workload's kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/pmc
WORKLOADS="search masks shares resolver resolve-masks batch" ./tools/pmc_traffic.sh || exit 1
find gpurun_out/pmc -name '*.csv' ! -name '*counter_collection.csv' -delete
du -sh gpurun_out/pmc
