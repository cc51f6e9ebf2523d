#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
./tools/gpu_r03gg.sh && ./tools/gpu_r03ff.sh
