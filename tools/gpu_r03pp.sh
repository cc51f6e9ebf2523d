#!/bin/bash
# batched kernel <8,2,2,2> energy decomposition: time, clock, MFMA busy of the shipped kernel and of its diagnostic
# builds (2 no LDS fragment reads, 3 no B loads, 4 no A loads/expansion, 5 no MFMAs, 6 B expansion for one chunk pair only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
./tools/batch_variants.sh 1024 ship:libiris_hip.so:4 d6:libiris_bd6.so:4 d2:libiris_bd2.so:4 d3:libiris_bd3.so:4 d4:libiris_bd4.so:4 d5:libiris_bd5.so:4 ship2:libiris_hip.so:4
