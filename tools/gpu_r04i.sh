# round 4: where the batched kernel's extra energy goes -- the shipped kernel against diagnostic builds with
# the query-tile (A) stream L2-hot (d7) and the template (B) stream L2-hot (d8), same box, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 bash tools/batch_variants.sh 1024 ship:libiris_hip.so:4 d7:libiris_d7.so:4 d8:libiris_d8.so:4 ship2:libiris_hip.so:4 d7b:libiris_d7.so:4 d8b:libiris_d8.so:4 || exit 1
