set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/batch_variants.sh 1024 "ship:libiris_hip.so:4" "nostag:libiris_nostag.so:4" "noroll:libiris_noroll.so:4" "ship2:libiris_hip.so:4" "r02:libiris_hip.so:2"
