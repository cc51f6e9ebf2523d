# round 4: the group / hooks changes first (group, attach, io, fuzz), then the whole GPU suite and smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread > $O/group.log 2>&1 || { echo "group rc=$?"; tail -40 $O/group.log; exit 1; }
tail -3 $O/group.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
