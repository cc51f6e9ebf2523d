"""CPU: bench.py's launcher contract.  `python bench.py --gpus N` without torchrun must
start N ranks itself and print ONE line with n_gpus == N (gloo dry run: rendezvous,
world-size check, all-gather + merge of a per-rank result, max-over-ranks timing, no GPU);
a request for more RCCL ranks than visible GPUs must fail loudly; a launcher whose
WORLD_SIZE disagrees with --gpus must fail.  Also the planted-answer placement."""
import json
import os
import pathlib
import socket
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [2, 3, 8])  # 8: the driver's scaling run, rehearsed on gloo
def test_self_launch_dry_run(n):
    env = dict(os.environ, IRIS_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--dry-run"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == n and d["ranks_seen"] == n and d["backend"] == "gloo"
    assert d["launcher"].startswith("bench.py") and d["dry_run"] and d["check"]["ok"]
    assert d["check"]["merged_index"] == 7  # equal distances: the lowest global index (rank 0) wins
    assert d["check"]["gathered_ranks"] == list(range(n))  # every rank's entry, in rank order


def test_too_many_rccl_ranks_fail_loudly():
    """--gpus 8 with the RCCL backend and fewer visible GPUs (none here) -> rc != 0, no line."""
    env = dict(os.environ)
    env.pop("IRIS_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert _lines(r.stdout) == []
    assert "visible" in r.stderr


def test_world_size_mismatch_fails():
    """torchrun with 2 ranks but --gpus 3: every rank refuses."""
    env = dict(os.environ, IRIS_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"), "--gpus", "3", "--dry-run"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert _lines(r.stdout) == []


def test_torchrun_launch_dry_run():
    """The driver's form: torch.distributed.run --nproc-per-node 2 bench.py --gpus 2."""
    env = dict(os.environ, IRIS_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"), "--gpus", "2", "--dry-run"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _lines(r.stdout)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["launcher"] == "torch.distributed.run"


def test_plant_sites_inside_database():
    import bench

    for total in (1, 2, 5, 100, 20_000, 49_000, 400_000, 10_000_000, 100_000_000):
        for count in (1, 4, 5):
            s = bench.plant_sites(total, count)
            assert len(s) == min(count, total) and len(set(s)) == len(s)
            assert all(0 <= x < total for x in s)
    # the single-query site of round 1 is kept where it fitted (10M: 7 512 345)
    assert bench.plant_sites(10_000_000, 1) == [7_512_345]
    # with 2+ ranks the first site lies in a later rank's shard
    assert bench.plant_sites(400_000, 1)[0] >= 200_000


def test_batch_plants_span_query_groups():
    import bench

    q = bench.batch_plant_queries(1024)
    assert len({x // 4 for x in q}) >= 4 and 0 in q and 1023 in q and 512 in q
    assert bench.batch_plant_queries(1) == [0]
    assert all(0 <= x < 9 for x in bench.batch_plant_queries(9))
