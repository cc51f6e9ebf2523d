"""GPU box: bench.py's multi-rank path end to end (torch.distributed.run, 2 ranks on
the one GPU, gloo exchange): each rank generates its shard, searches it, the ranks
all-gather and merge their minima, and rank 0 prints one JSON line whose planted
known answer (in rank 1's shard) must be found.  The 8-GPU RCCL run is the driver's;
this rehearses the same code with the exchange on CPU tensors."""
import json
import os
import pathlib
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("workload", ["search", "batch"])
def test_bench_two_ranks(workload):
    env = dict(os.environ, IRIS_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--n-per-gpu", "200000", "--no-cpu-baseline",
           "--workload", workload, "--queries", "8"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["check"]["ok"]
    assert d["config"]["total_templates"] == 400000
    assert d["ranks_seen"] == 2 and d["backend"] == "gloo"
    found = [d["check"]] if workload == "search" else d["check"]["planted_queries"]
    assert found[0]["planted_index"] >= 200000  # the first answer lives in rank 1's shard
    if workload == "batch":
        assert len(found) == 4 and len(d["check"]["query_groups"]) >= 2


def test_bench_eight_ranks_one_gpu():
    """The driver's 8-GPU scaling run rehearsed on the one GPU: `python bench.py --gpus 8`
    (self-launched, 8 ranks sharing the card over gloo, 200k templates each) prints one line
    with n_gpus 8 whose planted answer lies in a later rank's shard."""
    env = dict(os.environ, IRIS_DIST_BACKEND="gloo")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
           "--n-per-gpu", "200000", "--no-cpu-baseline", "--prewarm-s", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["ranks_seen"] == 8 and d["backend"] == "gloo" and d["check"]["ok"]
    assert d["config"]["total_templates"] == 1_600_000
    assert d["check"]["planted_index"] >= 200000


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` with no launcher starts both ranks itself (here on the one
    GPU, gloo exchange) and prints one line with n_gpus 2."""
    env = dict(os.environ, IRIS_DIST_BACKEND="gloo")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--n-per-gpu",
           "200000", "--no-cpu-baseline", "--prewarm-s", "0.2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["check"]["ok"]
    assert d["launcher"].startswith("bench.py")


def test_bench_more_gpus_than_visible_fails():
    """`python bench.py --gpus 8` on a one-GPU box (RCCL backend) refuses instead of
    printing a one-GPU line."""
    env = dict(os.environ)
    env.pop("IRIS_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--steps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_rccl_exchange_single_rank():
    """The RCCL form of the exchange (all_gather_into_tensor on device tensors) on a
    one-rank "nccl" process group: the code path the 8-GPU run takes."""
    code = f"""
import os, sys
sys.path[:0] = [{str(ROOT)!r}, {str(ROOT / 'mpc-iris-code_amd')!r}]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="{_free_port()}")
import torch, torch.distributed as dist
import iris_hip as ih, iris_dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
m = ih.Match(0.25, 1234, 5, 20, -3, 0)
r = iris_dist.allgather_merge(m, device="cuda:0")
assert (r.index, r.num, r.den, r.rotation) == (1234, 5, 20, -3) and r.distance == 0.25, r
dist.destroy_process_group()
print("rccl ok")
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout + r.stderr[-3000:]


def test_bench_rccl_single_rank():
    """bench.py's process-group path with the default "nccl" (RCCL) backend on one rank."""
    env = dict(os.environ, IRIS_FORCE_DIST="1", IRIS_DIST_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--steps", "3", "--warmup", "1", "--n-per-gpu", "300000", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["check"]["ok"]
