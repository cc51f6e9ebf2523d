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
    assert d["check"]["planted_index"] >= 200000  # the answer lives in rank 1's shard
