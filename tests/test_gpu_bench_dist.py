"""GPU box: bench.py's multi-GPU paths end to end on the one GPU: torch.distributed.run
ranks with the gloo rehearsal exchange (2 ranks, and the driver's 8-rank run sharing the card),
the default RCCL path on one rank (library communicator via ncclCommInitRank, gloo only for the
rendezvous) and the single-process library device group (--single-process).  Each run plants a
known answer (in a later rank's shard when there are several) that must be found."""
import json
import re
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
    k = d["kernel"]  # every rank's kernel time; the roofline is the slowest one's
    assert len(k["per_rank_kernel_ms"]) == 8 and k["kernel_ms_max"] == max(k["per_rank_kernel_ms"])
    assert k["avg_ms"] == k["kernel_ms_max"] and k["kernel_ms_min"] <= k["kernel_ms_max"]


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


def test_bench_single_process_group():
    """`bench.py --single-process`: one process, a library device group over --gpus devices
    (ncclCommInitAll + the RCCL all-gather of the shard winners + on-device merge), no
    torch; here a 1-device group, for the search (pipelined) and a 9-query batch."""
    for extra in ([], ["--workload", "batch", "--queries", "9"]):
        cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--single-process", "--steps", "3", "--warmup",
               "1", "--n-per-gpu", "300000", "--no-cpu-baseline", "--prewarm-s", "0.2", *extra]
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert d["n_gpus"] == 1 and d["check"]["ok"] and d["processes"] == 1
        assert d["backend"].startswith("rccl") and "RCCL" in d["config"]["exchange"]
        assert d["value_per_gpu"] == d["value"]


def test_bench_rccl_single_rank():
    """bench.py's process-group path with the default RCCL backend on one rank: gloo for the
    rendezvous, the library's own communicator (ncclCommInitRank, id broadcast over gloo)
    for the exchange."""
    env = dict(os.environ, IRIS_FORCE_DIST="1", IRIS_DIST_BACKEND="nccl")
    for extra in ([], ["--workload", "batch", "--queries", "5"]):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
               "--steps", "3", "--warmup", "1", "--n-per-gpu", "300000", "--no-cpu-baseline", *extra]
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert d["n_gpus"] == 1 and d["check"]["ok"] and d["ranks_seen"] == 1
        assert "helper-thread ncclCommInitRank (bounded)" in d["backend"] and "RCCL" in d["config"]["exchange"]
        # the formation's wall time and bound, for the first multi-GPU record to say what ran
        assert 0 < d["group_form_s"] < d["rccl_init_timeout_ms"] / 1e3
        assert d["rccl_init_timeout_ms"] == 120000
        # what the library's communicator saw: one rank, on this box's GPU (its PCI bus id)
        assert d["rccl_nranks"] == 1 and len(d["rccl_devices"]) == 1
        assert re.fullmatch(r"[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-9a-fA-F]", d["rccl_devices"][0])


def test_bench_rccl_fallback_when_group_cannot_form():
    """Two torch.distributed.run ranks with the default RCCL backend on the box's one GPU (each
    rank told that GPU is its own): RCCL refuses two ranks on one device, every rank learns that
    over gloo, and the run still searches and exchanges its winners over gloo, saying so in the
    line (backend, rccl_error, exchange) -- the 8-GPU record is then a measured line with the
    reason, not a missing one.  IRIS_RCCL_FALLBACK=0 turns the refusal into an error exit."""
    base = dict(os.environ, HIP_VISIBLE_DEVICES="0", IRIS_GROUP_TIMEOUT_MS="30000")
    base.pop("IRIS_DIST_BACKEND", None)

    def run(env):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
               "--gpus", "2", "--steps", "2", "--warmup", "1", "--n-per-gpu", "200000", "--no-cpu-baseline",
               "--prewarm-s", "0"]
        return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)

    r = run(base)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["check"]["ok"]
    assert d["check"]["planted_index"] >= 200000  # found in rank 1's shard, over the gloo exchange
    assert "fallback" in d["backend"] and d["rccl_error"] and d["rccl_nranks"] is None
    assert d["config"]["exchange"].endswith("(fallback)")

    r = run(dict(base, IRIS_RCCL_FALLBACK="0"))
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "did not form" in r.stderr
