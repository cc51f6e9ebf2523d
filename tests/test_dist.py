"""CPU: the multi-GPU path's exchange step, rehearsed with the gloo backend at
world_size 2.  Each rank searches its contiguous shard (here with the CPU
oracle standing in for the GPU kernel, since this runs without a GPU), then
all ranks all-gather their 32-byte iris_match_t records and merge them with
the library's native iris_match_merge — exactly what bench.py does over RCCL."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, seed, q, plants, result_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
    import iris_dist
    import iris_hip as ih
    from oracle import oracle_c as oc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = iris_dist.shard_range(n, rank, world)
    db = oc.gen_templates(seed, lo, hi - lo)
    for dst, src in plants:  # copies of record src planted at global index dst
        if lo <= dst < hi:
            db[dst - lo] = oc.gen_templates(seed, src, 1)[0]
    d = oc.template_distances(q, db, threads=1)
    best, idx = oc.argmin(d)
    if idx != 2**64 - 1:
        num, den = oc.template_counts(q, db[idx:idx + 1], threads=1)
        k = min(range(31), key=lambda k: (num[0, k] / den[0, k]) if den[0, k] else np.inf)
        local = ih.Match(best, lo + idx, int(num[0, k]), int(den[0, k]), k - 15, 0)
    else:
        local = ih.Match(float("inf"), 2**64 - 1, 0, 0, 0, 0)
    merged = iris_dist.allgather_merge(local)
    # the batched form: one all-gather of every query's Match
    inf = ih.Match(float("inf"), 2**64 - 1, 0, 0, 0, 0)
    ranked = ih.Match(0.5 - 0.1 * rank, lo, 5 - rank, 10, 0, 0)
    many = iris_dist.allgather_merge_many([local, inf, ranked])
    if rank == 0:
        np.save(result_path, np.array([merged.distance, float(merged.index), merged.num, merged.den,
                                       many[0].distance, float(many[0].index), many[1].distance,
                                       float(many[1].index), many[2].distance, float(many[2].index)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_shard_merge(tmp_path, world):
    sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
    import iris_dist
    from oracle import oracle_c as oc

    n, seed = 3000, 77
    full = oc.gen_templates(seed, 0, n)
    q = full[1234].copy()
    q[:200] ^= np.uint64(1)  # near-duplicate of 1234
    # plant a second, equal-distance copy of 1234 in the LAST shard, so the global minimum
    # is tied across shards and only the lowest-index rule (src/main.rs:616-621, strict <
    # in a sequential scan) applied by iris_match_merge picks 1234
    plants = [(2500, 1234)]
    full[2500] = full[1234]
    d_full = oc.template_distances(q, full)
    spans = [iris_dist.shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] <= 1234 < spans[0][1] and spans[-1][0] <= 2500 < spans[-1][1]
    shard_min = [oc.argmin(d_full[lo:hi]) for lo, hi in spans]
    assert shard_min[0][0] == shard_min[-1][0]  # a real cross-shard tie
    assert shard_min[-1][1] + spans[-1][0] == 2500
    result = tmp_path / "r.npy"
    mp.spawn(_worker, args=(world, _free_port(), n, seed, q, plants, str(result)), nprocs=world, join=True)
    got = np.load(result)
    want_d, want_i = oc.argmin(d_full)
    assert want_i == 1234
    assert got[0] == want_d and int(got[1]) == want_i
    assert got[4] == got[0] and got[5] == got[1]              # batched merge == single merge
    assert got[6] == np.inf and got[7] == float(2**64 - 1)     # no candidate on any rank
    last_lo = iris_dist.shard_range(n, world - 1, world)[0]
    assert np.isclose(got[8], 0.5 - 0.1 * (world - 1)) and int(got[9]) == last_lo
    # shards tile the range exactly
    spans = [iris_dist.shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_shard_range_ragged():
    sys.path.insert(0, str(ROOT / "mpc-iris-code_amd"))
    import iris_dist

    for n in (0, 1, 63, 64, 65, 100_000_000):
        for world in (1, 2, 3, 8):
            spans = [iris_dist.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert sum(h - l for l, h in spans) == n
            assert all(l <= h for l, h in spans)
