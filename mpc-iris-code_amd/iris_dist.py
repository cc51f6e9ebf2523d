"""iris_dist — the CPU (gloo) rehearsal of the multi-GPU exchange.

The product exchange is the library's own: a device group (iris_group_*,
csrc/iris_group.hip) all-gathers the 24-byte per-shard winners with RCCL and merges
them on every device.  This module is what bench.py's IRIS_DIST_BACKEND=gloo
rehearsal and the world_size-2 CPU tests use instead (several ranks may share one
GPU, which an RCCL communicator refuses): one torch.distributed all-gather over gloo
of every rank's 32-byte iris_match_t, merged by the native iris_match_merge (min
fraction, then lowest global index — the resolver's rule, src/main.rs:616-621).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

import iris_hip as ih

RECORD_BYTES = ctypes.sizeof(ih.Match)  # 32


def shard_range(n, rank, world):
    """Contiguous shard [lo, hi) of n records for `rank` (balanced, ragged-safe); the
    library's iris_group_db_create splits the same way (s * n / S)."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def _gather(raw):
    t = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy())
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.numpy().tobytes() for o in out]


def allgather_merge_many(locals_):
    """Per query: merge of every rank's Match, for a list of per-query Matches (a batched
    search), with ONE all-gather of len(locals_) x 32 bytes per rank."""
    nq = len(locals_)
    if nq == 0:
        return []
    per_rank = _gather(b"".join(bytes(m) for m in locals_))
    return [ih.merge_matches([ih.Match.from_buffer_copy(r[q * RECORD_BYTES:(q + 1) * RECORD_BYTES])
                              for r in per_rank]) for q in range(nq)]


def allgather_merge(local):
    """All-gather every rank's Match and merge."""
    return ih.merge_matches([ih.Match.from_buffer_copy(r) for r in _gather(bytes(local))])
