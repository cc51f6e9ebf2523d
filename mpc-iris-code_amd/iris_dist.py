"""iris_dist — multi-GPU sharding of the template database.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).  The
database is partitioned into contiguous index ranges, each rank searches its
own shard with no data-path communication, and the only exchange is one
all-gather of the 32-byte per-shard iris_match_t records, merged with the
native iris_match_merge (min fraction, then lowest global index — the
resolver's rule, src/main.rs:616-621).  The reference has no equivalent
(its participants each hold the full DB and talk TCP, src/main.rs:384-578).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

import iris_hip as ih

RECORD_BYTES = ctypes.sizeof(ih.Match)  # 32


def shard_range(n, rank, world):
    """Contiguous shard [lo, hi) of n records for `rank` (balanced, ragged-safe)."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def allgather_merge(local, device=None):
    """All-gather every rank's Match and merge.  `device` is the torch device the
    exchange tensor lives on (a cuda device for RCCL, cpu for gloo)."""
    buf = np.frombuffer(bytes(local), dtype=np.uint8).copy()
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    world = dist.get_world_size()
    if t.is_cuda:  # RCCL: one [world * 32] byte tensor, one device-to-host copy
        flat = torch.empty(world * RECORD_BYTES, dtype=torch.uint8, device=t.device)
        dist.all_gather_into_tensor(flat, t)
        raw = flat.cpu().numpy().tobytes()
        recs = [ih.Match.from_buffer_copy(raw[i * RECORD_BYTES:(i + 1) * RECORD_BYTES]) for i in range(world)]
    else:
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        recs = [ih.Match.from_buffer_copy(o.numpy().tobytes()) for o in out]
    return ih.merge_matches(recs)
