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


_BUFS = {}


def _exchange_buffers(device, world, nbytes):
    """Per (device, world, size) exchange tensors, allocated once: the per-step cost
    is then one small H2D copy, the all-gather and one D2H copy into pinned memory."""
    key = (str(device), world, nbytes)
    if key not in _BUFS:
        if len(_BUFS) >= 8:  # many distinct batch sizes: keep the cache bounded
            _BUFS.clear()
        _BUFS[key] = (torch.empty(nbytes, dtype=torch.uint8, device=device),
                      torch.empty(world * nbytes, dtype=torch.uint8, device=device),
                      torch.empty(world * nbytes, dtype=torch.uint8).pin_memory())
    return _BUFS[key]


def allgather_merge_many(locals_, device=None):
    """Per query: merge of every rank's Match, for a list of per-query Matches
    (a batched search), with ONE all-gather of len(locals_) x 32 bytes per rank."""
    nq = len(locals_)
    if nq == 0:
        return []
    buf = np.frombuffer(b"".join(bytes(m) for m in locals_), dtype=np.uint8).copy()
    t = torch.from_numpy(buf)
    world = dist.get_world_size()
    if device is not None and torch.device(device).type == "cuda":
        send, flat, host = _exchange_buffers(device, world, nq * RECORD_BYTES)
        send.copy_(t)
        dist.all_gather_into_tensor(flat, send)
        host.copy_(flat)
        raw = host.numpy().tobytes()
    else:
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        raw = b"".join(o.numpy().tobytes() for o in out)
    per_rank = nq * RECORD_BYTES
    return [ih.merge_matches([ih.Match.from_buffer_copy(raw[r * per_rank + q * RECORD_BYTES:
                                                            r * per_rank + (q + 1) * RECORD_BYTES])
                              for r in range(world)]) for q in range(nq)]


def allgather_merge(local, device=None):
    """All-gather every rank's Match and merge.  `device` is the torch device the
    exchange tensor lives on (a cuda device for RCCL, cpu for gloo)."""
    buf = np.frombuffer(bytes(local), dtype=np.uint8).copy()
    t = torch.from_numpy(buf)
    world = dist.get_world_size()
    if device is not None and torch.device(device).type == "cuda":
        # RCCL: one [world * 32] byte all-gather into a device tensor, one D2H copy
        send, flat, host = _exchange_buffers(device, world, RECORD_BYTES)
        send.copy_(t)
        dist.all_gather_into_tensor(flat, send)
        host.copy_(flat)
        raw = host.numpy().tobytes()
        recs = [ih.Match.from_buffer_copy(raw[i * RECORD_BYTES:(i + 1) * RECORD_BYTES]) for i in range(world)]
    else:
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        recs = [ih.Match.from_buffer_copy(o.numpy().tobytes()) for o in out]
    return ih.merge_matches(recs)
