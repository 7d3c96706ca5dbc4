"""Frame sharding across GPUs of one node.

Frame pairs are independent, so a batch of N pairs is split into contiguous shards, one per rank,
with no data-path collective.  The only cross-rank traffic is control (RCCL "nccl" on GPU, gloo on CPU):

* ``broadcast_params`` -- rank 0's ``ofdis_params`` (~100 B) to every rank, so all shards run one config;
* ``max_over_ranks``   -- the per-rank elapsed time of the timed region (the job ends with the slowest);
* ``sum_over_ranks``   -- whole-job counters: frames, sum of end-point differences vs the CPU oracle,
  bit-exact frames, per-kernel device time.
"""
from __future__ import annotations

import ctypes as C


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous [start, stop) of the frames owned by `rank`; sizes differ by at most one."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def broadcast_params(p, device=None, src: int = 0):
    """Broadcast a ctypes parameter struct (``ofdis_params``) from rank `src` in place; returns it."""
    import torch
    import torch.distributed as dist
    n = C.sizeof(p)
    raw = torch.tensor(list(C.string_at(C.addressof(p), n)), dtype=torch.uint8, device=device)
    dist.broadcast(raw, src=src)
    C.memmove(C.addressof(p), bytes(raw.cpu().tolist()), n)
    return p


def all_gather_objects(obj):
    """Every rank's `obj` (small, picklable: shard bounds, counters) in rank order."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
