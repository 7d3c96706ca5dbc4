"""Frame sharding across GPUs of one node.

Frame pairs are independent, so a batch of N pairs is split into contiguous shards, one per rank,
with no data-path collective.  The only cross-rank traffic is control: a barrier and the max of the
per-rank elapsed times (and optional counters), over RCCL ("nccl") on GPU or gloo on CPU.
"""
from __future__ import annotations


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
