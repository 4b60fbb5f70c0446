"""Multi-GPU plumbing for the hot path: one process per GPU, independent
frames / sequences per rank (weak scaling), one broadcast of the shared read-only state from
rank 0, and max-over-ranks timing. No per-frame collective exists on this path.

Backend "nccl" is RCCL over xGMI on ROCm; "gloo" is used for the CPU tests.
"""
from __future__ import annotations

import os


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_units: int, world: int, rank: int) -> range:
    """Contiguous block of sequences / frames owned by `rank` (balanced, covers all units)."""
    base, extra = divmod(n_units, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def broadcast_shared(values, device, dist) -> list:
    """Broadcast rank 0's shared state (ORB params, camera) to every rank (once)."""
    import torch
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist is not None:
        dist.broadcast(t, src=0)
    return t.tolist()


def max_over_ranks(x: float, device, dist) -> float:
    import torch
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, device, dist) -> float:
    import torch
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
