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


def broadcast_map(arrays, device, dist) -> dict:
    """Broadcast rank 0's map snapshot: a dict of numpy arrays -- keyframe
    poses, map point positions and descriptors, observations -- packed into one byte tensor
    and sent over RCCL (xGMI) from rank 0 in two collectives (sizes, then payload). Other
    ranks pass None and get an identical dict back. Read-only shared state: sent once before
    the timed region, never per frame."""
    import json

    import numpy as np
    import torch
    if dist is None:
        return arrays
    rank = dist.get_rank()
    if rank == 0:
        names = sorted(arrays)
        header = json.dumps([[k, arrays[k].dtype.str, list(arrays[k].shape)] for k in names]).encode()
        payload = b"".join(np.ascontiguousarray(arrays[k]).tobytes() for k in names)
        sizes = torch.tensor([len(header), len(payload)], dtype=torch.int64, device=device)
    else:
        sizes = torch.zeros(2, dtype=torch.int64, device=device)
    dist.broadcast(sizes, src=0)
    nh, npl = (int(v) for v in sizes.tolist())
    buf = torch.empty(nh + npl, dtype=torch.uint8, device=device)
    if rank == 0:
        buf.copy_(torch.from_numpy(np.frombuffer(header + payload, np.uint8).copy()))
    dist.broadcast(buf, src=0)
    raw = buf.cpu().numpy().tobytes()
    out, off = {}, nh
    for k, dt, shape in json.loads(raw[:nh].decode()):
        dt = np.dtype(dt)
        n = int(np.prod(shape)) * dt.itemsize
        out[k] = np.frombuffer(raw, dt, count=int(np.prod(shape)), offset=off).reshape(shape).copy()
        off += n
    return out
