"""gloo runs of the multi-GPU plumbing used by bench.py (CPU, no GPU) at world size 2 and at the
8 ranks of the driver's C5 run (one per GPU of a node): shared-state broadcast from rank 0,
map-snapshot broadcast (C5), sequence sharding, max / sum over ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from orbslam2_amd import dist as odist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    state = [2000, 1.2, 8, 20, 7, 386.1448, 718.856] if rank == 0 else [0] * 7
    got = odist.broadcast_shared(state, "cpu", dist)
    mine = list(odist.shard(8, world, rank))   # C5: 8 sequences over the ranks
    mx = odist.max_over_ranks(float(rank + 1), "cpu", dist)
    tot = odist.sum_over_ranks(float(len(mine)), "cpu", dist)
    from orbslam2_amd import synth
    snap = synth.localba_problem(seed=4, n_kf=10, n_points=200) if rank == 0 else None
    snap = odist.broadcast_map(snap, "cpu", dist)
    digest = {k: (v.dtype.str, v.shape, v.tobytes()) for k, v in snap.items()}
    q.put((rank, got, mine, mx, tot, digest))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world2(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owned = []
    from orbslam2_amd import synth
    want = synth.localba_problem(seed=4, n_kf=10, n_points=200)
    for rank, got, mine, mx, tot, digest in res:
        assert sorted(digest) == sorted(want)
        for k, a in want.items():   # map snapshot identical on every rank (dtype, shape, bytes)
            assert digest[k] == (a.dtype.str, a.shape, a.tobytes()), k
        assert got == pytest.approx([2000, 1.2, 8, 20, 7, 386.1448, 718.856])
        assert mx == world
        assert tot == 8
        owned += mine
    assert sorted(owned) == list(range(8))


def test_shard_balanced():
    for n in range(0, 20):
        for w in range(1, 9):
            parts = [odist.shard(n, w, r) for r in range(w)]
            assert sum(len(p) for p in parts) == n
            assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1
