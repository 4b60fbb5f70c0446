"""Parity at the headline launch shape of bench.py's C2 leg (shapes.C2_*): StereoPipeline with
C2_ENGINES engines over C2_BATCH KITTI-size pairs per batch, fed from SURVEY §8d's 512-frame
stream (left seed 2 + t, disparity seed 1002 + t, noise seed 2002 + t) exactly as bench.py
feeds it: the stream resident twice back to back, step k = frames (k * 384) mod 512 .. + 383.
Two consecutive steps (frames 0..383, then 384..511 and 0..255: every frame of the stream, 384
distinct pairs per batch), every pair's left / right keypoints, descriptors, mvuRight and mvDepth
bit-exact against the oracle's ORBextractor + Frame::ComputeStereoMatches
(ORBextractor.cc:1543-1658, Frame.cc:831-1128). A third run puts a batch flush against the end
of an allocation whose size is a 2 MiB multiple: the extractor reads no byte past the caller's
images (include/orbslam2_amd.h)."""
import numpy as np
import pytest

from orbslam2_amd import shapes, synth

pytestmark = pytest.mark.gpu
KITTI_BF, KITTI_FX = 386.1448, 718.856
H, W, B, E, N = shapes.C2_H, shapes.C2_W, shapes.C2_BATCH, shapes.C2_ENGINES, shapes.C2_STREAM_FRAMES


@pytest.fixture(scope="module")
def stream():
    return synth.stereo_stream(H, W, N)


@pytest.fixture(scope="module")
def stream_ref(stream, oracle_mod):
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    return oracle_mod.stereo_frames(stream, range(N), 2000, KITTI_BF, mb)


def _check_batch(pl, frames, ref, tag):
    matched = 0
    for i, j in enumerate(frames):
        kL, dL, kR, dR, u_ref, d_ref = ref[j]
        gkL, gdL, gkR, gdR = pl.fetch(i)
        assert gkL.tobytes() == kL.tobytes() and np.array_equal(gdL, dL), f"{tag} pair {i} (frame {j}) left"
        assert gkR.tobytes() == kR.tobytes() and np.array_equal(gdR, dR), f"{tag} pair {i} (frame {j}) right"
        u, d = pl.stereo_fetch(i)
        n = len(kL)
        assert u[:n].tobytes() == u_ref.tobytes() and d[:n].tobytes() == d_ref.tobytes(), f"{tag} pair {i} stereo"
        matched += int((u_ref >= 0).sum())
    assert matched > 100 * len(frames)


def test_headline_pipeline_stream(amd, stream, stream_ref):
    import torch
    assert (B, E, N) == (384, 3, 512)
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    imgs = np.empty((4 * N, H, W), np.uint8)   # bench.c2_stream_buffer: the stream twice
    for i in range(2 * N):
        imgs[2 * i], imgs[2 * i + 1] = stream[i % N]
    dev = torch.from_numpy(imgs).cuda()
    del imgs
    pl = amd.StereoPipeline(2000, n_engines=E)
    pl.reserve(W, H, B)
    assert [pl.chunk(i)[2] for i in range(E)] == [0] * E
    seen = set()
    for k in (0, 1):
        frames = shapes.c2_batch_frames(k, B, N)
        seen.update(frames)
        torch.cuda.synchronize()
        pl.stereo_batch(dev.data_ptr() + 2 * frames[0] * W * H, B, W, H, W, W * H, KITTI_BF, mb)
        assert [pl.chunk(i)[2] for i in range(E)] == [B // E] * E
        _check_batch(pl, frames, stream_ref, f"step {k}")
    assert seen == set(range(N))
    pl.close()
    del dev


def test_headline_batch_ends_at_allocation_end(amd, stream, stream_ref):
    """The C2 pipeline's 384 pairs placed flush against the end of a fresh 2 MiB-multiple
    allocation (the batch's last right image ends on the allocation's last byte; when that is also
    the end of the mapping, any read past it faults): every pair oracle-equal."""
    import torch
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    frames = shapes.c2_batch_frames(2, B, N)
    nbytes = 2 * B * W * H
    alloc = -(-nbytes // (2 << 20)) * (2 << 20)
    torch.cuda.empty_cache()
    dev = torch.empty(alloc, dtype=torch.uint8, device="cuda")
    off = alloc - nbytes
    imgs = np.empty((2 * B, H, W), np.uint8)
    for i, j in enumerate(frames):
        imgs[2 * i], imgs[2 * i + 1] = stream[j]
    dev[off:].copy_(torch.from_numpy(imgs.reshape(-1)))
    del imgs
    pl = amd.StereoPipeline(2000, n_engines=E)
    pl.reserve(W, H, B)
    torch.cuda.synchronize()
    pl.stereo_batch(dev.data_ptr() + off, B, W, H, W, W * H, KITTI_BF, mb)
    amd.device_sync()
    _check_batch(pl, frames, stream_ref, "flush")
    pl.close()
    del dev
