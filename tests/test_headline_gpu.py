"""Parity at the headline launch shape of bench.py's C2 leg: StereoPipeline(n_engines=3) over
384 KITTI-size pairs per batch (128 pairs = 256 images per engine launch), the batches built
exactly as bench.py builds its rotating input buffers (8 distinct synthetic pairs, buffer k uses
pair (i + 3k) % 8 rolled by 7k columns). Two consecutive batches (k = 0, 1), every pair's left /
right keypoints, descriptors, mvuRight and mvDepth bit-exact against the oracle's ORBextractor +
Frame::ComputeStereoMatches (ORBextractor.cc:1543-1658, Frame.cc:831-1128)."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu
KITTI_BF, KITTI_FX = 386.1448, 718.856
H, W, B, POOL = 376, 1241, 384, 8


def _pair(pool, i, k):
    L, R = pool[(i + 3 * k) % len(pool)]
    if k:
        L, R = np.roll(L, 7 * k, axis=1), np.roll(R, 7 * k, axis=1)
    return L, R


def test_headline_pipeline_384_pairs(amd, oracle_mod):
    import torch
    pool = [synth.stereo_pair(H, W, 2 + t) for t in range(POOL)]
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    pl = amd.StereoPipeline(2000, n_engines=3)
    pl.reserve(W, H, B)
    assert [pl.chunk(i)[2] for i in range(3)] == [0, 0, 0]
    for k in (0, 1):
        imgs = np.empty((2 * B, H, W), np.uint8)
        for i in range(B):
            imgs[2 * i], imgs[2 * i + 1] = _pair(pool, i, k)
        dev = torch.from_numpy(imgs).cuda()
        torch.cuda.synchronize()
        pl.stereo_batch(dev.data_ptr(), B, W, H, W, W * H, KITTI_BF, mb)
        assert [pl.chunk(i)[2] for i in range(3)] == [128, 128, 128]
        refs = {}
        for src in range(POOL):   # the 8 distinct pairs of this buffer
            L, R = _pair(pool, (src - 3 * k) % POOL, k)
            exL, exR = oracle_mod.Extractor(2000), oracle_mod.Extractor(2000)
            kL, dL = exL.extract(L)
            kR, dR = exR.extract(R)
            u, d = oracle_mod.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, mb)
            refs[src] = (kL, dL, kR, dR, u, d)
        matched = 0
        for i in range(B):
            kL, dL, kR, dR, u_ref, d_ref = refs[(i + 3 * k) % POOL]
            gkL, gdL, gkR, gdR = pl.fetch(i)
            assert gkL.tobytes() == kL.tobytes() and np.array_equal(gdL, dL), f"batch {k} pair {i} left"
            assert gkR.tobytes() == kR.tobytes() and np.array_equal(gdR, dR), f"batch {k} pair {i} right"
            u, d = pl.stereo_fetch(i)
            n = len(kL)
            assert u[:n].tobytes() == u_ref.tobytes() and d[:n].tobytes() == d_ref.tobytes(), f"batch {k} pair {i} stereo"
            matched += int((u_ref >= 0).sum())
        assert matched > 100 * B
        del dev
    pl.close()
