"""GPU parity of Frame::ComputeStereoMatches (Frame.cc:831-1128) and the Hamming core
(ORBmatcher.cc:2123-2143) against the CPU oracle: mvuRight / mvDepth bit-exact."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu

KITTI_BF = 386.1448       # Stereo/KITTI00-02.yaml:25 (Camera.bf)
KITTI_FX = 718.856        # Stereo/KITTI00-02.yaml:8


def _stereo_ref(oracle_mod, L, R, nf):
    exL = oracle_mod.Extractor(nf, 1.2, 8, 20, 7)
    exR = oracle_mod.Extractor(nf, 1.2, 8, 20, 7)
    kL, dL = exL.extract(L)
    kR, dR = exR.extract(R)
    mb = np.float32(KITTI_BF) / np.float32(KITTI_FX)
    u, d = oracle_mod.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, float(mb))
    return kL, u, d, float(mb)


@pytest.mark.parametrize("t", [0, 3])
def test_stereo_single_pair(amd, oracle_mod, t):
    L, R = synth.stereo_pair(376, 1241, t)
    kL, u_ref, d_ref, mb = _stereo_ref(oracle_mod, L, R, 2000)
    exL = amd.ORBextractor(2000)
    exR = amd.ORBextractor(2000)
    k, _ = exL(L)
    exR(R)
    assert len(k) == len(kL)
    u, d = amd.compute_stereo_matches(exL, exR, len(k), KITTI_BF, mb)
    assert (u_ref >= 0).sum() > 100, "synthetic pair should produce stereo matches"
    np.testing.assert_array_equal(u.view(np.uint32), u_ref.view(np.uint32))
    np.testing.assert_array_equal(d.view(np.uint32), d_ref.view(np.uint32))


@pytest.mark.parametrize("nf", [90, 300])
def test_stereo_few_features(amd, oracle_mod, nf):
    """Keypoint counts that leave the last staged workgroup (32 left keypoints, 8 per wavefront)
    partly filled, and images with few candidates per band."""
    L, R = synth.stereo_pair(376, 1241, 5)
    kL, u_ref, d_ref, mb = _stereo_ref(oracle_mod, L, R, nf)
    exL = amd.ORBextractor(nf)
    exR = amd.ORBextractor(nf)
    k, _ = exL(L)
    exR(R)
    assert len(k) == len(kL)
    u, d = amd.compute_stereo_matches(exL, exR, len(k), KITTI_BF, mb)
    np.testing.assert_array_equal(u.view(np.uint32), u_ref.view(np.uint32))
    np.testing.assert_array_equal(d.view(np.uint32), d_ref.view(np.uint32))


@pytest.mark.parametrize("rows", [36, 160])
def test_stereo_dense_rows(amd, oracle_mod, rows):
    """Keypoints packed into a band of rows: with 36 rows every candidate band holds far more
    right keypoints than a workgroup stages (ST_SCAP, orb_stereo.hip), so the staged matcher
    takes its global-memory scan; with 160 rows both forms occur."""
    h, w = 376, 1241
    rng = np.random.default_rng(rows)
    L = np.full((h, w), 40, np.uint8)
    y0 = (h - rows) // 2
    L[y0:y0 + rows] = rng.integers(0, 256, size=(rows, w), dtype=np.uint8)
    R = np.roll(L, -17, axis=1)
    R[:, -17:] = 40
    kL, u_ref, d_ref, mb = _stereo_ref(oracle_mod, L, R, 2000)
    exL = amd.ORBextractor(2000)
    exR = amd.ORBextractor(2000)
    k, _ = exL(L)
    exR(R)
    assert len(k) == len(kL)
    u, d = amd.compute_stereo_matches(exL, exR, len(k), KITTI_BF, mb)
    assert (u_ref >= 0).sum() > 50
    np.testing.assert_array_equal(u.view(np.uint32), u_ref.view(np.uint32))
    np.testing.assert_array_equal(d.view(np.uint32), d_ref.view(np.uint32))


def test_stereo_batch(amd, oracle_mod):
    import torch
    h, w, P = 376, 1241, 3
    pairs = [synth.stereo_pair(h, w, 10 + p) for p in range(P)]
    imgs = np.stack([im for pr in pairs for im in pr])
    dev = torch.from_numpy(imgs).cuda()
    ex = amd.BatchExtractor(2000)
    ex.reserve(w, h, 2 * P)
    torch.cuda.synchronize()
    ex.extract_device(dev.data_ptr(), 2 * P, w, h, w, h * w)
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    ex.stereo_batch(P, KITTI_BF, mb)
    for p in range(P):
        kL, u_ref, d_ref, _ = _stereo_ref(oracle_mod, *pairs[p], 2000)
        u, d = ex.stereo_fetch(p)
        n = len(kL)
        np.testing.assert_array_equal(u[:n].view(np.uint32), u_ref.view(np.uint32))
        np.testing.assert_array_equal(d[:n].view(np.uint32), d_ref.view(np.uint32))


def test_hamming_best2(amd, oracle_mod):
    rng = np.random.default_rng(3)
    db = rng.integers(0, 256, size=(1500, 32), dtype=np.uint8)
    q = db[rng.integers(0, 1500, 300)].copy()
    q[::2, 0] ^= 0x5A  # near-duplicates and exact duplicates
    dbd = np.concatenate([db, db[:50]])  # duplicate rows -> ties resolved to first index
    bi, bd, sd = amd.ORBmatcher.hamming_best2(q, dbd)
    ri, rd, rs = oracle_mod.hamming_best2(q, dbd)
    np.testing.assert_array_equal(bi, ri)
    np.testing.assert_array_equal(bd, rd)
    np.testing.assert_array_equal(sd, rs)


@pytest.mark.parametrize("P,k", [(5, 3), (2, 3), (4, 2)])
def test_stereo_pipeline(amd, oracle_mod, P, k):
    """orbx_pipeline_*: k engines on k streams, chunks of consecutive pairs (uneven and empty
    chunks included), two batches back to back (the second's phase 1 waits on the first's),
    every pair bit-exact with the oracle's extraction + ComputeStereoMatches."""
    import torch
    h, w = 376, 1241
    pairs = [synth.stereo_pair(h, w, 20 + p) for p in range(P)]
    imgs = np.stack([im for pr in pairs for im in pr])
    dev = torch.from_numpy(imgs).cuda()
    dev2 = torch.flip(dev, dims=[0]).contiguous()   # second batch: pairs reversed, L / R swapped
    pl = amd.StereoPipeline(2000, n_engines=k)
    pl.reserve(w, h, P)
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    torch.cuda.synchronize()
    pl.stereo_batch(dev2.data_ptr(), P, w, h, w, h * w, KITTI_BF, mb)
    pl.stereo_batch(dev.data_ptr(), P, w, h, w, h * w, KITTI_BF, mb)
    torch.cuda.synchronize()
    assert sum(pl.chunk(i)[2] for i in range(k)) == P
    for p in range(P):
        kL, u_ref, d_ref, _ = _stereo_ref(oracle_mod, *pairs[p], 2000)
        gkL, gdL, gkR, gdR = pl.fetch(p)
        assert gkL.tobytes() == kL.tobytes()
        u, d = pl.stereo_fetch(p)
        n = len(kL)
        np.testing.assert_array_equal(u[:n].view(np.uint32), u_ref.view(np.uint32))
        np.testing.assert_array_equal(d[:n].view(np.uint32), d_ref.view(np.uint32))
    pl.close()


def test_stereo_pipeline_opencv32(amd, oracle_mod):
    """The pipeline under the reference's documented platform (OpenCV 3.2 on x86-64, README.md:9):
    the SSE2 resize layout (resize_mode 1) and the half-even GaussianBlur column pass (blur_mode 1),
    12 pairs over 3 engines: keypoints, descriptors, mvuRight and mvDepth bit-exact against the
    oracle in the same variants."""
    import torch
    h, w, P, k = 376, 1241, 12, 3
    pairs = [synth.stereo_pair(h, w, 50 + p) for p in range(P)]
    dev = torch.from_numpy(np.stack([im for pr in pairs for im in pr])).cuda()
    pl = amd.StereoPipeline(2000, n_engines=k, resize_mode=1, blur_mode=1)
    pl.reserve(w, h, P)
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    torch.cuda.synchronize()
    pl.stereo_batch(dev.data_ptr(), P, w, h, w, h * w, KITTI_BF, mb)
    torch.cuda.synchronize()
    for p in range(P):
        L, R = pairs[p]
        exL = oracle_mod.Extractor(2000, resize_mode=1, blur_mode=1)
        exR = oracle_mod.Extractor(2000, resize_mode=1, blur_mode=1)
        kL, dL = exL.extract(L)
        kR, dR = exR.extract(R)
        u, d = oracle_mod.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, mb)
        _check_pair((*pl.fetch(p), *[a[:len(kL)] for a in pl.stereo_fetch(p)]), (kL, dL, kR, dR, u, d), f"pair {p}")
    pl.close()


def test_stereo_pipeline_host_mode(amd, oracle_mod):
    """orbx_pipeline_stereo_batch_host: host (pinned) images in, host outputs out, the H2D of the
    next batch overlapping the current one, three batches back to back into two output buffers
    (two device input slots): every pair bit-exact with the oracle."""
    h, w, P, k = 376, 1241, 7, 3
    pairs = [synth.stereo_pair(h, w, 40 + p) for p in range(P)]
    ins = []
    for b in range(3):
        a = amd.host_empty((2 * P, h, w), np.uint8)
        for p in range(P):
            L, R = pairs[(p + b) % P]
            a[2 * p], a[2 * p + 1] = L, R
        ins.append(a)
    pl = amd.StereoPipeline(2000, n_engines=k)
    pl.reserve(w, h, P)
    cap = pl.capacity()
    outs = [amd.StereoHostBatch(P, cap), amd.StereoHostBatch(P, cap)]
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    refs = [_stereo_ref_full(oracle_mod, *pairs[p]) for p in range(P)]
    pl.stereo_batch_host(ins[0], P, w, h, w, w * h, KITTI_BF, mb, outs[0])
    pl.stereo_batch_host(ins[1], P, w, h, w, w * h, KITTI_BF, mb, outs[1])
    pl.wait()
    got1 = [outs[1].pair(p) for p in range(P)]
    got1 = [tuple(np.array(x) for x in g) for g in got1]
    for b, out in ((0, outs[0]),):
        for p in range(P):
            _check_pair(out.pair(p), refs[(p + b) % P], f"batch {b} pair {p}")
    pl.stereo_batch_host(ins[2], P, w, h, w, w * h, KITTI_BF, mb, outs[0])
    pl.wait()
    for p in range(P):
        _check_pair(got1[p], refs[(p + 1) % P], f"batch 1 pair {p}")
        _check_pair(outs[0].pair(p), refs[(p + 2) % P], f"batch 2 pair {p}")
    pl.close()


def _stereo_ref_full(oracle_mod, L, R):
    exL, exR = oracle_mod.Extractor(2000), oracle_mod.Extractor(2000)
    kL, dL = exL.extract(L)
    kR, dR = exR.extract(R)
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    u, d = oracle_mod.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, mb)
    return kL, dL, kR, dR, u, d


def _check_pair(got, ref, what):
    gkL, gdL, gkR, gdR, gu, gd = got
    kL, dL, kR, dR, u, d = ref
    assert gkL.tobytes() == kL.tobytes() and np.array_equal(gdL, dL), what + " left"
    assert gkR.tobytes() == kR.tobytes() and np.array_equal(gdR, dR), what + " right"
    assert gu.tobytes() == u.tobytes() and gd.tobytes() == d.tobytes(), what + " stereo"


def test_stereo_pipeline_host_mode_varying_stride(amd, oracle_mod):
    """host-mode batches (10 pairs, stride S), (5, S), (10, S), (5, 2S) -- slot 1 is reused
    with the same pair count but a larger image stride while it is already big enough, so chunk j's
    upload covers byte ranges that engines j+1.. read in slot 1's previous batch: the upload must wait
    for every engine's reads, not only engines 0..j (the layout is keyed on count and stride)."""
    h, w, k = 376, 1241, 3
    S = w * h
    pairs = [synth.stereo_pair(h, w, 80 + p) for p in range(10)]
    refs = [_stereo_ref_full(oracle_mod, *pr) for pr in pairs]
    plan = ((10, 1), (5, 1), (10, 1), (5, 2))   # (pairs, stride in images)
    order = [[(p * 7 + b) % 10 for p in range(P)] for b, (P, _) in enumerate(plan)]
    ins = []
    for b, (P, m) in enumerate(plan):
        a = amd.host_empty((2 * P, m * h, w), np.uint8)
        a[...] = 0xA5                             # the gap rows of the wide stride are never read
        for p, q in enumerate(order[b]):
            a[2 * p, :h], a[2 * p + 1, :h] = pairs[q]
        ins.append(a)
    pl = amd.StereoPipeline(2000, n_engines=k)
    pl.reserve(w, h, 10)
    cap = pl.capacity()
    outs = [amd.StereoHostBatch(P, cap) for P, _ in plan]
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    for b, (P, m) in enumerate(plan):
        pl.stereo_batch_host(ins[b], P, w, h, w, m * S, KITTI_BF, mb, outs[b])
    pl.wait()
    for b, (P, _) in enumerate(plan):
        for p, q in enumerate(order[b]):
            _check_pair(outs[b].pair(p), refs[q], f"batch {b} pair {p}")
    pl.close()


def test_stereo_pipeline_host_mode_varying_batches(amd, oracle_mod):
    """Host-mode batches of 10, 5 and 8 pairs (slot 0, slot 1, slot 0 again): the third batch's
    chunk ranges in slot 0 straddle the first batch's, so its uploads must wait for every engine's
    reads of the first batch, not only engines 0..j. Then a device-input batch is enqueued before
    wait(): its phase 2 must not overwrite outputs still draining to the host."""
    import torch
    h, w, k = 376, 1241, 3
    pairs = [synth.stereo_pair(h, w, 60 + p) for p in range(10)]
    refs = [_stereo_ref_full(oracle_mod, *pr) for pr in pairs]
    sizes = (10, 5, 8)
    order = [[(p * 3 + b) % 10 for p in range(P)] for b, P in enumerate(sizes)]
    ins = []
    for b, P in enumerate(sizes):
        a = amd.host_empty((2 * P, h, w), np.uint8)
        for p, q in enumerate(order[b]):
            a[2 * p], a[2 * p + 1] = pairs[q]
        ins.append(a)
    pl = amd.StereoPipeline(2000, n_engines=k)
    pl.reserve(w, h, 10)
    cap = pl.capacity()
    outs = [amd.StereoHostBatch(P, cap) for P in sizes]
    with pytest.raises(ValueError):
        pl.stereo_batch_host(ins[0], 10, w, h, w, w * h, KITTI_BF, 0.5, amd.StereoHostBatch(4, cap))
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    for b, P in enumerate(sizes):
        pl.stereo_batch_host(ins[b], P, w, h, w, w * h, KITTI_BF, mb, outs[b])
    dev = torch.from_numpy(np.flip(ins[0], axis=0).copy()).cuda()   # reversed: other content per engine
    torch.cuda.synchronize()
    pl.stereo_batch(dev.data_ptr(), 10, w, h, w, h * w, KITTI_BF, mb)
    pl.wait()
    for b, P in enumerate(sizes):
        for p, q in enumerate(order[b]):
            _check_pair(outs[b].pair(p), refs[q], f"batch {b} pair {p}")
    torch.cuda.synchronize()
    pl.close()
