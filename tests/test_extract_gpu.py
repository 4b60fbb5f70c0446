"""GPU parity of the HIP ORBextractor against the CPU oracle (bit-exact).

Follows ORBextractor::operator() (ORBextractor.cc:1543-1658): keypoints (all 7 cv::KeyPoint
fields), the 32-byte descriptors, their order (level-major, quadtree list order) and the
image pyramid must be identical to the oracle's on the same seeded inputs.
"""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu


def _assert_same_kps(got, ref, tag=""):
    gk, gd = got
    rk, rd = ref
    assert len(gk) == len(rk), f"{tag}: count {len(gk)} != oracle {len(rk)}"
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = gk[f], rk[f]
        bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
        assert bad.size == 0, f"{tag}: field {f} differs at {bad[:8]} got {a[bad[:4]]} want {b[bad[:4]]}"
    bad = np.nonzero((gd != rd).any(axis=1))[0]
    assert bad.size == 0, f"{tag}: descriptor rows differ at {bad[:8]}"


# mode = resize_mode + 2 * blur_mode (SURVEY A.2 / A.3 variants; 3 = the OpenCV 3.2 x86 platform of
# README.md:9: SSE2 resize prefix and half-even blur prefix)
CASES = [
    ("kitti", 376, 1241, 2000, 0, 2),
    ("kitti_sse", 376, 1241, 2000, 1, 5),
    ("kitti_cv32", 376, 1241, 2000, 3, 2),
    ("tum_blur32", 480, 640, 1000, 2, 3),
    ("odd_cv32", 333, 517, 800, 3, 26),
    ("tum", 480, 640, 1000, 0, 3),
    ("tum_b", 480, 640, 1000, 0, 11),
    ("kitti_04", 370, 1226, 2000, 0, 21),    # KITTI04-12.yaml resolution
    ("euroc", 480, 752, 1200, 0, 22),        # EuRoC.yaml
    ("qvga", 240, 320, 500, 0, 23),
    ("fullhd", 1080, 1920, 4000, 0, 24),
    ("odd", 333, 517, 800, 1, 25),
]


@pytest.mark.parametrize("name,h,w,nf,mode,seed", CASES)
def test_extract_parity(amd, oracle_mod, name, h, w, nf, mode, seed):
    img = synth.textured_image(h, w, seed)
    rm, bm = mode & 1, mode >> 1
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, resize_mode=rm, blur_mode=bm)
    ref = oracle_mod.Extractor(nf, 1.2, 8, 20, 7, resize_mode=rm, blur_mode=bm)
    got = ex(img)
    want = ref.extract(img)
    for l in range(8):
        lev = ref.level(l)
        np.testing.assert_array_equal(ex.pyramid_level(l), lev, err_msg=f"pyramid level {l}")
        # E6 directly: the MFMA blur's every pixel, borders included, against the
        # GaussianBlur restatement (ORBextractor.cc:1617-1625) in the same variant
        np.testing.assert_array_equal(ex.blurred_level(l), oracle_mod.gaussian_blur9(lev, bm),
                                      err_msg=f"blurred level {l}")
    _assert_same_kps(got, want, name)


@pytest.mark.parametrize("blur_mode", [0, 1])
@pytest.mark.parametrize("h,w", [(376, 1241), (480, 640), (240, 320), (333, 517), (241, 1023)])
def test_blurred_pyramid_noise(amd, oracle_mod, h, w, blur_mode):
    """Blurred pyramid of uniform noise (every byte value) and of 0/255 vertical stripes (the largest
    row sums, full-scale outputs), byte for byte at every level, odd sizes included (smallest level
    >= 62 rows, the extractor's limit for one FAST cell row), in both SURVEY A.3 variants. Noise
    holds exact rounding ties, where the OpenCV 3.2 variant (blur_mode 1) differs from the
    default: the test checks that it does somewhere, so both roundings are really exercised."""
    rng = np.random.default_rng(h * 1000 + w)
    ties = 0
    for img in (rng.integers(0, 256, size=(h, w), dtype=np.uint8),
                np.broadcast_to(((np.arange(w) // 8) % 2 * 255).astype(np.uint8), (h, w)).copy()):
        ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, blur_mode=blur_mode)
        ex(img)
        ref = oracle_mod.Extractor(1000, 1.2, 8, 20, 7)
        ref.extract(img)
        for l in range(8):
            lev = ref.level(l)
            if lev.size == 0:
                continue
            want = oracle_mod.gaussian_blur9(lev, blur_mode)
            ties += int((want != oracle_mod.gaussian_blur9(lev, 1 - blur_mode)).sum())
            np.testing.assert_array_equal(ex.blurred_level(l), want, err_msg=f"{h}x{w} blurred level {l}")
    assert ties > 0


def test_extract_noise_many_candidates(amd, oracle_mod):
    """Uniform noise: thousands of FAST candidates per level (quadtree global-memory path)."""
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, size=(376, 1241), dtype=np.uint8)
    ex = amd.ORBextractor(2000, 1.2, 8, 20, 7)
    ref = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    _assert_same_kps(ex(img), ref.extract(img), "noise")


@pytest.mark.parametrize("env", [{"ORBX_QT_LDS_KB": "16"}, {"ORBX_QT_LDS_KB": "160"},
                                 {"ORBX_QT_NODES_LDS": "1", "ORBX_QT_LDS_KB": "96"}])
def test_extract_quadtree_layouts(amd, oracle_mod, monkeypatch, env):
    """The quadtree's memory layouts (read when an engine sizes its geometry): keys in global
    scratch for levels above a 16 KB LDS budget, every level in LDS at 160 KB, node arrays in LDS;
    each with its rank-sort stage (the idle key buffer, or the key area) -- all bit-exact."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(8)
    for img in (synth.textured_image(376, 1241, 31), rng.integers(0, 256, size=(376, 1241), dtype=np.uint8)):
        ex = amd.ORBextractor(2000, 1.2, 8, 20, 7)
        ref = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
        _assert_same_kps(ex(img), ref.extract(img), str(env))


def test_extract_flat_and_sparse(amd, oracle_mod):
    """Flat image: every cell retries at minThFAST and finds nothing -> 0 keypoints.
    Sparse image: a few isolated corners (tiny quadtree, size-1 roots)."""
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7)
    ref = oracle_mod.Extractor(1000, 1.2, 8, 20, 7)
    flat = np.full((480, 640), 128, np.uint8)
    k, d = ex(flat)
    assert len(k) == 0 and d.shape == (0, 32)
    _assert_same_kps((k, d), ref.extract(flat), "flat")
    sparse = flat.copy()
    for (y, x) in [(100, 100), (300, 500), (250, 320), (60, 600)]:
        sparse[y:y + 12, x:x + 12] = 250
    _assert_same_kps(ex(sparse), ref.extract(sparse), "sparse")


def test_extract_empty_image(amd):
    ex = amd.ORBextractor(1000)
    k, d = ex(np.zeros((0, 0), np.uint8))
    assert len(k) == 0


@pytest.mark.parametrize("nf,levels", [(500, 4), (3000, 8), (1200, 6), (8000, 8)])
def test_extract_param_sweep(amd, oracle_mod, nf, levels):
    img = synth.textured_image(480, 752, 21 + nf)
    ex = amd.ORBextractor(nf, 1.2, levels, 20, 7)
    ref = oracle_mod.Extractor(nf, 1.2, levels, 20, 7)
    _assert_same_kps(ex(img), ref.extract(img), f"nf{nf}_L{levels}")


def test_levels_tables(amd, oracle_mod):
    ex = amd.ORBextractor(2000, 1.2, 8, 20, 7)
    ref = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    np.testing.assert_array_equal(ex.GetScaleFactors(), ref.scale_factors)
    np.testing.assert_array_equal(ex.GetInverseScaleFactors(), ref.inv_scale_factors)
    assert ex.features_per_level() == ref.features_per_level


def test_batch_device_matches_single(amd, oracle_mod):
    """Batched device path (many images per launch) == oracle per image."""
    import torch
    h, w, n = 376, 1241, 6
    imgs = np.stack([synth.textured_image(h, w, 40 + i) for i in range(n)])
    dev = torch.from_numpy(imgs).cuda()
    ex = amd.BatchExtractor(2000, 1.2, 8, 20, 7)
    ex.reserve(w, h, n)
    torch.cuda.synchronize()
    ex.extract_device(dev.data_ptr(), n, w, h, w, h * w)
    ref = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    for i in range(n):
        _assert_same_kps(ex.fetch(i), ref.extract(imgs[i]), f"batch[{i}]")


@pytest.mark.parametrize("h,w,pitch,off", [(333, 517, 517, 1), (333, 517, 519, 3), (240, 322, 322, 2)])
def test_batch_device_unaligned(amd, oracle_mod, h, w, pitch, off):
    """Images at any byte: an odd image stride (w * h odd), an odd row pitch and a batch starting
    `off` bytes into the allocation put every image's first pixel, and its rows, at every
    alignment modulo 4 (the level-1 resize reads its source rows as aligned dwords through a
    buffer descriptor starting at the dword of the image's first byte)."""
    import torch
    n = 5
    stride = pitch * (h - 1) + w + (1 if (pitch * (h - 1) + w) % 2 == 0 else 0)   # odd stride
    imgs = [synth.textured_image(h, w, 90 + i) for i in range(n)]
    buf = np.full(off + n * stride + 64, 0x5A, np.uint8)
    for i, im in enumerate(imgs):
        for y in range(h):
            buf[off + i * stride + y * pitch: off + i * stride + y * pitch + w] = im[y]
    dev = torch.from_numpy(buf).cuda()
    ex = amd.BatchExtractor(800, 1.2, 8, 20, 7)
    ex.reserve(w, h, n)
    torch.cuda.synchronize()
    ex.extract_device(dev.data_ptr() + off, n, w, h, pitch, stride)
    ref = oracle_mod.Extractor(800, 1.2, 8, 20, 7)
    for i in range(n):
        _assert_same_kps(ex.fetch(i), ref.extract(imgs[i]), f"unaligned[{i}]")


def test_large_batch_matches_oracle(amd, oracle_mod):
    """A bench-sized batch (160 images, more workgroups than the chip holds at once): every
    image must still equal the oracle."""
    import torch
    h, w, n, k = 376, 1241, 160, 5
    src = [synth.textured_image(h, w, 60 + i) for i in range(k)]
    imgs = np.stack([src[i % k] for i in range(n)])
    dev = torch.from_numpy(imgs).cuda()
    ex = amd.BatchExtractor(2000, 1.2, 8, 20, 7)
    ex.reserve(w, h, n)
    torch.cuda.synchronize()
    ex.extract_device(dev.data_ptr(), n, w, h, w, h * w)
    ref = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    want = [ref.extract(im) for im in src]
    for i in range(n):
        _assert_same_kps(ex.fetch(i), want[i % k], f"batch[{i}]")


def test_batch_ends_at_allocation_end(amd, oracle_mod):
    """512 VGA frames are exactly 75 x 2 MiB, so the batch's last image ends where its allocation
    (and possibly the mapped memory) ends. The level-1 resize reads source rows as 12-byte windows;
    the last row's last window of that image must not reach past the buffer (it did: a memory fault
    at `bench.py --rgbd-batch 512`), and the guarded dword loads that replace it there must keep
    every image equal to the oracle."""
    import torch
    h, w, n = 480, 640, 512
    assert n * h * w == 75 * 2 * 1024 * 1024
    src = [synth.rgbd_frame(h, w, t)[0] for t in range(4)]
    dev = torch.empty(n * h * w, dtype=torch.uint8, device="cuda")
    dev.view(n, h, w).copy_(torch.from_numpy(np.stack([src[i % 4] for i in range(n)])))
    ex = amd.BatchExtractor(1000, 1.2, 8, 20, 7)
    ex.reserve(w, h, n)
    torch.cuda.synchronize()
    ex.extract_device(dev.data_ptr(), n, w, h, w, h * w)
    amd.device_sync()
    ref = oracle_mod.Extractor(1000, 1.2, 8, 20, 7)
    for i in (0, n - 3, n - 1):
        _assert_same_kps(ex.fetch(i), ref.extract(src[i % 4]), f"batch[{i}]")


def test_golden_c1_c2_on_device(amd):
    """HIP path == committed golden fixtures (independent of the oracle at run time)."""
    from test_golden_cpu import load_c1, load_c2
    img, g = load_c1()
    k, d = amd.ORBextractor(1000)(img)
    assert k.tobytes() == g["kps"].tobytes() and np.array_equal(d, g["desc"])
    L, R, g2 = load_c2()
    exL, exR = amd.ORBextractor(2000), amd.ORBextractor(2000)
    kL, dL = exL(L)
    kR, _ = exR(R)
    assert kL.tobytes() == g2["kps_left"].tobytes() and np.array_equal(dL, g2["desc_left"])
    assert kR.tobytes() == g2["kps_right"].tobytes()
    bf, fx, mb = g2["camera"]
    u, dep = amd.compute_stereo_matches(exL, exR, len(kL), float(bf), float(mb))
    assert u.tobytes() == g2["u_right"].tobytes() and dep.tobytes() == g2["depth"].tobytes()


@pytest.mark.parametrize("case", ["wide", "tall", "small_level", "scale_factor", "bad_mode"])
def test_extract_input_limits(amd, case):
    """The extractor's documented input range (include/orbslam2_amd.h, orbx_params): width / height
    <= 4000, every pyramid level >= 40 x 40, scaleFactor <= 2, resize_mode / blur_mode in {0, 1}.
    Outside it the call fails with ORBX_EINVAL (status -1) and the engine stays usable."""
    if case == "bad_mode":
        with pytest.raises(amd.OrbslamError, match="status -1"):
            amd.ORBextractor(1000, blur_mode=2)
        return
    shape, kw = {"wide": ((400, 4001), {}), "tall": ((4001, 400), {}), "small_level": ((120, 160), {}),
                 "scale_factor": ((480, 640), {"scaleFactor": 2.5, "nlevels": 3})}[case]
    ex = amd.ORBextractor(1000, **kw)
    with pytest.raises(amd.OrbslamError, match="status -1"):
        ex(np.zeros(shape, np.uint8))
    if case != "scale_factor":   # a refused size leaves the engine usable
        k, _ = ex(synth.textured_image(480, 640, 3))
        assert len(k) > 0
