"""CPU-only checks of the oracle (test infrastructure) — no GPU.

* the C oracle's FAST / IC_Angle / BRIEF / blur / Hamming against the independent numpy
  restatement (oracle/np_ref.py);
* the reformulated quadtree used by the HIP kernel (descending creation order, SURVEY.md
  §8a E4) modelled in Python against the oracle's literal std::list restatement;
* extractor tables against the values derived in SURVEY.md §8.
"""
import numpy as np
import pytest

import np_ref

SURVEY_SCALES = [1, 1.2, 1.44, 1.728, 2.0736, 2.48832, 2.98598, 3.58318]


def test_tables_match_survey(oracle_mod):
    ex = oracle_mod.Extractor(1000)
    assert ex.features_per_level == [217, 181, 151, 126, 105, 87, 73, 60]
    ex2 = oracle_mod.Extractor(2000)
    assert ex2.features_per_level == [434, 362, 302, 251, 209, 175, 145, 122]
    np.testing.assert_allclose(ex.scale_factors, SURVEY_SCALES, rtol=2e-6)
    assert list(ex.umax) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    assert list(np_ref.umax_table()) == list(ex.umax)
    pat = ex.pattern.reshape(256, 4)
    assert np.abs(pat).max() <= 13 and pat[0].tolist() == [8, -3, 9, 5]


@pytest.mark.parametrize("seed", range(6))
def test_fast_roi_vs_numpy(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    h, w = rng.integers(7, 44), rng.integers(7, 44)
    if seed % 2:
        roi = rng.integers(0, 256, (h, w), dtype=np.uint8)
    else:
        roi = np.clip(rng.normal(128, 40, (h, w)), 0, 255).astype(np.uint8)
    for th in (7, 20, 0, 1, 60):
        x1, y1, s1 = oracle_mod.fast_roi(roi, th)
        x2, y2, s2 = np_ref.fast_roi(roi, th)
        np.testing.assert_array_equal(x1, x2)
        np.testing.assert_array_equal(y1, y2)
        np.testing.assert_array_equal(s1, s2)


def test_blur_vs_numpy(oracle_mod):
    rng = np.random.default_rng(1)
    for h, w in [(40, 50), (105, 346), (9, 9)]:
        img = rng.integers(0, 256, (h, w), dtype=np.uint8)
        np.testing.assert_array_equal(oracle_mod.gaussian_blur9(img), np_ref.gaussian_blur9(img))


def test_ic_angle_and_brief_vs_numpy(oracle_mod):
    from orbslam2_amd import synth
    img = synth.textured_image(120, 160, 4)
    blur = oracle_mod.gaussian_blur9(img)
    ex = oracle_mod.Extractor(500)
    um, pat = ex.umax, ex.pattern
    rng = np.random.default_rng(2)
    for _ in range(200):
        x, y = int(rng.integers(20, 140)), int(rng.integers(20, 100))
        a1 = np.float32(oracle_mod.ic_angle(img, x, y, um))
        a2 = np_ref.ic_angle(img, x, y, um)
        assert a1.view(np.uint32) == a2.view(np.uint32)
        ang = np.float32(a1) * np.float32(np.pi / 180.0)
        ca = np.float32(oracle_mod.lib().orc_cosf(ang))
        sa = np.float32(oracle_mod.lib().orc_sinf(ang))
        d1 = oracle_mod.orb_descriptor(blur, x, y, float(a1), pat)
        d2 = np_ref.brief(blur, x, y, ca, sa, pat)
        np.testing.assert_array_equal(d1, d2)


def test_fast_atan2_vs_numpy(oracle_mod):
    rng = np.random.default_rng(5)
    vals = np.concatenate([rng.integers(-200000, 200000, (500, 2)), [[0, 0], [0, 5], [5, 0], [-3, 0], [0, -3], [7, 7], [-7, 7]]])
    for y, x in vals:
        a = np.float32(oracle_mod.lib().orc_fast_atan2(float(y), float(x)))
        b = np_ref.fast_atan2(np.float32(y), np.float32(x))
        assert a.view(np.uint32) == b.view(np.uint32), (y, x, a, b)


def test_hamming_vs_numpy(oracle_mod):
    rng = np.random.default_rng(9)
    a = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    ref = np_ref.hamming(a, b)
    got = [oracle_mod.descriptor_distance(a[i], b[i]) for i in range(100)]
    np.testing.assert_array_equal(got, ref)


def test_sincosf_restatement_matches_libm(oracle_mod):
    """Spot check here (full exhaustive pin: oracle/tools/check_sincosf.c)."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.cosf.restype = libm.sinf.restype = ctypes.c_float
    libm.cosf.argtypes = libm.sinf.argtypes = [ctypes.c_float]
    rng = np.random.default_rng(3)
    degs = np.concatenate([rng.uniform(0, 360, 20000).astype(np.float32), np.float32([0, 45, 90, 180, 270, 359.99997, 360])])
    fpi = np.float32(np.pi / 180.0)
    for d in degs:
        x = float(np.float32(d) * fpi)
        assert np.float32(libm.cosf(x)) == np.float32(oracle_mod.lib().orc_cosf(x))
        assert np.float32(libm.sinf(x)) == np.float32(oracle_mod.lib().orc_sinf(x))


# ---------------------------------------------------------------------------
# Quadtree reformulation model (what quadtree_kernel implements)
# ---------------------------------------------------------------------------
def qt_model(keys, minX, maxX, minY, maxY, N):
    f = np.float32
    nIni = int(np.floor(abs(f(maxX - minX) / f(maxY - minY)) + f(0.5)))
    hX = f(maxX - minX) / f(nIni)
    H = maxY - minY
    roots = [[] for _ in range(nIni)]
    for k in keys:
        roots[min(int(f(k["x"]) / hX), nIni - 1)].append(k)
    out, active = [], []
    live, next_id = 0, nIni
    for r in range(nIni):
        if not roots[r]:
            continue
        live += 1
        box = (int(hX * f(r)), 0, int(hX * f(r + 1)), H)
        if len(roots[r]) == 1:
            out.append((-1 - r, roots[r][0]))
        else:
            active.append((box, roots[r], -1 - r))

    def divide(node):
        (x0, y0, x1, y1), ks, _ = node
        hx = int(np.ceil(f(x1 - x0) / f(2)))
        hy = int(np.ceil(f(y1 - y0) / f(2)))
        mx, my = x0 + hx, y0 + hy
        boxes = [(x0, y0, mx, my), (mx, y0, x1, my), (x0, my, mx, y1), (mx, my, x1, y1)]
        ch = [[], [], [], []]
        for k in ks:
            ch[(1 if k["x"] >= mx else 0) + (2 if k["y"] >= my else 0)].append(k)
        return list(zip(boxes, ch))

    def best(ks):
        b = ks[0]
        for k in ks[1:]:
            if k["response"] > b["response"]:
                b = k
        return b

    def split(node, sink):
        nonlocal live, next_id
        ne = 0
        for box, ks in divide(node):
            if not ks:
                continue
            ne += 1
            nid = next_id
            next_id += 1
            if len(ks) == 1:
                out.append((nid, ks[0]))
            else:
                sink.append((box, ks, nid))
        live += ne - 1

    reverse = False
    final = False
    while True:
        prev = live
        new = []
        for node in (active[::-1] if reverse else active):
            split(node, new)
        active, reverse = new, True
        if live >= N or live == prev:
            break
        if live + 3 * len(active) > N:
            final = True
            break
    if final:
        while True:
            prev = live
            srt = sorted(active, key=lambda n: (len(n[1]), n[2]), reverse=True)
            new = []
            crossed = False
            for node in srt:
                if crossed:
                    out.append((node[2], best(node[1])))
                    continue
                split(node, new)
                if live >= N:
                    crossed = True
            active = new
            if live >= N or live == prev:
                break
    for node in active:
        out.append((node[2], best(node[1])))
    out.sort(key=lambda t: t[0], reverse=True)
    return [k for _, k in out]


def _rand_keys(rng, n, w, h, dup=False):
    from oracle import KP_DTYPE
    xs = rng.integers(3, w - 3, n * 3)
    ys = rng.integers(3, h - 3, n * 3)
    pts = list(dict.fromkeys(zip(xs.tolist(), ys.tolist())))[:n]
    if dup and pts:
        pts += pts[: max(1, len(pts) // 10)]
    k = np.zeros(len(pts), KP_DTYPE)
    k["x"] = [p[0] for p in pts]
    k["y"] = [p[1] for p in pts]
    k["response"] = rng.integers(7, 40, len(pts))   # many response ties
    k["size"] = 7
    k["angle"] = -1
    k["class_id"] = -1
    return k


@pytest.mark.parametrize("seed", range(40))
def test_quadtree_model_matches_list_restatement(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    W = int(rng.choice([147, 314, 608, 1002, 1209]))
    Hh = int(rng.choice([73, 120, 281, 344, 448]))
    if W / Hh < 0.5:          # nIni == 0: the reference divides by zero (ORBextractor.cc:703)
        W, Hh = Hh, W
    n = int(rng.choice([0, 1, 2, 5, 40, 300, 1500]))
    N = int(rng.choice([0, 1, 3, 60, 217, 434, 2000]))
    keys = _rand_keys(rng, n, W, Hh, dup=(seed % 7 == 3))
    ref = oracle_mod.distribute_octtree(keys, 16, 16 + W, 16, 16 + Hh, N)
    got = qt_model(keys, 16, 16 + W, 16, 16 + Hh, N)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert (g["x"], g["y"], g["response"]) == (r["x"], r["y"], r["response"])
