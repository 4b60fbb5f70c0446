"""ORBmatcher handle entries (orbm_create / orbm_*) vs the CPU oracle.

* SearchForInitialization on two independently built host frames, called frame after frame
  against a fixed initial frame with vbPrevMatched carried between calls, exactly as
  Tracking::MonocularInitialization does (Tracking.cc:893-897, 929-933; ORBmatcher.cc:580-748,
  the window centre read at :627 and rewritten at :742-745). Bit-exact vnMatches12, return value
  and vbPrevMatched after every call.
* The candidate-list Hamming scan (SURVEY.md §8b orbm_hamming_best2(q, db, cand_off, cand_idx))
  against the reference's best / second-best loop (ORBmatcher.cc:639-668) restated below.
"""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu
K_TUM = [517.306408, 516.469215, 318.643040, 255.313989]
D_TUM = [0.262383, -0.953104, -0.005358, 0.002628, 1.163314]


def _frame(oracle_mod, t, nfeat=1000, dist=D_TUM):
    gray, _ = synth.rgbd_frame(480, 640, t)
    k, d = oracle_mod.Extractor(nfeat).extract(gray)
    ku = k.copy()
    if dist[0] != 0:
        xy = oracle_mod.undistort_points(np.stack([k["x"], k["y"]], 1), K_TUM, dist)
        ku["x"], ku["y"] = xy[:, 0], xy[:, 1]
    return ku, d


@pytest.mark.parametrize("t0,steps,window,nnratio,check_ori", [(0, 5, 100, 0.9, True), (30, 5, 50, 0.9, True),
                                                               (60, 4, 200, 0.7, False)])
def test_search_for_initialization_chain(amd, oracle_mod, t0, steps, window, nnratio, check_ori):
    bounds = oracle_mod.image_bounds(640, 480, K_TUM, D_TUM)
    ku1, d1 = _frame(oracle_mod, t0)
    G1 = oracle_mod.Grid(ku1, d1, bounds)
    prev_ref = np.stack([ku1["x"], ku1["y"]], 1).astype(np.float32)   # mvbPrevMatched = F1 keysUn
    prev_gpu = prev_ref.copy()
    m = amd.ORBmatcher(nnratio, check_ori)
    total = 0
    for s in range(1, steps + 1):
        ku2, d2 = _frame(oracle_mod, t0 + s)
        G2 = oracle_mod.Grid(ku2, d2, bounds)
        nm, m12, prev_ref = oracle_mod.search_for_initialization(G1, G2, prev_ref, window, nnratio, check_ori)
        gn, gm = m.SearchForInitialization((ku1, d1, bounds), (ku2, d2, bounds), prev_gpu, window)
        assert gn == nm, f"call {s}"
        np.testing.assert_array_equal(gm, m12)
        assert prev_gpu.tobytes() == prev_ref.tobytes(), f"vbPrevMatched after call {s}"
        total += nm
    assert total > 40, "consecutive synthetic frames should match"
    m.close()


def test_search_for_initialization_edges(amd, oracle_mod):
    bounds = oracle_mod.image_bounds(640, 480, K_TUM, D_TUM)
    ku1, d1 = _frame(oracle_mod, 3)
    m = amd.ORBmatcher(0.9, True)
    empty = (ku1[:0], d1[:0], bounds)
    # empty F2: no candidates, prev untouched
    prev = np.stack([ku1["x"], ku1["y"]], 1).astype(np.float32)
    before = prev.copy()
    n, m12 = m.SearchForInitialization((ku1, d1, bounds), empty, prev, 100)
    assert n == 0 and (m12 == -1).all() and prev.tobytes() == before.tobytes()
    # empty F1: empty vnMatches12
    n, m12 = m.SearchForInitialization(empty, (ku1, d1, bounds), np.zeros((0, 2), np.float32), 100)
    assert n == 0 and len(m12) == 0
    # a frame against itself: every octave-0 keypoint finds itself unless ratio / duplicates reject it
    prev = np.stack([ku1["x"], ku1["y"]], 1).astype(np.float32)
    prev_ref = prev.copy()
    G1 = oracle_mod.Grid(ku1, d1, bounds)
    nm, r12, prev_ref = oracle_mod.search_for_initialization(G1, G1, prev_ref, 100, 0.9, True)
    n, m12 = m.SearchForInitialization((ku1, d1, bounds), (ku1, d1, bounds), prev, 100)
    assert n == nm and np.array_equal(m12, r12) and prev.tobytes() == prev_ref.tobytes()


def _best2_ref(q, db, off, idx):
    """ORBmatcher.cc:639-668 loop over each candidate list, in list order."""
    qa = np.unpackbits(q, axis=1).astype(np.int32)
    da = np.unpackbits(db, axis=1).astype(np.int32)
    bi = np.full(len(q), -1, np.int32)
    bd = np.full(len(q), 2**31 - 1, np.int32)
    sd = np.full(len(q), 2**31 - 1, np.int32)
    for i in range(len(q)):
        cand = idx[off[i]:off[i + 1]]
        if len(cand) == 0:
            continue
        dists = (qa[i][None, :] != da[cand]).sum(1)
        best, best2, bidx = 2**31 - 1, 2**31 - 1, -1
        for c, d in zip(cand, dists):
            if d < best:
                best2, best, bidx = best, int(d), int(c)
            elif d < best2:
                best2 = int(d)
        bi[i], bd[i], sd[i] = bidx, best, best2
    return bi, bd, sd


def test_hamming_best2_candidate_lists(amd):
    rng = np.random.default_rng(11)
    db = rng.integers(0, 256, size=(3000, 32), dtype=np.uint8)
    db[2000:2100] = db[:100]                       # duplicate rows: equal distances at two indices
    nq = 700
    q = db[rng.integers(0, 3000, nq)].copy()
    q[::3, 5] ^= 0x11
    lens = rng.integers(0, 90, nq)
    lens[::17] = 0                                  # empty lists
    lens[5] = 1
    lens[7] = 300                                   # longer than a wavefront
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    idx = rng.integers(0, 3000, off[-1]).astype(np.int32)
    # lists that hold the same row twice and both duplicates: first minimum in list order wins
    idx[off[9]:off[9] + 4] = [2050, 50, 50, 2050]
    q[9] = db[50]
    m = amd.ORBmatcher()
    bi, bd, sd = m.hamming_best2_cand(q, db, off, idx)
    ri, rd, rs = _best2_ref(q, db, off, idx)
    np.testing.assert_array_equal(bi, ri)
    np.testing.assert_array_equal(bd, rd)
    np.testing.assert_array_equal(sd, rs)
    assert bi[9] == 2050 and bd[9] == 0 and sd[9] == 0
    # without lists = the brute-force entry
    bi2, bd2, sd2 = m.hamming_best2_cand(q, db)
    fi, fd, fs = amd.ORBmatcher.hamming_best2(q, db)
    assert np.array_equal(bi2, fi) and np.array_equal(bd2, fd) and np.array_equal(sd2, fs)
    m.close()


def _random_frame(rng, n, bounds):
    """n keypoints spread over the image, every third of octave 0 (the ones SearchForInitialization
    queries), random angles / descriptors."""
    k = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    k["x"] = rng.uniform(bounds[0], bounds[1], n).astype(np.float32)
    k["y"] = rng.uniform(bounds[2], bounds[3], n).astype(np.float32)
    k["size"] = 31
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["octave"] = np.where(np.arange(n) % 3 == 0, 0, rng.integers(1, 8, n))
    k["class_id"] = -1
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return k, d


@pytest.mark.parametrize("n", [4094, 4096])
def test_search_for_initialization_max_frame(amd, oracle_mod, n):
    """The documented limit F1->n, F2->n <= 4096 (orbslam2_amd.h) holds at the limit; 4097 is refused."""
    rng = np.random.default_rng(n)
    bounds = oracle_mod.image_bounds(640, 480, K_TUM, D_TUM)
    k1, d1 = _random_frame(rng, n, bounds)
    k2 = k1.copy()                                   # F2: F1 shifted by < 2 px, descriptors with a few flips
    k2["x"] += rng.uniform(-2, 2, n).astype(np.float32)
    k2["y"] += rng.uniform(-2, 2, n).astype(np.float32)
    k2["angle"] = np.mod(k2["angle"] + rng.uniform(-5, 5, n), 360).astype(np.float32)
    d2 = d1.copy()
    d2[:, 3] ^= rng.integers(0, 256, n, dtype=np.uint8) & 0x21
    G1, G2 = oracle_mod.Grid(k1, d1, bounds), oracle_mod.Grid(k2, d2, bounds)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    nm, r12, prev_ref = oracle_mod.search_for_initialization(G1, G2, prev.copy(), 20, 0.9, True)
    m = amd.ORBmatcher(0.9, True)
    gn, g12 = m.SearchForInitialization((k1, d1, bounds), (k2, d2, bounds), prev, 20)
    assert gn == nm and nm > n // 6
    np.testing.assert_array_equal(g12, r12)
    assert prev.tobytes() == prev_ref.tobytes()
    k3, d3 = _random_frame(rng, 4097, bounds)
    with pytest.raises(amd.OrbslamError):
        m.SearchForInitialization((k3, d3, bounds), (k2, d2, bounds), np.zeros((4097, 2), np.float32), 20)
    m.close()
