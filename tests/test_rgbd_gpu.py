"""GPU C3 path vs the CPU oracle: UndistortKeyPoints + ComputeStereoFromRGBD (Frame.cc:725-776,
1131-1169) and SearchForInitialization over consecutive frames (ORBmatcher.cc:580-748) with
the TUM1 camera (Examples/RGB-D/TUM1.yaml). Bit-exact keypoints / depths / match indices."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu
K_TUM = [517.306408, 516.469215, 318.643040, 255.313989]
D_TUM = [0.262383, -0.953104, -0.005358, 0.002628, 1.163314]
BF_TUM = 40.0


def _oracle_frame(oracle_mod, gray, depth, K, D):
    ex = oracle_mod.Extractor(1000)
    k, d = ex.extract(gray)
    if D[0] != 0:
        xy = oracle_mod.undistort_points(np.stack([k["x"], k["y"]], 1), K, D)
        ku = k.copy()
        ku["x"], ku["y"] = xy[:, 0], xy[:, 1]
    else:
        ku = k.copy()
    u, dep = oracle_mod.stereo_from_rgbd(k, ku, depth, BF_TUM)
    return k, d, ku, u, dep


@pytest.mark.parametrize("dist", [D_TUM, [0, 0, 0, 0, 0]])
def test_rgbd_and_search_init(amd, oracle_mod, dist):
    import torch
    T = 4
    frames = [synth.rgbd_frame(480, 640, t) for t in range(T)]
    grays = np.stack([f[0] for f in frames])
    depths = np.stack([f[1] for f in frames])
    dg = torch.from_numpy(grays).cuda()
    dd = torch.from_numpy(depths).cuda()
    ex = amd.BatchExtractor(1000)
    ex.reserve(640, 480, T)
    torch.cuda.synchronize()
    ex.extract_device(dg.data_ptr(), T, 640, 480, 640, 640 * 480)
    ex.rgbd_device(dd.data_ptr(), 640 * 480, 640, K_TUM, dist, BF_TUM)
    ex.search_init_device(T - 1, 0, 1, 1, 1, K_TUM, dist, 100, 0.9, True)
    bounds = oracle_mod.image_bounds(640, 480, K_TUM, dist)
    ref = [_oracle_frame(oracle_mod, grays[t], depths[t], K_TUM, dist) for t in range(T)]
    for t in range(T):
        k, d, ku, u, dep = ref[t]
        gku, gu, gd = ex.rgbd_fetch(t)
        n = len(k)
        assert gku[:n].tobytes() == ku.tobytes(), f"keysUn frame {t}"
        assert gu[:n].tobytes() == u.tobytes() and gd[:n].tobytes() == dep.tobytes(), f"depth frame {t}"
    for p in range(T - 1):
        k1, d1, ku1, _, _ = ref[p]
        k2, d2, ku2, _, _ = ref[p + 1]
        G1 = oracle_mod.Grid(ku1, d1, bounds)
        G2 = oracle_mod.Grid(ku2, d2, bounds)
        prev = np.stack([ku1["x"], ku1["y"]], 1)
        nm, m12, prev_out = oracle_mod.search_for_initialization(G1, G2, prev, 100, 0.9, True)
        gn, gm, gxy = ex.search_init_fetch(p)
        n1 = len(k1)
        assert nm > 20, "consecutive synthetic frames should match"
        np.testing.assert_array_equal(gm[:n1], m12)
        assert gn == nm
        assert gxy[:n1].tobytes() == prev_out.tobytes()


def test_rgbd_host_path(amd, oracle_mod):
    gray, depth = synth.rgbd_frame(480, 640, 5)
    ex = amd.ORBextractor(1000)
    k, _ = ex(gray)
    ku, u, d = amd.compute_stereo_from_rgbd(ex, len(k), depth, K_TUM, D_TUM, BF_TUM)
    rk, rd, rku, ru, rdep = _oracle_frame(oracle_mod, gray, depth, K_TUM, D_TUM)
    assert ku.tobytes() == rku.tobytes() and u.tobytes() == ru.tobytes() and d.tobytes() == rdep.tobytes()


@pytest.mark.parametrize("window,nnratio,check_ori,gap", [(50, 0.9, True, 1), (200, 0.9, True, 2),
                                                          (100, 0.7, False, 1), (100, 0.95, True, 3)])
def test_search_init_variants(amd, oracle_mod, window, nnratio, check_ori, gap):
    """Two-phase GPU SearchForInitialization (candidate lists, then the greedy claim walk) vs the
    oracle over windows, ratios, rotation check on/off and frames `gap` apart (larger motion,
    more evictions)."""
    import torch
    T = 6
    frames = [synth.rgbd_frame(480, 640, 10 + t) for t in range(T)]
    grays = np.stack([f[0] for f in frames])
    depths = np.stack([f[1] for f in frames])
    dg = torch.from_numpy(grays).cuda()
    dd = torch.from_numpy(depths).cuda()
    ex = amd.BatchExtractor(1000)
    ex.reserve(640, 480, T)
    torch.cuda.synchronize()
    ex.extract_device(dg.data_ptr(), T, 640, 480, 640, 640 * 480)
    ex.rgbd_device(dd.data_ptr(), 640 * 480, 640, K_TUM, D_TUM, BF_TUM)
    n_pairs = T - gap
    ex.search_init_device(n_pairs, 0, 1, gap, 1, K_TUM, D_TUM, window, nnratio, check_ori)
    bounds = oracle_mod.image_bounds(640, 480, K_TUM, D_TUM)
    ref = [_oracle_frame(oracle_mod, grays[t], depths[t], K_TUM, D_TUM) for t in range(T)]
    for p in range(n_pairs):
        k1, d1, ku1, _, _ = ref[p]
        k2, d2, ku2, _, _ = ref[p + gap]
        G1 = oracle_mod.Grid(ku1, d1, bounds)
        G2 = oracle_mod.Grid(ku2, d2, bounds)
        prev = np.stack([ku1["x"], ku1["y"]], 1)
        nm, m12, prev_out = oracle_mod.search_for_initialization(G1, G2, prev, window, nnratio, check_ori)
        gn, gm, gxy = ex.search_init_fetch(p)
        n1 = len(k1)
        np.testing.assert_array_equal(gm[:n1], m12)
        assert gn == nm
        assert gxy[:n1].tobytes() == prev_out.tobytes()


@pytest.mark.parametrize("flush", [False, True], ids=["resident", "flush_at_allocation_end"])
def test_c3_production_shape(amd, oracle_mod, flush):
    """C3 at bench.py's production shape (shapes.C3_BATCH frames per batch, shapes.C3_ENGINES
    engines -- the constants bench.py's defaults read): consecutive batches
    alternating over the engines on their own streams with no synchronisation between them
    (bench_rgbd), each batch = extract(1000) + UndistortKeyPoints + ComputeStereoFromRGBD +
    SearchForInitialization over its 255 consecutive pairs. E + 1 batches (engine 0 reused while the
    others are in flight), batch b from the 8-frame pool shifted by 3b: every frame's keysUn /
    mvuRight / mvDepth and every pair's vnMatches12 / vbPrevMatched / count bit-exact. `flush`: each
    batch's gray images and depth maps end on the last byte of their own fresh 2 MiB-multiple
    allocation (256 VGA images are 75 MiB: the gray batch starts 1 MiB into a 76 MiB allocation).
    Reference: Frame.cc:725-776, 1131-1169; ORBmatcher.cc:580-748."""
    import torch
    from orbslam2_amd import shapes
    T, E = shapes.C3_BATCH, shapes.C3_ENGINES
    NB = E + 1
    assert (T, E) == (256, 4)
    pool = [synth.rgbd_frame(480, 640, t) for t in range(8)]
    ref = [_oracle_frame(oracle_mod, g, d, K_TUM, D_TUM) for g, d in pool]
    bounds = oracle_mod.image_bounds(640, 480, K_TUM, D_TUM)
    pair_ref = {}
    for a in range(8):
        b = (a + 1) % 8
        k1, d1, ku1, _, _ = ref[a]
        _, d2, ku2, _, _ = ref[b]
        prev = np.stack([ku1["x"], ku1["y"]], 1)
        pair_ref[a] = oracle_mod.search_for_initialization(oracle_mod.Grid(ku1, d1, bounds),
                                                           oracle_mod.Grid(ku2, d2, bounds), prev, 100, 0.9, True)
    def flush_copy(a):   # a device copy of `a` ending on the last byte of a 2 MiB-multiple allocation
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        alloc = -(-raw.size // (2 << 20)) * (2 << 20)
        buf = torch.empty(alloc, dtype=torch.uint8, device="cuda")
        buf[alloc - raw.size:].copy_(torch.from_numpy(raw))
        return buf, buf.data_ptr() + alloc - raw.size

    torch.cuda.empty_cache()
    ins = []
    for bi in range(NB):
        idx = [(t + 3 * bi) % 8 for t in range(T)]
        gs, ds = np.stack([pool[i][0] for i in idx]), np.stack([pool[i][1] for i in idx])
        if flush:
            (gb, gp), (db, dp) = flush_copy(gs), flush_copy(ds)
        else:
            gb, db = torch.from_numpy(gs).cuda(), torch.from_numpy(ds).cuda()
            gp, dp = gb.data_ptr(), db.data_ptr()
        ins.append((idx, gb, db, gp, dp))
    exs = [amd.BatchExtractor(1000) for _ in range(E)]
    for ex in exs:
        ex.reserve(640, 480, T)
    torch.cuda.synchronize()
    for bi in range(NB):   # bench_rgbd's step, back to back
        _, _, _, gp, dp = ins[bi]
        ex = exs[bi % E]
        ex.extract_device(gp, T, 640, 480, 640, 640 * 480)
        ex.rgbd_device(dp, 640 * 480, 640, K_TUM, D_TUM, BF_TUM)
        ex.search_init_device(T - 1, 0, 1, 1, 1, K_TUM, D_TUM, 100, 0.9, True)
    amd.device_sync()
    for bi in range(1, NB):   # batch 0's engine was reused by batch E
        idx = ins[bi][0]
        ex = exs[bi % E]
        for t in range(T):
            k, _, ku, u, dep = ref[idx[t]]
            gku, gu, gd = ex.rgbd_fetch(t)
            n = len(k)
            assert gku[:n].tobytes() == ku.tobytes(), f"keysUn batch {bi} frame {t}"
            assert gu[:n].tobytes() == u.tobytes() and gd[:n].tobytes() == dep.tobytes(), f"depth batch {bi} frame {t}"
        for p in range(T - 1):
            nm, m12, prev_out = pair_ref[idx[p]]
            gn, gm, gxy = ex.search_init_fetch(p)
            n1 = len(ref[idx[p]][0])
            assert gn == nm, f"batch {bi} pair {p}"
            np.testing.assert_array_equal(gm[:n1], m12)
            assert gxy[:n1].tobytes() == prev_out.tobytes(), f"vbPrevMatched batch {bi} pair {p}"


def test_golden_c3_on_device(amd):
    """HIP C3 path == the committed fixture tests/golden/c3_rgbd_640x480.npz (no oracle at run time)."""
    import torch
    from test_golden_cpu import load_c3
    frames, g = load_c3()
    cam = g["camera"]
    K, D, bf = list(cam[:4]), list(cam[4:9]), float(cam[9])
    dg = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    dd = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    ex = amd.BatchExtractor(1000)
    ex.reserve(640, 480, 2)
    torch.cuda.synchronize()
    ex.extract_device(dg.data_ptr(), 2, 640, 480, 640, 640 * 480)
    ex.rgbd_device(dd.data_ptr(), 640 * 480, 640, K, D, bf)
    ex.search_init_device(1, 0, 1, 1, 1, K, D, 100, 0.9, True)
    for t in (0, 1):
        gku, gu, gd = ex.rgbd_fetch(t)
        n = len(g[f"keys_un{t}"])
        assert gku[:n].tobytes() == g[f"keys_un{t}"].tobytes()
        assert gu[:n].tobytes() == g[f"u_right{t}"].tobytes() and gd[:n].tobytes() == g[f"depth_out{t}"].tobytes()
    gn, gm, gxy = ex.search_init_fetch(0)
    n1 = len(g["matches12"])
    assert gn == int(g["nmatches"])
    assert gm[:n1].tobytes() == g["matches12"].tobytes() and gxy[:n1].tobytes() == g["prev_matched"].tobytes()
