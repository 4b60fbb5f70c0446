"""CPU checks of the tracking-matcher oracle (oracle/track_oracle.c) and its host plumbing."""
import ctypes
import ctypes.util

import numpy as np

from orbslam2_amd import synth


def test_logf_restatement_matches_libm(oracle_mod):
    """Spot check (full exhaustive pin over every positive float: oracle/tools/check_logf.c)."""
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.logf.argtypes = [ctypes.c_float]
    libm.logf.restype = ctypes.c_float
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(0.05, 20, 3000), 1.2 ** np.arange(-20, 20), [1.0, 1e-40, 3e38]]).astype(np.float32)
    for x in xs:
        assert np.float32(oracle_mod.logf(float(x))) == np.float32(libm.logf(float(x))), x


def _tiny(flags0=2, flags1=2):
    """Two map points at the same place, one keypoint: the greedy claim order decides."""
    p = synth.tracking_problem(1, n_kp=50, n_mp=20)
    fr = p["frame"]
    kp = fr["keys_un"].copy()
    kp["octave"] = 0
    R = np.asarray(fr["Tcw"], np.float64)[:, :3]
    t = np.asarray(fr["Tcw"], np.float64)[:, 3]
    Pc = np.array([0.5, 0.2, 10.0])
    Xw = R.T @ (Pc - t)
    u = fr["fx"] * Pc[0] / Pc[2] + fr["cx"]
    v = fr["fy"] * Pc[1] / Pc[2] + fr["cy"]
    kp["x"][0], kp["y"][0] = u + 0.3, v - 0.2
    kp["x"][1:] = 5.0
    kp["y"][1:] = 5.0
    desc = fr["desc"].copy()
    mdesc = np.stack([desc[0], desc[0]])
    mdesc[1, 0] ^= 1
    Ow = np.asarray(fr["Ow"], np.float64)
    d = np.linalg.norm(Xw - Ow)
    nrm = (Xw - Ow) / d
    mp = {"Xw": np.stack([Xw, Xw]).astype(np.float32), "normal": np.stack([nrm, nrm]).astype(np.float32),
          "max_dist": np.array([0.999 * d, 0.999 * d], np.float32), "min_dist": np.array([d / 4, d / 4], np.float32),
          "desc": mdesc, "flags": np.array([flags0, flags1], np.uint8)}
    fr = dict(fr, keys_un=kp, desc=desc, u_right=np.full(len(kp), -1, np.float32))
    return dict(p, frame=fr, map=mp, kp_blocked=None)


def test_local_greedy_claim_order(oracle_mod):
    nm, own, view = oracle_mod.search_local_points(_tiny(2, 2))
    assert view["in_view"].tolist() == [1, 1] and view["level"].tolist() == [0, 0]
    assert nm == 1 and own[0] == 0              # the second point finds the keypoint claimed
    nm, own, _ = oracle_mod.search_local_points(_tiny(0, 2))
    assert nm == 2 and own[0] == 1              # first owner has no observations: overwritten
    nm, own, _ = oracle_mod.search_local_points(_tiny(1, 2))
    assert nm == 1 and own[0] == 1              # a bad point is skipped
    nm, own, view = oracle_mod.search_local_points(_tiny(4 | 2, 2))
    assert view["in_view"][0] == 0 and own[0] == 1   # already in the frame: not projected


def test_frame_matcher_runs_all_motions(oracle_mod):
    for motion in ("forward", "backward", "static"):
        p = synth.tracking_problem(3, motion=motion)
        nm, own = oracle_mod.search_by_projection_frame(p)
        assert (own >= 0).sum() > 0 and (own == -2).sum() > 0
        assert nm > 0


def test_crowd_claims_in_order(oracle_mod):
    from track_cases import crowd_problem
    p = crowd_problem()
    nm, own, view = oracle_mod.search_local_points(p)
    assert view["in_view"].all() and (view["level"] == 1).all()
    # keypoint j (distance 8j <= 100 -> j <= 12) goes to map point j, in the greedy order
    assert nm == 12 and own[:12].tolist() == list(range(12))
    nm, own = oracle_mod.search_by_projection_frame(p, th=15.0, check_ori=False)
    assert nm > 4 and own[0] == 0


def test_reloc_projection_rules(oracle_mod):
    """ORBmatcher.cc:1922-2066 invariants on the oracle: points in sAlreadyFound or bad never
    match, keypoints holding a map point on entry are never reassigned, every claim is
    exclusive (a keypoint is owned by one point), distances respect ORBdist."""
    import numpy as np
    from orbslam2_amd import synth
    p = synth.reloc_problem(42)
    flags = p["map"]["flags"]
    for th, od in ((10.0, 100), (3.0, 64)):
        nm, own = oracle_mod.search_by_projection_keyframe(p, th=th, orb_dist=od, check_ori=False)
        got = own[own >= 0]
        assert nm == len(got) > 50
        assert len(np.unique(got)) == len(got)
        assert not (flags[got] & (synth.MP_FOUND | synth.MP_BAD)).any()
        assert (own[p["kp_blocked"] == 1] == -1).all()
        d = np.unpackbits(p["map"]["desc"][got] ^ p["frame"]["desc"][own >= 0], axis=1).sum(1)
        assert (d <= od).all()
