"""GPU tracking matchers vs the CPU oracle, bit-exact.

Frame::isInFrustum (Frame.cc:490-578) outputs (mbTrackInView, mTrackProjX/Y/XR,
mTrackViewCos, mnTrackScaleLevel) and the keypoint -> map point assignment of both
ORBmatcher::SearchByProjection overloads used by Tracking (ORBmatcher.cc:78-176,
1741-1904), including the greedy claim order and the rotation-consistency removals, must
equal the oracle's bytes. Inputs are seeded synthetic frames / maps (synth.tracking_problem;
keypoints are projections of map points with noise, not extracted) -- the reference ships no
fixtures for these functions: parity against a real build is unpinned.
"""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tracker(amd):
    t = amd.Tracker()
    yield t
    t.close()


def _cmp_view(got, ref):
    for k in ("in_view", "proj_x", "proj_y", "proj_xr", "view_cos", "level"):
        assert got[k].tobytes() == ref[k].tobytes(), k


@pytest.mark.parametrize("seed,n_kp,n_mp,th,stereo", [
    (5, 2000, 3000, 1.0, True), (6, 2000, 3000, 3.0, True), (7, 1000, 1500, 5.0, False),
    (8, 4000, 6000, 1.0, True), (9, 300, 200, 1.0, True), (10, 2000, 3000, 1.0, False)])
def test_search_local_points(tracker, oracle_mod, seed, n_kp, n_mp, th, stereo):
    p = synth.tracking_problem(seed, n_kp=n_kp, n_mp=n_mp, stereo=stereo)
    nm_r, own_r, view_r = oracle_mod.search_local_points(p, th=th, nnratio=0.8)
    nm_g, own_g, view_g = tracker.search_local_points(p, th=th, nnratio=0.8)
    _cmp_view(view_g, view_r)
    assert nm_g == nm_r
    assert np.array_equal(own_g, own_r)
    assert nm_r > 50


@pytest.mark.parametrize("seed,motion,mono,check_ori,th", [
    (11, "forward", False, True, 15.0), (12, "backward", False, True, 15.0), (13, "static", False, True, 15.0),
    (14, "forward", True, True, 7.0), (15, "static", False, False, 15.0), (16, "forward", False, True, 30.0)])
def test_search_by_projection_frame(tracker, oracle_mod, seed, motion, mono, check_ori, th):
    p = synth.tracking_problem(seed, motion=motion, stereo=not mono)
    nm_r, own_r = oracle_mod.search_by_projection_frame(p, th=th, mono=mono, check_ori=check_ori)
    nm_g, own_g = tracker.search_by_projection_frame(p, th=th, mono=mono, check_ori=check_ori)
    assert nm_g == nm_r
    assert np.array_equal(own_g, own_r)
    assert (own_r >= 0).sum() > 20


@pytest.mark.parametrize("seed,th,orb_dist,check_ori,stereo", [
    (40, 10.0, 100, True, True), (41, 3.0, 64, True, True), (42, 10.0, 100, False, True),
    (43, 10.0, 100, True, False), (44, 3.0, 64, False, False), (45, 20.0, 256, True, True)])
def test_search_by_projection_keyframe(tracker, oracle_mod, seed, th, orb_dist, check_ori, stereo):
    """Tracking::Relocalization's SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist)
    (ORBmatcher.cc:1922-2066): greedy claims by every point, sAlreadyFound filter."""
    p = synth.reloc_problem(seed, stereo=stereo)
    nm_r, own_r = oracle_mod.search_by_projection_keyframe(p, th=th, orb_dist=orb_dist, check_ori=check_ori)
    nm_g, own_g = tracker.search_by_projection_keyframe(p, th=th, orb_dist=orb_dist, check_ori=check_ori)
    assert nm_g == nm_r
    assert np.array_equal(own_g, own_r)
    assert (own_r >= 0).sum() > 20


def test_reloc_batched_slots(amd, oracle_mod):
    t = amd.Tracker()
    probs = [synth.reloc_problem(200 + s, n_kp=1200 + 200 * s, n_mp=1800 + 300 * s) for s in range(5)]
    t.reserve(len(probs), 2100, 3300)
    for s, p in enumerate(probs):
        t.stage(s, p)
    t.run_reloc_batch(len(probs), th=10.0, orb_dist=100)
    for s, p in enumerate(probs):
        nm_g, own_g, _ = t.fetch(s, len(p["frame"]["keys_un"]))
        nm_r, own_r = oracle_mod.search_by_projection_keyframe(p, th=10.0, orb_dist=100)
        assert nm_g == nm_r and np.array_equal(own_g, own_r), s
    t.close()


def test_batched_slots(amd, oracle_mod):
    t = amd.Tracker()
    probs = [synth.tracking_problem(100 + s, n_kp=1500 + 100 * s, n_mp=2000 + 150 * s,
                                    motion=("forward", "backward", "static")[s % 3]) for s in range(6)]
    t.reserve(len(probs), 2100, 3000)
    for s, p in enumerate(probs):
        t.stage(s, p)
    t.run_local_batch(len(probs), th=1.0, nnratio=0.8)
    for s, p in enumerate(probs):
        nm, own, view = t.fetch(s, len(p["frame"]["keys_un"]), len(p["map"]["Xw"]))
        nm_r, own_r, view_r = oracle_mod.search_local_points(p, th=1.0, nnratio=0.8)
        assert nm == nm_r and np.array_equal(own, own_r)
        _cmp_view(view, view_r)
    t.run_frame_batch(len(probs), th=15.0)
    for s, p in enumerate(probs):
        nm, own, _ = t.fetch(s, len(p["frame"]["keys_un"]))
        nm_r, own_r = oracle_mod.search_by_projection_frame(p, th=15.0)
        assert nm == nm_r and np.array_equal(own, own_r)
    t.close()


def test_edge_cases(tracker, oracle_mod):
    p = synth.tracking_problem(21, n_kp=500, n_mp=400)
    # every keypoint already owned by a map point with observations: nothing can match
    q = dict(p, kp_blocked=np.ones(len(p["frame"]["keys_un"]), np.uint8))
    assert tracker.search_local_points(q)[0] == oracle_mod.search_local_points(q)[0] == 0
    # no map point has observations: later points may overwrite earlier claims
    m = dict(p["map"], flags=np.zeros_like(p["map"]["flags"]))
    q = dict(p, map=m)
    nm_r, own_r, _ = oracle_mod.search_local_points(q)
    nm_g, own_g, _ = tracker.search_local_points(q)
    assert nm_g == nm_r and np.array_equal(own_g, own_r)
    nm_r, own_r = oracle_mod.search_by_projection_frame(q)
    nm_g, own_g = tracker.search_by_projection_frame(q)
    assert nm_g == nm_r and np.array_equal(own_g, own_r)
    # empty map / empty last frame
    e = {k: v[:0] for k, v in p["map"].items()}
    q = dict(p, map=e, last_mp=np.full_like(p["last_mp"], -1))
    assert tracker.search_local_points(q)[0] == 0
    assert tracker.search_by_projection_frame(q)[0] == 0


def test_crowd_fallback_rescan(tracker, oracle_mod):
    """More claims than kept candidates: the resolve kernels' exact rescan path."""
    from track_cases import crowd_problem
    p = crowd_problem()
    nm_r, own_r, view_r = oracle_mod.search_local_points(p)
    nm_g, own_g, view_g = tracker.search_local_points(p)
    _cmp_view(view_g, view_r)
    assert nm_g == nm_r == 12 and np.array_equal(own_g, own_r)
    for ori in (False, True):
        nm_r, own_r = oracle_mod.search_by_projection_frame(p, th=15.0, check_ori=ori)
        nm_g, own_g = tracker.search_by_projection_frame(p, th=15.0, check_ori=ori)
        assert nm_g == nm_r and np.array_equal(own_g, own_r)


@pytest.mark.parametrize("seed,n_kp,n_mp,th", [(31, 2000, 3000, 3.0), (32, 1000, 1500, 3.0), (33, 4000, 6000, 5.0),
                                               (34, 300, 200, 1.0)])
def test_fuse_candidates(tracker, oracle_mod, seed, n_kp, n_mp, th):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th) search half (ORBmatcher.cc:1139-1240)."""
    p = synth.tracking_problem(seed, n_kp=n_kp, n_mp=n_mp)
    bi_r, bd_r = oracle_mod.fuse_candidates(p, th)
    bi_g, bd_g = tracker.fuse_candidates(p, th)
    assert np.array_equal(bi_g, bi_r) and np.array_equal(bd_g, bd_r)
    assert (bd_r <= 50).sum() > 20


def test_fuse_batched(amd, oracle_mod):
    t = amd.Tracker()
    probs = [synth.tracking_problem(40 + s, n_kp=1200 + 100 * s, n_mp=1500 + 200 * s) for s in range(5)]
    t.reserve(len(probs), 1700, 2500)
    for s, p in enumerate(probs):
        t.stage(s, p)
    t.run_fuse_batch(len(probs), 3.0)
    for s, p in enumerate(probs):
        bi, bd = t.fetch_fuse(s, len(p["map"]["Xw"]))
        bi_r, bd_r = oracle_mod.fuse_candidates(p, 3.0)
        assert np.array_equal(bi, bi_r) and np.array_equal(bd, bd_r)
    t.close()
