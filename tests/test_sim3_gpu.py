"""GPU loop-closing projection search ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
(ORBmatcher.cc:431-560, LoopClosing::ComputeSim3 th = 10) vs the CPU oracle, bit-exact: the Sim3
pose unscaled as cv::Mat evaluates it, queries = map points in vpPoints order, KeyFrame::IsInImage /
GetFeaturesInArea, levels [l - 1, l], every claim blocks later points, first minimum <= TH_LOW.
vpMatched enters as indices into the point table (-1 = NULL, -2 = a point outside vpPoints)."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu


def sim3_problem(seed, scale=1.37, pre_frac=0.1, outside_frac=0.03, **kw):
    p = synth.tracking_problem(seed, **kw)
    rng = np.random.default_rng(seed + 104729)
    T = np.asarray(p["frame"]["Tcw"], np.float32).reshape(-1)[:12].reshape(3, 4)
    Scw = np.eye(4, dtype=np.float32)
    Scw[:3, :4] = (np.float32(scale) * T).astype(np.float32)
    n = len(p["frame"]["keys_un"])
    m = len(p["map"]["Xw"])
    matched = np.full(n, -1, np.int32)
    pre = rng.random(n) < pre_frac
    matched[pre] = rng.integers(0, m, int(pre.sum()))
    matched[rng.random(n) < outside_frac] = -2
    return {"frame": p["frame"], "map": p["map"], "Scw": Scw, "matched": matched}


@pytest.mark.parametrize("seed,th,kw", [(60, 10, {}), (61, 10, dict(stereo=False)), (62, 5, dict(motion="forward")),
                                        (63, 10, dict(n_kp=3000, n_mp=5000)), (64, 15, dict(clone_frac=0.4))])
def test_search_by_projection_sim3(amd, oracle_mod, seed, th, kw):
    prob = sim3_problem(seed, **kw)
    nm_r, m_r = oracle_mod.search_by_projection_sim3(prob, th)
    nm_g, m_g = amd.Tracker().search_by_projection_sim3(prob, th)
    assert nm_r > 20
    assert nm_g == nm_r
    np.testing.assert_array_equal(m_g, m_r)


def test_sim3_batched(amd, oracle_mod):
    probs = [sim3_problem(70 + s, scale=0.8 + 0.2 * s) for s in range(4)]
    t = amd.Tracker()
    t.reserve(len(probs), 2000, 3000)
    for s, p in enumerate(probs):
        t.stage_sim3(s, p)
    t.run_sim3_batch(len(probs), 10)
    for s, p in enumerate(probs):
        nm, m = t.fetch_sim3(s, p)
        nm_r, m_r = oracle_mod.search_by_projection_sim3(p, 10)
        assert nm == nm_r
        np.testing.assert_array_equal(m, m_r)


@pytest.mark.parametrize("seed,th", [(90, 4.0), (91, 4.0), (92, 8.0)])
def test_fuse_sim3_candidates(amd, oracle_mod, seed, th):
    """LoopClosing's Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) search half (ORBmatcher.cc:1321-1437)."""
    prob = sim3_problem(seed, scale=1.21)
    bi_r, bd_r = oracle_mod.fuse_sim3_candidates(prob, th)
    bi_g, bd_g = amd.Tracker().fuse_sim3_candidates(prob, th)
    assert (bd_r <= 50).sum() > 20
    np.testing.assert_array_equal(bi_g, bi_r)
    np.testing.assert_array_equal(bd_g, bd_r)


@pytest.mark.parametrize("seed,s12,th", [(80, 1.0, 7.5), (81, 1.0, 10.0), (82, 1.03, 7.5), (83, 1.0, 4.0)])
def test_search_by_sim3(amd, oracle_mod, seed, s12, th):
    """ORBmatcher::SearchBySim3 (ORBmatcher.cc:1472-1723): both projections + mutual agreement."""
    prob = synth.sim3_pair_problem(seed, s12=s12)
    nf_r, m_r = oracle_mod.search_by_sim3(prob, th)
    nf_g, m_g = amd.Tracker().search_by_sim3(prob, th)
    assert nf_r > 20
    assert nf_g == nf_r
    np.testing.assert_array_equal(m_g, m_r)


def test_search_by_sim3_batched(amd, oracle_mod):
    probs = [synth.sim3_pair_problem(84 + s, n=900 + 200 * s, n_points=800 + 150 * s) for s in range(3)]
    t = amd.Tracker()
    t.reserve(2 * len(probs), 1500, 1200)
    for k, p in enumerate(probs):
        t.stage_search_by_sim3(k, p)
    t.run_sim3_match_batch(len(probs), 7.5)
    for k, p in enumerate(probs):
        nf, m = t.fetch_search_by_sim3(k, p)
        nf_r, m_r = oracle_mod.search_by_sim3(p, 7.5)
        assert nf == nf_r
        np.testing.assert_array_equal(m, m_r)
