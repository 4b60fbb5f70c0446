"""GPU BoW-guided matchers vs the CPU oracle, bit-exact:
ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (ORBmatcher.cc:236-353) and
SearchForTriangulation (ORBmatcher.cc:915-1089) on seeded synthetic keyframe pairs
(synth.bow_match_problem; FeatureVectors are synthetic node groupings). No reference fixtures
exist for these functions: parity against a real build is unpinned."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bm(amd):
    m = amd.BowMatcher()
    yield m
    m.close()


@pytest.mark.parametrize("seed,n,nnratio,ori", [(3, 2000, 0.7, True), (4, 2000, 0.75, True), (5, 1000, 0.7, False),
                                                (6, 3000, 0.9, True), (7, 300, 0.6, True)])
def test_search_by_bow(bm, oracle_mod, seed, n, nnratio, ori):
    p = synth.bow_match_problem(seed, n=n, n_points=int(0.8 * n))
    nm_r, m_r = oracle_mod.search_by_bow(p, nnratio, ori)
    nm_g, m_g = bm.search_by_bow(p, nnratio, ori)
    assert nm_g == nm_r and np.array_equal(m_g, m_r)
    assert nm_r > 20


@pytest.mark.parametrize("seed,n,stereo,ori", [(3, 2000, False, True), (8, 2000, True, True), (9, 1500, False, False),
                                               (10, 3000, False, True), (11, 400, False, True)])
def test_search_for_triangulation(bm, oracle_mod, seed, n, stereo, ori):
    p = synth.bow_match_problem(seed, n=n, n_points=int(0.8 * n))
    r = oracle_mod.search_for_triangulation(p, stereo, ori)
    g = bm.search_for_triangulation(p, stereo, ori)
    assert np.array_equal(g, r)
    assert len(r) > 5


def test_bowmatch_batched(amd, oracle_mod):
    m = amd.BowMatcher()
    probs = [synth.bow_match_problem(50 + s, n=800 + 200 * s, n_points=700 + 150 * s) for s in range(6)]
    m.reserve(len(probs), 2000)
    for s, p in enumerate(probs):
        m.stage(s, p)
    m.run_bow_batch(len(probs), 0.7, True)
    for s, p in enumerate(probs):
        nm, out = m.fetch(s, False, len(p["B"]["keys_un"]))
        nm_r, out_r = oracle_mod.search_by_bow(p, 0.7, True)
        assert nm == nm_r and np.array_equal(out, out_r)
    m.run_tri_batch(len(probs), False, True)
    for s, p in enumerate(probs):
        assert np.array_equal(m.fetch(s, True, len(p["A"]["keys_un"])), oracle_mod.search_for_triangulation(p))
    m.close()


def test_no_shared_nodes(bm, oracle_mod):
    p = synth.bow_match_problem(12, n=500, n_points=400)
    B = dict(p["B"], fv_nodes=p["B"]["fv_nodes"] + 1000)
    q = dict(p, B=B)
    assert bm.search_by_bow(q)[0] == oracle_mod.search_by_bow(q)[0] == 0
    assert len(bm.search_for_triangulation(q)) == 0


@pytest.mark.parametrize("seed,n,nnratio,ori,mpb", [(13, 2000, 0.75, True, 0.6), (14, 2000, 0.75, False, 0.8),
                                                    (15, 1000, 0.9, True, 0.5), (16, 3000, 0.6, True, 0.7)])
def test_search_by_bow_kf(bm, oracle_mod, seed, n, nnratio, ori, mpb):
    """SearchByBoW(KeyFrame*, KeyFrame*) (ORBmatcher.cc:760-903, LoopClosing::ComputeSim3)."""
    p = synth.bow_match_problem(seed, n=n, n_points=int(0.8 * n), mp_frac_b=mpb)
    nm_r, m_r = oracle_mod.search_by_bow_kf(p, nnratio, ori)
    nm_g, m_g = bm.search_by_bow_kf(p, nnratio, ori)
    assert nm_g == nm_r and np.array_equal(m_g, m_r)
    assert nm_r > 20


def test_bow_kf_batched(amd, oracle_mod):
    m = amd.BowMatcher()
    probs = [synth.bow_match_problem(70 + s, n=900 + 150 * s, n_points=800 + 100 * s, mp_frac_b=0.6) for s in range(5)]
    m.reserve(len(probs), 2000)
    for s, p in enumerate(probs):
        m.stage(s, p)
    m.run_bowkf_batch(len(probs), 0.75, True)
    for s, p in enumerate(probs):
        nm, out = m.fetch(s, 2, len(p["A"]["keys_un"]))
        nm_r, out_r = oracle_mod.search_by_bow_kf(p, 0.75, True)
        assert nm == nm_r and np.array_equal(out, out_r)
    m.close()
