"""GPU triangulation of new map points (LocalMapping::CreateNewMapPoints, LocalMapping.cc:396-600)
vs the CPU oracle through the C-ABI: accept flags, the count and every accepted point's float bits
identical (parallax test with glibc atan2f / cosf restated, OpenCV's float Jacobi SVD, stereo
unprojection from the distorted keypoint, chi2 / scale gates)."""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu


def _check(prob, got, ref):
    n, x, ok = got
    rn, rx, rok = ref
    assert n == rn
    np.testing.assert_array_equal(ok, rok)
    assert x.tobytes() == rx.tobytes()


@pytest.mark.parametrize("kw", [
    dict(seed=21),                                   # KITTI stereo, 60 % stereo keypoints
    dict(seed=22, cam="tum"),                        # RGB-D: depth measured, distorted mvKeys
    dict(seed=23, stereo_frac=0.0),                  # monocular: SVD only, parallax gate
    dict(seed=24, stereo_frac=1.0, baseline=0.15),   # low parallax: stereo unprojection wins
    dict(seed=25, baseline=3.0, wrong_frac=0.3),     # wide baseline, many wrong partners
    dict(seed=26, n=3000, n_points=2800, zmax=150.0),
])
def test_triangulate_parity(amd, oracle_mod, kw):
    prob = synth.newpoints_problem(**kw)
    got = amd.NewMapPoints().triangulate(prob)
    ref = oracle_mod.triangulate(prob)
    assert ref[0] > 0
    _check(prob, got, ref)


def test_triangulate_batch_slots(amd, oracle_mod):
    probs = [synth.newpoints_problem(seed=30 + s, cam="kitti" if s % 2 else "tum", n=800 + 100 * s,
                                     n_points=700 + 90 * s) for s in range(6)]
    nm = amd.NewMapPoints()
    nm.reserve(len(probs), 1400, 1400)
    for s, p in enumerate(probs):
        nm.stage(s, p)
    nm.run_batch(len(probs))
    for s, p in enumerate(probs):
        _check(p, nm.fetch(s, len(p["pairs"])), oracle_mod.triangulate(p))


def test_triangulate_empty_and_bad_input(amd):
    prob = synth.newpoints_problem(seed=3)
    prob["pairs"] = prob["pairs"][:0]
    n, x, ok = amd.NewMapPoints().triangulate(prob)
    assert n == 0 and len(ok) == 0
    bad = synth.newpoints_problem(seed=3)
    bad["pairs"] = bad["pairs"].copy()
    bad["pairs"][0, 1] = 10 ** 6   # out-of-range idx2 must be refused on the host
    with pytest.raises(Exception):
        amd.NewMapPoints().triangulate(bad)
