"""CPU checks of the new-map-points oracle (LocalMapping::CreateNewMapPoints, LocalMapping.cc:396-600):
the restated OpenCV Jacobi SVD against numpy, accepted points against the synthetic ground truth,
and the pin of the device restatements of glibc atan2f / hypot (libm_restate.h) against the live
libm (oracle/tools/check_atan2f_hypot.c; the full run covers 1.56e9 atan2f and 2e8 hypot inputs
with 0 mismatches, this test a bounded sample)."""
import subprocess
from pathlib import Path

import numpy as np

from orbslam2_amd import synth

ROOT = Path(__file__).resolve().parents[1]


def test_svd4_matches_numpy(oracle_mod):
    rng = np.random.default_rng(0)
    for _ in range(200):
        A = rng.normal(size=(4, 4)).astype(np.float32)
        vt, w = oracle_mod.svd4_vt(A)
        _, s, v = np.linalg.svd(A.astype(np.float64))
        assert np.all(np.diff(w) <= 0), "singular values sorted descending"
        np.testing.assert_allclose(w, s, rtol=1e-5, atol=1e-5)
        # last right singular vector up to sign
        d = min(np.abs(vt[3] - v[3]).max(), np.abs(vt[3] + v[3]).max())
        assert d < 1e-4


def test_triangulation_recovers_points(oracle_mod):
    for cam in ("kitti", "tum"):
        prob = synth.newpoints_problem(seed=5, cam=cam, wrong_frac=0.0)
        nnew, x3d, ok = oracle_mod.triangulate(prob)
        assert nnew == int(ok.sum()) and nnew > 0.4 * len(prob["pairs"])
        # accepted points reproject into kf1 near the observed keypoint
        k1 = prob["kf1"]
        T = np.asarray(k1["Tcw"], np.float64).reshape(3, 4)
        P = x3d[ok == 1].astype(np.float64) @ T[:, :3].T + T[:, 3]
        u = k1["fx"] * P[:, 0] / P[:, 2] + k1["cx"]
        idx1 = prob["pairs"][ok == 1, 0]
        assert np.median(np.abs(u - k1["keys_un"]["x"][idx1])) < 2.0


def test_wrong_partners_rejected(oracle_mod):
    prob = synth.newpoints_problem(seed=9, wrong_frac=0.5)
    nnew, x3d, ok = oracle_mod.triangulate(prob)
    clean = synth.newpoints_problem(seed=9, wrong_frac=0.0)
    n2, _, ok2 = oracle_mod.triangulate(clean)
    assert nnew < n2


def test_libm_restatements_pinned(tmp_path):
    exe = tmp_path / "check_atan2f_hypot"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(ROOT / "oracle/tools/check_atan2f_hypot.c"), "-lm"],
                   check=True)
    r = subprocess.run([str(exe), "2000000", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "0 mismatches; hypot" in r.stdout and r.stdout.strip().endswith("0 mismatches")
