"""CPU checks of the PoseOptimization oracle (oracle/lba_oracle.c pose_oracle_optimize)."""
import ctypes as C

import numpy as np

from orbslam2_amd import synth


def test_ldlt_restatement_solves(oracle_mod):
    L = oracle_mod.lib()
    L.orc_ldlt_solve6.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(0)
    for _ in range(50):
        A = rng.normal(size=(6, 6)) * rng.uniform(0.1, 1e3, 6)
        H = np.ascontiguousarray(A @ A.T + 1e-3 * np.eye(6))
        b = rng.normal(size=6)
        x = np.zeros(6)
        assert L.orc_ldlt_solve6(H.ctypes.data, b.ctypes.data, x.ctypes.data) == 1
        np.testing.assert_allclose(H @ x, b, rtol=1e-6, atol=1e-9 * np.abs(b).max())
    H = -np.eye(6)
    assert L.orc_ldlt_solve6(np.ascontiguousarray(H).ctypes.data, b.ctypes.data, x.ctypes.data) == 0


def test_pose_oracle_recovers_pose(oracle_mod):
    for seed in range(3):
        p = synth.pose_problem(seed, n=500, outlier_frac=0.1)
        r = oracle_mod.pose_optimization(p)
        assert np.abs(r["Tcw"] - p["true_Tcw"]).max() < 0.02
        # most planted outliers are flagged
        assert r["outlier"][p["is_outlier"]].mean() > 0.9
        assert r["n_inliers"] == len(p["Xw"]) - int(r["outlier"].sum())


def test_pose_oracle_few_edges(oracle_mod):
    p = synth.pose_problem(1, n=2)
    r = oracle_mod.pose_optimization(p)
    assert r["n_inliers"] == 0 and np.array_equal(r["Tcw"], p["Tcw"]) and not r["outlier"].any()
    p = synth.pose_problem(1, n=8)
    r = oracle_mod.pose_optimization(p)
    assert r["iterations"][0] > 0 and r["iterations"][1:] == (-1, -1, -1)   # edges < 10: one round
