"""CPU checks of the LocalBA oracle (test infrastructure): convergence on the C4 graph."""
import numpy as np

from orbslam2_amd import synth


def test_lba_oracle_converges(oracle_mod):
    prob = synth.localba_problem(seed=4)
    r = oracle_mod.lba_solve(prob)
    assert r["iterations"][0] == 5 and 1 <= r["iterations"][1] <= 10
    assert r["chi2"][1] < r["chi2"][0]
    T0 = prob["pose_Tcw"].reshape(-1, 4, 4)
    T1 = r["pose_Tcw"].reshape(-1, 4, 4)
    Tt = prob["truth_Tcw"]
    e0 = np.abs(T0[:, :3, 3] - Tt[:, :3, 3]).mean()
    e1 = np.abs(T1[:, :3, 3] - Tt[:, :3, 3]).mean()
    assert e1 < 0.5 * e0          # poses pulled towards the truth
    frac = r["edge_erase"].mean()
    assert 0.05 < frac < 0.2      # 5 % injected outliers + chi2 tail


def test_lba_oracle_stop_flag(oracle_mod):
    prob = synth.localba_problem(seed=7, n_kf=8, n_points=300)
    r = oracle_mod.lba_solve(prob, stop=True)
    assert r["stopped"] == 2
    assert np.array_equal(r["pose_Tcw"], prob["pose_Tcw"].reshape(-1, 16))
