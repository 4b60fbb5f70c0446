"""CPU checks of the LocalBA oracle (test infrastructure): convergence on the C4 graph; and of the
product's host-side structure build (lba_host.h)."""
from pathlib import Path

import numpy as np

from orbslam2_amd import synth

ROOT = Path(__file__).resolve().parents[1]


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


def _rejecting_problem(seed, sigma, n_kf=8, n_points=300):
    """A C4-shaped graph whose points are scattered by `sigma` m: LM trials get rejected (rho < 0),
    so the trial loop's terminate() check (levenberg.cpp:149) is reached."""
    prob = synth.localba_problem(seed=seed, n_kf=n_kf, n_points=n_points)
    rng = np.random.default_rng(seed)
    prob["point_Xw"] = (prob["point_Xw"] + rng.normal(0, sigma, prob["point_Xw"].shape)).astype(np.float32)
    return prob


def test_lba_oracle_stop_hook_semantics(oracle_mod):
    """The oracle's pbStopFlag hook (lba_oracle_solve_hook) against g2o's control flow
    (sparse_optimizer.cpp:376, optimization_algorithm_levenberg.cpp:96-164, Optimizer.cc:902-917):
    a flag raised after trial T of phase 1 ends phase 1 with the iteration holding trial T and skips
    phase 2; raised in phase 2, it ends phase 2 the same way; a trial count the phase never reaches
    changes nothing."""
    prob = _rejecting_problem(61, 3.0)
    full = oracle_mod.lba_solve(prob)
    assert full["trials"][0] > full["iterations"][0], "the problem must reject a phase-1 trial"
    for never in ((2, 99), (1, full["trials"][0] + 1)):   # a trial the phase never reaches raises nothing
        r = oracle_mod.lba_solve(prob, hook=never)
        assert r["pose_Tcw"].tobytes() == full["pose_Tcw"].tobytes() and r["stopped"] == 0, never
    r0 = oracle_mod.lba_solve(prob, hook=(1, 0))
    assert r0["iterations"] == (0, 0) and r0["stopped"] == 1
    rej = None
    for T in range(1, full["trials"][0] + 1):
        r = oracle_mod.lba_solve(prob, hook=(1, T))
        assert r["trials"] == (T, 0) and r["stopped"] == 1 and r["iterations"][1] == 0
        prev = oracle_mod.lba_solve(prob, hook=(1, T - 1))
        if r["iterations"][0] == prev["iterations"][0] + 1 and r["chi2"][0] == prev["chi2"][0] and T > 1:
            rej = T   # trial T was rejected and the flag ended its iteration there
    assert rej is not None
    for T in range(0, full["trials"][1]):
        r = oracle_mod.lba_solve(prob, hook=(2, T))
        assert r["trials"] == (full["trials"][0], T) and r["stopped"] == 1


def test_host_structure_invariants(tmp_path):
    """LocalBA's host structure build (csrc/lba_host.h: the active set and the Schur tile-pair row
    lists, built per call before the device trials) on landmark-major and shuffled edge orders,
    unsorted vertex ids and extra fixed poses: hessian order by id, CSR lists in slot order, inverse
    maps, the landmark-major fast path's aliasing, and every tile pair's landmark rows
    (tests/cpp/lba_host_check.cpp). CPU only."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = tmp_path / "lba_host_check"
    subprocess.run([hipcc, "-O2", "-I", str(ROOT / "orb-slam2-noted_amd" / "csrc"),
                    str(ROOT / "tests" / "cpp" / "lba_host_check.cpp"), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok 8"), r.stdout + r.stderr


def test_chol16_include_is_generated():
    """csrc/lba_chol16.inc (the software-pipelined diagonal-tile Cholesky, lba.hip LBA_DIAG_PIPE) is the
    output of tools/gen_chol16.py: a hand edit of either would drift from the other."""
    import subprocess
    import sys
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "gen_chol16.py")], capture_output=True, text=True,
                         check=True).stdout
    inc = (ROOT / "orb-slam2-noted_amd" / "csrc" / "lba_chol16.inc").read_text()
    assert out.rstrip("\n") == inc.rstrip("\n")
    # every instruction of the pipelined tile is an ordered (volatile) statement; the column
    # updates: 120 of L and 120 of its inverse
    assert inc.count("v_fmac_f64_dpp") == 240 and inc.count("v_rsq_f64") == 16
