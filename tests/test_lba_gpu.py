"""GPU LocalBA (Optimizer::LocalBundleAdjustment, Optimizer.cc:646-1049) vs the CPU oracle.

Tolerance (BASELINE.json north_star): poses and points within 1e-4 relative; the outlier
set (vToErase) identical; same LM iteration counts.
"""
import numpy as np
import pytest

from orbslam2_amd import synth

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-12)


# 6P <= 128 runs the single-workgroup LDS Cholesky; 22 / 40 / 64 / 93 free KFs (6P = 132, 240,
# 384, 558) the single-workgroup Cholesky over a global work matrix (chol_global_body); 100 free
# KFs (6P = 600) the multi-launch blocked Cholesky (ORB-SLAM2's covisibility window is not bounded). 8 and 16 free KFs (6P = 48, 96) put the appended
# right-hand-side row first in its 16-row tile (the diagonal tile's pivot limit is 0).
@pytest.mark.parametrize("seed,n_kf,n_pts", [(4, 20, 3000), (5, 10, 800), (6, 20, 1500), (9, 21, 1500),
                                             (10, 22, 2000), (11, 40, 4000), (12, 64, 6000),
                                             (13, 16, 1500), (14, 8, 600), (16, 93, 7000), (17, 100, 7000)])
def test_lba_matches_oracle(amd, oracle_mod, seed, n_kf, n_pts):
    prob = synth.localba_problem(seed=seed, n_kf=n_kf, n_points=n_pts)
    ref = oracle_mod.lba_solve(prob)
    got = amd.LocalBundleAdjustment().solve(prob)
    print("iters", got["iterations"], ref["iterations"], "chi2", got["chi2"], ref["chi2"],
          "erase diff", int((got["edge_erase"] != ref["edge_erase"]).sum()),
          "pose rel", _rel(got["pose_Tcw"], ref["pose_Tcw"]), "pt rel", _rel(got["point_Xw"], ref["point_Xw"]))
    assert got["iterations"] == ref["iterations"]
    np.testing.assert_allclose(got["chi2"], ref["chi2"], rtol=1e-5)
    assert _rel(got["pose_Tcw"], ref["pose_Tcw"]) < RTOL
    assert _rel(got["point_Xw"], ref["point_Xw"]) < RTOL
    # per point relative (scale-aware) check too
    d = np.linalg.norm(got["point_Xw"] - ref["point_Xw"], axis=1)
    n = np.linalg.norm(ref["point_Xw"], axis=1)
    assert (d / n).max() < RTOL
    assert np.array_equal(got["edge_erase"], ref["edge_erase"])


@pytest.mark.parametrize("order", ["shuffled", "reversed_ids"])
def test_lba_edge_orders(amd, oracle_mod, order):
    """Edges not landmark by landmark (the general path: landmark-major records gathered, their own
    position arrays), and vertex ids against index order (the hessian sorted by id): same results
    as the oracle on the same problem. ORB-SLAM2 itself adds the edges map point by map point
    (Optimizer.cc:766-848), the fast path every other test takes."""
    prob = dict(synth.localba_problem(seed=13, n_kf=12, n_points=1200))
    rng = np.random.default_rng(1)
    if order == "shuffled":
        perm = rng.permutation(len(prob["edge_point"]))
        for k in ("edge_point", "edge_pose", "edge_obs", "edge_inv_sigma2"):
            prob[k] = np.ascontiguousarray(np.asarray(prob[k])[perm])
    else:
        prob["point_id"] = np.ascontiguousarray(np.asarray(prob["point_id"])[::-1])
        prob["pose_id"] = np.ascontiguousarray(np.asarray(prob["pose_id"])[::-1])
    ref = oracle_mod.lba_solve(prob)
    got = amd.LocalBundleAdjustment().solve(prob)
    assert got["iterations"] == ref["iterations"]
    assert _rel(got["pose_Tcw"], ref["pose_Tcw"]) < RTOL
    assert _rel(got["point_Xw"], ref["point_Xw"]) < RTOL
    assert np.array_equal(got["edge_erase"], ref["edge_erase"])


def _near_singular_problem(seed=21, keep=2):
    """A window whose free keyframe 5 keeps only `keep` mono observations: its 6 x 6 pose block has
    rank 2 keep < 6 and the Schur system is positive definite only through the LM damping, so the
    Cholesky pivots of that block are ~lambda (the pivot's v_rsq_f64 + Newton step)."""
    prob = dict(synth.localba_problem(seed=seed, n_kf=10, n_points=800))
    ep = np.asarray(prob["edge_pose"])
    pose_idx = int(np.flatnonzero(np.asarray(prob["pose_id"]) == 5)[0])
    mine = np.flatnonzero(ep == pose_idx)
    drop = np.zeros(len(ep), bool)
    drop[mine[keep:]] = True
    for k in ("edge_point", "edge_pose", "edge_obs", "edge_inv_sigma2"):
        prob[k] = np.ascontiguousarray(np.asarray(prob[k])[~drop])
    obs = np.array(prob["edge_obs"], np.float32).reshape(-1, 3)
    obs[np.asarray(prob["edge_pose"]) == pose_idx, 2] = -1.0   # mono
    prob["edge_obs"] = np.ascontiguousarray(obs.reshape(np.asarray(prob["edge_obs"]).shape))
    return prob


@pytest.mark.parametrize("keep", [1, 2])
def test_lba_near_singular(amd, oracle_mod, keep):
    prob = _near_singular_problem(keep=keep)
    ref = oracle_mod.lba_solve(prob)
    got = amd.LocalBundleAdjustment().solve(prob)
    assert got["iterations"] == ref["iterations"] and got["trials"] == ref["trials"]
    assert _rel(got["pose_Tcw"], ref["pose_Tcw"]) < RTOL
    assert _rel(got["point_Xw"], ref["point_Xw"]) < RTOL
    assert np.array_equal(got["edge_erase"], ref["edge_erase"])


def test_lba_stop_flag(amd, oracle_mod):
    prob = synth.localba_problem(seed=7, n_kf=8, n_points=300)
    got = amd.LocalBundleAdjustment().solve(prob, stop=True)
    assert got["stopped"] == 2 and got["iterations"] == (0, 0)
    assert np.array_equal(got["pose_Tcw"], prob["pose_Tcw"].reshape(-1, 16))
    assert got["edge_erase"].sum() == 0


def test_lba_mono_only_and_fixed(amd, oracle_mod):
    prob = synth.localba_problem(seed=8, n_kf=12, n_points=1000, stereo_frac=0.0)
    ref = oracle_mod.lba_solve(prob)
    got = amd.LocalBundleAdjustment().solve(prob)
    assert got["iterations"] == ref["iterations"]
    assert _rel(got["pose_Tcw"], ref["pose_Tcw"]) < RTOL
    assert _rel(got["point_Xw"], ref["point_Xw"]) < RTOL
    assert np.array_equal(got["edge_erase"], ref["edge_erase"])


def test_golden_c4_on_device(amd):
    """HIP LocalBA == the committed fixture tests/golden/c4_localba.npz within 1e-4, same LM
    iterations and erase set (no oracle at run time)."""
    from test_golden_cpu import load_c4
    prob, g = load_c4()
    got = amd.LocalBundleAdjustment().solve(prob)
    assert tuple(got["iterations"]) == tuple(g["iterations"])
    assert _rel(got["pose_Tcw"], g["pose_Tcw"]) < RTOL and _rel(got["point_Xw"], g["point_Xw"]) < RTOL
    assert np.array_equal(got["edge_erase"], g["edge_erase"])


def _rejecting_problem(seed, sigma, n_kf=8, n_points=300):
    from test_lba_cpu import _rejecting_problem as mk
    return mk(seed, sigma, n_kf, n_points)


def _same(got, ref, what):
    assert got["iterations"] == ref["iterations"], (what, got["iterations"], ref["iterations"])
    assert got["trials"] == ref["trials"], (what, got["trials"], ref["trials"])
    assert got["stopped"] == ref["stopped"], (what, got["stopped"], ref["stopped"])
    assert _rel(got["pose_Tcw"], ref["pose_Tcw"]) < RTOL, what
    assert _rel(got["point_Xw"], ref["point_Xw"]) < RTOL, what
    assert np.array_equal(got["edge_erase"], ref["edge_erase"]), what


@pytest.mark.parametrize("case", ["c4", "reject1", "reject2"])
def test_lba_stop_hook_every_trial(amd, oracle_mod, case):
    """pbStopFlag raised after every LM trial of both phases: the device's LM
    decision reads the flag where g2o does (levenberg.cpp:149 after a rejected trial,
    sparse_optimizer.cpp:376 before each iteration) and the host skips phase 2 (Optimizer.cc:913-917).
    `reject1` / `reject2` reject a trial in phase 1 / phase 2, so the trial-loop check is reached.
    GPU == oracle within 1e-4 with the same iterations, trials, stopped code and erase set."""
    if case == "c4":
        prob = synth.localba_problem(seed=4)
    else:
        prob = _rejecting_problem(61, 3.0) if case == "reject1" else _rejecting_problem(78, 4.0)
    full = oracle_mod.lba_solve(prob)
    if case != "c4":
        p = 0 if case == "reject1" else 1
        assert full["trials"][p] > full["iterations"][p]
    lba = amd.LocalBundleAdjustment()
    for phase in (1, 2):
        for T in range(0, full["trials"][phase - 1] + 2):
            lba.set_stop_hook(phase, T)
            _same(lba.solve(prob), oracle_mod.lba_solve(prob, hook=(phase, T)), (case, phase, T))
    lba.set_stop_hook(0, 0)
    _same(lba.solve(prob), full, (case, "no hook"))


def test_lba_stop_flag_live(amd, oracle_mod):
    """A second thread raises the flag while lba_solve runs (LocalMapping's mbAbortBA, set by
    Tracking::NeedNewKeyFrame / InsertKeyFrame): the call returns early with stopped = 1, and its
    result equals the oracle stopped at the same point (the trial the device observed)."""
    import ctypes
    import threading
    import time
    prob = synth.localba_problem(seed=12, n_kf=64, n_points=6000)
    lba = amd.LocalBundleAdjustment()
    full = lba.solve(prob)
    t0 = time.perf_counter()
    lba.solve(prob, stop=ctypes.c_uint8(0))
    t_full = time.perf_counter() - t0
    stopped_early = 0
    for frac in (0.5, 0.3, 0.15, 0.05):
        flag = ctypes.c_uint8(0)
        th = threading.Timer(frac * t_full, lambda: setattr(flag, "value", 1))
        th.start()
        got = lba.solve(prob, stop=flag)
        th.join()
        assert flag.value == 1
        if got["stopped"] == 0:
            assert got["trials"] == full["trials"]   # raised after the last check: a complete run
            continue
        assert got["stopped"] == 1
        stopped_early += 1
        hook = (1, got["trials"][0]) if got["iterations"][1] == 0 and got["trials"][1] == 0 else (2, got["trials"][1])
        ref = oracle_mod.lba_solve(prob, hook=hook)   # (2, 0) and (1, all) give the same outputs
        _same(got, ref, ("live", frac, hook))
        print("live stop", frac, t_full, got["iterations"], got["trials"])
    if stopped_early == 0:   # timer jitter on a loaded host: the deterministic test below covers it
        pytest.skip(f"no timer attempt landed mid-call (call {t_full * 1e3:.2f} ms)")


def test_lba_stop_flag_live_deterministic(amd, oracle_mod):
    """The live flag at a deterministic point (lba_set_stop_hook phase 3): once the call has read back
    its first chunk of trials (phase 1's five), while phase 2 is still queued, the word the device reads
    turns raised -- the same mirrored word a second thread's write reaches (an engine-owned flag ORed
    in: the caller's const flag is not written). The call must return stopped = 1 and equal
    the oracle stopped at the trial the device observed."""
    import ctypes
    prob = synth.localba_problem(seed=12, n_kf=64, n_points=6000)
    lba = amd.LocalBundleAdjustment()
    full = lba.solve(prob)
    chunk = 1
    lba.set_stop_hook(3, chunk)
    flag = ctypes.c_uint8(0)
    got = lba.solve(prob, stop=flag)
    lba.set_stop_hook(0, 0)
    assert flag.value == 0, "the hook wrote the caller's flag"
    assert got["stopped"] == 1, (got["iterations"], got["trials"], full["trials"])
    hook = (1, got["trials"][0]) if got["iterations"][1] == 0 and got["trials"][1] == 0 else (2, got["trials"][1])
    assert sum(got["trials"]) < sum(full["trials"])
    _same(got, oracle_mod.lba_solve(prob, hook=hook), ("live-hook", chunk, hook))


@pytest.mark.parametrize("seed,n_kf,n_pts", [(4, 20, 3000), (9, 21, 1500), (14, 8, 600), (10, 22, 2000), (11, 40, 4000)])
def test_lba_fused_finish_bit_identical(amd, seed, n_kf, n_pts):
    """lba_finish_chol (the Schur finish blocks hand Hs to the Cholesky block inside one launch, for the
    LDS Cholesky (<= 21 free keyframes) and the global-work-matrix one (22..93):
    write-through stores, an agent-scope counter, sc1 loads) against the two-launch path
    (lba_schur_finish, then lba_chol_tiled, ordered by the kernel boundary): identical bits in every
    output (the hand-off's memory ordering is checked, not assumed)."""
    prob = synth.localba_problem(seed=seed, n_kf=n_kf, n_points=n_pts)
    lba = amd.LocalBundleAdjustment()
    fused = lba.solve(prob)
    lba.set_test_option(lba.LBA_OPT_FUSE_FINISH, 0)
    split = lba.solve(prob)
    lba.set_test_option(lba.LBA_OPT_FUSE_FINISH, 1)
    again = lba.solve(prob)
    for k in ("pose_Tcw", "point_Xw", "edge_erase"):
        assert np.asarray(fused[k]).tobytes() == np.asarray(split[k]).tobytes(), k
        assert np.asarray(fused[k]).tobytes() == np.asarray(again[k]).tobytes(), k
    assert fused["iterations"] == split["iterations"] and fused["trials"] == split["trials"]
    assert fused["chi2"] == split["chi2"]


def test_lba_handoff_timeout_is_an_error(amd, oracle_mod):
    """A hand-off wait that times out (LBA_OPT_SPIN_LIMIT 0: every wait does) must not pass for a
    rejected LM trial: lba_solve returns ORBX_EDEVICE. The engine is usable afterwards:
    with the default bound the next call equals the oracle."""
    prob = synth.localba_problem(seed=9, n_kf=21, n_points=1500)
    lba = amd.LocalBundleAdjustment()
    lba.set_test_option(lba.LBA_OPT_SPIN_LIMIT, 0)
    with pytest.raises(amd.OrbslamError, match="status -2"):
        lba.solve(prob)
    lba.set_test_option(lba.LBA_OPT_SPIN_LIMIT, -1)
    _same(lba.solve(prob), oracle_mod.lba_solve(prob), "after the fault")
