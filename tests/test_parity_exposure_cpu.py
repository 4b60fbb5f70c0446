"""The conditions of the "bit-exact" claim, measured: how often each oracle
pin that the reference does not fix decides an output, on (a quick cut of) the benchmark
workloads. Full numbers: tools/parity_exposure.py -> profiles/r02_parity_exposure.json.

Stated conditions, checked here:
* quadtree tie key: the final-phase order of equal-size nodes decides the keypoint ORDER of
  (nearly) every level, and the keypoint SET of most levels, yet a different key still shares
  >= 95 % of each image's keypoints -- bit-exactness is against the creation-sequence pin;
* cv::resize vertical pass: the SSE2 layout changes the keypoints (>= 85 % shared), so parity is
  per pin (both are implemented on the GPU, resize_mode 0 / 1);
* GaussianBlur rounding: OpenCV 3.2's SSE2 half-even column pass never moves a keypoint and
  changes at most a few descriptor rows per image;
* LocalBA: no Schur solve meets a non-positive pivot, so the dense LLT and Eigen's LDLT accept and
  reject the same LM trials.
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))


def test_parity_exposure_quick(oracle_mod, monkeypatch, capsys):
    import json
    import parity_exposure
    monkeypatch.setattr(sys, "argv", ["parity_exposure.py", "--quick"])
    parity_exposure.main()
    rep = json.loads(capsys.readouterr().out)
    for w in ("C1", "C2", "C3"):
        r = rep[w]
        assert r["final_phase_levels"] == r["quadtree_levels"] > 0
        assert r["order_exposed_levels"] >= r["quadtree_levels"] // 2
        for k in ("tie_reversed", "tie_hashed"):
            assert r[k]["min_keypoint_set_shared"] >= 0.95
        assert r["resize_sse2_vs_pin"]["min_keypoint_set_shared"] >= 0.85
        b = r["blur_cv32_sse2_vs_pin"]
        assert b["min_keypoint_set_shared"] == 1.0 and b["descriptor_rows_differing_same_keypoints"] <= 3 * b["images"]
    assert rep["C4"]["nonpositive_pivot"] == 0 and rep["C4"]["min_pivot_ratio"] > 1e-3
    # the instruments are off again: the pinned oracle is unchanged
    img_ok = rep["C1"]["quadtree_levels"] == 8
    assert img_ok


def test_glibc_pointer_order_harness(oracle_mod):
    """oracle/tools/qt_glibc_order.cpp: with creation-order ties it reproduces
    orc_distribute_octtree exactly; with real heap addresses (std::list<ExtractorNode> in fresh
    std::threads) the result is a quadtree output of (within the cut's overshoot) the same size that shares >= 95 % of
    each image's keypoints with the pin. Full run: tools/qt_glibc_order.py ->
    profiles/r02_parity_exposure.json["glibc_pointer_order"]."""
    import qt_glibc_order as q
    from orbslam2_amd import synth
    L = q.harness()
    inputs = [q.level_inputs(im) for im in synth.stereo_pair(376, 1241, 0)]
    pin, _ = q.run(L, inputs, 0, 1)
    for i, levels in enumerate(inputs):
        for l, (cand, _, b, N, _) in enumerate(levels):
            assert oracle_mod.distribute_octtree(cand, b[0], b[1], b[2], b[3], N).tobytes() == pin[i][l].tobytes()
    for ctx in (0, 1, 2):
        real, st = q.run(L, inputs, ctx, 0)
        c = q.compare(real, pin)
        assert st["levels_reaching_final_phase"] == 16 and st["equal_size_pairs"] > 0
        assert c["min_keypoint_set_shared"] >= 0.95
        # the final-phase cut may overshoot N by up to 3 nodes, differently per order
        assert all(abs(len(a) - len(b)) <= 3 for a, b in zip(real[0], pin[0]))
