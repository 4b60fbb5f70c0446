#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle (test infrastructure).

The reference ships no golden vectors and cannot be built here (no OpenCV / Eigen,
SURVEY.md §8c), so these fixtures pin the oracle's current output on seeded synthetic
inputs (regression anchor for both the oracle and the HIP path). Inputs are regenerated
from their seeds and checked against the stored SHA-256, so generator drift fails loudly
instead of silently changing the pinned case.

  c1_mono_640x480.npz   C1: ORBextractor(1000,1.2,8,20,7) on textured_image(480,640,seed=1)
  c2_stereo_1241x376.npz C2: ORBextractor(2000,...) on stereo_pair(376,1241,t=0) left/right +
                         Frame::ComputeStereoMatches (KITTI bf/fx)
  c3_rgbd_640x480.npz    C3: ORBextractor(1000) on rgbd_frame(480,640,t) t = 0, 1 + UndistortKeyPoints
                         (TUM1 K / distortion) + ComputeStereoFromRGBD (bf 40) per frame, and
                         SearchForInitialization(F0, F1, vbPrevMatched = F0 keysUn, 100) with
                         ORBmatcher(0.9, true): vnMatches12, vbPrevMatched out, the count
  c4_localba.npz         C4: LocalBundleAdjustment on synth.localba_problem(seed=4) (20 KF x 3000 MP):
                         optimised Tcw, points, the erase set, LM iterations and chi2
"""
import sys
from pathlib import Path

import hashlib

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))

import oracle  # noqa: E402
from orbslam2_amd import synth  # noqa: E402

KITTI_BF, KITTI_FX = 386.1448, 718.856
K_TUM = [517.306408, 516.469215, 318.643040, 255.313989]
D_TUM = [0.262383, -0.953104, -0.005358, 0.002628, 1.163314]
BF_TUM = 40.0


def problem_sha(prob: dict) -> np.ndarray:
    h = hashlib.sha256()
    for k in sorted(prob):
        h.update(k.encode() + np.ascontiguousarray(prob[k]).tobytes())
    return np.array(h.hexdigest())


def c3_frame(t):
    """(gray, depth, kps, desc, keysUn, uRight, depth) of C3 frame t through the oracle."""
    gray, depth = synth.rgbd_frame(480, 640, t)
    k, d = oracle.Extractor(1000).extract(gray)
    xy = oracle.undistort_points(np.stack([k["x"], k["y"]], 1), K_TUM, D_TUM)
    ku = k.copy()
    ku["x"], ku["y"] = xy[:, 0], xy[:, 1]
    u, dep = oracle.stereo_from_rgbd(k, ku, depth, BF_TUM)
    return gray, depth, k, d, ku, u, dep


def sha(a: np.ndarray) -> np.ndarray:
    return np.array(hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest())


def main():
    img = synth.textured_image(480, 640, 1)
    ex = oracle.Extractor(1000, 1.2, 8, 20, 7)
    k, d = ex.extract(img)
    np.savez_compressed(HERE / "c1_mono_640x480.npz", image_sha256=sha(img), kps=k, desc=d)
    L, R = synth.stereo_pair(376, 1241, 0)
    exL, exR = oracle.Extractor(2000), oracle.Extractor(2000)
    kL, dL = exL.extract(L)
    kR, dR = exR.extract(R)
    mb = float(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    u, dep = oracle.stereo_matches(exL, exR, kL, dL, kR, dR, KITTI_BF, mb)
    np.savez_compressed(HERE / "c2_stereo_1241x376.npz", left_sha256=sha(L), right_sha256=sha(R),
                        kps_left=kL, desc_left=dL, kps_right=kR, u_right=u, depth=dep,
                        camera=np.array([KITTI_BF, KITTI_FX, mb], np.float64))
    f0, f1 = c3_frame(0), c3_frame(1)
    bounds = oracle.image_bounds(640, 480, K_TUM, D_TUM)
    prev = np.stack([f0[4]["x"], f0[4]["y"]], 1)
    nm, m12, prev_out = oracle.search_for_initialization(oracle.Grid(f0[4], f0[3], bounds),
                                                         oracle.Grid(f1[4], f1[3], bounds), prev, 100, 0.9, True)
    np.savez_compressed(HERE / "c3_rgbd_640x480.npz",
                        gray0_sha256=sha(f0[0]), depth0_sha256=sha(f0[1]), gray1_sha256=sha(f1[0]),
                        depth1_sha256=sha(f1[1]), kps0=f0[2], desc0=f0[3], keys_un0=f0[4], u_right0=f0[5],
                        depth_out0=f0[6], kps1=f1[2], keys_un1=f1[4], u_right1=f1[5], depth_out1=f1[6],
                        matches12=m12, prev_matched=prev_out, nmatches=np.int32(nm),
                        camera=np.array(K_TUM + D_TUM + [BF_TUM], np.float64))
    prob = synth.localba_problem(seed=4)
    r = oracle.lba_solve(prob)
    np.savez_compressed(HERE / "c4_localba.npz", problem_sha256=problem_sha(prob), pose_Tcw=r["pose_Tcw"],
                        point_Xw=r["point_Xw"], edge_erase=r["edge_erase"],
                        iterations=np.array(r["iterations"], np.int32), chi2=np.array(r["chi2"], np.float64))
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
