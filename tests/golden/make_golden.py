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
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
