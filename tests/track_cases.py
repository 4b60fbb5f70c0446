"""Hand-built tracking-matcher cases shared by the CPU and GPU tests."""
import numpy as np

from orbslam2_amd import synth


def crowd_problem(n_kp_near: int = 12, n_mp: int = 20):
    """n_mp map points at one 3D location competing for n_kp_near keypoints around its
    projection. Keypoint j's descriptor is the map descriptor with 8*j flipped bits and
    octaves alternate 0/1 (so the ratio test never fires: best and second are on different
    levels). The greedy order then assigns keypoint j to map point j while the best distance
    stays <= TH_HIGH -- after 4 claims every map point's kept top-4 candidates are claimed,
    so this exercises the GPU resolve kernels' exact rescan fallback."""
    p = synth.tracking_problem(1, n_kp=64, n_mp=20)
    fr = p["frame"]
    rng = np.random.default_rng(3)
    R = np.asarray(fr["Tcw"], np.float64)[:, :3]
    t = np.asarray(fr["Tcw"], np.float64)[:, 3]
    Pc = np.array([1.0, 0.5, 12.0])
    Xw = R.T @ (Pc - t)
    u = fr["fx"] * Pc[0] / Pc[2] + fr["cx"]
    v = fr["fy"] * Pc[1] / Pc[2] + fr["cy"]
    kp = fr["keys_un"].copy()
    kp["x"] = rng.uniform(0, 1241, len(kp))
    kp["y"] = rng.uniform(0, 376, len(kp))
    kp["x"][:n_kp_near] = u + rng.uniform(-1.5, 1.5, n_kp_near)
    kp["y"][:n_kp_near] = v + rng.uniform(-1.5, 1.5, n_kp_near)
    kp["octave"][:n_kp_near] = np.arange(n_kp_near) % 2
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    desc = fr["desc"].copy()
    for j in range(n_kp_near):
        desc[j] = synth._flip_bits(rng, base, 8 * j)
    Ow = np.asarray(fr["Ow"], np.float64)
    d = np.linalg.norm(Xw - Ow)
    nrm = (Xw - Ow) / d
    mp = {"Xw": np.tile(Xw, (n_mp, 1)).astype(np.float32), "normal": np.tile(nrm, (n_mp, 1)).astype(np.float32),
          "max_dist": np.full(n_mp, 1.2 * 0.999 * d, np.float32), "min_dist": np.full(n_mp, 0.3 * d, np.float32),
          "desc": np.tile(base, (n_mp, 1)), "flags": np.full(n_mp, synth.MP_HAS_OBS, np.uint8)}
    fr = dict(fr, keys_un=kp, desc=desc, u_right=np.full(len(kp), -1, np.float32))
    # frame-to-frame: the last frame sees every map point once, same octave 0, angles equal
    nl = n_mp
    lk = np.zeros(nl, kp.dtype)
    lk["octave"] = 0
    lk["angle"] = kp["angle"][0]
    last = dict(p["last"], keys_un=lk, u_right=np.full(nl, -1, np.float32), desc=np.zeros((nl, 32), np.uint8))
    return dict(p, frame=fr, map=mp, last=last, last_mp=np.arange(nl, dtype=np.int32),
                last_outlier=np.zeros(nl, np.uint8), kp_blocked=None)
