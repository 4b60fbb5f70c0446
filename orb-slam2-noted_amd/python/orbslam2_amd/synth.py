"""Seeded synthetic inputs for the benchmark configs.

No datasets exist on the build or GPU boxes, so every workload is synthetic:

* ``textured_image``  — value noise (4 octaves, base 64 px) + 200 rectangles (axis-aligned
  and rotated) + 100 discs with random u8 intensities + uniform noise in [-4, 4], clamped
  to u8 (C1/C2/C3 generator).
* ``stereo_pair``     — the left image plus a right image warped by a piecewise-planar
  disparity field d(x, y) in [2, 96] px built from 8 random planes, with +-2 noise (C2).
* ``rgbd_frame``      — gray frame + float depth (metres) from a piecewise-planar Z field in
  [0.5, 4] m with 5 % zero holes (C3; depth = u16/5000 as TUM1.yaml:35 / Tracking.cc:334).
"""
from __future__ import annotations

import numpy as np


def _value_noise(rng: np.random.Generator, h: int, w: int, base: int = 64, octaves: int = 4) -> np.ndarray:
    out = np.zeros((h, w), np.float64)
    amp, total = 1.0, 0.0
    for o in range(octaves):
        step = max(2, base >> o)
        gh, gw = h // step + 2, w // step + 2
        grid = rng.random((gh, gw))
        ys = np.arange(h) / step
        xs = np.arange(w) / step
        y0 = ys.astype(int)
        x0 = xs.astype(int)
        fy = (ys - y0)[:, None]
        fx = (xs - x0)[None, :]
        g00 = grid[y0][:, x0]
        g01 = grid[y0][:, x0 + 1]
        g10 = grid[y0 + 1][:, x0]
        g11 = grid[y0 + 1][:, x0 + 1]
        out += amp * ((1 - fy) * ((1 - fx) * g00 + fx * g01) + fy * ((1 - fx) * g10 + fx * g11))
        total += amp
        amp *= 0.5
    return out / total


def textured_image(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = 40.0 + 175.0 * _value_noise(rng, h, w)
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(200):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        hw, hh = rng.uniform(4, 40), rng.uniform(4, 40)
        val = rng.integers(0, 256)
        if rng.random() < 0.5:
            x0, x1 = int(max(cx - hw, 0)), int(min(cx + hw, w))
            y0, y1 = int(max(cy - hh, 0)), int(min(cy + hh, h))
            img[y0:y1, x0:x1] = val
        else:
            th = rng.uniform(0, np.pi)
            r = int(np.ceil(np.hypot(hw, hh))) + 1
            x0, x1 = int(max(cx - r, 0)), int(min(cx + r, w))
            y0, y1 = int(max(cy - r, 0)), int(min(cy + r, h))
            if x1 <= x0 or y1 <= y0:
                continue
            dx = xx[y0:y1, x0:x1] - cx
            dy = yy[y0:y1, x0:x1] - cy
            u = dx * np.cos(th) + dy * np.sin(th)
            v = -dx * np.sin(th) + dy * np.cos(th)
            m = (np.abs(u) <= hw) & (np.abs(v) <= hh)
            img[y0:y1, x0:x1][m] = val
    for _ in range(100):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        r = rng.uniform(3, 30)
        val = rng.integers(0, 256)
        x0, x1 = int(max(cx - r, 0)), int(min(cx + r + 1, w))
        y0, y1 = int(max(cy - r, 0)), int(min(cy + r + 1, h))
        if x1 <= x0 or y1 <= y0:
            continue
        m = (xx[y0:y1, x0:x1] - cx) ** 2 + (yy[y0:y1, x0:x1] - cy) ** 2 <= r * r
        img[y0:y1, x0:x1][m] = val
    img += rng.integers(-4, 5, size=(h, w))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def _planar_field(rng: np.random.Generator, h: int, w: int, lo: float, hi: float, nplanes: int = 8) -> np.ndarray:
    sx, sy = rng.uniform(0, w, nplanes), rng.uniform(0, h, nplanes)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    d2 = (xx[None] - sx[:, None, None]) ** 2 + (yy[None] - sy[:, None, None]) ** 2
    lab = np.argmin(d2, axis=0)
    a = rng.uniform(lo, hi, nplanes)
    bx = rng.uniform(-0.02, 0.02, nplanes) * (hi - lo) / 10
    by = rng.uniform(-0.02, 0.02, nplanes) * (hi - lo) / 10
    f = a[lab] + bx[lab] * (xx - sx[lab]) + by[lab] * (yy - sy[lab])
    return np.clip(f, lo, hi)


def stereo_pair(h: int, w: int, t: int, base_seed: int = 2) -> tuple[np.ndarray, np.ndarray]:
    """C2 generator: left = textured_image(seed 2+t); right = left warped by disparity."""
    left = textured_image(h, w, base_seed + t)
    rng = np.random.default_rng(1000 + base_seed + t)
    disp = _planar_field(rng, h, w, 2.0, 96.0)
    xs = np.arange(w)[None, :] + disp
    xi = np.clip(np.rint(xs).astype(int), 0, w - 1)
    right = np.take_along_axis(left, xi, axis=1).astype(np.int32)
    nrng = np.random.default_rng(2000 + base_seed + t)
    right += nrng.integers(-2, 3, size=(h, w))
    return left, np.clip(right, 0, 255).astype(np.uint8)


def _stream_part(args):
    h, w, ts, base_seed = args
    return [stereo_pair(h, w, t, base_seed) for t in ts]


def stream_workers() -> int:
    """Generator processes for stereo_stream: the usable host threads, at most 16 (the GPU box's
    CPU share; OMP_NUM_THREADS is 16 there)."""
    import os
    n = len(os.sched_getaffinity(0))
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, min(16, n))


def stereo_stream(h: int, w: int, n: int, base_seed: int = 2, t_step: int = 1,
                  workers: int | None = None) -> list[tuple[np.ndarray, np.ndarray]]:
    """SURVEY §8d's C2 input stream: frame t (t = 0 .. n-1) = stereo_pair(h, w, t_step * t,
    base_seed), i.e. left seed base_seed + t_step * t, disparity seed 1000 + that, noise seed
    2000 + that. C2: base_seed 2, t_step 1, n = 512; C5 rank r: base_seed 10 + r, t_step 8 (no two
    ranks share a frame). Generated by `workers` spawned processes (numpy only; the parent may
    already hold the GPU, so no fork), identical to the serial loop."""
    ts = [t_step * t for t in range(n)]
    workers = stream_workers() if workers is None else max(1, workers)
    if workers == 1 or n < 8:
        return _stream_part((h, w, ts, base_seed))
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    k = max(1, -(-n // (4 * workers)))   # ~4 parts per worker
    parts = [(h, w, ts[i:i + k], base_seed) for i in range(0, n, k)]
    with ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
        out = []
        for p in ex.map(_stream_part, parts):
            out.extend(p)
    return out


def rgbd_frame(h: int, w: int, t: int, base_seed: int = 3) -> tuple[np.ndarray, np.ndarray]:
    """C3 generator: gray frame shifted 0-3 px per frame + float depth (m), 5 % holes."""
    base = textured_image(h + 64, w + 64, base_seed)
    sx = (t * 3) % 32
    sy = (t * 2) % 32
    gray = np.ascontiguousarray(base[sy:sy + h, sx:sx + w])
    rng = np.random.default_rng(5000 + base_seed + t)
    z = _planar_field(rng, h, w, 0.5, 4.0)
    depth_u16 = np.rint(z * 5000.0).astype(np.uint16)
    holes = rng.random((h, w)) < 0.05
    depth_u16[holes] = 0
    depth = (depth_u16.astype(np.float32) * np.float32(1.0 / 5000.0)).astype(np.float32)
    return gray, depth


# ---------------------------------------------------------------------------------------
# C4: synthetic LocalBundleAdjustment graph, after the homework simulator
# pattern (orbslam_homework/hw4_answer/src/utils.cpp:35-69, demo/main.cpp:28-86):
# 20 local KFs on a forward path 1 m apart with +-2 deg yaw (mnId 1..20, free) plus two fixed
# cameras (mnId 0 and 21); 3000 points at 4-40 m, each seen by a contiguous run of 3..8 KFs;
# 70 % stereo observations; octave ~ features per level, pixel noise sigma = scale[octave];
# 5 % outliers (+-20 px); initial poses perturbed 0.5 deg / 5 cm, points 10 cm.
# ---------------------------------------------------------------------------------------
KITTI_CAM = (718.856, 718.856, 607.1928, 185.2157, 386.1448)   # Stereo/KITTI00-02.yaml


def _rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _small_rot(rng, deg):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = np.deg2rad(deg) * rng.uniform(-1, 1)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def localba_problem(seed: int = 4, n_kf: int = 20, n_points: int = 3000, stereo_frac: float = 0.7,
                    outlier_frac: float = 0.05, W: int = 1241, H: int = 376):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = KITTI_CAM
    scales = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    inv_sigma2 = (np.float32(1) / (scales * scales)).astype(np.float32)
    feat = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    oct_p = feat / feat.sum()
    ids = list(range(0, n_kf + 2))                       # 0 = fixed, 1..n_kf free, n_kf+1 fixed
    Rwc, Cw = [], []
    for i in ids:
        Rwc.append(_rot_y(np.deg2rad(rng.uniform(-2, 2))))
        Cw.append(np.array([rng.normal(0, 0.05), rng.normal(0, 0.02), float(i)]))
    Tcw_true = []
    for R, C in zip(Rwc, Cw):
        Rcw = R.T
        T = np.eye(4)
        T[:3, :3] = Rcw
        T[:3, 3] = -Rcw @ C
        Tcw_true.append(T)
    pts, obs = [], []
    for p in range(n_points):
        k = int(rng.integers(3, 9))
        first = int(rng.integers(1, n_kf - k + 2))
        run = list(range(first, first + k))
        if first == 1 and rng.random() < 0.5:
            run = [0] + run
        if run[-1] == n_kf and rng.random() < 0.5:
            run = run + [n_kf + 1]
        last = run[-1]
        z = rng.uniform(4, 40)
        u = rng.uniform(0.3 * W, 0.7 * W)
        v = rng.uniform(0.3 * H, 0.7 * H)
        Xc = np.array([(u - cx) / fx * z, (v - cy) / fy * z, z])
        T = Tcw_true[last]
        Xw = T[:3, :3].T @ (Xc - T[:3, 3])
        pts.append(Xw)
        for kf in run:
            T = Tcw_true[kf]
            Xc = T[:3, :3] @ Xw + T[:3, 3]
            if Xc[2] <= 0.5:
                continue
            o = int(rng.choice(8, p=oct_p))
            sig = float(scales[o])
            uu = fx * Xc[0] / Xc[2] + cx + rng.normal(0, sig)
            vv = fy * Xc[1] / Xc[2] + cy + rng.normal(0, sig)
            uR = -1.0
            if rng.random() < stereo_frac:
                uR = uu - bf / Xc[2] + rng.normal(0, sig)
            if rng.random() < outlier_frac:
                du, dv = rng.uniform(-20, 20, 2)
                uu += du
                vv += dv
                if uR >= 0:
                    uR += du
            obs.append((p, kf, uu, vv, uR, inv_sigma2[o]))
    # perturbed initial estimates (what LocalBA starts from)
    Tcw0 = []
    for i, T in enumerate(Tcw_true):
        T0 = T.copy()
        if 1 <= i <= n_kf:
            Rw = T[:3, :3].T @ _small_rot(rng, 0.5)
            Cc = -T[:3, :3].T @ T[:3, 3] + rng.uniform(-0.05, 0.05, 3)
            T0[:3, :3] = Rw.T
            T0[:3, 3] = -Rw.T @ Cc
        Tcw0.append(T0)
    X0 = np.array(pts) + rng.uniform(-0.1, 0.1, (n_points, 3))
    maxKFid = max(ids)
    obs.sort(key=lambda o: (o[0], o[1]))                  # point list order, then KF order
    ob = np.array(obs, dtype=np.float64)
    return {
        "pose_id": np.array(ids, np.int32),
        "pose_fixed": np.array([1 if (i == 0 or i == n_kf + 1) else 0 for i in ids], np.uint8),
        "pose_Tcw": np.array(Tcw0, np.float32).reshape(-1, 16),
        "pose_cam": np.tile(np.array(KITTI_CAM, np.float32), (len(ids), 1)),
        "point_id": (np.arange(n_points) + maxKFid + 1).astype(np.int32),
        "point_Xw": X0.astype(np.float32),
        "edge_point": ob[:, 0].astype(np.int32),
        "edge_pose": ob[:, 1].astype(np.int32),
        "edge_obs": ob[:, 2:5].astype(np.float32),
        "edge_inv_sigma2": ob[:, 5].astype(np.float32),
        "truth_Tcw": np.array(Tcw_true, np.float64),
        "truth_Xw": np.array(pts, np.float64),
    }


# ---------------------------------------------------------------------------------------
# Tracking matchers: one current frame + a local map (+ the last
# frame for the motion-model matcher). Keypoints are synthetic (not extracted): projections
# of map points with pixel noise sigma = scale[octave], descriptors = the map point's with
# 0..60 flipped bits, plus clones competing for the same keypoints (exercises the greedy
# claim order) and uniformly random distractors. Octaves ~ features per level.
# ---------------------------------------------------------------------------------------
TRACK_KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
MP_BAD, MP_HAS_OBS, MP_IN_FRAME, MP_FOUND = 1, 2, 4, 8


def _flip_bits(rng, d: np.ndarray, k: int) -> np.ndarray:
    d = d.copy()
    for b in rng.choice(256, size=k, replace=False):
        d[b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def _pose_dict(R: np.ndarray, t: np.ndarray):
    Rf = R.astype(np.float32)
    tf = t.astype(np.float32)
    T = np.concatenate([Rf, tf[:, None]], axis=1).astype(np.float32)
    Ow = (-(Rf.astype(np.float64).T @ tf.astype(np.float64))).astype(np.float32)
    return T, Ow


def tracking_problem(seed: int = 5, n_kp: int = 2000, n_mp: int = 3000, W: int = 1241, H: int = 376,
                     stereo: bool = True, motion: str = "forward", clone_frac: float = 0.15,
                     n_last: int = 1500):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = (np.float32(v) for v in KITTI_CAM)
    mb = np.float32(bf / fx)
    nl = 8
    sf = np.ones(nl, np.float32)
    for i in range(1, nl):
        sf[i] = np.float32(sf[i - 1] * np.float32(1.2))
    feat = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    oct_p = feat / feat.sum()
    Rcw = _small_rot(rng, 2.0)
    tcw = rng.normal(0, 0.3, 3)
    Tcw, Ow = _pose_dict(Rcw, tcw)
    Rwc = Rcw.T
    n_true = int(n_mp * (1 - clone_frac))
    # map points: projections (some outside the image), depth 3..45 m (some behind)
    u = rng.uniform(-30, W + 30, n_true)
    v = rng.uniform(-30, H + 30, n_true)
    z = rng.uniform(3, 45, n_true)
    z[rng.random(n_true) < 0.03] *= -1
    Pc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (Pc - tcw) @ Rcw            # Rwc (Pc - tcw)
    octv = rng.choice(nl, size=n_true, p=oct_p)
    Ocw = -Rwc @ tcw
    dist = np.linalg.norm(Xw - Ocw, axis=1)
    maxd = dist * (1.2 ** octv) * rng.uniform(0.92, 1.08, n_true)
    maxd[rng.random(n_true) < 0.04] *= 0.3                         # out of the scale range
    # viewing direction of a reference keyframe: mostly close, some beyond 60 degrees
    ref = Ocw + rng.normal(0, 0.5, (n_true, 3))
    nrm = Xw - ref
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    wild = rng.random(n_true) < 0.08
    nrm[wild] = rng.normal(size=(int(wild.sum()), 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    mdesc = rng.integers(0, 256, (n_true, 32), dtype=np.uint8)
    # clones: another map point at nearly the same place with a similar descriptor
    n_clone = n_mp - n_true
    src = rng.integers(0, n_true, n_clone)
    Xw = np.concatenate([Xw, Xw[src] + rng.normal(0, 0.02, (n_clone, 3))])
    nrm = np.concatenate([nrm, nrm[src]])
    maxd = np.concatenate([maxd, maxd[src]])
    octv = np.concatenate([octv, octv[src]])
    mdesc = np.concatenate([mdesc, np.stack([_flip_bits(rng, mdesc[s], int(rng.integers(0, 30))) for s in src])
                            if n_clone else np.zeros((0, 32), np.uint8)])
    perm = rng.permutation(n_mp)
    Xw, nrm, maxd, octv, mdesc = Xw[perm], nrm[perm], maxd[perm], octv[perm], mdesc[perm]
    mind = maxd / sf[nl - 1]
    flags = np.where(rng.random(n_mp) < 0.9, MP_HAS_OBS, 0).astype(np.uint8)
    flags[rng.random(n_mp) < 0.03] |= MP_BAD
    flags[rng.random(n_mp) < 0.05] |= MP_IN_FRAME
    # keypoints
    kps, kdesc, kur, kgen = [], [], [], []
    Pcm = Xw @ Rcw.T + tcw
    for m in range(n_mp):
        if len(kps) >= int(0.75 * n_kp) or Pcm[m, 2] <= 0.1 or rng.random() < 0.3:
            continue
        uu = fx * Pcm[m, 0] / Pcm[m, 2] + cx
        vv = fy * Pcm[m, 1] / Pcm[m, 2] + cy
        for _ in range(1 + int(rng.random() < 0.2)):             # sometimes two detections
            o = int(np.clip(octv[m] + rng.integers(-1, 2), 0, nl - 1))
            s = float(sf[o])
            x = uu + rng.normal(0, s)
            y = vv + rng.normal(0, s)
            if not (0 <= x < W and 0 <= y < H):
                continue
            kps.append((x, y, 31 * s, rng.uniform(0, 360), 0, o, -1))
            kdesc.append(_flip_bits(rng, mdesc[m], int(rng.integers(0, 60))))
            ur = x - bf / Pcm[m, 2] + rng.normal(0, 0.5) if (stereo and rng.random() < 0.6) else -1.0
            kur.append(ur)
            kgen.append(m)
    while len(kps) < n_kp:
        o = int(rng.choice(nl, p=oct_p))
        kps.append((rng.uniform(0, W), rng.uniform(0, H), 31 * float(sf[o]), rng.uniform(0, 360), 0, o, -1))
        kdesc.append(rng.integers(0, 256, 32, dtype=np.uint8))
        kur.append(float(rng.uniform(0, W)) if (stereo and rng.random() < 0.5) else -1.0)
        kgen.append(-1)
    kps = kps[:n_kp]
    order = rng.permutation(len(kps))
    keys = np.array([kps[i] for i in order], TRACK_KP_DTYPE)
    kdesc = np.stack([kdesc[i] for i in order]).astype(np.uint8)
    kur = np.array([kur[i] for i in order], np.float32)
    kgen = np.array([kgen[i] for i in order], np.int64)
    frame = {"keys_un": keys, "u_right": kur, "desc": kdesc, "Tcw": Tcw, "Ow": Ow, "fx": fx, "fy": fy, "cx": cx,
             "cy": cy, "mbf": bf, "mb": mb, "min_x": 0.0, "max_x": float(W), "min_y": 0.0, "max_y": float(H),
             "nlevels": nl, "log_scale_factor": np.float32(np.log(np.float32(1.2))), "scale_factors": sf,
             "inv_level_sigma2": (np.float32(1) / (sf * sf)).astype(np.float32)}
    mp = {"Xw": Xw.astype(np.float32), "normal": nrm.astype(np.float32), "min_dist": mind.astype(np.float32),
          "max_dist": maxd.astype(np.float32), "desc": mdesc, "flags": flags}
    # last frame (motion model): the camera 1 m behind / ahead / in place along its optical axis
    shift = {"forward": 1.0, "backward": -1.0, "static": 0.2}[motion]
    Rlw = Rcw @ _small_rot(rng, 1.0)
    Olw = Ocw - shift * Rwc[:, 2]
    tlw = -Rlw @ Olw
    lTcw, lOw = _pose_dict(Rlw, tlw)
    nL = n_last
    last_mp = np.full(nL, -1, np.int32)
    pick = rng.choice(n_mp, size=min(n_mp, int(0.8 * nL)), replace=False)
    slots = rng.choice(nL, size=len(pick), replace=False)
    last_mp[slots] = pick
    lk = np.zeros(nL, TRACK_KP_DTYPE)
    lk["x"] = rng.uniform(0, W, nL)
    lk["y"] = rng.uniform(0, H, nL)
    lk["octave"] = rng.choice(nl, size=nL, p=oct_p)
    lk["octave"][slots] = np.clip(octv[pick] + rng.integers(-1, 2, len(pick)), 0, nl - 1)
    lk["angle"] = rng.uniform(0, 360, nL).astype(np.float32)
    lk["size"] = 31.0
    lk["class_id"] = -1
    # a consistent in-plane rotation (12 +- 3 deg) between the last and the current keypoint of
    # the same map point for most matches, random for the rest (rotation-histogram check)
    first_kp = {}
    for i, g in enumerate(kgen):
        if g >= 0 and g not in first_kp:
            first_kp[int(g)] = i
    for i in slots:
        j = first_kp.get(int(last_mp[i]))
        if j is not None and rng.random() < 0.8:
            lk["angle"][i] = np.float32((float(keys["angle"][j]) + 12.0 + rng.normal(0, 3)) % 360.0)
    last = {"keys_un": lk, "u_right": np.full(nL, -1, np.float32), "desc": np.zeros((nL, 32), np.uint8),
            "Tcw": lTcw, "Ow": lOw, **{k: frame[k] for k in ("fx", "fy", "cx", "cy", "mbf", "mb", "min_x", "max_x",
                                                               "min_y", "max_y", "nlevels", "log_scale_factor",
                                                               "scale_factors", "inv_level_sigma2")}}
    last_out = (rng.random(nL) < 0.05).astype(np.uint8)
    kp_blocked = (rng.random(len(keys)) < 0.05).astype(np.uint8)
    return {"frame": frame, "map": mp, "last": last, "last_mp": last_mp, "last_outlier": last_out,
            "kp_blocked": kp_blocked}


# ---------------------------------------------------------------------------------------
# Optimizer::PoseOptimization: one frame's map-point matches. KITTI
# camera; points 3..45 m in front; observations = projections of the true pose with noise
# sigma = scale[octave] (uR from the true depth for stereo edges), `outlier_frac` of them
# moved 8..60 px; the starting pose is the true one perturbed by ~1 deg / 10 cm (a motion-
# model prediction).
# ---------------------------------------------------------------------------------------
def pose_problem(seed: int = 7, n: int = 600, stereo_frac: float = 0.6, outlier_frac: float = 0.15,
                 W: int = 1241, H: int = 376, rot_deg: float = 1.0, trans_m: float = 0.1):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = KITTI_CAM
    sf = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    inv_s2 = (np.float32(1) / (sf * sf)).astype(np.float32)
    feat = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    Rt = _small_rot(rng, 3.0)
    tt = rng.normal(0, 1.0, 3)
    u = rng.uniform(0, W, n)
    v = rng.uniform(0, H, n)
    z = rng.uniform(3, 45, n)
    Pc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (Pc - tt) @ Rt
    octv = rng.choice(8, size=n, p=feat / feat.sum())
    s = sf[octv].astype(np.float64)
    ou = u + rng.normal(0, 1, n) * s
    ov = v + rng.normal(0, 1, n) * s
    ur = ou - bf / z + rng.normal(0, 1, n) * s
    st = rng.random(n) < stereo_frac
    bad = rng.random(n) < outlier_frac
    ang = rng.uniform(0, 2 * np.pi, int(bad.sum()))
    mag = rng.uniform(8, 60, int(bad.sum()))
    ou[bad] += mag * np.cos(ang)
    ov[bad] += mag * np.sin(ang)
    obs = np.stack([ou, ov, np.where(st, ur, -1.0)], 1).astype(np.float32)
    R0 = Rt @ _small_rot(rng, rot_deg)
    t0 = tt + rng.normal(0, trans_m, 3)
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = R0
    T[:3, 3] = t0
    return {"Xw": Xw.astype(np.float32), "obs": obs, "inv_sigma2": inv_s2[octv].astype(np.float32),
            "Tcw": T, "cam": (np.float32(fx), np.float32(fy), np.float32(cx), np.float32(cy), np.float32(bf)),
            "true_Tcw": np.concatenate([np.concatenate([Rt, tt[:, None]], 1), [[0, 0, 0, 1]]]).astype(np.float32),
            "is_outlier": bad}


# ---------------------------------------------------------------------------------------
# DBoW2 vocabulary. ORBvoc.txt is not in the reference tree
# (.MISSING_LARGE_BLOBS), so a synthetic vocabulary of the same shape is generated: a full
# k-ary tree of depth L in breadth-first node order (DBoW2's saveToTextFile order), each child
# descriptor = its parent's with each bit flipped with probability p_level (coarse-to-fine
# clusters), leaf weights = IDF-like values in [0.5, 8] with `stop_frac` stopped (weight 0)
# words, internal weights 0; scoring L1_NORM, weighting TF_IDF (ORBvoc.txt header 10 6 0 0).
# ---------------------------------------------------------------------------------------
def vocabulary(seed: int = 11, k: int = 10, L: int = 6, stop_frac: float = 0.02):
    rng = np.random.default_rng(seed)
    sizes = [k ** l for l in range(L + 1)]
    n = sum(sizes)
    parent = np.full(n, -1, np.int32)
    desc = np.zeros((n, 32), np.uint8)
    leaf = np.zeros(n, np.uint8)
    weight = np.zeros(n, np.float64)
    desc[0] = rng.integers(0, 256, 32, dtype=np.uint8)
    start_prev, start = 0, 1
    for l in range(1, L + 1):
        m = sizes[l]
        parent[start:start + m] = np.repeat(np.arange(start_prev, start_prev + sizes[l - 1], dtype=np.int32), k)
        p = 0.35 / (1.0 + 0.6 * (l - 1))
        flips = np.packbits(rng.random((m, 256)) < p, axis=1, bitorder="little")
        desc[start:start + m] = desc[parent[start:start + m]] ^ flips
        start_prev, start = start, start + m
    leaf[n - sizes[L]:] = 1
    w = rng.uniform(0.5, 8.0, sizes[L])
    w[rng.random(sizes[L]) < stop_frac] = 0.0
    weight[n - sizes[L]:] = w
    return {"k": k, "L": L, "scoring": 0, "weighting": 0, "parent": parent, "is_leaf": leaf, "desc": desc,
            "weight": weight}


def vocabulary_text(voc: dict) -> str:
    """TemplatedVocabulary::saveToTextFile layout (TemplatedVocabulary.h:1479-1530)."""
    lines = [f"{voc['k']} {voc['L']} {voc['scoring']} {voc['weighting']}"]
    for i in range(1, len(voc["parent"])):
        d = " ".join(str(int(b)) for b in voc["desc"][i])
        lines.append(f"{int(voc['parent'][i])} {int(voc['is_leaf'][i])} {d} {float(voc['weight'][i])!r}")
    return "\n".join(lines) + "\n"


def bow_features(voc: dict, seed: int, n: int = 2000, noise_bits: int = 24, random_frac: float = 0.2):
    """Descriptors near random leaves (each bit flipped w.p. noise_bits/256) plus random ones."""
    rng = np.random.default_rng(seed)
    leaves = np.nonzero(voc["is_leaf"])[0]
    pick = rng.choice(leaves, size=n)
    flips = np.packbits(rng.random((n, 256)) < noise_bits / 256.0, axis=1, bitorder="little")
    d = voc["desc"][pick] ^ flips
    r = rng.random(n) < random_frac
    d[r] = rng.integers(0, 256, (int(r.sum()), 32), dtype=np.uint8)
    return np.ascontiguousarray(d)


# ---------------------------------------------------------------------------------------
# BoW-guided matchers: two keyframes A, B of a common scene (KITTI
# camera, B ~0.8 m ahead of A). Keypoints of the same 3D point share a base descriptor
# (0..40 flipped bits), a consistent in-plane rotation (+10 deg) and, mostly, a FeatureVector
# node (node = point id mod 100 -- the level-2 nodes of a k=10 vocabulary at levelsup 4);
# distractor keypoints fill up to n. A's keypoints carry map points (some bad) for
# SearchByBoW; both frames carry some for SearchForTriangulation. F12 / Cw1 / T2w follow
# LocalMapping::ComputeF12 and KeyFrame::GetCameraCenter.
# ---------------------------------------------------------------------------------------
def _fv_from_nodes(nodes: np.ndarray):
    order = np.lexsort((np.arange(len(nodes)), nodes))
    sn = nodes[order]
    uniq, start = np.unique(sn, return_index=True)
    return (uniq.astype(np.uint32), np.append(start, len(nodes)).astype(np.int32), order.astype(np.int32))


def bow_match_problem(seed: int = 3, n: int = 2000, n_points: int = 1600, stereo_frac: float = 0.5,
                      mp_frac_a: float = 0.6, mp_frac_b: float = 0.3, W: int = 1241, H: int = 376):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = (np.float32(v) for v in KITTI_CAM)
    sf = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    s2 = (sf * sf).astype(np.float32)
    feat = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    oct_p = feat / feat.sum()
    Ra = _small_rot(rng, 2.0)
    ta = rng.normal(0, 0.5, 3)
    Rb = Ra @ _small_rot(rng, 2.0)
    Ca = -Ra.T @ ta
    Cb = Ca + Ra.T @ np.array([rng.normal(0, 0.1), rng.normal(0, 0.05), 0.8])
    tb = -Rb @ Cb
    z = rng.uniform(4, 40, n_points)
    u = rng.uniform(0, W, n_points)
    v = rng.uniform(0, H, n_points)
    Pa = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Pw = (Pa - ta) @ Ra
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    ang = rng.uniform(0, 360, n_points)
    node = (np.arange(n_points) % 100).astype(np.int64)

    def frame(R, t, dang, frac, mp_frac):
        kps, desc, ur, nodes, mp = [], [], [], [], []
        Pc = Pw @ R.T + t
        for p in range(n_points):
            if rng.random() > frac or Pc[p, 2] <= 0.5:
                continue
            uu = fx * Pc[p, 0] / Pc[p, 2] + cx
            vv = fy * Pc[p, 1] / Pc[p, 2] + cy
            o = int(rng.choice(8, p=oct_p))
            s = float(sf[o])
            x, y = uu + rng.normal(0, 0.7 * s), vv + rng.normal(0, 0.7 * s)
            if not (0 <= x < W and 0 <= y < H):
                continue
            kps.append((x, y, 31 * s, (ang[p] + dang + rng.normal(0, 2)) % 360, 0, o, -1))
            desc.append(_flip_bits(rng, base[p], int(rng.integers(0, 40))))
            ur.append(x - bf / Pc[p, 2] if rng.random() < stereo_frac else -1.0)
            nodes.append(node[p] if rng.random() < 0.9 else int(rng.integers(0, 100)))
            mp.append(p if rng.random() < mp_frac else -1)
        while len(kps) < n:
            o = int(rng.choice(8, p=oct_p))
            kps.append((rng.uniform(0, W), rng.uniform(0, H), 31 * float(sf[o]), rng.uniform(0, 360), 0, o, -1))
            desc.append(rng.integers(0, 256, 32, dtype=np.uint8))
            ur.append(float(rng.uniform(0, W)) if rng.random() < stereo_frac else -1.0)
            nodes.append(int(rng.integers(0, 100)))
            mp.append(int(rng.integers(0, n_points)) if rng.random() < mp_frac * 0.5 else -1)
        perm = rng.permutation(len(kps))[:n]
        keys = np.array([kps[i] for i in perm], TRACK_KP_DTYPE)
        fvn, fvs, fvf = _fv_from_nodes(np.array([nodes[i] for i in perm], np.int64))
        mpa = np.array([mp[i] for i in perm], np.int32)
        return {"keys_un": keys, "desc": np.stack([desc[i] for i in perm]).astype(np.uint8),
                "u_right": np.array([ur[i] for i in perm], np.float32), "mp": mpa,
                "mp_bad": ((rng.random(len(perm)) < 0.05) & (mpa >= 0)).astype(np.uint8),
                "fv_nodes": fvn, "fv_start": fvs, "fv_features": fvf, "fx": fx, "fy": fy, "cx": cx, "cy": cy,
                "nlevels": 8, "scale_factors": sf, "level_sigma2": s2}

    A = frame(Ra, ta, 0.0, 0.85, mp_frac_a)
    B = frame(Rb, tb, -10.0, 0.85, mp_frac_b)
    # LocalMapping::ComputeF12 (float): F12 = K1^-T [t12]x R12 K2^-1
    R1, t1, R2, t2 = Ra.astype(np.float32), ta.astype(np.float32), Rb.astype(np.float32), tb.astype(np.float32)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]], np.float32)
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)
    Kinv = np.linalg.inv(K.astype(np.float64)).astype(np.float32)
    F12 = (Kinv.T @ tx @ R12 @ Kinv).astype(np.float32)
    T2w = np.concatenate([R2, t2[:, None]], 1).astype(np.float32)
    Cw1 = (-(R1.astype(np.float64).T @ t1.astype(np.float64))).astype(np.float32)
    return {"A": A, "B": B, "F12": F12, "Cw1": Cw1, "T2w": T2w}


def reloc_problem(seed: int = 40, found_frac: float = 0.2, blocked_frac: float = 0.1, **kw):
    """Tracking::Relocalization's projection search (ORBmatcher.cc:1922-2066): a tracking
    problem whose last frame plays the candidate keyframe (its keypoint angles and map point
    matches), ~found_frac of the map points in sAlreadyFound (MP_FOUND) and ~blocked_frac of
    the current keypoints already holding a map point (kp_blocked)."""
    p = tracking_problem(seed, **kw)
    rng = np.random.default_rng(seed + 7919)
    m = p["map"]
    flags = np.array(m["flags"], np.uint8, copy=True)
    flags[rng.random(len(flags)) < found_frac] |= MP_FOUND
    p["map"] = dict(m, flags=flags)
    n = len(p["frame"]["keys_un"])
    p["kp_blocked"] = (rng.random(n) < blocked_frac).astype(np.uint8)
    return p


# ---------------------------------------------------------------------------------------
# New map points (LocalMapping::CreateNewMapPoints): the current
# keyframe and one neighbour observing a shared cloud, keypoints = projections with pixel noise
# 0.5 x scale[octave], stereo / RGB-D depth on a fraction of them, plus the matched pairs in
# SearchForTriangulation's idx1 order with ~wrong_frac wrong partners (rejected by the
# reprojection gates). cam = "kitti" (rectified stereo: mvKeys == mvKeysUn) or "tum" (RGB-D,
# measured depth, mvKeys = distorted positions != mvKeysUn).
# ---------------------------------------------------------------------------------------
TUM1_CAM = (517.306408, 516.469215, 318.643040, 255.313989, 40.0)   # RGB-D/TUM1.yaml


def newpoints_problem(seed: int = 21, n: int = 1500, n_points: int = 1400, stereo_frac: float = 0.6,
                      baseline: float = 0.8, wrong_frac: float = 0.08, cam: str = "kitti", zmax: float = 60.0):
    rng = np.random.default_rng(seed)
    if cam == "kitti":
        fx, fy, cx, cy, bf = (np.float32(v) for v in KITTI_CAM)
        W, H = 1241, 376
    else:
        fx, fy, cx, cy, bf = (np.float32(v) for v in TUM1_CAM)
        W, H = 640, 480
    mb = np.float32(bf / fx)
    sf = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    s2 = (sf * sf).astype(np.float32)
    feat = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    oct_p = feat / feat.sum()
    R1 = _small_rot(rng, 2.0)
    t1 = rng.normal(0, 0.5, 3)
    C1 = -R1.T @ t1
    C2 = C1 + R1.T @ np.array([rng.normal(0, 0.3), rng.normal(0, 0.05), baseline])
    R2 = R1 @ _small_rot(rng, 3.0)
    t2 = -R2 @ C2
    z = np.where(rng.random(n_points) < 0.8, rng.uniform(2, 25, n_points), rng.uniform(25, zmax, n_points))
    u = rng.uniform(0, W, n_points)
    v = rng.uniform(0, H, n_points)
    Pw = (np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1) - t1) @ R1

    def keyframe(R, t):
        Pc = Pw @ R.T + t
        rows, owner = [], []
        for p in range(n_points):
            if Pc[p, 2] <= 0.5:
                continue
            o = int(rng.choice(8, p=oct_p))
            s = float(sf[o])
            x = fx * Pc[p, 0] / Pc[p, 2] + cx + rng.normal(0, 0.5 * s)
            y = fy * Pc[p, 1] / Pc[p, 2] + cy + rng.normal(0, 0.5 * s)
            if not (0 <= x < W and 0 <= y < H):
                continue
            if rng.random() < stereo_frac:
                d = Pc[p, 2] * (1 + rng.normal(0, 0.01))
                ur = x - bf / d
            else:
                d, ur = -1.0, -1.0
            rows.append((x, y, o, ur, d))
            owner.append(p)
        while len(rows) < n:
            o = int(rng.choice(8, p=oct_p))
            rows.append((rng.uniform(0, W), rng.uniform(0, H), o, -1.0, -1.0))
            owner.append(-1)
        perm = rng.permutation(len(rows))[:n]
        keys_un = np.zeros(n, TRACK_KP_DTYPE)
        for i, j in enumerate(perm):
            x, y, o, ur, d = rows[j]
            keys_un[i] = (x, y, 31 * float(sf[o]), rng.uniform(0, 360), 0, o, -1)
        keys = keys_un.copy()
        if cam != "kitti":   # mvKeys: the distorted positions (UnprojectStereo reads them)
            keys["x"] += rng.normal(0, 1.5, n).astype(np.float32)
            keys["y"] += rng.normal(0, 1.5, n).astype(np.float32)
        ur = np.array([rows[j][3] for j in perm], np.float32)
        dep = np.array([rows[j][4] for j in perm], np.float32)
        if cam != "kitti":   # RGB-D: uR = xUn - mbf / d (Frame::ComputeStereoFromRGBD)
            ok = dep > 0
            ur = np.where(ok, keys_un["x"] - bf / np.where(ok, dep, 1), -1).astype(np.float32)
        else:                # stereo: depth = mbf / disparity
            ok = ur >= 0
            disp = keys_un["x"] - ur
            dep = np.where(ok, bf / np.where(ok, disp, 1), -1).astype(np.float32)
        T, Ow = _pose_dict(R, t)
        kf = {"keys": keys, "keys_un": keys_un, "u_right": ur, "depth": dep, "Tcw": T.reshape(-1), "Ow": Ow,
              "fx": fx, "fy": fy, "cx": cx, "cy": cy, "invfx": np.float32(1) / fx, "invfy": np.float32(1) / fy,
              "mb": mb, "mbf": bf, "nlevels": 8, "scale_factors": sf, "level_sigma2": s2}
        return kf, np.array([owner[j] for j in perm], np.int64)

    k1, own1 = keyframe(R1, t1)
    k2, own2 = keyframe(R2, t2)
    where2 = {int(p): i for i, p in enumerate(own2) if p >= 0}
    pairs = []
    for i1 in range(n):
        p = int(own1[i1])
        if p >= 0 and p in where2:
            pairs.append((i1, where2[p] if rng.random() >= wrong_frac else int(rng.integers(0, n))))
    return {"kf1": k1, "kf2": k2, "pairs": np.array(pairs, np.int32).reshape(-1, 2),
            "ratio_factor": np.float32(1.5) * np.float32(1.2)}


# ---------------------------------------------------------------------------------------
# Loop closing (SearchBySim3): two keyframes of a KITTI-like camera 1.5 m apart observing a
# shared cloud, each keypoint of an observed point carries the point (GetMapPointMatches) with
# probability 0.9, descriptors = the point's with 0..40 flipped bits, distractors fill to n;
# (s12, R12, t12) = the relative pose of camera 2 in camera 1 (s12 = 1 unless given);
# matches12 = ~10 % of the shared points already matched (SearchByBoW's output).
# ---------------------------------------------------------------------------------------
def sim3_pair_problem(seed: int = 80, n: int = 1500, n_points: int = 1300, s12: float = 1.0, W: int = 1241,
                      H: int = 376, pre_frac: float = 0.1):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = (np.float32(v) for v in KITTI_CAM)
    mb = np.float32(bf / fx)
    nl = 8
    sf = np.ones(nl, np.float32)
    for i in range(1, nl):
        sf[i] = np.float32(sf[i - 1] * np.float32(1.2))
    feat = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    oct_p = feat / feat.sum()
    R1 = _small_rot(rng, 2.0)
    t1 = rng.normal(0, 0.3, 3)
    C1 = -R1.T @ t1
    C2 = C1 + R1.T @ np.array([rng.normal(0, 0.3), rng.normal(0, 0.05), 1.5])
    R2 = R1 @ _small_rot(rng, 4.0)
    t2 = -R2 @ C2
    z = rng.uniform(3, 40, n_points)
    u = rng.uniform(-20, W + 20, n_points)
    v = rng.uniform(-20, H + 20, n_points)
    Pw = (np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1) - t1) @ R1
    octv = rng.choice(nl, size=n_points, p=oct_p)
    dist = np.linalg.norm(Pw - C1, axis=1)
    maxd = (dist * (1.2 ** octv) * rng.uniform(0.9, 1.12, n_points)).astype(np.float32)
    mind = (maxd / sf[nl - 1]).astype(np.float32)
    nrm = (Pw - C1) / dist[:, None]
    mdesc = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    flags = np.where(rng.random(n_points) < 0.03, MP_BAD, 0).astype(np.uint8)

    def keyframe(R, t):
        Pc = Pw @ R.T + t
        rows = []
        for p in range(n_points):
            if Pc[p, 2] <= 0.5 or rng.random() < 0.15:
                continue
            o = int(np.clip(octv[p] + rng.integers(-1, 2), 0, nl - 1))
            s = float(sf[o])
            x = fx * Pc[p, 0] / Pc[p, 2] + cx + rng.normal(0, 0.7 * s)
            y = fy * Pc[p, 1] / Pc[p, 2] + cy + rng.normal(0, 0.7 * s)
            if not (0 <= x < W and 0 <= y < H):
                continue
            rows.append((x, y, o, _flip_bits(rng, mdesc[p], int(rng.integers(0, 40))), p if rng.random() < 0.9 else -1))
        while len(rows) < n:
            o = int(rng.choice(nl, p=oct_p))
            rows.append((rng.uniform(0, W), rng.uniform(0, H), o, rng.integers(0, 256, 32, dtype=np.uint8), -1))
        perm = rng.permutation(len(rows))[:n]
        keys = np.zeros(n, TRACK_KP_DTYPE)
        for i, j in enumerate(perm):
            x, y, o, _, _ = rows[j]
            keys[i] = (x, y, 31 * float(sf[o]), rng.uniform(0, 360), 0, o, -1)
        T, Ow = _pose_dict(R, t)
        fr = {"keys_un": keys, "u_right": np.full(n, -1, np.float32),
              "desc": np.stack([rows[j][3] for j in perm]).astype(np.uint8), "Tcw": T, "Ow": Ow, "fx": fx, "fy": fy,
              "cx": cx, "cy": cy, "mbf": bf, "mb": mb, "min_x": 0.0, "max_x": float(W), "min_y": 0.0,
              "max_y": float(H), "nlevels": nl, "log_scale_factor": np.float32(np.log(np.float32(1.2))),
              "scale_factors": sf, "inv_level_sigma2": (np.float32(1) / (sf * sf)).astype(np.float32)}
        return fr, np.array([rows[j][4] for j in perm], np.int32)

    k1, mp1 = keyframe(R1, t1)
    k2, mp2 = keyframe(R2, t2)
    R1f, t1f, R2f, t2f = (a.astype(np.float32) for a in (R1, t1, R2, t2))
    R12 = (R1f @ R2f.T).astype(np.float32)
    t12 = (-R12 @ t2f + t1f).astype(np.float32)
    in2 = set(int(p) for p in mp2 if p >= 0)
    m12 = np.full(n, -1, np.int32)
    for i in range(n):
        if mp1[i] >= 0 and int(mp1[i]) in in2 and rng.random() < pre_frac:
            m12[i] = mp1[i]
    mp = {"Xw": Pw.astype(np.float32), "normal": nrm.astype(np.float32), "min_dist": mind, "max_dist": maxd,
          "desc": mdesc, "flags": flags}
    return {"kf1": k1, "kf1_mp": mp1, "kf2": k2, "kf2_mp": mp2, "map": mp, "s12": np.float32(s12), "R12": R12,
            "t12": t12, "matches12": m12}
