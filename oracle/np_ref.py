"""ORACLE CROSS-CHECK — TEST INFRASTRUCTURE ONLY.

An independent, vectorised numpy restatement of the integer / float32 kernels of the
extractor, written from the definitions rather than from the C oracle's loop structure, so
that an indexing or ordering slip in either one shows up as a mismatch:

* FAST-9/16 corner test and cornerScore as "largest t for which the pixel is still a
  corner" (cornerScore<16> of OpenCV fast_score.cpp), 3x3 strict NMS inside
  the ROI, row-major emission
* IC_Angle moments over the circular patch (ORBextractor.cc:94-141) + fastAtan2 (A.4)
* steered BRIEF sampling (ORBextractor.cc:153-204) given cos/sin
* 9x9 sigma-2 fixed-point Gaussian blur, reflect-101 (A.3)
* DescriptorDistance (ORBmatcher.cc:2123-2143)
"""
from __future__ import annotations

import numpy as np

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]  # (dx, dy)


def fast_roi(roi: np.ndarray, th: int):
    """cv::FAST(roi, kps, th, nonmax=true) -> (xs, ys, scores) in emission order."""
    th = int(min(max(th, 0), 255))
    img = roi.astype(np.int32)
    rows, cols = img.shape
    if rows < 7 or cols < 7:
        return np.zeros(0, int), np.zeros(0, int), np.zeros(0, int)
    ys, xs = np.mgrid[3:rows - 3, 3:cols - 3]
    v = img[ys, xs]
    d = np.stack([v - img[ys + dy, xs + dx] for dx, dy in RING], axis=-1)   # v - ring
    dd = np.concatenate([d, d[..., :8]], axis=-1)                            # circular
    arcs_min = np.stack([dd[..., s:s + 9].min(-1) for s in range(16)], -1)   # min d over arc
    arcs_nmin = np.stack([(-dd[..., s:s + 9]).min(-1) for s in range(16)], -1)
    M = np.maximum(arcs_min.max(-1), arcs_nmin.max(-1))
    corner = M > th
    score = np.where(corner, np.maximum(th, M) - 1, 0) & 0xFF
    smap = np.zeros((rows, cols), np.int32)
    smap[3:rows - 3, 3:cols - 3] = score
    s = smap[1:-1, 1:-1]
    nb = [smap[1 + dy:rows - 1 + dy, 1 + dx:cols - 1 + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dx or dy]
    keep = np.ones_like(s, bool)
    for n in nb:
        keep &= s > n
    keep &= s > 0
    yy, xx = np.nonzero(keep)
    yy = yy + 1
    xx = xx + 1
    return xx, yy, smap[yy, xx]


def fast_atan2(y: np.float32, x: np.float32) -> np.float32:
    f = np.float32
    r2d = f(180.0 / np.pi)
    p1 = f(0.9997878412794807) * r2d
    p3 = f(-0.3258083974640975) * r2d
    p5 = f(0.1555786518463281) * r2d
    p7 = f(-0.04432655554792128) * r2d
    eps = f(np.finfo(np.float64).eps)
    ax, ay = abs(f(x)), abs(f(y))
    if ax >= ay:
        c = ay / (ax + eps)
        c2 = c * c
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    else:
        c = ax / (ay + eps)
        c2 = c * c
        a = f(90.0) - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    if x < 0:
        a = f(180.0) - a
    if y < 0:
        a = f(360.0) - a
    return f(a)


def umax_table():
    hp = 15
    vmax = int(np.floor(np.float32(hp) * np.sqrt(np.float32(2)) / np.float32(2) + np.float32(1)))
    vmin = int(np.ceil(np.float32(hp) * np.sqrt(np.float32(2)) / np.float32(2)))
    u = [0] * (hp + 1)
    for v in range(vmax + 1):
        u[v] = int(np.rint(np.sqrt(hp * hp - v * v)))
    v0 = 0
    for v in range(hp, vmin - 1, -1):
        while u[v0] == u[v0 + 1]:
            v0 += 1
        u[v] = v0
        v0 += 1
    return np.array(u)


def ic_angle(img: np.ndarray, x: int, y: int, umax) -> np.float32:
    vs, us = np.mgrid[-15:16, -15:16]
    mask = np.abs(us) <= np.asarray(umax)[np.abs(vs)]
    patch = img[y - 15:y + 16, x - 15:x + 16].astype(np.int64)
    m10 = int((us * patch)[mask].sum())
    m01 = int((vs * patch)[mask].sum())
    return fast_atan2(np.float32(m01), np.float32(m10))


def brief(blur: np.ndarray, x: int, y: int, a: np.float32, b: np.float32, pattern: np.ndarray) -> np.ndarray:
    f = np.float32
    p = pattern.reshape(256, 4).astype(np.float32)
    a, b = f(a), f(b)

    def sample(px, py):
        r = np.rint(px * b + py * a).astype(int)
        c = np.rint(px * a - py * b).astype(int)
        return blur[y + r, x + c].astype(int)

    bits = (sample(p[:, 0], p[:, 1]) < sample(p[:, 2], p[:, 3])).astype(np.uint8)
    return np.packbits(bits.reshape(32, 8)[:, ::-1], axis=1).reshape(32)


def gaussian_blur9(img: np.ndarray) -> np.ndarray:
    k = np.array([7, 17, 32, 46, 52, 46, 32, 17, 7], np.int64)
    h, w = img.shape

    def refl(idx, n):
        idx = np.abs(idx)
        return np.where(idx >= n, 2 * n - 2 - idx, idx)

    xs = refl(np.arange(w)[:, None] + np.arange(-4, 5)[None, :], w)
    rows = (img.astype(np.int64)[:, xs] * k).sum(-1)
    ys = refl(np.arange(h)[:, None] + np.arange(-4, 5)[None, :], h)
    cols = (rows[ys, :] * k[None, :, None]).sum(1)
    return np.minimum((cols + 32768) >> 16, 255).astype(np.uint8)


def hamming(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.unpackbits(np.bitwise_xor(a, b), axis=-1).sum(-1)
