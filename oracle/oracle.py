"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of the CPU restatement in oracle/_build/liborb_oracle.so (built by
oracle/Makefile). Imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liborb_oracle.so"

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
MAXL = 16


class OrcExtractor(C.Structure):
    _fields_ = [
        ("nfeatures", C.c_int), ("scaleFactor", C.c_double), ("nlevels", C.c_int),
        ("iniThFAST", C.c_int), ("minThFAST", C.c_int), ("resize_mode", C.c_int), ("blur_mode", C.c_int),
        ("mvScaleFactor", C.c_float * MAXL), ("mvInvScaleFactor", C.c_float * MAXL),
        ("mvLevelSigma2", C.c_float * MAXL), ("mvInvLevelSigma2", C.c_float * MAXL),
        ("mnFeaturesPerLevel", C.c_int * MAXL), ("umax", C.c_int * 16), ("pattern", C.c_int * 1024),
        ("lw", C.c_int * MAXL), ("lh", C.c_int * MAXL),
        ("level", C.POINTER(C.c_uint8) * MAXL), ("blurred", C.POINTER(C.c_uint8) * MAXL),
    ]


class OrcGrid(C.Structure):
    _fields_ = [("N", C.c_int), ("keysUn", C.c_void_p), ("desc", C.c_void_p),
                ("minX", C.c_float), ("maxX", C.c_float), ("minY", C.c_float), ("maxY", C.c_float),
                ("gridInvW", C.c_float), ("gridInvH", C.c_float),
                ("cell_start", C.c_void_p), ("cell_items", C.c_void_p)]


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        P = C.c_void_p
        L.orc_extractor_init.argtypes = [C.POINTER(OrcExtractor), C.c_int, C.c_float, C.c_int, C.c_int, C.c_int]
        L.orc_extractor_free.argtypes = [C.POINTER(OrcExtractor)]
        L.orc_extract.argtypes = [C.POINTER(OrcExtractor), P, C.c_int, C.c_int, C.c_int, P, P, C.c_int]
        L.orc_resize_linear.argtypes = [P, C.c_int, C.c_int, C.c_int, P, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_fast_roi.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, C.c_int]
        L.orc_gaussian_blur9.argtypes = [P, C.c_int, C.c_int, P]
        L.orc_gaussian_blur9_mode.argtypes = [P, C.c_int, C.c_int, P, C.c_int]
        L.orc_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.orc_fast_atan2.restype = C.c_float
        L.orc_cosf.argtypes = [C.c_float]
        L.orc_cosf.restype = C.c_float
        L.orc_sinf.argtypes = [C.c_float]
        L.orc_sinf.restype = C.c_float
        L.orc_ic_angle.argtypes = [P, C.c_int, C.c_float, C.c_float, P]
        L.orc_ic_angle.restype = C.c_float
        L.orc_orb_descriptor.argtypes = [P, C.c_int, C.c_float, C.c_float, C.c_float, P, P]
        L.orc_descriptor_distance.argtypes = [P, P]
        L.orc_level_candidates.argtypes = [C.POINTER(OrcExtractor), C.c_int, P, C.c_int]
        L.orc_level_candidates_cells.argtypes = [C.POINTER(OrcExtractor), C.c_int, P, C.c_int, P, P]
        L.orc_distribute_octtree.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int]
        L.orc_stereo_matches.argtypes = [C.POINTER(OrcExtractor), C.POINTER(OrcExtractor), P, P, C.c_int,
                                         P, P, C.c_int, C.c_float, C.c_float, P, P]
        L.orc_image_bounds.argtypes = [C.c_int, C.c_int, P, P, P, P, P, P]
        L.orc_grid_build.argtypes = [C.POINTER(OrcGrid), P, P, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float]
        L.orc_grid_free.argtypes = [C.POINTER(OrcGrid)]
        L.orc_features_in_area.argtypes = [C.POINTER(OrcGrid), C.c_float, C.c_float, C.c_float, C.c_int, C.c_int, P, C.c_int]
        L.orc_search_for_initialization.argtypes = [C.POINTER(OrcGrid), C.POINTER(OrcGrid), P, P, C.c_int, C.c_float, C.c_int]
        L.orc_undistort_points.argtypes = [P, P, C.c_int, P, P]
        L.orc_stereo_from_rgbd.argtypes = [P, P, C.c_int, P, C.c_int, C.c_float, P, P]
        L.orc_hamming_best2.argtypes = [P, C.c_int, P, C.c_int, P, P, P]
        L.orc_qt_tie_stats.argtypes = [P, C.c_int]
        L.orc_qt_tie_stats.restype = None
        L.orc_set_blur_mode.argtypes = [C.c_int]
        L.orc_set_blur_mode.restype = None
        L.orc_set_tie_mode.argtypes = [C.c_int]
        L.orc_set_tie_mode.restype = None
        _lib = L
    return _lib


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def qt_tie_stats(reset: bool = False) -> dict:
    """Quadtree tie-pin exposure counters of the calling thread (orc_qt_tie_stats)."""
    a = np.zeros(4, np.int64)
    lib().orc_qt_tie_stats(_p(a), 1 if reset else 0)
    return {"calls": int(a[0]), "final_phase": int(a[1]), "order_exposed": int(a[2]), "set_exposed": int(a[3])}


def set_tie_mode(mode: int):
    """Quadtree final-phase tie key: 0 = creation sequence (pin), 1 = reversed, 2 = hashed."""
    lib().orc_set_tie_mode(int(mode))


def set_blur_mode(mode: int):
    """0 = pinned blur (OpenCV >= 3.4 / scalar rounding), 1 = OpenCV 3.2 SSE2 half-even prefix."""
    lib().orc_set_blur_mode(int(mode))


class Extractor:
    """Python face of the oracle ORBextractor (ORBextractor.h:89-158)."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, resize_mode=0, blur_mode=0):
        self.s = OrcExtractor()
        rc = lib().orc_extractor_init(C.byref(self.s), nfeatures, scale_factor, nlevels, ini_th, min_th)
        if rc != 0:
            raise ValueError("bad extractor params")
        self.s.resize_mode = resize_mode
        self.s.blur_mode = blur_mode   # 1 = OpenCV 3.2's half-even SSE2 column pass
        self.nfeatures = nfeatures
        self.nlevels = nlevels

    def __del__(self):
        try:
            lib().orc_extractor_free(C.byref(self.s))
        except Exception:
            pass

    @property
    def scale_factors(self):
        return np.array(self.s.mvScaleFactor[: self.nlevels], np.float32)

    @property
    def inv_scale_factors(self):
        return np.array(self.s.mvInvScaleFactor[: self.nlevels], np.float32)

    @property
    def features_per_level(self):
        return list(self.s.mnFeaturesPerLevel[: self.nlevels])

    @property
    def umax(self):
        return np.array(self.s.umax[:], np.int32)

    @property
    def pattern(self):
        return np.array(self.s.pattern[:], np.int32)

    def extract(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        cap = self.nfeatures * 2 + 256
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = lib().orc_extract(C.byref(self.s), _p(img), w, h, w, _p(kps), _p(desc), cap)
        if n < 0:
            raise RuntimeError("oracle capacity exceeded")
        return kps[:n].copy(), desc[:n].copy()

    def level(self, l: int) -> np.ndarray:
        w, h = self.s.lw[l], self.s.lh[l]
        buf = C.cast(self.s.level[l], C.POINTER(C.c_uint8 * (w * h))).contents
        return np.frombuffer(buf, np.uint8).reshape(h, w).copy()

    def level_candidates(self, l: int):
        cap = self.s.lw[l] * self.s.lh[l] // 2 + 16
        out = np.zeros(cap, KP_DTYPE)
        n = lib().orc_level_candidates(C.byref(self.s), l, _p(out), cap)
        return out[:n].copy()

    def level_candidates_cells(self, l: int):
        """(candidates, per-visited-cell candidate counts) of level l after extract()."""
        w, h = self.s.lw[l], self.s.lh[l]
        cap = w * h // 2 + 16
        out = np.zeros(cap, KP_DTYPE)
        counts = np.zeros((w // 30 + 2) * (h // 30 + 2), np.int32)
        nc = C.c_int()
        n = lib().orc_level_candidates_cells(C.byref(self.s), l, _p(out), cap, _p(counts), C.byref(nc))
        return out[:n].copy(), counts[: nc.value].copy()


def stereo_matches(exL: Extractor, exR: Extractor, kL, dL, kR, dR, mbf, mb):
    nL = len(kL)
    uR = np.zeros(max(nL, 1), np.float32)
    dep = np.zeros(max(nL, 1), np.float32)
    kL = np.ascontiguousarray(kL)
    kR = np.ascontiguousarray(kR)
    dL = np.ascontiguousarray(dL)
    dR = np.ascontiguousarray(dR)
    lib().orc_stereo_matches(C.byref(exL.s), C.byref(exR.s), _p(kL), _p(dL), nL, _p(kR), _p(dR), len(kR),
                             mbf, mb, _p(uR), _p(dep))
    return uR[:nL], dep[:nL]


def stereo_frames(pool, idx, nfeatures=2000, mbf=386.1448, mb=None, threads=None, **ex_kw):
    """{j: (kL, dL, kR, dR, uR, depth)} for the stereo pairs pool[j], j in idx: ORBextractor on
    L and R + Frame::ComputeStereoMatches, one pair per task on a thread pool (the C calls release
    the GIL). mb defaults to KITTI's mbf / fx in float (Frame.cc:136)."""
    from concurrent.futures import ThreadPoolExecutor
    if mb is None:
        mb = float(np.float32(mbf) / np.float32(718.856))

    def one(j):
        L, R = pool[j]
        exL, exR = Extractor(nfeatures, **ex_kw), Extractor(nfeatures, **ex_kw)
        kL, dL = exL.extract(L)
        kR, dR = exR.extract(R)
        u, d = stereo_matches(exL, exR, kL, dL, kR, dR, mbf, mb)
        return j, (kL, dL, kR, dR, u, d)
    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    with ThreadPoolExecutor(threads) as ex:
        return dict(ex.map(one, sorted(set(idx))))


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orc_descriptor_distance(_p(a), _p(b))


def hamming_best2(q: np.ndarray, db: np.ndarray):
    q = np.ascontiguousarray(q, np.uint8)
    db = np.ascontiguousarray(db, np.uint8)
    n = len(q)
    bi = np.zeros(max(n, 1), np.int32)
    bd = np.zeros(max(n, 1), np.int32)
    sd = np.zeros(max(n, 1), np.int32)
    lib().orc_hamming_best2(_p(q), n, _p(db), len(db), _p(bi), _p(bd), _p(sd))
    return bi[:n], bd[:n], sd[:n]


def undistort_points(xy: np.ndarray, K, dist):
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    out = np.zeros_like(xy)
    Ka = np.asarray(K, np.float32)
    Da = np.asarray(dist, np.float32)
    lib().orc_undistort_points(_p(xy), _p(out), len(xy), _p(Ka), _p(Da))
    return out


def image_bounds(cols, rows, K, dist):
    Ka = np.asarray(K, np.float32)
    Da = np.asarray(dist, np.float32)
    vals = [C.c_float() for _ in range(4)]
    lib().orc_image_bounds(cols, rows, _p(Ka), _p(Da), *[C.byref(v) for v in vals])
    return tuple(v.value for v in vals)


def stereo_from_rgbd(keys, keys_un, depth: np.ndarray, mbf):
    n = len(keys)
    uR = np.zeros(max(n, 1), np.float32)
    dep = np.zeros(max(n, 1), np.float32)
    depth = np.ascontiguousarray(depth, np.float32)
    lib().orc_stereo_from_rgbd(_p(np.ascontiguousarray(keys)), _p(np.ascontiguousarray(keys_un)), n, _p(depth),
                               depth.shape[1], mbf, _p(uR), _p(dep))
    return uR[:n], dep[:n]


class Grid:
    def __init__(self, keys_un, desc, bounds):
        self.keys_un = np.ascontiguousarray(keys_un)
        self.desc = np.ascontiguousarray(desc, np.uint8)
        self.g = OrcGrid()
        lib().orc_grid_build(C.byref(self.g), _p(self.keys_un), _p(self.desc), len(self.keys_un), *bounds)

    def __del__(self):
        try:
            lib().orc_grid_free(C.byref(self.g))
        except Exception:
            pass

    def features_in_area(self, x, y, r, min_level=-1, max_level=-1):
        out = np.zeros(len(self.keys_un) + 1, np.int32)
        n = lib().orc_features_in_area(C.byref(self.g), x, y, r, min_level, max_level, _p(out), len(out))
        return out[:n].copy()


def search_for_initialization(F1: Grid, F2: Grid, prev_xy: np.ndarray, window=100, nnratio=0.9, check_ori=True):
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.zeros(max(len(F1.keys_un), 1), np.int32)
    n = lib().orc_search_for_initialization(C.byref(F1.g), C.byref(F2.g), _p(prev), _p(m12), window, nnratio,
                                            1 if check_ori else 0)
    return n, m12[: len(F1.keys_un)], prev


def distribute_octtree(keys: np.ndarray, minX: int, maxX: int, minY: int, maxY: int, N: int):
    """ExtractorNode quadtree (ORBextractor.cc:696-1042) on cell-offset candidates."""
    keys = np.ascontiguousarray(keys, KP_DTYPE)
    cap = max(N, 0) + 4 * 64 + len(keys) + 16
    out = np.zeros(cap, KP_DTYPE)
    n = lib().orc_distribute_octtree(_p(keys), len(keys), minX, maxX, minY, maxY, N, _p(out), cap)
    if n < 0:
        raise ValueError("nIni == 0")
    return out[:n].copy()


def fast_roi(roi: np.ndarray, th: int):
    roi = np.ascontiguousarray(roi, np.uint8)
    h, w = roi.shape
    cap = h * w + 1
    xs, ys, sc = (np.zeros(cap, np.int32) for _ in range(3))
    n = lib().orc_fast_roi(_p(roi), w, h, w, th, _p(xs), _p(ys), _p(sc), cap)
    return xs[:n].copy(), ys[:n].copy(), sc[:n].copy()


def gaussian_blur9(img: np.ndarray, mode: int | None = None) -> np.ndarray:
    """mode None: the process-wide set_blur_mode(); 0 / 1: that variant."""
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros_like(img)
    if mode is None:
        lib().orc_gaussian_blur9(_p(img), img.shape[1], img.shape[0], _p(out))
    else:
        lib().orc_gaussian_blur9_mode(_p(img), img.shape[1], img.shape[0], _p(out), int(mode))
    return out


def resize_linear(src: np.ndarray, dw: int, dh: int, mode: int = 0) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib().orc_resize_linear(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(out), dw, dh, dw, mode)
    return out


def ic_angle(img: np.ndarray, x: float, y: float, umax) -> float:
    img = np.ascontiguousarray(img, np.uint8)
    um = np.ascontiguousarray(umax, np.int32)
    return lib().orc_ic_angle(_p(img), img.shape[1], x, y, _p(um))


def orb_descriptor(blur: np.ndarray, x: float, y: float, angle: float, pattern) -> np.ndarray:
    blur = np.ascontiguousarray(blur, np.uint8)
    pat = np.ascontiguousarray(pattern, np.int32)
    out = np.zeros(32, np.uint8)
    lib().orc_orb_descriptor(_p(blur), blur.shape[1], x, y, angle, _p(pat), _p(out))
    return out


class LbaProblem(C.Structure):
    _fields_ = [("n_poses", C.c_int32), ("pose_id", C.c_void_p), ("pose_fixed", C.c_void_p),
                ("pose_Tcw", C.c_void_p), ("pose_cam", C.c_void_p), ("n_points", C.c_int32),
                ("point_id", C.c_void_p), ("point_Xw", C.c_void_p), ("n_edges", C.c_int32),
                ("edge_point", C.c_void_p), ("edge_pose", C.c_void_p), ("edge_obs", C.c_void_p),
                ("edge_inv_sigma2", C.c_void_p)]


class LbaResult(C.Structure):
    _fields_ = [("pose_Tcw", C.c_void_p), ("point_Xw", C.c_void_p), ("edge_erase", C.c_void_p),
                ("iterations", C.c_int32 * 2), ("chi2", C.c_double * 2), ("stopped", C.c_int32),
                ("trials", C.c_int32 * 2)]


def make_lba_structs(prob: dict):
    """Build (LbaProblem, keepalive arrays) from a synth.localba_problem dict."""
    keep = {}
    for k in ("pose_id", "pose_fixed", "pose_Tcw", "pose_cam", "point_id", "point_Xw", "edge_point",
              "edge_pose", "edge_obs", "edge_inv_sigma2"):
        keep[k] = np.ascontiguousarray(prob[k])
    P = LbaProblem(len(keep["pose_id"]), keep["pose_id"].ctypes.data, keep["pose_fixed"].ctypes.data,
                   keep["pose_Tcw"].ctypes.data, keep["pose_cam"].ctypes.data, len(keep["point_id"]),
                   keep["point_id"].ctypes.data, keep["point_Xw"].ctypes.data, len(keep["edge_point"]),
                   keep["edge_point"].ctypes.data, keep["edge_pose"].ctypes.data, keep["edge_obs"].ctypes.data,
                   keep["edge_inv_sigma2"].ctypes.data)
    return P, keep


def make_lba_result(prob: dict):
    out = {"pose_Tcw": np.zeros((len(prob["pose_id"]), 16), np.float32),
           "point_Xw": np.zeros((len(prob["point_id"]), 3), np.float32),
           "edge_erase": np.zeros(len(prob["edge_point"]), np.uint8)}
    R = LbaResult(out["pose_Tcw"].ctypes.data, out["point_Xw"].ctypes.data, out["edge_erase"].ctypes.data)
    return R, out


def lba_chol_stats(reset: bool = False) -> dict:
    """Dense-Cholesky pin exposure counters of the calling thread (lba_oracle_chol_stats)."""
    L = lib()
    L.lba_oracle_chol_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.lba_oracle_chol_stats.restype = None
    a = np.zeros(2, np.int64)
    r = C.c_double()
    L.lba_oracle_chol_stats(_p(a), C.byref(r), 1 if reset else 0)
    return {"schur_solves": int(a[0]), "nonpositive_pivot": int(a[1]), "min_pivot_ratio": r.value}


def lba_solve(prob: dict, stop: bool = False, hook=None):
    """Optimizer::LocalBundleAdjustment optimisation core on the CPU (double precision).
    hook = (phase, trial): pbStopFlag raised after LM trial `trial` of optimize() call `phase`
    (lba_oracle_solve_hook; the GPU's lba_set_stop_hook)."""
    L = lib()
    L.lba_oracle_solve_hook.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    P, keep = make_lba_structs(prob)
    R, out = make_lba_result(prob)
    flag = C.c_uint8(1 if stop else 0)
    hp, ht = hook if hook else (0, 0)
    L.lba_oracle_solve_hook(C.byref(P), C.byref(R), C.byref(flag), int(hp), int(ht))
    out["iterations"] = tuple(R.iterations)
    out["chi2"] = tuple(R.chi2)
    out["stopped"] = R.stopped
    out["trials"] = tuple(R.trials)
    return out


# ---- tracking matchers (track_oracle.c): Frame::isInFrustum + both per-frame
# ORBmatcher::SearchByProjection overloads. Problems are the dicts of synth.tracking_problem.
class OrbtFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("u_right", C.c_void_p), ("desc", C.c_void_p),
                ("Tcw", C.c_float * 12), ("Ow", C.c_float * 3), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("mbf", C.c_float), ("mb", C.c_float),
                ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float),
                ("nlevels", C.c_int32), ("log_scale_factor", C.c_float), ("scale_factors", C.c_float * 16),
                ("inv_level_sigma2", C.c_float * 16)]


class OrbtMapPoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("Xw", C.c_void_p), ("normal", C.c_void_p), ("min_dist", C.c_void_p),
                ("max_dist", C.c_void_p), ("desc", C.c_void_p), ("flags", C.c_void_p)]


class OrbtView(C.Structure):
    _fields_ = [("in_view", C.c_void_p), ("proj_x", C.c_void_p), ("proj_y", C.c_void_p),
                ("proj_xr", C.c_void_p), ("view_cos", C.c_void_p), ("level", C.c_void_p)]


def make_orbt_frame(fr: dict):
    keep = {"keys_un": np.ascontiguousarray(fr["keys_un"], KP_DTYPE),
            "u_right": np.ascontiguousarray(fr["u_right"], np.float32),
            "desc": np.ascontiguousarray(fr["desc"], np.uint8)}
    F = OrbtFrame()
    F.n = len(keep["keys_un"])
    F.keys_un, F.u_right, F.desc = (keep[k].ctypes.data for k in ("keys_un", "u_right", "desc"))
    F.Tcw[:] = [float(v) for v in np.asarray(fr["Tcw"], np.float32).reshape(-1)[:12]]
    F.Ow[:] = [float(v) for v in np.asarray(fr["Ow"], np.float32)]
    for k in ("fx", "fy", "cx", "cy", "mbf", "mb", "min_x", "max_x", "min_y", "max_y", "log_scale_factor"):
        setattr(F, k, float(fr[k]))
    F.nlevels = int(fr["nlevels"])
    sf = np.zeros(16, np.float32)
    sf[: F.nlevels] = fr["scale_factors"]
    F.scale_factors[:] = [float(v) for v in sf]
    isg = np.zeros(16, np.float32)
    isg[: F.nlevels] = fr["inv_level_sigma2"] if "inv_level_sigma2" in fr else \
        (np.float32(1) / (np.asarray(fr["scale_factors"], np.float32) ** 2)).astype(np.float32)
    F.inv_level_sigma2[:] = [float(v) for v in isg]
    return F, keep


def make_orbt_map(mp: dict):
    keep = {"Xw": np.ascontiguousarray(mp["Xw"], np.float32), "normal": np.ascontiguousarray(mp["normal"], np.float32),
            "min_dist": np.ascontiguousarray(mp["min_dist"], np.float32),
            "max_dist": np.ascontiguousarray(mp["max_dist"], np.float32),
            "desc": np.ascontiguousarray(mp["desc"], np.uint8), "flags": np.ascontiguousarray(mp["flags"], np.uint8)}
    M = OrbtMapPoints(len(keep["Xw"]), *(keep[k].ctypes.data for k in ("Xw", "normal", "min_dist", "max_dist", "desc",
                                                                        "flags")))
    return M, keep


def logf(x: float) -> float:
    L = lib()
    L.orc_logf.argtypes = [C.c_float]
    L.orc_logf.restype = C.c_float
    return L.orc_logf(x)


def search_local_points(prob: dict, cos_limit=0.5, th=1.0, nnratio=0.8):
    """Tracking::SearchLocalPoints core: isInFrustum + SearchByProjection(F, vpMapPoints, th)."""
    L = lib()
    L.orc_search_local_points.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_float, C.c_float, C.c_void_p,
                                          C.c_void_p, C.c_void_p]
    F, k1 = make_orbt_frame(prob["frame"])
    M, k2 = make_orbt_map(prob["map"])
    n, m = F.n, M.n
    view = {"in_view": np.zeros(max(m, 1), np.uint8), "proj_x": np.zeros(max(m, 1), np.float32),
            "proj_y": np.zeros(max(m, 1), np.float32), "proj_xr": np.zeros(max(m, 1), np.float32),
            "view_cos": np.zeros(max(m, 1), np.float32), "level": np.zeros(max(m, 1), np.int32)}
    V = OrbtView(*(view[k].ctypes.data for k in ("in_view", "proj_x", "proj_y", "proj_xr", "view_cos", "level")))
    owner = np.zeros(max(n, 1), np.int32)
    blk = prob.get("kp_blocked")
    blk = np.ascontiguousarray(blk, np.uint8) if blk is not None else None
    nm = L.orc_search_local_points(C.byref(F), C.byref(M), cos_limit, th, nnratio,
                                   blk.ctypes.data if blk is not None else None, C.byref(V), owner.ctypes.data)
    return nm, owner[:n], {k: v[:m] for k, v in view.items()}


def search_by_projection_frame(prob: dict, th=15.0, mono=False, check_ori=True):
    """ORBmatcher(0.9, checkOri).SearchByProjection(CurrentFrame, LastFrame, th, bMono)."""
    L = lib()
    L.orc_search_by_projection_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                 C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    F, k1 = make_orbt_frame(prob["frame"])
    Lf, k2 = make_orbt_frame(prob["last"])
    M, k3 = make_orbt_map(prob["map"])
    last_mp = np.ascontiguousarray(prob["last_mp"], np.int32)
    last_out = np.ascontiguousarray(prob["last_outlier"], np.uint8)
    owner = np.zeros(max(F.n, 1), np.int32)
    blk = prob.get("kp_blocked")
    blk = np.ascontiguousarray(blk, np.uint8) if blk is not None else None
    nm = L.orc_search_by_projection_frame(C.byref(F), C.byref(Lf), last_mp.ctypes.data, last_out.ctypes.data,
                                          C.byref(M), th, 1 if mono else 0, 1 if check_ori else 0,
                                          blk.ctypes.data if blk is not None else None, owner.ctypes.data)
    return nm, owner[: F.n]


def search_by_projection_keyframe(prob: dict, th=10.0, orb_dist=100, check_ori=True):
    """ORBmatcher(0.9, checkOri).SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)."""
    L = lib()
    L.orc_search_by_projection_kf.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_int,
                                              C.c_int, C.c_void_p, C.c_void_p]
    F, k1 = make_orbt_frame(prob["frame"])
    Kf, k2 = make_orbt_frame(prob["last"])
    M, k3 = make_orbt_map(prob["map"])
    kf_mp = np.ascontiguousarray(prob["last_mp"], np.int32)
    owner = np.zeros(max(F.n, 1), np.int32)
    blk = prob.get("kp_blocked")
    blk = np.ascontiguousarray(blk, np.uint8) if blk is not None else None
    nm = L.orc_search_by_projection_kf(C.byref(F), C.byref(Kf), kf_mp.ctypes.data, C.byref(M), th, int(orb_dist),
                                       1 if check_ori else 0, blk.ctypes.data if blk is not None else None,
                                       owner.ctypes.data)
    return nm, owner[: F.n]


def search_by_projection_sim3(prob: dict, th=10):
    """LoopClosing's SearchByProjection(pKF = prob["frame"], Scw, vpPoints = prob["map"], vpMatched, th):
    (nmatches, vpMatched out as point indices, -1 = NULL, -2 = a point outside vpPoints)."""
    L = lib()
    L.orc_search_by_projection_sim3.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    F, k1 = make_orbt_frame(prob["frame"])
    M, k2 = make_orbt_map(prob["map"])
    Scw = np.ascontiguousarray(prob["Scw"], np.float32).reshape(16)
    matched = np.array(prob["matched"], np.int32, copy=True)
    nm = L.orc_search_by_projection_sim3(C.byref(F), Scw.ctypes.data, C.byref(M), int(th), matched.ctypes.data)
    return nm, matched[: F.n]


def fuse_sim3_candidates(prob: dict, th=4.0):
    """LoopClosing's Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) search half: (best_idx, best_dist)."""
    L = lib()
    L.orc_fuse_sim3_candidates.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]
    F, k1 = make_orbt_frame(prob["frame"])
    M, k2 = make_orbt_map(prob["map"])
    Scw = np.ascontiguousarray(prob["Scw"], np.float32).reshape(16)
    bi = np.zeros(max(M.n, 1), np.int32)
    bd = np.zeros(max(M.n, 1), np.int32)
    L.orc_fuse_sim3_candidates(C.byref(F), Scw.ctypes.data, C.byref(M), th, bi.ctypes.data, bd.ctypes.data)
    return bi[: M.n], bd[: M.n]


def search_by_sim3(prob: dict, th=7.5):
    """ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th): (nFound, matches12 out)."""
    L = lib()
    L.orc_search_by_sim3.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p,
                                     C.c_void_p, C.c_float, C.c_void_p]
    F1, k1 = make_orbt_frame(prob["kf1"])
    F2, k2 = make_orbt_frame(prob["kf2"])
    M, k3 = make_orbt_map(prob["map"])
    mp1 = np.ascontiguousarray(prob["kf1_mp"], np.int32)
    mp2 = np.ascontiguousarray(prob["kf2_mp"], np.int32)
    R12 = np.ascontiguousarray(prob["R12"], np.float32).reshape(9)
    t12 = np.ascontiguousarray(prob["t12"], np.float32).reshape(3)
    m12 = np.array(prob["matches12"], np.int32, copy=True)
    nf = L.orc_search_by_sim3(C.byref(F1), mp1.ctypes.data, C.byref(F2), mp2.ctypes.data, C.byref(M), float(prob["s12"]),
                              R12.ctypes.data, t12.ctypes.data, th, m12.ctypes.data)
    return nf, m12[: F1.n]


# ---- Optimizer::PoseOptimization (lba_oracle.c pose_oracle_optimize)
class OrbpFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("Xw", C.c_void_p), ("obs", C.c_void_p), ("inv_sigma2", C.c_void_p),
                ("Tcw", C.c_float * 16), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float)]


class OrbpResult(C.Structure):
    _fields_ = [("Tcw", C.c_float * 16), ("outlier", C.c_void_p), ("n_inliers", C.c_int32),
                ("iterations", C.c_int32 * 4)]


def make_orbp_frame(prob: dict):
    keep = {k: np.ascontiguousarray(prob[k], np.float32) for k in ("Xw", "obs", "inv_sigma2")}
    F = OrbpFrame()
    F.n = len(keep["Xw"])
    F.Xw, F.obs, F.inv_sigma2 = (keep[k].ctypes.data for k in ("Xw", "obs", "inv_sigma2"))
    F.Tcw[:] = [float(v) for v in np.asarray(prob["Tcw"], np.float32).reshape(-1)]
    F.fx, F.fy, F.cx, F.cy, F.bf = (float(v) for v in prob["cam"])
    return F, keep


def pose_optimization(prob: dict):
    L = lib()
    L.pose_oracle_optimize.argtypes = [C.c_void_p, C.c_void_p]
    F, keep = make_orbp_frame(prob)
    out = np.zeros(max(F.n, 1), np.uint8)
    R = OrbpResult()
    R.outlier = out.ctypes.data
    L.pose_oracle_optimize(C.byref(F), C.byref(R))
    return {"Tcw": np.array(R.Tcw[:], np.float32).reshape(4, 4), "outlier": out[: F.n].copy(),
            "n_inliers": R.n_inliers, "iterations": tuple(R.iterations)}


# ---- DBoW2 vocabulary transform (bow_oracle.c)
class OrcVocab(C.Structure):
    _fields_ = [("k", C.c_int), ("L", C.c_int), ("scoring", C.c_int), ("weighting", C.c_int), ("n_nodes", C.c_int),
                ("n_words", C.c_int), ("child_start", C.c_void_p), ("children", C.c_void_p), ("desc", C.c_void_p),
                ("weight", C.c_void_p), ("word_id", C.c_void_p)]


class Vocabulary:
    """Oracle TemplatedVocabulary (from synth.vocabulary arrays or a text file)."""

    def __init__(self, voc: dict | None = None, path: str | None = None):
        L = lib()
        L.orc_vocab_build.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
        L.orc_vocab_load_text.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_vocab_free.argtypes = [C.c_void_p]
        L.orc_bow_transform.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        self.v = OrcVocab()
        if path is not None:
            rc = L.orc_vocab_load_text(C.byref(self.v), str(path).encode())
        else:
            par = np.ascontiguousarray(voc["parent"], np.int32)
            leaf = np.ascontiguousarray(voc["is_leaf"], np.uint8)
            desc = np.ascontiguousarray(voc["desc"], np.uint8)
            w = np.ascontiguousarray(voc["weight"], np.float64)
            rc = L.orc_vocab_build(C.byref(self.v), voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(par),
                                   par.ctypes.data, leaf.ctypes.data, desc.ctypes.data, w.ctypes.data)
        if rc != 0:
            raise ValueError("bad vocabulary")

    def __del__(self):
        try:
            lib().orc_vocab_free(C.byref(self.v))
        except Exception:
            pass

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        desc = np.ascontiguousarray(desc, np.uint8)
        n = len(desc)
        m = max(n, 1)
        words = np.zeros(m, np.uint32)
        vals = np.zeros(m, np.float64)
        fvn = np.zeros(m, np.uint32)
        fvs = np.zeros(m + 1, np.int32)
        fvf = np.zeros(m, np.int32)
        nw, nf = C.c_int(), C.c_int()
        lib().orc_bow_transform(C.byref(self.v), desc.ctypes.data, n, levelsup, words.ctypes.data, vals.ctypes.data,
                                C.byref(nw), fvn.ctypes.data, fvs.ctypes.data, fvf.ctypes.data, C.byref(nf))
        return {"words": words[: nw.value].copy(), "values": vals[: nw.value].copy(),
                "fv_nodes": fvn[: nf.value].copy(), "fv_start": fvs[: nf.value + 1].copy(),
                "fv_features": fvf[: fvs[nf.value]].copy()}


# ---- BoW-guided matchers (track_oracle.c)
class OrbbKeyFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("u_right", C.c_void_p), ("desc", C.c_void_p),
                ("mp", C.c_void_p), ("mp_bad", C.c_void_p), ("n_fv", C.c_int32), ("fv_nodes", C.c_void_p),
                ("fv_start", C.c_void_p), ("fv_features", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("nlevels", C.c_int32), ("scale_factors", C.c_float * 16),
                ("level_sigma2", C.c_float * 16)]


def make_orbb_keyframe(k: dict):
    keep = {"keys_un": np.ascontiguousarray(k["keys_un"], KP_DTYPE), "u_right": np.ascontiguousarray(k["u_right"], np.float32),
            "desc": np.ascontiguousarray(k["desc"], np.uint8), "mp": np.ascontiguousarray(k["mp"], np.int32),
            "mp_bad": np.ascontiguousarray(k["mp_bad"], np.uint8), "fv_nodes": np.ascontiguousarray(k["fv_nodes"], np.uint32),
            "fv_start": np.ascontiguousarray(k["fv_start"], np.int32),
            "fv_features": np.ascontiguousarray(k["fv_features"], np.int32)}
    K = OrbbKeyFrame()
    K.n = len(keep["keys_un"])
    for f in ("keys_un", "u_right", "desc", "mp", "mp_bad", "fv_nodes", "fv_start", "fv_features"):
        setattr(K, f, keep[f].ctypes.data)
    K.n_fv = len(keep["fv_nodes"])
    K.fx, K.fy, K.cx, K.cy = (float(k[f]) for f in ("fx", "fy", "cx", "cy"))
    K.nlevels = int(k["nlevels"])
    for f in ("scale_factors", "level_sigma2"):
        a = np.zeros(16, np.float32)
        a[: K.nlevels] = k[f]
        getattr(K, f)[:] = [float(x) for x in a]
    return K, keep


def search_by_bow(prob: dict, nnratio=0.7, check_ori=True):
    L = lib()
    L.orc_search_by_bow.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_int, C.c_void_p]
    A, k1 = make_orbb_keyframe(prob["A"])
    B, k2 = make_orbb_keyframe(prob["B"])
    out = np.zeros(max(B.n, 1), np.int32)
    nm = L.orc_search_by_bow(C.byref(A), C.byref(B), nnratio, 1 if check_ori else 0, out.ctypes.data)
    return nm, out[: B.n]


def search_by_bow_kf(prob: dict, nnratio=0.75, check_ori=True):
    """SearchByBoW(KeyFrame* pKF1 = A, KeyFrame* pKF2 = B): (nmatches, matches12[A.n])."""
    L = lib()
    L.orc_search_by_bow_kf.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_int, C.c_void_p]
    A, k1 = make_orbb_keyframe(prob["A"])
    B, k2 = make_orbb_keyframe(prob["B"])
    out = np.zeros(max(A.n, 1), np.int32)
    nm = L.orc_search_by_bow_kf(C.byref(A), C.byref(B), nnratio, 1 if check_ori else 0, out.ctypes.data)
    return nm, out[: A.n]


def search_for_triangulation(prob: dict, only_stereo=False, check_ori=True):
    L = lib()
    L.orc_search_for_triangulation.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                               C.c_int, C.c_void_p]
    A, k1 = make_orbb_keyframe(prob["A"])
    B, k2 = make_orbb_keyframe(prob["B"])
    F12 = np.ascontiguousarray(prob["F12"], np.float32)
    Cw = np.ascontiguousarray(prob["Cw1"], np.float32)
    T2w = np.ascontiguousarray(prob["T2w"], np.float32)
    pairs = np.zeros((max(A.n, 1), 2), np.int32)
    npairs = L.orc_search_for_triangulation(C.byref(A), C.byref(B), F12.ctypes.data, Cw.ctypes.data, T2w.ctypes.data,
                                            1 if only_stereo else 0, 1 if check_ori else 0, pairs.ctypes.data)
    return pairs[:npairs].copy()


def fuse_candidates(prob: dict, th=3.0):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th) search half: (best_idx, best_dist) per map point."""
    L = lib()
    L.orc_fuse_candidates.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]
    F, k1 = make_orbt_frame(prob["frame"])
    M, k2 = make_orbt_map(prob["map"])
    bi = np.zeros(max(M.n, 1), np.int32)
    bd = np.zeros(max(M.n, 1), np.int32)
    L.orc_fuse_candidates(C.byref(F), C.byref(M), th, bi.ctypes.data, bd.ctypes.data)
    return bi[: M.n], bd[: M.n]


# ---- new map points (newpts_oracle.c)
class OrbnKeyFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys", C.c_void_p), ("keys_un", C.c_void_p), ("u_right", C.c_void_p),
                ("depth", C.c_void_p), ("Tcw", C.c_float * 12), ("Ow", C.c_float * 3), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("invfx", C.c_float), ("invfy", C.c_float),
                ("mb", C.c_float), ("mbf", C.c_float), ("nlevels", C.c_int32), ("scale_factors", C.c_float * 16),
                ("level_sigma2", C.c_float * 16)]


def make_orbn_keyframe(k: dict):
    keep = {"keys": np.ascontiguousarray(k["keys"], KP_DTYPE), "keys_un": np.ascontiguousarray(k["keys_un"], KP_DTYPE),
            "u_right": np.ascontiguousarray(k["u_right"], np.float32), "depth": np.ascontiguousarray(k["depth"], np.float32)}
    K = OrbnKeyFrame()
    K.n = len(keep["keys_un"])
    for f in ("keys", "keys_un", "u_right", "depth"):
        setattr(K, f, keep[f].ctypes.data)
    K.Tcw[:] = [float(x) for x in np.asarray(k["Tcw"], np.float32).reshape(-1)]
    K.Ow[:] = [float(x) for x in np.asarray(k["Ow"], np.float32).reshape(-1)]
    for f in ("fx", "fy", "cx", "cy", "invfx", "invfy", "mb", "mbf"):
        setattr(K, f, float(k[f]))
    K.nlevels = int(k["nlevels"])
    for f in ("scale_factors", "level_sigma2"):
        a = np.zeros(16, np.float32)
        a[: K.nlevels] = k[f]
        getattr(K, f)[:] = [float(x) for x in a]
    return K, keep


def triangulate(prob: dict):
    """LocalMapping::CreateNewMapPoints' per-match body: (nnew, x3d[n][3], ok[n])."""
    L = lib()
    L.orc_triangulate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_float, C.c_void_p, C.c_void_p]
    A, k1 = make_orbn_keyframe(prob["kf1"])
    B, k2 = make_orbn_keyframe(prob["kf2"])
    pairs = np.ascontiguousarray(prob["pairs"], np.int32)
    n = len(pairs)
    x3d = np.zeros((max(n, 1), 3), np.float32)
    ok = np.zeros(max(n, 1), np.uint8)
    nnew = L.orc_triangulate(C.byref(A), C.byref(B), pairs.ctypes.data, n, float(prob["ratio_factor"]),
                             x3d.ctypes.data, ok.ctypes.data)
    return nnew, x3d[:n], ok[:n]


def svd4_vt(A: np.ndarray):
    """cv::SVD::compute(A 4x4 CV_32F, MODIFY_A | FULL_UV) -> (vt, w) as restated."""
    L = lib()
    L.orc_svd4_vt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    a = np.ascontiguousarray(A, np.float32).reshape(16)
    vt = np.zeros(16, np.float32)
    w = np.zeros(4, np.float32)
    L.orc_svd4_vt(a.ctypes.data, vt.ctypes.data, w.ctypes.data)
    return vt.reshape(4, 4), w
