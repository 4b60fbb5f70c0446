"""orbslam2_amd — Python face of the MI355X-native ORB-SLAM2 hot path.

Thin ctypes binding of the C-ABI in include/orbslam2_amd.h (liborbslam2_amd.so, built
in-tree by orb-slam2-noted_amd/Makefile). The classes mirror the reference classes the
C-ABI replaces so tests read like the reference's call sites:

* ``ORBextractor``   — ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST),
                        ``__call__(image) -> (keypoints, descriptors)`` (ORBextractor.h:89-158)
* ``ORBmatcher``     — ``DescriptorDistance`` and the brute-force best/second-best scan
                        (ORBmatcher.h:57-65)
* ``compute_stereo_matches`` — Frame::ComputeStereoMatches (Frame.h:249)
* ``BatchExtractor`` — the batched, device-resident path used by bench.py

There is no CPU fallback: if the shared library or a GPU is missing, constructing any of
these raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parents[2]          # orb-slam2-noted_amd/
# ORBSLAM_AMD_LIB: an instrumented build of the same sources (tools/*: profiling variants)
LIB_PATH = Path(os.environ["ORBSLAM_AMD_LIB"]) if os.environ.get("ORBSLAM_AMD_LIB") else PKG_ROOT / "liborbslam2_amd.so"

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

ORBX_OK, ORBX_EINVAL, ORBX_EDEVICE, ORBX_ECAP, ORBX_ESTATE = 0, -1, -2, -3, -4


class OrbxParams(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("resize_mode", C.c_int32),
                ("blur_mode", C.c_int32)]


class OrbslamError(RuntimeError):
    pass


_lib = None

# (name, restype, argtypes) of every exported C-ABI symbol declared in include/orbslam2_amd.h
_P = C.c_void_p
_I = C.c_int
_F = C.c_float
SIGNATURES = [
    ("orbx_create", _I, [C.POINTER(OrbxParams), C.POINTER(C.c_void_p)]),
    ("orbx_destroy", None, [_P]),
    ("orbx_levels", _I, [_P, _P, _P, _P, _P, _P, _P]),
    ("orbx_extract", _I, [_P, _P, _I, _I, _I, _P, _P, _I, _P]),
    ("orbx_pyramid_level", _I, [_P, _I, _I, _P, _P, _P]),
    ("orbx_blurred_level", _I, [_P, _I, _I, _P, _P, _P]),
    ("orbx_reserve", _I, [_P, _I, _I, _I]),
    ("orbx_extract_batch_device", _I, [_P, _P, _I, _I, _I, _I, C.c_size_t, _P]),
    ("orbx_extract_batch_device_phase", _I, [_P, _P, _I, _I, _I, _I, C.c_size_t, _P, _I]),
    ("orbx_pipeline_create", _I, [_P, _I, _P]),
    ("orbx_pipeline_destroy", None, [_P]),
    ("orbx_pipeline_engines", _I, [_P]),
    ("orbx_pipeline_reserve", _I, [_P, _I, _I, _I]),
    ("orbx_pipeline_stereo_batch", _I, [_P, _P, _I, _I, _I, _I, C.c_size_t, _F, _F, _P]),
    ("orbx_pipeline_chunk", _I, [_P, _I, _P, _P, _P]),
    ("orbx_pipeline_capacity", _I, [_P, _P]),
    ("orbx_capacity", _I, [_P, _P]),
    ("orbx_pipeline_stereo_batch_host", _I, [_P, _P, _I, _I, _I, _I, C.c_size_t, _F, _F, _P]),
    ("orbx_pipeline_wait", _I, [_P]),
    ("orbx_host_alloc", _I, [C.c_size_t, _P]),
    ("orbx_host_free", _I, [_P]),
    ("orbx_pipeline_join", _I, [_P, _P]),
    ("orbx_batch_results", _I, [_P, _P, _P, _P, _P]),
    ("orbx_batch_fetch", _I, [_P, _I, _P, _P, _I, _P]),
    ("orbx_stream", _P, [_P]),
    ("orbm_stereo_match", _I, [_P, _P, _F, _F, _P, _P, _I]),
    ("orbm_stereo_match_batch_device", _I, [_P, _I, _F, _F, _P]),
    ("orbm_stereo_results", _I, [_P, _P, _P]),
    ("orbm_stereo_fetch", _I, [_P, _I, _P, _P, _I]),
    ("orbm_hamming_best2", _I, [_P, _I, _P, _I, _P, _P, _P]),
    ("orbm_create", _I, [_F, _I, _P]),
    ("orbm_destroy", None, [_P]),
    ("orbm_hamming_best2_cand", _I, [_P, _P, _I, _P, _I, _P, _P, _P, _P, _P]),
    ("orbm_hamming_best2_cand_device", _I, [_P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P]),
    ("orbm_search_for_initialization", _I, [_P, _P, _P, _P, _P, _I, _P]),
    ("orbslam2_amd_version", C.c_char_p, []),
    ("orbx_build_id", C.c_char_p, []),
    ("orbslam2_amd_device_count", _I, []),
    ("orbslam2_amd_device_sync", _I, []),
    ("orbslam2_amd_set_device", _I, [_I]),
    ("orbx_profile", _I, [_P, _I]),
    ("lba_profile", _I, [_P, _I]),
    ("lba_profile_read", _I, [_P, _I, C.c_char_p, _I, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    ("orbf_rgbd", _I, [_P, _P, _I, _P, _P, _F, _P, _P, _P, _I]),
    ("orbf_rgbd_batch_device", _I, [_P, _P, C.c_size_t, _I, _P, _P, _F, _P]),
    ("orbf_rgbd_fetch", _I, [_P, _I, _P, _P, _P, _I]),
    ("orbm_search_init_batch_device", _I, [_P, _I, _I, _I, _I, _I, _P, _P, _I, _F, _I, _P]),
    ("orbm_search_init_fetch", _I, [_P, _I, _P, _P, _I, _P]),
    ("lba_create", _I, [C.POINTER(C.c_void_p)]),
    ("lba_destroy", None, [_P]),
    ("lba_solve", _I, [_P, _P, _P, _P]),
    ("lba_set_stop_hook", _I, [_P, _I, _I]),
    ("lba_set_test_option", _I, [_P, _I, C.c_longlong]),
    ("orbx_profile_read", _I, [_P, _I, C.c_char_p, _I, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    ("orbt_create", _I, [C.POINTER(C.c_void_p)]),
    ("orbt_destroy", None, [_P]),
    ("orbt_search_local_points", _I, [_P, _P, _P, _F, _F, _F, _P, _P, _P, _P]),
    ("orbt_search_by_projection_frame", _I, [_P, _P, _P, _P, _P, _P, _F, _I, _I, _P, _P, _P]),
    ("orbt_reserve", _I, [_P, _I, _I, _I]),
    ("orbt_stage", _I, [_P, _I, _P, _P, _P, _P, _P, _P]),
    ("orbt_run_local_batch", _I, [_P, _I, _F, _F, _F, _P]),
    ("orbt_run_frame_batch", _I, [_P, _I, _F, _I, _I, _P]),
    ("orbt_run_reloc_batch", _I, [_P, _I, _F, _I, _I, _P]),
    ("orbt_search_by_projection_keyframe", _I, [_P, _P, _P, _P, _P, _F, _I, _I, _P, _P, _P]),
    ("orbt_fetch", _I, [_P, _I, _P, _P, _P]),
    ("orbt_fuse_candidates", _I, [_P, _P, _P, _F, _P, _P]),
    ("orbt_run_fuse_batch", _I, [_P, _I, _F, _P]),
    ("orbt_fetch_fuse", _I, [_P, _I, _P, _P]),
    ("orbt_search_by_projection_sim3", _I, [_P, _P, _P, _P, _I, _P, _P]),
    ("orbt_stage_sim3", _I, [_P, _I, _P, _P, _P, _P]),
    ("orbt_run_sim3_batch", _I, [_P, _I, _I, _P]),
    ("orbt_fuse_sim3_candidates", _I, [_P, _P, _P, _P, _F, _P, _P]),
    ("orbt_stage_fuse_sim3", _I, [_P, _I, _P, _P, _P]),
    ("orbt_run_fuse_sim3_batch", _I, [_P, _I, _F, _P]),
    ("orbt_search_by_sim3", _I, [_P, _P, _P, _P, _P, _P, _F, _P, _P, _F, _P, _P]),
    ("orbt_stage_search_by_sim3", _I, [_P, _I, _P, _P, _P, _P, _P, _F, _P, _P, _P]),
    ("orbt_run_sim3_match_batch", _I, [_P, _I, _F, _P]),
    ("orbt_fetch_search_by_sim3", _I, [_P, _I, _P, _P, _P]),
    ("orbp_create", _I, [C.POINTER(C.c_void_p)]),
    ("orbp_destroy", None, [_P]),
    ("orbp_pose_optimization", _I, [_P, _P, _P]),
    ("orbp_reserve", _I, [_P, _I, _I]),
    ("orbp_stage", _I, [_P, _I, _P]),
    ("orbp_run_batch", _I, [_P, _I, _P]),
    ("orbp_fetch", _I, [_P, _I, _P]),
    ("orbv_create", _I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, C.POINTER(C.c_void_p)]),
    ("orbv_load_text", _I, [C.c_char_p, C.POINTER(C.c_void_p)]),
    ("orbv_destroy", None, [_P]),
    ("orbv_info", _I, [_P, _P, _P, _P, _P]),
    ("orbv_transform", _I, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    ("orbv_transform_batch_device", _I, [_P, _P, _P, _I, _I, C.c_size_t, _I, _P]),
    ("orbv_batch_fetch", _I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    ("orbb_create", _I, [C.POINTER(C.c_void_p)]),
    ("orbb_destroy", None, [_P]),
    ("orbb_search_by_bow", _I, [_P, _P, _P, _F, _I, _P, _P]),
    ("orbb_search_for_triangulation", _I, [_P, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
    ("orbb_reserve", _I, [_P, _I, _I]),
    ("orbb_stage", _I, [_P, _I, _P, _P, _P, _P, _P]),
    ("orbb_run_bow_batch", _I, [_P, _I, _F, _I, _P]),
    ("orbb_run_tri_batch", _I, [_P, _I, _I, _I, _P]),
    ("orbb_fetch", _I, [_P, _I, _I, _P, _P]),
    ("orbb_search_by_bow_kf", _I, [_P, _P, _P, _F, _I, _P, _P]),
    ("orbb_run_bowkf_batch", _I, [_P, _I, _F, _I, _P]),
    ("orbn_create", _I, [C.POINTER(C.c_void_p)]),
    ("orbn_destroy", None, [_P]),
    ("orbn_triangulate", _I, [_P, _P, _P, _P, _I, _F, _P, _P, _P]),
    ("orbn_reserve", _I, [_P, _I, _I, _I]),
    ("orbn_stage", _I, [_P, _I, _P, _P, _P, _I, _F]),
    ("orbn_run_batch", _I, [_P, _I, _P]),
    ("orbn_fetch", _I, [_P, _I, _P, _P, _P]),
]


def _init_torch_runtime_first():
    """torch-ROCm ships its own HIP runtime (torch/lib/libamdhip64.so) while this library
    links /opt/rocm's. Both coexist in one process -- and device pointers are shared -- only
    if torch's runtime initialises the device first (probed on MI355X by
    tools/probe_runtime.py), so touch torch.cuda before loading our library when torch is
    importable. Without torch nothing is needed."""
    if os.environ.get("ORBSLAM2_AMD_NO_TORCH"):
        return
    try:
        import torch
    except Exception:
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def lib() -> C.CDLL:
    """Load the in-tree HIP library (fails loudly: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        _init_torch_runtime_first()
        if not LIB_PATH.exists():
            raise OrbslamError(f"{LIB_PATH} missing: build it with `make -C {PKG_ROOT}` "
                               "(or __graft_entry__.build())")
        L = C.CDLL(str(LIB_PATH))
        ab = bool(os.environ.get("ORBSLAM_AMD_LIB"))   # an A/B or variant build may predate some entries
        for name, res, args in SIGNATURES:
            if ab and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != ORBX_OK:
        raise OrbslamError(f"{what} failed with status {rc}")


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def build_id() -> str:
    """Hash of the sources the loaded library was built from (tools/src_hash.py)."""
    return lib().orbx_build_id().decode()


def device_count() -> int:
    return lib().orbslam2_amd_device_count()


def set_device(device: int):
    _check(lib().orbslam2_amd_set_device(device), "set_device")


def device_sync():
    _check(lib().orbslam2_amd_device_sync(), "device_sync")


class ORBextractor:
    """ORBextractor (include/ORBextractor.h:80-216) backed by the HIP kernels."""

    def __init__(self, nfeatures: int, scaleFactor: float = 1.2, nlevels: int = 8,
                 iniThFAST: int = 20, minThFAST: int = 7, resize_mode: int = 0, blur_mode: int = 0):
        self._h = C.c_void_p()
        p = OrbxParams(C.sizeof(OrbxParams), nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, resize_mode, blur_mode)
        _check(lib().orbx_create(C.byref(p), C.byref(self._h)), "orbx_create")
        self.nfeatures = nfeatures
        self.nlevels = nlevels

    def close(self):
        if getattr(self, "_view", False):   # engine owned by a StereoPipeline
            return
        if getattr(self, "_h", None) and self._h.value:
            lib().orbx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def _levels(self):
        L = self.nlevels
        arrs = [np.zeros(L, np.float32) for _ in range(4)] + [np.zeros(L, np.int32)]
        n = C.c_int()
        _check(lib().orbx_levels(self._h, C.byref(n), *[_p(a) for a in arrs]), "orbx_levels")
        return arrs

    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactors(self):
        return self._levels()[0]

    def GetInverseScaleFactors(self):
        return self._levels()[1]

    def GetScaleSigmaSquares(self):
        return self._levels()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._levels()[3]

    def features_per_level(self):
        return list(self._levels()[4])

    def __call__(self, image: np.ndarray, mask=None):
        """operator()(image, mask, keypoints, descriptors); returns (keypoints, descriptors)."""
        img = np.ascontiguousarray(image, np.uint8)
        if img.ndim != 2:
            raise ValueError("expects a single-channel u8 image (ORBextractor.cc:1553)")
        h, w = img.shape
        cap = max(64, self.nfeatures * 2 + 512)
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int()
        _check(lib().orbx_extract(self._h, _p(img), w, h, w, _p(kps), _p(desc), cap, C.byref(n)),
               "orbx_extract")
        return kps[: n.value].copy(), desc[: n.value].copy()

    def pyramid_level(self, level: int, image: int = 0) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        _check(lib().orbx_pyramid_level(self._h, image, level, None, C.byref(w), C.byref(h)), "pyramid")
        out = np.zeros((h.value, w.value), np.uint8)
        _check(lib().orbx_pyramid_level(self._h, image, level, _p(out), None, None), "pyramid")
        return out

    def blurred_level(self, level: int, image: int = 0) -> np.ndarray:
        """The 9x9 GaussianBlur of pyramid level `level` that the descriptors sample."""
        w, h = C.c_int(), C.c_int()
        _check(lib().orbx_blurred_level(self._h, image, level, None, C.byref(w), C.byref(h)), "blurred")
        out = np.zeros((h.value, w.value), np.uint8)
        _check(lib().orbx_blurred_level(self._h, image, level, _p(out), None, None), "blurred")
        return out


class BatchExtractor(ORBextractor):
    """Batched device-resident extraction: many frames per launch (bench / throughput)."""

    def reserve(self, w: int, h: int, max_images: int):
        _check(lib().orbx_reserve(self._h, w, h, max_images), "orbx_reserve")

    def extract_device(self, d_ptr: int, n_images: int, w: int, h: int, pitch: int,
                       image_stride: int, stream: int | None = None):
        _check(lib().orbx_extract_batch_device(self._h, C.c_void_p(d_ptr), n_images, w, h, pitch,
                                               image_stride, C.c_void_p(stream or 0)),
               "orbx_extract_batch_device")

    def extract_device_phase(self, d_ptr: int, n_images: int, w: int, h: int, pitch: int,
                             image_stride: int, phase: int, stream: int | None = None):
        """Phase 1 (pyramid + FAST map + blur) or 2 (NMS, quadtree, descriptors) of extract_device."""
        _check(lib().orbx_extract_batch_device_phase(self._h, C.c_void_p(d_ptr), n_images, w, h, pitch,
                                                     image_stride, C.c_void_p(stream or 0), phase),
               "orbx_extract_batch_device_phase")

    def stream(self) -> int:
        return lib().orbx_stream(self._h) or 0

    def profile(self, enable: bool):
        _check(lib().orbx_profile(self._h, 1 if enable else 0), "orbx_profile")

    def profile_read(self) -> dict:
        """{kernel name: (total ms, launches)} of the hipEvent records since profile(True)."""
        out = {}
        i = 0
        buf = C.create_string_buffer(64)
        while True:
            ms, n = C.c_double(), C.c_int()
            rc = lib().orbx_profile_read(self._h, i, buf, 64, C.byref(ms), C.byref(n))
            if rc == ORBX_ESTATE:
                break
            _check(rc, "orbx_profile_read")
            out[buf.value.decode()] = (ms.value, n.value)
            i += 1
        return out

    def fetch(self, image: int):
        cap = max(64, self.nfeatures * 2 + 512)
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int()
        _check(lib().orbx_batch_fetch(self._h, image, _p(kps), _p(desc), cap, C.byref(n)), "orbx_batch_fetch")
        return kps[: n.value].copy(), desc[: n.value].copy()

    def results(self):
        cnt, kps, desc, cap = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int()
        _check(lib().orbx_batch_results(self._h, C.byref(cnt), C.byref(kps), C.byref(desc), C.byref(cap)),
               "orbx_batch_results")
        return cnt.value, kps.value, desc.value, cap.value

    def stereo_batch(self, n_pairs: int, mbf: float, mb: float, stream: int | None = None):
        _check(lib().orbm_stereo_match_batch_device(self._h, n_pairs, mbf, mb, C.c_void_p(stream or 0)),
               "orbm_stereo_match_batch_device")

    def rgbd_device(self, d_depth: int, depth_stride: int, dpitch: int, K, dist, mbf: float, stream=None):
        Ka, Da = np.asarray(K, np.float32), np.asarray(dist, np.float32)
        _check(lib().orbf_rgbd_batch_device(self._h, C.c_void_p(d_depth), depth_stride, dpitch, _p(Ka), _p(Da),
                                            mbf, C.c_void_p(stream or 0)), "orbf_rgbd_batch_device")

    def rgbd_fetch(self, image: int):
        cap = max(64, self.nfeatures * 2 + 512)
        ku = np.zeros(cap, KP_DTYPE)
        u = np.zeros(cap, np.float32)
        d = np.zeros(cap, np.float32)
        _check(lib().orbf_rgbd_fetch(self._h, image, _p(ku), _p(u), _p(d), cap), "orbf_rgbd_fetch")
        return ku, u, d

    def search_init_device(self, n_pairs, f1_base, f1_step, f2_base, f2_step, K, dist, window=100,
                           nnratio=0.9, check_ori=True, stream=None):
        Ka, Da = np.asarray(K, np.float32), np.asarray(dist, np.float32)
        _check(lib().orbm_search_init_batch_device(self._h, n_pairs, f1_base, f1_step, f2_base, f2_step, _p(Ka),
                                                   _p(Da), window, nnratio, 1 if check_ori else 0,
                                                   C.c_void_p(stream or 0)), "orbm_search_init_batch_device")

    def search_init_fetch(self, pair: int):
        cap = max(64, self.nfeatures * 2 + 512)
        m = np.zeros(cap, np.int32)
        xy = np.zeros(2 * cap, np.float32)
        n = C.c_int()
        _check(lib().orbm_search_init_fetch(self._h, pair, _p(m), _p(xy), cap, C.byref(n)), "orbm_search_init_fetch")
        return n.value, m, xy.reshape(-1, 2)

    def stereo_fetch(self, pair: int):
        cap = max(64, self.nfeatures * 2 + 512)
        u = np.zeros(cap, np.float32)
        d = np.zeros(cap, np.float32)
        _check(lib().orbm_stereo_fetch(self._h, pair, _p(u), _p(d), cap), "orbm_stereo_fetch")
        return u, d


class StereoHostOut(C.Structure):
    """orbx_stereo_host_out (include/orbslam2_amd.h)."""
    _fields_ = [("counts", C.c_void_p), ("kps", C.c_void_p), ("desc", C.c_void_p), ("u_right", C.c_void_p),
                ("depth", C.c_void_p)]


class _HostBlock:
    """Owner of one orbx_host_alloc block; numpy views keep it alive via .base chains."""

    def __init__(self, nbytes: int):
        self.p = C.c_void_p()
        self.nbytes = max(int(nbytes), 1)
        _check(lib().orbx_host_alloc(self.nbytes, C.byref(self.p)), "orbx_host_alloc")

    def __del__(self):
        try:
            if self.p.value:
                lib().orbx_host_free(self.p)
        except Exception:
            pass


def host_empty(shape, dtype) -> np.ndarray:
    """numpy array over page-locked host memory (orbx_host_alloc), for the host-mode pipeline."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    blk = _HostBlock(n)
    buf = (C.c_char * blk.nbytes).from_address(blk.p.value)
    buf.owner = blk   # the array's base chain ends at buf, which keeps the block alive
    return np.frombuffer(buf, np.uint8, n).view(dt).reshape(shape)


class StereoHostBatch:
    """Page-locked host outputs of one stereo batch (orbx_stereo_host_out)."""

    def __init__(self, n_pairs: int, cap: int):
        self.n_pairs, self.cap = n_pairs, cap
        self.counts = host_empty((2 * n_pairs,), np.int32)
        self.kps = host_empty((2 * n_pairs, cap), KP_DTYPE)
        self.desc = host_empty((2 * n_pairs, cap, 32), np.uint8)
        self.u_right = host_empty((n_pairs, cap), np.float32)
        self.depth = host_empty((n_pairs, cap), np.float32)
        self.c = StereoHostOut(self.counts.ctypes.data, self.kps.ctypes.data, self.desc.ctypes.data,
                               self.u_right.ctypes.data, self.depth.ctypes.data)

    def pair(self, p: int):
        """(kL, dL, kR, dR, mvuRight, mvDepth) of pair p, trimmed to the keypoint counts."""
        nL, nR = int(self.counts[2 * p]), int(self.counts[2 * p + 1])
        return (self.kps[2 * p, :nL], self.desc[2 * p, :nL], self.kps[2 * p + 1, :nR], self.desc[2 * p + 1, :nR],
                self.u_right[p, :nL], self.depth[p, :nL])


class StereoPipeline:
    """Batched stereo Frame construction (extract L + R, ComputeStereoMatches) over k engines on
    k HIP streams, their pyramid / FAST / blur phases in turn (orbx_pipeline_*, orb_pipeline.hip).
    Pair p of the last batch lives on engine chunk_of(p)."""

    def __init__(self, nfeatures: int = 2000, scaleFactor: float = 1.2, nlevels: int = 8,
                 iniThFAST: int = 20, minThFAST: int = 7, n_engines: int = 3, resize_mode: int = 0,
                 blur_mode: int = 0):
        self._h = C.c_void_p()
        p = OrbxParams(C.sizeof(OrbxParams), nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, resize_mode, blur_mode)
        _check(lib().orbx_pipeline_create(C.byref(p), n_engines, C.byref(self._h)), "orbx_pipeline_create")
        self.nfeatures, self.nlevels = nfeatures, nlevels
        self.engines = []
        for i in range(lib().orbx_pipeline_engines(self._h)):
            e = C.c_void_p()
            _check(lib().orbx_pipeline_chunk(self._h, i, C.byref(e), None, None), "orbx_pipeline_chunk")
            v = BatchExtractor.__new__(BatchExtractor)
            v._h, v._view, v.nfeatures, v.nlevels = e, True, nfeatures, nlevels
            self.engines.append(v)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().orbx_pipeline_destroy(self._h)
            self._h = C.c_void_p()
            self.engines = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, w: int, h: int, max_pairs: int):
        _check(lib().orbx_pipeline_reserve(self._h, w, h, max_pairs), "orbx_pipeline_reserve")

    def stereo_batch(self, d_ptr: int, n_pairs: int, w: int, h: int, pitch: int, image_stride: int,
                     mbf: float, mb: float, stream: int | None = None):
        _check(lib().orbx_pipeline_stereo_batch(self._h, C.c_void_p(d_ptr), n_pairs, w, h, pitch, image_stride,
                                                mbf, mb, C.c_void_p(stream or 0)), "orbx_pipeline_stereo_batch")

    def capacity(self) -> int:
        cap = C.c_int()
        _check(lib().orbx_pipeline_capacity(self._h, C.byref(cap)), "orbx_pipeline_capacity")
        return cap.value

    def stereo_batch_host(self, h_imgs: np.ndarray, n_pairs: int, w: int, h: int, pitch: int, image_stride: int,
                          mbf: float, mb: float, out: "StereoHostBatch"):
        """Host images in (ideally host_empty memory), host outputs into `out`; asynchronous until wait()."""
        # the C side uploads whole image_stride blocks (2 * n_pairs of them) and writes
        # 2 * n_pairs * capacity() records into out's page-locked arrays, with no sizes to check against
        if not h_imgs.flags.c_contiguous or h_imgs.nbytes < 2 * n_pairs * image_stride:
            raise ValueError("h_imgs must be a contiguous buffer of 2 * n_pairs images")
        if not isinstance(out, StereoHostBatch) or out.n_pairs < n_pairs or out.cap != self.capacity():
            raise ValueError("out must be a StereoHostBatch of >= n_pairs pairs with cap == capacity()")
        _check(lib().orbx_pipeline_stereo_batch_host(self._h, C.c_void_p(h_imgs.ctypes.data), n_pairs, w, h, pitch,
                                                     image_stride, mbf, mb, C.byref(out.c)),
               "orbx_pipeline_stereo_batch_host")

    def wait(self):
        _check(lib().orbx_pipeline_wait(self._h), "orbx_pipeline_wait")

    def join(self, stream: int | None = None):
        """Make `stream` (default: the legacy default stream) wait for the last batch."""
        _check(lib().orbx_pipeline_join(self._h, C.c_void_p(stream or 0)), "orbx_pipeline_join")

    def chunk(self, i: int):
        first, n = C.c_int(), C.c_int()
        _check(lib().orbx_pipeline_chunk(self._h, i, None, C.byref(first), C.byref(n)), "orbx_pipeline_chunk")
        return self.engines[i], first.value, n.value

    def chunk_of(self, pair: int):
        for i in range(len(self.engines)):
            ex, first, n = self.chunk(i)
            if first <= pair < first + n:
                return ex, pair - first
        raise IndexError(pair)

    def fetch(self, pair: int):
        """(left keypoints, left descriptors, right keypoints, right descriptors) of a pair."""
        ex, p = self.chunk_of(pair)
        return (*ex.fetch(2 * p), *ex.fetch(2 * p + 1))

    def stereo_fetch(self, pair: int):
        ex, p = self.chunk_of(pair)
        return ex.stereo_fetch(p)

    def profile(self, enable: bool):
        for ex in self.engines:
            ex.profile(enable)

    def profile_read(self) -> dict:
        """{kernel name: (total ms, launches)} summed over the engines."""
        out = {}
        for ex in self.engines:
            for k, (ms, n) in ex.profile_read().items():
                a, b = out.get(k, (0.0, 0))
                out[k] = (a + ms, b + n)
        return out


def compute_stereo_from_rgbd(ex: ORBextractor, n: int, depth: np.ndarray, K, dist, mbf: float):
    """UndistortKeyPoints + ComputeStereoFromRGBD for the extractor's last image ->
    (mvKeysUn, mvuRight, mvDepth)."""
    depth = np.ascontiguousarray(depth, np.float32)
    Ka, Da = np.asarray(K, np.float32), np.asarray(dist, np.float32)
    ku = np.zeros(max(n, 1), KP_DTYPE)
    u = np.zeros(max(n, 1), np.float32)
    d = np.zeros(max(n, 1), np.float32)
    _check(lib().orbf_rgbd(ex.handle, _p(depth), depth.shape[1], _p(Ka), _p(Da), mbf, _p(ku), _p(u), _p(d), n),
           "orbf_rgbd")
    return ku[:n], u[:n], d[:n]


def compute_stereo_matches(left: ORBextractor, right: ORBextractor, n_left: int, mbf: float, mb: float):
    """Frame::ComputeStereoMatches over the two extractors' last frames -> (mvuRight, mvDepth)."""
    u = np.zeros(max(n_left, 1), np.float32)
    d = np.zeros(max(n_left, 1), np.float32)
    _check(lib().orbm_stereo_match(left.handle, right.handle, mbf, mb, _p(u), _p(d), n_left), "orbm_stereo_match")
    return u[:n_left], d[:n_left]


class OrbmFrame(C.Structure):
    """orbm_frame: the Frame members SearchForInitialization reads (include/Frame.h)."""
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("desc", C.c_void_p), ("min_x", C.c_float),
                ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


class ORBmatcher:
    """ORBmatcher(nnratio=0.6, checkOri=True) (ORBmatcher.h:57): a matcher handle with its own HIP
    stream (orbm_create), DescriptorDistance scans and SearchForInitialization on host frames."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self.mfNNratio = nnratio
        self.mbCheckOrientation = checkOri
        self._h = C.c_void_p()
        _check(lib().orbm_create(nnratio, 1 if checkOri else 0, C.byref(self._h)), "orbm_create")

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().orbm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def hamming_best2(q: np.ndarray, db: np.ndarray):
        """Brute force over db (orbm_hamming_best2, per-thread matcher)."""
        q = np.ascontiguousarray(q, np.uint8)
        db = np.ascontiguousarray(db, np.uint8)
        n = len(q)
        bi = np.zeros(max(n, 1), np.int32)
        bd = np.zeros(max(n, 1), np.int32)
        sd = np.zeros(max(n, 1), np.int32)
        _check(lib().orbm_hamming_best2(_p(q), n, _p(db), len(db), _p(bi), _p(bd), _p(sd)), "orbm_hamming_best2")
        return bi[:n], bd[:n], sd[:n]

    def hamming_best2_cand(self, q: np.ndarray, db: np.ndarray, cand_off=None, cand_idx=None):
        """Best / second over CSR candidate lists cand_idx[cand_off[i]:cand_off[i+1]] (None: all of db)."""
        q = np.ascontiguousarray(q, np.uint8)
        db = np.ascontiguousarray(db, np.uint8)
        n = len(q)
        bi = np.zeros(max(n, 1), np.int32)
        bd = np.zeros(max(n, 1), np.int32)
        sd = np.zeros(max(n, 1), np.int32)
        off = idx = None
        if cand_off is not None:
            off = np.ascontiguousarray(cand_off, np.int32)
            if off.ndim != 1 or len(off) != n + 1:
                raise ValueError("cand_off must hold len(q) + 1 offsets")
            idx = np.ascontiguousarray(cand_idx if cand_idx is not None else np.zeros(0), np.int32)
            if off[0] < 0 or np.any(np.diff(off) < 0) or off[-1] > len(idx):
                raise ValueError("cand_off must be non-decreasing offsets into cand_idx")
            if len(idx) == 0:
                idx = np.zeros(1, np.int32)
        _check(lib().orbm_hamming_best2_cand(self._h, _p(q), n, _p(db), len(db), _p(off) if off is not None else None,
                                             _p(idx) if idx is not None else None, _p(bi), _p(bd), _p(sd)),
               "orbm_hamming_best2_cand")
        return bi[:n], bd[:n], sd[:n]

    def SearchForInitialization(self, F1, F2, vbPrevMatched: np.ndarray, windowSize: int = 10):
        """SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) on host frames.
        F = (keys_un KP_DTYPE array, desc n x 32, (minX, maxX, minY, maxY)). vbPrevMatched (n1 x 2
        float32) is updated in place, as the reference's reference argument. -> (nmatches, vnMatches12)."""
        def frame(F):
            ku, de, b = F
            ku = np.ascontiguousarray(ku, KP_DTYPE)
            de = np.ascontiguousarray(de, np.uint8)
            return OrbmFrame(len(ku), ku.ctypes.data if len(ku) else None, de.ctypes.data if len(ku) else None,
                             *[float(v) for v in b]), (ku, de)
        f1, keep1 = frame(F1)
        f2, keep2 = frame(F2)
        if (vbPrevMatched.dtype != np.float32 or not vbPrevMatched.flags.c_contiguous
                or vbPrevMatched.size < 2 * f1.n):
            raise ValueError("vbPrevMatched must be a C-contiguous float32 (n1, 2) array (updated in place)")
        m12 = np.full(max(f1.n, 1), -1, np.int32)
        n = C.c_int32()
        _check(lib().orbm_search_for_initialization(self._h, C.byref(f1), C.byref(f2), _p(vbPrevMatched), _p(m12),
                                                    int(windowSize), C.byref(n)), "orbm_search_for_initialization")
        return n.value, m12[: f1.n]


class LbaProblem(C.Structure):
    """lba_problem (include/orbslam2_amd.h): the graph Optimizer::LocalBundleAdjustment builds."""
    _fields_ = [("n_poses", C.c_int32), ("pose_id", C.c_void_p), ("pose_fixed", C.c_void_p),
                ("pose_Tcw", C.c_void_p), ("pose_cam", C.c_void_p), ("n_points", C.c_int32),
                ("point_id", C.c_void_p), ("point_Xw", C.c_void_p), ("n_edges", C.c_int32),
                ("edge_point", C.c_void_p), ("edge_pose", C.c_void_p), ("edge_obs", C.c_void_p),
                ("edge_inv_sigma2", C.c_void_p)]


class LbaResult(C.Structure):
    _fields_ = [("pose_Tcw", C.c_void_p), ("point_Xw", C.c_void_p), ("edge_erase", C.c_void_p),
                ("iterations", C.c_int32 * 2), ("chi2", C.c_double * 2), ("stopped", C.c_int32),
                ("trials", C.c_int32 * 2)]


_LBA_FIELDS = ("pose_id", "pose_fixed", "pose_Tcw", "pose_cam", "point_id", "point_Xw", "edge_point",
               "edge_pose", "edge_obs", "edge_inv_sigma2")
_LBA_DTYPES = {"pose_id": np.int32, "pose_fixed": np.uint8, "pose_Tcw": np.float32, "pose_cam": np.float32,
               "point_id": np.int32, "point_Xw": np.float32, "edge_point": np.int32, "edge_pose": np.int32,
               "edge_obs": np.float32, "edge_inv_sigma2": np.float32}


class LocalBundleAdjustment:
    """Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap) (Optimizer.h:112) on the GPU.

    ``solve(problem)`` takes the flattened graph (see synth.localba_problem) and returns the
    optimised poses (Tcw 4x4 float), points and the per-edge erase flags (vToErase)."""

    def __init__(self):
        self._h = C.c_void_p()
        _check(lib().lba_create(C.byref(self._h)), "lba_create")

    def close(self):
        if getattr(self, "_view", False):   # engine owned by a StereoPipeline
            return
        if getattr(self, "_h", None) and self._h.value:
            lib().lba_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stop_hook(self, phase: int = 0, trial: int = 0):
        """lba_set_stop_hook: act as if pbStopFlag were raised after trial `trial` of optimize() call
        `phase` (1 or 2; 0 removes the hook)."""
        _check(lib().lba_set_stop_hook(self._h, int(phase), int(trial)), "lba_set_stop_hook")

    LBA_OPT_FUSE_FINISH = 1
    LBA_OPT_SPIN_LIMIT = 2
    LBA_OPT_STREAM_PRIORITY = 3

    def set_test_option(self, option: int, value: int):
        """lba_set_test_option: LBA_OPT_FUSE_FINISH (1 fused, 0 two launches) or LBA_OPT_SPIN_LIMIT
        (< 0 default, 0 fault injection: every in-launch hand-off wait times out)."""
        _check(lib().lba_set_test_option(self._h, int(option), int(value)), "lba_set_test_option")

    def solve(self, prob: dict, stop=False) -> dict:
        """`stop`: a bool (the flag's value for the whole call) or a ctypes.c_uint8 shared with
        another thread that may raise it while the call runs (ctypes releases the GIL)."""
        keep = {k: np.ascontiguousarray(prob[k], _LBA_DTYPES[k]) for k in _LBA_FIELDS}
        P = LbaProblem(len(keep["pose_id"]), keep["pose_id"].ctypes.data, keep["pose_fixed"].ctypes.data,
                       keep["pose_Tcw"].ctypes.data, keep["pose_cam"].ctypes.data, len(keep["point_id"]),
                       keep["point_id"].ctypes.data, keep["point_Xw"].ctypes.data, len(keep["edge_point"]),
                       keep["edge_point"].ctypes.data, keep["edge_pose"].ctypes.data,
                       keep["edge_obs"].ctypes.data, keep["edge_inv_sigma2"].ctypes.data)
        out = {"pose_Tcw": np.zeros((len(keep["pose_id"]), 16), np.float32),
               "point_Xw": np.zeros((len(keep["point_id"]), 3), np.float32),
               "edge_erase": np.zeros(len(keep["edge_point"]), np.uint8)}
        R = LbaResult(out["pose_Tcw"].ctypes.data, out["point_Xw"].ctypes.data, out["edge_erase"].ctypes.data)
        flag = stop if isinstance(stop, C.c_uint8) else C.c_uint8(1 if stop else 0)
        _check(lib().lba_solve(self._h, C.byref(P), C.byref(R), C.byref(flag)), "lba_solve")
        out["iterations"] = tuple(R.iterations)
        out["chi2"] = tuple(R.chi2)
        out["stopped"] = R.stopped
        out["trials"] = tuple(R.trials)
        return out

    def profile(self, enable: bool):
        _check(lib().lba_profile(self._h, 1 if enable else 0), "lba_profile")

    def profile_read(self) -> dict:
        """{kernel group: (total ms, launches)} since profile(True)."""
        out, i = {}, 0
        buf = C.create_string_buffer(64)
        while True:
            ms, n = C.c_double(), C.c_int()
            rc = lib().lba_profile_read(self._h, i, buf, 64, C.byref(ms), C.byref(n))
            if rc == ORBX_ESTATE:
                break
            _check(rc, "lba_profile_read")
            out[buf.value.decode()] = (ms.value, n.value)
            i += 1
        return out


# ---- tracking matchers (orbt_*): Frame::isInFrustum + ORBmatcher::SearchByProjection --------
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


def _orbt_frame(fr: dict):
    keep = {"keys_un": np.ascontiguousarray(fr["keys_un"]).view(KP_DTYPE),
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


def _orbt_map(mp: dict):
    keep = {k: np.ascontiguousarray(mp[k], np.uint8 if k in ("desc", "flags") else np.float32)
            for k in ("Xw", "normal", "min_dist", "max_dist", "desc", "flags")}
    M = OrbtMapPoints(len(keep["Xw"]), *(keep[k].ctypes.data for k in ("Xw", "normal", "min_dist", "max_dist",
                                                                        "desc", "flags")))
    return M, keep


class Tracker:
    """The per-frame tracking matchers of ORBmatcher (ORBmatcher.h:82,102) plus
    Frame::isInFrustum, on the GPU. Problems are dicts shaped like synth.tracking_problem:
    {"frame", "map", "last", "last_mp", "last_outlier", "kp_blocked"}."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().orbt_create(C.byref(h)), "orbt_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _blk(prob):
        b = prob.get("kp_blocked")
        return np.ascontiguousarray(b, np.uint8) if b is not None else None

    def search_local_points(self, prob: dict, cos_limit=0.5, th=1.0, nnratio=0.8):
        F, k1 = _orbt_frame(prob["frame"])
        M, k2 = _orbt_map(prob["map"])
        n, m = F.n, M.n
        view = {"in_view": np.zeros(max(m, 1), np.uint8), "proj_x": np.zeros(max(m, 1), np.float32),
                "proj_y": np.zeros(max(m, 1), np.float32), "proj_xr": np.zeros(max(m, 1), np.float32),
                "view_cos": np.zeros(max(m, 1), np.float32), "level": np.zeros(max(m, 1), np.int32)}
        V = OrbtView(*(view[k].ctypes.data for k in ("in_view", "proj_x", "proj_y", "proj_xr", "view_cos", "level")))
        owner = np.zeros(max(n, 1), np.int32)
        nm = C.c_int32()
        blk = self._blk(prob)
        _check(lib().orbt_search_local_points(self._h, C.byref(F), C.byref(M), cos_limit, th, nnratio,
                                              blk.ctypes.data if blk is not None else None, C.byref(V),
                                              owner.ctypes.data, C.byref(nm)), "orbt_search_local_points")
        return nm.value, owner[:n], {k: v[:m] for k, v in view.items()}

    def search_by_projection_frame(self, prob: dict, th=15.0, mono=False, check_ori=True):
        F, k1 = _orbt_frame(prob["frame"])
        Lf, k2 = _orbt_frame(prob["last"])
        M, k3 = _orbt_map(prob["map"])
        last_mp = np.ascontiguousarray(prob["last_mp"], np.int32)
        last_out = np.ascontiguousarray(prob["last_outlier"], np.uint8)
        owner = np.zeros(max(F.n, 1), np.int32)
        nm = C.c_int32()
        blk = self._blk(prob)
        _check(lib().orbt_search_by_projection_frame(self._h, C.byref(F), C.byref(Lf), last_mp.ctypes.data,
                                                     last_out.ctypes.data, C.byref(M), th, 1 if mono else 0,
                                                     1 if check_ori else 0,
                                                     blk.ctypes.data if blk is not None else None,
                                                     owner.ctypes.data, C.byref(nm)),
               "orbt_search_by_projection_frame")
        return nm.value, owner[: F.n]

    def search_by_projection_keyframe(self, prob: dict, th=10.0, orb_dist=100, check_ori=True):
        """ORBmatcher(0.9, checkOri).SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
        ORBdist) (Tracking::Relocalization); prob["last"] / prob["last_mp"] are the keyframe and
        its map point matches, map flags ORBT_MP_FOUND = sAlreadyFound."""
        F, k1 = _orbt_frame(prob["frame"])
        Kf, k2 = _orbt_frame(prob["last"])
        M, k3 = _orbt_map(prob["map"])
        kf_mp = np.ascontiguousarray(prob["last_mp"], np.int32)
        owner = np.zeros(max(F.n, 1), np.int32)
        nm = C.c_int32()
        blk = self._blk(prob)
        _check(lib().orbt_search_by_projection_keyframe(self._h, C.byref(F), C.byref(Kf), kf_mp.ctypes.data,
                                                        C.byref(M), th, int(orb_dist), 1 if check_ori else 0,
                                                        blk.ctypes.data if blk is not None else None,
                                                        owner.ctypes.data, C.byref(nm)),
               "orbt_search_by_projection_keyframe")
        return nm.value, owner[: F.n]

    def run_reloc_batch(self, n_slots: int, th=10.0, orb_dist=100, check_ori=True, stream=None):
        _check(lib().orbt_run_reloc_batch(self._h, n_slots, th, int(orb_dist), 1 if check_ori else 0, stream),
               "orbt_run_reloc_batch")

    def search_by_projection_sim3(self, prob: dict, th=10):
        """LoopClosing's SearchByProjection(pKF, Scw, vpPoints, vpMatched, th): prob = {"frame" (pKF),
        "map" (vpPoints), "Scw" (4x4), "matched" (vpMatched as point indices, -1 NULL, -2 outside)}.
        Returns (nmatches, vpMatched out)."""
        F, k1 = _orbt_frame(prob["frame"])
        M, k2 = _orbt_map(prob["map"])
        Scw = np.ascontiguousarray(prob["Scw"], np.float32).reshape(16)
        matched = np.array(prob["matched"], np.int32, copy=True)
        nm = C.c_int32()
        _check(lib().orbt_search_by_projection_sim3(self._h, C.byref(F), Scw.ctypes.data, C.byref(M), int(th),
                                                    matched.ctypes.data, C.byref(nm)), "orbt_search_by_projection_sim3")
        return nm.value, matched[: F.n]

    def stage_sim3(self, slot: int, prob: dict):
        F, k1 = _orbt_frame(prob["frame"])
        M, k2 = _orbt_map(prob["map"])
        Scw = np.ascontiguousarray(prob["Scw"], np.float32).reshape(16)
        matched = np.ascontiguousarray(prob["matched"], np.int32)
        _check(lib().orbt_stage_sim3(self._h, slot, C.byref(F), Scw.ctypes.data, C.byref(M), matched.ctypes.data),
               "orbt_stage_sim3")

    def run_sim3_batch(self, n_slots: int, th=10, stream=None):
        _check(lib().orbt_run_sim3_batch(self._h, n_slots, int(th), stream), "orbt_run_sim3_batch")

    def fetch_sim3(self, slot: int, prob: dict):
        n = len(prob["frame"]["keys_un"])
        nm, owner, _ = self.fetch(slot, n)
        matched = np.array(prob["matched"], np.int32, copy=True)[:n]
        matched[owner >= 0] = owner[owner >= 0]
        return nm, matched

    def fuse_sim3_candidates(self, prob: dict, th=4.0):
        """LoopClosing's Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) search half -> (best_idx, best_dist)."""
        F, k1 = _orbt_frame(prob["frame"])
        M, k2 = _orbt_map(prob["map"])
        Scw = np.ascontiguousarray(prob["Scw"], np.float32).reshape(16)
        bi = np.zeros(max(M.n, 1), np.int32)
        bd = np.zeros(max(M.n, 1), np.int32)
        _check(lib().orbt_fuse_sim3_candidates(self._h, C.byref(F), Scw.ctypes.data, C.byref(M), th, bi.ctypes.data,
                                               bd.ctypes.data), "orbt_fuse_sim3_candidates")
        return bi[: M.n], bd[: M.n]

    @staticmethod
    def _sim3_args(prob):
        F1, k1 = _orbt_frame(prob["kf1"])
        F2, k2 = _orbt_frame(prob["kf2"])
        M, k3 = _orbt_map(prob["map"])
        keep = {"mp1": np.ascontiguousarray(prob["kf1_mp"], np.int32), "mp2": np.ascontiguousarray(prob["kf2_mp"], np.int32),
                "R12": np.ascontiguousarray(prob["R12"], np.float32).reshape(9),
                "t12": np.ascontiguousarray(prob["t12"], np.float32).reshape(3), "k": (k1, k2, k3)}
        return F1, F2, M, keep

    def search_by_sim3(self, prob: dict, th=7.5):
        """ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) -> (nFound, matches12 out)."""
        F1, F2, M, kp = self._sim3_args(prob)
        m12 = np.array(prob["matches12"], np.int32, copy=True)
        nf = C.c_int32()
        _check(lib().orbt_search_by_sim3(self._h, C.byref(F1), kp["mp1"].ctypes.data, C.byref(F2), kp["mp2"].ctypes.data,
                                         C.byref(M), float(prob["s12"]), kp["R12"].ctypes.data, kp["t12"].ctypes.data, th,
                                         m12.ctypes.data, C.byref(nf)), "orbt_search_by_sim3")
        return nf.value, m12[: F1.n]

    def stage_search_by_sim3(self, pair: int, prob: dict):
        F1, F2, M, kp = self._sim3_args(prob)
        m12 = np.ascontiguousarray(prob["matches12"], np.int32)
        _check(lib().orbt_stage_search_by_sim3(self._h, pair, C.byref(F1), kp["mp1"].ctypes.data, C.byref(F2),
                                               kp["mp2"].ctypes.data, C.byref(M), float(prob["s12"]),
                                               kp["R12"].ctypes.data, kp["t12"].ctypes.data, m12.ctypes.data),
               "orbt_stage_search_by_sim3")

    def run_sim3_match_batch(self, n_pairs: int, th=7.5, stream=None):
        _check(lib().orbt_run_sim3_match_batch(self._h, n_pairs, th, stream), "orbt_run_sim3_match_batch")

    def fetch_search_by_sim3(self, pair: int, prob: dict):
        mp2 = np.ascontiguousarray(prob["kf2_mp"], np.int32)
        m12 = np.array(prob["matches12"], np.int32, copy=True)
        nf = C.c_int32()
        _check(lib().orbt_fetch_search_by_sim3(self._h, pair, mp2.ctypes.data, m12.ctypes.data, C.byref(nf)),
               "orbt_fetch_search_by_sim3")
        return nf.value, m12

    def fuse_candidates(self, prob: dict, th=3.0):
        """ORBmatcher::Fuse(pKF, vpMapPoints, th) search half; prob["frame"] is the KeyFrame."""
        F, k1 = _orbt_frame(prob["frame"])
        M, k2 = _orbt_map(prob["map"])
        bi = np.zeros(max(M.n, 1), np.int32)
        bd = np.zeros(max(M.n, 1), np.int32)
        _check(lib().orbt_fuse_candidates(self._h, C.byref(F), C.byref(M), th, bi.ctypes.data, bd.ctypes.data),
               "orbt_fuse_candidates")
        return bi[: M.n], bd[: M.n]

    def run_fuse_batch(self, n_slots: int, th=3.0, stream=None):
        _check(lib().orbt_run_fuse_batch(self._h, n_slots, th, stream), "orbt_run_fuse_batch")

    def fetch_fuse(self, slot: int, n_mp: int):
        bi = np.zeros(max(n_mp, 1), np.int32)
        bd = np.zeros(max(n_mp, 1), np.int32)
        _check(lib().orbt_fetch_fuse(self._h, slot, bi.ctypes.data, bd.ctypes.data), "orbt_fetch_fuse")
        return bi[:n_mp], bd[:n_mp]

    # batched device-resident path (bench.py)
    def reserve(self, n_slots: int, cap_kp: int, cap_mp: int):
        _check(lib().orbt_reserve(self._h, n_slots, cap_kp, cap_mp), "orbt_reserve")

    def stage(self, slot: int, prob: dict):
        F, k1 = _orbt_frame(prob["frame"])
        Lf, k2 = _orbt_frame(prob["last"])
        M, k3 = _orbt_map(prob["map"])
        last_mp = np.ascontiguousarray(prob["last_mp"], np.int32)
        last_out = np.ascontiguousarray(prob["last_outlier"], np.uint8)
        blk = self._blk(prob)
        _check(lib().orbt_stage(self._h, slot, C.byref(F), C.byref(M), C.byref(Lf), last_mp.ctypes.data,
                                last_out.ctypes.data, blk.ctypes.data if blk is not None else None), "orbt_stage")

    def run_local_batch(self, n_slots: int, cos_limit=0.5, th=1.0, nnratio=0.8, stream=None):
        _check(lib().orbt_run_local_batch(self._h, n_slots, cos_limit, th, nnratio, stream), "orbt_run_local_batch")

    def run_frame_batch(self, n_slots: int, th=15.0, mono=False, check_ori=True, stream=None):
        _check(lib().orbt_run_frame_batch(self._h, n_slots, th, 1 if mono else 0, 1 if check_ori else 0, stream),
               "orbt_run_frame_batch")

    def fetch(self, slot: int, n_kp: int, n_mp: int = 0):
        owner = np.zeros(max(n_kp, 1), np.int32)
        nm = C.c_int32()
        view = None
        V = None
        if n_mp:
            view = {"in_view": np.zeros(n_mp, np.uint8), "proj_x": np.zeros(n_mp, np.float32),
                    "proj_y": np.zeros(n_mp, np.float32), "proj_xr": np.zeros(n_mp, np.float32),
                    "view_cos": np.zeros(n_mp, np.float32), "level": np.zeros(n_mp, np.int32)}
            V = OrbtView(*(view[k].ctypes.data for k in ("in_view", "proj_x", "proj_y", "proj_xr", "view_cos",
                                                         "level")))
        _check(lib().orbt_fetch(self._h, slot, C.byref(V) if V is not None else None, owner.ctypes.data,
                                C.byref(nm)), "orbt_fetch")
        return nm.value, owner[:n_kp], view


# ---- Optimizer::PoseOptimization (orbp_*) ----------------------------------------------------
class OrbpFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("Xw", C.c_void_p), ("obs", C.c_void_p), ("inv_sigma2", C.c_void_p),
                ("Tcw", C.c_float * 16), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float)]


class OrbpResult(C.Structure):
    _fields_ = [("Tcw", C.c_float * 16), ("outlier", C.c_void_p), ("n_inliers", C.c_int32),
                ("iterations", C.c_int32 * 4)]


def _orbp_frame(prob: dict):
    keep = {k: np.ascontiguousarray(prob[k], np.float32) for k in ("Xw", "obs", "inv_sigma2")}
    F = OrbpFrame()
    F.n = len(keep["Xw"])
    F.Xw, F.obs, F.inv_sigma2 = (keep[k].ctypes.data for k in ("Xw", "obs", "inv_sigma2"))
    F.Tcw[:] = [float(v) for v in np.asarray(prob["Tcw"], np.float32).reshape(-1)]
    F.fx, F.fy, F.cx, F.cy, F.bf = (float(v) for v in prob["cam"])
    return F, keep


class PoseOptimizer:
    """Optimizer::PoseOptimization (Optimizer.h:105) on the GPU: the whole 4-round
    Levenberg-Marquardt solve in one workgroup per frame. Problems are dicts shaped like
    synth.pose_problem: {"Xw", "obs", "inv_sigma2", "Tcw", "cam"}."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().orbp_create(C.byref(h)), "orbp_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _result(n):
        out = np.zeros(max(n, 1), np.uint8)
        R = OrbpResult()
        R.outlier = out.ctypes.data
        return R, out

    @staticmethod
    def _pack(R, out, n):
        return {"Tcw": np.array(R.Tcw[:], np.float32).reshape(4, 4), "outlier": out[:n].copy(),
                "n_inliers": R.n_inliers, "iterations": tuple(R.iterations)}

    def optimize(self, prob: dict) -> dict:
        F, keep = _orbp_frame(prob)
        R, out = self._result(F.n)
        _check(lib().orbp_pose_optimization(self._h, C.byref(F), C.byref(R)), "orbp_pose_optimization")
        return self._pack(R, out, F.n)

    def reserve(self, n_slots: int, cap_edges: int):
        _check(lib().orbp_reserve(self._h, n_slots, cap_edges), "orbp_reserve")

    def stage(self, slot: int, prob: dict):
        F, keep = _orbp_frame(prob)
        _check(lib().orbp_stage(self._h, slot, C.byref(F)), "orbp_stage")

    def run_batch(self, n_slots: int, stream=None):
        _check(lib().orbp_run_batch(self._h, n_slots, stream), "orbp_run_batch")

    def fetch(self, slot: int, n: int) -> dict:
        R, out = self._result(n)
        _check(lib().orbp_fetch(self._h, slot, C.byref(R)), "orbp_fetch")
        return self._pack(R, out, n)


# ---- DBoW2 vocabulary transform (orbv_*): Frame::ComputeBoW ---------------------------------
class Vocabulary:
    """ORBVocabulary (DBoW2 TemplatedVocabulary<FORB>) resident in HBM. Built from the arrays
    of synth.vocabulary or loaded from a DBoW2 text file (loadFromTextFile format).
    ``transform(desc, levelsup=4)`` = Frame::ComputeBoW -> (BowVector, FeatureVector)."""

    def __init__(self, voc: dict | None = None, path: str | None = None):
        h = C.c_void_p()
        if path is not None:
            _check(lib().orbv_load_text(str(path).encode(), C.byref(h)), "orbv_load_text")
        else:
            par = np.ascontiguousarray(voc["parent"], np.int32)
            leaf = np.ascontiguousarray(voc["is_leaf"], np.uint8)
            desc = np.ascontiguousarray(voc["desc"], np.uint8)
            w = np.ascontiguousarray(voc["weight"], np.float64)
            _check(lib().orbv_create(voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(par), par.ctypes.data,
                                     leaf.ctypes.data, desc.ctypes.data, w.ctypes.data, C.byref(h)), "orbv_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        vals = [C.c_int() for _ in range(4)]
        _check(lib().orbv_info(self._h, *[C.byref(v) for v in vals]), "orbv_info")
        return dict(zip(("n_nodes", "n_words", "k", "L"), (v.value for v in vals)))

    @staticmethod
    def _bufs(n):
        m = max(n, 1)
        return (np.zeros(m, np.uint32), np.zeros(m, np.float64), np.zeros(m, np.uint32), np.zeros(m + 1, np.int32),
                np.zeros(m, np.int32))

    @staticmethod
    def _pack(b, nw, nf):
        words, vals, fvn, fvs, fvf = b
        return {"words": words[:nw].copy(), "values": vals[:nw].copy(), "fv_nodes": fvn[:nf].copy(),
                "fv_start": fvs[: nf + 1].copy(), "fv_features": fvf[: fvs[nf]].copy()}

    def transform(self, desc: np.ndarray, levelsup: int = 4) -> dict:
        desc = np.ascontiguousarray(desc, np.uint8)
        n = len(desc)
        b = self._bufs(n)
        nw, nf = C.c_int32(), C.c_int32()
        _check(lib().orbv_transform(self._h, desc.ctypes.data if n else None, n, levelsup, *(x.ctypes.data for x in b[:2]),
                                    C.byref(nw), *(x.ctypes.data for x in b[2:]), C.byref(nf)), "orbv_transform")
        return self._pack(b, nw.value, nf.value)

    def transform_batch_device(self, d_desc: int, d_counts: int, n_frames: int, cap: int, frame_stride: int,
                               levelsup: int = 4, stream=None):
        _check(lib().orbv_transform_batch_device(self._h, C.c_void_p(d_desc), C.c_void_p(d_counts), n_frames, cap,
                                                 frame_stride, levelsup, stream), "orbv_transform_batch_device")

    def batch_fetch(self, frame: int, cap: int) -> dict:
        b = self._bufs(cap)
        nw, nf = C.c_int32(), C.c_int32()
        _check(lib().orbv_batch_fetch(self._h, frame, b[0].ctypes.data, b[1].ctypes.data, C.byref(nw),
                                      b[2].ctypes.data, b[3].ctypes.data, b[4].ctypes.data, C.byref(nf)),
               "orbv_batch_fetch")
        return self._pack(b, nw.value, nf.value)


# ---- BoW-guided matchers (orbb_*): SearchByBoW(KF, F) + SearchForTriangulation -------------
class OrbbKeyFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("u_right", C.c_void_p), ("desc", C.c_void_p),
                ("mp", C.c_void_p), ("mp_bad", C.c_void_p), ("n_fv", C.c_int32), ("fv_nodes", C.c_void_p),
                ("fv_start", C.c_void_p), ("fv_features", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("nlevels", C.c_int32), ("scale_factors", C.c_float * 16),
                ("level_sigma2", C.c_float * 16)]


def _orbb_keyframe(k: dict):
    keep = {"keys_un": np.ascontiguousarray(k["keys_un"]).view(KP_DTYPE),
            "u_right": np.ascontiguousarray(k["u_right"], np.float32), "desc": np.ascontiguousarray(k["desc"], np.uint8),
            "mp": np.ascontiguousarray(k["mp"], np.int32), "mp_bad": np.ascontiguousarray(k["mp_bad"], np.uint8),
            "fv_nodes": np.ascontiguousarray(k["fv_nodes"], np.uint32),
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


class BowMatcher:
    """ORBmatcher::SearchByBoW(KeyFrame*, Frame&) and SearchForTriangulation on the GPU.
    Problems are dicts shaped like synth.bow_match_problem: {"A", "B", "F12", "Cw1", "T2w"}."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().orbb_create(C.byref(h)), "orbb_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def search_by_bow(self, prob: dict, nnratio=0.7, check_ori=True):
        A, k1 = _orbb_keyframe(prob["A"])
        B, k2 = _orbb_keyframe(prob["B"])
        out = np.zeros(max(B.n, 1), np.int32)
        nm = C.c_int32()
        _check(lib().orbb_search_by_bow(self._h, C.byref(A), C.byref(B), nnratio, 1 if check_ori else 0,
                                        out.ctypes.data, C.byref(nm)), "orbb_search_by_bow")
        return nm.value, out[: B.n]

    def search_by_bow_kf(self, prob: dict, nnratio=0.75, check_ori=True):
        """SearchByBoW(KeyFrame* pKF1 = A, KeyFrame* pKF2 = B) -> (nmatches, matches12[A.n])."""
        A, k1 = _orbb_keyframe(prob["A"])
        B, k2 = _orbb_keyframe(prob["B"])
        out = np.zeros(max(A.n, 1), np.int32)
        nm = C.c_int32()
        _check(lib().orbb_search_by_bow_kf(self._h, C.byref(A), C.byref(B), nnratio, 1 if check_ori else 0,
                                           out.ctypes.data, C.byref(nm)), "orbb_search_by_bow_kf")
        return nm.value, out[: A.n]

    def run_bowkf_batch(self, n_slots: int, nnratio=0.75, check_ori=True, stream=None):
        _check(lib().orbb_run_bowkf_batch(self._h, n_slots, nnratio, 1 if check_ori else 0, stream),
               "orbb_run_bowkf_batch")

    def search_for_triangulation(self, prob: dict, only_stereo=False, check_ori=True):
        A, k1 = _orbb_keyframe(prob["A"])
        B, k2 = _orbb_keyframe(prob["B"])
        g = {k: np.ascontiguousarray(prob[k], np.float32) for k in ("F12", "Cw1", "T2w")}
        pairs = np.zeros((max(A.n, 1), 2), np.int32)
        n = C.c_int32()
        _check(lib().orbb_search_for_triangulation(self._h, C.byref(A), C.byref(B), g["F12"].ctypes.data,
                                                   g["Cw1"].ctypes.data, g["T2w"].ctypes.data, 1 if only_stereo else 0,
                                                   1 if check_ori else 0, pairs.ctypes.data, C.byref(n)),
               "orbb_search_for_triangulation")
        return pairs[: n.value].copy()

    def reserve(self, n_slots: int, cap_kp: int):
        _check(lib().orbb_reserve(self._h, n_slots, cap_kp), "orbb_reserve")

    def stage(self, slot: int, prob: dict):
        A, k1 = _orbb_keyframe(prob["A"])
        B, k2 = _orbb_keyframe(prob["B"])
        g = {k: np.ascontiguousarray(prob[k], np.float32) for k in ("F12", "Cw1", "T2w")}
        _check(lib().orbb_stage(self._h, slot, C.byref(A), C.byref(B), g["F12"].ctypes.data, g["Cw1"].ctypes.data,
                                g["T2w"].ctypes.data), "orbb_stage")

    def run_bow_batch(self, n_slots: int, nnratio=0.7, check_ori=True, stream=None):
        _check(lib().orbb_run_bow_batch(self._h, n_slots, nnratio, 1 if check_ori else 0, stream), "orbb_run_bow_batch")

    def run_tri_batch(self, n_slots: int, only_stereo=False, check_ori=True, stream=None):
        _check(lib().orbb_run_tri_batch(self._h, n_slots, 1 if only_stereo else 0, 1 if check_ori else 0, stream),
               "orbb_run_tri_batch")

    def fetch(self, slot: int, tri, n_out: int):
        """tri: False / 0 = SearchByBoW(KF, F) matches, True / 1 = triangulation pairs,
        2 = SearchByBoW(KF1, KF2) matches12."""
        mode = int(tri)
        out = np.zeros(max(2 * n_out, 1), np.int32)
        n = C.c_int32()
        _check(lib().orbb_fetch(self._h, slot, mode, out.ctypes.data, C.byref(n)), "orbb_fetch")
        if mode == 1:
            return out[: 2 * n.value].reshape(-1, 2).copy()
        return n.value, out[:n_out].copy()


# ---- new map points (orbn_*): the triangulation loop of LocalMapping::CreateNewMapPoints ----
class OrbnKeyFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys", C.c_void_p), ("keys_un", C.c_void_p), ("u_right", C.c_void_p),
                ("depth", C.c_void_p), ("Tcw", C.c_float * 12), ("Ow", C.c_float * 3), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("invfx", C.c_float), ("invfy", C.c_float),
                ("mb", C.c_float), ("mbf", C.c_float), ("nlevels", C.c_int32), ("scale_factors", C.c_float * 16),
                ("level_sigma2", C.c_float * 16)]


def orbn_keyframe(k: dict):
    """ctypes KeyFrame view of a synth.newpoints_problem keyframe dict (+ the arrays it points into)."""
    keep = {"keys": np.ascontiguousarray(k["keys"]).view(KP_DTYPE),
            "keys_un": np.ascontiguousarray(k["keys_un"]).view(KP_DTYPE),
            "u_right": np.ascontiguousarray(k["u_right"], np.float32),
            "depth": np.ascontiguousarray(k["depth"], np.float32)}
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


class NewMapPoints:
    """LocalMapping::CreateNewMapPoints' per-match triangulation on the GPU. Problems are dicts
    shaped like synth.newpoints_problem: {"kf1", "kf2", "pairs", "ratio_factor"}."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().orbn_create(C.byref(h)), "orbn_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbn_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def triangulate(self, prob: dict):
        A, k1 = orbn_keyframe(prob["kf1"])
        B, k2 = orbn_keyframe(prob["kf2"])
        pairs = np.ascontiguousarray(prob["pairs"], np.int32)
        n = len(pairs)
        x3d = np.zeros((max(n, 1), 3), np.float32)
        ok = np.zeros(max(n, 1), np.uint8)
        nnew = C.c_int32()
        _check(lib().orbn_triangulate(self._h, C.byref(A), C.byref(B), pairs.ctypes.data, n,
                                      float(prob["ratio_factor"]), x3d.ctypes.data, ok.ctypes.data, C.byref(nnew)),
               "orbn_triangulate")
        return nnew.value, x3d[:n], ok[:n]

    def reserve(self, n_slots: int, cap_kp: int, cap_pairs: int):
        _check(lib().orbn_reserve(self._h, n_slots, cap_kp, cap_pairs), "orbn_reserve")

    def stage(self, slot: int, prob: dict):
        A, k1 = orbn_keyframe(prob["kf1"])
        B, k2 = orbn_keyframe(prob["kf2"])
        pairs = np.ascontiguousarray(prob["pairs"], np.int32)
        _check(lib().orbn_stage(self._h, slot, C.byref(A), C.byref(B), pairs.ctypes.data, len(pairs),
                                float(prob["ratio_factor"])), "orbn_stage")

    def run_batch(self, n_slots: int, stream=None):
        _check(lib().orbn_run_batch(self._h, n_slots, stream), "orbn_run_batch")

    def fetch(self, slot: int, n_pairs: int):
        x3d = np.zeros((max(n_pairs, 1), 3), np.float32)
        ok = np.zeros(max(n_pairs, 1), np.uint8)
        nnew = C.c_int32()
        _check(lib().orbn_fetch(self._h, slot, x3d.ctypes.data, ok.ctypes.data, C.byref(nnew)), "orbn_fetch")
        return nnew.value, x3d[:n_pairs], ok[:n_pairs]
