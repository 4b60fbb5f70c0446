"""Provenance stamp of a profiles/ summary: the hash of the library's sources (tools/src_hash.py),
checked against the built library's orbx_build_id() so a summary is never stamped with sources the
library was not built from, plus the commit (GIT_HEAD, passed in by the gpurun command line: the
GPU box has no .git) and the configuration the counters belong to."""
import ctypes
import os
from pathlib import Path

from src_hash import src_hash

LIB = Path(__file__).resolve().parent.parent / "orb-slam2-noted_amd" / "liborbslam2_amd.so"


def stamp(**config) -> dict:
    """The library checked is the one the profiled run loaded: ORBSLAM_AMD_LIB when set (the Python
    binding's override), else the product build. Its build id must be the bare source hash: a
    variant or EXTRA-flag build carries a suffix (Makefile) and is refused."""
    h = src_hash()
    built = ctypes.CDLL(os.environ.get("ORBSLAM_AMD_LIB") or str(LIB))
    built.orbx_build_id.restype = ctypes.c_char_p
    lib_id = built.orbx_build_id().decode()
    if lib_id != h:
        raise SystemExit(f"library build id {lib_id}, tree is {h}: profile a product build of this tree")
    st = {"src_hash": h, "commit": os.environ.get("GIT_HEAD", "unknown"),
          "resize_mode": int(os.environ.get("RESIZE_MODE", "0")),
          "blur_mode": int(os.environ.get("BLUR_MODE", "0"))}
    st.update(config)
    return st
