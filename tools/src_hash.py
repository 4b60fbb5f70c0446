#!/usr/bin/env python3
"""Hash of the sources liborbslam2_amd.so is built from (provenance stamp).

The Makefile bakes it into the library (orbx_build_id(), orb_pipeline.hip); the PMC summaries
under profiles/ carry the hash of the library they were measured on, and bench.py reports a
committed counter figure only when the two agree (VERDICT r2 "next" item 1).
Hashed: csrc/*.hip, csrc/*.h, csrc/*.inc, include/orbslam2_amd.h and the library Makefile, in
sorted order, each as its repo-relative path, a NUL, its bytes, a NUL. 16 hex digits of SHA-256.
"""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "orb-slam2-noted_amd"


def source_files():
    files = []
    for pat in ("*.hip", "*.h", "*.inc"):
        files += (PKG / "csrc").glob(pat)
    files += [ROOT / "include" / "orbslam2_amd.h", PKG / "Makefile"]
    return sorted(files, key=lambda p: p.relative_to(ROOT).as_posix())


def src_hash() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(f.relative_to(ROOT).as_posix().encode() + b"\0")
        h.update(f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(src_hash() + "\n")
