"""Every preprocessor switch left in the product sources (orb-slam2-noted_amd/csrc) selects an
instrumented build of the shipped code -- a profile printout, a bounds trap, an experiment that
compiles one part of fast_blur_kernel out -- never an alternative algorithm (the
measured-and-rejected variants live in tools/archive/pruned_r06.patch). This test compiles each
instrumented configuration for gfx950 on the CPU, so none of them rots unseen, and checks that no
other switch has crept back in. (CPU only: nothing is run.)"""
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "orb-slam2-noted_amd"
HIPCC = "/opt/rocm/bin/hipcc"

# (source, defines): the instrumented builds tools/ use (make variant VDEFS=...)
VARIANTS = [
    ("orb_extract.hip", ["-DORBX_BOUNDS_CHECK=1", "-DORBX_QT_PROFILE", "-DORBX_EXPERIMENTS=1"]),
    ("orb_extract.hip", ["-DFB_SKIP_PRE", "-DFB_SKIP_BLUR", "-DFB_SKIP_EXACT"]),
    ("lba.hip", ["-DLBA_PROFILE"]),
    ("orb_pose.hip", ["-DORBP_PROFILE"]),
]
# every switch the product sources may test, and what it is
ALLOWED = {
    "ORBX_BOUNDS_CHECK": "trap on an LDS list overflow (debug build)",
    "ORBX_QT_PROFILE": "quadtree phase timestamps (printf)",
    "FB_SKIP_PRE": "fast_blur VALU split (tools/gpu_fb_parts.sh)",
    "FB_SKIP_BLUR": "fast_blur VALU split",
    "FB_SKIP_EXACT": "fast_blur VALU split",
    "LBA_PROFILE": "LocalBA Cholesky phase timestamps (printf)",
    "ORBP_PROFILE": "PoseOptimization phase timestamps",
    "ORBX_EXPERIMENTS": "environment-read experiment knobs (make variant builds only)",
    "ORBX_BUILD_SUFFIX": "build id suffix of a non-product build",
    "ORB_LIBM_RESTATE_H": "include guard",
    "__HIPCC__": "libm_restate.h shared with the C oracle tools",
}


def test_no_unlisted_switch():
    pat = re.compile(r"^\s*#\s*(?:if|ifdef|ifndef|elif)\b(.*)$")
    found = {}
    for f in sorted((PKG / "csrc").glob("*")):
        if f.suffix not in (".hip", ".h", ".inc"):
            continue
        for n, line in enumerate(f.read_text().splitlines(), 1):
            m = pat.match(line)
            if m:
                for name in re.findall(r"[A-Za-z_][A-Za-z0-9_]*", m.group(1).split("//")[0]):
                    if name != "defined":
                        found.setdefault(name, []).append(f"{f.name}:{n}")
    extra = {k: v for k, v in found.items() if k not in ALLOWED}
    assert not extra, f"switches outside the instrumented set: {extra}"


@pytest.mark.skipif(shutil.which(HIPCC) is None, reason="hipcc not installed")
def test_instrumented_builds_compile(tmp_path):
    def build(i):
        src, defs = VARIANTS[i]
        cmd = [HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-ffp-contract=off",
               f"-I{ROOT / 'include'}", f"-I{PKG / 'csrc'}", f"-I{PKG / 'build'}", "-mllvm",
               "-amdgpu-mfma-vgpr-form=1", *defs, "-c", str(PKG / "csrc" / src), "-o", str(tmp_path / f"v{i}.o")]
        r = subprocess.run(cmd, capture_output=True, text=True)
        return src, defs, r.returncode, r.stderr[-2000:]
    with ThreadPoolExecutor(4) as ex:
        for src, defs, rc, err in ex.map(build, range(len(VARIANTS))):
            assert rc == 0, f"{src} {defs}:\n{err}"
