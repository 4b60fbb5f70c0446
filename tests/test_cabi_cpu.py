"""The C-ABI library loads without a GPU and exports every symbol include/orbslam2_amd.h
declares (no compute calls here)."""
import ctypes
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "orbslam2_amd.h"
LIB = ROOT / "orb-slam2-noted_amd" / "liborbslam2_amd.so"


def declared_symbols():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*([a-z_0-9]+)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n.startswith(("orbx_", "orbm_", "lba_", "orbslam2_amd_"))))


def test_header_declares_abi():
    syms = declared_symbols()
    for must in ("orbx_create", "orbx_extract", "orbx_extract_batch_device", "orbm_stereo_match",
                 "orbm_hamming_best2"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    if not LIB.exists():
        import __graft_entry__
        __graft_entry__.build()
    lib = ctypes.CDLL(str(LIB))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"not exported: {missing}"


def test_python_binding_covers_abi():
    import orbslam2_amd
    bound = {name for name, _, _ in orbslam2_amd.SIGNATURES}
    assert set(declared_symbols()) <= bound, set(declared_symbols()) - bound
