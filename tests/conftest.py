"""Test configuration: registers the `gpu` marker and makes the in-tree packages importable.

`-m "not gpu"` runs here (no GPU): oracle pins, golden fixtures, host logic and the C-ABI
symbol check. `-m gpu` runs on an MI355X and compares the HIP path (through the C-ABI)
with the CPU oracle.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam2-noted_amd" / "python"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and liborbslam2_amd.so")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def amd():
    import orbslam2_amd
    if orbslam2_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests must run on the MI355X box")
    return orbslam2_amd
