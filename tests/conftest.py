"""pytest configuration: markers, import paths, and on-demand native builds.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, and
the C-ABI library's exports.  `-m gpu` runs on an MI355X through gpurun: the
parity tests proper, calling the HIP kernels through the C ABI.
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "whisper-burn_amd")
for p in (REPO, PKG, os.path.join(PKG, "tools"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu through gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built() -> None:
    """Build oracle/ (gcc) and libwq4.so (hipcc, cross-compiles without a GPU)
    if a fresh checkout lacks them.  On the GPU box the prebuilt .so files
    travel with the snapshot and this is a no-op."""
    if not os.path.exists(os.path.join(REPO, "oracle", "build", "libq4oracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    if not os.path.exists(os.path.join(PKG, "lib", "libwq4.so")):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    return np.load(os.path.join(REPO, "tests", "golden", "q4_golden.npz"))
