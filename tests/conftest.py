import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_sessionstart(session):
    """Build the in-tree native libraries if a fresh checkout lacks them
    (hipcc cross-compiles gfx950 without a GPU; g++ for the engine/oracle)."""
    from korali_amd import _build
    if not (os.path.exists(_build.LIB) and os.path.exists(_build.PYMOD) and os.path.exists(_build.ENGINE_LIB)):
        _build.build()
    if not os.path.exists(os.path.join(ROOT, "oracle", "librefcpu.so")):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
