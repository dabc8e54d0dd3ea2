"""CPU-side checks of the C-ABI boundary: the shared library builds for
gfx950, loads without a GPU, and exports exactly what include/*.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            syms |= set(re.findall(r"^\s*(?:const\s+char\s*\*|int)\s*(kg_\w+)\s*\(", src, re.M))
    return syms


@pytest.fixture(scope="module")
def lib():
    from korali_amd import _build
    _build.build()
    return ctypes.CDLL(_build.LIB)


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "kg_cmaes_generation" in syms and "kg_tmcmc_generation" in syms and "kg_last_error" in syms
    assert len(syms) >= 30


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in sorted(declared_symbols()) if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from korali_amd import native
    assert set(native.EXPORTED) == declared_symbols()


def test_abi_version(lib):
    lib.kg_abi_version.restype = ctypes.c_int
    assert lib.kg_abi_version() == 3


def test_code_object_targets_gfx950():
    from korali_amd import _build
    data = open(_build.LIB, "rb").read()
    assert b"gfx950" in data
