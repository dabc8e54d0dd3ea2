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
    assert lib.kg_abi_version() == 8


def test_code_object_targets_gfx950():
    from korali_amd import _build
    data = open(_build.LIB, "rb").read()
    assert b"gfx950" in data


def test_code_object_has_no_sdwa_or_indexed_register_forms(lib, tmp_path):
    """No VGPR-indexing mode anywhere: a runtime-indexed private-array write
    inside a longer loop (round 2's CartPole reset, `if (i <= 8) lo[i] = x`
    for i < 405) was if-converted into an unconditional indexed register write
    v[base + i] far past the array, which memory-faulted on MI355X; every
    private-array index is now a compile-time constant.  And no SDWA forms:
    the library builds without any -amdgpu-sdwa-peephole switch."""
    import shutil
    import subprocess
    llvm = "/opt/rocm/lib/llvm/bin"
    if not (shutil.which("objcopy") and os.path.exists(f"{llvm}/clang-offload-bundler")):
        pytest.skip("objcopy / clang-offload-bundler not available")
    fat, co = tmp_path / "fat.bin", tmp_path / "co.o"
    from korali_amd import _build
    subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", _build.LIB, str(fat)])
    subprocess.check_call([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    dis = subprocess.run([f"{llvm}/llvm-objdump", "-d", "--mcpu=gfx950", str(co)], check=True,
                         capture_output=True, text=True).stdout
    assert "v_add_f64" in dis
    assert not re.search(r"\bv_\w+_sdwa\b", dis)
    assert not re.search(r"\bs_set_gpr_idx_on\b|\bv_movrel\w*\b", dis)
