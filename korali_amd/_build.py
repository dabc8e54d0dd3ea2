"""Build the in-tree native libraries (no JIT cache, nothing installed).

  korali_amd/libkorali_amd.so      HIP kernels + C-ABI (include/korali_amd.h),
                                   gfx950 code objects, hipcc
  korali_amd/libkorali_engine.so   C++ korali::Engine / Experiment / Sample
                                   (korali_amd/engine/korali.hpp) on the C-ABI
  korali_amd/libkorali*.so         the `libkorali` Python module (pybind11)
"""
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libkorali_amd.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KORALI_AMD_ARCH", "gfx950")
# -ffp-contract=off: no implicit FMA anywhere (bit-faithful replay of the
# reference's x86-64 SSE2 double arithmetic); explicit fma() is kept.
# (No SDWA flag: the two places the SDWA peephole used to fire — the
# CartPole reset's tempering and k_vr_meta's byte flags, kg_vracer.hip — keep
# their values opaque to it locally; tests/test_abi.py checks that the code
# object holds no SDWA instruction.)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}",
         "-Wno-unused-result"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".cpp", ".inc")))


# host-core code of the library (the GSL-order tridiagonalisation,
# kg_host_tridiag.cpp): g++, no FMA, one body per instruction set
HOST_SRC = os.path.join(CSRC, "kg_host_tridiag.cpp")
HOST_OBJ = os.path.join(CSRC, "kg_host_tridiag.o")
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-ffp-contract=off", "-fno-math-errno", "-Wall", "-Wno-psabi"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


ENGINE = os.path.join(PKG, "engine")
ENGINE_LIB = os.path.join(PKG, "libkorali_engine.so")
PYMOD = os.path.join(PKG, "libkorali" + sysconfig.get_config_var("EXT_SUFFIX"))
CXX = os.environ.get("CXX", "g++")
CXXFLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-result"]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)


def build(force=False, verbose=False):
    deps = sources() + [os.path.join(ROOT, "include", "korali_amd.h")]
    if force or _stale(LIB, deps):
        _run(["g++"] + HOST_FLAGS + ["-c", "-o", HOST_OBJ, HOST_SRC], verbose)
        _run([HIPCC] + FLAGS + ["-o", LIB, os.path.join(CSRC, "korali_amd.hip"), "-Wl," + HOST_OBJ, "-pthread"], verbose)
    build_engine(force, verbose)
    return LIB


def build_engine(force=False, verbose=False):
    srcs = [os.path.join(ENGINE, f) for f in ("json.cpp", "engine.cpp", "likelihood.cpp", "distributed.cpp")]
    hdrs = [os.path.join(ENGINE, f) for f in ("json.hpp", "korali.hpp", "distributed.hpp")] + [os.path.join(ROOT, "include", "korali_amd.h")]
    link = ["-L" + PKG, "-lkorali_amd", "-Wl,-rpath,$ORIGIN", "-ldl"]  # -ldl: librccl is opened at run time
    if force or _stale(ENGINE_LIB, srcs + hdrs + [LIB]):
        _run([CXX] + CXXFLAGS + ["-o", ENGINE_LIB] + srcs + link, verbose)
    pysrc = os.path.join(ENGINE, "pybind.cpp")
    if force or _stale(PYMOD, srcs + hdrs + [pysrc, LIB]):
        import pybind11
        inc = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]
        _run([CXX] + CXXFLAGS + ["-fvisibility=hidden"] + inc + ["-o", PYMOD, pysrc] + srcs + link, verbose)
    build_cxx_example(force, verbose)
    return PYMOD


# a C++ problem definition in the reference's own idioms, linked against the
# engine (tests/test_cxx_api.py runs it)
CXX_EXAMPLE_SRC = os.path.join(ROOT, "tests", "cxx", "reference_idioms.cpp")
CXX_EXAMPLE = os.path.join(ROOT, "tests", "cxx", "reference_idioms")


def build_cxx_example(force=False, verbose=False):
    hdrs = [os.path.join(ENGINE, f) for f in ("json.hpp", "korali.hpp")]
    if os.path.exists(CXX_EXAMPLE_SRC) and (force or _stale(CXX_EXAMPLE, [CXX_EXAMPLE_SRC, ENGINE_LIB] + hdrs)):
        _run([CXX, "-O1", "-std=c++17", "-I" + ENGINE, "-o", CXX_EXAMPLE, CXX_EXAMPLE_SRC, "-L" + PKG,
              "-lkorali_engine", "-Wl,-rpath," + PKG], verbose)
    return CXX_EXAMPLE


if __name__ == "__main__":
    build(force=True, verbose=True)
