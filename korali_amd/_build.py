"""Build the in-tree native libraries (no JIT cache, nothing installed).

  korali_amd/libkorali_amd.so   HIP kernels + C-ABI (include/korali_amd.h),
                                gfx950 code objects, hipcc
"""
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libkorali_amd.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KORALI_AMD_ARCH", "gfx950")
# -ffp-contract=off: no implicit FMA anywhere (bit-faithful replay of the
# reference's x86-64 SSE2 double arithmetic); explicit fma() is kept.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}",
         "-Wno-unused-result"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp")))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    deps = sources() + [os.path.join(ROOT, "include", "korali_amd.h")]
    if force or _stale(LIB, deps):
        cmd = [HIPCC] + FLAGS + ["-o", LIB, os.path.join(CSRC, "korali_amd.hip")]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    build(force=True, verbose=True)
