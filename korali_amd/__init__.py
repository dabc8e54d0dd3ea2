"""korali_amd — MI355X-native engine for Korali's population-based solver
generation loop (CMA-ES, TMCMC).  See DESIGN.md."""
import ctypes as _ctypes
import importlib.util as _ilu
import os as _os

__version__ = "0.1.0"


def _one_hip_runtime():
    """Bind this package's libraries to the HIP runtime PyTorch ships.

    libkorali_amd.so needs ``libamdhip64.so.7``; torch's HIP libraries need
    ``libamdhip64.so`` from their own directory.  Loaded in the order
    ``import korali`` then ``import torch``, the process maps TWO HIP runtimes
    and two HSA runtimes (/opt/rocm's and torch's), each with its own view of
    the device; the occupancy query of the first then answered 0 blocks per
    CU for the multi-workgroup tridiagonalisation (round 3's "occupancy
    anomaly", seen only in a pytest process that had imported every test
    module).  Loading torch's runtime first (by file, RTLD_GLOBAL, without
    importing torch) makes our ``libamdhip64.so.7`` dependency resolve to it,
    and torch later finds the same file already mapped: one runtime per
    process, whatever the import order.  KORALI_AMD_HIP_RUNTIME=system keeps
    /opt/rocm's (processes that never import torch).

    A process in which an HSA runtime is ALREADY mapped keeps that one's HIP:
    under rocprofv3 the profiler's preloaded tool maps /opt/rocm's
    libhsa-runtime64.so.1 before Python starts, and loading torch's HIP on top
    (whose HSA calls then bind to /opt/rocm's HSA while torch's own HSA is
    mapped too) made every profiled process that had made a cooperative launch
    fault in the HIP runtime's exit handler (profiles/r5/c4_teardown_segv.txt).
    Our libamdhip64.so.7 dependency then resolves to /opt/rocm's HIP over the
    HSA already there: one HIP + HSA pair (tests/test_one_runtime.py)."""
    if _os.environ.get("KORALI_AMD_HIP_RUNTIME", "") == "system":
        return
    spec = _ilu.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    try:
        with open("/proc/self/maps") as f:
            mapped = [l.split()[-1] for l in f if "libhsa-runtime64" in l]
    except OSError:
        mapped = []
    torch_dirs = [_os.path.realpath(_os.path.join(b, "lib")) for b in spec.submodule_search_locations]
    if any(not any(_os.path.realpath(m).startswith(d + _os.sep) for d in torch_dirs) for m in mapped):
        return  # a system HSA runtime is already mapped (a profiler's tool): keep its HIP
    for base in spec.submodule_search_locations:
        lib = _os.path.join(base, "lib", "libamdhip64.so")
        if _os.path.exists(lib):
            _ctypes.CDLL(lib, mode=_ctypes.RTLD_GLOBAL)
            return


_one_hip_runtime()
