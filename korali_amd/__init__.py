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
    /opt/rocm's (processes that never import torch)."""
    if _os.environ.get("KORALI_AMD_HIP_RUNTIME", "") == "system":
        return
    spec = _ilu.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for base in spec.submodule_search_locations:
        lib = _os.path.join(base, "lib", "libamdhip64.so")
        if _os.path.exists(lib):
            _ctypes.CDLL(lib, mode=_ctypes.RTLD_GLOBAL)
            return


_one_hip_runtime()
