"""korali — the Korali Python API (reference: python/korali/__init__.py, which
re-exports the pybind11 module `libkorali`) served by the MI355X-native
engine: korali_amd/engine (C++ Engine / Experiment / Sample) over the
korali_amd C-ABI (HIP kernels, gfx950).

    import korali
    k = korali.Engine()
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Function"] = model      # or "Objective Kernel": "Negative Rosenbrock"
    e["Variables"][0]["Name"] = "X"
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 32
    k.run(e)

There is no CPU fallback: the native modules must be built
(`python -m korali_amd._build`).
"""
import os as _os
import sys as _sys

_root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _root not in _sys.path:
    _sys.path.insert(0, _root)

try:
    from korali_amd.libkorali import Engine, Experiment, KoraliError, Sample, koraliJson  # noqa: F401
    # timing hook of this engine (not a reference API): the last run's
    # generation completion marks, kept out of the experiment's JSON
    from korali_amd.libkorali import _generation_completion_times  # noqa: F401
except ImportError as _e:  # pragma: no cover
    raise ImportError(f"korali: the native engine is not built ({_e}); run `python -m korali_amd._build`") from _e

__all__ = ["Engine", "Experiment", "Sample", "KoraliError", "koraliJson"]
