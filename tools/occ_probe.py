"""Which CMA-ES handle configurations at the C4 shape can create their
eigensolver (co-residency of the multi-workgroup tridiagonalisation)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KORALI_AMD_DEBUG_OCC"] = "1"
if "torch" in sys.argv:  # torch's bundled HIP runtime loaded first (as in the pytest process)
    import torch  # noqa: F401
import numpy as np
from korali_amd.native import CmaesDevice

mode = sys.argv[1]
lam = 65536
try:
    dev = CmaesDevice(512, lam, initial_value=np.full(512, 2.0), initial_std=np.ones(512), normal_seed=1337,
                      uniform_seed=1338, cov_mode=mode)
    dev.generation(1, "ackley")
    dev.synchronize()
    print(mode, lam, "ok", flush=True)
    dev.close()
except Exception as e:
    print(mode, lam, "FAILED", e, flush=True)
