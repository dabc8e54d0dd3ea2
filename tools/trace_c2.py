"""Per-phase s_memtime counters of the tridiagonalisation (C2 workload)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KORALI_AMD_TRACE_EIGEN"] = "1"
import numpy as np
from korali_amd.native import CmaesDevice

dev = CmaesDevice(128, 4096, initial_value=np.zeros(128), initial_std=np.ones(128), normal_seed=1337,
                  uniform_seed=1338, cov_mode="mfma")
for g in range(1, 11):
    dev.generation(g, "rosenbrock")
dev.synchronize()
