"""Per-phase s_memtime counters of the eigensolver (C4 shape, N=512)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KORALI_AMD_TRACE_EIGEN"] = "1"
import numpy as np
from korali_amd.native import CmaesDevice

dev = CmaesDevice(512, 65536, initial_value=np.full(512, 2.0), initial_std=np.ones(512), normal_seed=1337,
                  uniform_seed=1338, cov_mode="mfma")
for g in range(1, 5):
    dev.generation(g, "ackley")
dev.synchronize()
