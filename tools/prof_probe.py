"""A few C2-shaped CMA-ES generations through the C-ABI (rocprofv3 teardown
probe: tools/../scripts/diag_prof.sh)."""
import numpy as np

from korali_amd.native import CmaesDevice

N, lam = 128, 4096
d = CmaesDevice(N, lam, initial_value=np.zeros(N), initial_std=np.ones(N), normal_seed=1337, uniform_seed=1338)
for g in range(1, 4):
    d.generation(g, "negative rosenbrock")
d.synchronize()
print("best", d["Best Ever Value"][0], flush=True)
d.close()
