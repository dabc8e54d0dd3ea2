"""A few C3-shaped TMCMC generations through the C-ABI (rocprofv3 teardown probe)."""
import numpy as np

from korali_amd.native import TmcmcDevice

N, P = 4, 10000
d = TmcmcDevice(N, P, prior_min=np.full(N, -10.0), prior_max=np.full(N, 10.0), max_chain_length=1)
for g in range(1, 4):
    d.generation(g)
d.synchronize()
print("exponent", d["Annealing Exponent"][0], flush=True)
d.close()
