"""First generation of a discrete-variable CMA-ES on the device and in the
oracle: where the populations differ (debugging aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np
import refcpu as R
from korali_amd.native import CmaesDevice

for use_gran in (0, 1):
    Nv, lam, seed = 10, 8, 1701
    gran = np.zeros(Nv)
    if use_gran:
        gran[[0, 1, 3, 6]] = 1.0
    lb, ub = np.full(Nv, -19.0), np.full(Nv, 21.0)
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"] = np.ones(Nv)
    o["Initial Standard Deviation"] = (ub - lb) * 0.3
    o["Lower Bound"], o["Upper Bound"], o["Granularity"] = lb, ub, gran
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = CmaesDevice(Nv, lam, initial_value=np.ones(Nv), initial_std=(ub - lb) * 0.3, lower_bound=lb, upper_bound=ub,
                      granularity=gran, normal_seed=seed, uniform_seed=seed + 1)
    for g in (1, 2, 3):
        o.generation(g, "sphere")
        dev.generation(g, "sphere")
        dev.synchronize()
        X, Y = dev["Sample Population"].reshape(lam, Nv), o["Sample Population"].reshape(lam, Nv)
        bad = np.argwhere(X != Y)
        print("gran", use_gran, "gen", g, "mismatches", len(bad), "infeasible dev/oracle",
              dev["Infeasible Sample Count"][0], o["Infeasible Sample Count"][0], flush=True)
        for r, c in bad[:6]:
            print("   row", r, "col", c, repr(X[r, c]), repr(Y[r, c]), flush=True)
        if len(bad):
            print("   dev row", X[bad[0][0]], "\n   orc row", Y[bad[0][0]], flush=True)
            break
    dev.close()
