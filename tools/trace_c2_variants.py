"""k_tridiag_1wg experiment switches (KORALI_AMD_T1_FLAGS) on the C2 workload:
per variant, the eigen stage times (HIP events) and the s_memtime phase
counters, and a bit-identity check of B against variant 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KORALI_AMD_TRACE_EIGEN"] = "1"
import numpy as np
from korali_amd.native import CmaesDevice

variants = [int(a) for a in sys.argv[1:]] or [0, 1, 2, 5]
ref = None
for fl in variants:
    os.environ["KORALI_AMD_T1_FLAGS"] = str(fl)
    dev = CmaesDevice(128, 4096, initial_value=np.zeros(128), initial_std=np.ones(128), normal_seed=1337,
                      uniform_seed=1338, cov_mode="mfma")
    for g in range(1, 6):
        dev.generation(g, "rosenbrock")
    dev.synchronize()
    dev.profile(True)
    for st in ("eigen_tridiag", "eigen_unpack", "eigen_apply"):
        dev.profile_read(st)
    for g in range(6, 26):
        dev.generation(g, "rosenbrock")
    dev.synchronize()
    out = {st: round(dev.profile_read(st)[0] / 20, 4) for st in ("eigen_tridiag", "eigen_unpack", "eigen_apply")}
    B = dev["Covariance Matrix"].copy()
    same = None if ref is None else bool(np.array_equal(B, ref))
    if ref is None:
        ref = B
    print(f"flags={fl} {out} identical_to_first={same}", flush=True)
    dev.close()
