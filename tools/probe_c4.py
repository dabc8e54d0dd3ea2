"""C4 single-GPU probe: stage times of CMA-ES N=512, lambda=65536, Ackley."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from korali_amd.native import CmaesDevice

N, L = int(sys.argv[1]) if len(sys.argv) > 1 else 512, int(sys.argv[2]) if len(sys.argv) > 2 else 65536
gens = int(sys.argv[3]) if len(sys.argv) > 3 else 4
cov = sys.argv[4] if len(sys.argv) > 4 else "mfma"
dev = CmaesDevice(N, L, initial_value=np.full(N, 2.0), initial_std=np.ones(N), normal_seed=1337, uniform_seed=1338,
                  cov_mode=cov)
t0 = time.perf_counter()
dev.generation(1, "ackley"); dev.synchronize()
print("gen1 %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
t0 = time.perf_counter()
for g in range(2, 2 + gens):
    dev.generation(g, "ackley")
dev.synchronize()
print("gens/s %.2f  ms/gen %.2f" % (gens / (time.perf_counter() - t0), (time.perf_counter() - t0) / gens * 1e3), flush=True)
dev.profile(True)
STAGES = ("eigen", "eigen_tridiag", "eigen_unpack", "eigen_dsd_wait", "eigen_chase_host", "eigen_apply", "rng_polar", "transform",
          "rng_consume", "objective", "sort", "mean_paths", "covariance", "sigma")
for st in ("init",) + STAGES:
    dev.profile_read(st)
g0 = 2 + gens
for g in range(g0, g0 + 2):
    dev.generation(g, "ackley")
dev.synchronize()
for st in STAGES:
    ms, n = dev.profile_read(st)
    if n:
        print("%-18s %8.3f ms" % (st, ms / n))
print("best", dev["Best Ever Value"][0])
