"""Time the host core's tridiagonalisation (kg_debug_host_tridiag) at the
C2 / C4 orders for each instruction-set body, one process per ISA (the ISA
is picked once per process).  Usage: python tools/time_host_tridiag.py [isa]"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(isa):
    from korali_amd.native import lib
    L = lib()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    out = {}
    for N, reps in ((128, 400), (512, 12)):
        rng = np.random.default_rng(N)
        Y = rng.standard_normal((N, 2 * N))
        C = np.ascontiguousarray(Y @ Y.T / (2 * N))
        H = np.zeros((N, N))
        tau, d, sd = np.zeros(N), np.zeros(N), np.zeros(N)
        for _ in range(3):
            L.kg_debug_host_tridiag(N, vp(C), vp(H), vp(tau), vp(d), vp(sd))
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            L.kg_debug_host_tridiag(N, vp(C), vp(H), vp(tau), vp(d), vp(sd))
            ts.append(time.perf_counter() - t0)
        out[N] = (1e6 * float(np.median(ts)), 1e6 * float(np.min(ts)))
    print(f"{isa}: " + ", ".join(f"N={N} median {m:.1f} us min {mn:.1f} us" for N, (m, mn) in out.items()), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        cpu = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][:1]
        print("cpu:", cpu, flush=True)
        for isa in ("avx512", "avx2", "sse2"):
            env = dict(os.environ, KORALI_AMD_HOST_TRIDIAG_ISA=isa)
            subprocess.run(["taskset", "-c", str(min(os.sched_getaffinity(0))), sys.executable, __file__, isa],
                           env=env, check=True)
