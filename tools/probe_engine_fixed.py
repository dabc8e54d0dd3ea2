"""Fixed cost of a korali.Engine run at the C2 shape: handle creation,
initialisation and the first generation, against the steady per-generation
time (bench.py's engine_end_to_end line).  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import bench
from korali_amd.native import CmaesDevice


def main():
    import korali
    out = {}
    # the C-ABI: create / initialise / first generations
    for rep in range(3):
        t0 = time.perf_counter()
        d = CmaesDevice(128, 4096, initial_value=np.zeros(128), initial_std=np.ones(128), normal_seed=1337 + rep,
                        uniform_seed=1338 + rep, cov_mode="exact")
        d.synchronize()
        t1 = time.perf_counter()
        d.generation(1, "rosenbrock")
        d.synchronize()
        t2 = time.perf_counter()
        for g in range(2, 12):
            d.generation(g, "rosenbrock")
        d.synchronize()
        t3 = time.perf_counter()
        d.close()
        t4 = time.perf_counter()
        out[f"capi_rep{rep}"] = {"create_ms": (t1 - t0) * 1e3, "gen1_ms": (t2 - t1) * 1e3,
                                 "gen_ms": (t3 - t2) * 1e3 / 10, "close_ms": (t4 - t3) * 1e3}
    k = korali.Engine()
    for n in (1, 1, 21, 21):
        e = bench.c2_experiment("exact", n)
        t0 = time.perf_counter()
        k.run(e)
        out.setdefault("engine_run_ms", []).append([n, (time.perf_counter() - t0) * 1e3])
        marks = korali._generation_completion_times(e)
        out.setdefault("engine_marks_ms", []).append([round(m * 1e3, 3) for m in marks[:3]] + [round(marks[-1] * 1e3, 3)])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
