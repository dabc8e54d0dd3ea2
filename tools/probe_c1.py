"""C1 (N=8, lambda=16) through korali.Engine: wall time of runs of growing
length, device objective then the Python model (bench.py c1_line)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench


def main():
    import korali
    k = korali.Engine()
    for obj, gens in (("kernel", 10), ("kernel", 100), ("kernel", 1000), ("python", 10), ("python", 100),
                      ("python", 1000)):
        e = bench.c1_experiment(obj)
        e["Solver"]["Termination Criteria"]["Max Generations"] = gens
        t0 = time.perf_counter()
        k.run(e)
        print(obj, gens, f"{(time.perf_counter() - t0) * 1e3:.1f} ms", e["Current Generation"],
              e["Results"]["Best Sample"]["F(x)"], flush=True)


if __name__ == "__main__":
    main()
