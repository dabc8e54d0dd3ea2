"""C1 through korali.Engine (device objective), 200 generations, for a
rocprofv3 kernel trace of the small-problem generation."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench


def main():
    import korali
    k = korali.Engine()
    e = bench.c1_experiment("kernel")
    e["Solver"]["Termination Criteria"]["Max Generations"] = 200
    k.run(e)
    print(e["Current Generation"], flush=True)


if __name__ == "__main__":
    main()
