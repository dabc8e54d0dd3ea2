import os, sys
sys.path.insert(0, os.getcwd())
os.environ["KORALI_AMD_TRACE_TMCMC"] = "1"
import bench
dev = bench.c3_experiment(1337)
for g in range(1, 6):
    dev.generation(g)
dev.synchronize()
dev.close()
