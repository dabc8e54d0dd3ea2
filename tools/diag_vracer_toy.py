"""Diagnostic: the multi-action host-environment toy of
tests/test_gpu_vracer_host_env.py, printing where non-finite actions appear.

    python tools/diag_vracer_toy.py [start_size] [distribution]
"""
import sys

import numpy as np

sys.path.insert(0, "tests")
import korali  # noqa: E402

step = [0]


def env(s):
    rs = np.random.RandomState(s["Sample Id"])
    x = rs.uniform(-1, 1, 3)
    s["State"] = x.tolist()
    for _ in range(12):
        s.update()
        a = np.array(s["Action"])
        step[0] += 1
        if not np.all(np.isfinite(a)):
            print("non-finite action at env step", step[0], "sample", s["Sample Id"], a, flush=True)
            a = np.zeros(2)
        s["Reward"] = -float(np.sum((a - x[:2]) ** 2))
        x = rs.uniform(-1, 1, 3)
        s["State"] = x.tolist()
    s["Termination"] = "Truncated"


def main():
    start = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    dist = sys.argv[2] if len(sys.argv) > 2 else "Clipped Normal"
    e = korali.Experiment()
    e["Problem"]["Type"] = "Reinforcement Learning / Continuous"
    e["Problem"]["Environment Function"] = env
    for i in range(3):
        e["Variables"][i]["Name"] = f"x{i}"
        e["Variables"][i]["Type"] = "State"
    for i in range(2):
        v = e["Variables"][3 + i]
        v["Name"], v["Type"] = f"a{i}", "Action"
        v["Lower Bound"], v["Upper Bound"], v["Initial Exploration Noise"] = -1.0, 1.0, 0.5
    sv = e["Solver"]
    sv["Type"] = "Agent / Continuous / VRACER"
    sv["Experiences Between Policy Updates"] = 1
    sv["Episodes Per Generation"] = 4
    sv["Concurrent Environments"] = 2
    sv["Experience Replay"]["Start Size"] = start
    sv["Experience Replay"]["Maximum Size"] = 4096
    sv["Learning Rate"] = 1e-3
    sv["Mini Batch"]["Size"] = 32
    sv["Policy"]["Distribution"] = dist
    for j in range(2):
        sv["Neural Network"]["Hidden Layers"][2 * j]["Type"] = "Layer/Linear"
        sv["Neural Network"]["Hidden Layers"][2 * j]["Output Channels"] = 32
        sv["Neural Network"]["Hidden Layers"][2 * j + 1]["Type"] = "Layer/Activation"
        sv["Neural Network"]["Hidden Layers"][2 * j + 1]["Function"] = "Elementwise/Tanh"
    sv["Termination Criteria"]["Max Generations"] = 10
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    korali.Engine().run(e)
    print("episodes", sv["Current Episode"], "experiences", sv["Experience Count"], "updates",
          sv["Policy Update Count"])
    pol = np.array(sv["Training"]["Current Policy"]["Policy"])
    print("policy finite", np.all(np.isfinite(pol)), "rewards", np.array(sv["Training"]["Reward History"])[:8])


if __name__ == "__main__":
    main()
