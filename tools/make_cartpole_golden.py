"""Golden CartPole trajectories from the reference's own environment
(examples/learning/reinforcement/cartpole/_model/cartpole.py: numpy-seeded
reset, scipy `ode(...).set_integrator('dopri5')` advance), imported here from
/root/reference as a module.  Writes tests/golden/cartpole_dopri5.json:

  resets:       seed -> CartPole.reset(seed).u (the seeds env.py uses,
                sampleId * 1024 + launchId)
  trajectories: u0, the forces applied (some beyond the +-10 clip), and after
                every advance the state u, the isOver flag and the reward,
                until the pole falls or `steps` advances.

    python tools/make_cartpole_golden.py
"""
import importlib.util
import json
import os

import numpy as np

REF = "/root/reference/examples/learning/reinforcement/cartpole/_model/cartpole.py"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "cartpole_dopri5.json")


def load_cartpole():
    spec = importlib.util.spec_from_file_location("ref_cartpole", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CartPole


def main():
    CartPole = load_cartpole()
    cart = CartPole()
    seeds = [0, 1, 2, 1024, 1025, 3 * 1024 + 7, 123456789, 2**32 - 1]
    resets = []
    for s in seeds:
        cart.reset(s)
        resets.append({"seed": s, "u": [float(v) for v in cart.u]})
    rng = np.random.default_rng(20261017)
    trajectories = []
    for t in range(12):
        seed = t * 1024 + 3
        cart.reset(seed)
        u0 = [float(v) for v in cart.u]
        scale = [2.0, 6.0, 12.0, 25.0][t % 4]  # 25: the clip to +-10 is exercised
        steps = 60 if t < 8 else 200
        forces, states, over, rewards = [], [], [], []
        for k in range(steps):
            if t % 3:
                f = float(rng.uniform(-scale, scale))
            else:  # a balancing feedback (long trajectories; saturates at the clip)
                x, v, th, w = cart.u
                f = float(1.0 * x + 2.0 * v + 30.0 * th + 5.0 * w + rng.uniform(-0.5, 0.5))
            done = cart.advance([f])
            forces.append(f)
            states.append([float(v) for v in cart.u])
            over.append(int(done))
            rewards.append(float(cart.getReward()))
            if done:
                break
        trajectories.append({"seed": seed, "u0": u0, "force": forces, "u": states, "over": over, "reward": rewards})
    with open(OUT, "w") as f:
        json.dump({"source": "examples/learning/reinforcement/cartpole/_model/cartpole.py (scipy dopri5)",
                   "dt": 0.02, "resets": resets, "trajectories": trajectories}, f, indent=1)
    print(OUT, sum(len(t["u"]) for t in trajectories), "states")


if __name__ == "__main__":
    main()
