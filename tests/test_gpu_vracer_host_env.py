"""VRACER with a host 'Environment Function' (the reference's own interface:
examples/learning/reinforcement/cartpole/run-vracer.py sets
e["Problem"]["Environment Function"] = env).  The engine runs each concurrent
environment's function as a coroutine (reinforcementLearning.cpp.base:66-88,
:90-209, :332-393); the device keeps the policy, the episode buffers and the
replay memory (kg_vracer_host_launch / _act / _feed).

Parity: an environment function whose dynamics are the device CartPole's
(kg_debug_cartpole_at, one step at a time) and whose resets, environment ids
and rewards are env.py's must train exactly like the CartPole kernel: same
reward history, same policy, bit for bit.  The reference's own environment
(scipy dopri5) runs run-vracer.py's configuration unchanged."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

vp = ctypes.c_void_p


def device_advance(u, t, force):
    """one CartPole step on the device's dynamics (cp_advance)"""
    from korali_amd import native
    u0 = np.ascontiguousarray(u, np.float64)
    t0 = np.array([t], np.float64)
    f = np.array([force], np.float64)
    out = np.zeros(4)
    t1 = np.zeros(1)
    over = np.zeros(1, np.int32)
    L = native.lib()
    assert L.kg_debug_cartpole_at(0, u0.ctypes.data_as(vp), t0.ctypes.data_as(vp), f.ctypes.data_as(vp), 1, 1,
                                  out.ctypes.data_as(vp), t1.ctypes.data_as(vp), over.ctypes.data_as(vp)) == 0
    assert over[0] >= 0
    return out, float(t1[0]), bool(over[0])


def device_cartpole_env(s):
    """env.py's episode (numpy-seeded reset with Sample Id * 1024 + Launch Id,
    environment id = Sample Id % 3 in training, the three reward variants,
    500 steps at most) on the device's CartPole dynamics"""
    sid, lid = s["Sample Id"], s["Launch Id"]
    env_id = sid % 3 if s["Mode"] == "Training" else 0
    u = np.random.RandomState(sid * 1024 + lid).uniform(-0.05, 0.05, 4)
    t = 0.0
    s["Environment Id"] = env_id
    s["State"] = u.tolist()
    step, over = 0, False
    while not over and step < 500:
        s.update()
        u, t, over = device_advance(u, t, s["Action"][0])
        r = 1.0 - 1.0 * over
        s["Reward"] = r if env_id == 0 else (r - 1 if env_id == 1 else r * 0.1)
        s["State"] = u.tolist()
        step += 1
    s["Termination"] = "Terminal" if over else "Truncated"


class ScipyCartPole:
    """The reference example's CartPole (cartpole.py: scipy's dopri5 from t to
    t + 0.02 per action, force clipped to [-10, 10], numpy-seeded reset),
    written here as that module behaves."""

    def __init__(self):
        from scipy.integrate import ode
        self.ode = ode(self.rhs).set_integrator("dopri5")
        self.u, self.t = np.zeros(4), 0.0

    @staticmethod
    def rhs(t, y, F):
        mp, mc, l, g = 0.1, 1.0, 0.5, 9.81
        x, v, th, w = y
        c, s = np.cos(th), np.sin(th)
        M = mp + mc
        tmp = (F + l * w ** 2 * s) / M
        wdot = (g * s - c * tmp) / (l * (4.0 / 3.0 - mp * c ** 2 / M))
        return [v, tmp - l * wdot * c / M, w, wdot]

    def reset(self, seed):
        np.random.seed(seed)
        self.u, self.t = np.random.uniform(-0.05, 0.05, 4), 0.0

    def failed(self):
        return abs(self.u[0]) > 2.4 or abs(self.u[2]) > math.pi / 15

    def advance(self, action):
        F = min(10.0, max(-10.0, action[0]))
        self.ode.set_initial_value(self.u, self.t).set_f_params(F)
        self.u = self.ode.integrate(self.t + 0.02)
        self.t += 0.02
        return self.failed()


_cart = ScipyCartPole()


def scipy_cartpole_env(s):
    """env.py's environment function, on the scipy CartPole"""
    sid, lid = s["Sample Id"], s["Launch Id"]
    env_id = sid % 3 if s["Mode"] == "Training" else 0
    _cart.reset(sid * 1024 + lid)
    s["Environment Id"] = env_id
    s["State"] = _cart.u.tolist()
    step, done = 0, False
    while not done and step < 500:
        s.update()
        done = _cart.advance(s["Action"])
        r = 1.0 - 1.0 * _cart.failed()
        s["Reward"] = r if env_id == 0 else (r - 1 if env_id == 1 else r * 0.1)
        s["State"] = _cart.u.tolist()
        step += 1
    s["Termination"] = "Terminal" if _cart.failed() else "Truncated"


def host_experiment(env, **kw):
    from vracer_cases import cartpole_vracer
    e = cartpole_vracer(kernel=None, **kw)
    e["Problem"]["Environment Function"] = env
    return e


@pytest.mark.parametrize("environments,policy,rescale", [(1, "Clipped Normal", False), (4, "Normal", False),
                                                         (3, "Clipped Normal", True)])
def test_host_environment_trains_exactly_like_the_cartpole_kernel(environments, policy, rescale):
    """The same experiment, once with the device CartPole kernel and once with
    a host environment function on the same dynamics: every episode, every
    policy update and the final policy equal (the host path shares the
    policy evaluation, action noise, episode bookkeeping, replay memory and
    updates with the kernel path; only the transitions cross the boundary)."""
    import korali
    from vracer_cases import cartpole_vracer
    runs = []
    for kernel in ("CartPole", None):
        e = cartpole_vracer(max_generations=15, environments=environments, hidden=32, policy=policy, kernel=kernel)
        if kernel is None:
            e["Problem"]["Environment Function"] = device_cartpole_env
        e["Solver"]["Experience Replay"]["Start Size"] = 300
        e["Solver"]["State Rescaling"]["Enabled"] = rescale
        e["Solver"]["Reward"]["Rescaling"]["Enabled"] = rescale
        korali.Engine().run(e)
        runs.append(json.loads(e.dump())["Solver"])
    a, b = runs
    assert a["Policy Update Count"] > 0
    for k in ("Current Episode", "Experience Count", "Policy Update Count", "Current Learning Rate",
              "Current Sample ID"):
        assert a[k] == b[k], k
    assert a["Training"]["Reward History"] == b["Training"]["Reward History"]
    assert a["Training"]["Current Policy"]["Policy"] == b["Training"]["Current Policy"]["Policy"]
    assert a["Experience Replay"]["Off Policy"] == b["Experience Replay"]["Off Policy"]
    assert a["State Rescaling"]["Means"] == b["State Rescaling"]["Means"]
    assert a["Reward"]["Rescaling"]["Sigma"] == b["Reward"]["Rescaling"]["Sigma"]


def test_reference_example_runs_unchanged():
    """run-vracer.py's experiment as the reference writes it (Environment
    Function = env.py's env on the scipy CartPole, Environment Count 3,
    Actions Between Policy Updates 1, one concurrent environment), fewer
    generations: every episode of 10 per generation processed, policy
    updates once 1000 experiences are stored."""
    import korali
    e = host_experiment(scipy_cartpole_env, max_generations=20)
    korali.Engine().run(e)
    sv = e["Solver"]
    assert e["Current Generation"] == 20 and sv["Current Episode"] == 200
    assert sv["Current Sample ID"] == 201  # 200 episodes processed, one in flight
    hist = np.array(sv["Training"]["Reward History"])
    assert hist.size == 200 and np.all(np.isfinite(hist))
    assert sv["Experience Count"] > 1000 and sv["Policy Update Count"] == sv["Experience Count"] - 1000
    assert len(sv["Training"]["Current Policy"]["Policy"]) == (4 * 32 + 32) + (32 * 32 + 32) + (32 * 3 + 3)
    # env ids: sample id % 3 -> rewards 1 / 0 / 0.1 per surviving step
    for j, r in enumerate(hist):
        if j % 3 == 1:
            assert r <= 0.0


def test_host_testing_mode_equals_the_kernel_testing_episodes():
    """Testing mode with a host environment (runTestingEpisode: the policy's
    mode on the state rescaled with the agent's moments, Launch Id counted
    from 0): rewards equal the CartPole kernel's testing episodes with the
    same policy."""
    import korali
    from vracer_cases import cartpole_vracer
    e = cartpole_vracer(max_generations=5, environments=8, hidden=32)
    e["Solver"]["State Rescaling"]["Enabled"] = True
    e["Solver"]["Experience Replay"]["Start Size"] = 200
    korali.Engine().run(e)
    res = {}
    for kernel in ("CartPole", None):
        t = cartpole_vracer(max_generations=5, environments=8, hidden=32, kernel=kernel)
        if kernel is None:
            t["Problem"]["Environment Function"] = device_cartpole_env
        t["Solver"]["State Rescaling"]["Enabled"] = True
        t["Solver"]["Experience Replay"]["Start Size"] = 200
        t["Solver"]["Mode"] = "Testing"
        t["Solver"]["Testing"]["Sample Ids"] = list(range(10))
        t["Solver"]["Training"]["Current Policy"]["Policy"] = e["Solver"]["Training"]["Current Policy"]["Policy"]
        t["Solver"]["State Rescaling"]["Means"] = e["Solver"]["State Rescaling"]["Means"]
        t["Solver"]["State Rescaling"]["Sigmas"] = e["Solver"]["State Rescaling"]["Sigmas"]
        korali.Engine().run(t)
        res[kernel] = list(t["Solver"]["Testing"]["Reward"])
    assert res["CartPole"] == res[None]
    assert all(r >= 1.0 for r in res[None])


def toy_env(s):
    """3 state variables, 2 actions: the state is a target the actions chase;
    reward -|a - target|^2; 12 steps then Truncated"""
    rs = np.random.RandomState(s["Sample Id"])
    x = rs.uniform(-1, 1, 3)
    s["State"] = x.tolist()
    for _ in range(12):
        s.update()
        a = np.array(s["Action"])
        assert a.shape == (2,)
        s["Reward"] = -float(np.sum((a - x[:2]) ** 2))
        x = rs.uniform(-1, 1, 3)
        s["State"] = x.tolist()
    s["Termination"] = "Truncated"


def test_host_environment_any_state_and_action_sizes():
    """A host environment with 3 state and 2 action variables (the CartPole
    kernel is 4 / 1): the policy has the reference's layer sizes, every
    episode of 12 steps is stored, the actions respect Clipped Normal's
    bounds."""
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Reinforcement Learning / Continuous"
    e["Problem"]["Environment Function"] = toy_env
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
    sv["Experience Replay"]["Start Size"] = 96
    sv["Experience Replay"]["Maximum Size"] = 4096
    sv["Learning Rate"] = 1e-3
    sv["Mini Batch"]["Size"] = 32
    sv["Policy"]["Distribution"] = "Clipped Normal"
    for j in range(2):
        sv["Neural Network"]["Hidden Layers"][2 * j]["Type"] = "Layer/Linear"
        sv["Neural Network"]["Hidden Layers"][2 * j]["Output Channels"] = 32
        sv["Neural Network"]["Hidden Layers"][2 * j + 1]["Type"] = "Layer/Activation"
        sv["Neural Network"]["Hidden Layers"][2 * j + 1]["Function"] = "Elementwise/Tanh"
    sv["Termination Criteria"]["Max Generations"] = 10
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    korali.Engine().run(e)
    assert sv["Current Episode"] == 40 and sv["Experience Count"] == 40 * 12
    assert sv["Policy Update Count"] == 40 * 12 - 96
    assert len(sv["Training"]["Current Policy"]["Policy"]) == (3 * 32 + 32) + (32 * 32 + 32) + (32 * 5 + 5)
    hist = np.array(sv["Training"]["Reward History"])
    assert hist.size == 40 and np.all(hist <= 0.0) and np.all(np.isfinite(hist))


def _bad(kind):
    def env(s):
        s["State"] = [0.0, 0.0, 0.0] if kind == "size" else [0.0] * 4
        if kind == "envid":
            s["Environment Id"] = 7
        if kind == "raise":
            raise ValueError("the environment broke")
        s.update()
        s["Reward"] = float("nan") if kind == "nan" else 1.0
        s["State"] = [0.0] * 4
        if kind == "status":
            s["Termination"] = "Done"
        # "unset": returns without a termination status
    return env


@pytest.mark.parametrize("kind,msg", [
    ("unset", "termination status \\(success or truncated\\) was not set"),
    ("status", "neither 'Terminal' nor 'Truncated'"),
    ("size", "wrong size: 3, expected: 4"),
    ("envid", "exceeds the maximum environment count"),
    ("nan", "reward returned an invalid value"),
    ("raise", "the environment broke"),
])
def test_host_environment_errors(kind, msg):
    """The reference's checks on what an environment function returns
    (reinforcementLearning.cpp.base:77-83, :131-134, :351-392); a Python
    exception inside the function ends the run with its message, and the
    engine leaves no coroutine behind."""
    import korali
    e = host_experiment(_bad(kind), max_generations=2)
    with pytest.raises(Exception, match=msg):
        korali.Engine().run(e)


def test_host_environment_resume(tmp_path):
    """Experiment.loadState of a host-environment run: the replay memory,
    policy and counters continue from state.bin; the episodes in flight are
    relaunched (the reference loses them with the run as well), the sample
    ids continuing where they were."""
    import korali
    e = host_experiment(device_cartpole_env, max_generations=4, environments=2)
    e["Solver"]["Experience Replay"]["Start Size"] = 150
    e["File Output"]["Enabled"] = True
    e["File Output"]["Path"] = str(tmp_path)
    korali.Engine().run(e)
    first = json.load(open(tmp_path / "latest"))["Solver"]
    r = korali.Experiment()
    assert r.loadState(str(tmp_path / "latest"))
    r["Problem"]["Environment Function"] = device_cartpole_env
    r["Solver"]["Termination Criteria"]["Max Generations"] = 7
    korali.Engine().run(r)
    sv = json.load(open(tmp_path / "latest"))["Solver"]
    n0, n1 = first["Current Episode"], sv["Current Episode"]
    assert 40 <= n0 <= 41 and 70 <= n1 <= 71  # 10 per generation, two environments finishing together
    assert len(sv["Training"]["Reward History"]) == n1
    assert sv["Training"]["Reward History"][:n0] == first["Training"]["Reward History"]
    assert sv["Experience Count"] > first["Experience Count"]
    assert sv["Policy Update Count"] > first["Policy Update Count"]
    # the two relaunched environments, then one launch per episode
    assert sv["Current Sample ID"] == first["Current Sample ID"] + 2 + (n1 - n0)
    assert os.path.exists(tmp_path / "state.bin")
