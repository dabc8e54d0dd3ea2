"""CPU checks of the VRACER oracle (oracle/vracer_ref.py) — the checker of the
device agent (korali_amd/csrc/kg_vracer.hip).  The CartPole environment is
pinned to the reference's own module (tests/golden/cartpole_dopri5.json,
written by tools/make_cartpole_golden.py from cartpole.py with scipy's
dopri5): resets and trajectories bit-exact.  The agent's pieces are pinned
against independent definitions: Random123's philox known answers, numpy's
own RandomState for the resets, finite differences for the backward pass,
and the reference's formulas checked term by term."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import vracer_ref as V  # noqa: E402

f32 = np.float32


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert V.philox4x32((0, 0, 0, 0), 0, 0) == (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)
    assert V.philox4x32((0xffffffff,) * 4, 0xffffffff, 0xffffffff) == (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)
    assert V.philox4x32((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), 0xa4093822, 0x299f31d0) == (
        0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)


def test_normal_stream_moments():
    z = np.array([V.philox_normals(11, 0x4E4F, s, 0) for s in range(4000)], np.float64).ravel()
    assert abs(z.mean()) < 0.05 and abs(z.std() - 1.0) < 0.05
    u = np.array(V.minibatch_uniforms(3, 0, 4000), np.float64)
    assert u.min() >= 0.0 and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.02


def mt_reset(seed):
    """The device's restatement of numpy's legacy seeding (kg_vracer.hip cp_reset)."""
    x, mt = seed & 0xFFFFFFFF, []
    for i in range(405):
        if i:
            x = (1812433253 * (x ^ (x >> 30)) + i) & 0xFFFFFFFF
        mt.append(x)
    out = []
    for i in range(8):
        y = (mt[i] & 0x80000000) | (mt[i + 1] & 0x7FFFFFFF)
        z = mt[i + 397] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        z ^= z >> 11
        z ^= (z << 7) & 0x9D2C5680
        z ^= (z << 15) & 0xEFC60000
        z ^= z >> 18
        out.append(z & 0xFFFFFFFF)
    d = [((out[2 * k] >> 5) * 67108864.0 + (out[2 * k + 1] >> 6)) / 9007199254740992.0 for k in range(4)]
    return np.array([-0.05 + (0.05 - -0.05) * v for v in d])


@pytest.mark.parametrize("sid", [0, 1, 2, 17, 4095, 4096, 123457, 4000000])
def test_cartpole_reset_equals_numpy_random_state(sid):
    c = V.CartPole()
    c.reset(sid * 1024 + sid)  # env.py: cart.reset(sampleId * 1024 + launchId)
    assert np.array_equal(mt_reset(sid * 1024 + sid), c.u)


def cartpole_golden():
    import json
    return json.load(open(os.path.join(ROOT, "tests", "golden", "cartpole_dopri5.json")))


def test_cartpole_resets_match_reference_goldens():
    for r in cartpole_golden()["resets"]:
        c = V.CartPole()
        c.reset(r["seed"])
        assert list(c.u) == r["u"], r["seed"]
        assert list(mt_reset(r["seed"])) == r["u"], r["seed"]  # the device's restatement


def test_cartpole_dopri5_matches_reference_trajectories():
    """The oracle's DOPRI5 restatement reproduces scipy's dopri5 bit for bit
    on every state of every golden trajectory (clip at +-10 included)."""
    g = cartpole_golden()
    assert sum(len(t["u"]) for t in g["trajectories"]) > 500
    for t in g["trajectories"]:
        c = V.CartPole()
        c.reset(t["seed"])
        assert list(c.u) == t["u0"]
        for k, (f, u, over, rew) in enumerate(zip(t["force"], t["u"], t["over"], t["reward"])):
            assert int(c.advance(f)) == over
            assert list(c.u) == u, (t["seed"], k)
            assert c.reward(0) == rew


def test_backward_matches_finite_differences():
    S, H, L, A = 4, 8, 2, 1
    rng = np.random.default_rng(0)
    n = V.hyperparameter_count(S, H, L, A)
    th = (rng.standard_normal(n) * 0.5).astype(f32)
    X = rng.standard_normal((5, S)).astype(f32)
    G = rng.standard_normal((5, 1 + 2 * A)).astype(f32)
    out, acts = V.forward(th, X, S, H, L, A, 1.0)
    g = V.backward(th, acts, out, G, S, H, L, A, 1.0).astype(np.float64)
    f = lambda t: float((V.forward(t.astype(f32), X, S, H, L, A, 1.0)[0].astype(np.float64) * G).sum())
    for seed in range(3):
        d = np.random.default_rng(seed + 1).standard_normal(n).astype(f32)
        eps = 1e-2
        fd = (f(th + eps * d) - f(th - eps * d)) / (2 * eps)
        assert abs(fd - g @ d) <= 5e-3 * max(1.0, abs(fd))


def test_initial_hyperparameters_layout_and_scaling():
    S, H, L, A = 4, 16, 2, 1
    n = V.hyperparameter_count(S, H, L, A)
    assert n == (S * H + H) + (H * H + H) + (H * 3 + 3)
    th = V.initial_hyperparameters(S, H, L, A, np.ones(n, f32))
    W1 = th[:S * H]
    assert np.allclose(W1, np.sqrt(6.0) / np.sqrt(H + S), rtol=1e-6)
    assert np.all(th[S * H:S * H + H] == 0)
    Wout = th[-(3 + 3 * H):-3]
    assert np.allclose(Wout, 0.001 * np.sqrt(6.0) / np.sqrt(3 + H), rtol=1e-6)


def test_normal_policy_terms():
    # continuous.cpp.base:404-440 gradient of exp(logp_cur - logp_old) wrt (mean, sigma)
    a, cm, cs, om, os_ = f32(0.3), f32(0.1), f32(0.7), f32(-0.2), f32(0.9)
    g = V.importance_weight_gradient([a], [cm, cs], [om, os_], 1).astype(np.float64)
    a, cm, cs, om, os_ = (float(v) for v in (a, cm, cs, om, os_))
    lp = lambda m, s: -0.5 * np.log(2 * np.pi * s * s) - 0.5 * ((a - m) / s) ** 2
    iw = lambda m, s: np.exp(lp(m, s) - lp(om, os_))
    e = 1e-4
    assert np.isclose(g[0] / iw(cm, cs), (np.log(iw(cm + e, cs)) - np.log(iw(cm - e, cs))) / (2 * e), rtol=1e-3)
    assert np.isclose(g[1] / iw(cm, cs), (np.log(iw(cm, cs + e)) - np.log(iw(cm, cs - e))) / (2 * e), rtol=1e-3)
    # KL(old || cur) gradient wrt the current parameters (continuous.cpp.base:697-732)
    kl = lambda m, s: np.log(s / os_) + (os_ ** 2 + (om - m) ** 2) / (2 * s * s) - 0.5
    k = V.kl_gradient([f32(om), f32(os_)], [f32(cm), f32(cs)], 1).astype(np.float64)
    assert np.isclose(k[0], (kl(cm + e, cs) - kl(cm - e, cs)) / (2 * e), rtol=1e-3)
    assert np.isclose(k[1], (kl(cm, cs + e) - kl(cm, cs - e)) / (2 * e), rtol=1e-3)
    # importance weights are clamped at exp(+-7) (continuous.cpp.base:389-390)
    assert V.importance_weight([f32(50.0)], [f32(0.0), f32(1.0)], [f32(50.0), f32(1.0)], 1) == f32(np.exp(f32(-7.0)))


def test_adam_ascends():
    ad = V.Adam(3, eta=0.1)
    th = np.zeros(3, f32)
    g = np.array([1.0, -2.0, 0.0], f32)
    th = ad.step(th, g)
    assert th[0] > 0 and th[1] < 0 and th[2] == 0  # fAdam.cpp:87-89 (first moment of -gradient)


def test_initial_retrace_covers_last_two_entries():
    """agent.cpp.base:527: startId = endId - episode.size() + 1 with the episode
    JSON holding two keys — only the last two replay entries get a value."""
    S, H, L, A = 4, 8, 1, 1
    th = np.zeros(V.hyperparameter_count(S, H, L, A), f32)
    ag = V.Agent(S, A, H, L, th, max_size=100, discount=0.5)
    st = [np.zeros(S, f32)] * 4
    ag.process_episode(0, st, [[0.0]] * 4, [1.0, 2.0, 3.0, 4.0], [[0.0, 1.0]] * 4, [0.0] * 4, V.TERMINAL)
    assert [float(r) for r in ag.er["ret"]] == [0.0, 0.0, 3.0 + 0.5 * 4.0, 4.0]
    ag.process_episode(0, st[:1], [[0.0]], [8.0], [[0.0, 1.0]], [0.0], V.TERMINAL)
    # a one-experience episode also rewrites the previous episode's last entry
    assert [float(r) for r in ag.er["ret"]] == [0.0, 0.0, 5.0, 4.0 + 0.5 * 8.0, 8.0]


def test_rollouts_and_update_run():
    S, H, L, A = 4, 16, 2, 1
    n = V.hyperparameter_count(S, H, L, A)
    th = V.initial_hyperparameters(S, H, L, A, np.random.default_rng(0).uniform(-1, 1, n))
    ag = V.Agent(S, A, H, L, th, max_size=300)
    ro = V.Rollouts(ag, 8, max_steps=30)
    for s in range(50):
        ro.step(V.action_noise(5, s, 8, A))
    assert 100 < ag.size() <= 300 and ag.current_episode > 8
    ids = ag.minibatch_ids(V.minibatch_uniforms(5, 0, 32))
    G, grad = ag.train_policy(ids)
    assert np.all(np.isfinite(G)) and np.all(np.isfinite(grad)) and ag.update_count == 1


@pytest.mark.parametrize("a", [-0.5, 0.1, 0.5])  # stored actions are clipped to the bounds
def test_clipped_normal_iw_gradient_matches_finite_differences(a):
    """continuous.cpp.base:482-560: below the lower bound the weight is the
    CDF's, above the upper the CCDF's, inside the density's."""
    bounds = (np.array([-0.5], f32), np.array([0.5], f32))
    cm, cs, om, os_ = f32(0.1), f32(0.6), f32(-0.1), f32(0.8)
    g = V.importance_weight_gradient([f32(a)], [cm, cs], [om, os_], 1, bounds).astype(np.float64)
    from scipy.stats import norm

    def logp(m, s):
        if a <= -0.5:
            return norm.logcdf(-0.5, m, s)
        if a >= 0.5:
            return norm.logsf(0.5, m, s)
        return norm.logpdf(a, m, s)

    iw = np.exp(logp(float(cm), float(cs)) - logp(float(om), float(os_)))
    e = 1e-5
    dm = (logp(float(cm) + e, float(cs)) - logp(float(cm) - e, float(cs))) / (2 * e)
    ds = (logp(float(cm), float(cs) + e) - logp(float(cm), float(cs) - e)) / (2 * e)
    assert np.isclose(g[0], iw * dm, rtol=2e-3) and np.isclose(g[1], iw * ds, rtol=2e-3)


def test_clipped_normal_log_cdf_tails():
    # auxiliar/math.hpp:297-328 far in the tails (the asymptotic log erfc branch)
    from scipy.stats import norm
    for x in (-40.0, -8.0, 0.0, 8.0, 40.0):
        assert np.isclose(V.normal_logcdf(f32(x), f32(0), f32(1)), norm.logcdf(x), rtol=1e-6, atol=1e-6)
        assert np.isclose(V.normal_logccdf(f32(x), f32(0), f32(1)), norm.logsf(x), rtol=1e-6, atol=1e-6)


def test_policy_description_matches_reference_result_files():
    """The continuous agent's policy description (continuous.cpp.base:9-60)
    and the network's hyperparameter layout against the reference's own
    VRACER result files (tests/python/rlview/abf2d_vracer{1,2}, 4 states,
    3 actions, 2 x 64 tanh; facts extracted by tests/golden/make_vracer_golden.py)."""
    import korali
    from korali_amd import libkorali
    runs = json.load(open(os.path.join(ROOT, "tests", "golden", "vracer_abf2d.json")))
    for run, r in runs.items():
        e = korali.Experiment()
        for i, v in enumerate(r["variables"]):
            for k, val in v.items():
                e["Variables"][i][k] = val
        e["Solver"]["Policy"]["Distribution"] = r["solver"]["Policy"]["Distribution"]
        e["Solver"]["Neural Network"]["Hidden Layers"] = r["solver"]["Neural Network"]["Hidden Layers"]
        d = libkorali._vracer_policy_description(e)
        ex = r["expected"]
        for k, v in ex["Policy"].items():
            assert d["Solver"]["Policy"][k] == v, (run, k)
        assert d["Solver"]["Action Shifts"] == ex["Action Shifts"] and d["Solver"]["Action Scales"] == ex["Action Scales"]
        for k, v in r["problem"].items():
            assert d["Problem"][k] == v, (run, k)
        hp = r["hyperparameters"]
        assert d["Hyperparameter Count"] == hp["count"] == hp["covered"] == 4935
        assert d["Layer Sizes"] == hp["layer_sizes"]
        # initial hyperparameters: [W (out x in), b] per layer, zero biases,
        # Xavier-bounded weights, the output layer scaled by 0.001 -- the
        # pattern of the reference's generation-0 vector
        theta = np.array(libkorali._vracer_initial_hyperparameters(hp["layer_sizes"], 7))
        assert theta.size == hp["count"]
        k = 0
        for L, (ic, oc) in zip(hp["layers"], zip(hp["layer_sizes"][:-1], hp["layer_sizes"][1:])):
            W, b = theta[k:k + ic * oc], theta[k + ic * oc:k + ic * oc + oc]
            k += ic * oc + oc
            bound = np.sqrt(6.0) / np.sqrt(ic + oc) * (0.001 if oc == hp["layer_sizes"][-1] else 1.0)
            assert L["bias_all_zero"] and np.all(b == 0.0)
            assert L["weights_nonzero"] == ic * oc and np.all(W != 0.0)
            # both vectors fill the same Xavier interval (largest |w| within 5% of the bound)
            assert 0.95 * bound < L["weight_max_abs"] <= bound * (1 + 1e-6)
            assert 0.95 * bound < np.abs(W).max() <= bound * (1 + 1e-6)
