"""GPU parity of the VRACER agent (korali_amd/csrc/kg_vracer.hip) against the
oracle's restatement (oracle/vracer_ref.py), through the C-ABI.

Float32 like the reference; the device reassociates the matrix products
(MFMA 16x16x4 tiles) and uses the device libm, so values are compared with
float32 tolerances (written per check); discrete outcomes (termination,
episode ids, mini-batch ids, on-policy flags, counters) must be equal.
Reference parity is unpinned (no VRACER fixtures in the reference)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import vracer_ref as V  # noqa: E402

pytestmark = pytest.mark.gpu
f32 = np.float32
S, A = 4, 1


def theta_for(H, L, seed, spread=0.15):
    n = V.hyperparameter_count(S, H, L, A)
    rng = np.random.default_rng(seed)
    th = V.initial_hyperparameters(S, H, L, A, rng.uniform(-1, 1, n))
    return (th + spread * rng.standard_normal(n) / np.sqrt(H)).astype(f32)


def device(**kw):
    from korali_amd.vracer import VracerDevice
    return VracerDevice(**kw)


def close(a, b, rtol, atol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    # NaN on both sides is agreement (a NaN rescaling sigma, see
    # test_environment_steps_match_oracle); NaN on one side is not
    both = np.isnan(a) & np.isnan(b)
    assert not np.any(np.isnan(a) ^ np.isnan(b)), "NaN on one side only"
    a, b = np.where(both, 0.0, a), np.where(both, 0.0, b)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    assert err.max() <= 0, f"max excess {err.max():.3e} at {np.unravel_index(err.argmax(), err.shape)}"


@pytest.mark.parametrize("H,L,n", [(64, 1, 37), (256, 2, 500), (128, 3, 4096), (32, 2, 300), (100, 1, 77)])
def test_run_policy_matches_oracle(H, L, n):
    th = theta_for(H, L, 1, spread=1.0)
    d = device(hidden_size=H, hidden_layers=L, environments=4096, mini_batch_size=64, replay_maximum_size=1024,
               replay_start_size=512, initial_exploration_noise=0.7, hyperparameters=th)
    X = np.random.default_rng(2).standard_normal((n, S)).astype(f32)
    out = d.run_policy(X)
    ref, _ = V.forward(th, X, S, H, L, A, 0.7)
    close(out, ref, 2e-5, 2e-5)  # float32 sums of <= 256 terms in another order
    assert np.all(out[:, 2] > 0)


@pytest.mark.parametrize("H,L,n", [(64, 1, 37), (256, 2, 500), (128, 3, 4096), (32, 2, 300), (100, 1, 77)])
def test_fused_forward_equals_per_layer_kernels(monkeypatch, H, L, n):
    """k_vr_fwd_fused (one launch per forward pass) forms every output with the
    per-layer kernels' operations in their order: equal bit for bit."""
    th = theta_for(H, L, 1, spread=1.0)
    d = device(hidden_size=H, hidden_layers=L, environments=4096, mini_batch_size=64, replay_maximum_size=1024,
               replay_start_size=512, initial_exploration_noise=0.7, hyperparameters=th)
    X = np.random.default_rng(5).standard_normal((n, S)).astype(f32)
    monkeypatch.setenv("KORALI_AMD_VR_FUSED", "1")
    fused = d.run_policy(X)
    monkeypatch.setenv("KORALI_AMD_VR_FUSED", "0")
    per_layer = d.run_policy(X)
    assert np.array_equal(fused, per_layer)


def test_fused_update_equals_per_layer_kernels(monkeypatch):
    """Policy updates with drawn mini-batches: the fused draw + forward launch
    (and the draw counter advanced by the metadata kernel) leaves every
    hyperparameter, Adam moment and replay field equal to the separate
    k_vr_minibatch + per-layer forward bit for bit; so do the retrace walks
    staged through LDS against the one-thread walks."""
    ag, th = fill_replay(64, 2, 8, 90, 600)
    runs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("KORALI_AMD_VR_FUSED", fused)
        monkeypatch.setenv("KORALI_AMD_VR_STAGED", fused)  # (staged walks with the fused forward)
        d = device(hidden_size=64, hidden_layers=2, environments=8, mini_batch_size=64, replay_maximum_size=600,
                   replay_start_size=100, hyperparameters=th)
        load_replay(d, ag)
        d.train_policy(7)
        runs.append((d.hyperparameters, d.get("retrace")[:ag.size()], d.get("importance_weight")[:ag.size()],
                     d.get("loss_gradient")))
        d.close()
    for a, b in zip(*runs):
        assert np.array_equal(a, b)


def test_draw_with_input_layer_equals_separate_kernels(monkeypatch):
    """The mini-batch draw fused with the input layer (k_vr_minibatch_in,
    many workgroups, the draw counter advanced by k_vr_meta) against the
    one-workgroup draw + k_vr_fwd_in (the default): every update's results
    bit for bit."""
    ag, th = fill_replay(64, 2, 8, 90, 600)
    runs = []
    monkeypatch.setenv("KORALI_AMD_VR_FUSED", "0")
    for v in ("1", "0"):
        monkeypatch.setenv("KORALI_AMD_VR_DRAW_IN", v)
        d = device(hidden_size=64, hidden_layers=2, environments=8, mini_batch_size=64, replay_maximum_size=600,
                   replay_start_size=100, hyperparameters=th)
        load_replay(d, ag)
        d.train_policy(9)
        runs.append((d.hyperparameters, d.get("retrace")[:ag.size()], d.get("importance_weight")[:ag.size()],
                     d.get("loss_gradient")))
        d.close()
    for a, b in zip(*runs):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("glen,ahead", [("4", "0"), ("5", "0"), ("4", "1"), ("5", "1")])
def test_graph_replayed_updates_equal_kernel_launches(monkeypatch, glen, ahead):
    """trainPolicy's updates replayed from a captured graph of glen updates
    (11 updates: whole graphs, then the rest launched kernel by kernel) leave
    the hyperparameters, Adam moments, retrace values and importance weights
    equal to launching every update's kernels, bit for bit."""
    ag, th = fill_replay(64, 2, 8, 90, 600)
    runs = []
    monkeypatch.setenv("KORALI_AMD_VR_FUSED", "0")
    monkeypatch.setenv("KORALI_AMD_VR_DRAW_AHEAD", ahead)  # (the graph's mini-batches drawn up front)
    for g in (glen, "0"):
        monkeypatch.setenv("KORALI_AMD_VR_GRAPH", g)
        d = device(hidden_size=64, hidden_layers=2, environments=8, mini_batch_size=64, replay_maximum_size=600,
                   replay_start_size=100, hyperparameters=th)
        load_replay(d, ag)
        d.train_policy(11)
        d.train_policy(int(glen))  # the captured graph replayed again
        runs.append((d.hyperparameters, d.get("retrace")[:ag.size()], d.get("importance_weight")[:ag.size()],
                     d.get("loss_gradient")))
        d.close()
    for a, b in zip(*runs):
        assert np.array_equal(a, b)


CLIP = (np.array([-0.5], f32), np.array([0.5], f32))  # narrow bounds: every clipping branch is taken


def clip_kw(clipped):
    return dict(policy_distribution="Clipped Normal", action_lower_bound=-0.5, action_upper_bound=0.5) if clipped \
        else {}


def fill_replay(H, L, E, steps, max_size, seed=3, bounds=None):
    th = theta_for(H, L, seed)
    ag = V.Agent(S, A, H, L, th, max_size=max_size, bounds=bounds)
    ro = V.Rollouts(ag, E, max_steps=40)
    for s in range(steps):
        ro.step(V.action_noise(seed, s, E, A))
    return ag, th


def load_replay(d, ag):
    er, n = ag.er, ag.size()
    d.set("state", np.stack(er["state"]))
    d.set("action", np.stack(er["action"]))
    d.set("reward", np.array(er["reward"], f32))
    d.set("environment_id", np.array(er["env"]))
    d.set("termination", np.array(er["term"]))
    d.set("truncated_state", np.stack(er["tstate"]))
    d.set("exp_policy", np.stack(er["exp_pol"]))
    d.set("cur_policy", np.stack(er["cur_pol"]))
    d.set("exp_state_value", np.array(er["exp_v"], f32))
    d.set("state_value", np.array(er["v"], f32))
    d.set("retrace", np.array(er["ret"], f32))
    d.set("importance_weight", np.array(er["iw"], f32))
    d.set("truncated_importance_weight", np.array(er["tiw"], f32))
    d.set("truncated_state_value", np.array(er["tv"], f32))
    d.set("on_policy", np.array(er["onp"], np.int32))
    d.set("episode_id", np.array(er["ep_id"], np.int64))
    d.set("episode_pos", np.array(er["ep_pos"], np.int32))
    d.set_scalar("total", n)
    d.set_scalar("size", n)
    d.set_scalar("off_policy_count", ag.off_count)
    d.set_scalar("current_episode", ag.current_episode)
    d.set_scalar("experience_count", ag.experience_count)


@pytest.mark.parametrize("H,L,B,clipped", [(64, 2, 32, False), (256, 2, 256, False), (64, 2, 64, True),
                                           (32, 2, 32, True)])
def test_policy_updates_match_oracle(H, L, B, clipped):
    """VRACER::trainPolicy on a replay memory filled by the oracle's rollouts:
    five updates with given sorted mini-batches (metadata, retrace, loss
    gradient, backward, fAdam and the REF-ER schedule)."""
    ag, th = fill_replay(H, L, 8, 90, 600, bounds=CLIP if clipped else None)
    d = device(hidden_size=H, hidden_layers=L, environments=8, mini_batch_size=B, replay_maximum_size=600,
               replay_start_size=100, hyperparameters=th, **clip_kw(clipped))
    if clipped:
        acts = np.concatenate(ag.er["action"])
        assert np.any(acts <= -0.5) and np.any(acts >= 0.5) and np.any(np.abs(acts) < 0.5)
    load_replay(d, ag)
    rng = np.random.default_rng(9)
    for u in range(5):
        ids = np.sort(rng.integers(0, ag.size() - 1, B)).astype(np.uint32)
        ids[1] = ids[0]  # a duplicate entry (updateExperienceMetadata's unique filter)
        ids.sort()
        G, grad = ag.train_policy([int(i) for i in ids])
        d.train_minibatch(ids)
        close(d.get("loss_gradient").reshape(B, -1), G, 1e-3, 1e-4)
        close(d.get("gradient"), grad, 2e-3, 2e-3 * np.abs(grad).max())
        close(d.hyperparameters, ag.theta, 1e-4, 1e-6)
        assert np.array_equal(d.get("on_policy")[:ag.size()], np.array(ag.er["onp"], np.int32))
        close(d.get("retrace")[:ag.size()], np.array(ag.er["ret"], f32), 1e-4, 1e-5)
        close(d.get("importance_weight")[:ag.size()], np.array(ag.er["iw"], f32), 1e-4, 1e-6)
        assert d.scalar("policy_update_count") == ag.update_count
        assert d.scalar("off_policy_count") == ag.off_count
        assert np.isclose(d.scalar("refer_beta"), float(ag.beta), rtol=1e-6)
        assert np.isclose(d.scalar("learning_rate"), float(ag.lr), rtol=1e-7)
        assert np.isclose(d.scalar("off_policy_cutoff"), float(ag.cutoff), rtol=1e-7)


def fill_synthetic(Sx, Ax, H, L, n_eps, seed, bounds=None, max_size=600):
    """An oracle agent's replay memory filled with synthetic episodes of Sx
    state and Ax action variables (a host environment's shapes): states and
    rewards from a seeded generator, actions drawn from the agent's own
    policy (clipped to the bounds), the policy and value stored as
    processEpisode stores them; terminal and truncated endings alternate."""
    n = V.hyperparameter_count(Sx, H, L, Ax)
    rng = np.random.default_rng(seed)
    th = (V.initial_hyperparameters(Sx, H, L, Ax, rng.uniform(-1, 1, n))
          + 0.15 * rng.standard_normal(n) / np.sqrt(H)).astype(f32)
    ag = V.Agent(Sx, Ax, H, L, th, max_size=max_size, bounds=bounds)
    for ep in range(n_eps):
        T = int(rng.integers(1, 30))
        states = rng.uniform(-1, 1, (T, Sx)).astype(f32)
        out = ag.policy(states)
        acts = (out[:, 1:1 + Ax] + out[:, 1 + Ax:] * rng.standard_normal((T, Ax)).astype(f32)).astype(f32)
        if bounds is not None:
            acts = np.clip(acts, bounds[0], bounds[1]).astype(f32)
        rewards = rng.normal(0, 1, T).astype(f32)
        term = V.TERMINAL if ep % 2 else V.TRUNCATED
        ag.process_episode(ep % 3, states, acts, rewards, out[:, 1:], out[:, 0], term,
                           tstate=rng.uniform(-1, 1, Sx).astype(f32))
    return ag, th


@pytest.mark.parametrize("Sx,Ax,clipped", [(3, 2, False), (3, 2, True), (5, 4, True), (2, 3, False)])
def test_multi_action_policy_updates_match_oracle(Sx, Ax, clipped):
    """VRACER::trainPolicy with several action components (a host
    environment's agent): the importance weights and their gradients sum the
    components' log-densities in order (continuous.cpp.base:278-397,
    :399-560), the KL gradient is per component (:697-777); five updates
    against the oracle as test_policy_updates_match_oracle."""
    H, L, B = 64, 2, 64
    bounds = (np.full(Ax, -0.5, f32), np.full(Ax, 0.5, f32)) if clipped else None
    ag, th = fill_synthetic(Sx, Ax, H, L, 60, 11, bounds)
    kw = dict(policy_distribution="Clipped Normal", action_lower_bound=-0.5, action_upper_bound=0.5) if clipped \
        else {}
    d = device(state_size=Sx, action_size=Ax, hidden_size=H, hidden_layers=L, environments=8, mini_batch_size=B,
               replay_maximum_size=600, replay_start_size=100, hyperparameters=th, host_environment=True, **kw)
    if clipped:
        acts = np.concatenate(ag.er["action"])
        assert np.any(acts <= -0.5) and np.any(acts >= 0.5) and np.any(np.abs(acts) < 0.5)
    load_replay(d, ag)
    rng = np.random.default_rng(5)
    for u in range(5):
        ids = np.sort(rng.integers(0, ag.size() - 1, B)).astype(np.uint32)
        G, grad = ag.train_policy([int(i) for i in ids])
        d.train_minibatch(ids)
        close(d.get("loss_gradient").reshape(B, -1), G, 1e-3, 1e-4)
        close(d.get("gradient"), grad, 2e-3, 2e-3 * np.abs(grad).max())
        close(d.hyperparameters, ag.theta, 1e-4, 1e-6)
        assert np.array_equal(d.get("on_policy")[:ag.size()], np.array(ag.er["onp"], np.int32))
        close(d.get("importance_weight")[:ag.size()], np.array(ag.er["iw"], f32), 1e-4, 1e-6)
        close(d.get("cur_policy").reshape(-1, 2 * Ax)[:ag.size()], np.stack(ag.er["cur_pol"]), 1e-4, 1e-6)
        assert d.scalar("off_policy_count") == ag.off_count


@pytest.mark.parametrize("clipped,R,T,rr,K", [(False, 700, 40, False, 3), (True, 700, 40, False, 3),
                                             (False, 40, 5, False, 3), (False, 700, 40, True, 3),
                                             (False, 40, 5, True, 3), (False, 700, 40, True, 100),
                                             (False, 40, 5, True, 257)])
def test_environment_steps_match_oracle(clipped, R, T, rr, K):
    """Concurrent CartPole environments with the same action noise: episodes,
    terminations, the replay memory in processEpisode order, initial retrace
    values, relaunch sample ids — 120 steps, eviction included; (R=40, T=5):
    one step appends more experiences than the replay memory holds.  rr:
    Reward Rescaling (the per-environment sums, counts and sigmas in
    processEpisode order, bit for bit, and the scaled initial retrace); K:
    Environment Count (above 64 the per-id tables stay in device memory)."""
    H, L, E = 64, 2, 16
    th = theta_for(H, L, 4, spread=0.6)
    ag = V.Agent(S, A, H, L, th, max_size=R, bounds=CLIP if clipped else None, reward_rescaling=rr,
                 env_count=max(K, 8))
    ro = V.Rollouts(ag, E, env_count=K, max_steps=T)
    d = device(hidden_size=H, hidden_layers=L, environments=E, mini_batch_size=32, replay_maximum_size=R,
               replay_start_size=R, max_episode_steps=T, hyperparameters=th, seed=4, reward_rescaling=rr,
               environment_count=K, **clip_kw(clipped))
    rng = np.random.default_rng(5)
    total = 0
    for s in range(120):
        z = rng.standard_normal((E, A)).astype(f32)
        new_ref, _ = ro.step(z)
        new_dev = d.environment_step(noise=z)
        assert new_dev == new_ref, s
        total += new_ref
    assert total > R  # the ring wrapped
    n = ag.size()
    assert d.scalar("size") == n and d.scalar("total") == total and d.scalar("current_episode") == ag.current_episode
    # device ring -> logical order
    start = (total - n) % R
    order = (start + np.arange(n)) % R
    er = ag.er
    assert np.array_equal(d.get("termination")[order], np.array(er["term"]))
    assert np.array_equal(d.get("episode_id")[order], np.array(er["ep_id"]))
    assert np.array_equal(d.get("episode_pos")[order], np.array(er["ep_pos"]))
    assert np.array_equal(d.get("environment_id")[order], np.array(er["env"]))
    assert np.array_equal(d.get("reward")[order], np.array(er["reward"], f32))
    close(d.get("state").reshape(R, S)[order], np.stack(er["state"]), 1e-5, 1e-6)
    close(d.get("action")[order], np.concatenate(er["action"]), 1e-5, 1e-5)
    close(d.get("exp_policy").reshape(R, 2)[order], np.stack(er["exp_pol"]), 1e-5, 1e-6)
    close(d.get("retrace")[order], np.array(er["ret"], f32), 1e-5, 1e-5)
    close(d.get("truncated_state").reshape(R, S)[order], np.stack(er["tstate"]), 1e-5, 1e-6)
    assert np.array_equal(d.get("env_sample_ids"), np.array(ro.sample, np.uint64))
    if rr:
        assert np.array_equal(d.get("reward_rescaling_count")[:K], ag.rcnt[:K])
        assert np.array_equal(d.get("reward_rescaling_sum")[:K], ag.rsum[:K])
        # (an id whose squared-reward sum cancels to a tiny negative value gets
        # a NaN sigma on both sides, as the reference's sqrt would give)
        assert np.array_equal(d.get("reward_rescaling_sigma")[:K], ag.rsig[:K], equal_nan=True)
        assert np.any(ag.rsig[:K] != 1.0)
    # actions differ in the last float32 bits (reassociated MFMA sums), so do
    # the fp64 states: round 2 measured at most 3.8e-8 after 30 steps
    close(d.get("env_u").reshape(E, 4), np.stack([c.u for c in ro.carts]), 1e-6, 2e-7)


@pytest.mark.parametrize("rr,srs", [(False, False), (True, False), (False, True), (True, True)])
def test_training_loop_matches_oracle_end_to_end(rr, srs):
    """kg_vracer_training_step with the device's own streams (action noise,
    mini-batch uniforms; the oracle draws the same philox blocks) — the
    body of Agent::trainingGeneration: environment step, then as many updates
    as Experiences Between Policy Updates allows once the start size is
    reached.  rr: Reward Rescaling (scaled rewards in the retrace chains and
    the policy gradient's Qret); srs: State Rescaling (the replay memory's
    moments at the start size, every stored state rescaled, episodes launched
    from then on scaling their states)."""
    H, L, E, R, B = 64, 2, 8, 400, 32
    th = theta_for(H, L, 6)
    seed = 77
    ag = V.Agent(S, A, H, L, th, max_size=R, reward_rescaling=rr, state_rescaling=srs)
    ro = V.Rollouts(ag, E, max_steps=30)
    d = device(hidden_size=H, hidden_layers=L, environments=E, mini_batch_size=B, replay_maximum_size=R,
               replay_start_size=150, max_episode_steps=30, experiences_between_policy_updates=4.0,
               hyperparameters=th, seed=seed, reward_rescaling=rr, state_rescaling=srs)
    session_exp, updates, mb_ctr, rescaled = 0, 0, 0, 0
    for s in range(70):
        new_ref, _ = ro.step(V.action_noise(seed, s, E, A))
        session_exp += new_ref
        n = 0
        if ag.experience_count >= 150:
            if ag.maybe_rescale_states(150):
                ro.relaunched_take_moments()
                rescaled += 1
            while session_exp > 4.0 * (updates + n) + 150:
                n += 1
        for _ in range(n):
            ids = ag.minibatch_ids(V.minibatch_uniforms(seed, mb_ctr, B))
            mb_ctr += B
            ag.train_policy(ids)
        updates += n
        new_dev, n_dev = d.training_step()
        assert (new_dev, n_dev) == (new_ref, n), s
    assert updates > 10
    close(d.hyperparameters, ag.theta, 1e-3, 1e-5)
    assert d.scalar("policy_update_count") == ag.update_count
    if rr:
        assert np.array_equal(d.get("reward_rescaling_sigma")[:3], ag.rsig[:3])
    if srs:
        assert rescaled >= 1
        close(d.get("state_rescaling_means"), ag.smean, 1e-5, 1e-6)
        close(d.get("state_rescaling_sigmas"), ag.ssdev, 1e-5, 1e-6)
        assert np.all(ag.ssdev != 1.0)
        n = ag.size()
        total = int(d.scalar("total"))
        order = ((total - n) % R + np.arange(n)) % R
        close(d.get("state").reshape(R, S)[order], np.stack(ag.er["state"]), 1e-4, 1e-5)


def test_c5_shape_runs():
    """Config C5: 4096 concurrent environments, 2x256 hidden layers, mini-batch
    256 — a few training steps with updates; all values finite, counters
    consistent with the reference's update rule."""
    d = device(environments=4096, hidden_size=256, hidden_layers=2, mini_batch_size=256,
               replay_maximum_size=262144, replay_start_size=8192, experiences_between_policy_updates=64.0, seed=1)
    th = theta_for(256, 2, 8)
    d.set("hyperparameters", th)
    tot, ups = 0, 0
    for _ in range(40):
        n, u = d.training_step()
        tot += n
        ups += u
    assert tot == d.scalar("experience_count") and ups == d.scalar("policy_update_count") > 0
    assert np.all(np.isfinite(d.hyperparameters))
    assert np.all(np.isfinite(d.get("retrace")[:int(d.scalar("size"))]))


def test_device_cartpole_matches_reference_trajectories():
    """The device CartPole (kg_vracer.hip cp_advance: DOPRI5 restated as
    scipy runs it) on the forces of the reference's own trajectories
    (tests/golden/cartpole_dopri5.json, from cartpole.py + scipy dopri5).
    The oracle's restatement is bit-exact on these (test_vracer_cpu.py); the
    device differs only through its cos / sin / pow roundings (ocml vs glibc,
    within an ulp), which the falling-pole trajectories amplify: measured
    max |diff| 4.7e-12 with 86 of 631 states bit-identical, every termination
    flag equal."""
    import ctypes
    import json
    from korali_amd import native
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "cartpole_dopri5.json")))
    tr = g["trajectories"]
    n, steps = len(tr), max(len(t["force"]) for t in tr)
    u0 = np.array([t["u0"] for t in tr], np.float64)
    force = np.zeros((n, steps))
    for j, t in enumerate(tr):
        force[j, :len(t["force"])] = t["force"]
    u = np.zeros((n, steps, 4))
    over = np.zeros((n, steps), np.int32)
    vp = ctypes.c_void_p
    L = native.lib()
    assert L.kg_debug_cartpole(0, u0.ctypes.data_as(vp), force.ctypes.data_as(vp), n, steps, u.ctypes.data_as(vp),
                               over.ctypes.data_as(vp)) == 0, L.kg_last_error()
    worst, exact = 0.0, 0
    for j, t in enumerate(tr):
        m = len(t["u"])
        ref = np.array(t["u"])
        assert np.array_equal(over[j, :m], np.array(t["over"])), j
        worst = max(worst, float(np.abs(u[j, :m] - ref).max()))
        exact += int(np.sum(np.all(u[j, :m] == ref, axis=1)))
    print(f"device CartPole vs scipy dopri5: max |diff| {worst:.3e}, {exact} of "
          f"{sum(len(t['u']) for t in tr)} states bit-identical")
    assert worst <= 2e-11


@pytest.mark.parametrize("H,L,clipped,spread", [(64, 2, False, 0.0), (64, 2, True, 0.0), (128, 2, False, 0.15),
                                                (32, 1, True, 0.15)])
def test_testing_episodes_match_oracle(H, L, clipped, spread):
    """Testing mode (Agent::testingGeneration): one deterministic CartPole
    episode per sample id, the policy's mode as the action.  spread 0: every
    weight but the output biases zero, so the actions do not depend on the
    float32 forward's summation order and the episodes equal the oracle's
    exactly; otherwise the mode moves by float32 rounding, which may shift a
    failure by a step."""
    n = V.hyperparameter_count(S, H, L, A)
    rng = np.random.default_rng(5)
    if spread == 0.0:
        th = np.zeros(n, f32)
        th[n - 3:] = np.array([0.1, 0.35 if not clipped else 0.8, 0.0], f32)  # output biases: V, mean, sigma
    else:
        th = theta_for(H, L, 7, spread=spread)
    kw = clip_kw(clipped)
    d = device(hidden_size=H, hidden_layers=L, environments=64, mini_batch_size=32, replay_maximum_size=1024,
               replay_start_size=512, initial_exploration_noise=0.5, hyperparameters=th, **kw)
    sids = np.array([0, 1, 2, 7, 11, 40, 41, 99] + list(range(200, 290)), np.uint64)
    lids = np.arange(sids.size, dtype=np.uint64)
    got = d.test_episodes(sids, lids)
    ref = V.testing_episodes(th, sids, lids, S, H, L, A, 0.5, 500, clipped=clipped,
                             lb=CLIP[0][0] if clipped else None, ub=CLIP[1][0] if clipped else None)
    if spread == 0.0:
        assert np.array_equal(got, ref), (got, ref)
    else:
        assert np.abs(got - ref).max() <= 1.0, (got, ref)
        assert np.mean(got == ref) >= 0.9
    assert np.all(got >= 1.0)
    d.close()


def test_engine_training_resume_is_bit_exact(tmp_path):
    """Experiment.loadState of a VRACER training run's latest result file
    (+ the training state the engine writes beside it, state.bin: replay
    memory, the episodes in flight, policy and Adam moments, counters;
    agent.cpp.base:849-976 serialize / deserialize the replay memory the
    same way) continues it: 3 + 3 generations end exactly like 6."""
    import json
    import os
    import korali
    from vracer_cases import cartpole_vracer

    def experiment(gens, out):
        e = cartpole_vracer(max_generations=gens, environments=4, hidden=32)
        e["Solver"]["Experience Replay"]["Start Size"] = 150
        e["File Output"]["Enabled"] = True
        e["File Output"]["Path"] = str(out)
        return e

    a = experiment(6, tmp_path / "a")
    korali.Engine().run(a)
    korali.Engine().run(experiment(3, tmp_path / "b"))
    assert os.path.exists(tmp_path / "b" / "state.bin")
    r = korali.Experiment()
    assert r.loadState(str(tmp_path / "b" / "latest"))
    r["Solver"]["Termination Criteria"]["Max Generations"] = 6
    korali.Engine().run(r)
    sa = json.load(open(tmp_path / "a" / "latest"))["Solver"]
    sb = json.load(open(tmp_path / "b" / "latest"))["Solver"]
    assert sb["Policy Update Count"] > 0 and sa["Policy Update Count"] == sb["Policy Update Count"]
    for k in ("Experience Count", "Current Episode", "Current Learning Rate"):
        assert sa[k] == sb[k], k
    assert sa["Training"]["Current Policy"]["Policy"] == sb["Training"]["Current Policy"]["Policy"]
    assert sa["Training"]["Reward History"] == sb["Training"]["Reward History"]
    assert sa["Experience Replay"]["Off Policy"] == sb["Experience Replay"]["Off Policy"]
    # a missing training state fails as the reference does (agent.cpp.base:914-915)
    os.remove(tmp_path / "b" / "state.bin")
    r2 = korali.Experiment()
    assert r2.loadState(str(tmp_path / "b" / "latest"))
    r2["Solver"]["Termination Criteria"]["Max Generations"] = 8
    with pytest.raises(korali.KoraliError, match="could not find or deserialize agent's state"):
        korali.Engine().run(r2)
