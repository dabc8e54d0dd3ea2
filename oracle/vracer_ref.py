"""VRACER oracle — TEST INFRASTRUCTURE ONLY.

A NumPy restatement of the reference's VRACER agent for the continuous
"Normal" policy, used by tests/ and bench.py's CPU-baseline leg as the
checker of the HIP path (korali_amd/csrc/kg_vracer.hip).  Nothing in the
product path imports it.

What it restates (reference paths relative to the korali root):

* critic/policy network: DeepSupervisor's layer list (deepSupervisor.cpp.base:21-60)
  = input, user hidden layers (Linear + Elementwise/Tanh), a Linear layer to
  1 + 2A outputs with Weight Scaling 0.001 (VRACER.cpp.base:38), Output layer
  with Identity / Softplus masks, Scale and Shift (continuous.cpp.base:34-61,
  output.cpp.base:140-160 forward, :170-210 backward); Linear forward /
  backward (linear.cpp.base:219-231, :284-291, :337-350: weight gradients
  summed over the batch, not averaged); Xavier initial hyperparameters
  (linear.cpp.base:28-49) in Korali's hyperparameter order [W (out x in), b]
  per layer; fAdam::processResult (fAdam.cpp:64-91; the optimizer ascends);
* agent bookkeeping: processEpisode (agent.cpp.base:376-572: replay append,
  initial retrace values, off-policy count on eviction), generateMiniBatch
  (:574-597), updateExperienceMetadata (:599-735: importance weights,
  on-policy flags, REF-ER cutoff, truncated state values, retrace chains),
  the REF-ER learning-rate / beta schedule (:221-231);
* VRACER::calculatePolicyGradients (VRACER.cpp.base:89-181) with the Normal
  policy's importance weight, its gradient and the KL gradient
  (continuous.cpp.base:278-440, :697-732), normalLogDensity (auxiliar/math.hpp:269-274);
* the CartPole environment of examples/learning/reinforcement/cartpole/_model
  (cartpole.py, env.py): dynamics, 3 reward variants, numpy-seeded resets.

Parity status: **unpinned against the reference** — the reference holds no
VRACER fixtures and its C++ (GSL, Eigen/oneDNN) is not buildable here.  The
restatement follows the reference's float32 formulas; the device is checked
against it within float32 tolerances (matrix products are reassociated on
the MFMA units).  Deviations by design, documented in DESIGN.md: the
CartPole ODE is integrated with a fixed-step RK4 instead of scipy's adaptive
dopri5, and the random streams (action noise, mini-batch uniforms) come from
a counter-based generator (philox4x32-10) instead of GSL's, so tests feed
the same noise / ids to both sides.
"""
import math

import numpy as np

f32 = np.float32
KORALI_EPSILON = 0.00000000001

NON_TERMINAL, TERMINAL, TRUNCATED = 0, 1, 2


# ----------------------------------------------------------------- network
def layer_sizes(S, H, L, A):
    return [S] + [H] * L + [1 + 2 * A]


def hyperparameter_count(S, H, L, A):
    s = layer_sizes(S, H, L, A)
    return sum(s[i] * s[i + 1] + s[i + 1] for i in range(len(s) - 1))


def initial_hyperparameters(S, H, L, A, uniforms, output_scaling=0.001):
    """linear.cpp.base:28-49: W = weightScaling * sqrt(6)/sqrt(out+in) * U(-1,1), b = 0;
    hidden layers Weight Scaling 1.0, the last Linear layer 0.001 (VRACER.cpp.base:38)."""
    s = layer_sizes(S, H, L, A)
    out, k = [], 0
    for i in range(len(s) - 1):
        ic, oc = s[i], s[i + 1]
        scale = f32(output_scaling if i == len(s) - 2 else 1.0)
        xav = f32(np.sqrt(f32(6.0)) / np.sqrt(f32(oc + ic)))
        u = np.asarray(uniforms[k:k + ic * oc], dtype=f32)
        k += ic * oc
        out.append((scale * xav * u).astype(f32))
        out.append(np.zeros(oc, f32))
    return np.concatenate(out)


def unpack(theta, S, H, L, A):
    s = layer_sizes(S, H, L, A)
    layers, k = [], 0
    for i in range(len(s) - 1):
        ic, oc = s[i], s[i + 1]
        W = theta[k:k + ic * oc].reshape(oc, ic)
        k += ic * oc
        b = theta[k:k + oc]
        k += oc
        layers.append((W, b))
    return layers


def output_transform(A, initial_noise, mean_shift=None):
    """continuous.cpp.base:34-61 (Normal): [V | means | sigmas]; means Identity,
    scale 1, shift = action shift (0 for the unbounded Normal policy); sigmas
    Softplus with scale 2 * Initial Exploration Noise."""
    noise = np.broadcast_to(np.asarray(initial_noise, dtype=f32), (A,))
    scale = np.concatenate([[f32(1.0)], np.ones(A, f32), f32(2.0) * noise]).astype(f32)
    shift = np.zeros(1 + 2 * A, f32)
    if mean_shift is not None:
        shift[1:1 + A] = mean_shift
    soft = np.concatenate([[False], np.zeros(A, bool), np.ones(A, bool)])
    return scale, shift, soft


def forward(theta, X, S, H, L, A, initial_noise, mean_shift=None):
    """NeuralNetwork::forward of the critic/policy net; returns (out, acts)."""
    layers = unpack(theta, S, H, L, A)
    scale, shift, soft = output_transform(A, initial_noise, mean_shift)
    acts = [np.asarray(X, dtype=f32)]
    h = acts[0]
    for W, b in layers[:-1]:
        h = np.tanh((h @ W.T + b).astype(f32)).astype(f32)
        acts.append(h)
    W, b = layers[-1]
    z = (h @ W.T + b).astype(f32)
    x = z.astype(np.float64)
    x = np.where(soft, 0.5 * (x + np.sqrt(1.0 + x * x)), x)
    out = (x.astype(f32) * scale + shift).astype(f32)
    return out, acts


def backward(theta, acts, out, G, S, H, L, A, initial_noise, mean_shift=None):
    """Output-layer gradient preprocessing (output.cpp.base:170-210), then the
    Linear/Tanh backward; returns the hyperparameter gradient vector."""
    layers = unpack(theta, S, H, L, A)
    scale, shift, soft = output_transform(A, initial_noise, mean_shift)
    x = ((out - shift) / scale).astype(f32)
    g = (np.asarray(G, f32) * scale).astype(f32)
    nnx = (x - f32(0.25) / x).astype(np.float64)
    gs = (g.astype(np.float64) * 0.5 * (1.0 + nnx / np.sqrt(nnx * nnx + 1.0))).astype(f32)
    g = np.where(soft, gs, g).astype(f32)
    grads = [None] * (2 * len(layers))
    for li in range(len(layers) - 1, -1, -1):
        W, b = layers[li]
        a = acts[li]
        grads[2 * li] = (g.T @ a).astype(f32)
        grads[2 * li + 1] = g.sum(axis=0, dtype=f32)
        if li > 0:
            g = ((g @ W) * (f32(1.0) - a * a)).astype(f32)
    return np.concatenate([x.ravel() for x in grads]).astype(f32)


class Adam:
    """korali::fAdam (fAdam.cpp:20-91): the first moment accumulates -gradient,
    so the update ascends the gradient."""

    def __init__(self, n, eta=1e-3):
        self.b1, self.b2, self.eps = f32(0.9), f32(0.999), f32(1e-8)
        self.b1p, self.b2p = f32(1.0), f32(1.0)
        self.m = np.zeros(n, f32)
        self.v = np.zeros(n, f32)
        self.eta = f32(eta)

    def step(self, theta, grad):
        self.b1p = f32(self.b1p * self.b1)
        self.b2p = f32(self.b2p * self.b2)
        f1 = f32(1.0) / (f32(1.0) - self.b1p)
        f2 = f32(1.0) / (f32(1.0) - self.b2p)
        self.m = (self.b1 * self.m - (f32(1.0) - self.b1) * grad).astype(f32)
        self.v = (self.b2 * self.v + (f32(1.0) - self.b2) * grad * grad).astype(f32)
        return (theta - self.eta / (np.sqrt(self.v * f2) + self.eps) * self.m * f1).astype(f32)


# ------------------------------------------------------- Normal policy math
def normal_logp(x, mean, sigma):
    """auxiliar/math.hpp:269-274 with T = float (the 2*M_PI and KORALI_EPSILON
    terms promote to double before the float result)."""
    x, mean, sigma = (np.asarray(v, f32) for v in (x, mean, sigma))
    norm = (-0.5 * np.log(2 * np.pi * sigma.astype(np.float64) * sigma.astype(np.float64))).astype(f32)
    d = ((x - mean).astype(np.float64) / (sigma.astype(np.float64) + KORALI_EPSILON)).astype(f32)
    return (norm.astype(np.float64) - 0.5 * d.astype(np.float64) * d.astype(np.float64)).astype(f32)


def log_erfc(x):
    """gsl_sf_log_erfc restated as log(erfc(x)), asymptotic series where erfc
    underflows (GSL parity unpinned: GSL 2.6 is absent)."""
    from scipy.special import erfc
    x = float(x)
    if x < 26.0:
        return float(np.log(erfc(x)))
    x2, h = x * x, 1.0 / (2.0 * x * x)
    return -x2 - np.log(x) - 0.57236494292470008707 + np.log(1.0 - h + 3.0 * h * h - 15.0 * h * h * h)


def normal_logcdf(x, mean, sigma):
    """auxiliar/math.hpp:297-301 with T = float."""
    z = f32((np.float64(f32(f32(x) - f32(mean)))) / (np.float64(f32(sigma)) * np.sqrt(2.0)))
    return f32(np.log(0.5) + log_erfc(-np.float64(z)))


def normal_logccdf(x, mean, sigma):
    """auxiliar/math.hpp:324-328 with T = float."""
    z = f32((np.float64(f32(f32(x) - f32(mean)))) / (np.float64(f32(sigma)) * np.sqrt(2.0)))
    return f32(np.log(0.5) + log_erfc(np.float64(z)))


def policy_logp(i, a, m, s, bounds):
    """One action component's log-density (continuous.cpp.base:283-340);
    bounds = None (Normal) or (lb, ub) arrays (Clipped Normal)."""
    if bounds is not None:
        lb, ub = f32(bounds[0][i]), f32(bounds[1][i])
        if a <= lb:
            return normal_logcdf(lb, m, s)
        if ub <= a:
            return normal_logccdf(ub, m, s)
    return normal_logp(a, m, s)


def importance_weight(action, cur, old, A, bounds=None):
    """continuous.cpp.base:278-340, :385-397 (clamped log weight)."""
    lc, lo = f32(0.0), f32(0.0)
    for i in range(A):
        lc = f32(lc + policy_logp(i, f32(action[i]), cur[i], cur[A + i], bounds))
        lo = f32(lo + policy_logp(i, f32(action[i]), old[i], old[A + i], bounds))
    liw = f32(lc - lo)
    liw = min(max(liw, f32(-7.0)), f32(7.0))
    return f32(np.exp(liw))


def importance_weight_gradient(action, cur, old, A, bounds=None):
    """continuous.cpp.base:404-440 (Normal) and :482-560 (Clipped Normal); the
    log weight is not clamped here."""
    if bounds is not None:
        return _clipped_iw_gradient(action, cur, old, A, bounds)
    g = np.zeros(2 * A, f32)
    lc, lo = f32(0.0), f32(0.0)
    for i in range(A):
        m, s = f32(cur[i]), f32(cur[A + i])
        dif = f32(f32(action[i]) - m)
        inv_var = f32(f32(1.0) / f32(s * s))
        g[i] = f32(dif * inv_var)
        g[A + i] = f32(f32(dif * dif) * f32(inv_var / s) - f32(1.0) / s)
        lc = f32(lc + normal_logp(action[i], m, s))
        lo = f32(lo + normal_logp(action[i], old[i], old[A + i]))
    iw = f32(np.exp(f32(lc - lo)))
    return (g * iw).astype(f32)


def _clipped_iw_gradient(action, cur, old, A, bounds):
    g = np.zeros(2 * A, f32)
    lc, lo = f32(0.0), f32(0.0)
    for i in range(A):
        a, m, s, om, os_ = f32(action[i]), f32(cur[i]), f32(cur[A + i]), f32(old[i]), f32(old[A + i])
        lb, ub = f32(bounds[0][i]), f32(bounds[1][i])
        inv_sig = f32(f32(1.0) / s)
        dif = f32(a - m)
        if a <= lb:
            lcdf = normal_logcdf(lb, m, s)
            r = f32(np.exp(f32(normal_logp(lb, m, s) - lcdf)))
            g[i] = -r
            g[A + i] = f32(f32(-dif * inv_sig) * r)
            lc, lo = f32(lc + lcdf), f32(lo + normal_logcdf(lb, om, os_))
        elif ub <= a:
            lccdf = normal_logccdf(ub, m, s)
            r = f32(np.exp(f32(normal_logp(ub, m, s) - lccdf)))
            g[i] = r
            g[A + i] = f32(f32(dif * inv_sig) * r)
            lc, lo = f32(lc + lccdf), f32(lo + normal_logccdf(ub, om, os_))
        else:
            inv_sig3 = f32(f32(inv_sig * inv_sig) * inv_sig)
            g[i] = f32(f32(dif * inv_sig) * inv_sig)
            g[A + i] = f32(f32(f32(dif * dif) * inv_sig3) - inv_sig)
            lc, lo = f32(lc + normal_logp(a, m, s)), f32(lo + normal_logp(a, om, os_))
    iw = f32(np.exp(f32(lc - lo)))
    return (g * iw).astype(f32)


def clipped_kl_gradient(old, cur, A, bounds):
    """continuous.cpp.base:734-777 (Clipped Normal)."""
    from math import erf
    g = np.zeros(2 * A, f32)
    for i in range(A):
        om, osd, cm, cs = f32(old[i]), f32(old[A + i]), f32(cur[i]), f32(cur[A + i])
        lb, ub = f32(bounds[0][i]), f32(bounds[1][i])
        old_var, old_inv_sig, cur_inv_sig = f32(osd * osd), f32(f32(1) / osd), f32(f32(1) / cs)
        cur_inv_var, cur_inv_sig3 = f32(f32(1) / f32(cs * cs)), f32(f32(1) / f32(f32(cs * cs) * cs))
        mu_dif = f32(om - cm)
        inv_sqrt_2pi = f32(np.sqrt(0.5) * np.sqrt(1.0 / np.pi))
        o_lb, o_ub = f32(f32(lb - om) * old_inv_sig), f32(f32(ub - om) * old_inv_sig)
        c_lb, c_ub = f32(f32(lb - cm) * cur_inv_sig), f32(f32(ub - cm) * cur_inv_sig)
        erf_lb, erf_ub = f32(erf(np.sqrt(0.5) * float(o_lb))), f32(erf(np.sqrt(0.5) * float(o_ub)))
        exp_lb, exp_ub = f32(np.exp(f32(f32(f32(-0.5) * o_lb) * o_lb))), f32(np.exp(f32(f32(f32(-0.5) * o_ub) * o_ub)))
        cdf_a = f32(np.exp(f32(f32(normal_logcdf(lb, om, osd) + normal_logp(lb, cm, cs)) - normal_logcdf(lb, cm, cs))))
        ccdf_b = f32(np.exp(f32(f32(normal_logccdf(ub, om, osd) + normal_logp(ub, cm, cs)) - normal_logccdf(ub, cm, cs))))
        km = cdf_a
        km = f32(km - f32(f32(f32(f32(0.5) * mu_dif) * cur_inv_var) * f32(erf_ub - erf_lb)))
        km = f32(km + f32(f32(f32(inv_sqrt_2pi * osd) * cur_inv_var) * f32(exp_ub - exp_lb)))
        km = f32(km - ccdf_b)
        ks = f32(c_lb * cdf_a)
        ks = f32(ks + f32(f32(f32(0.5) * f32(f32(cur_inv_sig - f32(f32(mu_dif * mu_dif) * cur_inv_sig3)) -
                                               f32(old_var * cur_inv_sig3))) * f32(erf_ub - erf_lb)))
        ks = f32(ks + f32(f32(f32(inv_sqrt_2pi * cur_inv_sig3) * f32(f32(old_var * o_ub) + f32(f32(2) * osd * mu_dif)))
                          * exp_ub))
        ks = f32(ks - f32(f32(f32(inv_sqrt_2pi * cur_inv_sig3) * f32(f32(old_var * o_lb) + f32(f32(2) * osd * mu_dif)))
                          * exp_lb))
        ks = f32(ks - f32(c_ub * ccdf_b))
        g[i], g[A + i] = km, ks
    return g


def kl_gradient(old, cur, A, bounds=None):
    """continuous.cpp.base:697-732 (Normal); :734-777 for Clipped Normal."""
    if bounds is not None:
        return clipped_kl_gradient(old, cur, A, bounds)
    g = np.zeros(2 * A, f32)
    for i in range(A):
        om, osd, cm, cs = f32(old[i]), f32(old[A + i]), f32(cur[i]), f32(cur[A + i])
        inv_sig = f32(1.0 / np.float64(cs))
        inv_var = f32(1.0 / np.float64(f32(cs * cs)))
        inv_sig3 = f32(1.0 / np.float64(f32(f32(cs * cs) * cs)))
        d = f32(cm - om)
        g[i] = f32(d * inv_var)
        g[A + i] = f32(f32(f32(-inv_sig3 * osd) * osd) + f32(-f32(d * d) * inv_sig3)) + inv_sig
    return g.astype(f32)


# --------------------------------------------------------------- the agent
class Agent:
    """Replay memory + REF-ER bookkeeping of agent.cpp.base, Normal policy VRACER.
    The replay memory is kept in logical order (index 0 = oldest), exactly
    the reference's cBuffer view (auxiliar/cbuffer.hpp:97-142)."""

    FIELDS = ("state", "action", "reward", "env", "term", "tstate", "exp_pol", "exp_v", "cur_pol", "v",
              "ret", "iw", "tiw", "tv", "onp", "ep_id", "ep_pos")

    def __init__(self, S, A, H=256, L=2, theta=None, *, max_size=4096, discount=0.995, learning_rate=1e-4,
                 iw_truncation=1.0, cutoff_scale=4.0, off_target=0.1, annealing_rate=0.0, refer_beta=0.3,
                 initial_noise=1.0, l2_enabled=False, l2_importance=1e-4, bounds=None, reward_rescaling=False,
                 env_count=8, state_rescaling=False):
        """bounds = None: Normal policy; (lb, ub) arrays: Clipped Normal.
        reward_rescaling: Reward / Rescaling / Enabled (agent.cpp.base:96-98,
        :423-437, :557-563; getScaledReward, agent.hpp:711-719)."""
        self.S, self.A, self.H, self.L = S, A, H, L
        self.bounds = None if bounds is None else (np.broadcast_to(np.asarray(bounds[0], f32), (A,)),
                                                   np.broadcast_to(np.asarray(bounds[1], f32), (A,)))
        self.theta = np.asarray(theta, f32).copy()
        self.adam = Adam(self.theta.size)
        self.max_size = max_size
        self.gamma = f32(discount)
        self.lr0 = f32(learning_rate)
        self.lr = f32(learning_rate)
        self.iw_trunc = f32(iw_truncation)
        self.cutoff_scale = f32(cutoff_scale)
        self.cutoff = f32(cutoff_scale)
        self.off_target = f32(off_target)
        self.anneal = f32(annealing_rate)
        self.beta = f32(refer_beta)
        self.noise = initial_noise
        self.l2 = (bool(l2_enabled), f32(l2_importance))
        self.off_count = 0
        self.off_ratio = f32(0.0)
        self.update_count = 0
        self.current_episode = 0
        self.experience_count = 0
        self.er = {k: [] for k in self.FIELDS}
        # per environment id: the sum of squared rewards and the experience
        # count in the replay memory (kept whether or not rescaling is on, as
        # the reference does), and the rescaling sigma (1.0 unless enabled)
        self.reward_rescaling = bool(reward_rescaling)
        self.rsum = np.zeros(env_count, f32)
        self.rcnt = np.zeros(env_count, np.int64)
        self.rsig = np.ones(env_count, f32)
        # State Rescaling (agent.cpp.base:92-94, :204-207, :291-322): the
        # moments the environments scale their states with (identity until set)
        self.state_rescaling = bool(state_rescaling)
        self.smean = np.zeros(S, f32)
        self.ssdev = np.ones(S, f32)

    # ---- helpers
    def size(self):
        return len(self.er["reward"])

    def shift(self):
        """Bounded distributions shift the means by (ub + lb) / 2 (continuous.cpp.base:20-30, :53-54)."""
        if self.bounds is None:
            return None
        return ((self.bounds[1] + self.bounds[0]) * f32(0.5)).astype(f32)

    def policy(self, X):
        out, _ = forward(self.theta, np.atleast_2d(X), self.S, self.H, self.L, self.A, self.noise, self.shift())
        return out

    def scaled_reward(self, i):
        """getScaledReward (agent.hpp:711-719) of replay entry i: float division"""
        return f32(self.er["reward"][i] / self.rsig[self.er["env"][i]])

    def _add(self, **kw):
        # agent.cpp.base:423-437: the new reward's square in, then (memory
        # full) the evicted one's out
        r, env = f32(kw["reward"]), kw["env"]
        self.rsum[env] = f32(self.rsum[env] + f32(r * r))
        self.rcnt[env] += 1
        if self.size() == self.max_size:
            ev, rv = self.er["env"][0], f32(self.er["reward"][0])
            self.rsum[ev] = f32(self.rsum[ev] - f32(rv * rv))
            self.rcnt[ev] -= 1
            if not self.er["onp"][0]:
                self.off_count -= 1
            for k in self.FIELDS:
                self.er[k].pop(0)
        for k in self.FIELDS:
            self.er[k].append(kw[k])

    def process_episode(self, env_id, states, actions, rewards, pols, vals, termination, tstate=None):
        """agent.cpp.base:376-572 (no reward rescaling / outbound penalty)."""
        n = len(rewards)
        for t in range(n):
            term = termination if t == n - 1 else NON_TERMINAL
            ts = np.asarray(tstate, f32) if term == TRUNCATED else np.zeros(self.S, f32)
            self._add(state=np.asarray(states[t], f32), action=np.asarray(actions[t], f32), reward=f32(rewards[t]),
                      env=env_id, term=term, tstate=ts, exp_pol=np.asarray(pols[t], f32), exp_v=f32(vals[t]),
                      cur_pol=np.asarray(pols[t], f32), v=f32(vals[t]), ret=f32(0.0), iw=f32(1.0), tiw=f32(1.0),
                      tv=f32(0.0), onp=True, ep_id=self.current_episode, ep_pos=t)
        ret = f32(0.0)
        end = self.size() - 1
        if termination == TRUNCATED:
            tv = self.policy(np.asarray(tstate, f32))[0, 0]
            ret = f32(ret + f32(self.gamma * tv))
        # agent.cpp.base:527 takes startId = endId - episode.size() + 1 where
        # `episode` is the JSON object {"Environment Id", "Experiences"}: its
        # size() is 2, so the initial retrace covers the last two replay
        # entries (the previous episode's last one when this episode has a
        # single experience); every other entry keeps the 0.0 placeholder
        # until a mini-batch retrace chain reaches it.  Reproduced as is.
        for e in range(end, max(end - 2, -1), -1):
            ret = f32(f32(self.gamma * ret) + self.scaled_reward(e))
            self.er["ret"][e] = ret
        if self.reward_rescaling:  # agent.cpp.base:557-563 (float sums, double quotient and sqrt)
            for i in range(self.rsig.size):
                q = np.float64(self.rsum[i]) / (np.float64(np.float32(self.rcnt[i])) + 1e-9)
                self.rsig[i] = f32(np.sqrt(q) + 1e-9)
        self.current_episode += 1
        self.experience_count += n

    def rescale_states(self):
        """rescaleStates (agent.cpp.base:291-322): float sums over the replay
        memory in order, the moments, then every stored state rescaled (the
        truncated states are not)"""
        st = self.er["state"]
        ssum = np.zeros(self.S, f32)
        ssq = np.zeros(self.S, f32)
        for x in st:
            for d in range(self.S):
                ssum[d] = f32(ssum[d] + x[d])
                ssq[d] = f32(ssq[d] + f32(x[d] * x[d]))
        n = f32(len(st))
        with np.errstate(all="ignore"):
            for d in range(self.S):
                m = f32(ssum[d] / n)
                if not np.isfinite(m):
                    m = f32(0.0)
                sg = f32(np.sqrt(f32(f32(ssq[d] / n) - f32(m * m))))
                if not np.isfinite(sg):
                    sg = f32(1.0)
                if sg <= 1e-9:
                    sg = f32(1.0)
                self.smean[d], self.ssdev[d] = m, sg
        for i in range(len(st)):
            st[i] = ((st[i] - self.smean) / self.ssdev).astype(f32)

    def maybe_rescale_states(self, start_size):
        """agent.cpp.base:201-207: at the training loop, once the start size is
        reached and before the first policy update (every time until then)"""
        if self.state_rescaling and self.experience_count >= start_size and self.update_count == 0:
            self.rescale_states()
            return True
        return False

    def minibatch_ids(self, uniforms):
        """generateMiniBatch (agent.cpp.base:574-597) for given uniforms."""
        ids = [int(np.floor(f32(f32(u) * f32(self.size() - 1)))) for u in uniforms]
        return sorted(ids)

    def train_policy(self, mb):
        """VRACER::trainPolicy (VRACER.cpp.base:65-87) for a given sorted mini-batch;
        returns (G, grad) for inspection."""
        er, A, B = self.er, self.A, len(mb)
        X = np.stack([er["state"][i] for i in mb])
        out, acts = forward(self.theta, X, self.S, self.H, self.L, A, self.noise, self.shift())
        # updateExperienceMetadata (agent.cpp.base:599-735)
        delta = 0
        for b in range(B):
            if b > 0 and mb[b] == mb[b - 1]:
                continue
            e = mb[b]
            cur = out[b, 1:]
            iw = importance_weight(er["action"][e], cur, er["exp_pol"][e], A, self.bounds)
            tiw = min(self.iw_trunc, iw)
            onp = bool(iw > f32(1.0) / self.cutoff and iw < self.cutoff)
            if er["onp"][e] and not onp:
                delta += 1
            if not er["onp"][e] and onp:
                delta -= 1
            er["cur_pol"][e] = cur.copy()
            er["v"][e] = out[b, 0]
            er["tv"][e] = f32(0.0)
            er["iw"][e] = iw
            er["onp"][e] = onp
            er["tiw"][e] = tiw
        for b in range(B):
            if b > 0 and mb[b] == mb[b - 1]:
                continue
            e = mb[b]
            if er["term"][e] == TRUNCATED:
                er["tv"][e] = self.policy(er["tstate"][e])[0, 0]
        self.off_count += delta
        self.off_ratio = f32(f32(self.off_count) / f32(self.size()))
        self.cutoff = f32(self.cutoff_scale / f32(f32(1.0) + f32(self.anneal * f32(self.update_count))))
        rmb = [mb[B - 1]] + [mb[i] for i in range(B - 2, -1, -1) if er["ep_id"][mb[i]] != er["ep_id"][mb[i + 1]]]
        for end in rmb:
            start = max(end - er["ep_pos"][end], 0)
            ret = f32(0.0)
            if er["term"][end] == TRUNCATED:
                ret = er["tv"][end]
            if er["term"][end] == NON_TERMINAL:
                ret = er["ret"][end + 1]
            for c in range(end, start - 1, -1):
                v = er["v"][c]
                ret = f32(v + f32(er["tiw"][c] * f32(f32(self.scaled_reward(c) + f32(self.gamma * ret)) - v)))
                er["ret"][c] = ret
        # calculatePolicyGradients (VRACER.cpp.base:89-181)
        G = np.zeros((B, 1 + 2 * A), f32)
        for b, e in enumerate(mb):
            V, cur, old = er["v"][e], er["cur_pol"][e], er["exp_pol"][e]
            G[b, 0] = f32(er["ret"][e] - V)
            if er["onp"][e]:
                q = self.scaled_reward(e)
                if er["term"][e] == NON_TERMINAL:
                    q = f32(q + f32(self.gamma * er["ret"][e + 1]))
                if er["term"][e] == TRUNCATED:
                    q = f32(q + f32(self.gamma * er["tv"][e]))
                loss = f32(q - V)
                pg = importance_weight_gradient(er["action"][e], cur, old, A, self.bounds)
                G[b, 1:] = (self.beta * loss * pg).astype(f32)
            klg = kl_gradient(old, cur, A, self.bounds)
            G[b, 1:] = (G[b, 1:] + f32(-(f32(1.0) - self.beta)) * klg).astype(f32)
        if not np.all(np.isfinite(G)):
            raise FloatingPointError("Gradient loss returned an invalid value")
        # DeepSupervisor::runGeneration (deepSupervisor.cpp.base:97-161), Direct Gradient
        grad = backward(self.theta, acts, out, G, self.S, self.H, self.L, A, self.noise, self.shift())
        if self.l2[0]:
            grad = (grad - self.l2[1] * self.theta).astype(f32)
        self.adam.eta = self.lr
        self.theta = self.adam.step(self.theta, grad)
        # agent.cpp.base:221-231
        self.update_count += 1
        self.lr = f32(self.lr0 / f32(f32(1.0) + f32(self.anneal * f32(self.update_count))))
        if self.off_ratio > self.off_target:
            self.beta = f32(f32(f32(1.0) - self.lr) * self.beta)
        else:
            self.beta = f32(f32(f32(f32(1.0) - self.lr) * self.beta) + self.lr)
        return G, grad


# ------------------------------------------------------------- environment
class CartPole:
    """examples/learning/reinforcement/cartpole/_model/cartpole.py: numpy-seeded
    reset and scipy's `ode(system).set_integrator('dopri5')` advance, restated
    below (dopri5_advance); pinned by tests/golden/cartpole_dopri5.json,
    which the reference's own module produced (tools/make_cartpole_golden.py)."""

    dt, x_threshold, th_threshold = 0.02, 2.4, np.pi / 15

    def __init__(self):
        self.u = np.zeros(4)
        self.t = 0.0
        self.step = 0

    def reset(self, seed):
        rs = np.random.RandomState(seed)
        self.u = rs.uniform(-0.05, 0.05, 4)
        self.t = 0.0
        self.step = 0

    @staticmethod
    def system(y, act):
        # cartpole.py:37-46, the same operation order (w**2 and costh**2 squared first)
        mp, mc, l, g = 0.1, 1.0, 0.5, 9.81
        x, v, th, w = y
        c, s = np.cos(th), np.sin(th)
        tot = mp + mc
        tmp = (act + l * (w * w) * s) / tot
        wdot = (g * s - c * tmp) / (l * (4.0 / 3.0 - mp * (c * c) / tot))
        vdot = tmp - l * wdot * c / tot
        return [float(v), float(vdot), float(w), float(wdot)]

    def failed(self):
        return abs(self.u[0]) > self.x_threshold or abs(self.u[2]) > self.th_threshold

    def advance(self, action):
        # cartpole.py:48-62: F clipped to [-10, 10], ODE from t to t + dt
        F = min(max(float(action), -10.0), 10.0)
        self.u = np.array(dopri5_advance(lambda y: self.system(y, F), [float(v) for v in self.u], self.t,
                                         self.t + self.dt))
        self.t = self.t + self.dt
        self.step += 1
        return self.failed()

    def reward(self, env_id):
        r = 1.0 - 1.0 * self.failed()
        return (r, r - 1.0, r * 0.1)[env_id % 3]


def testing_episodes(theta, sample_ids, launch_ids, S, H, L, A, initial_noise, max_steps, clipped=False, lb=None,
                     ub=None):
    """Agent::testingGeneration (agent.cpp.base:267-289) with the CartPole
    environment: ReinforcementLearning::runTestingEpisode
    (reinforcementLearning.cpp.base:207-255) adds environment 0's reward (the
    testing branch of env.py) of every step taken with the policy's mode
    (continuous.cpp.base:219-260: Normal mean; Clipped Normal: clipped to
    the bounds) until the pole falls or max_steps; reset seed
    sample_id * 1024 + launch_id (env.py).  Returns the cumulative rewards."""
    rewards = []
    for sid, lid in zip(sample_ids, launch_ids):
        cp = CartPole()
        cp.reset(int(sid) * 1024 + int(lid))
        total = f32(0.0)
        for _ in range(max_steps):
            out, _ = forward(theta, cp.u.astype(f32)[None, :], S, H, L, A, initial_noise)
            act = out[0, 1]
            if clipped:  # (continuous.cpp.base:242-252's order)
                if act >= f32(ub):
                    act = f32(ub)
                if act <= f32(lb):
                    act = f32(lb)
            done = cp.advance(float(act))
            total = f32(total + f32(cp.reward(0)))
            if done:
                break
        rewards.append(total)
    return np.array(rewards, f32)


# scipy.integrate.ode 'dopri5' = E. Hairer & G. Wanner's DOPRI5 (dopri5.f,
# Dormand-Prince 5(4)), as scipy calls it for one integrate(): rtol 1e-6,
# atol 1e-12 (scalars: ITOL 0), WORK = (UROUND 0 -> 2.3e-16, SAFE 0.9,
# FAC1 0.2, FAC2 10, BETA 0 -> 0.04, HMAX 0 -> XEND - X, H 0 -> HINIT),
# NMAX 500, no dense output.  Stiffness detection only prints, so it is left
# out.  Fortran's left-to-right evaluation order is kept term by term.
DP_C2, DP_C3, DP_C4, DP_C5 = 0.2, 0.3, 0.8, 8.0 / 9.0
DP_A21 = 0.2
DP_A31, DP_A32 = 3.0 / 40.0, 9.0 / 40.0
DP_A41, DP_A42, DP_A43 = 44.0 / 45.0, -56.0 / 15.0, 32.0 / 9.0
DP_A51, DP_A52, DP_A53, DP_A54 = 19372.0 / 6561.0, -25360.0 / 2187.0, 64448.0 / 6561.0, -212.0 / 729.0
DP_A61, DP_A62, DP_A63, DP_A64, DP_A65 = 9017.0 / 3168.0, -355.0 / 33.0, 46732.0 / 5247.0, 49.0 / 176.0, \
    -5103.0 / 18656.0
DP_A71, DP_A73, DP_A74, DP_A75, DP_A76 = 35.0 / 384.0, 500.0 / 1113.0, 125.0 / 192.0, -2187.0 / 6784.0, 11.0 / 84.0
DP_E1, DP_E3, DP_E4, DP_E5, DP_E6, DP_E7 = 71.0 / 57600.0, -71.0 / 16695.0, 71.0 / 1920.0, -17253.0 / 339200.0, \
    22.0 / 525.0, -1.0 / 40.0
DP_RTOL, DP_ATOL, DP_UROUND, DP_SAFE, DP_FAC1, DP_FAC2, DP_BETA, DP_NMAX = 1e-6, 1e-12, 2.3e-16, 0.9, 0.2, 10.0, \
    0.04, 500


def dopri5_hinit(f, x, y, f0, hmax):
    """DOPRI5's HINIT (initial step: explicit Euler probe, order 5)."""
    n = len(y)
    dnf = dny = 0.0
    for i in range(n):
        sk = DP_ATOL + DP_RTOL * abs(y[i])
        dnf = dnf + (f0[i] / sk) ** 2
        dny = dny + (y[i] / sk) ** 2
    h = 1.0e-6 if (dnf <= 1.0e-10 or dny <= 1.0e-10) else math.sqrt(dny / dnf) * 0.01
    h = min(h, hmax)
    y1 = [y[i] + h * f0[i] for i in range(n)]
    f1 = f(y1)
    der2 = 0.0
    for i in range(n):
        sk = DP_ATOL + DP_RTOL * abs(y[i])
        der2 = der2 + ((f1[i] - f0[i]) / sk) ** 2
    der2 = math.sqrt(der2) / h
    der12 = max(abs(der2), math.sqrt(dnf))
    h1 = max(1.0e-6, abs(h) * 1.0e-3) if der12 <= 1.0e-15 else (0.01 / der12) ** (1.0 / 5)
    return min(100 * abs(h), h1, hmax)


def dopri5_advance(f, y, x, xend):
    """DOPRI5's DOPCOR from x to xend (forward): returns y(xend)."""
    n = len(y)
    y = list(y)
    expo1 = 0.2 - DP_BETA * 0.75
    facc1, facc2 = 1.0 / DP_FAC1, 1.0 / DP_FAC2
    facold = 1.0e-4
    hmax = abs(xend - x)
    k1 = f(y)
    h = dopri5_hinit(f, x, y, k1, hmax)
    last, reject, naccpt, nstep = False, False, 0, 0
    while True:
        if nstep > DP_NMAX:
            raise RuntimeError("dopri5: more than NMAX steps")
        if 0.1 * abs(h) <= abs(x) * DP_UROUND:
            raise RuntimeError("dopri5: step size too small")
        if (x + 1.01 * h - xend) > 0.0:
            h = xend - x
            last = True
        nstep += 1
        y1 = [y[i] + h * DP_A21 * k1[i] for i in range(n)]
        k2 = f(y1)
        y1 = [y[i] + h * (DP_A31 * k1[i] + DP_A32 * k2[i]) for i in range(n)]
        k3 = f(y1)
        y1 = [y[i] + h * (DP_A41 * k1[i] + DP_A42 * k2[i] + DP_A43 * k3[i]) for i in range(n)]
        k4 = f(y1)
        y1 = [y[i] + h * (DP_A51 * k1[i] + DP_A52 * k2[i] + DP_A53 * k3[i] + DP_A54 * k4[i]) for i in range(n)]
        k5 = f(y1)
        ysti = [y[i] + h * (DP_A61 * k1[i] + DP_A62 * k2[i] + DP_A63 * k3[i] + DP_A64 * k4[i] + DP_A65 * k5[i])
                for i in range(n)]
        xph = x + h
        k6 = f(ysti)
        y1 = [y[i] + h * (DP_A71 * k1[i] + DP_A73 * k3[i] + DP_A74 * k4[i] + DP_A75 * k5[i] + DP_A76 * k6[i])
              for i in range(n)]
        k2 = f(y1)
        k4 = [(DP_E1 * k1[i] + DP_E3 * k3[i] + DP_E4 * k4[i] + DP_E5 * k5[i] + DP_E6 * k6[i] + DP_E7 * k2[i]) * h
              for i in range(n)]
        err = 0.0
        for i in range(n):
            sk = DP_ATOL + DP_RTOL * max(abs(y[i]), abs(y1[i]))
            err = err + (k4[i] / sk) ** 2
        err = math.sqrt(err / n)
        fac11 = err ** expo1
        fac = fac11 / facold ** DP_BETA
        fac = max(facc2, min(facc1, fac / DP_SAFE))
        hnew = h / fac
        if err <= 1.0:
            facold = max(err, 1.0e-4)
            naccpt += 1
            k1, y = k2, y1
            x = xph
            if last:
                return y
            if abs(hnew) > hmax:
                hnew = hmax
            if reject:
                hnew = min(abs(hnew), abs(h))
            reject = False
        else:
            hnew = h / min(facc1, fac11 / DP_SAFE)
            reject = True
            last = False
        h = hnew


# ------------------------------------------------------ counter-based streams
def philox4x32(c, k0, k1):
    """philox4x32-10 (Salmon et al., SC'11), as kg_vracer.hip's philox4x32."""
    M = 0xFFFFFFFF
    x, y, z, w = c
    for _ in range(10):
        p0, p1 = 0xD2511F53 * x, 0xCD9E8D57 * z
        x, y, z, w = ((p1 >> 32) ^ y ^ k0) & M, p1 & M, ((p0 >> 32) ^ w ^ k1) & M, p0 & M
        k0, k1 = (k0 + 0x9E3779B9) & M, (k1 + 0xBB67AE85) & M
    return x, y, z, w


def philox_normals(seed, purpose, a, b):
    r = philox4x32((a & 0xFFFFFFFF, a >> 32, b, purpose), seed & 0xFFFFFFFF, seed >> 32)
    u1 = (r[0] + 1.0) * 2.3283064365386963e-10
    u2 = r[1] * 2.3283064365386963e-10
    rad = np.sqrt(-2.0 * np.log(u1))
    return f32(rad * np.cos(6.283185307179586 * u2)), f32(rad * np.sin(6.283185307179586 * u2))


def philox_uniform24(seed, ctr):
    r = philox4x32((ctr & 0xFFFFFFFF, ctr >> 32, 0, 0x4D42), seed & 0xFFFFFFFF, seed >> 32)
    return f32(f32(r[0] >> 8) * f32(5.9604644775390625e-08))


def action_noise(seed, env_step, E, A):
    """The device's action-noise stream: normals of environment e, action i
    from block (env_step, e * 4 + i) (two normals per block)."""
    z = np.zeros((E, A), f32)
    for e in range(E):
        for i in range(0, A, 2):
            n0, n1 = philox_normals(seed, 0x4E4F, env_step, e * 4 + i)
            z[e, i] = n0
            if i + 1 < A:
                z[e, i + 1] = n1
    return z


def minibatch_uniforms(seed, ctr, B):
    return [philox_uniform24(seed, ctr + i) for i in range(B)]


# ------------------------------------------------ concurrent environments
class Rollouts:
    """Agent::trainingGeneration's concurrent environments (agent.cpp.base:176-199)
    with the CartPole env of env.py: every running environment takes one action
    per step; environments whose episode ended are processed in environment
    order and relaunched with the next sample ids (launch id = sample id)."""

    def __init__(self, agent, E, env_count=3, max_steps=500):
        self.agent, self.E, self.env_count, self.T = agent, E, env_count, max_steps
        self.carts = [CartPole() for _ in range(E)]
        self.sample = list(range(E))
        for e in range(E):
            self._launch(e, e)
        self.next_sample = E

    def _launch(self, e, sid):
        self.carts[e].reset(sid * 1024 + sid)
        self.sample[e] = sid
        # the State Rescaling moments the episode runs with (agent.cpp.base:186-187)
        self.pm = getattr(self, "pm", [None] * self.E)
        self.ps = getattr(self, "ps", [None] * self.E)
        self.pm[e], self.ps[e] = self.agent.smean.copy(), self.agent.ssdev.copy()
        self.buf = getattr(self, "buf", [None] * self.E)
        self.buf[e] = dict(states=[], actions=[], rewards=[], pols=[], vals=[], cum=f32(0.0))

    def env_id(self, e):
        return self.sample[e] % self.env_count

    def scaled_state(self, e, u):
        """requestNewPolicy's normalisation (reinforcementLearning.cpp.base:361-370)"""
        return ((u.astype(f32) - self.pm[e]) / self.ps[e]).astype(f32)

    def relaunched_take_moments(self):
        """the reference relaunches finished agents at the top of the next loop
        iteration, after a rescaling in this one: environments that have not
        acted since their relaunch take the current moments"""
        for e, c in enumerate(self.carts):
            if c.step == 0:
                self.pm[e], self.ps[e] = self.agent.smean.copy(), self.agent.ssdev.copy()

    def step(self, noise):
        A, ag = self.agent.A, self.agent
        X = np.stack([self.scaled_state(e, c.u) for e, c in enumerate(self.carts)])
        out = ag.policy(X)
        finished = []
        for e, cart in enumerate(self.carts):
            b = self.buf[e]
            act = np.array([f32(out[e, 1 + i] + f32(out[e, 1 + A + i] * f32(noise[e, i]))) for i in range(A)], f32)
            if ag.bounds is not None:  # continuous.cpp.base:172-183
                act = np.minimum(np.maximum(act, ag.bounds[0]), ag.bounds[1]).astype(f32)
            b["states"].append(X[e].copy())
            b["actions"].append(act)
            b["pols"].append(out[e, 1:].copy())
            b["vals"].append(out[e, 0])
            failed = cart.advance(act[0])
            r = f32(cart.reward(self.env_id(e)))
            b["rewards"].append(r)
            b["cum"] = f32(b["cum"] + r)
            if failed:
                finished.append((e, TERMINAL))
            elif cart.step >= self.T:
                finished.append((e, TRUNCATED))
        new, rewards = 0, []
        for e, term in finished:
            b = self.buf[e]
            ag.process_episode(self.env_id(e), b["states"], b["actions"], b["rewards"], b["pols"], b["vals"], term,
                               tstate=self.scaled_state(e, self.carts[e].u))
            new += len(b["rewards"])
            rewards.append(b["cum"])
        for e, _ in finished:
            self._launch(e, self.next_sample)
            self.next_sample += 1
        return new, rewards
