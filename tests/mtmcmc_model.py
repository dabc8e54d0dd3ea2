"""The reference's mTMCMC example as plain numpy, for the oracle / device
parity tests: examples/bayesian.inference/reference/run-mtmcmc.py with
_model/model.py:modelWithGradients (y = a x + b, standard deviation sig,
three Uniform(0, 5) priors) and the Normal likelihood of
problem/bayesian/reference/reference.cpp.base (loglikelihood :57-79,
gradient :251-286, Fisher information :533-566), in the reference's
operation order."""
import numpy as np

X = np.array([1.0, 2.0, 3.0, 4.0, 5.0])
Y = np.array([3.21, 4.14, 4.94, 6.06, 6.84])
LOG2PI = 1.83787706640934533908193770912476
PMIN, PMAX = 0.0, 5.0


def log_prior(th):
    """Bayesian::evaluateLogPrior with Univariate/Uniform priors: sum of
    -log(max - min) inside the support, -inf outside."""
    lp = 0.0
    for v in th:
        lp += -np.log(PMAX - PMIN) if (PMIN <= v <= PMAX) else -np.inf
    return lp


def model(th):
    a, b, sig = th
    f = a * X + b
    g = np.full(X.size, sig)
    gF = np.stack([X, np.ones_like(X), np.zeros_like(X)], axis=1)
    gG = np.tile(np.array([0.0, 0.0, 1.0]), (X.size, 1))
    return f, g, gF, gG


def loglik(th):
    f, g, _, _ = model(th)
    sse = 0.0
    for i in range(X.size):
        diff = (Y[i] - f[i]) / g[i]
        sse += diff * diff
    ll = 0.0
    for i in range(X.size):
        ll -= np.log(max(g[i], 1e-11))
    return ll - 0.5 * (X.size * LOG2PI + sse)


def gradient(th):
    f, g, gF, gG = model(th)
    out = np.zeros(3)
    for i in range(X.size):
        inv = 1.0 / g[i]
        inv2 = inv * inv
        inv3 = inv2 * inv
        dif = Y[i] - f[i]
        for d in range(3):
            out[d] += -inv * gG[i][d] + inv2 * dif * gF[i][d] + inv3 * dif * dif * gG[i][d]
    return out


def fisher(th):
    f, g, gF, gG = model(th)
    F = np.zeros((3, 3))
    for i in range(X.size):
        var = g[i] * g[i]
        vinv = 1.0 / var
        for k in range(3):
            for l in range(k):
                t = vinv * gF[i][k] * gF[i][l] + 2.0 * vinv * gG[i][k] * gG[i][l]
                F[k, l] += t
                F[l, k] += t
            F[k, k] += vinv * gF[i][k] * gF[i][k] + 2.0 * vinv * gG[i][k] * gG[i][k]
    return F


def evaluate(cands):
    """(log-priors, log-likelihoods, gradients, Fisher informations) of P
    candidates; the likelihood and its derivatives only where the prior is
    finite (Bayesian::evaluate skips the model otherwise)."""
    P = cands.shape[0]
    lp, ll = np.empty(P), np.empty(P)
    gr, fim = np.zeros((P, 3)), np.zeros((P, 3, 3))
    for c in range(P):
        lp[c] = log_prior(cands[c])
        if np.isfinite(lp[c]):
            ll[c] = loglik(cands[c])
            gr[c] = gradient(cands[c])
            fim[c] = fisher(cands[c])
        else:
            ll[c] = -np.inf
    return lp, ll, gr, fim
