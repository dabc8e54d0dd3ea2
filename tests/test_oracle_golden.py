"""Pin the CPU oracle (oracle/refcpu.c) against the reference's own committed
generation files (golden vectors, tests/golden/).  Every comparison here is
bit-exact (np.array_equal on float64).

CMA-ES fixture: reference tests/python/plot/cmaes, N=10, lambda=32, mu=16,
Logarithmic weights, seeds Normal 790510 / Uniform 790511, bounds +-25.
TMCMC fixture: reference tests/python/plot/tmcmc, N=3, P=50, TargetCOV 0.8.
"""
import numpy as np
import pytest

import refcpu as R
from golden_util import (CMAES_STATE_SCALARS, CMAES_STATE_VECTORS, cmaes_variables, load_cmaes, load_tmcmc,
                         population)

CM = load_cmaes()
TM = load_tmcmc()
N, LAM, MU = 10, 32, 16


def by_gen(gens, g):
    for x in gens:
        if x["Current Generation"] == g:
            return x
    raise KeyError(g)


def cmaes_from_fixture(g):
    """Oracle CMA-ES handle holding the full state saved after generation g."""
    st = by_gen(CM, g)
    o = R.CMAES(N, LAM, MU)
    o.option("Max Infeasible Resamplings", 10000)
    for k, v in cmaes_variables(st).items():
        o[k] = v
    s = st["Solver"]
    for k in CMAES_STATE_VECTORS:
        o[k] = s[k]
    for k in CMAES_STATE_SCALARS:
        o[k] = s[k]
    o.rng(0).from_hex(s["Normal Generator"]["Range"])
    o.rng(1).from_hex(s["Uniform Generator"]["Range"])
    return o


def test_mt19937_seeding_matches_fixture():
    s = by_gen(CM, 0)["Solver"]
    # gen 0 is written before the solver ran: its RNGs are freshly seeded
    for name, seed in (("Normal Generator", 790510), ("Uniform Generator", 790511)):
        r = R.Rng(seed=seed)
        assert r.to_hex() == s[name]["Range"]


def test_tmcmc_seeding_matches_fixture():
    g0 = TM[0]
    for dist in g0["Distributions"]:
        r = R.Rng(seed=dist["Random Seed"] & 0xFFFFFFFF)
        assert r.to_hex() == dist["Range"]
    for name in ("Multinomial Generator", "Multivariate Generator", "Uniform Generator"):
        gs = g0["Solver"][name]
        assert R.Rng(seed=gs["Random Seed"] & 0xFFFFFFFF).to_hex() == gs["Range"]


def test_hypot_is_fdlibm():
    L = R.lib()
    assert L.kr_hypot(3.0, 4.0) == 5.0
    assert L.kr_hypot(0.0, 0.0) == 0.0
    assert L.kr_hypot(1e300, 1e300) == pytest.approx(1.4142135623730951e300, rel=1e-15)
    assert L.kr_hypot(1e-310, 0.0) == 1e-310
    assert np.isinf(L.kr_hypot(np.inf, np.nan))


@pytest.mark.parametrize("k", range(1, 100))
def test_eigensystem_bit_exact(k):
    """gen k's C -> gen k+1's B (Covariance Eigenvector Matrix) and D."""
    C = np.array(by_gen(CM, k)["Solver"]["Covariance Matrix"]).reshape(N, N)
    nxt = by_gen(CM, k + 1)["Solver"]
    A = np.tril(C) + np.tril(C, -1).T
    ev, Q = R.eigen_symmv(A)
    assert np.array_equal(Q.reshape(-1), np.array(nxt["Covariance Eigenvector Matrix"]))
    assert np.array_equal(np.sqrt(ev), np.array(nxt["Axis Lengths"]))


@pytest.mark.parametrize("k", [1, 2, 19, 49, 99])
def test_cmaes_generation_teacher_forced(k):
    """State after gen k + gen k+1's fitness values -> gen k+1 bit-exact:
    eigensystem, the whole population (MT19937 + polar + B*D*z), sorting
    index, mean, paths, covariance, sigma."""
    o = cmaes_from_fixture(k)
    nxt = by_gen(CM, k + 1)["Solver"]
    o.prepare()
    assert np.array_equal(o["Covariance Eigenvector Matrix"], np.array(nxt["Covariance Eigenvector Matrix"]))
    assert np.array_equal(o["Sample Population"], population(by_gen(CM, k + 1)).reshape(-1))
    assert o["Infeasible Sample Count"][0] == nxt["Infeasible Sample Count"]
    o["Value Vector"] = nxt["Value Vector"]
    o.update(k + 1)
    assert list(o.sorting_index()) == nxt["Sorting Index"]
    for key in ("Current Mean", "Previous Mean", "Evolution Path", "Conjugate Evolution Path", "Covariance Matrix"):
        assert np.array_equal(o[key], np.array(nxt[key])), key
    for key in ("Sigma", "Conjugate Evolution Path L2 Norm", "Best Ever Value", "Current Best Value",
                "Maximum Diagonal Covariance Matrix Element", "Minimum Diagonal Covariance Matrix Element",
                "Current Min Standard Deviation", "Current Max Standard Deviation"):
        assert o[key][0] == nxt[key], key


def test_cmaes_values_are_negative_sphere():
    """The fixture objective is F = -0.5*sum(x^2); check the builtin."""
    st = by_gen(CM, 5)["Solver"]
    X = np.array(st["Sample Population"])
    F = [R.objective("sphere", x) for x in X]
    assert np.array_equal(np.array(F), np.array(st["Value Vector"]))


def test_cmaes_initialize_matches_gen1_constants():
    st1 = by_gen(CM, 1)
    o = R.CMAES(N, LAM, MU)
    for k, v in cmaes_variables(st1).items():
        o[k] = v
    o.initialize()
    s = st1["Solver"]
    for key in ("Effective Mu", "Cumulative Covariance", "Sigma Cumulation Factor", "Damp Factor",
                "Chi Square Number", "Trace"):
        assert o[key][0] == s[key], key
    assert np.array_equal(o["Mu Weights"], np.array(s["Mu Weights"]))


def test_cmaes_full_run_from_seed_reproduces_fixture():
    """Seeded from scratch (experiment seed 790510), the oracle reproduces
    generations 1..100 of the fixture with the fixture objective."""
    st0 = by_gen(CM, 0)
    o = R.CMAES(N, LAM, MU)
    o.option("Max Infeasible Resamplings", 10000)
    for k, v in cmaes_variables(st0).items():
        o[k] = v
    R.lib().kr_rng_seed(o.rng(0).ptr, 790510)
    R.lib().kr_rng_seed(o.rng(1).ptr, 790511)
    for g in range(1, 101):
        o.generation(g, "sphere")
        s = by_gen(CM, g)["Solver"]
        assert list(o.sorting_index()) == s["Sorting Index"], g
        assert np.array_equal(o["Sample Population"], population(by_gen(CM, g)).reshape(-1)), g
        assert np.array_equal(o["Covariance Matrix"], np.array(s["Covariance Matrix"])), g
        assert o["Sigma"][0] == s["Sigma"], g
    assert o.rng(0).to_hex() == by_gen(CM, 100)["Solver"]["Normal Generator"]["Range"]


# ------------------------------------------------------------------ TMCMC
TN, TP = 3, 50


def tmcmc_from_fixture(g):
    st = by_gen(TM, g)
    s = st["Solver"]
    o = R.TMCMC(TN, TP)
    o.option("Target Coefficient Of Variation", s["Target Coefficient Of Variation"])
    o.option("Covariance Scaling", s["Covariance Scaling"])
    o["Prior Minimum"] = [d["Minimum"] for d in st["Distributions"]]
    o["Prior Maximum"] = [d["Maximum"] for d in st["Distributions"]]
    for k in ("Chain Leaders", "Chain Leaders LogLikelihoods", "Chain Leaders LogPriors", "Covariance Matrix",
              "Chain Lengths"):
        if len(s[k]):
            o[k] = s[k]
    for k in ("Annealing Exponent", "Previous Annealing Exponent", "LogEvidence", "Chain Count"):
        o[k] = s[k]
    o.rng(0).from_hex(s["Multinomial Generator"]["Range"])
    o.rng(1).from_hex(s["Multivariate Generator"]["Range"])
    o.rng(2).from_hex(s["Uniform Generator"]["Range"])
    for i, d in enumerate(st["Distributions"]):
        o.rng(3 + i).from_hex(d["Range"])
    return o


@pytest.mark.parametrize("k", range(0, 7))
def test_tmcmc_generation_teacher_forced(k):
    """State after gen k + gen k+1's candidate log-likelihoods (the reference
    problem used a Python model) -> gen k+1 bit-exact: Cholesky + candidate
    draws, accept/reject, annealing exponent (nmsimplex), log-evidence,
    multinomial resampling -> chain leaders, mean and covariance."""
    o = tmcmc_from_fixture(k)
    nxt = by_gen(TM, k + 1)["Solver"]
    g = k + 1
    if g == 1:
        o.initialize()
    o.prepare(g)
    cand = np.array(nxt["Chain Candidates"]).reshape(-1)
    assert np.array_equal(o["Chain Candidates"], cand)
    o["Chain Candidates LogLikelihoods"] = nxt["Chain Candidates LogLikelihoods"]
    o["Chain Candidates LogPriors"] = nxt["Chain Candidates LogPriors"]
    o.process_candidates(g)
    assert o["Accepted Samples Count"][0] == nxt["Accepted Samples Count"]
    assert np.array_equal(o["Sample LogLikelihood Database"], np.array(nxt["Sample LogLikelihood Database"]))
    o.process_generation()
    for key in ("Annealing Exponent", "LogEvidence", "Coefficient Of Variation", "Max Loglikelihood",
                "Selection Acceptance Rate", "Proposals Acceptance Rate", "Chain Count"):
        assert o[key][0] == nxt[key], key
    for key in ("Chain Leaders", "Chain Leaders LogLikelihoods", "Chain Lengths", "Covariance Matrix", "Mean Theta"):
        assert np.array_equal(o[key], np.array(nxt[key]).reshape(-1)), key
    assert o.rng(0).to_hex() == nxt["Multinomial Generator"]["Range"]
    assert o.rng(1).to_hex() == nxt["Multivariate Generator"]["Range"]
    assert o.rng(2).to_hex() == nxt["Uniform Generator"]["Range"]


def test_binomial_btpe_statistics():
    """BTPE branch (n*p >= 14) is pinned by no fixture: check moments."""
    r = R.Rng(seed=1337)
    L = R.lib()
    n, p = 2000, 0.3
    xs = np.array([L.kr_ran_binomial(r.ptr, p, n) for _ in range(20000)], dtype=np.float64)
    assert abs(xs.mean() - n * p) < 0.5
    assert abs(xs.var() / (n * p * (1 - p)) - 1.0) < 0.05
    assert xs.min() >= 0 and xs.max() <= n


def test_multinomial_conserves_total():
    r = R.Rng(seed=7)
    w = np.random.default_rng(3).random(8192)
    w /= w.sum()
    n = R.multinomial(r, w, 8192)
    assert int(n.sum()) == 8192


def _decimal_cos(x):
    """cos(x) to ~70 digits (decimal Taylor after reduction by a 110-digit
    pi/2): the exact value the correctly-rounded cos must round."""
    from decimal import Decimal as D, localcontext
    with localcontext() as ctx:
        ctx.prec = 80
        pi = D("3.14159265358979323846264338327950288419716939937510582097494459230781640628620899862803482534211706798")
        xd = D(x)
        k = (xd / (pi / 2)).to_integral_value()
        r = xd - k * (pi / 2)
        q = int(k) % 4
        odd = q % 2 == 1
        s, t, n = D(0), (r if odd else D(1)), (1 if odd else 0)
        while abs(t) > D(10) ** -75:
            s += t
            t = -t * r * r / ((n + 1) * (n + 2))
            n += 2
        return float(-s if q in (1, 2) else s)


def test_cos_is_correctly_rounded():
    """kr_cos_cr (the Ackley objective's cos; the device runs the same
    sequence) equals the correctly rounded cos, including arguments next
    to multiples of pi/2 that 2*pi*x produces for x on a quarter grid."""
    import ctypes
    f = R.lib().kr_cos_cr
    f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
    rng = np.random.default_rng(11)
    xs = list(rng.uniform(-80, 80, 400)) + list(2 * np.pi * np.arange(-40, 41) / 4) + [0.0, 1e-300, -3e-9]
    for x in xs:
        assert f(float(x)) == _decimal_cos(float(x)), x


def test_oracle_mtmcmc_posterior_of_the_reference_example():
    """The oracle's mTMCMC restatement on the reference's mTMCMC example
    (run-mtmcmc.py, P = 400): it reaches annealing exponent 1 with the
    gradient proposals in use and a posterior mean near the least-squares
    fit of the example's data (a = 0.907, b = 2.307).  Statistical only:
    no reference fixture covers mTMCMC."""
    from mtmcmc_model import evaluate
    N, P = 3, 400
    o = R.TMCMC(N, P)
    o["Prior Minimum"] = np.zeros(N)
    o["Prior Maximum"] = np.full(N, 5.0)
    o.option("Version", 1)
    o.option("Step Size", 0.1)
    o.option("Domain Extension Factor", 0.2)
    o.set_prior_map([0, 0, 0])
    for w in range(4):
        R.lib().kr_rng_seed(o.rng(w).ptr, 100 + w)
    for g in range(1, 40):
        if g == 1:
            o.initialize()
        o.prepare(g)
        lp, ll, gr, fim = evaluate(o["Chain Candidates"].reshape(P, N).copy())
        o["Chain Candidates LogPriors"] = lp
        o["Chain Candidates LogLikelihoods"] = ll
        if g > 1:
            o.set_gradients(gr, fim)
        o.process_candidates(g)
        o.process_generation()
        if o["Previous Annealing Exponent"][0] >= 1.0:
            break
    assert o["Previous Annealing Exponent"][0] >= 1.0
    assert np.count_nonzero(o["Chain Leaders Errors"] == 0) > P // 2
    m = o["Mean Theta"]
    assert abs(m[0] - 0.907) < 0.25 and abs(m[1] - 2.307) < 0.8 and 0.05 < m[2] < 2.0, m
    assert R.lib().kr_chi2inv_068(3) == 3.505882355768179


def test_oracle_discrete_variables_stay_on_their_grid():
    """The oracle's discrete-variable path (CMAES.cpp.base:515-544, :834-867)
    on examples/optimization/discrete/run-cmaes.py's setup: discrete
    coordinates on the integers, masks switching on as sigma shrinks, the
    Uniform Generator consumed only once discrete mutations exist."""
    Nv, lam = 10, 8
    o = R.CMAES(Nv, lam, 0)
    gran = np.zeros(Nv)
    gran[[0, 1, 3, 6]] = 1.0
    o["Initial Value"], o["Lower Bound"], o["Upper Bound"] = np.ones(Nv), np.full(Nv, -19.0), np.full(Nv, 21.0)
    o["Initial Standard Deviation"] = np.full(Nv, 12.0)
    o["Granularity"] = gran
    R.lib().kr_rng_seed(o.rng(0).ptr, 5)
    R.lib().kr_rng_seed(o.rng(1).ptr, 6)
    u0 = o.rng(1).get_bytes()
    o.generation(1, "sphere")
    assert o.rng(1).get_bytes() == u0  # no discrete mutations in generation 1
    seen = 0
    for g in range(1, 200):
        if g > 1:
            o.generation(g, "sphere")
        X = o["Sample Population"].reshape(lam, Nv)
        assert np.array_equal(X[:, gran > 0], np.round(X[:, gran > 0]))
        seen += o["Number Masking Matrix Entries"][0] > 0
        assert o["Number Of Discrete Mutations"][0] <= lam // 2 - 1
    assert seen > 0 and o.rng(1).get_bytes() != u0
