"""GPU parity: the HIP TMCMC path (through the C-ABI) against the oracle and
the reference's golden generation files (tests/python/plot/tmcmc).

Bar: bit-exact (np.array_equal / ==) for candidates, accept decisions, the
annealing exponent, coefficient of variation, log-evidence, multinomial
selections -> chain leaders, weighted mean and covariance, and the exported
GSL generator states.
"""
import numpy as np
import pytest

import refcpu as R
from golden_util import load_tmcmc

pytestmark = pytest.mark.gpu

TM = load_tmcmc()
TN, TP = 3, 50


def by_gen(g):
    for x in TM:
        if x["Current Generation"] == g:
            return x
    raise KeyError(g)


def fixture_device(g):
    from korali_amd.native import TmcmcDevice
    st = by_gen(g)
    s = st["Solver"]
    dev = TmcmcDevice(TN, TP, prior_min=[d["Minimum"] for d in st["Distributions"]],
                      prior_max=[d["Maximum"] for d in st["Distributions"]],
                      target_cov=s["Target Coefficient Of Variation"], covariance_scaling=s["Covariance Scaling"])
    for k in ("Chain Leaders", "Chain Leaders LogLikelihoods", "Chain Leaders LogPriors", "Covariance Matrix",
              "Chain Lengths"):
        if len(s[k]):
            dev[k] = s[k]
    for k in ("Annealing Exponent", "Previous Annealing Exponent", "LogEvidence", "Chain Count"):
        dev[k] = [s[k]]
    dev.set_rng(0, bytes.fromhex(s["Multinomial Generator"]["Range"]))
    dev.set_rng(1, bytes.fromhex(s["Multivariate Generator"]["Range"]))
    dev.set_rng(2, bytes.fromhex(s["Uniform Generator"]["Range"]))
    for i, d in enumerate(st["Distributions"]):
        dev.set_rng(3 + i, bytes.fromhex(d["Range"]))
    return dev


@pytest.mark.parametrize("k", range(0, 7))
def test_tmcmc_teacher_forced_generation_bit_exact(k):
    """Fixture state after gen k + gen k+1's candidate log-likelihoods (the
    reference problem used a Python model) -> gen k+1 on the device."""
    dev = fixture_device(k)
    nxt = by_gen(k + 1)["Solver"]
    g = k + 1
    dev.prepare(g)
    assert np.array_equal(dev["Chain Candidates"], np.array(nxt["Chain Candidates"]).reshape(-1))
    dev.set_evaluations(np.array(nxt["Chain Candidates LogPriors"]), np.array(nxt["Chain Candidates LogLikelihoods"]))
    dev.process(g)
    dev.synchronize()
    assert dev["Accepted Samples Count"][0] == nxt["Accepted Samples Count"]
    assert np.array_equal(dev["Sample LogLikelihood Database"], np.array(nxt["Sample LogLikelihood Database"]))
    for key in ("Annealing Exponent", "LogEvidence", "Coefficient Of Variation", "Max Loglikelihood",
                "Selection Acceptance Rate", "Proposals Acceptance Rate", "Chain Count"):
        assert dev[key][0] == nxt[key], key
    for key in ("Chain Leaders", "Chain Leaders LogLikelihoods", "Chain Lengths", "Covariance Matrix", "Mean Theta"):
        assert np.array_equal(dev[key], np.array(nxt[key]).reshape(-1)), key
    assert dev.get_rng(0).hex().upper() == nxt["Multinomial Generator"]["Range"]
    assert dev.get_rng(1).hex().upper() == nxt["Multivariate Generator"]["Range"]
    assert dev.get_rng(2).hex().upper() == nxt["Uniform Generator"]["Range"]


VEC_KEYS = ("Chain Candidates", "Chain Candidates LogLikelihoods", "Chain Candidates LogPriors", "Chain Leaders",
            "Chain Leaders LogLikelihoods", "Chain Leaders LogPriors", "Chain Lengths", "Mean Theta",
            "Covariance Matrix", "Sample Database", "Sample LogLikelihood Database", "Num Selections")
SCA_KEYS = ("Annealing Exponent", "Previous Annealing Exponent", "LogEvidence", "Coefficient Of Variation",
            "Max Loglikelihood", "Chain Count", "Accepted Samples Count", "Proposals Acceptance Rate",
            "Selection Acceptance Rate", "Model Evaluation Count", "Min Search Iterations")


def seeded_pair(N, P, shared, seed=1337, target_cov=1.0, max_chain_length=1, burn_in=0, per_generation_burn_in=()):
    """C3-style experiment: every variable with a U(-5, 5) prior, Gaussian
    loglik -0.5|x|^2; seeds in Korali's consumption order (distributions,
    then the solver's Multinomial, Multivariate, Uniform generators)."""
    from korali_amd.native import TmcmcDevice
    ndist = 1 if shared else N
    pdist = [0] * N if shared else list(range(N))
    seeds = [seed + k for k in range(ndist)]
    sm, sv, su = seed + ndist, seed + ndist + 1, seed + ndist + 2
    dev = TmcmcDevice(N, P, prior_min=[-5.0] * N, prior_max=[5.0] * N, prior_seeds=seeds, prior_distribution=pdist,
                      multinomial_seed=sm, multivariate_seed=sv, uniform_seed=su, target_cov=target_cov,
                      max_chain_length=max_chain_length, default_burn_in=burn_in,
                      per_generation_burn_in=per_generation_burn_in)
    o = R.TMCMC(N, P)
    o.option("Target Coefficient Of Variation", target_cov)
    o.option("Max Chain Length", max_chain_length)
    o.option("Default Burn In", burn_in)
    if len(per_generation_burn_in):
        o.set_per_generation_burn_in(per_generation_burn_in)
    o["Prior Minimum"] = [-5.0] * N
    o["Prior Maximum"] = [5.0] * N
    o.set_prior_map(pdist)
    for k in range(ndist):
        R.lib().kr_rng_seed(o.rng(3 + k).ptr, seeds[k])
    R.lib().kr_rng_seed(o.rng(0).ptr, sm)
    R.lib().kr_rng_seed(o.rng(1).ptr, sv)
    R.lib().kr_rng_seed(o.rng(2).ptr, su)
    return dev, o, ndist


@pytest.mark.parametrize("N,P,gens,shared", [(4, 256, 12, True), (3, 500, 10, False), (32, 2048, 6, True)])
def test_tmcmc_seeded_run_matches_oracle(N, P, gens, shared):
    dev, o, ndist = seeded_pair(N, P, shared)
    for g in range(1, gens + 1):
        dev.generation(g)
        o.generation(g)
        dev.synchronize()
        for key in VEC_KEYS:
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in SCA_KEYS:
            a, b = dev[key][0], o[key][0]
            assert a == b or (np.isnan(a) and np.isnan(b)), (g, key, a, b)
        if o["Annealing Exponent"][0] >= 1.0:
            break
    for which in range(3 + ndist):
        assert dev.get_rng(which).hex().upper() == o.rng(which).to_hex(), which


PRIOR_SETS = {
    # variable -> distribution, kind (enum kg_prior_kind), the two parameters
    "normal": ([0, 1, 2, 2], [1, 0, 1, 1], [0.5, -5.0, -1.0, -1.0], [2.0, 5.0, 0.7, 0.7]),
    "all": ([0, 1, 2, 3, 4, 4], [2, 3, 4, 5, 1, 1], [-1.0, 0.3, 0.0, 0.0, -1.0, -1.0], [2.0, 1.5, 0.5, 0.5, 0.7, 0.7]),
}


@pytest.mark.parametrize("mcl,burn,priors", [(1, 0, "normal"), (3, 1, "normal"), (1, 0, "all"), (2, 1, "all")])
def test_tmcmc_normal_priors_match_oracle(mcl, burn, priors):
    """Univariate/Normal priors (normal.cpp.base: mean + gsl_ran_gaussian(sd)
    draws at generation 1, log-density logNormalization - 0.5 d^2) mixed with
    Uniform ones, one Normal distribution shared by two variables (its draws
    interleave sample-major); and Exponential, Laplace, Cauchy and LogNormal
    priors beside a shared Normal: the whole run bit-exact vs the oracle, the
    prior generators' exported states included."""
    from korali_amd.native import TmcmcDevice
    pdist, kinds, pmin, pmax = PRIOR_SETS[priors]
    N, P, seed = len(pdist), 600, 2024
    nd = max(pdist) + 1
    seeds = [seed + k for k in range(nd)]
    sm, sv, su = seed + nd, seed + nd + 1, seed + nd + 2
    dev = TmcmcDevice(N, P, prior_min=pmin, prior_max=pmax, prior_seeds=seeds, prior_distribution=pdist,
                      prior_kind=kinds, multinomial_seed=sm, multivariate_seed=sv, uniform_seed=su,
                      max_chain_length=mcl, default_burn_in=burn)
    o = R.TMCMC(N, P)
    o.option("Max Chain Length", mcl)
    o.option("Default Burn In", burn)
    o["Prior Minimum"] = pmin
    o["Prior Maximum"] = pmax
    o.set_prior_map(pdist)
    o.set_prior_kinds(kinds)
    for k in range(nd):
        R.lib().kr_rng_seed(o.rng(3 + k).ptr, seeds[k])
    R.lib().kr_rng_seed(o.rng(0).ptr, sm)
    R.lib().kr_rng_seed(o.rng(1).ptr, sv)
    R.lib().kr_rng_seed(o.rng(2).ptr, su)
    for g in range(1, 9):
        dev.generation(g)
        o.generation(g)
        dev.synchronize()
        for key in VEC_KEYS:
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in SCA_KEYS:
            a, b = dev[key][0], o[key][0]
            assert a == b or (np.isnan(a) and np.isnan(b)), (g, key, a, b)
        if g == 1 and priors == "normal":  # the Normal variables' draws are unbounded and centred on the mean
            x = np.asarray(dev["Sample Database"]).reshape(-1, N)
            assert abs(x[:, 0].mean() - 0.5) < 0.3 and abs(x[:, 2].mean() + 1.0) < 0.15
        if g == 1 and priors == "all":  # Exponential >= location, LogNormal > 0, Laplace around its mean
            x = np.asarray(dev["Sample Database"]).reshape(-1, N)
            assert x[:, 0].min() >= -1.0 and x[:, 3].min() > 0 and abs(np.median(x[:, 1]) - 0.3) < 0.3
        if o["Annealing Exponent"][0] >= 1.0:
            break
    for which in range(3 + nd):
        assert dev.get_rng(which).hex().upper() == o.rng(which).to_hex(), which


@pytest.mark.parametrize("seed,target_cov", [(11, 0.5), (12, 2.0), (13, 1.0)])
def test_tmcmc_interval_search_equals_exact_search(monkeypatch, seed, target_cov):
    """The annealing search decides on interval estimates and falls back to
    the host's exact evaluation only when they overlap, with the simplex loop
    on the device (default: k_tm_nm_search, relaunched with host-exact
    values) or on the host (min_search): both runs must equal the all-exact
    search and the oracle."""
    N, P = 6, 1024
    runs = []
    # (device search: the symmetric form, k_tm_nm_sym, and the controller form, KORALI_AMD_NM_SYM=0)
    for exact, host, sym in (("0", "0", "1"), ("1", "0", "1"), ("0", "1", "1"), ("0", "0", "0")):
        monkeypatch.setenv("KORALI_AMD_TMCMC_EXACT_SEARCH", exact)
        monkeypatch.setenv("KORALI_AMD_TMCMC_HOST_SEARCH", host)
        monkeypatch.setenv("KORALI_AMD_NM_SYM", sym)
        dev, o, ndist = seeded_pair(N, P, shared=True, seed=seed, target_cov=target_cov)
        hist = []
        for g in range(1, 30):
            dev.generation(g)
            hist.append((dev["Annealing Exponent"][0], dev["Coefficient Of Variation"][0], dev["LogEvidence"][0],
                         dev["Covariance Matrix"].tobytes(), dev["Min Search Iterations"][0]))
            if dev["Annealing Exponent"][0] >= 1.0:
                break
        runs.append((hist, dev["Exact Search Evaluations"][0]))
        if exact == "0" and host == "0" and sym == "1":
            for g in range(1, len(hist) + 1):
                o.generation(g)
                assert o["Annealing Exponent"][0] == hist[g - 1][0], g
                assert o["Coefficient Of Variation"][0] == hist[g - 1][1], g
                assert o["LogEvidence"][0] == hist[g - 1][2], g
                assert o["Covariance Matrix"].tobytes() == hist[g - 1][3], g
    assert runs[0][0] == runs[1][0]
    assert runs[2][0] == runs[1][0]
    assert runs[3] == runs[0]  # the two device forms: the same searches, the same exact evaluations
    # the interval paths need far fewer exact host evaluations
    assert runs[0][1] < runs[1][1] and runs[2][1] < runs[1][1]


@pytest.mark.parametrize("N,P", [(6, 1000), (32, 1024), (3, 37)])
def test_row_chain_sums_and_deferred_tail_match_oracle(monkeypatch, N, P):
    """The weighted mean / covariance on row chains (k_tm_wsum_rows, P padded
    to the slot pitch) and the stored minimum's exact value formed on the
    host worker (HostTail) against the round-2 LDS-tile sums with the value
    formed before going on (KORALI_AMD_TM_WSUM=lds, KORALI_AMD_TM_DEFER_TAIL=0)
    and the oracle: the same bits every generation; the next generation's
    first-step normals formed ahead on the side stream leave the Multivariate
    generator where the plain order leaves it."""
    runs, states = [], []
    for wsum, defer in (("rows", "1"), ("lds", "0")):
        monkeypatch.setenv("KORALI_AMD_TM_WSUM", wsum)
        monkeypatch.setenv("KORALI_AMD_TM_DEFER_TAIL", defer)
        monkeypatch.setenv("KORALI_AMD_TM_NORMALS_AHEAD", defer)  # (first-step normals formed ahead, or not)
        dev, o, ndist = seeded_pair(N, P, shared=True, seed=5)
        hist = []
        for g in range(1, 40):
            dev.generation(g)
            hist.append((dev["Annealing Exponent"][0], dev["Coefficient Of Variation"][0], dev["LogEvidence"][0],
                         dev["Mean Theta"].tobytes(), dev["Covariance Matrix"].tobytes()))
            if wsum == "rows":
                o.generation(g)
                compare_state(dev, o, g)
            if dev["Annealing Exponent"][0] >= 1.0:
                break
        runs.append((hist, dev["Deferred Search Evaluations"][0]))
        states.append(bytes(dev.get_rng(1)))  # the Multivariate generator after the run
    assert runs[0][0] == runs[1][0]
    assert runs[1][1] == 0
    assert states[0] == states[1]


def compare_state(dev, o, g):
    for key in VEC_KEYS:
        assert np.array_equal(dev[key], o[key]), (g, key)
    for key in SCA_KEYS + ("Current Burn In", "Database Entries"):
        a, b = dev[key][0], o[key][0]
        assert a == b or (np.isnan(a) and np.isnan(b)), (g, key, a, b)


@pytest.mark.parametrize("N,P,mcl,burn,pergen", [(4, 256, 1, 2, ()), (3, 500, 3, 0, ()), (5, 300, 4, 1, (3, 0, 2)),
                                                 (32, 1024, 2, 1, ())])
def test_tmcmc_chain_steps_match_oracle(N, P, mcl, burn, pergen):
    """Max Chain Length > 1 / Burn In / Per Generation Burn In: several steps
    per chain in the Sequential conduit's chain-major RNG order, leader
    splitting, database and counters — bit-exact against the oracle."""
    dev, o, ndist = seeded_pair(N, P, True, seed=99, max_chain_length=mcl, burn_in=burn, per_generation_burn_in=pergen)
    split = False
    for g in range(1, 30):
        dev.generation(g)
        o.generation(g)
        dev.synchronize()
        compare_state(dev, o, g)
        split |= o["Chain Count"][0] < P
        if o["Previous Annealing Exponent"][0] >= 1.0:
            break
    if mcl > 1:
        assert split
    for which in range(3 + ndist):
        assert dev.get_rng(which).hex().upper() == o.rng(which).to_hex(), which


def test_tmcmc_host_evaluated_rounds_match_oracle():
    """The host-callback protocol (evaluate_prior -> pending -> candidates ->
    set_evaluations -> advance, repeated while chains are pending) with the
    likelihood formed in Python, against the oracle's builtin run."""
    N, P = 3, 400
    dev, o, ndist = seeded_pair(N, P, True, seed=5, max_chain_length=3, burn_in=2)
    for g in range(1, 12):
        lens, cc = dev["Chain Lengths"], int(dev["Chain Count"][0])
        dev.prepare(g)
        rounds = 0
        while True:
            dev.evaluate_prior()
            pend = dev.pending()
            X = dev.candidates()
            lp = dev["Chain Candidates LogPriors"]
            ll = np.full(P, -np.inf)
            for i in np.nonzero(pend)[0]:
                if np.isinf(lp[i]) and lp[i] < 0:
                    continue
                ss = 0.0
                for x in X[i]:
                    ss += x * x
                ll[i] = -0.5 * ss
            dev.set_evaluations(lp, ll)
            rounds += 1
            if dev.advance(g) == 0:
                break
        dev.process(g)
        dev.synchronize()
        o.generation(g)
        compare_state(dev, o, g)
        assert rounds == (1 if g == 1 else int(np.max(lens[:cc])) + 2)
        if o["Previous Annealing Exponent"][0] >= 1.0:
            break
