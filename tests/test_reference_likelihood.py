"""Bayesian/Reference likelihood models (korali_amd/engine/likelihood.cpp,
reference.cpp.base:25-229) on the CPU.

* Normal is pinned bit-exact by the reference's own TMCMC result files
  (tests/python/plot/tmcmc: Bayesian/Reference, Likelihood Model "Normal",
  the linear model of tests/statistical/bayesian/_model/model.py with
  reference points x = 1..5): every candidate with a finite prior has its
  committed "Chain Candidates LogLikelihoods" reproduced exactly.
* The other models restate GSL's pdf/cdf algorithms; no reference fixture
  covers them (parity with GSL's special functions is unpinned), so they are
  checked against scipy.stats at 1e-12 relative.
"""
import math

import numpy as np
import pytest
import scipy.stats as st

import korali
from golden_util import load_tmcmc
from korali_amd import libkorali as L

# tests/statistical/bayesian/_model/model.py getReferenceData / getReferencePoints
Y = [3.21, 4.14, 4.94, 6.06, 6.84]
X = [1.0, 2.0, 3.0, 4.0, 5.0]


def linear_model(p):  # model.py:8-21
    a, b, sig = p
    return {"Reference Evaluations": [a * x + b for x in X], "Standard Deviation": [sig] * len(X),
            "Degrees Of Freedom": [1] * len(X), "Dispersion": [100.0] * len(X)}


def test_normal_reproduces_reference_fixture_loglikelihoods():
    n = 0
    for gen in load_tmcmc():
        s = gen["Solver"]
        if not len(s.get("Chain Candidates LogLikelihoods", [])):
            continue
        for c, ll, lp in zip(s["Chain Candidates"], s["Chain Candidates LogLikelihoods"], s["Chain Candidates LogPriors"]):
            if lp == -math.inf:
                continue
            assert L._reference_loglikelihood("Normal", Y, linear_model(c)) == ll, (gen["Current Generation"], c)
            n += 1
    assert n > 300


def test_normal_standard_deviation_clamp_applies_to_the_log_only():
    """reference.cpp.base:64-75: the SSE divides by the raw deviation, only the
    log term sees the STDEV_EPSILON clamp."""
    ll = L._reference_loglikelihood("Normal", [1.0, 2.0], {"Reference Evaluations": [1.0, 2.5],
                                                           "Standard Deviation": [1e-12, 0.5]})
    assert math.isnan(ll) is False
    assert ll == -(math.log(1e-11) + math.log(0.5)) - 0.5 * (2 * 1.83787706640934533908193770912476 + 1.0)
    assert math.isnan(L._reference_loglikelihood("Normal", [1.0], {"Reference Evaluations": [1.0],
                                                                   "Standard Deviation": [0.0]}))


rng = np.random.default_rng(7)
CASES = [(rng.uniform(0.5, 8.0, 6), rng.uniform(0.5, 8.0, 6), rng.uniform(0.3, 3.0, 6)) for _ in range(20)]


@pytest.mark.parametrize("k", range(len(CASES)))
def test_continuous_models_match_scipy(k):
    y, f, sd = CASES[k]
    y, f, sd = list(y), list(f), list(sd)
    nu = [float(v) for v in np.round(np.array(sd) * 3 + 1)]
    ref = {
        "Normal": st.norm.logpdf(y, f, sd).sum(),
        "Positive Normal": (st.norm.logpdf(y, f, sd) - np.log(st.norm.sf(0.0, f, sd))).sum(),
        "StudentT": st.t.logpdf(np.subtract(y, f), nu).sum(),
        "Positive StudentT": (st.t.logpdf(np.subtract(y, f), nu) - np.log(1.0 - st.t.cdf(-np.array(f), nu))).sum(),
    }
    ent = {"Reference Evaluations": f, "Standard Deviation": sd, "Degrees Of Freedom": nu}
    for model, want in ref.items():
        got = L._reference_loglikelihood(model, y, ent)
        assert got == pytest.approx(want, rel=1e-12, abs=1e-12), model


@pytest.mark.parametrize("k", range(10))
def test_count_models_match_scipy(k):
    r = np.random.default_rng(100 + k)
    y = [float(v) for v in r.integers(0, 30, 8)]
    f = list(r.uniform(0.5, 20.0, 8))
    disp = list(r.uniform(0.5, 50.0, 8))
    ent = {"Reference Evaluations": f, "Dispersion": disp}
    got = L._reference_loglikelihood("Poisson", y, ent)
    assert got == pytest.approx(st.poisson.logpmf(y, f).sum(), rel=1e-12)
    # gsl_ran_geometric_pdf(y + 1, 1 / (1 + f)): scipy's geom counts trials from 1
    got = L._reference_loglikelihood("Geometric", y, ent)
    assert got == pytest.approx(st.geom.logpmf(np.add(y, 1), 1.0 / (1.0 + np.array(f))).sum(), rel=1e-12)
    # p = m / (m + r): y failures before r successes with success prob 1 - p
    got = L._reference_loglikelihood("Negative Binomial", y, ent)
    p = np.array(f) / (np.array(f) + np.array(disp))
    assert got == pytest.approx(st.nbinom.logpmf(y, disp, 1.0 - p).sum(), rel=1e-11)


def test_negative_binomial_nonpositive_mean_is_minus_infinity():
    assert L._reference_loglikelihood("Negative Binomial", [1.0, 2.0], {"Reference Evaluations": [1.0, 0.0],
                                                                          "Dispersion": [1.0, 1.0]}) == -math.inf


@pytest.mark.parametrize("model,ent,msg", [
    ("Normal", {"Reference Evaluations": [1.0, 2.0]}, "requires a 'Standard Deviation'"),
    ("Normal", {"Reference Evaluations": [1.0, 2.0], "Standard Deviation": [1.0]}, "2-sized Standard Deviation"),
    ("Normal", {"Reference Evaluations": [1.0, 2.0], "Standard Deviation": [1.0, -1.0]}, "Negative"),
    ("Positive Normal", {"Reference Evaluations": [1.0, -2.0], "Standard Deviation": [1.0, 1.0]}, "Reference Evaluation"),
    ("Poisson", {"Reference Evaluations": [1.0, 0.0]}, "Negative value"),
    ("Laplace", {"Reference Evaluations": [1.0, 2.0]}, "not recognized"),
])
def test_malformed_model_output_fails_loudly(model, ent, msg):
    with pytest.raises(korali.KoraliError, match=msg):
        L._reference_loglikelihood(model, [1.0, 2.0], ent)


def reference_experiment():
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Reference"
    e["Problem"]["Likelihood Model"] = "Normal"
    e["Problem"]["Reference Data"] = Y
    e["Problem"]["Computational Model"] = lambda s: None
    for i, n in enumerate(("a", "b", "[Sigma]")):
        e["Distributions"][i]["Name"] = "Uniform %d" % i
        e["Distributions"][i]["Type"] = "Univariate/Uniform"
        e["Distributions"][i]["Minimum"] = 0.0
        e["Distributions"][i]["Maximum"] = 5.0
        e["Variables"][i]["Name"] = n
        e["Variables"][i]["Prior Distribution"] = "Uniform %d" % i
    e["Solver"]["Type"] = "Sampler/TMCMC"
    e["Solver"]["Population Size"] = 50
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    return e


@pytest.mark.parametrize("key,value,msg", [("Reference Data", [], "require defining reference data"),
                                           ("Likelihood Model", "Cauchy", "not recognized"),
                                           ("Computational Model", None, "Computational Model")])
def test_reference_problem_configuration_errors_before_device(key, value, msg):
    e = reference_experiment()
    e["Problem"][key] = value
    with pytest.raises(korali.KoraliError, match=msg):
        korali.Engine().run(e)


def test_sample_entries_extend_in_place():
    """model.py's `s[k] = []; s[k] += [v]` idiom on a korali Sample."""
    s = L.Sample()
    s["Reference Evaluations"] = []
    s["Reference Evaluations"] += [1.5]
    s["Reference Evaluations"] += [2.5]
    assert s["Reference Evaluations"] == [1.5, 2.5]


def test_cmaes_bayesian_prior_validation_before_device():
    e = reference_experiment()
    e["Solver"] = {"Type": "Optimizer/CMAES", "Population Size": 8}
    e["Distributions"][2]["Type"] = "Univariate/Beta"
    with pytest.raises(korali.KoraliError, match="Univariate/Normal"):
        korali.Engine().run(e)


def test_bayesian_evaluate_reference_and_priors():
    """Bayesian::evaluate (bayesian.cpp.base:24-84) as CMA-ES sees it: Uniform
    log-density -log(max - min), the model skipped outside the support."""
    calls = []

    def model(s):
        calls.append(1)
        a, b, sig = s["Parameters"][0], s["Parameters"][1], s["Parameters"][2]
        s["Reference Evaluations"] = [a * x + b for x in X]
        s["Standard Deviation"] = [sig] * len(X)

    e = reference_experiment()
    e["Problem"]["Computational Model"] = model
    out = L._bayesian_evaluate(e, [0.9, 2.2, 0.3])
    lp = 0.0
    for _ in range(3):
        lp += -math.log(5.0)
    ll = L._reference_loglikelihood("Normal", Y, linear_model([0.9, 2.2, 0.3]))
    assert out["logPrior"] == lp and out["logLikelihood"] == ll
    assert out["F(x)"] == out["logPosterior"] == out["logP(x)"] == lp + ll
    assert len(calls) == 1
    out = L._bayesian_evaluate(e, [0.9, 2.2, -0.1])  # sigma outside Uniform(0, 5)
    assert out["F(x)"] == -math.inf and out["logLikelihood"] == -math.inf and len(calls) == 1


def test_bayesian_evaluate_custom_with_normal_prior():
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    e["Problem"]["Likelihood Model"] = lambda s: s.__setitem__("logLikelihood", -2.0 * s["Parameters"][0] ** 2)
    e["Distributions"][0]["Name"] = "N"
    e["Distributions"][0]["Type"] = "Univariate/Normal"
    e["Distributions"][0]["Mean"] = 1.0
    e["Distributions"][0]["Standard Deviation"] = 2.0
    e["Variables"][0]["Name"] = "x"
    e["Variables"][0]["Prior Distribution"] = "N"
    out = L._bayesian_evaluate(e, [0.5])
    d = (0.5 - 1.0) / 2.0
    assert out["logPrior"] == (-0.5 * math.log(2 * math.pi) - math.log(2.0)) - 0.5 * d * d
    assert out["F(x)"] == out["logPrior"] + (-0.5)
    assert out["logPrior"] == pytest.approx(st.norm.logpdf(0.5, 1.0, 2.0), rel=1e-15)


@pytest.mark.parametrize("dist,params,x,ref", [
    ("Univariate/Exponential", {"Location": -1.0, "Mean": 2.0}, 0.5, lambda x: st.expon.logpdf(x, -1.0, 2.0)),
    ("Univariate/Laplace", {"Mean": 0.3, "Width": 1.5}, -0.4, lambda x: st.laplace.logpdf(x, 0.3, 1.5)),
    ("Univariate/Cauchy", {"Location": 0.0, "Scale": 0.5}, 0.7, lambda x: st.cauchy.logpdf(x, 0.0, 0.5)),
    ("Univariate/LogNormal", {"Mu": 0.2, "Sigma": 0.5}, 1.3, lambda x: st.lognorm.logpdf(x, 0.5, scale=math.exp(0.2)))])
def test_bayesian_evaluate_custom_with_other_priors(dist, params, x, ref):
    """The other univariate priors' getLogDensity (exponential / laplace /
    cauchy / logNormal .cpp.base) in the MAP evaluator: the reference's
    expression order exactly, and the density itself against scipy."""
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    e["Problem"]["Likelihood Model"] = lambda s: s.__setitem__("logLikelihood", 0.0)
    e["Distributions"][0]["Name"] = "P"
    e["Distributions"][0]["Type"] = dist
    for k, v in params.items():
        e["Distributions"][0][k] = v
    e["Variables"][0]["Name"] = "x"
    e["Variables"][0]["Prior Distribution"] = "P"
    lp = L._bayesian_evaluate(e, [x])["logPrior"]
    a, b = list(params.values())
    exact = {"Univariate/Exponential": lambda: -math.log(b) - (x - a) / b,
             "Univariate/Laplace": lambda: -math.log(2.0 * b) - abs(x - a) / b,
             "Univariate/Cauchy": lambda: -math.log(b * math.pi) - math.log(1.0 + (x - a) * (x - a) / (b * b)),
             "Univariate/LogNormal": lambda: (-0.5 * math.log(2 * math.pi) - math.log(b)) - math.log(x)
             - 0.5 * ((math.log(x) - a) / b) ** 2}[dist]()
    assert lp == exact
    assert lp == pytest.approx(ref(x), rel=1e-13)


@pytest.mark.parametrize("dist,drop", [("Univariate/Normal", "Standard Deviation"), ("Univariate/Normal", "Mean"),
                                       ("Univariate/Uniform", "Minimum"), ("Univariate/Uniform", "Maximum")])
def test_bayesian_prior_mandatory_settings(dist, drop):
    """A missing prior parameter fails at configuration time with the
    generated setConfiguration's message (source_builders.py:72-75)."""
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    e["Problem"]["Likelihood Model"] = lambda s: s.__setitem__("logLikelihood", 0.0)
    e["Distributions"][0]["Name"] = "P"
    e["Distributions"][0]["Type"] = dist
    params = {"Mean": 0.0, "Standard Deviation": 1.0} if "Normal" in dist else {"Minimum": 0.0, "Maximum": 1.0}
    for k, v in params.items():
        if k != drop:
            e["Distributions"][0][k] = v
    e["Variables"][0]["Name"] = "x"
    e["Variables"][0]["Prior Distribution"] = "P"
    with pytest.raises(korali.KoraliError, match="No value provided for mandatory setting: \\['%s'\\]" % drop):
        L._bayesian_evaluate(e, [0.5])


def test_reference_likelihood_rejects_scalar_where_array_expected():
    """KORALI_GET(std::vector<double>, ...) does not convert a scalar."""
    s = linear_model([0.9, 2.2, 0.3])
    s["Standard Deviation"] = 0.3
    with pytest.raises(korali.KoraliError, match="Standard Deviation"):
        L._reference_loglikelihood("Normal", Y, s)
