"""GPU tests of the korali API (korali/ -> korali_amd/engine, C++ over the
C-ABI): the reference's own statistical scripts, re-run through `import
korali`, and parity of the engine's result files with the reference's
committed ones (tests/python/plot/cmaes, same configuration and seed).
"""
import json
import math
import os

import numpy as np
import pytest

from golden_util import cmaes_variables, load_cmaes

pytestmark = pytest.mark.gpu

CM = load_cmaes()


def by_gen(g):
    for x in CM:
        if x["Current Generation"] == g:
            return x
    raise KeyError(g)


# tests/statistical/optimizers/correctness/model: minimum -0.5 area
def evalmodel(s):
    x = s["Parameters"][0]
    r = x * x + math.sin(x)
    s["F(x)"] = -r


# examples/optimization/stochastic/_model/model.py negative_sphere (F part)
def negative_sphere(p):
    x = p["Parameters"]
    res = 0.
    for i in range(len(x)):
        res += x[i]**2
    p["F(x)"] = -0.5 * res


def lgaussian_custom(s):  # tests/statistical/samplers/mean/model/model.py
    x0 = s["Parameters"][0]
    r = -0.5 * ((x0 + 2.0)**2 / (9.0)) - 0.5 * math.log(2 * math.pi * 9)
    s["logLikelihood"] = r


def cmaes_1d(**solver):
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Function"] = evalmodel
    e["Variables"][0]["Name"] = "X"
    e["Variables"][0]["Lower Bound"] = -10.0
    e["Variables"][0]["Upper Bound"] = +10.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 8
    e["Solver"]["Termination Criteria"]["Max Generations"] = 100
    for k, v in solver.items():
        e["Solver"][k.replace("_", " ")] = v
    e["Console Output"]["Verbosity"] = "Silent"
    e["File Output"]["Enabled"] = False
    e["Random Seed"] = 1337
    return e


@pytest.mark.parametrize("cfg,tol", [({}, 1e-4), ({"Diagonal Covariance": True}, 1e-4), ({"Mu Type": "Linear"}, 1e-4),
                                     ({"Mu Type": "Logarithmic"}, 1e-4),
                                     ({"Mu Type": "Proportional", "Population Size": 64}, 1e-3),
                                     ({"Mu Type": "Equal", "Population Size": 64}, 1e-3)])
def test_statistical_cmaes_correctness(cfg, tol):
    """tests/statistical/optimizers/correctness/run-cmaes.py: checkMin(e, 0.23246, tol)."""
    import korali
    e = cmaes_1d()
    for k, v in cfg.items():
        e["Solver"][k] = v
    korali.Engine().run(e)
    assert np.isclose(0.23246, e["Solver"]["Best Ever Value"], atol=tol)
    assert e["Results"]["Best Sample"]["F(x)"] == e["Solver"]["Best Ever Value"]


def test_unsupported_features_fail_loudly():
    import korali
    e = cmaes_1d()
    e["Problem"]["Constraints"] = [lambda s: None]  # a constraint that sets no F(x)
    with pytest.raises(korali.KoraliError, match="did not assign 'F\\(x\\)'"):
        korali.Engine().run(e)
    e = cmaes_1d()
    e["Problem"]["Constraints"] = [lambda s: s.__setitem__("F(x)", 1.0)]
    e["Solver"]["Mirrored Sampling"] = True
    with pytest.raises(korali.KoraliError, match="Mirrored Sampling not applicable"):
        korali.Engine().run(e)
    e = cmaes_1d()
    e["Variables"][0]["Granularity"] = -0.5
    with pytest.raises(korali.KoraliError, match="Negative granularity"):
        korali.Engine().run(e)


@pytest.mark.parametrize("mirrored", [False, True])
def test_statistical_cmaes_discrete(mirrored, tmp_path):
    """tests/statistical/optimizers/correctness/run-cmaes.py, corner case
    'Discrete with Mirrored Sampling' (Granularity 0.0001, Population Size
    64, 10 generations): checkMin(e, 0.23246, 1e-3); and the discrete state in
    the result files."""
    import json
    import korali
    e = cmaes_1d(**{"Population Size": 64, "Mirrored Sampling": mirrored})
    e["Variables"][0]["Initial Value"] = 1.0
    e["Variables"][0]["Granularity"] = 0.0001
    e["Solver"]["Termination Criteria"]["Max Generations"] = 10
    e["File Output"]["Enabled"] = True
    e["File Output"]["Path"] = str(tmp_path)
    korali.Engine().run(e)
    assert np.isclose(0.23246, e["Solver"]["Best Ever Value"], atol=1e-3)
    x = e["Solver"]["Best Ever Variables"][0]
    assert x == round(x / 0.0001) * 0.0001
    st = json.load(open(tmp_path / "latest"))["Solver"]
    assert st["Has Discrete Variables"] is True or st["Has Discrete Variables"] == 1
    for k in ("Masking Matrix", "Masking Matrix Sigma", "Number Of Discrete Mutations", "Number Masking Matrix Entries",
              "Chi Square Number Discrete Mutations", "Discrete Mutations"):
        assert k in st, k


def test_statistical_tmcmc_gaussian():
    """tests/statistical/samplers/mean/run-tmcmc-gaussian.py."""
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    e["Problem"]["Likelihood Model"] = lgaussian_custom
    e["Solver"]["Type"] = "Sampler/TMCMC"
    e["Solver"]["Population Size"] = 5000
    e["Distributions"][0]["Name"] = "Uniform 0"
    e["Distributions"][0]["Type"] = "Univariate/Uniform"
    e["Distributions"][0]["Minimum"] = -15.0
    e["Distributions"][0]["Maximum"] = +15.0
    e["Variables"][0]["Name"] = "a"
    e["Variables"][0]["Prior Distribution"] = "Uniform 0"
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    e["Random Seed"] = 1337
    korali.Engine().run(e)
    samples = np.reshape(e["Solver"]["Sample Database"], (-1, 1))
    assert np.isclose(-2.0, samples.mean(), atol=0.05)
    assert np.isclose(3.0, samples.std(), atol=0.05)
    assert e["Solver"]["Annealing Exponent"] == 1.0
    # TMCMC::finalize (TMCMC.cpp.base:791-795)
    assert np.array_equal(np.reshape(e["Results"]["Sample Database"], (-1, 1)), samples)


def fixture_experiment(path, max_gen=100):
    """The configuration behind tests/python/plot/cmaes (gen00000000.json)."""
    import korali
    v = cmaes_variables(by_gen(0))
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Function"] = negative_sphere
    for i in range(10):
        e["Variables"][i]["Name"] = "X" + str(i)
        e["Variables"][i]["Lower Bound"] = v["Lower Bound"][i]
        e["Variables"][i]["Upper Bound"] = v["Upper Bound"][i]
        e["Variables"][i]["Initial Standard Deviation"] = v["Initial Standard Deviation"][i]
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 32
    e["Solver"]["Termination Criteria"]["Max Generations"] = max_gen
    e["Solver"]["Termination Criteria"]["Min Value Difference Threshold"] = 1e-32
    e["Solver"]["Termination Criteria"]["Max Infeasible Resamplings"] = 10000
    e["Random Seed"] = 790510
    e["Console Output"]["Verbosity"] = "Silent"
    e["File Output"]["Path"] = str(path)
    return e


def read_gen(path, g):
    with open(os.path.join(path, "gen%08d.json" % g)) as f:
        return json.load(f)


def test_engine_reproduces_reference_result_files(tmp_path):
    """Same experiment as the reference's committed CMA-ES result files:
    every committed generation's population, sorting index, mean,
    covariance, sigma and generator states are reproduced bit for bit."""
    import korali
    out = tmp_path / "res"
    e = fixture_experiment(out)
    korali.Engine().run(e)
    assert e["Current Generation"] == 100
    marks = korali._generation_completion_times(e)  # (bench.py's C4 engine timing)
    assert len(marks) == 101 and all(b >= a for a, b in zip(marks, marks[1:]))
    # the timing marks stay out of the saved experiment (the reference's
    # setConfiguration rejects unknown keys, experiment.cpp:416)
    assert "Generation Completion Times" not in read_gen(out, 100).get("Internal", {})
    for ref in CM:
        g = ref["Current Generation"]
        if g == 0:
            continue
        mine = read_gen(out, g)["Solver"]
        s = ref["Solver"]
        assert np.array_equal(np.array(mine["Sample Population"]), np.array(s["Sample Population"])), g
        assert mine["Sorting Index"] == s["Sorting Index"], g
        for k in ("Current Mean", "Covariance Matrix", "Evolution Path", "Conjugate Evolution Path"):
            assert np.array_equal(np.array(mine[k]), np.array(s[k])), (g, k)
        assert mine["Sigma"] == s["Sigma"], g
        assert mine["Best Ever Value"] == s["Best Ever Value"], g
        if "Normal Generator" in s:
            assert mine["Normal Generator"]["Range"] == s["Normal Generator"]["Range"], g
    final = read_gen(out, 100)
    assert final["Is Finished"] is True
    assert os.path.exists(os.path.join(out, "latest"))


def test_engine_resume_from_result_file_is_bit_exact(tmp_path):
    """Experiment.loadState + Preserve Random Number Generator States: a run
    resumed from generation 50's file ends exactly like the straight run."""
    import korali
    a = tmp_path / "a"
    e = fixture_experiment(a)
    korali.Engine().run(e)
    r = korali.Experiment()
    assert r.loadState(str(a / "gen00000050.json"))
    r["Preserve Random Number Generator States"] = True
    r["Problem"]["Objective Function"] = negative_sphere
    r["File Output"]["Path"] = str(tmp_path / "b")
    korali.Engine().run(r)
    sa, sb = read_gen(a, 100)["Solver"], read_gen(tmp_path / "b", 100)["Solver"]
    for k in ("Sample Population", "Current Mean", "Covariance Matrix", "Sigma", "Best Ever Value"):
        assert sa[k] == sb[k], k
    assert sa["Normal Generator"]["Range"] == sb["Normal Generator"]["Range"]


def test_objective_kernel_equals_callback():
    """The device-batched objective (extension key) gives the same run as
    the host callback of the same function."""
    import korali
    runs = []
    for kernel in (False, True):
        e = korali.Experiment()
        e["Problem"]["Type"] = "Optimization"
        if kernel:
            e["Problem"]["Objective Kernel"] = "Negative Sphere"
        else:
            e["Problem"]["Objective Function"] = negative_sphere
        for i in range(6):
            e["Variables"][i]["Name"] = "X" + str(i)
            e["Variables"][i]["Initial Value"] = 1.0
            e["Variables"][i]["Initial Standard Deviation"] = 0.5
        e["Solver"]["Type"] = "Optimizer/CMAES"
        e["Solver"]["Population Size"] = 24
        e["Solver"]["Termination Criteria"]["Max Generations"] = 40
        e["Random Seed"] = 4242
        e["Console Output"]["Verbosity"] = "Silent"
        e["File Output"]["Enabled"] = False
        korali.Engine().run(e)
        runs.append((e["Solver"]["Best Ever Value"], e["Solver"]["Covariance Matrix"], e["Solver"]["Sigma"]))
    assert runs[0] == runs[1]


def test_tmcmc_normal_prior_through_the_api():
    """A Univariate/Normal prior through korali.Engine (Bayesian/Custom with
    a host likelihood): N(0.5, 2^2) prior x exp(-x^2/2) likelihood is the
    N(0.1, 0.8) posterior; LogEvidence is its closed form
    log N(0; 0.5, 1 + 4) + 0.5 log(2 pi) within the sampler's noise."""
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    e["Problem"]["Likelihood Model"] = lambda s: s.__setitem__("logLikelihood", -0.5 * s["Parameters"][0] ** 2)
    e["Distributions"][0]["Name"] = "N"
    e["Distributions"][0]["Type"] = "Univariate/Normal"
    e["Distributions"][0]["Mean"] = 0.5
    e["Distributions"][0]["Standard Deviation"] = 2.0
    e["Variables"][0]["Name"] = "x"
    e["Variables"][0]["Prior Distribution"] = "N"
    e["Solver"]["Type"] = "Sampler/TMCMC"
    e["Solver"]["Population Size"] = 5000
    e["Random Seed"] = 99
    e["Console Output"]["Verbosity"] = "Silent"
    e["File Output"]["Enabled"] = False
    korali.Engine().run(e)
    x = np.asarray(e["Solver"]["Sample Database"], dtype=float)
    assert abs(x.mean() - 0.1) < 0.05 and abs(x.var() - 0.8) < 0.08, (x.mean(), x.var())
    logz = -0.5 * np.log(2 * np.pi * 5.0) - 0.5 * 0.25 / 5.0 + 0.5 * np.log(2 * np.pi)
    assert abs(e["Solver"]["LogEvidence"] - logz) < 0.05, (e["Solver"]["LogEvidence"], logz)


def test_tmcmc_likelihood_kernel_equals_callback():
    import korali

    def lg(s):
        ss = 0.0
        for x in s["Parameters"]:
            ss += x**2
        s["logLikelihood"] = -0.5 * ss

    runs = []
    for kernel in (False, True):
        e = korali.Experiment()
        e["Problem"]["Type"] = "Bayesian/Custom"
        if kernel:
            e["Problem"]["Likelihood Kernel"] = "Gaussian"
        else:
            e["Problem"]["Likelihood Model"] = lg
        e["Distributions"][0]["Name"] = "Uniform 0"
        e["Distributions"][0]["Type"] = "Univariate/Uniform"
        e["Distributions"][0]["Minimum"] = -5.0
        e["Distributions"][0]["Maximum"] = 5.0
        for i in range(4):
            e["Variables"][i]["Name"] = "X" + str(i)
            e["Variables"][i]["Prior Distribution"] = "Uniform 0"
        e["Solver"]["Type"] = "Sampler/TMCMC"
        e["Solver"]["Population Size"] = 1000
        e["Random Seed"] = 7
        e["Console Output"]["Verbosity"] = "Silent"
        e["File Output"]["Enabled"] = False
        korali.Engine().run(e)
        runs.append((e["Solver"]["LogEvidence"], e["Solver"]["Covariance Matrix"], e["Solver"]["Sample Database"]))
    assert runs[0] == runs[1]


def tmcmc_1d(model, **solver):
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Custom"
    if model is None:
        e["Problem"]["Likelihood Kernel"] = "Gaussian"
    else:
        e["Problem"]["Likelihood Model"] = model
    e["Distributions"][0]["Name"] = "Uniform 0"
    e["Distributions"][0]["Type"] = "Univariate/Uniform"
    e["Distributions"][0]["Minimum"] = -20.0
    e["Distributions"][0]["Maximum"] = +20.0
    e["Variables"][0]["Name"] = "X"
    e["Variables"][0]["Prior Distribution"] = "Uniform 0"
    e["Solver"]["Type"] = "Sampler/TMCMC"
    for k, v in solver.items():
        e["Solver"][k] = v
    e["Console Output"]["Verbosity"] = "Silent"
    e["File Output"]["Enabled"] = False
    e["Random Seed"] = 0xC0FFEE
    return e


def test_statistical_run_tmcmc_2_burn_in():
    """tests/statistical/samplers/correctness/run-tmcmc-2.py (Burn In 3):
    checkMean(e, 0.0, 0.05), checkStd(e, 1.0, 0.05)."""
    import korali

    def model(s):  # correctness/model/model.py
        v = s["Parameters"][0]
        s["logLikelihood"] = -0.5 * v * v

    e = tmcmc_1d(model, **{"Population Size": 5000, "Covariance Scaling": 0.01, "Burn In": 3,
                           "Target Coefficient Of Variation": 0.4})
    korali.Engine().run(e)
    samples = np.array(e["Solver"]["Sample Database"])
    assert np.isclose(0.0, samples.mean(), atol=0.05)
    assert np.isclose(1.0, samples.std(), atol=0.05)


def test_tmcmc_specifics_burn_in_and_rho_updates(tmp_path):
    """tests/statistical/samplers/detailed/tmcmc/tmcmc-specifics.py: Burn In 5,
    Per Generation Burn In [10, 7], rho updates within [1e-3, 0.2]; the
    result files carry Burn In and Current Burn In per generation."""
    import korali

    def model(s):  # detailed/tmcmc/helpers: loglik -v^2
        v = s["Parameters"][0]
        s["logLikelihood"] = -v * v

    e = tmcmc_1d(model, **{"Population Size": 5000, "Covariance Scaling": 0.001, "Burn In": 5,
                           "Per Generation Burn In": [10, 7], "Max Chain Length": 1,
                           "Target Coefficient Of Variation": 0.5, "Min Annealing Exponent Update": 1e-3,
                           "Max Annealing Exponent Update": 0.2})
    e["Distributions"][0]["Minimum"] = -10.0
    e["Distributions"][0]["Maximum"] = +10.0
    e["Random Seed"] = 314
    e["File Output"]["Enabled"] = True
    e["File Output"]["Path"] = str(tmp_path)
    korali.Engine().run(e)
    files = sorted(f for f in os.listdir(tmp_path) if f.startswith("gen"))
    assert len(files) > 5
    burn = [0, 0, 10, 7] + [5] * 100
    prev = 0.0
    for f in files:
        with open(os.path.join(tmp_path, f)) as fh:
            d = json.load(fh)
        g = d["Current Generation"]
        if g == 0:
            continue
        assert d["Solver"]["Burn In"] == 5
        assert d["Solver"]["Current Burn In"] == burn[g]
        rho = d["Solver"]["Annealing Exponent"]
        assert rho - prev <= 0.2 + 1e-12
        assert rho >= prev + 1e-3 - 1e-12 or rho == 1.0
        prev = rho


@pytest.mark.parametrize("solver", [{"Burn In": 2, "Max Chain Length": 3}, {"Max Chain Length": 4},
                                    {"Burn In": 1, "Per Generation Burn In": [3, 0]}])
def test_tmcmc_chain_steps_kernel_equals_callback(solver):
    """Multi-step chains through the engine: the host-callback rounds
    (WAITANY loop) and the device likelihood kernel give identical runs."""
    import korali

    def model(s):
        v = s["Parameters"][0]
        s["logLikelihood"] = -0.5 * v * v

    runs = []
    for m in (model, None):
        e = tmcmc_1d(m, **{"Population Size": 700, **solver})
        korali.Engine().run(e)
        runs.append((e["Solver"]["LogEvidence"], e["Solver"]["Covariance Matrix"], e["Solver"]["Sample Database"],
                     e["Solver"]["Model Evaluation Count"], e["Solver"]["Chain Lengths"]))
    assert runs[0] == runs[1]


def run_with_conduit(e, conduit):
    import korali
    k = korali.Engine()
    for key, v in conduit.items():
        k["Conduit"][key] = v
    k.run(e)
    return e


@pytest.mark.parametrize("jobs", [2, 8])
def test_concurrent_conduit_equals_sequential_cmaes(jobs):
    """f3: host-callback objectives through the Concurrent conduit (a thread
    pool sharing each generation's batch) give the Sequential run bit for bit."""
    import korali

    def model(s):
        x = np.asarray(s["Parameters"])
        s["F(x)"] = -float(np.sum(100.0 * (x[1:] - x[:-1] ** 2) ** 2 + (1.0 - x[:-1]) ** 2))

    runs = []
    for conduit in ({"Type": "Sequential"}, {"Type": "Concurrent", "Concurrent Jobs": jobs}):
        e = korali.Experiment()
        e["Problem"]["Type"] = "Optimization"
        e["Problem"]["Objective Function"] = model
        for i in range(8):
            e["Variables"][i]["Name"] = "X" + str(i)
            e["Variables"][i]["Initial Value"] = 0.0
            e["Variables"][i]["Initial Standard Deviation"] = 1.0
        e["Solver"]["Type"] = "Optimizer/CMAES"
        e["Solver"]["Population Size"] = 64
        e["Solver"]["Termination Criteria"]["Max Generations"] = 30
        e["Random Seed"] = 1337
        e["Console Output"]["Verbosity"] = "Silent"
        e["File Output"]["Enabled"] = False
        run_with_conduit(e, conduit)
        runs.append((e["Solver"]["Best Ever Value"], e["Solver"]["Covariance Matrix"], e["Solver"]["Sigma"],
                     e["Solver"]["Current Mean"]))
    assert runs[0] == runs[1]


def test_concurrent_conduit_equals_sequential_tmcmc_chain_rounds():
    """TMCMC chain rounds (Burn In, Max Chain Length) through the Concurrent
    conduit: the Sequential conduit's chain-major result, bit for bit (the
    reference's Concurrent run is completion-order dependent here)."""

    def model(s):
        v = s["Parameters"][0]
        s["logLikelihood"] = -0.5 * v * v

    runs = []
    for conduit in ({"Type": "Sequential"}, {"Type": "Concurrent", "Concurrent Jobs": 6}):
        e = tmcmc_1d(model, **{"Population Size": 600, "Burn In": 2, "Max Chain Length": 3})
        run_with_conduit(e, conduit)
        runs.append((e["Solver"]["LogEvidence"], e["Solver"]["Sample Database"], e["Solver"]["Chain Lengths"],
                     e["Solver"]["Model Evaluation Count"]))
    assert runs[0] == runs[1]


def test_concurrent_conduit_raises_the_callback_error():
    import korali

    def model(s):
        if s["Sample Id"] == 17:
            raise ValueError("model failed on sample 17")
        s["F(x)"] = -float(np.sum(np.asarray(s["Parameters"]) ** 2))

    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Function"] = model
    e["Variables"][0]["Name"] = "X"
    e["Variables"][0]["Initial Value"] = 0.0
    e["Variables"][0]["Initial Standard Deviation"] = 1.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 32
    e["Solver"]["Termination Criteria"]["Max Generations"] = 3
    e["Console Output"]["Verbosity"] = "Silent"
    e["File Output"]["Enabled"] = False
    with pytest.raises(ValueError, match="sample 17"):
        run_with_conduit(e, {"Type": "Concurrent", "Concurrent Jobs": 4})


# tests/statistical/bayesian/_model/model.py: linear model a*x + b with noise sigma
REF_X = [1.0, 2.0, 3.0, 4.0, 5.0]
REF_Y = [3.21, 4.14, 4.94, 6.06, 6.84]


def linear_reference_model(s):  # model.py:8-21, the reference's own list-append idiom
    a = s["Parameters"][0]
    b = s["Parameters"][1]
    sig = s["Parameters"][2]
    s["Reference Evaluations"] = []
    s["Standard Deviation"] = []
    for x in REF_X:
        s["Reference Evaluations"] += [a * x + b]
        s["Standard Deviation"] += [sig]


def test_bayesian_reference_reproduces_reference_tmcmc_result_files(tmp_path):
    """The experiment behind tests/python/plot/tmcmc (Bayesian/Reference,
    Normal likelihood, 3 Uniform(0,5) priors, P=50, Target CoV 0.8, seed of
    gen00000000.json) run through korali.Engine: every committed generation's
    candidates, likelihoods, accept counts, annealing exponent, evidence,
    chain leaders, mean, covariance and generator states, bit for bit."""
    import korali
    from golden_util import load_tmcmc
    TM = load_tmcmc()
    g0 = TM[0]
    e = korali.Experiment()
    e["Problem"]["Type"] = "Bayesian/Reference"
    e["Problem"]["Likelihood Model"] = "Normal"
    e["Problem"]["Reference Data"] = REF_Y
    e["Problem"]["Computational Model"] = linear_reference_model
    for i, d in enumerate(g0["Distributions"]):
        e["Distributions"][i]["Name"] = d["Name"]
        e["Distributions"][i]["Type"] = "Univariate/Uniform"
        e["Distributions"][i]["Minimum"] = d["Minimum"]
        e["Distributions"][i]["Maximum"] = d["Maximum"]
    for i, v in enumerate(g0["Variables"]):
        e["Variables"][i]["Name"] = v["Name"]
        e["Variables"][i]["Prior Distribution"] = v["Prior Distribution"]
    e["Solver"]["Type"] = "Sampler/TMCMC"
    e["Solver"]["Population Size"] = 50
    e["Solver"]["Target Coefficient Of Variation"] = 0.8
    e["Random Seed"] = g0["Distributions"][0]["Random Seed"]
    e["Store Sample Information"] = True
    e["Console Output"]["Verbosity"] = "Silent"
    out = tmp_path / "tm"
    e["File Output"]["Path"] = str(out)
    korali.Engine().run(e)
    assert e["Current Generation"] == TM[-1]["Current Generation"]
    for ref in TM[1:]:
        g = ref["Current Generation"]
        mine, s = read_gen(out, g)["Solver"], ref["Solver"]
        # log-priors are not compared: the committed files were written by a
        # reference version whose Uniform log-density was 0 inside the support
        # (every LogPriors entry is 0.0); the current uniform.cpp.base gives
        # -log(max - min).  A constant prior cancels in every acceptance ratio
        # (TMCMC.cpp.base:632), so nothing else depends on it.
        for k in ("Chain Candidates", "Chain Candidates LogLikelihoods", "Chain Leaders",
                  "Chain Leaders LogLikelihoods", "Chain Lengths", "Mean Theta", "Covariance Matrix",
                  "Sample Database", "Sample LogLikelihood Database"):
            assert np.array_equal(np.array(mine[k], dtype=float), np.array(s[k], dtype=float)), (g, k)
        for k in ("Annealing Exponent", "LogEvidence", "Coefficient Of Variation", "Max Loglikelihood",
                  "Accepted Samples Count", "Chain Count", "Proposals Acceptance Rate", "Selection Acceptance Rate"):
            assert mine[k] == s[k], (g, k)
        for k in ("Multinomial Generator", "Multivariate Generator", "Uniform Generator"):
            assert mine[k]["Range"] == s[k]["Range"], (g, k)


def ref_linear_experiment(problem_type):
    """examples/bayesian.inference/reference/run-cmaes.py (MAP estimate)."""
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = problem_type
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 24
    e["Solver"]["Termination Criteria"]["Max Generations"] = 100
    e["Distributions"][0]["Name"] = "Uniform 0"
    e["Distributions"][0]["Type"] = "Univariate/Uniform"
    e["Distributions"][0]["Minimum"] = 0.0
    e["Distributions"][0]["Maximum"] = +5.0
    for i, n in enumerate(("a", "b", "[Sigma]")):
        e["Variables"][i]["Name"] = n
        e["Variables"][i]["Prior Distribution"] = "Uniform 0"
        e["Variables"][i]["Initial Value"] = +2.5
        e["Variables"][i]["Initial Standard Deviation"] = +0.5
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    e["Random Seed"] = 1337
    return e


def test_cmaes_bayesian_reference_finds_the_analytic_map():
    """Uniform priors: the MAP is the least-squares line with sigma^2 = RSS/n;
    candidates outside the priors' support (sigma < 0 near the optimum) get
    F(x) = -inf, as Bayesian::evaluate gives them."""
    import korali
    e = ref_linear_experiment("Bayesian/Reference")
    e["Problem"]["Likelihood Model"] = "Normal"
    e["Problem"]["Reference Data"] = REF_Y
    e["Problem"]["Computational Model"] = linear_reference_model
    korali.Engine().run(e)
    A = np.stack([REF_X, np.ones(5)], 1)
    (a, b), rss = np.linalg.lstsq(A, np.array(REF_Y), rcond=None)[:2]
    sig = math.sqrt(rss[0] / 5)
    best = -3 * math.log(5.0) - 5 * math.log(sig) - 0.5 * (5 * math.log(2 * math.pi) + 5)
    p = e["Results"]["Best Sample"]["Parameters"]
    assert np.allclose(p, [a, b, sig], rtol=1e-3, atol=1e-3), (p, a, b, sig)
    assert e["Solver"]["Best Ever Value"] == pytest.approx(best, rel=1e-8)


def test_cmaes_bayesian_custom_equals_optimization_objective():
    """Bayesian/Custom through CMA-ES is the Optimization run of
    F = logPrior + logLikelihood (same seed, candidates inside the support):
    identical generations, bit for bit."""
    import korali

    def loglik(s):
        a, b, sig = s["Parameters"][0], s["Parameters"][1], s["Parameters"][2]
        s["logLikelihood"] = -sum((y - (a * x + b))**2 for x, y in zip(REF_X, REF_Y)) - 0.1 * sig * sig

    def objective(s):
        lp = 0.0
        for _ in range(3):
            lp += -math.log(5.0)
        loglik(s)
        s["F(x)"] = lp + s["logLikelihood"]

    eb = ref_linear_experiment("Bayesian/Custom")
    eb["Problem"]["Likelihood Model"] = loglik
    eb["Solver"]["Termination Criteria"]["Max Generations"] = 8
    eo = ref_linear_experiment("Optimization")
    eo["Problem"]["Objective Function"] = objective
    eo["Solver"]["Termination Criteria"]["Max Generations"] = 8
    for i in range(3):
        eo["Variables"][i]["Lower Bound"] = 0.0
        eo["Variables"][i]["Upper Bound"] = 5.0
        eb["Variables"][i]["Lower Bound"] = 0.0
        eb["Variables"][i]["Upper Bound"] = 5.0
    korali.Engine().run(eb)
    korali.Engine().run(eo)
    for k in ("Current Mean", "Covariance Matrix", "Sigma", "Best Ever Value", "Sample Population"):
        assert eb["Solver"][k] == eo["Solver"][k], k


def test_cmaes_gradient_information_through_the_api():
    """'Use Gradient Information' (CMAES.cpp.base:82-87, :199, :226,
    :611-621; Optimization::evaluateWithGradients): the objective receives
    Operation 'Evaluate With Gradients' and sets 'Gradient'; the run
    optimises a 6-dim negative sphere; a wrong gradient size and a
    non-positive step size fail with the reference's messages."""
    import korali
    ops = set()

    def sphere(s):
        ops.add(s["Operation"])
        x = np.array(s["Parameters"])
        s["F(x)"] = float(-0.5 * np.sum(x * x))
        s["Gradient"] = list(-x)

    def experiment(fn, step=0.1):
        e = korali.Experiment()
        e["Problem"]["Type"] = "Optimization"
        e["Problem"]["Objective Function"] = fn
        for i in range(6):
            e["Variables"][i]["Name"] = f"x{i}"
            e["Variables"][i]["Initial Value"] = 2.0
            e["Variables"][i]["Initial Standard Deviation"] = 0.5
        e["Solver"]["Type"] = "Optimizer/CMAES"
        e["Solver"]["Population Size"] = 16
        e["Solver"]["Use Gradient Information"] = True
        e["Solver"]["Gradient Step Size"] = step
        e["Solver"]["Termination Criteria"]["Max Generations"] = 60
        e["File Output"]["Enabled"] = False
        e["Console Output"]["Verbosity"] = "Silent"
        e["Random Seed"] = 5
        return e

    e = experiment(sphere)
    korali.Engine().run(e)
    assert ops == {"Evaluate With Gradients"}
    assert e["Results"]["Best Sample"]["F(x)"] > -1e-3

    def short_gradient(s):
        s["F(x)"] = 0.0
        s["Gradient"] = [0.0]

    with pytest.raises(Exception, match="Size of sample's gradient evaluations vector"):
        korali.Engine().run(experiment(short_gradient))
    with pytest.raises(Exception, match="Gradient Step Size must be larger than 0.0"):
        korali.Engine().run(experiment(sphere, step=0.0))


def test_run_vracer_example_configuration_unchanged():
    """examples/learning/reinforcement/cartpole/run-vracer.py exactly as its
    defaults run it (50 generations of 10 episodes, 1 concurrent environment,
    3 environment variants, two 32-wide tanh layers, Clipped Normal policy,
    learning rate 1e-4, mini-batch 32, replay 1000 / 10000, one update per
    experience), the host `env` replaced by the device CartPole kernel."""
    import korali
    from vracer_cases import cartpole_vracer
    e = cartpole_vracer()
    assert e["Solver"]["Neural Network"]["Hidden Layers"][0]["Output Channels"] == 32
    korali.Engine().run(e)
    sv = e["Solver"]
    assert e["Current Generation"] == 50 and sv["Current Episode"] == 500
    assert sv["Experience Count"] > 1000 and sv["Policy Update Count"] > 0
    pol = sv["Training"]["Current Policy"]["Policy"]
    assert len(pol) == (4 * 32 + 32) + (32 * 32 + 32) + (32 * 3 + 3)  # the reference's hyperparameter count
    assert np.all(np.isfinite(pol))
    hist = np.array(sv["Training"]["Reward History"])
    assert hist.size == 500 and np.all(np.isfinite(hist))


@pytest.mark.parametrize("policy", ["Normal", "Clipped Normal"])
def test_vracer_cartpole_through_korali_engine(policy):
    """examples/learning/reinforcement/cartpole/run-vracer.py's configuration
    (Normal policy, device CartPole kernel) through korali.Engine: generations
    of 10 episodes, policy updates once 1000 experiences are stored, the
    solver state written back (counters, reward history, current policy)."""
    import korali
    from vracer_cases import cartpole_vracer
    e = cartpole_vracer(max_generations=30, environments=64, hidden=64, policy=policy)
    korali.Engine().run(e)
    sv = e["Solver"]
    assert sv["Current Episode"] >= 290
    assert sv["Experience Count"] >= 1000 and sv["Policy Update Count"] > 0
    hist = np.array(sv["Training"]["Reward History"])
    assert hist.size == sv["Current Episode"] and np.all(np.isfinite(hist))
    assert len(sv["Training"]["Current Policy"]["Policy"]) == (4 * 64 + 64) + (64 * 64 + 64) + (64 * 3 + 3)
    assert np.isfinite(sv["Training"]["Average Reward"])


def test_vracer_testing_mode_after_training():
    """The reference's testing flow: train, then e["Solver"]["Mode"] =
    "Testing" with Testing / Sample Ids and run the same experiment again;
    one generation of deterministic episodes with the trained policy
    (agent.cpp.base:139-153, 267-289), rewards in Testing / Reward equal to
    the device's testing episodes run directly with that policy."""
    import korali
    from korali_amd.vracer import VracerDevice
    from vracer_cases import cartpole_vracer
    e = cartpole_vracer(max_generations=5, environments=16, hidden=32)
    korali.Engine().run(e)
    gen = e["Current Generation"]
    pol = np.array(e["Solver"]["Training"]["Current Policy"]["Policy"], np.float32)
    e["Solver"]["Mode"] = "Testing"
    e["Solver"]["Testing"]["Sample Ids"] = list(range(12))
    korali.Engine().run(e)
    assert e["Current Generation"] == gen + 1
    got = np.array(e["Solver"]["Testing"]["Reward"], np.float32)
    assert got.size == 12 and np.all(got >= 1.0)
    noise = e["Variables"][4]["Initial Exploration Noise"]
    bounds = dict(policy_distribution="Clipped Normal", action_lower_bound=e["Variables"][4]["Lower Bound"],
                  action_upper_bound=e["Variables"][4]["Upper Bound"]) \
        if e["Solver"]["Policy"]["Distribution"] == "Clipped Normal" else {}
    d = VracerDevice(hidden_size=32, hidden_layers=2, environments=16, mini_batch_size=32, replay_maximum_size=1024,
                     replay_start_size=512, initial_exploration_noise=noise, hyperparameters=pol, **bounds)
    assert np.array_equal(got, d.test_episodes(np.arange(12)))
    d.close()


def test_vracer_testing_mode_uses_the_state_rescaling_moments():
    """Testing after a State-Rescaling training run: the engine restores the
    experiment's State Rescaling Means / Sigmas into the agent before the
    testing episodes (agent.cpp.base:1266-1274, handed to every testing agent
    at :279-280); the rewards equal the device's testing episodes run
    directly with that policy and those moments."""
    import korali
    from korali_amd.vracer import VracerDevice
    from vracer_cases import cartpole_vracer
    e = cartpole_vracer(max_generations=5, environments=16, hidden=32)
    e["Solver"]["State Rescaling"]["Enabled"] = True
    korali.Engine().run(e)
    means = np.array(e["Solver"]["State Rescaling"]["Means"], np.float32)
    sigmas = np.array(e["Solver"]["State Rescaling"]["Sigmas"], np.float32)
    assert np.any(means != 0.0) and np.any(sigmas != 1.0)  # the moments were formed
    pol = np.array(e["Solver"]["Training"]["Current Policy"]["Policy"], np.float32)
    e["Solver"]["Mode"] = "Testing"
    e["Solver"]["Testing"]["Sample Ids"] = list(range(12))
    korali.Engine().run(e)
    got = np.array(e["Solver"]["Testing"]["Reward"], np.float32)
    noise = e["Variables"][4]["Initial Exploration Noise"]
    kw = dict(hidden_size=32, hidden_layers=2, environments=16, mini_batch_size=32, replay_maximum_size=1024,
              replay_start_size=512, initial_exploration_noise=noise, hyperparameters=pol,
              policy_distribution="Clipped Normal", action_lower_bound=e["Variables"][4]["Lower Bound"],
              action_upper_bound=e["Variables"][4]["Upper Bound"])
    d = VracerDevice(**kw)
    d.set("state_rescaling_means", means)
    d.set("state_rescaling_sigmas", sigmas)
    assert np.array_equal(got, d.test_episodes(np.arange(12)))
    d.close()
