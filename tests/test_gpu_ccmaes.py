"""GPU parity of CCMA-ES (Problem "Constraints"; CMAES.cpp.base:315-437,
:551-580, :724-731, :774-832): the device path (kg_cmaes_prepare_constrained:
host constraint callbacks, device covariance correction / eigensystem /
redraws) against the oracle's restatement, bit for bit, through whole runs
of the reference's own CCMA-ES test problems (run-ccmaes.py) and the
constraint corner cases of run-cmaes.py.  Objective and constraints are the
same Python functions on both sides."""
import numpy as np
import pytest

import refcpu as R
from ccmaes_cases import CONSTRAINTS, RUN_CCMAES, RUN_CCMAES_SETUP, evalmodel, evaluate_model
from test_oracle_ccmaes import ccmaes_oracle

pytestmark = pytest.mark.gpu


def device(N, lam, cons, viab, bound, seed, sigma_bounded=False, x0=None, max_res=float("inf")):
    from korali_amd.native import CmaesDevice
    return CmaesDevice(N, lam, lower_bound=np.full(N, -bound), upper_bound=np.full(N, bound),
                       initial_value=None if x0 is None else np.asarray(x0, dtype=float),
                       is_sigma_bounded=sigma_bounded, normal_seed=seed, uniform_seed=seed + 1,
                       max_infeasible_resamplings=max_res, constraints=[CONSTRAINTS[c] for c in cons],
                       viability_population_size=viab)


def run_pair(o, dev, gens, objective, stop=None):
    N = dev.N
    for g in range(1, gens + 1):
        o.ccmaes_generation(g, objective)
        if g == 1:
            dev.initialize()
        dev.prepare_constrained(g)
        lam = dev.lam
        assert lam == o.current_population_size(), g
        X = dev.candidates()
        assert np.array_equal(X.reshape(-1), o["Sample Population"]), g
        dev.set_fitness(np.array([objective(list(map(float, x))) for x in X]))
        dev.update(g)
        dev.synchronize()
        assert np.array_equal(dev.sorting_index(), o.sorting_index()[:lam]), g
        for key in ("Current Mean", "Covariance Matrix", "Covariance Eigenvector Matrix", "Axis Lengths"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in ("Sigma", "Best Ever Value", "Infeasible Sample Count", "Global Success Rate",
                    "Resampled Parameter Count"):
            assert dev[key][0] == o[key][0], (g, key)
        if True:  # (every case here has constraints)
            assert np.array_equal(dev["Viability Boundaries"], o["Viability Boundaries"]), g
            assert np.array_equal(dev["Best Constraint Evaluations"], o["Best Constraint Evaluations"]), g
            for key in ("Constraint Evaluation Count", "Covariance Matrix Adaptation Count"):
                assert dev[key][0] == o[key][0], (g, key)
            assert np.array_equal(dev["Normal Constraint Approximation"], o["Normal Constraint Approximation"]), g
        if stop and stop(o, g):
            break
    assert dev.get_rng(0) == o.rng(0).get_bytes()


@pytest.mark.parametrize("case", [c for c in RUN_CCMAES if c != "None"])
def test_run_ccmaes_cases_match_oracle_bit_exact(case):
    cons, lower = RUN_CCMAES[case]
    S = RUN_CCMAES_SETUP
    args = (S["N"], S["lam"], cons, S["viability_population_size"], S["bound"], S["seed"], S["sigma_bounded"])
    o, dev = ccmaes_oracle(*args), device(*args)
    run_pair(o, dev, S["generations"], evaluate_model)
    assert dev["Best Ever Value"][0] >= lower
    dev.close()


def test_unsatisfiable_constraint_corner_cases_match_oracle():
    o = ccmaes_oracle(1, 16, ["constraint1"], 2, 10.0, 1337, x0=[1.0])
    dev = device(1, 16, ["constraint1"], 2, 10.0, 1337, x0=[1.0])
    run_pair(o, dev, 10, evalmodel)
    assert dev["Infeasible Sample Count"][0] > 10
    dev.close()
    o = ccmaes_oracle(1, 16, ["constraint1"], 2, 10.0, 1337, x0=[1.0], max_res=50)
    dev = device(1, 16, ["constraint1"], 2, 10.0, 1337, x0=[1.0], max_res=50)
    run_pair(o, dev, 100, evalmodel, stop=lambda o, g: g > 1 and o["Infeasible Sample Count"][0] >= 50)
    dev.close()


def _sample_fn(f):
    def g(s):
        s["F(x)"] = f([s["Parameters"][d] for d in range(len(s["Parameters"]))])
    return g


@pytest.mark.parametrize("case,conduit", [("Active at Max 1", "Sequential"), ("Mixed", "Concurrent")])
def test_run_ccmaes_configuration_through_korali_engine(case, conduit):
    """run-ccmaes.py's experiment unchanged through korali.Engine (Python
    objective and constraint functions, Sequential or Concurrent conduit):
    the reference's bound holds and the result equals the oracle's run bit
    for bit."""
    import korali
    cons, lower = RUN_CCMAES[case]
    S = RUN_CCMAES_SETUP
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Function"] = _sample_fn(evaluate_model)
    e["Problem"]["Constraints"] = [_sample_fn(CONSTRAINTS[c]) for c in cons]
    for i, name in enumerate(("X", "Y")):
        e["Variables"][i]["Name"] = name
        e["Variables"][i]["Lower Bound"] = -10.0
        e["Variables"][i]["Upper Bound"] = +10.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 8
    e["Solver"]["Viability Population Size"] = 2
    e["Solver"]["Termination Criteria"]["Max Generations"] = 100
    e["Solver"]["Is Sigma Bounded"] = 1
    e["Console Output"]["Verbosity"] = "Silent"
    e["File Output"]["Enabled"] = False
    e["Random Seed"] = 1337
    k = korali.Engine()
    k["Conduit"]["Type"] = conduit
    if conduit == "Concurrent":
        k["Conduit"]["Concurrent Jobs"] = 4
    k.run(e)
    best = e["Solver"]["Best Ever Value"]
    assert best >= lower
    o = ccmaes_oracle(S["N"], S["lam"], cons, S["viability_population_size"], S["bound"], S["seed"], True)
    for g in range(1, S["generations"] + 1):
        o.ccmaes_generation(g, evaluate_model)
    assert best == o["Best Ever Value"][0]
    assert e["Solver"]["Constraint Evaluation Count"] == o["Constraint Evaluation Count"][0]
    assert list(e["Solver"]["Viability Boundaries"]) == list(o["Viability Boundaries"])
