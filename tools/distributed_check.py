"""One rank of the korali::Engine Distributed conduit check (tests/
test_gpu_distributed.py launches it with torch.distributed.run): runs the
experiment on the Distributed conduit, then the same experiment unsharded on
the Sequential conduit, after 1 and after 6 generations, and writes the
solver states to <out>/rank<r>.json.  The test compares them (TMCMC and
CMA-ES with the exact covariance update: bit-identical; CMA-ES with MFMA:
the first generation's samples, fitness and sort bit-identical and mean /
covariance / sigma within the partial-sum tolerance) and every rank's state
against rank 0's (bit-identical).

    distributed_check.py <out dir> cmaes|tmcmc builtin|host|grad|ccmaes|mtmcmc|c4 RCCL|Host [Exact|MFMA]

model grad (CMA-ES only): the host Rosenbrock objective with its "Gradient",
Use Gradient Information on (each rank evaluates its rows' gradients, the
engine all-gathers them).

model ccmaes (CMA-ES only): run-ccmaes.py's "Mixed" CCMA-ES experiment (host
objective, 8 constraints): the device state replicated, the objective and
constraint callbacks split over the ranks and their values all-gathered.

model mtmcmc (TMCMC only): run-mtmcmc.py's mTMCMC experiment (Bayesian/
Reference, gradient / Fisher-information proposals): the device state
replicated, each round's evaluations split over the ranks.

model c4 (CMA-ES only): the C4 shape, 512-dim negative Ackley at
lambda = 65536 (BASELINE.json configs[3]), after 1 and 4 generations.
"""
import json
import math
import os
import sys

import korali

KEYS = {"cmaes": ["Current Mean", "Covariance Matrix", "Sigma", "Sorting Index", "Best Ever Value",
                  "Evolution Path", "Conjugate Evolution Path", "Value Vector", "Model Evaluation Count"],
        "tmcmc": ["Sample Database", "Sample LogLikelihood Database", "Annealing Exponent", "LogEvidence",
                  "Chain Leaders", "Covariance Matrix", "Model Evaluation Count", "Accepted Samples Count"]}


def negative_rosenbrock(s):
    x = s["Parameters"]
    s["F(x)"] = -sum(100.0 * (x[i + 1] - x[i] * x[i]) ** 2 + (1.0 - x[i]) ** 2 for i in range(len(x) - 1))


def rosenbrock_with_gradient(s):  # Optimization::evaluateWithGradients: F(x) and its "Gradient"
    negative_rosenbrock(s)
    x = s["Parameters"]
    g = [0.0] * len(x)
    for i in range(len(x) - 1):
        t = x[i + 1] - x[i] * x[i]
        g[i] += 400.0 * t * x[i] + 2.0 * (1.0 - x[i])
        g[i + 1] -= 200.0 * t
    s["Gradient"] = g


def ccmaes_model(s):  # tests/ccmaes_cases.py evaluate_model (run-ccmaes.py's helpers)
    x1, x2 = s["Parameters"]
    s["F(x)"] = -x1**2 - x2**2 - math.sin(x1)**2 - math.sin(x2)**2


def constraint(fn):
    def c(s):
        s["F(x)"] = fn(s["Parameters"])
    return c


# run-ccmaes.py's "Mixed" case: active and inactive constraints at the maxima
CCMAES_CONSTRAINTS = [lambda x: -(x[0] - 1.0), lambda x: -(x[0] - 2.0), lambda x: -(x[1] - 1.0),
                      lambda x: -(x[1] - 2.0), lambda x: -math.cos(x[0]), lambda x: -math.sin(x[0]),
                      lambda x: -math.cos(x[1]), lambda x: -math.sin(x[1])]


REF_X, REF_Y = [1.0, 2.0, 3.0, 4.0, 5.0], [3.21, 4.14, 4.94, 6.06, 6.84]


def model_with_gradients(s):  # run-mtmcmc.py's _model/model.py: y = a x + b, sd sig, with gradients
    a, b, sig = s["Parameters"]
    s["Reference Evaluations"] = [a * x + b for x in REF_X]
    s["Standard Deviation"] = [sig] * len(REF_X)
    s["Gradient Mean"] = [[x, 1.0, 0.0] for x in REF_X]
    s["Gradient Standard Deviation"] = [[0.0, 0.0, 1.0] for x in REF_X]


def gaussian(s):  # the builtin Gaussian likelihood, -0.5 * sum(x^2)
    s["logLikelihood"] = -0.5 * sum(v * v for v in s["Parameters"])


_FAIL_CALLS = [0]


def failing_constraint(s):
    """ccmaes_fail: rank 1's constraint callback raises on its 40th call
    (a replicated CCMA-ES evaluation: every rank must leave with an error,
    none may be left waiting in the bootstrap gather)"""
    _FAIL_CALLS[0] += 1
    if int(os.environ["RANK"]) == 1 and _FAIL_CALLS[0] >= 40:
        raise RuntimeError("constraint failed on purpose on rank 1")
    s["F(x)"] = CCMAES_CONSTRAINTS[0](s["Parameters"])


def experiment(solver, model, gens, cov="Exact"):
    e = korali.Experiment()
    e["Random Seed"] = 4242
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    if solver == "cmaes" and model in ("ccmaes", "ccmaes_fail"):  # run-ccmaes.py's experiment
        e["Problem"]["Type"] = "Optimization"
        e["Problem"]["Objective Function"] = ccmaes_model
        e["Problem"]["Constraints"] = [constraint(c) for c in CCMAES_CONSTRAINTS]
        if model == "ccmaes_fail":
            e["Problem"]["Constraints"] = [failing_constraint] + e["Problem"]["Constraints"][1:]
        for i, name in enumerate(("X", "Y")):
            e["Variables"][i]["Name"] = name
            e["Variables"][i]["Lower Bound"] = -10.0
            e["Variables"][i]["Upper Bound"] = +10.0
        e["Solver"]["Type"] = "Optimizer/CMAES"
        e["Solver"]["Population Size"] = 8
        e["Solver"]["Viability Population Size"] = 2
        e["Solver"]["Is Sigma Bounded"] = 1
        e["Solver"]["Termination Criteria"]["Max Generations"] = gens
    elif solver == "cmaes":
        N = 512 if model == "c4" else 16
        e["Problem"]["Type"] = "Optimization"
        if model == "c4":
            e["Problem"]["Objective Kernel"] = "Negative Ackley"
        elif model == "builtin":
            e["Problem"]["Objective Kernel"] = "Negative Rosenbrock"
        elif model == "grad":
            e["Problem"]["Objective Function"] = rosenbrock_with_gradient
            e["Solver"]["Use Gradient Information"] = True
            e["Solver"]["Gradient Step Size"] = 1e-3
        else:
            e["Problem"]["Objective Function"] = negative_rosenbrock
        for i in range(N):
            e["Variables"][i]["Name"] = f"X{i}"
            e["Variables"][i]["Initial Value"] = 2.0 if model == "c4" else 0.0
            e["Variables"][i]["Initial Standard Deviation"] = 1.0
        e["Solver"]["Type"] = "Optimizer/CMAES"
        e["Solver"]["Population Size"] = 65536 if model == "c4" else 64
        e["Solver"]["Covariance Update"] = cov
        e["Solver"]["Termination Criteria"]["Max Generations"] = gens
    elif model == "mtmcmc":  # run-mtmcmc.py's experiment (P = 500)
        e["Problem"]["Type"] = "Bayesian/Reference"
        e["Problem"]["Likelihood Model"] = "Normal"
        e["Problem"]["Reference Data"] = REF_Y
        e["Problem"]["Computational Model"] = model_with_gradients
        e["Distributions"][0]["Name"] = "Uniform 0"
        e["Distributions"][0]["Type"] = "Univariate/Uniform"
        e["Distributions"][0]["Minimum"] = 0.0
        e["Distributions"][0]["Maximum"] = 5.0
        for i, n in enumerate(("a", "b", "[Sigma]")):
            e["Variables"][i]["Name"] = n
            e["Variables"][i]["Prior Distribution"] = "Uniform 0"
        e["Solver"]["Type"] = "Sampler/TMCMC"
        e["Solver"]["Version"] = "mTMCMC"
        e["Solver"]["Population Size"] = 500
        e["Solver"]["Termination Criteria"]["Max Generations"] = gens
    else:
        e["Problem"]["Type"] = "Bayesian/Custom"
        if model == "builtin":
            e["Problem"]["Likelihood Kernel"] = "Gaussian"
        else:
            e["Problem"]["Likelihood Model"] = gaussian
        e["Distributions"][0]["Name"] = "U"
        e["Distributions"][0]["Type"] = "Univariate/Uniform"
        e["Distributions"][0]["Minimum"] = -10.0
        e["Distributions"][0]["Maximum"] = 10.0
        for i in range(4):
            e["Variables"][i]["Name"] = f"a{i}"
            e["Variables"][i]["Prior Distribution"] = "U"
        e["Solver"]["Type"] = "Sampler/TMCMC"
        e["Solver"]["Population Size"] = 600
        e["Solver"]["Max Chain Length"] = 2
        e["Solver"]["Burn In"] = 1
        e["Solver"]["Termination Criteria"]["Max Generations"] = gens
    return e


CCMAES_KEYS = ["Viability Boundaries", "Constraint Evaluation Count", "Is Viability Regime", "Constraint Evaluations",
               "Current Population Size"]


MTMCMC_KEYS = ["Chain Leaders Errors", "Chain Leaders Covariance"]


def state(e, solver, model):
    keys = KEYS[solver] + {"ccmaes": CCMAES_KEYS, "mtmcmc": MTMCMC_KEYS}.get(model, [])
    return {k: e["Solver"][k] for k in keys} | {"Current Generation": e["Current Generation"]}


GENS = {"c4": (1, 4), "mtmcmc": (1, 3)}  # (mtmcmc reaches annealing exponent 1 at generation 5)


def main():
    out, solver, model, transport = sys.argv[1:5]
    cov = sys.argv[5] if len(sys.argv) > 5 else "Exact"
    rank = int(os.environ["RANK"])
    result = {}
    if model == "ccmaes_fail":
        k = korali.Engine()
        k["Conduit"]["Type"] = "Distributed"
        k["Conduit"]["Transport"] = transport
        try:
            k.run(experiment(solver, model, 6, cov))
            result["error"] = None
        except Exception as ex:  # noqa: BLE001 -- the test reads the message
            result["error"] = str(ex)
        with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
            json.dump(result, f)
        print(f"DISTRIBUTED_CHECK rank {rank} done", flush=True)
        return
    for gens in GENS.get(model, (1, 6)):  # one generation: same samples; more: the run as a whole
        k = korali.Engine()
        k["Conduit"]["Type"] = "Distributed"
        k["Conduit"]["Transport"] = transport
        e = experiment(solver, model, gens, cov)
        k.run(e)
        u = experiment(solver, model, gens, cov)
        korali.Engine().run(u)
        result[str(gens)] = {"sharded": state(e, solver, model), "unsharded": state(u, solver, model)}
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(result, f)
    print(f"DISTRIBUTED_CHECK rank {rank} done", flush=True)


if __name__ == "__main__":
    main()
