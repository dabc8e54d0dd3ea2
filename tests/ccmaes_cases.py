"""CCMA-ES test problems: the reference's own statistical test
tests/statistical/optimizers/detailed/ccmaes (run-ccmaes.py + helpers) and the
constraint corner cases of tests/statistical/optimizers/correctness/
run-cmaes.py, restated as plain functions of the parameter list (the
reference's take a Sample and set "F(x)")."""
import math


def evaluate_model(x):  # ccmaes/helpers: evaluateModel
    x1, x2 = x[0], x[1]
    return -x1**2 - x2**2 - math.sin(x1)**2 - math.sin(x2)**2


def evalmodel(x):  # correctness/model: evalmodel (minimum at -0.5)
    v = x[0]
    return -(v * v + math.sin(v))


CONSTRAINTS = {
    "inactive1": lambda x: -1,
    "inactive2": lambda x: -2,
    "activeMax1": lambda x: -(x[0] - 1.0),
    "activeMax2": lambda x: -(x[0] - 2.0),
    "activeMax3": lambda x: -(x[1] - 1.0),
    "activeMax4": lambda x: -(x[1] - 2.0),
    "inactiveMax1": lambda x: -math.cos(x[0]),
    "inactiveMax2": lambda x: -math.sin(x[0]),
    "inactiveMax3": lambda x: -math.cos(x[1]),
    "inactiveMax4": lambda x: -math.sin(x[1]),
    "constraint1": lambda x: 100.0,
}

# run-ccmaes.py: case -> (constraints, the reference's assert_greatereq bound on Best Ever Value)
RUN_CCMAES = {
    "None": ([], -6 * 1e-10),
    "Inactive": (["inactive1", "inactive2"], -1.8 * 1e-10),
    "Active at Max 1": (["activeMax1", "activeMax2"], -4.826824e+00),
    "Active at Max 2": (["activeMax1", "activeMax2", "activeMax3", "activeMax4"], -9.653645e+00),
    "Inactive at Max 1": (["inactiveMax1", "inactiveMax2"], -2.19963e-10),
    "Inactive at Max 2": (["inactiveMax1", "inactiveMax2", "inactiveMax3", "inactiveMax4"], -4.626392e-10),
    "Mixed": (["activeMax1", "activeMax2", "activeMax3", "activeMax4", "inactiveMax1", "inactiveMax2",
               "inactiveMax3", "inactiveMax4"], -7.895685e+01),
}

# run-ccmaes.py's experiment: 2 variables in [-10, 10], Population Size 8,
# Viability Population Size 2, Is Sigma Bounded, Random Seed 1337 (Normal
# 1337, Uniform 1338), 100 generations
RUN_CCMAES_SETUP = dict(N=2, lam=8, viability_population_size=2, bound=10.0, sigma_bounded=True, seed=1337,
                        generations=100)
