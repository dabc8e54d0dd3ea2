"""Helpers that load the committed golden fixtures (tests/golden/*.json,
extracted from the reference's tests/python/plot/{cmaes,tmcmc} by
tests/golden/make_golden.py) into oracle / device solver states."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CMAES_STATE_VECTORS = [
    "Current Mean", "Previous Mean", "Covariance Matrix", "Covariance Eigenvector Matrix", "Axis Lengths",
    "Evolution Path", "Conjugate Evolution Path", "Mu Weights", "Best Ever Variables",
]
CMAES_STATE_SCALARS = [
    "Sigma", "Trace", "Effective Mu", "Cumulative Covariance", "Sigma Cumulation Factor", "Damp Factor",
    "Chi Square Number", "Best Ever Value", "Current Best Value", "Infeasible Sample Count",
    "Previous Best Value", "Previous Best Ever Value",
]


def load_cmaes():
    with open(os.path.join(GOLDEN, "cmaes_golden.json")) as f:
        return json.load(f)["generations"]


def load_tmcmc():
    with open(os.path.join(GOLDEN, "tmcmc_golden.json")) as f:
        return json.load(f)["generations"]


def cmaes_variables(gen):
    vs = gen["Variables"]
    return {
        "Lower Bound": [v["Lower Bound"] for v in vs],
        "Upper Bound": [v["Upper Bound"] for v in vs],
        "Initial Value": [v["Initial Value"] for v in vs],
        "Initial Standard Deviation": [v["Initial Standard Deviation"] for v in vs],
        "Minimum Standard Deviation Update": [v["Minimum Standard Deviation Update"] for v in vs],
    }


def population(gen):
    return np.array(gen["Solver"]["Sample Population"], dtype=np.float64)
