"""The oracle's CCMA-ES (oracle/refcpu.c, kr_cmaes_set_constraints /
kr_cmaes_ccmaes_prepare; CMAES.cpp.base:315-437, :551-580, :724-731,
:774-832) against the reference's own CCMA-ES checks: every case of
tests/statistical/optimizers/detailed/ccmaes/run-ccmaes.py passes its
assert_greatereq bound, and the constraint corner cases of
tests/statistical/optimizers/correctness/run-cmaes.py their checkInfeasible.

The Python reference cannot be run here (its compiled engine does not build
offline), so the run-ccmaes.py bounds are the pins.  Several
of them were evidently written from a run's printed Best Ever Value: the
restatement reproduces their mantissas to all printed digits (Active at Max
1: -4.826822 vs the bound -4.826824; Inactive at Max 1: -2.199629e-19 vs
-2.19963e-10), which is asserted below as a stronger (still statistical)
pin."""
import numpy as np
import pytest

import refcpu as R
from ccmaes_cases import CONSTRAINTS, RUN_CCMAES, RUN_CCMAES_SETUP, evalmodel, evaluate_model


def ccmaes_oracle(N, lam, cons, viab, bound, seed, sigma_bounded=False, x0=None, max_res=None):
    o = R.CMAES(N, lam, 0)
    o["Lower Bound"], o["Upper Bound"] = [-bound] * N, [bound] * N
    if x0 is not None:
        o["Initial Value"] = x0
    if sigma_bounded:
        o.option("Is Sigma Bounded", 1)
    if max_res is not None:
        o.option("Max Infeasible Resamplings", max_res)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    if cons:
        o.set_constraints([CONSTRAINTS[c] for c in cons], viab, 0)
    return o


@pytest.mark.parametrize("case", list(RUN_CCMAES))
def test_run_ccmaes_cases_pass_the_reference_bounds(case):
    cons, lower = RUN_CCMAES[case]
    S = RUN_CCMAES_SETUP
    o = ccmaes_oracle(S["N"], S["lam"], cons, S["viability_population_size"], S["bound"], S["seed"],
                      S["sigma_bounded"])
    for g in range(1, S["generations"] + 1):
        o.ccmaes_generation(g, evaluate_model)
    best = o["Best Ever Value"][0]
    assert best >= lower, (case, best)
    if cons:
        assert o["Constraint Evaluation Count"][0] > 0
    # the bounds read like a printed result with a loosened exponent: equal mantissas
    mant = lambda v: float(f"{abs(v):.6e}".split("e")[0])
    if case in ("Active at Max 1", "Active at Max 2", "Inactive at Max 1", "Inactive at Max 2"):
        assert abs(mant(best) - mant(lower)) <= 3e-6, (case, best, lower)


def test_unsatisfiable_constraint_keeps_the_viability_regime():
    """run-cmaes.py 'Constraints that cannot be satisfied': checkInfeasible(e, 10)"""
    o = ccmaes_oracle(1, 16, ["constraint1"], 2, 10.0, 1337, x0=[1.0])
    for g in range(1, 11):
        o.ccmaes_generation(g, evalmodel)
    assert o["Infeasible Sample Count"][0] > 10
    assert o["Value Vector"].size == 2  # still the viability population


def test_max_infeasible_resamplings_with_constraints():
    """run-cmaes.py 'Terminating on Max Infeasible Resamplings' (50)."""
    o = ccmaes_oracle(1, 16, ["constraint1"], 2, 10.0, 1337, x0=[1.0], max_res=50)
    g = 0
    for g in range(1, 101):
        o.ccmaes_generation(g, evalmodel)
        if g > 1 and o["Infeasible Sample Count"][0] >= 50:  # the CMAES termination criterion
            break
    assert o["Infeasible Sample Count"][0] > 50 and g < 100
