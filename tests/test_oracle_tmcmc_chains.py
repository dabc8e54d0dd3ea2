"""CPU oracle: TMCMC chains with more than one step per generation (Burn In,
Per Generation Burn In, Max Chain Length > 1; TMCMC.cpp.base:107-157,
:229-252, :331-360, :781-789).

No reference fixture covers these settings (the committed TMCMC result
files use Max Chain Length 1 and Burn In 0), so parity with the reference is
unpinned here beyond the restatement; these tests pin the bookkeeping
invariants the reference's loop implies and reproduce the reference's own
statistical checks (tests/statistical/samplers/correctness/run-tmcmc-2.py:
mean 0 +- 0.05, std 1 +- 0.05 of the final sample database).
"""
import numpy as np
import pytest

import refcpu as R


def make(N, P, seed, lo, hi, **opts):
    o = R.TMCMC(N, P)
    o["Prior Minimum"] = [lo] * N
    o["Prior Maximum"] = [hi] * N
    o.set_prior_map([0] * N)
    pergen = opts.pop("Per Generation Burn In", None)
    for k, v in opts.items():
        o.option(k, v)
    if pergen is not None:
        o.set_per_generation_burn_in(pergen)
    # Korali's seed order: the experiment's distribution, then Multinomial,
    # Multivariate, Uniform (TMCMC.config Internal Settings order)
    for which, s in ((3, seed), (0, seed + 1), (1, seed + 2), (2, seed + 3)):
        R.lib().kr_rng_seed(o.rng(which).ptr, s)
    return o


def run(o, max_gens=60):
    hist = []
    for g in range(1, max_gens + 1):
        cc = int(o["Chain Count"][0]) if g > 1 else o.P
        lengths = o["Chain Lengths"].copy() if g > 1 else np.ones(o.P)
        evals0 = o["Model Evaluation Count"][0]
        o.generation(g)
        hist.append(dict(g=g, started=cc, lengths=lengths, burn=o["Current Burn In"][0],
                         evals=o["Model Evaluation Count"][0] - evals0, db=o["Database Entries"][0],
                         accepted=o["Accepted Samples Count"][0], rho=o["Annealing Exponent"][0],
                         prev=o["Previous Annealing Exponent"][0], cl=o["Chain Lengths"].copy(),
                         count=o["Chain Count"][0], mcl=None))
        # termination "Target Annealing Exponent" (TMCMC.config): the
        # generation after the exponent reached 1 samples the posterior
        if o["Previous Annealing Exponent"][0] >= 1.0:
            break
    return hist


def test_run_tmcmc_2_statistics():
    """run-tmcmc-2.py: N=1, U(-20, 20) prior, loglik -0.5 x^2, P=5000,
    Covariance Scaling 0.01, Burn In 3, Target CoV 0.4, seed 0xC0FFEE."""
    o = make(1, 5000, 0xC0FFEE, -20.0, 20.0, **{"Covariance Scaling": 0.01, "Default Burn In": 3,
                                                  "Target Coefficient Of Variation": 0.4})
    hist = run(o)
    assert hist[-1]["prev"] >= 1.0
    db = o["Sample Database"]
    assert abs(np.mean(db) - 0.0) <= 0.05
    assert abs(np.std(db) - 1.0) <= 0.05


@pytest.mark.parametrize("mcl,burn,pergen", [(1, 2, None), (3, 0, None), (4, 1, [3, 0, 2])])
def test_chain_bookkeeping(mcl, burn, pergen):
    N, P = 3, 400
    opts = {"Max Chain Length": mcl, "Default Burn In": burn, "Covariance Scaling": 0.04}
    if pergen is not None:
        opts["Per Generation Burn In"] = pergen
    o = make(N, P, 4242, -5.0, 5.0, **opts)
    hist = run(o, 25)
    for h in hist:
        g = h["g"]
        B = 0 if g == 1 else (pergen[g - 2] if pergen is not None and g - 2 < len(pergen) else burn)
        assert h["burn"] == B
        # every started chain runs Chain Lengths[c] + B steps; the lengths of
        # the started chains sum to P, so the database always holds P entries
        assert np.sum(h["lengths"][:h["started"]]) == P
        assert h["evals"] == P + h["started"] * B
        assert h["db"] == P
        assert 0 <= h["accepted"] <= P
        # leader expansion :331-360: lengths in [1, mcl] for count chains, 0 after
        cl, cnt = h["cl"], int(h["count"])
        assert np.all(cl[:cnt] >= 1) and np.all(cl[:cnt] <= mcl) and np.all(cl[cnt:] == 0)
        assert np.sum(cl) == P
    if mcl > 1:
        assert any(int(h["count"]) < P for h in hist)
