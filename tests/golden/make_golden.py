#!/usr/bin/env python3
"""Extract golden vectors from the reference's committed generation files.

Source (read-only, this container only):
  /root/reference/tests/python/plot/cmaes/gen000000{00..101}.json
  /root/reference/tests/python/plot/tmcmc/gen0000000{0..7}.json

These are full per-generation solver states written by the reference's
Experiment::saveState (experiment.cpp.base:120-148).  We keep only the numeric
fields the parity tests compare (data, not code), in two JSON files:

  tests/golden/cmaes_golden.json   every generation: C, B, D, mean, sigma,
                                   paths, population, values, sorting index;
                                   RNG 'Range' hex only where a draw test
                                   needs it (to keep the file small)
  tests/golden/tmcmc_golden.json   all 8 generations, full numeric state

Re-run:  python3 tests/golden/make_golden.py
"""
import json
import os

REF = "/root/reference/tests/python/plot"
OUT = os.path.dirname(os.path.abspath(__file__))

CMAES_KEYS = [
    "Covariance Matrix", "Covariance Eigenvector Matrix", "Axis Lengths", "Current Mean",
    "Previous Mean", "Sigma", "Evolution Path", "Conjugate Evolution Path", "Sample Population",
    "Value Vector", "Sorting Index", "Mu Weights", "Effective Mu", "Cumulative Covariance",
    "Sigma Cumulation Factor", "Damp Factor", "Chi Square Number", "Trace",
    "Conjugate Evolution Path L2 Norm", "Best Ever Value", "Current Best Value",
    "Infeasible Sample Count", "Minimum Covariance Eigenvalue", "Maximum Covariance Eigenvalue",
    "Maximum Diagonal Covariance Matrix Element", "Minimum Diagonal Covariance Matrix Element",
    "Current Min Standard Deviation", "Current Max Standard Deviation", "Best Ever Variables",
    "BDZ Matrix", "Mu Value", "Population Size", "Variable Count", "Mu Type",
    "Previous Best Value", "Previous Best Ever Value", "Model Evaluation Count",
]
RNG_GENS = {0, 1, 2, 3, 19, 20, 49, 50, 99, 100}

TMCMC_KEYS = [
    "Annealing Exponent", "Previous Annealing Exponent", "LogEvidence", "Coefficient Of Variation",
    "Chain Candidates", "Chain Candidates LogLikelihoods", "Chain Candidates LogPriors",
    "Chain Leaders", "Chain Leaders LogLikelihoods", "Chain Leaders LogPriors", "Chain Lengths",
    "Chain Count", "Covariance Matrix", "Mean Theta", "Sample Database",
    "Sample LogLikelihood Database", "Sample LogPrior Database", "Accepted Samples Count",
    "Proposals Acceptance Rate", "Selection Acceptance Rate", "Max Loglikelihood",
    "Population Size", "Variable Count", "Target Coefficient Of Variation", "Covariance Scaling",
    "Max Chain Length", "Min Annealing Exponent Update", "Max Annealing Exponent Update",
]


def load(path):
    with open(path) as f:
        return json.load(f)


def cmaes():
    gens = []
    files = sorted(f for f in os.listdir(f"{REF}/cmaes") if f.startswith("gen"))
    for fn in files:
        d = load(f"{REF}/cmaes/{fn}")
        g = d["Current Generation"]
        s = d["Solver"]
        rec = {"Current Generation": g, "Random Seed": d["Random Seed"], "Solver": {}}
        for k in CMAES_KEYS:
            if k in s:
                rec["Solver"][k] = s[k]
        if g in RNG_GENS:
            rec["Solver"]["Normal Generator"] = {k: s["Normal Generator"][k] for k in ("Random Seed", "Range")}
            rec["Solver"]["Uniform Generator"] = {k: s["Uniform Generator"][k] for k in ("Random Seed", "Range")}
        rec["Variables"] = d["Variables"]
        gens.append(rec)
    return gens


def tmcmc():
    gens = []
    files = sorted(f for f in os.listdir(f"{REF}/tmcmc") if f.startswith("gen"))
    for fn in files:
        d = load(f"{REF}/tmcmc/{fn}")
        s = d["Solver"]
        rec = {"Current Generation": d["Current Generation"], "Random Seed": d["Random Seed"], "Solver": {}}
        for k in TMCMC_KEYS:
            if k in s:
                rec["Solver"][k] = s[k]
        for gname in ("Multinomial Generator", "Multivariate Generator", "Uniform Generator"):
            if gname in s:
                rec["Solver"][gname] = {k: s[gname][k] for k in ("Random Seed", "Range") if k in s[gname]}
        rec["Distributions"] = [
            {k: v for k, v in dist.items() if k in ("Name", "Type", "Minimum", "Maximum", "Random Seed", "Range")}
            for dist in d.get("Distributions", [])
        ]
        rec["Variables"] = d["Variables"]
        gens.append(rec)
    return gens


if __name__ == "__main__":
    c = cmaes()
    with open(f"{OUT}/cmaes_golden.json", "w") as f:
        json.dump({"source": "reference tests/python/plot/cmaes", "generations": c}, f, allow_nan=True)
    t = tmcmc()
    with open(f"{OUT}/tmcmc_golden.json", "w") as f:
        json.dump({"source": "reference tests/python/plot/tmcmc", "generations": t}, f, allow_nan=True)
    print(len(c), "cmaes generations,", len(t), "tmcmc generations")
