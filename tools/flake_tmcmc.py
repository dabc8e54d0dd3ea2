"""Determinism probe for the device TMCMC path (no distributed): two
unsharded handles from the same seeds (Max Chain Length 3, Burn In 1) must
agree bit for bit every generation.  Prints the first difference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from korali_amd.native import TmcmcDevice

KEYS = ("Chain Candidates", "Chain Candidates LogLikelihoods", "Chain Leaders", "Sample Database", "Mean Theta",
        "Covariance Matrix", "Annealing Exponent", "Accepted Samples Count")


def main():
    N, P, gens = 3, 500, 8
    kw = dict(prior_min=[-5.0] * N, prior_max=[5.0] * N, prior_seeds=[77], prior_distribution=[0] * N,
              multinomial_seed=78, multivariate_seed=79, uniform_seed=80, max_chain_length=3, default_burn_in=1)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    bad = 0
    for rep in range(reps):
        a, b = TmcmcDevice(N, P, **kw), TmcmcDevice(N, P, **kw)
        for g in range(1, gens + 1):
            a.generation(g)
            b.generation(g)
            a.synchronize()
            b.synchronize()
            for k in KEYS:
                if a[k].tobytes() != b[k].tobytes():
                    print(f"rep {rep} gen {g}: {k} differs", flush=True)
                    bad += 1
            if bad:
                break
            for which in range(4):
                if a.get_rng(which) != b.get_rng(which):
                    print(f"rep {rep} gen {g}: rng {which} differs", flush=True)
                    bad += 1
            if a["Previous Annealing Exponent"][0] >= 1.0:
                break
        a.close()
        b.close()
        if bad:
            break
    print("FLAKE_CHECK", "FAIL" if bad else "PASS", flush=True)


if __name__ == "__main__":
    main()
