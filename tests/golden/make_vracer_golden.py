"""Extract (data only) the VRACER facts the reference's own result files hold
into tests/golden/vracer_abf2d.json.

Source: /root/reference/tests/python/rlview/abf2d_vracer{1,2}/gen0000000{0,50}.json
(Korali result files of a 4-state / 3-action VRACER run, 2 x 64 tanh layers,
Normal policy).  Kept: the Variables and Solver settings that define the
policy; the policy description Korali wrote (Parameter Count / Scaling /
Shifting / Transformation Masks, Action Shifts / Scales); the hyperparameter
vector's layout facts at generation 0 (length, which entries are exactly
zero, per-layer max |w|); the reward-rescaling record at generation 50.

    python tests/golden/make_vracer_golden.py
"""
import json
import os

SRC = "/root/reference/tests/python/rlview"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vracer_abf2d.json")


def layer_facts(theta, sizes):
    k, out = 0, []
    for ic, oc in zip(sizes[:-1], sizes[1:]):
        W, b = theta[k:k + ic * oc], theta[k + ic * oc:k + ic * oc + oc]
        k += ic * oc + oc
        out.append({"in": ic, "out": oc, "weight_max_abs": max(abs(x) for x in W),
                    "weights_nonzero": sum(1 for x in W if x != 0.0), "bias_all_zero": all(x == 0.0 for x in b)})
    return k, out


def main():
    runs = {}
    for run in ("abf2d_vracer1", "abf2d_vracer2"):
        g0 = json.load(open(os.path.join(SRC, run, "gen00000000.json")))
        g50 = json.load(open(os.path.join(SRC, run, "gen00000050.json")))
        s0, s50 = g0["Solver"], g50["Solver"]
        theta = s0["Training"]["Current Policy"]["Policy"]
        hl = s0["Neural Network"]["Hidden Layers"]
        sizes = [g0["Problem"]["State Vector Size"]] + [hl[2 * l]["Output Channels"] for l in range(len(hl) // 2)] + \
                [1 + s0["Policy"]["Parameter Count"]]
        used, layers = layer_facts(theta, sizes)
        runs[run] = {
            "variables": g0["Variables"],
            "problem": {k: g0["Problem"][k] for k in ("State Vector Size", "Action Vector Size", "State Vector Indexes",
                                                      "Action Vector Indexes")},
            "solver": {"Policy": {"Distribution": s0["Policy"]["Distribution"]},
                       "Neural Network": {"Hidden Layers": hl}},
            "expected": {"Policy": {k: s0["Policy"][k] for k in ("Parameter Count", "Parameter Scaling",
                                                                 "Parameter Shifting",
                                                                 "Parameter Transformation Masks")},
                         "Action Shifts": s0["Action Shifts"], "Action Scales": s0["Action Scales"]},
            "hyperparameters": {"count": len(theta), "layer_sizes": sizes, "covered": used, "layers": layers},
            "reward_rescaling_gen50": {"Sigma": s50["Reward"]["Rescaling"]["Sigma"],
                                       "Sum Squared Rewards": s50["Reward"]["Rescaling"]["Sum Squared Rewards"],
                                       "Experience Count Per Environment": s50["Experience Count Per Environment"],
                                       "Maximum Size": s50["Experience Replay"]["Maximum Size"]},
            "solver_keys_gen50": sorted(s50.keys()),
        }
    json.dump(runs, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
