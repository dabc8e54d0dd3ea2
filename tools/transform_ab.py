"""A/B of the transform kernel forms (KORALI_AMD_TRANSFORM = tile | bc8 | bc16 |
bc32): every form's populations must equal the 2-D tile form's bit for bit
over a few generations; prints the transform stage time of each."""
import sys, os, hashlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from korali_amd.native import CmaesDevice

CASES = [  # N, lambda, objective, kwargs, generations
    (128, 4096, "rosenbrock", dict(initial_value=np.zeros(128), initial_std=np.ones(128)), 6),
    (70, 1000, "ackley", dict(initial_value=np.full(70, 1.0), initial_std=np.ones(70),
                              lower_bound=np.full(70, -2.0), upper_bound=np.full(70, 3.0)), 5),
    (96, 512, "ackley", dict(initial_value=np.full(96, 1.0), initial_std=np.ones(96), mirrored=True), 5),
    (512, 65536, "ackley", dict(initial_value=np.full(512, 2.0), initial_std=np.ones(512), cov_mode="mfma"), 4),
]
if len(sys.argv) > 1:
    CASES = [c for c in CASES if str(c[0]) in sys.argv[1:]]
FORMS = ("tile", "bc8", "bc16", "bc32")


def run(case, form):
    N, L, obj, kw, G = case
    os.environ["KORALI_AMD_TRANSFORM"] = form
    dev = CmaesDevice(N, L, normal_seed=1337, uniform_seed=1338, **kw)
    h = hashlib.sha256()
    dev.initialize()
    for g in range(1, G + 1):
        dev.sample()
        h.update(np.ascontiguousarray(dev.candidates()).tobytes())
        dev.evaluate(obj)
        dev.update(g)
    dev.synchronize()
    dev.profile(True)
    dev.profile_read("transform")
    for g in range(G + 1, G + 4):
        dev.generation(g, obj)
    dev.synchronize()
    ms, n = dev.profile_read("transform")
    h.update(np.ascontiguousarray(dev["Current Mean"]).tobytes())
    dev.close()
    return h.hexdigest()[:16], ms / max(n, 1)


bad = 0
for case in CASES:
    ref = None
    for form in FORMS:
        dig, ms = run(case, form)
        ref = ref or dig
        ok = dig == ref
        bad += not ok
        print("N=%-4d lam=%-6d %-5s transform %.4f ms  %s %s" % (case[0], case[1], form, ms, dig, "ok" if ok else "MISMATCH"),
              flush=True)
sys.exit(1 if bad else 0)
