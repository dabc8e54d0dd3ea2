"""Device annealing search cost per evaluation: C3-shaped TMCMC runs at
several P, per generation the min_search time, simplex iterations and the
device evaluations (cv at one point over the P log-likelihoods)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from korali_amd.native import TmcmcDevice

for P in [int(a) for a in sys.argv[1:]] or [1024, 8192]:
    dev = TmcmcDevice(32, P, prior_min=[-5.0] * 32, prior_max=[5.0] * 32, prior_seeds=[1337],
                      prior_distribution=[0] * 32, multinomial_seed=1338, multivariate_seed=1339, uniform_seed=1340,
                      target_cov=1.0, covariance_scaling=0.04)
    dev.profile(True)
    dev.profile_read("min_search")
    tot_ms = tot_ev = tot_it = 0.0
    for g in range(1, 40):
        e0 = dev["Device Search Evaluations"][0]
        dev.generation(g)
        dev.synchronize()
        ms, n = dev.profile_read("min_search")
        ev = dev["Device Search Evaluations"][0] - e0
        it = dev["Min Search Iterations"][0]
        tot_ms += ms
        tot_ev += ev
        tot_it += it
        print(f"P={P} g={g} min_search {ms:.3f} ms iters {it:.0f} evals {ev:.0f} us/eval {1e3 * ms / max(ev, 1):.2f}",
              flush=True)
        if dev["Previous Annealing Exponent"][0] >= 1.0:
            break
    print(f"P={P} TOTAL {tot_ms:.2f} ms, {tot_ev:.0f} evals, {tot_it:.0f} iters, {1e3 * tot_ms / tot_ev:.2f} us/eval, "
          f"relaunches {dev['Device Search Relaunches'][0]:.0f}", flush=True)
    t = dev["Device Search Phase Times"]
    r = dev["Device Search Rounds"][0]
    print(f"P={P} per round (us): controller wait {1e3 * t[0] / r:.2f} combine {1e3 * t[1] / r:.2f} "
          f"logic {1e3 * t[2] / r:.2f}; worker wait {1e3 * t[3] / r:.2f} evaluate {1e3 * t[4] / r:.2f} "
          f"reduce+publish {1e3 * t[5] / r:.2f}; rounds {r:.0f}", flush=True)
    if os.environ.get("KORALI_AMD_NM_SYM", "1") != "0":
        print(f"P={P} symmetric kernel per round (us): hand-off wait {1e3 * t[0] / r:.2f}, simplex logic "
              f"{1e3 * t[1] / r:.2f}, evaluate + publish {1e3 * t[2] / r:.2f}, combine {1e3 * t[5] / r:.2f}; "
              f"whole launches {t[3]:.3f} ms, prologues {t[4]:.3f} ms (host-timed min_search {tot_ms:.3f} ms)",
              flush=True)
    dev.close()
