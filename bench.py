#!/usr/bin/env python3
"""bench.py — CMA-ES generation throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): CMA-ES, 128-dim negative
Rosenbrock (examples/optimization/stochastic/_model/model.py:23-34),
λ = 4096, μ = 2048 (Logarithmic), x0 = 0, σ0 = 1, seed 1337, bounds ±∞.
A step is one full generation (CMAES::runGeneration): GSL-faithful
eigendecomposition, mt19937 polar draw of λ·N normals, x = m + σ B(D∘z),
batched objective, sort, mean/paths, rank-μ covariance update, σ update.
Everything runs on the device; the host only enqueues.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--cov exact|mfma]

N > 1: one process per GPU — launched by torch.distributed.run (RANK /
WORLD_SIZE set), or, when WORLD_SIZE is unset, bench.py starts the N rank
processes itself before touching the GPU.  Every rank runs its own C2
experiment (seed 1337 + rank) — "replicas", weak scaling, no collective on
the data path (λ = 4096 fits one GPU many times over);
value = total generations/s over all ranks (max-over-ranks wall time).
Beside it, `c4_sharded`: the C4 experiment (512-dim Ackley, λ = 65536)
through korali.Engine on one rank and sharded over all N ranks (the
Distributed conduit, exact covariance order), its rates and speed-up, and
whether the two runs ended bit-identical.

The JSON line also carries `roofline` for the dominant kernel (algorithmic
FLOPs per launch / its HIP-event time on the solver's stream) and
`cpu_baseline` (the bit-exact CPU oracle, one core, bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_VARS, LAMBDA = 128, 4096
MU = LAMBDA // 2
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector == FP64 matrix (spec)
HBM_PEAK_GBS = 8000.0

# algorithmic FP64 work per launch of each stage at C2
def stage_flops(N, lam, mu):
    """Algorithmic FLOPs per launch of the profiled CMA-ES stages at (N, lambda, mu)."""
    return {"eigen": (8.0 / 3.0) * N ** 3 + 6.0 * 1.1 * N ** 3,
            "eigen_tridiag": (4.0 / 3.0) * N ** 3, "eigen_unpack": (4.0 / 3.0) * N ** 3,
            "eigen_apply": 6.0 * 1.1 * N ** 3,
            "transform": 2.0 * lam * N ** 2, "covariance": 1.0 * mu * N * (N + 1),
            "rankmu_mfma": 1.0 * mu * N * (N + 1), "objective": 8.0 * lam * N}


STAGE_FLOPS = {
    # GSL symmv pieces: tridiagonalisation (4/3)N^3, unpack 2N^3 (nominal),
    # Givens application 6 flops * N rows * ~1.1 N^2 rotations
    "eigen": (8.0 / 3.0) * N_VARS ** 3 + 6.0 * 1.1 * N_VARS ** 3,
    "eigen_tridiag": (4.0 / 3.0) * N_VARS ** 3,
    "eigen_unpack": (4.0 / 3.0) * N_VARS ** 3,  # householder_hm over N-2 reflectors: sum of 4 n^2
    "eigen_apply": 6.0 * 1.1 * N_VARS ** 3,
    "transform": 2.0 * LAMBDA * N_VARS ** 2,
    # rank-mu sum: the SYRK count mu N (N+1) (the lower triangle and the
    # diagonal, 2 flops per term), not the full-GEMM 2 mu N^2
    "covariance": 1.0 * MU * N_VARS * (N_VARS + 1),
    "rankmu_mfma": 1.0 * MU * N_VARS * (N_VARS + 1),
    "objective": 8.0 * LAMBDA * N_VARS,
}


# kernels behind each profiled stage (names as in profiles/<round>/*_pmc_traffic.csv)
STAGE_KERNELS = {
    # a tuple lists alternatives (the kernel the size selects); template
    # instances match their base name
    "eigen_tridiag": [("kg::k_tridiag_sq", "kg::k_tridiag_mw2", "kg::k_tridiag_1wg2", "kg::k_tridiag_1wg",
                       "kg::k_tridiag_mw", "kg::k_tridiag")],
    "eigen_unpack": [("kg::k_unpack_wv", "kg::k_unpack_mw", "kg::k_unpack")], "eigen_apply": ["kg::k_apply"],
    "transform": [("kg::k_transform_sc", "kg::k_transform")], "objective": [("kg::k_objective2", "kg::k_objective")],
    "covariance": ["kg::k_rankmu_prep", ("kg::k_adaptC_lane", "kg::k_adaptC_row", "kg::k_adaptC_exact3", "kg::k_adaptC_exact2")],
    "rankmu_mfma": ["kg::k_rankmu_tile"],
    "rng_polar": ["kg::k_polar_count", "kg::k_scan_counts", "kg::k_polar_scatter"],
    "mean_paths": ["kg::k_update_best", "kg::k_gather_selected", ("kg::k_mean3", "kg::k_mean2", "kg::k_mean"),
                   ("kg::k_paths3", "kg::k_paths2", "kg::k_paths")],
    # C3 (TMCMC): the weighted mean / covariance stage
    "mean_cov": [("kg::k_tm_factors_mean_t", "kg::k_tm_factors_mean"), ("kg::k_tm_wsum_rows<false>", "kg::k_tm_wsum<false>"),
                 ("kg::k_tm_factors_cov_t", "kg::k_tm_factors_cov"), ("kg::k_tm_wsum_rows<true>", "kg::k_tm_wsum<true>")],
    # C3: the annealing search (symmetric form by default)
    "min_search": [("kg::k_tm_nm_sym", "kg::k_tm_nm_search")],
}
# stages timed on the host core (wall clock), not device kernels
HOST_STAGES = ("eigen_chase_host", "eigen_tridiag_host", "eigen_c_wait", "eigen_dsd_wait")
# device stages whose duration the host sets: k_fetch_h spins until the host
# tridiagonalisation publishes the reflectors, k_apply replays the rotations
# as the host chase publishes them (its event time is the chase's)
HOST_FED = ("eigen_fetch_h", "eigen_apply", "eigen_publish_c")
# what bounds each stage that can come out dominant (the roofline's note)
STAGE_NOTES = {
    "eigen_unpack": "symmtd_unpack (Q from the N-2 Householder reflectors, householder_hm): per reflector an "
                    "ordered dot chain per column of Q in GSL order, so latency-bound far below the FP64 roof; it "
                    "runs beside the host core's Givens chase, off the generation's critical path",
    "eigen_tridiag": "GSL's Householder tridiagonalisation on the device (KORALI_AMD_TRIDIAG=sq/mw2): three ordered "
                     "FP64 add chains per step whose order the bit-exact contract fixes",
    "covariance": "adaptC's exact rank-mu sums: one ordered chain of mu Markstein quotients per lower-triangle "
                  "entry (the reference's order), so chain- and issue-bound, not HBM-bound",
    "mean_paths": "the mean / evolution paths: ordered sums over the mu selected rows (latency-bound chains)",
    "transform": "x = m + sigma B (D o z): FP64 VALU (no FMA, bit-exact), the ordered K loop per output",
}
PROFILE_ROUNDS = ("r6", "r5", "r4", "r3", "r2")
# the kernel behind a stage as rocprof names it (C2 shapes)
STAGE_KERNEL_NAME = {"eigen_tridiag": "kg::k_tridiag_sq", "eigen_unpack": "kg::k_unpack_wv",
                     "covariance": "kg::k_adaptC_row", "transform": "kg::k_transform",
                     "mean_paths": "kg::k_mean3 + kg::k_paths3 + kg::k_gather_selected + kg::k_update_best"}  # newest first: a PMC summary is read from the newest round that holds it


def profile_file(name):
    """(absolute path, repo-relative path) of the newest committed profiles/<round>/<name>."""
    for r in PROFILE_ROUNDS:
        path = os.path.join(ROOT, "profiles", r, name)
        if os.path.exists(path):
            return path, f"profiles/{r}/{name}"
    return os.path.join(ROOT, "profiles", PROFILE_ROUNDS[0], name), None


def pmc_traffic(stage, csv_name="c2_pmc_traffic.csv"):
    """HBM bytes per launch of a stage's kernels from the committed PMC passes
    (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE), or None."""
    import csv
    path, _ = profile_file(csv_name)
    if stage not in STAGE_KERNELS or not os.path.exists(path):
        return None, None
    rows = {r["kernel"]: r for r in csv.DictReader(open(path))}

    def find(k):
        for alt in (k if isinstance(k, tuple) else (k,)):
            for name, r in rows.items():
                if name == alt or name.startswith(alt + "<"):
                    return r
        return None

    tot, raw = 0.0, 0.0
    for k in STAGE_KERNELS[stage]:
        r = find(k)
        if r is None:
            return None, None
        tot += (float(r["fetch_KB_x2"]) + float(r["write_KB"])) * 1024
        raw += (float(r["fetch_KB_raw"]) + float(r["write_KB"])) * 1024
    return tot, raw


def rankmu_roofline(ms, mu, n, csv_name):
    """The rank-mu MFMA kernel (k_rankmu_tile) against the FP64 matrix peak:
    algorithmic work = the SYRK count mu N (N+1) (lower triangle with the
    diagonal, 2 flops per term); the kernel executes the lower 64x64 tiles
    (executed_flops_per_launch, slightly more: the diagonal tiles' upper
    halves); HIP events around its launch on its own stream."""
    flops = 1.0 * mu * n * (n + 1)
    nt = (n + 63) // 64
    executed = nt * (nt + 1) // 2 * 64 * 64 * 2.0 * mu
    achieved = flops / (ms * 1e-3) / 1e12
    traffic, raw = pmc_traffic("rankmu_mfma", csv_name)
    return {"kernel": "kg::k_rankmu_tile", "bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "avg_launch_ms": ms,
            "algorithmic_flops_per_launch": flops, "executed_flops_per_launch": executed,
            "executed_frac": executed / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
            "algorithmic_bytes_per_launch": 8.0 * (mu * n + n * n),
            "traffic": traffic, "traffic_source": profile_file(csv_name)[1] if traffic else None}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class pinned_core:
    """Pin the calling process to one core for the CPU-baseline timing
    (`taskset -c <core>`), restoring the affinity after."""

    def __init__(self):
        self.saved = os.sched_getaffinity(0)
        # the middle core of the allowed set: core 0 also takes the host's
        # interrupts and housekeeping, which showed up as window-to-window noise
        self.core = sorted(self.saved)[len(self.saved) // 2]

    def __enter__(self):
        os.sched_setaffinity(0, {self.core})
        return self.core

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.saved)


def _cmaes_oracle_rate(variant, warmup, gens_min, seconds_budget, N=N_VARS, lam=LAMBDA, objective="rosenbrock",
                       x0=0.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu as R

    R.lib(variant).kr_set_threads(1)  # the reference is single-threaded (no OpenMP in CMAES)
    o = R.CMAES(N, lam, lam // 2, variant=variant)
    o["Initial Value"] = np.full(N, x0)
    o["Initial Standard Deviation"] = np.ones(N)
    R.lib(variant).kr_rng_seed(o.rng(0).ptr, 1337)
    R.lib(variant).kr_rng_seed(o.rng(1).ptr, 1338)
    g = 0
    for _ in range(warmup):  # warm-up (includes initialisation)
        g += 1
        o.generation(g, objective)
    n, t0 = 0, time.perf_counter()
    while True:
        g += 1
        n += 1
        o.generation(g, objective)
        el = time.perf_counter() - t0
        if n >= gens_min and el > seconds_budget:
            break
        if el > 4 * seconds_budget:  # hard bound on a slow host
            break
    return n, el


def _dispatch_rate(seconds_budget):
    """BASELINE.md §2 variant (ii): generations/s of C2 with per-sample JSON
    dispatch (oracle/dispatch_baseline, built by `make -C oracle`), or None
    when the binary is absent."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "dispatch_baseline")
    if not os.path.exists(exe):
        return None
    r = subprocess.run([exe, str(N_VARS), str(LAMBDA), "10", "100", str(seconds_budget)], capture_output=True,
                       text=True, timeout=60 * seconds_budget + 120)
    if r.returncode != 0:
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])["generations_per_sec"]


def _cmaes_oracle_windows(variant, warmup, windows, gens_min, seconds_per_window):
    """Per-window generations/s of the oracle's C2 loop: `windows` back-to-back
    windows of at least `gens_min` generations and `seconds_per_window` each,
    after `warmup` generations (one experiment, so the state keeps evolving)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu as R

    R.lib(variant).kr_set_threads(1)
    o = R.CMAES(N_VARS, LAMBDA, LAMBDA // 2, variant=variant)
    o["Initial Value"] = np.zeros(N_VARS)
    o["Initial Standard Deviation"] = np.ones(N_VARS)
    R.lib(variant).kr_rng_seed(o.rng(0).ptr, 1337)
    R.lib(variant).kr_rng_seed(o.rng(1).ptr, 1338)
    g = 0
    for _ in range(warmup):
        g += 1
        o.generation(g, "rosenbrock")
    rates, total = [], 0
    for _ in range(windows):
        n, t0 = 0, time.perf_counter()
        while True:
            g += 1
            n += 1
            o.generation(g, "rosenbrock")
            el = time.perf_counter() - t0
            if (n >= gens_min and el > seconds_per_window) or el > 4 * seconds_per_window:
                break
        rates.append(n / el)
        total += n
    return rates, total


def cpu_baseline(seconds_budget=8.0, windows=5):
    """The reference's arithmetic on this host's CPU: the
    oracle restatement, -O3 without -march, one thread pinned to one core,
    10 warm-up generations, then `windows` timed windows of C2 (at least 20
    generations each); `value` is the MEDIAN window rate (min / max beside
    it: one window of a shared host can catch a neighbour's burst).  The build
    against the system libm (the speed the reference itself runs at here —
    the conservative baseline, variant (i): solver arithmetic with an inline
    objective, no per-sample dispatch); the bit-exact build (correctly rounded
    log/exp, slower) is reported beside it on a shorter sample."""
    progress("cpu baseline (oracle, one pinned core)")
    with pinned_core() as core:
        rates, gens = _cmaes_oracle_windows("libm", 10, windows, 20, seconds_budget / windows)
        gens_cr, el_cr = _cmaes_oracle_rate("cr", 2, 10, seconds_budget / 3)
        v2 = _dispatch_rate(seconds_budget / 2)
    med = float(np.median(rates))
    return {"value": med, "unit": "generations/s", "cores": 1, "kind": "port",
            "window_rates": rates, "min": min(rates), "max": max(rates),
            "samples_per_sec": med * LAMBDA,
            "bit_exact_port_value": gens_cr / el_cr,
            "variant_ii_value": v2,
            "variant_ii": "the same loop with every sample dispatched as a korali::Json Sample through a "
                          "Sequential-conduit loop (oracle/dispatch_baseline.cpp, -O3, system libm), 10 warm-up",
            "cpu": f"{cpu_model()}, 1 of {os.cpu_count()} cores (pinned to core {core})",
            "sample": f"{gens} generations of C2 (N=128, lambda=4096) in {windows} windows after 10 warm-up "
                      f"(value = median window), oracle/refcpu.c -O3 (no -march) with system libm, 1 thread, "
                      f"variant (i) inline objective; bit-exact CR build: {gens_cr} generations after 2 warm-up"}


def c2_experiment(cov, generations):
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Kernel"] = "Negative Rosenbrock"
    for i in range(N_VARS):
        e["Variables"][i]["Name"] = "X" + str(i)
        e["Variables"][i]["Initial Value"] = 0.0
        e["Variables"][i]["Initial Standard Deviation"] = 1.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = LAMBDA
    e["Solver"]["Covariance Update"] = "MFMA" if cov == "mfma" else "Exact"
    e["Solver"]["Termination Criteria"]["Max Generations"] = generations
    e["Random Seed"] = 1337
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    return e


def engine_rate(steps, warmup, cov):
    """The same C2 experiment through the korali API (C++ engine: termination
    checks and bookkeeping every generation, as Korali's Experiment::run
    does).  Returns (differential, end_to_end):
    * differential: fresh k.run(e) of `short` and of `long` generations
      (three of each, medians); their difference cancels the fixed cost of a
      run (handle creation, initialisation, the first generation), leaving
      the engine's per-generation rate;
    * end_to_end: one fresh k.run(e) of `steps` generations, wall clock,
      handle creation and initialisation included;
    * in_run: from that same run, generations `warmup`+1 .. `steps` by the
      engine's own completion marks (korali._generation_completion_times:
      when each generation's termination check returned), no subtraction
      of two runs."""
    import korali
    progress("engine rate (korali.Engine runs of C2)")
    k = korali.Engine()
    k.run(c2_experiment(cov, warmup))  # (first-use costs: module load, code objects)
    short, long_ = 50, 50 + max(steps, 300)
    med = {}
    for n in (short, long_):
        ts = []
        for _ in range(3):
            f = c2_experiment(cov, n)
            t0 = time.perf_counter()
            k.run(f)
            ts.append(time.perf_counter() - t0)
        med[n] = sorted(ts)[1]
    diff = (long_ - short) / (med[long_] - med[short])
    f = c2_experiment(cov, steps)
    t0 = time.perf_counter()
    k.run(f)
    e2e = steps / (time.perf_counter() - t0)
    marks = korali._generation_completion_times(f)
    w = min(warmup, steps - 1)
    in_run = (steps - w) / (marks[steps] - marks[w]) if len(marks) == steps + 1 else None
    # short runs: the fixed cost against 20 generations (median of five)
    ts = []
    for _ in range(5):
        f = c2_experiment(cov, 20)
        t0 = time.perf_counter()
        k.run(f)
        ts.append(time.perf_counter() - t0)
    e2e20 = 20 / sorted(ts)[2]
    return diff, e2e, in_run, e2e20


_T_START = time.perf_counter()


def progress(msg):
    """One line on stderr per phase (a long default run stays visibly alive;
    the JSON line alone goes to stdout)."""
    print(f"[bench {time.perf_counter() - _T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


C1_N, C1_LAMBDA, C1_GENS = 8, 16, 1000


def c1_experiment(objective):
    """CMA-ES, 8-dim negative Rosenbrock, lambda=16,
    x0=0, sigma0=1, Max Generations 1000, seed 1337, through korali.Engine.
    objective "kernel": the device objective; "python": the reference
    example's Python model (examples/optimization/model.py negative_rosenbrock)
    called per sample through the Sequential conduit."""
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    if objective == "kernel":
        e["Problem"]["Objective Kernel"] = "Negative Rosenbrock"
    else:
        def model(s):
            x = s["Parameters"]
            s["F(x)"] = -sum(100.0 * (x[i + 1] - x[i] ** 2) ** 2 + (1.0 - x[i]) ** 2 for i in range(len(x) - 1))
        e["Problem"]["Objective Function"] = model
    for i in range(C1_N):
        e["Variables"][i]["Name"] = "X" + str(i)
        e["Variables"][i]["Initial Value"] = 0.0
        e["Variables"][i]["Initial Standard Deviation"] = 1.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = C1_LAMBDA
    e["Solver"]["Termination Criteria"]["Max Generations"] = C1_GENS
    e["Random Seed"] = 1337
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    return e


def c1_line(cpu=True):
    """C1 beside the reference's CPU arithmetic: whole korali.Engine runs of
    1000 generations (creation, initialisation and the final state included),
    median of three, with the device objective and with the Python model;
    refcpu: the oracle restatement (-O3, system libm, one pinned core) on the
    same shape."""
    import korali
    progress("C1 line (korali.Engine, N=8, lambda=16)")
    k = korali.Engine()
    k.run(c1_experiment("kernel"))  # (first-use costs)
    out = {"workload": "C1: CMA-ES, 8-dim negative Rosenbrock, lambda=16, mu=8, x0=0, sigma0=1, "
                       "1000 generations, seed 1337, korali.Engine (Sequential conduit)"}
    for obj in ("kernel", "python"):
        ts = []
        for _ in range(3):
            e = c1_experiment(obj)
            t0 = time.perf_counter()
            k.run(e)
            ts.append(time.perf_counter() - t0)
        out[f"engine_{obj}_generations_per_sec"] = C1_GENS / sorted(ts)[1]
    if cpu:
        progress("C1 refcpu (whole 1000-generation runs, one pinned core)")
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import refcpu as R
        lib = R.lib("libm")
        lib.kr_set_threads(1)
        runs, t0 = 0, time.perf_counter()
        with pinned_core():
            # whole runs from a fresh state, like the engine's (a run continued
            # past its 1000 generations degenerates the covariance)
            while runs < 3 or time.perf_counter() - t0 < 1.0:
                o = R.CMAES(C1_N, C1_LAMBDA, C1_LAMBDA // 2, variant="libm")
                o["Initial Value"] = np.zeros(C1_N)
                o["Initial Standard Deviation"] = np.ones(C1_N)
                lib.kr_rng_seed(o.rng(0).ptr, 1337)
                lib.kr_rng_seed(o.rng(1).ptr, 1338)
                for g in range(1, C1_GENS + 1):
                    o.generation(g, "rosenbrock")
                runs += 1
        el = time.perf_counter() - t0
        out["refcpu_generations_per_sec"] = runs * C1_GENS / el
        out["refcpu_sample"] = (f"{runs} whole C1 runs of {C1_GENS} generations, oracle/refcpu.c -O3 (no -march), "
                                f"system libm, inline objective, 1 pinned core")
        out["engine_kernel_vs_refcpu"] = out["engine_kernel_generations_per_sec"] / out["refcpu_generations_per_sec"]
    return out


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets
    them) before this process touches the GPU, and exit with the worst
    return code.  Rank 0 prints the JSON line."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def rank_device(local_rank):
    """The GPU of a rank: LOCAL_RANK, folded onto the visible devices (several
    ranks share one device when there are fewer GPUs than ranks)."""
    import torch
    n = torch.cuda.device_count()  # (does not initialise the GPU on this image)
    return local_rank % max(1, n), n


EXCHANGE_STAGES = ("exchange_fitness", "exchange_rows", "exchange_covariance", "exchange_partials")


def exchange_ms(e, dist):
    """The sharded update's exchange collectives, device time per generation
    (HIP events around each RCCL call on the handle's stream, the engine's
    KORALI_AMD_EXCHANGE_PROFILE=1; mean over the run's generations), max over
    ranks.  None when the engine did not record them."""
    import torch
    got = {}
    try:
        em = e["Results"]["Exchange Milliseconds"]
        for st in EXCHANGE_STAGES:
            try:
                got[st] = float(em[st])
            except (KeyError, TypeError, IndexError, ValueError):
                pass
    except (KeyError, TypeError):
        pass
    v = torch.tensor([got.get(st, -1.0) for st in EXCHANGE_STAGES], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    out = {st: float(x) for st, x in zip(EXCHANGE_STAGES, v.tolist()) if x >= 0}
    return out or None


def c4_scaling(args, world, rank, dist):
    """The C4 experiment through korali.Engine on rank 0 alone (Sequential
    conduit) and sharded over all ranks (Distributed conduit, exact
    covariance order); generations/s of each over the last `steps`
    generations (the engine's completion marks, slowest rank), the speed-up,
    and whether both runs end in the same state bit for bit."""
    import korali
    import torch
    steps, w = max(2, min(args.steps, 10)), 2
    total = w + steps

    def rate(e):
        marks = korali._generation_completion_times(e)
        return marks[total] - marks[w]

    one, state1 = None, None
    if rank == 0:
        e1 = c4_experiment(total, "Exact")
        korali.Engine().run(e1)
        one = steps / rate(e1)
        state1 = [e1["Solver"][k] for k in ("Current Mean", "Covariance Matrix", "Sigma")]
    dist.barrier()
    devs = rank_device(int(os.environ.get("LOCAL_RANK", "0")))[1]
    transport = "RCCL" if devs >= world else "Host"  # (RCCL refuses two ranks on one device)
    k = korali.Engine()
    k["Conduit"]["Type"] = "Distributed"
    k["Conduit"]["Transport"] = transport
    eN = c4_experiment(total, "Exact")
    os.environ.setdefault("KORALI_AMD_EXCHANGE_PROFILE", "1")
    k.run(eN)
    exch = exchange_ms(eN, dist)
    t = torch.tensor([rate(eN)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank != 0:
        return None
    many = steps / float(t.item())
    same = state1 == [eN["Solver"][k] for k in ("Current Mean", "Covariance Matrix", "Sigma")]
    return {"workload": "C4: CMA-ES, 512-dim negative Ackley, lambda=65536, mu=32768, Exact covariance order, "
                        "korali.Engine", "ranks": world, "transport": transport, "steps": steps, "warmup": w,
            "generations_per_sec_1_rank": one, f"generations_per_sec_{world}_ranks": many, "speedup": many / one,
            "bit_identical_to_1_rank": bool(same), "scaling": "strong",
            "exchange_ms_per_generation": exch,
            "note": "the eigendecomposition (GSL order: host tridiagonalisation ~1.3 ms on 6 threads + Givens chase "
                    "~4.4 ms of an ~11.8 ms 1-GPU generation, profiles/r6/bench_c4.json) is replicated on every rank, "
                    "which bounds the speed-up at about 1.5x for any rank count (DESIGN.md §6)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--cov", default="exact", choices=["exact", "mfma"],
                    help="exact (default): bit-exact rank-mu order, the reference's trajectory; mfma: FP64 matrix "
                         "cores, <= 1e-12 per step (reported beside the exact rate)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 line (profiling runs: keeps the C2 kernels' "
                                                        "statistics free of the N=8 launches)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c2: the BASELINE metric (CMA-ES); c3: TMCMC N=32, P=8192; c4: CMA-ES 512-dim Ackley, "
                         "lambda=65536, population sharded over the ranks; c5: VRACER, 4096 CartPole rollouts")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.workload in ("c2", "c4"):
        sys.exit(spawn_ranks(args.gpus))
    if args.workload in ("c3", "c5") and args.gpus > 1:
        raise SystemExit(f"--workload {args.workload} runs on one GPU (replicas only: start one bench per GPU)")
    if args.workload == "c3":
        return run_c3(args)
    if args.workload == "c4":
        return run_c4(args)
    if args.workload == "c5":
        return run_c5(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = 0
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        dist = dist_mod
        device, _ = rank_device(local_rank)
        torch.cuda.set_device(device)
        # replicas: the process group only times (barrier, max over ranks);
        # no collective touches the solver's data
        dist.init_process_group("gloo")

    from korali_amd import _build
    from korali_amd.native import CmaesDevice

    if not os.path.exists(_build.LIB):
        _build.build()

    progress(f"C2 timed run ({args.steps} generations after {args.warmup} warm-up)")
    dev = CmaesDevice(N_VARS, LAMBDA, initial_value=np.zeros(N_VARS), initial_std=np.ones(N_VARS),
                      normal_seed=1337 + 2 * rank, uniform_seed=1338 + 2 * rank, cov_mode=args.cov, device=device)
    gen = 0
    for _ in range(args.warmup):
        gen += 1
        dev.generation(gen, "rosenbrock")
    dev.synchronize()

    def barrier():
        if dist is not None:
            dev.synchronize()
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gen += 1
        dev.generation(gen, "rosenbrock")
    dev.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-stage device times (HIP events on the solver's stream), separate pass
    dev.profile(True)
    prof_steps = min(args.steps, 20)
    STAGES = ("eigen", "eigen_tridiag", "eigen_publish_c", "eigen_c_wait", "eigen_tridiag_host", "eigen_fetch_h",
              "eigen_unpack", "eigen_chase_host", "eigen_apply", "rng_polar", "transform",
              "rng_consume", "objective", "sort", "mean_paths", "covariance", "rankmu_mfma", "sigma")
    for st in ("init",) + STAGES:
        dev.profile_read(st)
    for _ in range(prof_steps):
        gen += 1
        dev.generation(gen, "rosenbrock")
    dev.synchronize()
    stages = {}
    for st in STAGES:
        ms, n = dev.profile_read(st)
        if n:
            stages[st] = ms / n
    dev.profile(False)

    best = float(dev["Best Ever Value"][0])
    dev.close()
    eng, eng_e2e, eng_in_run, eng_e2e20 = (engine_rate(args.steps, args.warmup, args.cov) if world == 1
                                           else (None, None, None, None))
    # the other covariance mode on this rank alone (reported beside `value`)
    alt = "mfma" if args.cov == "exact" else "exact"
    progress(f"{alt} covariance rate")
    adev = CmaesDevice(N_VARS, LAMBDA, initial_value=np.zeros(N_VARS), initial_std=np.ones(N_VARS),
                       normal_seed=1337 + 2 * rank, uniform_seed=1338 + 2 * rank, cov_mode=alt, device=device)
    g2 = 0
    for _ in range(args.warmup):
        g2 += 1
        adev.generation(g2, "rosenbrock")
    adev.synchronize()
    ta = time.perf_counter()
    for _ in range(args.steps):
        g2 += 1
        adev.generation(g2, "rosenbrock")
    adev.synchronize()
    alt_rate = args.steps / (time.perf_counter() - ta)
    mfma_kernel = None
    if alt == "mfma" or args.cov == "mfma":
        pdev = adev if alt == "mfma" else None
        if pdev is not None:
            pdev.profile(True)
            pdev.profile_read("rankmu_mfma")
            for _ in range(20):
                g2 += 1
                pdev.generation(g2, "rosenbrock")
            pdev.synchronize()
            ms, n = pdev.profile_read("rankmu_mfma")
        else:
            ms, n = stages.get("rankmu_mfma", 0.0), 1
        if n:
            ms = ms / n if pdev is not None else ms
            mfma_kernel = rankmu_roofline(ms, MU, N_VARS, "c2_pmc_traffic.csv")
    adev.close()
    c4 = c4_scaling(args, world, rank, dist) if dist is not None else None
    c1 = c1_line(cpu=not args.no_cpu_baseline) if world == 1 and not args.no_c1 else None
    if rank != 0:
        dist.destroy_process_group()
        return

    gens_per_s = args.steps * world / elapsed
    # rankmu_mfma runs on the second stream, beside mean_paths
    kernels = {k: v for k, v in stages.items() if k not in HOST_STAGES + HOST_FED + ("eigen", "rankmu_mfma")}
    dominant = max(kernels, key=kernels.get)
    dom_ms = stages[dominant]
    flops = STAGE_FLOPS.get(dominant, 0.0)
    achieved = flops / (dom_ms * 1e-3) / 1e12
    traffic, traffic_raw = pmc_traffic(dominant)
    F_gen = 2 * LAMBDA * N_VARS ** 2 + 2 * MU * N_VARS ** 2 + 10 * N_VARS ** 3 + 8 * LAMBDA * N_VARS
    B_gen = 8 * (2 * LAMBDA * N_VARS + MU * N_VARS + 4 * N_VARS ** 2) + 24 * LAMBDA
    t_roof = max(F_gen / (FP64_PEAK_TFLOPS * 1e12), B_gen / (HBM_PEAK_GBS * 1e9))
    # the tridiagonalisation's dependency bound: three ordered chains of
    # n = N-1-i dependent FP64 adds per Householder step at the measured 14
    # shader cycles per add (tools/ubench_chain*.hip), 2.4 GHz
    chain_bound_ms = sum(3 * n for n in range(2, N_VARS)) * 14 / 2.4e9 * 1e3
    out = {
        "metric": "CMA-ES generations/sec + samples/sec, 128-dim Rosenbrock λ=4096, 1→8 GPUs",
        "value": gens_per_s,
        "unit": "generations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "C2: CMA-ES, 128-dim negative Rosenbrock, lambda=4096, mu=2048 Logarithmic, "
                               "x0=0, sigma0=1, seed 1337; one experiment per GPU",
                   "population": LAMBDA, "variables": N_VARS, "covariance_update": args.cov,
                   "parallelism": f"replicas{world}"},
        "samples_per_sec": gens_per_s * LAMBDA,
        "engine_generations_per_sec": eng,
        "engine_end_to_end_generations_per_sec": eng_e2e,
        "engine_in_run_generations_per_sec": eng_in_run,
        "engine_end_to_end_20_generations_per_sec": eng_e2e20,
        f"{alt}_covariance_generations_per_sec_per_gpu": alt_rate,
        "rankmu_mfma_roofline": mfma_kernel,
        "c4_sharded": c4,
        "c1": c1,
        "best_ever_value": best,
        "stage_ms": stages,
        "generation_roofline": {"T_roof_us": t_roof * 1e6, "frac": t_roof / (elapsed / args.steps * world / world)},
        "roofline": {"kernel": STAGE_KERNEL_NAME.get(dominant, dominant), "stage": dominant,
                     "bound": "mfma", "issued_on": "valu",
                     "bound_note": "the contract's compute roof, priced at the FP64 peak (MI355X FP64 vector peak == "
                                   "FP64 matrix peak, so the VALU kernel has the same roof; it issues no MFMA); "
                                   + STAGE_NOTES.get(dominant, ""),
                     "tridiag_device_chain_bound_ms": chain_bound_ms,
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_raw_fetch": traffic_raw,
                     "traffic_source": profile_file("c2_pmc_traffic.csv")[1] if traffic else None,
                     "algorithmic_flops_per_launch": flops, "avg_launch_ms": dom_ms},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


# ----------------------------------------------------------------- C3 TMCMC
C3_N, C3_P = 32, 8192


def c3_stage_flops(N, P):
    return {"draw": 2.0 * P * N * N / 2, "mean_cov": 3.0 * P * N * (N + 1) / 2 + 2.0 * P * N,
            "evaluate": 3.0 * P * N, "cholesky": N ** 3 / 3.0}


def c3_experiment(seed):
    from korali_amd.native import TmcmcDevice
    # one shared "Uniform 0" prior (U(-5,5)) for all 32 variables; seeds in
    # Korali's consumption order: distribution, then Multinomial,
    # Multivariate, Uniform generators of the solver
    return TmcmcDevice(C3_N, C3_P, prior_min=[-5.0] * C3_N, prior_max=[5.0] * C3_N, prior_seeds=[seed],
                       prior_distribution=[0] * C3_N, multinomial_seed=seed + 1, multivariate_seed=seed + 2,
                       uniform_seed=seed + 3, target_cov=1.0, covariance_scaling=0.04)


def c3_cpu_baseline(seconds_budget=30.0):
    """The whole C3 run (run to completion) on the libm
    oracle, one thread pinned to one core; the bit-exact build on its first
    3 generations beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import refcpu as R

    def rate(variant, budget, max_gens):
        L = R.lib(variant)
        L.kr_set_threads(1)
        o = R.TMCMC(C3_N, C3_P, variant=variant)
        o["Prior Minimum"] = [-5.0] * C3_N
        o["Prior Maximum"] = [5.0] * C3_N
        o.set_prior_map([0] * C3_N)
        for i, sd in enumerate([1338, 1339, 1340, 1337]):
            L.kr_rng_seed(o.rng(i).ptr, sd)
        g, t0 = 0, time.perf_counter()
        while True:
            g += 1
            o.generation(g)
            el = time.perf_counter() - t0
            # Korali terminates one generation after the exponent reaches 1
            if el > budget or g >= max_gens or o["Previous Annealing Exponent"][0] >= 1.0:
                return g, el

    with pinned_core() as core:
        g, el = rate("libm", seconds_budget, 40)
        gc, elc = rate("cr", seconds_budget / 4, 3)
    return {"value": g / el, "unit": "generations/s", "cores": 1, "kind": "port", "bit_exact_port_value": gc / elc,
            "chain_steps_per_sec": g * C3_P / el,
            "cpu": f"{cpu_model()}, 1 of {os.cpu_count()} cores (pinned to core {core})",
            "sample": f"the whole C3 run ({g} generations, N=32, P=8192, to termination), oracle/refcpu.c -O3 with "
                      f"system libm, 1 thread; bit-exact CR build: first {gc} generations"}


def run_c3(args):
    from korali_amd import _build
    if not os.path.exists(_build.LIB):
        _build.build()
    # warm-up: a throwaway run of W generations
    dev = c3_experiment(999)
    for g in range(1, args.warmup + 1):
        dev.generation(g)
        if dev["Annealing Exponent"][0] >= 1.0:
            break
    dev.synchronize()
    dev.close()
    # timed: K generations over successive complete runs (each run stops at
    # annealing exponent 1, as Korali's TMCMC termination does)
    exps = [c3_experiment(1337 + 10 * r) for r in range(max(2, args.steps // 8 + 2))]
    done, runs, r, g = 0, 0, 0, 0
    t0 = time.perf_counter()
    while done < args.steps:
        g += 1
        exps[r].generation(g)
        done += 1
        if exps[r]["Annealing Exponent"][0] >= 1.0:
            r, g, runs = r + 1, 0, runs + 1
            if r == len(exps):
                break
    exps[min(r, len(exps) - 1)].synchronize()
    elapsed = time.perf_counter() - t0
    for e in exps:
        e.close()
    # stage times on a fresh run
    dev = c3_experiment(4242)
    dev.profile(True)
    STAGES = ("cholesky", "prior_draw", "rng_polar", "draw", "evaluate", "accept", "min_search", "weights",
              "multinomial", "mean_cov", "expand")
    for g in range(1, 40):
        dev.generation(g)
        if dev["Annealing Exponent"][0] >= 1.0:
            break
    stages = {}
    for st in STAGES:
        ms, n = dev.profile_read(st)
        if n:
            stages[st] = ms / n
    search = {"generations": g, "exact_host_evaluations_per_generation": dev["Exact Search Evaluations"][0] / g,
              "of_which_deferred_to_host_worker": dev["Deferred Search Evaluations"][0] / g,
              "device_search_rounds_per_generation": dev["Device Search Rounds"][0] / g,
              "device_search_relaunches": dev["Device Search Relaunches"][0]}
    dev.close()
    flops = c3_stage_flops(C3_N, C3_P)
    # the annealing search (k_tm_nm_search): per simplex round at least two
    # candidate points, each P exponentials (~20 flops) + the weight sums'
    # double-double accumulation (~6 flops) per chain
    flops["min_search"] = search["device_search_rounds_per_generation"] * 2 * C3_P * 26.0
    # the dominant stage by time among every stage (GPU time; the annealing
    # search is the largest since the device search replaced the host loop)
    kernels = {k: v for k, v in stages.items() if k in flops}
    dominant = max(stages, key=stages.get)
    if dominant not in flops:
        dominant = max(kernels, key=kernels.get)
    achieved = flops[dominant] / (stages[dominant] * 1e-3) / 1e12
    c3_traffic, _ = pmc_traffic(dominant, "c3_pmc_traffic.csv")
    out = {
        "metric": "TMCMC generations/sec, 32-dim Gaussian posterior, P=8192 chains",
        "value": done / elapsed, "unit": "generations/s", "n_gpus": 1, "steps": done, "warmup": args.warmup,
        "ms_per_step": elapsed / done * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C3: TMCMC, 32 variables with one shared U(-5,5) prior, loglik -0.5|x|^2, "
                               "P=8192, Max Chain Length 1, Target CoV 1.0, Covariance Scaling 0.04; "
                               "successive runs to annealing exponent 1", "complete_runs": runs},
        "chain_steps_per_sec": done * C3_P / elapsed,
        "stage_ms": stages,
        "annealing_search": search,
        "roofline": {"kernel": {"min_search": "kg::k_tm_nm_sym"}.get(dominant, dominant), "stage": dominant,
                     "bound": "mfma",
                     "bound_note": "FP64 compute roof (MI355X FP64 vector peak == FP64 matrix peak); the stage is a "
                                   "chain of dependent rounds (GSL nmsimplex order, one cross-XCD hand-off per "
                                   "round), far below it by construction",
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "traffic": c3_traffic,
                     "traffic_source": profile_file("c3_pmc_traffic.csv")[1] if c3_traffic else None,
                     "algorithmic_flops_per_launch": flops[dominant], "avg_launch_ms": stages[dominant]},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = c3_cpu_baseline()
    print(json.dumps(out), flush=True)


# ----------------------------------------------------------------- C4 sharded
C4_N, C4_L = 512, 65536


def c4_cpu_baseline():
    """Bounded CPU sample for C4: the libm oracle, one pinned thread, N = 512
    Ackley at lambda = 8192 (one rank's shard at 8 GPUs; a full C4
    generation takes minutes on one core): 1 warm-up + 1 timed generation,
    reported as samples/s (comparable with the device's samples_per_sec)."""
    lam = 8192
    with pinned_core() as core:
        gens, el = _cmaes_oracle_rate("libm", 1, 1, 0.0, N=C4_N, lam=lam, objective="ackley", x0=2.0)
    return {"value": gens * lam / el, "unit": "samples/s", "cores": 1, "kind": "port",
            "generations_per_sec_at_sample": gens / el,
            "cpu": f"{cpu_model()}, 1 of {os.cpu_count()} cores (pinned to core {core})",
            "sample": f"{gens} generation(s) of N=512 Ackley at lambda=8192, mu=4096 (one rank's shard of C4) after "
                      f"1 warm-up, oracle/refcpu.c -O3 with system libm, 1 thread"}


def c4_experiment(generations, cov="MFMA"):
    import korali
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Kernel"] = "Negative Ackley"
    for i in range(C4_N):
        e["Variables"][i]["Name"] = "X" + str(i)
        e["Variables"][i]["Initial Value"] = 2.0
        e["Variables"][i]["Initial Standard Deviation"] = 1.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = C4_L
    e["Solver"]["Covariance Update"] = cov
    e["Solver"]["Termination Criteria"]["Max Generations"] = generations
    e["Random Seed"] = 1337
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    return e


def run_c4_engine(args, world, rank):
    """C4 through korali.Engine with the Distributed conduit (the C++ engine
    shards the population; RCCL all-gather of fitnesses and sum all-reduce of
    the mean / rank-mu partials on the handle's stream; Host transport when
    KORALI_AMD_C4_TRANSPORT=Host).  One run of warmup + steps generations;
    the engine records when each generation completed (its termination check
    returned, korali._generation_completion_times), and the timed region
    is the last `steps` generations of the slowest rank."""
    import korali
    import socket
    import torch
    import torch.distributed as tdist
    if "MASTER_PORT" not in os.environ:  # (one rank started without torch.distributed.run)
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world))
    tdist.init_process_group("gloo")  # (timing exchange only; the engine brings its own bootstrap + RCCL)
    os.environ.setdefault("KORALI_AMD_EXCHANGE_PROFILE", "1")
    transport = os.environ.get("KORALI_AMD_C4_TRANSPORT",
                               "RCCL" if rank_device(int(os.environ.get("LOCAL_RANK", "0")))[1] >= world else "Host")
    w = max(1, args.warmup)
    total = w + args.steps
    k = korali.Engine()
    k["Conduit"]["Type"] = "Distributed"
    k["Conduit"]["Transport"] = transport
    e = c4_experiment(total, "Exact" if args.cov == "exact" else "MFMA")
    tdist.barrier()
    k.run(e)
    marks = korali._generation_completion_times(e)
    gens = int(e["Current Generation"])
    if gens != total or len(marks) != total + 1:
        raise RuntimeError(f"engine ran {gens} generations ({len(marks)} marks), expected {total}")
    t = torch.tensor([marks[total] - marks[w]], dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    elapsed = float(t.item())
    best = float(e["Solver"]["Best Ever Value"])
    exch = exchange_ms(e, tdist)
    if rank == 0:
        print(json.dumps({
            "metric": "CMA-ES generations/sec, 512-dim Ackley lambda=65536 (C4)", "value": args.steps / elapsed,
            "unit": "generations/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "C4: CMA-ES, 512-dim negative Ackley, lambda=65536, mu=32768 Logarithmic, x0=2, "
                                   "sigma0=1, seed 1337; korali.Engine, Distributed conduit (" + transport + ")",
                       "parallelism": f"population-shard{world}", "covariance_update": args.cov},
            "samples_per_sec": args.steps / elapsed * C4_L, "best_ever_value": best,
            "timing": "generations %d-%d of one %d-generation engine run (engine completion marks), slowest rank"
                      % (w + 1, total, total),
            "exchange_ms_per_generation": exch or None,
            "cpu_baseline": None if args.no_cpu_baseline else c4_cpu_baseline()}), flush=True)
    tdist.destroy_process_group()


def c4_roofline(stages):
    """The dominant device kernel of a C4 generation (HIP-event stage times;
    the host chase, the eigen aggregate and the second-stream rank-mu MFMA
    excluded) against the FP64 peak, its HBM bytes per launch from the
    committed C4 PMC passes."""
    kern = {k: v for k, v in stages.items() if k not in HOST_STAGES + HOST_FED + ("eigen", "rankmu_mfma")}
    if not kern:
        return None
    dom = max(kern, key=kern.get)
    flops = stage_flops(C4_N, C4_L, C4_L // 2).get(dom, 0.0)
    ms = stages[dom]
    achieved = flops / (ms * 1e-3) / 1e12
    traffic, _ = pmc_traffic(dom, "c4_pmc_traffic.csv")
    names = {"eigen_tridiag": "kg::k_tridiag_mw2", "covariance": "kg::k_adaptC_lane", "eigen_unpack": "kg::k_unpack_mw",
             "transform": "kg::k_prescale_t + kg::k_transform_sc"}
    return {"kernel": names.get(dom, dom), "stage": dom, "bound": "mfma",
            "bound_note": "FP64 compute roof (vector = matrix FP64 peak on MI355X); " + STAGE_NOTES.get(dom, ""),
            "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
            "traffic": traffic, "traffic_source": profile_file("c4_pmc_traffic.csv")[1] if traffic else None,
            "algorithmic_flops_per_launch": flops, "avg_launch_ms": ms}


def run_c4(args):
    """BASELINE.json configs[3]: CMA-ES, 512-dim negative Ackley
    (model.py:37-62), λ = 65536, μ = 32768, x0 = 2, σ0 = 1, seed 1337.  With
    N > 1 ranks (or KORALI_AMD_C4_ENGINE=1) it runs through korali.Engine's
    Distributed conduit (run_c4_engine); one rank times the C-ABI loop
    (KORALI_AMD_C4_ENGINE=0 with N > 1: the Python sharded driver,
    korali_amd/sharded.py).  Total work is fixed, so scaling is strong."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    eng = os.environ.get("KORALI_AMD_C4_ENGINE", "1" if world > 1 else "0") == "1"
    if eng:
        return run_c4_engine(args, world, rank)
    kw = dict(initial_value=np.full(C4_N, 2.0), initial_std=np.ones(C4_N), normal_seed=1337, uniform_seed=1338)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        from korali_amd.sharded import ShardedCmaes
        solver = ShardedCmaes(C4_N, C4_L, dist, device=local_rank, transport="device", cov_mode=args.cov, **kw)
        dev = solver.dev
    else:
        from korali_amd.native import CmaesDevice
        dev = CmaesDevice(C4_N, C4_L, cov_mode=args.cov, **kw)
        solver = dev

    def step(g):
        solver.generation(g, "ackley")

    gen = 0
    for _ in range(args.warmup):
        gen += 1
        step(gen)
    dev.synchronize()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gen += 1
        step(gen)
    dev.synchronize()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    dev.profile(True)
    STAGES = ("eigen", "eigen_tridiag", "eigen_publish_c", "eigen_c_wait", "eigen_tridiag_host", "eigen_fetch_h",
              "eigen_unpack", "eigen_chase_host", "eigen_apply", "rng_polar", "transform",
              "objective", "sort", "mean_paths", "covariance", "rankmu_mfma", "sigma")
    for st in ("init",) + STAGES:
        dev.profile_read(st)
    for _ in range(2):
        gen += 1
        step(gen)
    dev.synchronize()
    stages = {}
    for st in STAGES:
        ms, n = dev.profile_read(st)
        if n:
            stages[st] = ms / n
    dev.profile(False)
    best = float(dev["Best Ever Value"][0])
    if rank == 0:
        print(json.dumps({
            "metric": "CMA-ES generations/sec, 512-dim Ackley lambda=65536 (C4)", "value": args.steps / elapsed,
            "unit": "generations/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "C4: CMA-ES, 512-dim negative Ackley, lambda=65536, mu=32768 Logarithmic, x0=2, "
                                   "sigma0=1, seed 1337", "parallelism": f"population-shard{world}",
                       "covariance_update": args.cov},
            "samples_per_sec": args.steps / elapsed * C4_L, "best_ever_value": best,
            "stage_ms_rank0": stages,
            "roofline": c4_roofline(stages),
            "rankmu_mfma_roofline": rankmu_roofline(stages["rankmu_mfma"], C4_L // 2, C4_N, "c4_pmc_traffic.csv")
            if "rankmu_mfma" in stages else None,
            "cpu_baseline": None if args.no_cpu_baseline else c4_cpu_baseline()}), flush=True)
    solver.close()  # (device memory and the chase thread released before the runtime's teardown)
    if dist is not None:
        dist.destroy_process_group()


# --------------------------------------------------------------- C5 VRACER
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 matrix (= FP32 vector) peak, MI355X_MICROARCH.md
C5 = dict(environments=4096, hidden_size=256, hidden_layers=2, mini_batch_size=256, replay_maximum_size=262144,
          replay_start_size=131072, experiences_between_policy_updates=1.0, max_episode_steps=500,
          environment_count=3, discount_factor=0.99, learning_rate=1e-4, initial_exploration_noise=1.0)


def c5_update_flops(S=4, H=256, L=2, A=1, B=256):
    """Algorithmic FLOPs of one VRACER::trainPolicy: the critic/policy forward on
    2B rows (mini-batch + truncated states) and the backward on B rows."""
    O = 1 + 2 * A
    fwd = 2 * (2 * B) * (S * H + (L - 1) * H * H + H * O)
    bwd = 2 * B * (H * O) * 2 + (L - 1) * 2 * (2 * B * H * H) + 2 * B * S * H
    return fwd + bwd


def c5_cpu_baseline(seconds_budget=15.0):
    """The NumPy restatement (oracle/vracer_ref.py) on one core: environment
    steps of the same 4096 CartPole rollouts and policy updates of the same
    network, timed separately on bounded samples."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vracer_ref as V
    try:
        from threadpoolctl import threadpool_limits
        limit = threadpool_limits(1)
    except Exception:  # noqa: BLE001
        limit = None
    S, A, H, L, E = 4, 1, C5["hidden_size"], C5["hidden_layers"], C5["environments"]
    n = V.hyperparameter_count(S, H, L, A)
    th = V.initial_hyperparameters(S, H, L, A, np.random.default_rng(0).uniform(-1, 1, n))
    ag = V.Agent(S, A, H, L, th, max_size=C5["replay_maximum_size"], discount=C5["discount_factor"],
                 learning_rate=C5["learning_rate"])
    ro = V.Rollouts(ag, E, max_steps=C5["max_episode_steps"])
    t0, steps, exps = time.perf_counter(), 0, 0
    while time.perf_counter() - t0 < seconds_budget / 2 or steps < 2:
        new, _ = ro.step(V.action_noise(1, steps, E, A))
        steps, exps = steps + 1, exps + new
    env_s = (time.perf_counter() - t0) / steps
    # policy updates on a replay memory of synthetic 50-step episodes (the
    # update cost does not depend on the values)
    rng = np.random.default_rng(2)
    while ag.size() < 8192:
        T = 50
        ag.process_episode(int(rng.integers(3)), rng.standard_normal((T, S)).astype(np.float32),
                           rng.standard_normal((T, A)).astype(np.float32), np.ones(T, np.float32),
                           np.abs(rng.standard_normal((T, 2 * A))).astype(np.float32) + 0.5,
                           rng.standard_normal(T).astype(np.float32), V.TERMINAL)
    t0, ups = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds_budget / 2 or ups < 3:
        ag.train_policy(ag.minibatch_ids(V.minibatch_uniforms(1, ups * C5["mini_batch_size"], C5["mini_batch_size"])))
        ups += 1
    upd_s = (time.perf_counter() - t0) / ups
    if limit is not None:
        limit.unregister() if hasattr(limit, "unregister") else None
    # steady state of the benchmark: one environment step of E actions plus
    # E / Experiences Between Policy Updates updates
    per_step = env_s + E / C5["experiences_between_policy_updates"] * upd_s
    return {"value": E / per_step, "unit": "experiences/s", "cores": 1, "kind": "port",
            "updates_per_sec": 1.0 / upd_s, "environment_step_ms": env_s * 1e3, "update_ms": upd_s * 1e3,
            "cpu": cpu_model(),
            "sample": f"oracle/vracer_ref.py (NumPy, 1 BLAS thread): {steps} environment steps of {E} CartPole "
                      f"rollouts and {ups} policy updates (mini-batch {C5['mini_batch_size']}, 2x{H} tanh); value = "
                      f"E / (env step + E/EBPU updates)"}


def run_c5(args):
    """BASELINE.json configs[4]: VRACER agent (Normal policy), 4096 concurrent
    CartPole environments (examples/learning/reinforcement/cartpole), critic/
    policy 2 x 256 tanh, mini-batch 256, Experiences Between Policy Updates 1
    (the cartpole example's), replay 262144 / start 131072.  A step is one
    iteration of Agent::trainingGeneration's loop: every environment takes an
    action, finished episodes enter the replay memory, then the policy
    updates the experience count allows (kg_vracer_training_step)."""
    from korali_amd.vracer import VracerDevice
    d = VracerDevice(seed=1337, **C5)
    # warm-up: fill the replay memory to its start size, then W steps
    filled = 0
    while d.scalar("experience_count") < C5["replay_start_size"]:
        d.training_step()
        filled += 1
    for _ in range(args.warmup):
        d.training_step()
    d.synchronize()
    exps, ups = 0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n, u = d.training_step()
        exps, ups = exps + n, ups + u
    d.synchronize()
    elapsed = time.perf_counter() - t0
    # stage timers on a few more steps
    m0 = d.get("meta_phase_ticks").astype(np.float64)
    u0 = d.scalar("policy_update_count")
    d.profile(True)
    for _ in range(3):
        d.training_step()
    d.synchronize()
    nu = max(1.0, d.scalar("policy_update_count") - u0)
    mt = (d.get("meta_phase_ticks").astype(np.float64) - m0) / nu
    meta_us = (mt[:3] * 0.01).tolist()  # 100 MHz ticks
    walks = {"longest_walk_entries": mt[3], "walked_entries": mt[4], "walks": mt[5],  # per update
             "us_walk_setup": mt[6] * 0.01, "us_staging_loads": mt[7] * 0.01, "us_walks": mt[8] * 0.01}
    stages = {}
    for st in ("environment_step", "update", "gemm_rollout", "gemm_update"):
        ms, cnt = d.profile_read(st)
        if cnt:
            stages[st] = ms / cnt
    d.profile(False)
    E, H = C5["environments"], C5["hidden_size"]
    gemm_flops = 2.0 * E * H * H * (C5["hidden_layers"] - 1)  # hidden-layer products of one rollout forward
    gemm_ms = stages.get("gemm_rollout")
    achieved = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms else None
    upd_flops = c5_update_flops(H=H, L=C5["hidden_layers"], B=C5["mini_batch_size"])
    upd_ms = stages.get("update")
    finished = d.get("finished_rewards")
    # HBM bytes per rollout-GEMM launch from the committed PMC passes (tools/pmc_c5.py)
    traffic = None
    tf = profile_file("c5_pmc_traffic.csv")[0]
    if os.path.exists(tf):
        import csv
        rows = list(csv.DictReader(open(tf)))
        if rows:
            traffic = (float(rows[0]["fetch_KB_x2"]) + float(rows[0]["write_KB"])) * 1024.0
    # HBM bytes of one policy update: every update kernel's FETCH_SIZE x2 +
    # WRITE_SIZE per dispatch (the kernels dispatched once per update) from the
    # committed PMC passes over all update kernels (tools/pmc_c5_update.py)
    upd_traffic, upd_traffic_src = None, None
    uf, upd_traffic_src = profile_file("c5_pmc_update_traffic.csv")
    if upd_traffic_src:
        import csv
        rows = list(csv.DictReader(open(uf)))
        top = max(int(r["dispatches"]) for r in rows)
        upd_traffic = sum((float(r["fetch_KB_x2"]) + float(r["write_KB"])) * 1024.0 for r in rows
                          if int(r["dispatches"]) * 2 >= top)
    out = {
        "metric": "VRACER experiences/sec, 4096 concurrent CartPole rollouts, 2x256 policy (C5)",
        "value": exps / elapsed, "unit": "experiences/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "C5: VRACER Normal policy, CartPole env (examples/learning/reinforcement/cartpole, "
                               "scipy dopri5 restated), 4096 concurrent environments, 2x256 tanh, mini-batch 256, EBPU 1, "
                               "replay 262144 (start 131072)", "fill_steps": filled},
        "policy_updates_per_sec": ups / elapsed, "updates": ups, "experiences": exps,
        "stage_ms": stages,
        "metadata_kernel_phases_us": {"setup_and_importance_weights": meta_us[0], "retrace_chains": meta_us[1],
                                      "loss_gradient_and_metadata": meta_us[2]},
        "retrace_walks_per_update": walks,
        "update_roofline": {"flops_per_update": upd_flops, "avg_update_ms": upd_ms,
                            "achieved_tflops": upd_flops / (upd_ms * 1e-3) / 1e12 if upd_ms else None,
                            "peak": FP32_PEAK_TFLOPS,
                            "frac": upd_flops / (upd_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS if upd_ms else None},
        # the metric's dominant work: one policy update (EBPU 1: one per
        # experience; the rollout GEMM below it is 1/4096 of an experience)
        "roofline": {"kernel": "VRACER policy update (mini-batch, forward, metadata, backward, Adam: one "
                               "trainPolicy step, its kernels back to back on the handle's stream)",
                     "bound": "mfma", "achieved": upd_flops / (upd_ms * 1e-3) / 1e12 if upd_ms else None,
                     "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": upd_flops / (upd_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS if upd_ms else None,
                     "traffic": upd_traffic, "traffic_source": upd_traffic_src,
                     "algorithmic_flops_per_launch": upd_flops, "avg_launch_ms": upd_ms},
        "rollout_gemm_roofline": {"kernel": "kg::vr::k_vr_gemm<1> (rollout forward, hidden layer)", "bound": "mfma",
                                  "achieved": achieved, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": achieved / FP32_PEAK_TFLOPS if achieved else None, "traffic": traffic,
                                  "traffic_source": profile_file("c5_pmc_traffic.csv")[1] if traffic else None,
                                  "algorithmic_flops_per_launch": gemm_flops, "avg_launch_ms": gemm_ms},
        "mean_recent_episode_reward": float(np.mean(finished[finished != 0])) if np.any(finished != 0) else None,
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = c5_cpu_baseline()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
