"""GPU parity: the HIP CMA-ES path (through the C-ABI) against the oracle and
the reference's golden generation files.

Bar: bit-exact (np.array_equal) for populations, sorting indices, means,
covariances and sigma in EXACT covariance mode; the MFMA covariance mode is
checked to 1e-12 relative on the covariance (north star: 1e-6) with the
sorting index of the next generation still exact.
"""
import numpy as np
import pytest

import refcpu as R
from golden_util import CMAES_STATE_SCALARS, CMAES_STATE_VECTORS, cmaes_variables, load_cmaes, population

pytestmark = pytest.mark.gpu

CM = load_cmaes()
N, LAM, MU = 10, 32, 16


def by_gen(g):
    for x in CM:
        if x["Current Generation"] == g:
            return x
    raise KeyError(g)


def device_solver(N, lam, **kw):
    from korali_amd.native import CmaesDevice
    return CmaesDevice(N, lam, **kw)


def fixture_device(k, cov_mode="exact"):
    st = by_gen(k)
    v = cmaes_variables(st)
    dev = device_solver(N, LAM, mu=MU, lower_bound=v["Lower Bound"], upper_bound=v["Upper Bound"],
                        initial_value=v["Initial Value"], initial_std=v["Initial Standard Deviation"],
                        max_infeasible_resamplings=10000, cov_mode=cov_mode)
    s = st["Solver"]
    for key in CMAES_STATE_VECTORS:
        dev[key] = s[key]
    for key in CMAES_STATE_SCALARS:
        dev[key] = [s[key]]
    dev.set_rng(0, bytes.fromhex(s["Normal Generator"]["Range"]))
    dev.set_rng(1, bytes.fromhex(s["Uniform Generator"]["Range"]))
    return dev


@pytest.mark.parametrize("k", [1, 2, 19, 49, 99])
def test_teacher_forced_generation_bit_exact(k):
    dev = fixture_device(k)
    nxt = by_gen(k + 1)["Solver"]
    dev.sample()
    dev.synchronize()
    assert np.array_equal(dev["Covariance Eigenvector Matrix"], np.array(nxt["Covariance Eigenvector Matrix"]))
    assert np.array_equal(dev["Axis Lengths"], np.array(nxt["Axis Lengths"]))
    assert np.array_equal(dev["Sample Population"], population(by_gen(k + 1)).reshape(-1))
    dev.set_fitness(np.array(nxt["Value Vector"]))
    dev.update(k + 1)
    dev.synchronize()
    assert list(dev.sorting_index()) == nxt["Sorting Index"]
    for key in ("Current Mean", "Previous Mean", "Evolution Path", "Conjugate Evolution Path", "Covariance Matrix"):
        assert np.array_equal(dev[key], np.array(nxt[key])), key
    for key in ("Sigma", "Conjugate Evolution Path L2 Norm", "Best Ever Value", "Current Best Value",
                "Maximum Diagonal Covariance Matrix Element", "Minimum Diagonal Covariance Matrix Element",
                "Current Min Standard Deviation", "Current Max Standard Deviation", "Infeasible Sample Count"):
        assert dev[key][0] == nxt[key], key
    # the exported GSL state continues the reference stream exactly
    if k + 1 in (2, 3, 20, 50, 100):
        assert dev.get_rng(0).hex().upper() == nxt["Normal Generator"]["Range"]


def test_seeded_100_generations_match_reference_fixture():
    """Experiment seed 790510 → Normal 790510 / Uniform 790511; builtin
    negative-sphere objective == the fixture's model; 100 generations."""
    v = cmaes_variables(by_gen(0))
    dev = device_solver(N, LAM, mu=MU, lower_bound=v["Lower Bound"], upper_bound=v["Upper Bound"],
                        initial_value=v["Initial Value"], initial_std=v["Initial Standard Deviation"],
                        max_infeasible_resamplings=10000, normal_seed=790510, uniform_seed=790511)
    for g in range(1, 101):
        dev.generation(g, "negative sphere")
        if g in (1, 2, 13, 50, 100):
            dev.synchronize()
            s = by_gen(g)["Solver"]
            assert list(dev.sorting_index()) == s["Sorting Index"], g
            assert np.array_equal(dev["Sample Population"], population(by_gen(g)).reshape(-1)), g
            assert np.array_equal(dev["Covariance Matrix"], np.array(s["Covariance Matrix"])), g
            assert dev["Sigma"][0] == s["Sigma"], g
    dev.synchronize()
    assert dev.get_rng(0).hex().upper() == by_gen(100)["Solver"]["Normal Generator"]["Range"]


def oracle_and_device(Nv, lam, objective, gens, cov_mode="exact", seed=1337, x0=0.0, s0=1.0, eigen_chase="host"):
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"] = np.full(Nv, x0)
    o["Initial Standard Deviation"] = np.full(Nv, s0)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=np.full(Nv, x0), initial_std=np.full(Nv, s0), normal_seed=seed,
                        uniform_seed=seed + 1, cov_mode=cov_mode, eigen_chase=eigen_chase)
    return o, dev


@pytest.mark.parametrize("Nv,lam,objective,gens,chase", [(8, 16, "rosenbrock", 30, "host"),
                                                         (32, 256, "ackley", 8, "host"),
                                                         (128, 4096, "rosenbrock", 3, "host"),
                                                         (128, 4096, "rosenbrock", 2, "device"),
                                                         (200, 512, "rosenbrock", 2, "host"),
                                                         (512, 1024, "rosenbrock", 2, "host")])
def test_seeded_run_matches_oracle_bit_exact(Nv, lam, objective, gens, chase):
    """N=200 and N=512 exercise the multi-workgroup eigensolver variant
    (rows / columns spread over workgroups, in-launch hand-offs)."""
    o, dev = oracle_and_device(Nv, lam, objective, gens, eigen_chase=chase)
    for g in range(1, gens + 1):
        o.generation(g, objective)
        dev.generation(g, objective)
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        # Ackley: correctly-rounded cos on both sides (kg_common.hpp cos_cr,
        # refcpu.c kr_cos_cr), so every objective value is bit-exact too
        assert np.array_equal(dev["Value Vector"], o["Value Vector"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Covariance Matrix", "Covariance Eigenvector Matrix", "Axis Lengths"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        assert dev["Sigma"][0] == o["Sigma"][0], g
    assert dev.get_rng(0) == o.rng(0).get_bytes()


def test_mfma_covariance_mode_within_tolerance():
    """Rank-μ sum on v_mfma_f64_16x16x4f64: one generation from identical
    state, covariance within 1e-12 relative of the sequential order; the
    population and sorting index of the generation are unaffected."""
    Nv, lam = 128, 4096
    o, dev = oracle_and_device(Nv, lam, "rosenbrock", 1, cov_mode="mfma")
    for g in (1, 2):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        C_o, C_d = o["Covariance Matrix"], dev["Covariance Matrix"]
        rel = np.max(np.abs(C_d - C_o)) / np.max(np.abs(C_o))
        assert rel < 1e-12, (g, rel)
        if g == 1:
            # re-sync the device covariance to the oracle so gen 2 starts equal
            dev["Covariance Matrix"] = C_o


def test_large_population_sort_matches_numpy():
    """λ = 65536 (> one LDS chunk): multi-pass bitonic network vs a stable
    descending argsort."""
    from korali_amd.native import CmaesDevice
    lam = 65536
    dev = CmaesDevice(4, lam, initial_value=np.zeros(4), initial_std=np.ones(4), normal_seed=5)
    dev.initialize()
    rng = np.random.default_rng(0)
    F = rng.standard_normal(lam)
    F[100:140] = F[7]  # ties: resolved by index
    dev.set_fitness(F)
    dev.update(1)
    dev.synchronize()
    ref = np.lexsort((np.arange(lam), -F))
    assert np.array_equal(dev.sorting_index(), ref)


@pytest.mark.parametrize("parts", ["1", "8", "13"])
def test_chunked_mt_producer_wraps_the_seed_slots(monkeypatch, parts):
    """Past 3K chunks (K = 256 chunks per launch, seed windows in 3K slots
    reused in turn; 45 generations of N = 64, lambda = 4096 draw ~30 M words
    in 2^15-word chunks): the chunk jumps split over 1, 8 or 13 workgroups
    keep the population and the exported generator state bit-exact."""
    monkeypatch.setenv("KORALI_AMD_MT_PARALLEL_MIN", "0")
    monkeypatch.setenv("KORALI_AMD_MT_CHUNK_LOG2", "15")
    monkeypatch.setenv("KORALI_AMD_MT_CHUNK_PARTS", parts)
    o, dev = oracle_and_device(64, 4096, "rosenbrock", 45)
    for g in range(1, 46):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        if g % 5 == 0 or g == 45:
            dev.synchronize()
            assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
    assert np.array_equal(dev["Current Mean"], o["Current Mean"])
    assert dev.get_rng(0) == o.rng(0).get_bytes()


@pytest.mark.parametrize("log2w", [15, 17])
def test_chunked_mt_producer_bit_exact(monkeypatch, log2w):
    """The multi-workgroup mt19937 producer (chunks of 2^log2w words seeded
    by GF(2) jumps, kg_mtjump.hip) forced on a C2-sized stream: populations,
    selection, update and the exported generator state stay bit-exact."""
    monkeypatch.setenv("KORALI_AMD_MT_PARALLEL_MIN", "0")
    monkeypatch.setenv("KORALI_AMD_MT_CHUNK_LOG2", str(log2w))
    o, dev = oracle_and_device(128, 4096, "rosenbrock", 3)
    for g in (1, 2, 3):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        assert np.array_equal(dev["Current Mean"], o["Current Mean"]), g
    assert dev.get_rng(0) == o.rng(0).get_bytes()
    assert dev.get_rng(1) == o.rng(1).get_bytes()


@pytest.mark.parametrize("Nv,lam", [(16, 64), (128, 4096)])
def test_multi_workgroup_eigen_forced_bit_exact(monkeypatch, Nv, lam):
    """The multi-workgroup tridiagonalisation / unpack (in-launch hand-offs,
    redundant pivot rows) forced below its default threshold: bit-exact."""
    monkeypatch.setenv("KORALI_AMD_EIGEN_MW_MIN", "0")
    o, dev = oracle_and_device(Nv, lam, "rosenbrock", 4)
    for g in (1, 2, 3, 4):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        for key in ("Covariance Eigenvector Matrix", "Axis Lengths", "Current Mean", "Covariance Matrix"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g


@pytest.mark.parametrize("Nv,lam", [(16, 64), (128, 4096)])
def test_unpack_streamed_reflector_rows_bit_exact(monkeypatch, Nv, lam):
    """The multi-workgroup unpack with reflector rows streamed step by step
    (the N > ~150 form) forced where the all-rows-in-LDS form is the default."""
    monkeypatch.setenv("KORALI_AMD_EIGEN_MW_MIN", "0")
    monkeypatch.setenv("KORALI_AMD_UNPACK_ALLH", "0")
    o, dev = oracle_and_device(Nv, lam, "rosenbrock", 4)
    for g in (1, 2, 3):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        for key in ("Covariance Eigenvector Matrix", "Axis Lengths", "Current Mean", "Covariance Matrix"):
            assert np.array_equal(dev[key], o[key]), (g, key)


@pytest.mark.parametrize("Nv,lam,kind", [(3, 8, "sq"), (5, 16, "sq"), (16, 64, "sq"), (67, 256, "sq"),
                                         (128, 4096, "sq"), (3, 8, "sq-dpp"), (5, 16, "sq-dpp"),
                                         (16, 64, "sq-dpp"), (67, 256, "sq-dpp"), (100, 300, "sq-dpp"),
                                         (128, 4096, "sq-dpp"), (16, 64, "1wg2"), (128, 4096, "1wg2"),
                                         (40, 128, "mw2"), (100, 512, "mw2"), (129, 256, "mw2"),
                                         (40, 128, "mw2-dpp"), (129, 256, "mw2-dpp"), (200, 400, "mw2-dpp"),
                                         (16, 64, "1wg"), (64, 256, "1wg"), (128, 4096, "1wg"), (100, 512, "mw"),
                                         (40, 128, "lds")])
def test_tridiagonalisation_kernels_bit_exact(monkeypatch, Nv, lam, kind):
    """Each tridiagonalisation kernel (one workgroup with the matrix in LDS,
    the multi-workgroup one, the older LDS one) forced: bit-exact B, D and
    the generation's outputs against the oracle."""
    monkeypatch.setenv("KORALI_AMD_TRIDIAG", kind.split("-")[0])
    monkeypatch.setenv("KORALI_AMD_SQ_DPP", "1" if kind.endswith("-dpp") else "0")
    o, dev = oracle_and_device(Nv, lam, "rosenbrock", 4)
    for g in (1, 2, 3, 4):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        for key in ("Covariance Eigenvector Matrix", "Axis Lengths", "Current Mean", "Covariance Matrix"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g


@pytest.mark.parametrize("Nv,lam,mirrored,bound", [(3, 8, False, None), (10, 64, False, None), (13, 100, True, None),
                                                  (128, 4096, False, None), (67, 300, False, 1.0),
                                                  (10, 64, True, 0.5)])
@pytest.mark.parametrize("width", ["8", "82"])
def test_scalar_operand_transform_bit_exact(monkeypatch, Nv, lam, mirrored, bound, width):
    """k_transform_sc (B in scalar registers, D o z prescaled k-major) forced:
    populations, selections and the updated state bit for bit against the
    oracle, for N not a multiple of the 4-k groups or of the 32-column
    workgroup, row counts not a multiple of 64, Mirrored Sampling and the
    bounded redraw rounds (k_select over the transformed reserve)."""
    monkeypatch.setenv("KORALI_AMD_TRANSFORM_SC", width)  # 8 columns per wave, 1 or 2 (82) rows per lane
    seed = 99
    x0 = np.full(Nv, 0.5 if bound == 0.5 else 0.0)
    # sigma0: bound 0.5 starts ON the bound (~10^3 draws per sample, the
    # redraw rounds); bound 1.0 at N = 67 leaves ~25% of the draws infeasible
    s0 = {None: 1.0, 0.5: 0.3, 1.0: 0.35}[bound]
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"], o["Initial Standard Deviation"] = x0, np.full(Nv, s0)
    kw = {}
    if bound is not None:
        o["Lower Bound"], o["Upper Bound"] = np.full(Nv, -bound), np.full(Nv, bound)
        kw = dict(lower_bound=np.full(Nv, -bound), upper_bound=np.full(Nv, bound))
    if mirrored:
        o.option("Mirrored Sampling", 1)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=x0, initial_std=np.full(Nv, s0),
                        mirrored=mirrored, normal_seed=seed, uniform_seed=seed + 1, **kw)
    for g in range(1, 5):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Covariance Matrix", "Axis Lengths"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        assert dev["Infeasible Sample Count"][0] == o["Infeasible Sample Count"][0], g
    dev.close()


@pytest.mark.parametrize("Nv,lam,bound,gens,diag", [(8, 16, None, 20, False), (8, 16, 1.5, 20, False),
                                                    (32, 256, 3.0, 6, False), (16, 64, 2.0, 10, True)])
def test_mirrored_sampling_matches_oracle_bit_exact(Nv, lam, bound, gens, diag):
    """Mirrored Sampling (CMAES.cpp.base:461-491): rows 2j / 2j+1 from z_j and
    -z_j, a pair redrawn only when both of its samples are infeasible (each
    infeasible draw counted); unbounded and bounded, full and diagonal
    covariance, against the oracle bit for bit."""
    seed = 77
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"] = np.zeros(Nv)
    o["Initial Standard Deviation"] = np.ones(Nv)
    o.option("Mirrored Sampling", 1)
    if diag:
        o.option("Diagonal Covariance", 1)
    kw = {}
    if bound is not None:
        o["Lower Bound"] = np.full(Nv, -bound)
        o["Upper Bound"] = np.full(Nv, bound)
        kw = dict(lower_bound=np.full(Nv, -bound), upper_bound=np.full(Nv, bound))
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=np.zeros(Nv), initial_std=np.ones(Nv), normal_seed=seed,
                        uniform_seed=seed + 1, mirrored=True, diagonal=diag, **kw)
    for g in range(1, gens + 1):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        X = dev["Sample Population"].reshape(lam, Nv)
        assert np.array_equal(X, o["Sample Population"].reshape(lam, Nv)), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Covariance Matrix", "Axis Lengths"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        assert dev["Sigma"][0] == o["Sigma"][0], g
        assert dev["Infeasible Sample Count"][0] == o["Infeasible Sample Count"][0], g
    if bound is not None:
        assert o["Infeasible Sample Count"][0] > 0  # the pair resampling ran
    assert dev.get_rng(0) == o.rng(0).get_bytes()
    dev.close()


def test_mfma_covariance_mode_trajectory():
    """The MFMA rank-mu mode over a whole trajectory (no re-sync): mean and
    covariance stay within 1e-6 relative of the bit-exact trajectory (the
    north star's tolerance) while the selection agrees, and the generation at
    which the first selection index differs is reported, not hidden."""
    Nv, lam, gens = 32, 256, 40
    seed = 9
    ex = device_solver(Nv, lam, initial_value=np.zeros(Nv), initial_std=np.ones(Nv), normal_seed=seed,
                       uniform_seed=seed + 1, cov_mode="exact")
    mf = device_solver(Nv, lam, initial_value=np.zeros(Nv), initial_std=np.ones(Nv), normal_seed=seed,
                       uniform_seed=seed + 1, cov_mode="mfma")
    first_split, worst = None, 0.0
    for g in range(1, gens + 1):
        ex.generation(g, "rosenbrock")
        mf.generation(g, "rosenbrock")
        ex.synchronize()
        mf.synchronize()
        same = np.array_equal(ex.sorting_index(), mf.sorting_index())
        if not same:
            first_split = g
            break
        for key in ("Current Mean", "Covariance Matrix"):
            a, b = ex[key], mf[key]
            rel = np.max(np.abs(a - b)) / np.max(np.abs(a))
            worst = max(worst, rel)
            assert rel < 1e-6, (g, key, rel)
    print(f"MFMA trajectory: max relative deviation {worst:.3e}; first differing selection at generation "
          f"{first_split} of {gens}")
    assert first_split is None or first_split > 3
    ex.close()
    mf.close()


def test_gradient_informed_mean_step_matches_oracle_bit_exact():
    """Use Gradient Information (CMAES.cpp.base:82-87, :611-621): the mean
    moves by sum_i w_i step / sqrt(N) g_(i) after recombination.  Fitness
    and gradients (negative sphere and its gradient, numpy) handed to both
    sides; 15 generations bit for bit."""
    Nv, lam, step, seed = 10, 32, 0.05, 21

    def fg(X):  # negative sphere, -0.5 |x|^2, and its gradient -x
        F = np.array([-0.5 * float(np.sum(x * x)) for x in X])
        return F, -X

    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"] = np.full(Nv, 0.5)
    o["Initial Standard Deviation"] = np.full(Nv, 0.3)
    o.option("Use Gradient Information", 1)
    o.option("Gradient Step Size", step)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=np.full(Nv, 0.5), initial_std=np.full(Nv, 0.3), normal_seed=seed,
                        uniform_seed=seed + 1, gradient_step_size=step)
    plain = device_solver(Nv, lam, initial_value=np.full(Nv, 0.5), initial_std=np.full(Nv, 0.3), normal_seed=seed,
                          uniform_seed=seed + 1)
    for g in range(1, 16):
        if g == 1:
            o.initialize()
            dev.initialize()
            plain.initialize()
        o.prepare()
        dev.sample()
        if g == 1:
            plain.sample()
        X = dev.candidates()
        assert np.array_equal(X.reshape(-1), o["Sample Population"]), g
        F, G = fg(X.reshape(lam, Nv))
        o["Value Vector"] = F
        o["Gradients"] = G
        dev.set_fitness(F)
        dev.set_gradients(G)
        if g == 1:
            plain.set_fitness(F)
            plain.update(g)
        o.update(g)
        dev.update(g)
        dev.synchronize()
        for key in ("Current Mean", "Covariance Matrix", "Evolution Path", "Conjugate Evolution Path"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        assert dev["Sigma"][0] == o["Sigma"][0], g
        if g == 1:  # the gradient step moved the mean
            assert not np.array_equal(dev["Current Mean"], plain["Current Mean"])
    dev.close()
    plain.close()


@pytest.mark.parametrize("Nv,lam,mirrored,bound,gens", [(10, 8, False, (-19.0, 21.0), 120), (12, 32, False, (-3.0, 3.0), 80),
                                                        (6, 16, True, (-3.0, 3.0), 80), (1, 64, True, (-10.0, 10.0), 10)])
def test_discrete_variables_match_oracle_bit_exact(Nv, lam, mirrored, bound, gens):
    """Discrete variables (Granularity; CMAES.cpp.base:44-50, sampleSingle's
    discrete mutations :515-544, discretize :861-867, the masking update
    :834-859 and the masked sigma step :729-735): populations, selections,
    masks, sigma and both generators' states bit-exact vs the oracle.  The
    first case is examples/optimization/discrete/run-cmaes.py's setup
    (variables 0, 1, 3, 6 on the integers), the last the reference's
    statistical corner case 'Discrete with Mirrored Sampling'."""
    seed = 1701
    gran = np.zeros(Nv)
    gran[[i for i in (0, 1, 3, 6) if i < Nv]] = 1.0
    if Nv == 1:
        gran[0] = 0.0001
    if Nv == 12:
        gran[::2] = 0.25
    lb, ub = np.full(Nv, bound[0]), np.full(Nv, bound[1])
    x0 = (lb + ub) / 2
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"] = x0
    o["Initial Standard Deviation"] = (ub - lb) * 0.3
    o["Lower Bound"], o["Upper Bound"], o["Granularity"] = lb, ub, gran
    if mirrored:
        o.option("Mirrored Sampling", 1)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=x0, initial_std=(ub - lb) * 0.3, lower_bound=lb,
                        upper_bound=ub, granularity=gran, mirrored=mirrored, normal_seed=seed, uniform_seed=seed + 1)
    mutated = 0
    for g in range(1, gens + 1):
        o.generation(g, "sphere")
        dev.generation(g, "sphere")
        dev.synchronize()
        X = dev["Sample Population"].reshape(lam, Nv)
        assert np.array_equal(X, o["Sample Population"].reshape(lam, Nv)), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Covariance Matrix", "Masking Matrix", "Masking Matrix Sigma"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in ("Sigma", "Infeasible Sample Count", "Number Of Discrete Mutations", "Number Masking Matrix Entries",
                    "Chi Square Number Discrete Mutations"):
            assert dev[key][0] == o[key][0], (g, key)
        # discrete coordinates sit on their grids
        d = gran > 0
        assert np.array_equal(X[:, d], np.round(X[:, d] / gran[d]) * gran[d]), g
        mutated += o["Number Masking Matrix Entries"][0] > 0
    assert dev.get_rng(0) == o.rng(0).get_bytes()
    assert dev.get_rng(1) == o.rng(1).get_bytes()  # the mutations' uniforms, consumed in the reference's order
    if Nv >= 10:
        assert mutated > 0  # masked variables took geometric mutations
    dev.close()


@pytest.mark.parametrize("Nv,lam,s0,mirrored,max_res,gens", [(10, 64, 0.3, False, float("inf"), 12),
                                                             (10, 64, 0.3, True, float("inf"), 12),
                                                             (4, 64, 1.0, False, float("inf"), 25),
                                                             (4, 64, 1.0, True, float("inf"), 25),
                                                             (10, 64, 0.3, False, 3000.0, 8)])
def test_resampling_past_the_first_round_matches_oracle_bit_exact(Nv, lam, s0, mirrored, max_res, gens):
    """prepareGeneration's redraw loop (CMAES.cpp.base:443-491) for any number
    of infeasible draws: the mean starts ON the upper bound of [-0.5, 0.5]^N
    and Rosenbrock's optimum (1, ..., 1) lies outside the box, so a generation
    draws thousands of infeasible samples, far more than the first round's
    max(256, lambda/4) reserve; the device continues the Normal stream round
    after round exactly where the reference's do/while would.  Populations,
    selections, infeasible counts, mean / covariance / sigma and the final
    generator state bit for bit, plain and mirrored, unlimited and with a
    finite Max Infeasible Resamplings (reached in generation 1)."""
    seed = 4242
    lb, ub, x0 = np.full(Nv, -0.5), np.full(Nv, 0.5), np.full(Nv, 0.5)
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"], o["Initial Standard Deviation"] = x0, np.full(Nv, s0)
    o["Lower Bound"], o["Upper Bound"] = lb, ub
    if mirrored:
        o.option("Mirrored Sampling", 1)
    o.option("Max Infeasible Resamplings", max_res)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=x0, initial_std=np.full(Nv, s0), lower_bound=lb, upper_bound=ub,
                        mirrored=mirrored, max_infeasible_resamplings=max_res, normal_seed=seed,
                        uniform_seed=seed + 1)
    reserve = max(256, lam // 4)
    prev, most = 0.0, 0.0
    for g in range(1, gens + 1):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Covariance Matrix", "Axis Lengths"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in ("Sigma", "Infeasible Sample Count", "Best Ever Value"):
            assert dev[key][0] == o[key][0], (g, key)
        cnt = o["Infeasible Sample Count"][0]
        most = max(most, cnt - prev)
        prev = cnt
    # more infeasible draws in one generation than the first round's reserve
    # holds: the walk continued into later rounds
    assert most > reserve, most
    assert dev.get_rng(0) == o.rng(0).get_bytes()
    dev.close()


def test_discrete_resampling_past_the_first_round_matches_oracle_bit_exact():
    """Discrete variables redraw through the same rounds (the walk stops at a
    block boundary and resumes with the next transformed blocks; its
    mutations' uniforms are re-peeked from the consumed position)."""
    Nv, lam, seed, gens = 8, 16, 99, 10
    lb, ub = np.full(Nv, -1.0), np.full(Nv, 1.0)
    x0, s0 = np.full(Nv, 1.0), np.full(Nv, 0.8)
    gran = np.zeros(Nv)
    gran[::2] = 0.5
    o = R.CMAES(Nv, lam, 0)
    o["Initial Value"], o["Initial Standard Deviation"] = x0, s0
    o["Lower Bound"], o["Upper Bound"], o["Granularity"] = lb, ub, gran
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = device_solver(Nv, lam, initial_value=x0, initial_std=s0, lower_bound=lb, upper_bound=ub,
                        granularity=gran, normal_seed=seed, uniform_seed=seed + 1)
    prev, most = 0.0, 0.0
    for g in range(1, gens + 1):
        o.generation(g, "rosenbrock")
        dev.generation(g, "rosenbrock")
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Covariance Matrix", "Masking Matrix"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in ("Sigma", "Infeasible Sample Count"):
            assert dev[key][0] == o[key][0], (g, key)
        cnt = o["Infeasible Sample Count"][0]
        most = max(most, cnt - prev)
        prev = cnt
    assert most > 256, most
    assert dev.get_rng(0) == o.rng(0).get_bytes()
    assert dev.get_rng(1) == o.rng(1).get_bytes()
    dev.close()


@pytest.mark.parametrize("mirrored", [False, True])
def test_overflowing_draws_are_redrawn_like_the_reference(mirrored):
    """Unbounded variables: the reference redraws a sample only when it is
    not finite (optimizer.cpp.base:5-14).  With sigma = 1e308 about a quarter
    of the draws overflow; the overflow guard sends the generation through
    the redraw rounds, and the population, infeasible count and generator
    state equal the oracle's.  Without the guard tripping (sigma = 1) the
    population is the first lambda blocks, as before."""
    Nv, lam, seed = 4, 16, 5
    for sigma, expect_redraw in ((1e308, True), (1.0, False)):
        o = R.CMAES(Nv, lam, 0)
        o["Initial Value"], o["Initial Standard Deviation"] = np.zeros(Nv), np.ones(Nv)
        if mirrored:
            o.option("Mirrored Sampling", 1)
        R.lib().kr_rng_seed(o.rng(0).ptr, seed)
        R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
        dev = device_solver(Nv, lam, initial_value=np.zeros(Nv), initial_std=np.ones(Nv), mirrored=mirrored,
                            normal_seed=seed, uniform_seed=seed + 1)
        o.initialize()
        dev.initialize()
        o["Sigma"] = [sigma]
        dev["Sigma"] = [sigma]
        o.prepare()
        dev.sample()
        dev.synchronize()
        X = dev["Sample Population"]
        assert np.all(np.isfinite(X))
        assert np.array_equal(X, o["Sample Population"])
        assert dev["Infeasible Sample Count"][0] == o["Infeasible Sample Count"][0]
        assert (o["Infeasible Sample Count"][0] > 0) == expect_redraw
        assert dev.get_rng(0) == o.rng(0).get_bytes()
        dev.close()


def test_handles_of_different_sizes_interleaved_bit_exact():
    """Kernel attributes are process-wide: a large handle (N = 512, the
    multi-workgroup tridiagonalisation and the streamed apply on a
    cooperative / capacity-checked launch) created BEFORE a smaller one
    (N = 200, same kernels, less LDS) must still launch after the small one
    was created and ran (round 3 lowered the dynamic-LDS limit per handle, and
    the runtime's occupancy query then answered 0 for the large launches).
    Interleaved generations, both bit-exact vs the oracle."""
    big_o, big = oracle_and_device(512, 1024, "rosenbrock", 2)
    small_o, small = oracle_and_device(200, 512, "rosenbrock", 2)
    tiny_o, tiny = oracle_and_device(16, 32, "rosenbrock", 2)
    for g in (1, 2):
        for o, dev in ((big_o, big), (small_o, small), (tiny_o, tiny)):
            o.generation(g, "rosenbrock")
            dev.generation(g, "rosenbrock")
            dev.synchronize()
            assert np.array_equal(dev["Sample Population"], o["Sample Population"]), (dev.N, g)
            for key in ("Covariance Eigenvector Matrix", "Axis Lengths", "Covariance Matrix"):
                assert np.array_equal(dev[key], o[key]), (dev.N, g, key)
    for dev in (big, small, tiny):
        dev.close()


@pytest.mark.gpu
def test_profile_mark_brackets_a_stage():
    """kg_cmaes_profile_mark (the engine's exchange timing): begin / end pairs
    on the handle's stream accumulate into one stage; an end without a begin
    is refused."""
    dev = device_solver(8, 16, initial_value=np.zeros(8), initial_std=np.ones(8), normal_seed=1, uniform_seed=2)
    try:
        assert dev.profile_mark("exchange_test", 1) == 1
        for g in range(1, 3):
            assert dev.profile_mark("exchange_test", 0) == 0
            dev.generation(g, "rosenbrock")
            assert dev.profile_mark("exchange_test", 1) == 0
        ms, n = dev.profile_read("exchange_test")
        assert n == 2 and ms > 0.0
        assert dev.profile_read("exchange_test") == (0.0, 0)
    finally:
        dev.close()
