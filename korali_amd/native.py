"""ctypes binding of the korali_amd C-ABI (include/korali_amd.h).

The product path: every call here goes to the HIP kernels in
korali_amd/libkorali_amd.so.  There is no CPU fallback — if the library is
missing or no HIP device is present, construction raises.
"""
import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libkorali_amd.so")
if os.environ.get("KORALI_AMD_LIB_VARIANT"):  # A/B builds (libkorali_amd_<variant>.so, same sources, other -D flags)
    LIB_PATH = os.path.join(_PKG, f"libkorali_amd_{os.environ['KORALI_AMD_LIB_VARIANT']}.so")
_LIB = None

MU_TYPES = {"logarithmic": 0, "linear": 1, "equal": 2, "proportional": 3}
OBJECTIVES = {"negative rosenbrock": 0, "negative ackley": 1, "negative sphere": 2,
              "rosenbrock": 0, "ackley": 1, "sphere": 2}
COV_MODES = {"exact": 0, "mfma": 1}


class KoraliDeviceError(RuntimeError):
    pass


class _CmaesCfg(C.Structure):
    _fields_ = [
        ("variable_count", C.c_size_t), ("population_size", C.c_size_t), ("mu_value", C.c_size_t),
        ("mu_type", C.c_int), ("initial_sigma_cumulation_factor", C.c_double),
        ("initial_damp_factor", C.c_double), ("initial_cumulative_covariance", C.c_double),
        ("is_sigma_bounded", C.c_int), ("diagonal_covariance", C.c_int), ("mirrored_sampling", C.c_int),
        ("max_infeasible_resamplings", C.c_double),
        ("lower_bound", C.POINTER(C.c_double)), ("upper_bound", C.POINTER(C.c_double)),
        ("initial_value", C.POINTER(C.c_double)), ("initial_std", C.POINTER(C.c_double)),
        ("min_std_update", C.POINTER(C.c_double)),
        ("normal_seed", C.c_uint64), ("uniform_seed", C.c_uint64), ("cov_mode", C.c_int), ("device", C.c_int),
        ("store_bdz", C.c_int), ("eigen_device_chase", C.c_int), ("shard_rank", C.c_int), ("shard_count", C.c_int),
        ("use_gradients", C.c_int), ("gradient_step_size", C.c_double),
        ("granularity", C.POINTER(C.c_double)),
        ("constraint_count", C.c_size_t), ("viability_population_size", C.c_size_t),
        ("viability_mu_value", C.c_size_t), ("max_covariance_matrix_corrections", C.c_double),
        ("target_success_rate", C.c_double), ("covariance_matrix_adaption_strength", C.c_double),
        ("global_success_learning_rate", C.c_double),
    ]


# int (*)(const double *X, size_t rows, size_t N, const size_t *ids, double *out, void *ctx)
CONSTRAINT_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_size_t, C.c_size_t, C.POINTER(C.c_size_t),
                            C.POINTER(C.c_double), C.c_void_p)


class _TmcmcCfg(C.Structure):
    _fields_ = [
        ("variable_count", C.c_size_t), ("population_size", C.c_size_t), ("max_chain_length", C.c_double),
        ("default_burn_in", C.c_double), ("target_cov", C.c_double), ("covariance_scaling", C.c_double),
        ("min_annealing_exponent_update", C.c_double), ("max_annealing_exponent_update", C.c_double),
        ("prior_min", C.POINTER(C.c_double)), ("prior_max", C.POINTER(C.c_double)),
        ("prior_distribution", C.POINTER(C.c_int)), ("distribution_count", C.c_size_t),
        ("prior_seeds", C.POINTER(C.c_uint64)), ("multinomial_seed", C.c_uint64),
        ("multivariate_seed", C.c_uint64), ("uniform_seed", C.c_uint64), ("likelihood", C.c_int),
        ("device", C.c_int), ("per_generation_burn_in", C.POINTER(C.c_double)),
        ("per_generation_burn_in_count", C.c_size_t), ("shard_rank", C.c_int), ("shard_count", C.c_int),
        ("version", C.c_int), ("step_size", C.c_double), ("domain_extension_factor", C.c_double),
        ("prior_kind", C.POINTER(C.c_int)),
    ]


EXPORTED = [
    "kg_last_error", "kg_abi_version", "kg_device_count",
    "kg_cmaes_create", "kg_cmaes_destroy", "kg_cmaes_initialize", "kg_cmaes_sample", "kg_cmaes_eval_builtin",
    "kg_cmaes_get_candidates", "kg_cmaes_set_fitness", "kg_cmaes_set_log_posterior", "kg_cmaes_update", "kg_cmaes_generation",
    "kg_cmaes_begin_sample", "kg_cmaes_wait_termination_fields", "kg_cmaes_set_gradients", "kg_cmaes_update_partial", "kg_cmaes_update_finalize",
    "kg_cmaes_shard_row_count", "kg_cmaes_update_rows",
    "kg_cmaes_synchronize", "kg_cmaes_field_size", "kg_cmaes_get_field", "kg_cmaes_set_field",
    "kg_cmaes_get_fields", "kg_cmaes_get_sorting_index", "kg_cmaes_get_rng", "kg_cmaes_set_rng", "kg_cmaes_device_ptr",
    "kg_cmaes_stream", "kg_cmaes_profile", "kg_cmaes_profile_read", "kg_cmaes_profile_mark",
    "kg_cmaes_set_constraints", "kg_cmaes_prepare_constrained", "kg_cmaes_population_size",
    "kg_tmcmc_create", "kg_tmcmc_destroy", "kg_tmcmc_generation", "kg_tmcmc_synchronize", "kg_tmcmc_field_size",
    "kg_tmcmc_get_field", "kg_tmcmc_set_field", "kg_tmcmc_get_rng", "kg_tmcmc_set_rng", "kg_tmcmc_prepare",
    "kg_tmcmc_evaluate", "kg_tmcmc_process", "kg_tmcmc_advance", "kg_tmcmc_get_pending",
    "kg_tmcmc_process_partial", "kg_tmcmc_process_finalize", "kg_tmcmc_device_ptr", "kg_tmcmc_stream", "kg_tmcmc_evaluate_prior", "kg_tmcmc_get_candidates", "kg_tmcmc_set_evaluations",
    "kg_tmcmc_set_gradients",
    "kg_tmcmc_profile", "kg_tmcmc_profile_read", "kg_debug_mt_jump", "kg_debug_multinomial", "kg_debug_cartpole",
    "kg_debug_cartpole_at",
    "kg_debug_host_tridiag", "kg_debug_host_chase",
    # VRACER (korali_amd/vracer.py binds their argument types)
    "kg_vracer_create", "kg_vracer_destroy", "kg_vracer_hyperparameter_count", "kg_vracer_field_size",
    "kg_vracer_get_field", "kg_vracer_set_field", "kg_vracer_get_scalar", "kg_vracer_set_scalar",
    "kg_vracer_run_policy", "kg_vracer_set_action_noise", "kg_vracer_environment_step", "kg_vracer_train_policy",
    "kg_vracer_train_policy_minibatch", "kg_vracer_training_step", "kg_vracer_test_episodes", "kg_vracer_rescale_states", "kg_vracer_synchronize", "kg_vracer_stream",
    "kg_vracer_profile", "kg_vracer_profile_read", "kg_vracer_save_state", "kg_vracer_load_state",
    "kg_vracer_train_pending", "kg_vracer_host_launch", "kg_vracer_host_act", "kg_vracer_host_feed",
]


def lib():
    """Load libkorali_amd.so (raises if it is absent: no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise KoraliDeviceError(f"{LIB_PATH} not built; run `python -m korali_amd._build` (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        vp, sz, dp, cp, ip = C.c_void_p, C.c_size_t, C.POINTER(C.c_double), C.c_char_p, C.c_int
        L.kg_last_error.restype = cp
        L.kg_abi_version.restype = ip
        L.kg_device_count.argtypes = [C.POINTER(C.c_int)]
        L.kg_cmaes_create.argtypes = [C.POINTER(_CmaesCfg), C.POINTER(vp)]
        for f in ("kg_cmaes_destroy", "kg_cmaes_initialize", "kg_cmaes_sample", "kg_cmaes_synchronize",
                  "kg_cmaes_begin_sample"):
            getattr(L, f).argtypes = [vp]
        L.kg_cmaes_eval_builtin.argtypes = [vp, ip]
        L.kg_cmaes_get_candidates.argtypes = [vp, dp, sz]
        L.kg_cmaes_set_fitness.argtypes = [vp, dp]
        L.kg_cmaes_set_log_posterior.argtypes = [vp, dp]
        L.kg_cmaes_set_gradients.argtypes = [vp, dp]
        L.kg_cmaes_update.argtypes = [vp, sz]
        L.kg_cmaes_update_partial.argtypes = [vp, sz]
        L.kg_cmaes_update_finalize.argtypes = [vp, sz]
        L.kg_cmaes_shard_row_count.argtypes = [vp, C.POINTER(sz)]
        L.kg_cmaes_update_rows.argtypes = [vp, sz]
        L.kg_debug_mt_jump.argtypes = [vp, C.c_uint64, vp]
        L.kg_debug_multinomial.argtypes = [C.c_uint64, C.c_size_t, C.c_uint, vp, C.c_size_t, vp, vp]
        L.kg_debug_cartpole.argtypes = [ip, vp, vp, sz, sz, vp, vp]
        L.kg_debug_cartpole_at.argtypes = [ip, vp, vp, vp, sz, sz, vp, vp, vp]
        L.kg_debug_host_tridiag.argtypes = [sz, vp, vp, vp, vp, vp]
        L.kg_debug_host_chase.argtypes = [sz, vp, vp, C.c_int, sz, vp, vp, vp, sz, vp, vp]
        L.kg_cmaes_generation.argtypes = [vp, sz, ip]
        L.kg_cmaes_field_size.argtypes = [vp, cp, C.POINTER(sz)]
        L.kg_cmaes_get_field.argtypes = [vp, cp, dp, sz]
        L.kg_cmaes_set_field.argtypes = [vp, cp, dp, sz]
        L.kg_cmaes_get_sorting_index.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.kg_cmaes_get_fields.argtypes = [vp, C.POINTER(cp), sz, dp]
        L.kg_cmaes_wait_termination_fields.argtypes = [vp, dp]
        L.kg_cmaes_set_constraints.argtypes = [vp, CONSTRAINT_FN, vp]
        L.kg_cmaes_prepare_constrained.argtypes = [vp, sz]
        L.kg_cmaes_population_size.argtypes = [vp, C.POINTER(sz), C.POINTER(sz)]
        L.kg_cmaes_get_rng.argtypes = [vp, ip, vp]
        L.kg_cmaes_set_rng.argtypes = [vp, ip, vp]
        L.kg_cmaes_device_ptr.argtypes = [vp, cp, C.POINTER(vp)]
        L.kg_cmaes_stream.argtypes = [vp, C.POINTER(vp)]
        L.kg_cmaes_profile.argtypes = [vp, ip]
        L.kg_cmaes_profile_read.argtypes = [vp, cp, dp, C.POINTER(sz)]
        L.kg_cmaes_profile_mark.argtypes = [vp, cp, ip]
        L.kg_tmcmc_create.argtypes = [C.POINTER(_TmcmcCfg), C.POINTER(vp)]
        for f in ("kg_tmcmc_destroy", "kg_tmcmc_synchronize", "kg_tmcmc_evaluate", "kg_tmcmc_evaluate_prior"):
            getattr(L, f).argtypes = [vp]
        L.kg_tmcmc_device_ptr.argtypes = [vp, cp, C.POINTER(vp)]
        L.kg_tmcmc_stream.argtypes = [vp, C.POINTER(vp)]
        for f in ("kg_tmcmc_generation", "kg_tmcmc_prepare", "kg_tmcmc_process", "kg_tmcmc_process_partial",
                  "kg_tmcmc_process_finalize"):
            getattr(L, f).argtypes = [vp, sz]
        L.kg_tmcmc_field_size.argtypes = [vp, cp, C.POINTER(sz)]
        L.kg_tmcmc_get_field.argtypes = [vp, cp, dp, sz]
        L.kg_tmcmc_set_field.argtypes = [vp, cp, dp, sz]
        L.kg_tmcmc_get_rng.argtypes = [vp, ip, vp]
        L.kg_tmcmc_set_rng.argtypes = [vp, ip, vp]
        L.kg_tmcmc_get_candidates.argtypes = [vp, dp, sz]
        L.kg_tmcmc_set_evaluations.argtypes = [vp, dp, dp]
        L.kg_tmcmc_set_gradients.argtypes = [vp, dp, dp]
        L.kg_tmcmc_advance.argtypes = [vp, sz, C.POINTER(sz)]
        L.kg_tmcmc_get_pending.argtypes = [vp, C.POINTER(C.c_ubyte)]
        L.kg_tmcmc_profile.argtypes = [vp, ip]
        L.kg_tmcmc_profile_read.argtypes = [vp, cp, dp, C.POINTER(sz)]
        _LIB = L
    return _LIB


def check(rc):
    if rc != 0:
        raise KoraliDeviceError(lib().kg_last_error().decode())


def device_count():
    n = C.c_int(0)
    check(lib().kg_device_count(C.byref(n)))
    return n.value


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _vec(x, n, default):
    if x is None:
        return np.full(n, default, dtype=np.float64)
    a = np.ascontiguousarray(np.broadcast_to(np.asarray(x, dtype=np.float64), (n,)))
    return a


class CmaesDevice:
    """One CMA-ES solver instance resident on one MI355X (kg_cmaes_t)."""

    def __init__(self, N, lam, mu=0, mu_type="Logarithmic", lower_bound=None, upper_bound=None, initial_value=None,
                 initial_std=None, min_std_update=None, normal_seed=0, uniform_seed=0, cov_mode="exact",
                 is_sigma_bounded=False, diagonal=False, max_infeasible_resamplings=float("inf"),
                 initial_sigma_cumulation_factor=-1.0, initial_damp_factor=-1.0,
                 initial_cumulative_covariance=-1.0, device=0, store_bdz=False, eigen_chase="host", shard_rank=0,
                 shard_count=1, mirrored=False, gradient_step_size=None, granularity=None, constraints=None,
                 viability_population_size=2, viability_mu_value=0, max_covariance_matrix_corrections=1e6,
                 target_success_rate=0.1818, covariance_matrix_adaption_strength=0.1,
                 global_success_learning_rate=0.2):
        """constraints: CCMA-ES constraint functions c(x) -> float (x: the
        sample as a list), evaluated in list order per sample; a sample
        violates c when c(x) > 0 (beyond the viability boundary)."""
        L = lib()
        self.N, self._lam_cfg = int(N), int(lam)
        self.mu = int(mu) if mu else self._lam_cfg // 2
        self._arrays = [
            _vec(lower_bound, self.N, -np.inf), _vec(upper_bound, self.N, np.inf),
            _vec(initial_value, self.N, np.nan), _vec(initial_std, self.N, np.nan),
            _vec(min_std_update, self.N, 0.0), _vec(granularity, self.N, 0.0),
        ]
        cfg = _CmaesCfg()
        cfg.variable_count, cfg.population_size, cfg.mu_value = self.N, self._lam_cfg, int(mu)
        cfg.mu_type = MU_TYPES[mu_type.lower()] if isinstance(mu_type, str) else int(mu_type)
        cfg.initial_sigma_cumulation_factor = initial_sigma_cumulation_factor
        cfg.initial_damp_factor = initial_damp_factor
        cfg.initial_cumulative_covariance = initial_cumulative_covariance
        cfg.is_sigma_bounded, cfg.diagonal_covariance = int(is_sigma_bounded), int(diagonal)
        cfg.mirrored_sampling = int(bool(mirrored))
        cfg.use_gradients, cfg.gradient_step_size = int(gradient_step_size is not None), float(gradient_step_size or 0.0)
        cfg.max_infeasible_resamplings = float(max_infeasible_resamplings)
        (cfg.lower_bound, cfg.upper_bound, cfg.initial_value, cfg.initial_std,
         cfg.min_std_update, cfg.granularity) = [_dptr(a) for a in self._arrays]
        cfg.normal_seed, cfg.uniform_seed = int(normal_seed), int(uniform_seed)
        cfg.cov_mode = COV_MODES[cov_mode.lower()] if isinstance(cov_mode, str) else int(cov_mode)
        cfg.device, cfg.store_bdz = int(device), int(store_bdz)
        cfg.eigen_device_chase = 1 if eigen_chase == "device" else 0
        cfg.shard_rank, cfg.shard_count = int(shard_rank), int(shard_count)
        self.shard_rank, self.shard_count = int(shard_rank), max(1, int(shard_count))
        self._constraints = list(constraints or [])
        cfg.constraint_count = len(self._constraints)
        cfg.viability_population_size, cfg.viability_mu_value = int(viability_population_size), int(viability_mu_value)
        cfg.max_covariance_matrix_corrections = float(max_covariance_matrix_corrections)
        cfg.target_success_rate = float(target_success_rate)
        cfg.covariance_matrix_adaption_strength = float(covariance_matrix_adaption_strength)
        cfg.global_success_learning_rate = float(global_success_learning_rate)
        h = C.c_void_p()
        check(L.kg_cmaes_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self._L = L
        if self._constraints:
            funcs = self._constraints

            def cb(X, rows, n, ids, out, ctx):
                try:
                    nc = len(funcs)
                    for r in range(rows):
                        x = [float(X[r * n + d]) for d in range(n)]
                        for c in range(nc):
                            out[r * nc + c] = float(funcs[c](x))
                    return 0
                except Exception:  # reported as a failed evaluation by the library
                    return 1

            self._cfn = CONSTRAINT_FN(cb)  # kept alive with the handle
            check(L.kg_cmaes_set_constraints(self.h, self._cfn, None))

    @property
    def lam(self):
        """the current population size (CCMA-ES: the viability one in its viability regime)"""
        n = C.c_size_t()
        check(self._L.kg_cmaes_population_size(self.h, C.byref(n), None))
        return n.value

    def prepare_constrained(self, generation):
        """CCMA-ES: regime check, draw, constraint evaluation and handling
        (kg_cmaes_prepare_constrained); then evaluate the current population."""
        check(self._L.kg_cmaes_prepare_constrained(self.h, int(generation)))

    def close(self):
        if getattr(self, "h", None):
            self._L.kg_cmaes_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # stages
    def initialize(self):
        check(self._L.kg_cmaes_initialize(self.h))

    def sample(self):
        check(self._L.kg_cmaes_sample(self.h))

    def evaluate(self, objective):
        check(self._L.kg_cmaes_eval_builtin(self.h, OBJECTIVES[objective.lower()] if isinstance(objective, str)
                                            else int(objective)))

    def update(self, generation):
        check(self._L.kg_cmaes_update(self.h, int(generation)))

    def update_partial(self, generation):
        check(self._L.kg_cmaes_update_partial(self.h, int(generation)))

    def update_finalize(self, generation):
        check(self._L.kg_cmaes_update_finalize(self.h, int(generation)))

    def shard_row_count(self):
        """Doubles per rank block of the "Shard Rows" all-gather (exact-order
        sharded update; waits for the packing)."""
        n = C.c_size_t(0)
        check(self._L.kg_cmaes_shard_row_count(self.h, C.byref(n)))
        return int(n.value)

    def update_rows(self, generation):
        check(self._L.kg_cmaes_update_rows(self.h, int(generation)))

    def begin_sample(self):
        """Enqueue the next generation's generator prefetch and the first
        eigendecomposition phases (workspace only) — what the korali engine
        does right after each update (kg_cmaes_begin_sample)."""
        check(self._L.kg_cmaes_begin_sample(self.h))

    def generation(self, generation, objective):
        obj = OBJECTIVES[objective.lower()] if isinstance(objective, str) else int(objective)
        check(self._L.kg_cmaes_generation(self.h, int(generation), obj))

    def synchronize(self):
        check(self._L.kg_cmaes_synchronize(self.h))

    # host-callback objectives
    def candidates(self):
        X = np.empty((self.lam, self.N))
        check(self._L.kg_cmaes_get_candidates(self.h, _dptr(X), self.N))
        return X

    def _fitness_arg(self, F):
        F = np.ascontiguousarray(F, dtype=np.float64)
        if F.shape != (self.lam,):
            raise ValueError("fitness vector has shape %s, expected (%d,)" % (F.shape, self.lam))
        return F

    def set_fitness(self, F):
        F = self._fitness_arg(F)
        check(self._L.kg_cmaes_set_fitness(self.h, _dptr(F)))

    def set_gradients(self, G):
        """Use Gradient Information: every sample's gradient (lambda x N)."""
        G = np.ascontiguousarray(G, dtype=np.float64)
        if G.size != self.lam * self.N:
            raise ValueError(f"set_gradients: expected {self.lam} x {self.N} gradients, got {G.shape}")
        check(self._L.kg_cmaes_set_gradients(self.h, _dptr(G)))

    def set_log_posterior(self, F):
        """Bayesian problems: F(x) = logPosterior, -inf allowed."""
        F = self._fitness_arg(F)
        check(self._L.kg_cmaes_set_log_posterior(self.h, _dptr(F)))

    # state
    def field_size(self, name):
        n = C.c_size_t()
        check(self._L.kg_cmaes_field_size(self.h, name.encode(), C.byref(n)))
        return n.value

    def __getitem__(self, name):
        n = self.field_size(name)
        out = np.empty(n)
        check(self._L.kg_cmaes_get_field(self.h, name.encode(), _dptr(out), n))
        return out

    def __setitem__(self, name, value):
        a = np.ascontiguousarray(np.asarray(value, dtype=np.float64).reshape(-1))
        check(self._L.kg_cmaes_set_field(self.h, name.encode(), _dptr(a), a.size))

    def get_prefix(self, name, n):
        """The first n doubles of an exchange buffer ("Shard Rows")."""
        out = np.empty(int(n))
        check(self._L.kg_cmaes_get_field(self.h, name.encode(), _dptr(out), int(n)))
        return out

    def sorting_index(self):
        out = np.empty(self.lam, dtype=np.uint64)
        check(self._L.kg_cmaes_get_sorting_index(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    def get_rng(self, which):
        buf = C.create_string_buffer(5000)
        check(self._L.kg_cmaes_get_rng(self.h, int(which), buf))
        return buf.raw

    def set_rng(self, which, state):
        assert len(state) == 5000
        buf = C.create_string_buffer(bytes(state), 5000)
        check(self._L.kg_cmaes_set_rng(self.h, int(which), buf))

    def device_ptr(self, name):
        p = C.c_void_p()
        check(self._L.kg_cmaes_device_ptr(self.h, name.encode(), C.byref(p)))
        return p.value

    def stream(self):
        p = C.c_void_p()
        check(self._L.kg_cmaes_stream(self.h, C.byref(p)))
        return p.value

    def profile(self, enable=True):
        check(self._L.kg_cmaes_profile(self.h, int(enable)))

    def profile_read(self, stage):
        ms, n = C.c_double(), C.c_size_t()
        check(self._L.kg_cmaes_profile_read(self.h, stage.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def profile_mark(self, stage, phase):
        """kg_cmaes_profile_mark: phase 0 begins, 1 ends a caller-bracketed
        stage on the handle's stream; returns the C-ABI status (1: an end
        without a begin)."""
        return int(self._L.kg_cmaes_profile_mark(self.h, stage.encode(), int(phase)))


class TmcmcDevice:
    """One TMCMC sampler instance (Version "TMCMC") on one MI355X (kg_tmcmc_t).

    prior_min / prior_max: the Univariate/Uniform prior of every variable
    (prior_kind[d] = 1: the Univariate/Normal prior's Mean / Standard Deviation);
    prior_distribution[d]: index of the distribution object variable d draws
    from (variables sharing a distribution share its generator); prior_seeds[k]:
    seed of distribution k.  Generator indices for get_rng / set_rng:
    0 Multinomial, 1 Multivariate, 2 Uniform, 3 + k prior distribution k."""

    def __init__(self, N, P, prior_min, prior_max, prior_seeds=None, prior_distribution=None,
                 multinomial_seed=0, multivariate_seed=0, uniform_seed=0, target_cov=1.0, covariance_scaling=0.04,
                 min_annealing_exponent_update=1e-5, max_annealing_exponent_update=1.0, max_chain_length=1,
                 default_burn_in=0, per_generation_burn_in=(), likelihood=0, device=0, shard_rank=0, shard_count=0,
                 version=0, step_size=0.1, domain_extension_factor=0.2, prior_kind=None):
        L = lib()
        self.N, self.P = int(N), int(P)
        pdist = (np.arange(self.N, dtype=np.int32) if prior_distribution is None
                 else np.ascontiguousarray(prior_distribution, dtype=np.int32))
        ndist = int(pdist.max()) + 1
        seeds = np.zeros(ndist, dtype=np.uint64) if prior_seeds is None else np.ascontiguousarray(
            np.broadcast_to(np.asarray(prior_seeds, dtype=np.uint64), (ndist,)))
        pgb = np.ascontiguousarray(per_generation_burn_in, dtype=np.float64).reshape(-1)
        pkind = None if prior_kind is None else np.ascontiguousarray(prior_kind, dtype=np.int32)
        self._arrays = [_vec(prior_min, self.N, 0.0), _vec(prior_max, self.N, 1.0), pdist, seeds, pgb, pkind]
        cfg = _TmcmcCfg()
        cfg.variable_count, cfg.population_size = self.N, self.P
        cfg.max_chain_length, cfg.default_burn_in = float(max_chain_length), float(default_burn_in)
        cfg.target_cov, cfg.covariance_scaling = float(target_cov), float(covariance_scaling)
        cfg.min_annealing_exponent_update = float(min_annealing_exponent_update)
        cfg.max_annealing_exponent_update = float(max_annealing_exponent_update)
        cfg.prior_min, cfg.prior_max = _dptr(self._arrays[0]), _dptr(self._arrays[1])
        cfg.prior_distribution = pdist.ctypes.data_as(C.POINTER(C.c_int))
        cfg.distribution_count = ndist
        cfg.prior_seeds = seeds.ctypes.data_as(C.POINTER(C.c_uint64))
        cfg.multinomial_seed, cfg.multivariate_seed, cfg.uniform_seed = (int(multinomial_seed),
                                                                        int(multivariate_seed), int(uniform_seed))
        cfg.likelihood, cfg.device = int(likelihood), int(device)
        cfg.per_generation_burn_in = _dptr(pgb) if pgb.size else None
        cfg.per_generation_burn_in_count = pgb.size
        cfg.shard_rank, cfg.shard_count = int(shard_rank), int(shard_count)
        cfg.version = 1 if version in (1, "mTMCMC") else 0
        cfg.step_size, cfg.domain_extension_factor = float(step_size), float(domain_extension_factor)
        cfg.prior_kind = None if pkind is None else pkind.ctypes.data_as(C.POINTER(C.c_int))
        h = C.c_void_p()
        check(L.kg_tmcmc_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self._L = L

    def close(self):
        if getattr(self, "h", None):
            self._L.kg_tmcmc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare(self, generation):
        check(self._L.kg_tmcmc_prepare(self.h, int(generation)))

    def evaluate(self):
        check(self._L.kg_tmcmc_evaluate(self.h))

    def process(self, generation):
        check(self._L.kg_tmcmc_process(self.h, int(generation)))

    def process_partial(self, generation):
        check(self._L.kg_tmcmc_process_partial(self.h, int(generation)))

    def process_finalize(self, generation):
        check(self._L.kg_tmcmc_process_finalize(self.h, int(generation)))

    def device_ptr(self, name):
        p = C.c_void_p()
        check(self._L.kg_tmcmc_device_ptr(self.h, name.encode(), C.byref(p)))
        return p.value

    def stream(self):
        p = C.c_void_p()
        check(self._L.kg_tmcmc_stream(self.h, C.byref(p)))
        return p.value

    def advance(self, generation):
        """One step of every unfinished chain; returns how many chains now
        have a candidate pending evaluation."""
        n = C.c_size_t()
        check(self._L.kg_tmcmc_advance(self.h, int(generation), C.byref(n)))
        return n.value

    def pending(self):
        m = np.zeros(self.P, dtype=np.uint8)
        check(self._L.kg_tmcmc_get_pending(self.h, m.ctypes.data_as(C.POINTER(C.c_ubyte))))
        return m.astype(bool)

    def generation(self, generation):
        check(self._L.kg_tmcmc_generation(self.h, int(generation)))

    def synchronize(self):
        check(self._L.kg_tmcmc_synchronize(self.h))

    def evaluate_prior(self):
        check(self._L.kg_tmcmc_evaluate_prior(self.h))

    def candidates(self):
        X = np.empty((self.P, self.N))
        check(self._L.kg_tmcmc_get_candidates(self.h, _dptr(X), self.N))
        return X

    def set_evaluations(self, log_prior, log_likelihood):
        lp = np.ascontiguousarray(log_prior, dtype=np.float64)
        ll = np.ascontiguousarray(log_likelihood, dtype=np.float64)
        check(self._L.kg_tmcmc_set_evaluations(self.h, _dptr(lp), _dptr(ll)))

    def set_gradients(self, grad, fisher):
        """mTMCMC: every candidate's log-likelihood gradient (P x N) and Fisher
        information (P x N x N); kg_tmcmc_set_gradients."""
        g = np.ascontiguousarray(grad, dtype=np.float64).reshape(-1)
        f = np.ascontiguousarray(fisher, dtype=np.float64).reshape(-1)
        if g.size != self.P * self.N or f.size != self.P * self.N * self.N:
            raise ValueError("set_gradients: expected P x N gradients and P x N x N Fisher informations")
        check(self._L.kg_tmcmc_set_gradients(self.h, _dptr(g), _dptr(f)))

    def field_size(self, name):
        n = C.c_size_t()
        check(self._L.kg_tmcmc_field_size(self.h, name.encode(), C.byref(n)))
        return n.value

    def __getitem__(self, name):
        n = self.field_size(name)
        out = np.empty(n)
        check(self._L.kg_tmcmc_get_field(self.h, name.encode(), _dptr(out), n))
        return out

    def __setitem__(self, name, value):
        a = np.ascontiguousarray(np.asarray(value, dtype=np.float64).reshape(-1))
        check(self._L.kg_tmcmc_set_field(self.h, name.encode(), _dptr(a), a.size))

    def get_rng(self, which):
        buf = C.create_string_buffer(5000)
        check(self._L.kg_tmcmc_get_rng(self.h, int(which), buf))
        return buf.raw

    def set_rng(self, which, state):
        assert len(state) == 5000
        buf = C.create_string_buffer(bytes(state), 5000)
        check(self._L.kg_tmcmc_set_rng(self.h, int(which), buf))

    def profile(self, enable=True):
        check(self._L.kg_tmcmc_profile(self.h, int(enable)))

    def profile_read(self, stage):
        ms, n = C.c_double(), C.c_size_t()
        check(self._L.kg_tmcmc_profile_read(self.h, stage.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value
