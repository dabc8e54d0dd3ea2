"""ctypes binding of the CPU oracle (oracle/librefcpu.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package korali_amd/.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS = {}
# "cr": the bit-exact oracle; "libm": timing-only build with the system libm
# log/exp/pow (the speed the reference itself would run at; not bit-exact)
_VARIANTS = {"cr": "librefcpu.so", "libm": "librefcpu_libm.so"}


# void (*)(const double *x, size_t N, double *out, size_t nc, void *ctx)
CONSTRAINT_FN = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_size_t, C.POINTER(C.c_double), C.c_size_t, C.c_void_p)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib(variant="cr"):
    if variant not in _LIBS:
        path = os.path.join(_HERE, _VARIANTS[variant])
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        vp, sz, dp, cp = C.c_void_p, C.c_size_t, C.POINTER(C.c_double), C.c_char_p
        L.kr_rng_seed.argtypes = [vp, C.c_uint64]
        L.kr_set_threads.argtypes = [C.c_int]
        L.kr_btpe_draws.restype = C.c_ulonglong
        L.kr_rng_get.argtypes = [vp]
        L.kr_rng_get.restype = C.c_uint32
        L.kr_ran_gaussian.argtypes = [vp, C.c_double]
        L.kr_ran_gaussian.restype = C.c_double
        L.kr_ran_flat.argtypes = [vp, C.c_double, C.c_double]
        L.kr_ran_flat.restype = C.c_double
        L.kr_ran_binomial.argtypes = [vp, C.c_double, C.c_uint]
        L.kr_ran_binomial.restype = C.c_uint
        L.kr_ran_multinomial.argtypes = [vp, sz, C.c_uint, dp, C.POINTER(C.c_uint)]
        L.kr_hypot.argtypes = [C.c_double, C.c_double]
        L.kr_hypot.restype = C.c_double
        L.kr_eigen_symmv.argtypes = [sz, dp, dp, dp]
        L.kr_eigen_symmv.restype = sz
        L.kr_qr_chase.argtypes = [sz, dp, dp, dp, sz]
        L.kr_symmtd_decomp.argtypes = [sz, dp, dp]
        L.kr_qr_chase.restype = sz
        L.kr_cholesky.argtypes = [sz, dp]
        L.kr_cholesky.restype = C.c_int
        L.kr_dtrmv_lower.argtypes = [sz, dp, dp]
        for f in ("kr_obj_negative_rosenbrock", "kr_obj_negative_ackley", "kr_obj_negative_sphere", "kr_loglik_gaussian"):
            getattr(L, f).argtypes = [dp, sz]
            getattr(L, f).restype = C.c_double
        L.kr_cmaes_new.argtypes = [sz, sz, sz]
        L.kr_cmaes_new.restype = vp
        L.kr_cmaes_free.argtypes = [vp]
        L.kr_cmaes_field.argtypes = [vp, cp, C.POINTER(sz)]
        L.kr_cmaes_field.restype = dp
        L.kr_cmaes_sorting_index.argtypes = [vp]
        L.kr_cmaes_sorting_index.restype = C.POINTER(sz)
        L.kr_cmaes_rng.argtypes = [vp, C.c_int]
        L.kr_cmaes_rng.restype = vp
        L.kr_cmaes_set_option.argtypes = [vp, cp, C.c_double]
        for f in ("kr_cmaes_initialize", "kr_cmaes_prepare", "kr_cmaes_eigen_only", "kr_cmaes_sample_only"):
            getattr(L, f).argtypes = [vp]
        L.kr_cmaes_evaluate.argtypes = [vp, C.c_int]
        L.kr_cmaes_update.argtypes = [vp, sz]
        L.kr_cmaes_generation.argtypes = [vp, sz, C.c_int]
        L.kr_cmaes_set_constraints.argtypes = [vp, sz, sz, sz, CONSTRAINT_FN, vp]
        L.kr_cmaes_check_mean_and_set_regime.argtypes = [vp]
        L.kr_cmaes_update_constraints.argtypes = [vp, sz]
        L.kr_cmaes_handle_constraints.argtypes = [vp]
        L.kr_cmaes_ccmaes_prepare.argtypes = [vp, sz]
        L.kr_cmaes_constraint_error.argtypes = [vp]
        L.kr_cmaes_constraint_error.restype = C.c_int
        L.kr_tmcmc_new.argtypes = [sz, sz]
        L.kr_tmcmc_new.restype = vp
        L.kr_tmcmc_free.argtypes = [vp]
        L.kr_tmcmc_field.argtypes = [vp, cp, C.POINTER(sz)]
        L.kr_tmcmc_field.restype = dp
        L.kr_tmcmc_rng.argtypes = [vp, C.c_int]
        L.kr_tmcmc_rng.restype = vp
        L.kr_tmcmc_set_option.argtypes = [vp, cp, C.c_double]
        L.kr_tmcmc_set_prior_map.argtypes = [vp, C.POINTER(C.c_int)]
        L.kr_tmcmc_set_prior_kinds.argtypes = [vp, C.POINTER(C.c_int)]
        L.kr_tmcmc_set_per_generation_burn_in.argtypes = [vp, dp, sz]
        L.kr_tmcmc_initialize.argtypes = [vp]
        L.kr_tmcmc_prepare.argtypes = [vp, sz]
        L.kr_tmcmc_evaluate.argtypes = [vp]
        L.kr_tmcmc_process_candidates.argtypes = [vp, sz]
        L.kr_tmcmc_process_generation.argtypes = [vp]
        L.kr_tmcmc_set_gradients.argtypes = [vp, dp, dp]
        L.kr_chi2inv_068.argtypes = [sz]
        L.kr_chi2inv_068.restype = C.c_double
        L.kr_tmcmc_generation.argtypes = [vp, sz]
        L.kr_tmcmc_minsearch.argtypes = [dp, sz, C.c_double, C.c_double, dp, dp]
        L.kr_tmcmc_minsearch.restype = sz
        L.kr_tmcmc_cv2.argtypes = [C.c_double, dp, sz, C.c_double, C.c_double]
        L.kr_tmcmc_cv2.restype = C.c_double
        _LIBS[variant] = L
    return _LIBS[variant]


RNG_BYTES = 5000


class Rng:
    """A GSL-compatible mt19937 state living in a ctypes buffer (or a view
    into a solver handle)."""

    def __init__(self, ptr=None, seed=None):
        if ptr is None:
            self._buf = C.create_string_buffer(RNG_BYTES)
            ptr = C.addressof(self._buf)
        self.ptr = ptr
        if seed is not None:
            lib().kr_rng_seed(self.ptr, seed)

    def get_bytes(self):
        return C.string_at(self.ptr, RNG_BYTES)

    def set_bytes(self, b):
        assert len(b) == RNG_BYTES
        C.memmove(self.ptr, b, RNG_BYTES)

    def to_hex(self):
        return self.get_bytes().hex().upper()

    def from_hex(self, h):
        self.set_bytes(bytes.fromhex(h))

    def words(self):
        """(mt[624] as uint32, mti)"""
        b = self.get_bytes()
        mt = np.frombuffer(b[: 624 * 8], dtype="<u8").astype(np.uint32)
        mti = int(np.frombuffer(b[624 * 8 : 624 * 8 + 4], dtype="<i4")[0])
        return mt, mti

    def set_words(self, mt, mti):
        b = bytearray(RNG_BYTES)
        b[: 624 * 8] = np.asarray(mt, dtype="<u8").tobytes()
        b[624 * 8 : 624 * 8 + 4] = np.int32(mti).tobytes()
        self.set_bytes(bytes(b))

    def get(self):
        return lib().kr_rng_get(self.ptr)

    def gaussian(self, sigma=1.0):
        return lib().kr_ran_gaussian(self.ptr, sigma)

    def flat(self, a, b):
        return lib().kr_ran_flat(self.ptr, a, b)


def _np_view(ptr, n):
    if n == 0:
        return np.zeros(0)
    return np.ctypeslib.as_array(ptr, shape=(n,))


class CMAES:
    MU_TYPES = {"Logarithmic": 0, "Linear": 1, "Equal": 2, "Proportional": 3}
    OBJECTIVES = {"rosenbrock": 0, "ackley": 1, "sphere": 2}

    def __init__(self, N, lam, mu=0, variant="cr"):
        self.L = lib(variant)
        self.h = self.L.kr_cmaes_new(N, lam, mu)
        self.N, self.lam = N, lam
        self.mu = mu if mu else lam // 2

    def __del__(self):
        try:
            self.L.kr_cmaes_free(self.h)
        except Exception:
            pass

    def field(self, name):
        n = C.c_size_t()
        p = self.L.kr_cmaes_field(self.h, name.encode(), C.byref(n))
        if not p:
            raise KeyError(name)
        return _np_view(p, n.value)

    def __getitem__(self, name):
        return self.field(name)

    def __setitem__(self, name, value):
        f = self.field(name)
        f[:] = np.asarray(value, dtype=np.float64).reshape(-1)

    def sorting_index(self):
        return np.ctypeslib.as_array(self.L.kr_cmaes_sorting_index(self.h), shape=(self.lam,)).copy()

    def rng(self, which):
        return Rng(self.L.kr_cmaes_rng(self.h, which))

    def option(self, name, value):
        self.L.kr_cmaes_set_option(self.h, name.encode(), float(value))

    def initialize(self):
        self.L.kr_cmaes_initialize(self.h)

    def prepare(self):
        self.L.kr_cmaes_prepare(self.h)

    def eigen(self):
        self.L.kr_cmaes_eigen_only(self.h)

    def sample(self):
        self.L.kr_cmaes_sample_only(self.h)

    def evaluate(self, objective):
        self.L.kr_cmaes_evaluate(self.h, self.OBJECTIVES[objective])

    def update(self, gen):
        self.L.kr_cmaes_update(self.h, gen)

    def generation(self, gen, objective):
        self.L.kr_cmaes_generation(self.h, gen, self.OBJECTIVES[objective])

    # ---- CCMA-ES (Problem "Constraints")
    def set_constraints(self, constraints, viability_population_size=2, viability_mu_value=0):
        """constraints: callables c(x) -> float, evaluated in list order per
        sample (optimization.cpp.base:11-24)."""
        funcs = list(constraints)

        def cb(x, n, out, nc, ctx):
            v = [float(x[i]) for i in range(n)]
            for c in range(nc):
                out[c] = float(funcs[c](v))

        self._cfn = CONSTRAINT_FN(cb)  # kept alive with the handle
        self.L.kr_cmaes_set_constraints(self.h, len(funcs), viability_population_size, viability_mu_value,
                                        self._cfn, None)

    def current_population_size(self):
        return self.field("Value Vector").size

    def ccmaes_prepare(self, gen):
        """runGeneration up to the objective (:188-196)."""
        self.L.kr_cmaes_ccmaes_prepare(self.h, gen)

    def ccmaes_generation(self, gen, objective):
        """one generation with a Python objective f(x) -> float over the
        current population (model evaluations counted as the reference)."""
        self.ccmaes_prepare(gen)
        lam = self.current_population_size()
        X = self.field("Sample Population").reshape(lam, self.N)
        self.field("Value Vector")[:] = [float(objective(list(map(float, x)))) for x in X]
        self.field("Model Evaluation Count")[0] += lam
        self.update(gen)
        if self.L.kr_cmaes_constraint_error(self.h):
            raise RuntimeError("CCMA-ES: no sample without constraint violations (the reference indexes out of range)")


class TMCMC:
    def __init__(self, N, P, variant="cr"):
        self.L = lib(variant)
        self.h = self.L.kr_tmcmc_new(N, P)
        self.N, self.P = N, P

    def __del__(self):
        try:
            self.L.kr_tmcmc_free(self.h)
        except Exception:
            pass

    def field(self, name):
        n = C.c_size_t()
        p = self.L.kr_tmcmc_field(self.h, name.encode(), C.byref(n))
        if not p:
            raise KeyError(name)
        return _np_view(p, n.value)

    def __getitem__(self, name):
        return self.field(name)

    def __setitem__(self, name, value):
        f = self.field(name)
        f[:] = np.asarray(value, dtype=np.float64).reshape(-1)

    def rng(self, which):
        return Rng(self.L.kr_tmcmc_rng(self.h, which))

    def option(self, name, value):
        self.L.kr_tmcmc_set_option(self.h, name.encode(), float(value))

    def set_prior_map(self, dist_of_var):
        m = (C.c_int * self.N)(*[int(v) for v in dist_of_var])
        self.L.kr_tmcmc_set_prior_map(self.h, m)

    def set_prior_kinds(self, kinds):  # 0 Uniform, 1 Normal (Prior Minimum / Maximum = Mean / sd)
        m = (C.c_int * self.N)(*[int(v) for v in kinds])
        self.L.kr_tmcmc_set_prior_kinds(self.h, m)

    def set_per_generation_burn_in(self, values):
        v = np.ascontiguousarray(values, dtype=np.float64)
        self.L.kr_tmcmc_set_per_generation_burn_in(self.h, v.ctypes.data_as(C.POINTER(C.c_double)), v.size)

    def initialize(self):
        self.L.kr_tmcmc_initialize(self.h)

    def prepare(self, gen):
        self.L.kr_tmcmc_prepare(self.h, gen)

    def evaluate(self):
        self.L.kr_tmcmc_evaluate(self.h)

    def set_gradients(self, grad, fim):
        """mTMCMC: every candidate's log-likelihood gradient (P x N) and Fisher
        information (P x N x N); kr_tmcmc_set_gradients."""
        g = np.ascontiguousarray(grad, dtype=np.float64).reshape(-1)
        f = np.ascontiguousarray(fim, dtype=np.float64).reshape(-1)
        dp = C.POINTER(C.c_double)
        self.L.kr_tmcmc_set_gradients(self.h, g.ctypes.data_as(dp), f.ctypes.data_as(dp))

    def process_candidates(self, gen):
        self.L.kr_tmcmc_process_candidates(self.h, gen)

    def process_generation(self):
        self.L.kr_tmcmc_process_generation(self.h)

    def generation(self, gen):
        self.L.kr_tmcmc_generation(self.h, gen)


def eigen_symmv(A):
    A = np.ascontiguousarray(A, dtype=np.float64).copy()
    n = A.shape[0]
    ev = np.zeros(n)
    Q = np.zeros((n, n))
    dp = C.POINTER(C.c_double)
    lib().kr_eigen_symmv(n, A.ctypes.data_as(dp), ev.ctypes.data_as(dp), Q.ctypes.data_as(dp))
    return ev, Q


def cholesky(A):
    A = np.ascontiguousarray(A, dtype=np.float64).copy()
    st = lib().kr_cholesky(A.shape[0], A.ctypes.data_as(C.POINTER(C.c_double)))
    return st, A


def objective(name, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    f = {"rosenbrock": lib().kr_obj_negative_rosenbrock, "ackley": lib().kr_obj_negative_ackley,
         "sphere": lib().kr_obj_negative_sphere, "gaussian": lib().kr_loglik_gaussian}[name]
    return f(x.ctypes.data_as(C.POINTER(C.c_double)), x.size)


def minsearch(loglike, exponent, target_cov):
    ll = np.ascontiguousarray(loglike, dtype=np.float64)
    xm, fm = C.c_double(), C.c_double()
    it = lib().kr_tmcmc_minsearch(ll.ctypes.data_as(C.POINTER(C.c_double)), ll.size, exponent, target_cov, C.byref(xm), C.byref(fm))
    return xm.value, fm.value, it


def multinomial(rng, p, N):
    p = np.ascontiguousarray(p, dtype=np.float64)
    n = np.zeros(p.size, dtype=np.uint32)
    lib().kr_ran_multinomial(rng.ptr, p.size, N, p.ctypes.data_as(C.POINTER(C.c_double)), n.ctypes.data_as(C.POINTER(C.c_uint)))
    return n
