"""TMCMC resampling: the interval-decided conditional-binomial walk the
handle uses (kg_tmcmc.hip multinomial_interval) against the exact walk and
the oracle's gsl_ran_multinomial restatement (oracle/refcpu.c
kr_ran_multinomial; TMCMC.cpp.base:303-309), several consecutive draws from
one generator, so the stream positions must agree too.  CPU only: the
library's host-only debug entry makes no device call."""
import ctypes

import numpy as np
import pytest

import refcpu as R


def weights(kind, K, rng):
    if kind == "flat":
        w = np.ones(K)
    elif kind == "lognormal":
        w = np.exp(rng.normal(0.0, 1.0, K))
    elif kind == "annealed":  # C3-like: exp(ll * drho - max)
        ll = -0.5 * rng.chisquare(32, K)
        w = np.exp((ll - ll.max()) * 0.05)
    elif kind == "heavy":  # a few categories with n p >= 14: the BTPE branch
        w = np.exp(rng.normal(0.0, 4.0, K))
    elif kind == "zeros":
        w = np.exp(rng.normal(0.0, 1.0, K))
        if K >= 3:
            w[::3] = 0.0
    else:
        raise ValueError(kind)
    return w / w.sum()


@pytest.mark.parametrize("kind", ["flat", "lognormal", "annealed", "heavy", "zeros"])
@pytest.mark.parametrize("K,N", [(1, 5), (7, 7), (500, 500), (8192, 8192), (300, 5000)])
def test_interval_walk_equals_exact_walk_and_oracle(kind, K, N):
    from korali_amd.native import lib
    L = lib()
    rng = np.random.default_rng(K * 31 + N)
    p = np.ascontiguousarray(weights(kind, K, rng))
    reps, seed = 3, 4242 + K
    ne = np.zeros(reps * K, dtype=np.uint32)
    ni = np.zeros(reps * K, dtype=np.uint32)
    assert L.kg_debug_multinomial(ctypes.c_uint64(seed), K, N, p.ctypes.data_as(ctypes.c_void_p), reps,
                                  ne.ctypes.data_as(ctypes.c_void_p), ni.ctypes.data_as(ctypes.c_void_p)) == 0
    o = R.Rng()
    R.lib().kr_rng_seed(o.ptr, seed)
    no = np.zeros(reps * K, dtype=np.uint32)
    for r in range(reps):
        out = (ctypes.c_uint * K)()
        R.lib().kr_ran_multinomial(o.ptr, K, N, p.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out)
        no[r * K:(r + 1) * K] = np.frombuffer(out, dtype=np.uint32)
    assert np.array_equal(ne, no)
    assert np.array_equal(ni, no)
    for r in range(reps):
        assert int(ni[r * K:(r + 1) * K].sum()) == N


def test_interval_walk_equals_exact_walk_many_seeds():
    """many generators and weight vectors: every count and the stream position
    (the next draw) of the interval walk equal the exact walk's"""
    from korali_amd.native import lib
    L = lib()
    K, N, reps = 2048, 2048, 2
    for seed in range(120):
        rng = np.random.default_rng(seed)
        p = np.ascontiguousarray(weights(["lognormal", "annealed", "heavy"][seed % 3], K, rng))
        ne = np.zeros(reps * K, dtype=np.uint32)
        ni = np.zeros(reps * K, dtype=np.uint32)
        assert L.kg_debug_multinomial(ctypes.c_uint64(seed), K, N, p.ctypes.data_as(ctypes.c_void_p), reps,
                                      ne.ctypes.data_as(ctypes.c_void_p), ni.ctypes.data_as(ctypes.c_void_p)) == 0
        assert np.array_equal(ne, ni), seed
