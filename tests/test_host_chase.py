"""The host core's Givens chase (phase C of CMAES::eigen: GSL eigen/symmv.c's
implicit-QR loop, qrstep.c, chop_small_elements; kg_eigen.hip qr_chase)
against the oracle's restatement (oracle/refcpu.c kr_qr_chase, pinned with
the whole eigensolver to the reference's 99 committed eigensystems), bit for
bit: every rotation (c, s), the QR-step count and the eigenvalues.  The
fused sweep (the chop test and the rotation record folded into qrstep) must
equal the separate-pass form exactly.  CPU only: kg_debug_host_chase runs no
device code."""
import ctypes

import numpy as np
import pytest

import refcpu as R


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _lib():
    from korali_amd.native import lib
    return lib()


def _chase(d, sd, fused):
    N = d.size
    eval_, perm = np.zeros(N), np.zeros(N, np.int32)
    cap = 2 * (8 * N * N + 65536)
    cs = np.zeros(cap)
    counts = np.zeros(3, np.int32)
    ns = np.zeros(1)
    d = np.ascontiguousarray(d, np.float64)
    sd = np.ascontiguousarray(np.append(sd, 0.0), np.float64)
    assert _lib().kg_debug_host_chase(N, _vp(d), _vp(sd), int(fused), 1, _vp(eval_), _vp(perm), _vp(cs), cap,
                                      _vp(counts), _vp(ns)) == 0
    assert counts[2] == 0
    return eval_, perm, cs[:2 * counts[1]], counts[:2]


def _oracle(d, sd):
    N = d.size
    dd = np.ascontiguousarray(d, np.float64).copy()
    ss = np.ascontiguousarray(np.append(sd, 0.0), np.float64)
    maxrot = 8 * N * N + 65536
    cs = np.zeros(2 * maxrot)
    p = ctypes.POINTER(ctypes.c_double)
    rot = R.lib().kr_qr_chase(N, dd.ctypes.data_as(p), ss.ctypes.data_as(p), cs.ctypes.data_as(p), maxrot)
    return dd, cs[:2 * rot]


def _tridiag(N, seed, kind):
    rng = np.random.default_rng(seed)
    if kind == "spd":  # the tridiagonal of a covariance-like matrix (host tridiagonalisation's output)
        Y = rng.standard_normal((N, 2 * N + 3))
        C = Y @ Y.T / Y.shape[1]
        A = C.copy()
        tau = np.zeros(max(N - 1, 1))
        R.lib().kr_symmtd_decomp(N, A.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                 tau.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return np.diag(A).copy(), np.diag(A, -1).copy()
    d = rng.standard_normal(N)
    sd = rng.standard_normal(N - 1)
    if kind == "split":  # zeros / negligible couplings: several unreduced blocks, deflation mid-matrix
        sd[::7] = 0.0
        sd[3::11] *= 1e-17
    if kind == "repeated":  # clustered eigenvalues
        d = np.round(d)
        sd *= 1e-9
    return d, sd


@pytest.mark.parametrize("kind", ["spd", "random", "split", "repeated"])
@pytest.mark.parametrize("N", [2, 3, 5, 8, 17, 64, 128, 200])
def test_host_chase_matches_oracle_and_fused_sweep(N, kind):
    d, sd = _tridiag(N, 3 * N + len(kind), kind)
    od, ocs = _oracle(d, sd)
    for fused in (False, True):
        ev, perm, cs, counts = _chase(d, sd, fused)
        assert np.array_equal(cs.view(np.uint64), ocs.view(np.uint64)), fused
        # the unsorted eigenvalues through the permutation (gsl_eigen_symmv_sort ABS_ASC)
        assert np.array_equal(ev.view(np.uint64), od[perm].view(np.uint64)), fused
    a, b = _chase(d, sd, False), _chase(d, sd, True)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
