"""The host core's tridiagonalisation (korali_amd/csrc/kg_host_tridiag.cpp,
GSL symmtd_decomp in gslcblas order, CMAES.cpp.base:896-938) against the
oracle's restatement (oracle/refcpu.c symmtd_decomp, pinned to the
reference's 99 committed eigensystems by test_oracle_golden.py), bit for
bit.  CPU only: kg_debug_host_tridiag runs no device code."""
import ctypes

import numpy as np
import pytest

import refcpu as R


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _oracle(C):
    N = C.shape[0]
    A = np.tril(C) + np.tril(C, -1).T  # CMAES::eigen mirrors the lower triangle (:913-918)
    A = np.ascontiguousarray(A)
    tau = np.zeros(max(N - 1, 1))
    R.lib().kr_symmtd_decomp(N, A.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             tau.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return A, tau


def _device_lib():
    from korali_amd.native import lib
    return lib()


def _check(C):
    N = C.shape[0]
    L = _device_lib()
    H = np.zeros((N, N))
    tau, d, sd = np.zeros(N), np.zeros(N), np.zeros(N)
    Cc = np.ascontiguousarray(C)
    assert L.kg_debug_host_tridiag(N, _vp(Cc), _vp(H), _vp(tau), _vp(d), _vp(sd)) == 0
    A, t_ref = _oracle(C)
    assert np.array_equal(d.view(np.uint64), np.diag(A).copy().view(np.uint64))
    assert np.array_equal(sd[:N - 1].view(np.uint64), np.diag(A, -1).copy().view(np.uint64))
    for i in range(N - 2):
        col = A[i + 1:, i]
        assert np.array_equal(H[i, :N - 1 - i].view(np.uint64), col.copy().view(np.uint64)), i
        assert tau[i].tobytes() == t_ref[i].tobytes(), i


def _spd(N, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    Y = rng.standard_normal((N, 2 * N + 3))
    C = Y @ Y.T / Y.shape[1] + 0.05 * np.eye(N)
    return C * scale


@pytest.mark.parametrize("N", [2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 33, 64, 70, 96, 127, 128, 130, 200])
def test_host_tridiag_matches_oracle_bit_exact(N):
    C = _spd(N, N)
    C[np.triu_indices(N, 1)] = np.nan  # only the lower triangle is read
    _check(C)


def test_host_tridiag_c4_order():
    _check(_spd(512, 7))


def test_host_tridiag_zero_columns_and_tiny_scales():
    """xnorm == 0 steps (tau = 0, the column left as it is), the two-stage
    scaling of a reflector whose |alpha - beta| is below DBL_MIN, and
    subnormal/huge magnitudes"""
    N = 24
    C = np.diag(np.arange(1.0, N + 1))
    C[10, 3] = C[3, 10] = 0.25  # some columns have nothing below the diagonal
    _check(C)
    _check(_spd(19, 3, scale=1e-300))
    _check(_spd(19, 4, scale=1e150))
    C = _spd(21, 5)
    C[:, 6] = C[6, :] = 0.0
    C[6, 6] = 2.0
    _check(C)


def test_host_tridiag_is_deterministic_across_sizes_in_one_process():
    for N in (40, 8, 130, 40):
        _check(_spd(N, 11 + N))


@pytest.mark.parametrize("threads", [2, 3, 5])
@pytest.mark.parametrize("N", [9, 16, 17, 33, 70, 128, 200, 257])
def test_multi_threaded_pass_matches_oracle_bit_exact(monkeypatch, N, threads):
    """The pass split over helper threads (two blocked copies of the lower
    triangle: column sums down column blocks, row chains along row blocks,
    the same operands in the same order per element) equals the oracle bit
    for bit, for any thread count, block remainders included."""
    monkeypatch.setenv("KORALI_AMD_HOST_TRIDIAG_THREADS", str(threads))
    C = _spd(N, N + threads)
    C[np.triu_indices(N, 1)] = np.nan
    _check(C)


def test_multi_threaded_pass_zero_columns_and_tiny_scales(monkeypatch):
    monkeypatch.setenv("KORALI_AMD_HOST_TRIDIAG_THREADS", "3")
    test_host_tridiag_zero_columns_and_tiny_scales()
    _check(_spd(512, 9))
