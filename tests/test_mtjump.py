"""mt19937 jump-ahead (host reference of the chunked device producer,
korali_amd/csrc/kg_mtjump.hip): the jumped window equals the words a
brute-force run of the recurrence reaches.  CPU only (no device call)."""
import ctypes

import numpy as np
import pytest

import refcpu as R


def untempered_stream(seed, n):
    """GSL mt19937 untempered words s_0..s_{n-1} (2002 seeding, rng/mt.c)."""
    s = np.zeros(n, dtype=np.uint64)
    s[0] = seed & 0xffffffff
    for i in range(1, 624):
        s[i] = (1812433253 * (int(s[i - 1]) ^ (int(s[i - 1]) >> 30)) + i) & 0xffffffff
    mag = np.uint64(0x9908b0df)
    for j0 in range(624, n, 227):
        j1 = min(j0 + 227, n)
        y = (s[j0 - 624:j1 - 624] & np.uint64(0x80000000)) | (s[j0 - 623:j1 - 623] & np.uint64(0x7fffffff))
        s[j0:j1] = s[j0 - 227:j1 - 227] ^ (y >> np.uint64(1)) ^ np.where((y & np.uint64(1)) == 1, mag, np.uint64(0))
    return s.astype(np.uint32)


def temper(y):
    y = y.astype(np.uint64)
    y ^= y >> np.uint64(11)
    y ^= (y << np.uint64(7)) & np.uint64(0x9d2c5680)
    y ^= (y << np.uint64(15)) & np.uint64(0xefc60000)
    y ^= y >> np.uint64(18)
    return (y & np.uint64(0xffffffff)).astype(np.uint32)


def test_brute_force_stream_matches_oracle():
    """pin the test's own generator to the oracle's GSL mt19937"""
    s = untempered_stream(790510, 624 + 2000)
    rng = R.Rng()
    R.lib().kr_rng_seed(rng.ptr, 790510)
    words = [R.lib().kr_rng_get(rng.ptr) for _ in range(2000)]
    assert np.array_equal(temper(s[624:2624]), np.array(words, dtype=np.uint32))


@pytest.mark.parametrize("start,J", [(624, 1), (1000, 12345), (3120, 2 ** 19), (7777, 1_500_000)])
def test_jump_matches_brute_force(start, J):
    from korali_amd.native import lib
    L = lib()
    s = untempered_stream(1337, start + J + 624 + 1)
    win = np.ascontiguousarray(s[start:start + 624])
    out = np.zeros(624, dtype=np.uint32)
    assert L.kg_debug_mt_jump(win.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(J),
                              out.ctypes.data_as(ctypes.c_void_p)) == 0
    assert np.array_equal(out, s[start + J:start + J + 624])
