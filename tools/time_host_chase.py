"""Wall time of the host core's Givens chase (kg_debug_host_chase: the
product's qr_chase) on the tridiagonal of a covariance-like matrix, separate
chop pass vs the fused sweep:  python tools/time_host_chase.py [N ...]"""
import ctypes
import os
import sys

import numpy as np

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_R, "tests"), os.path.join(_R, "oracle"), _R]
from test_host_chase import _tridiag, _vp  # noqa: E402
from korali_amd.native import lib  # noqa: E402


def main():
    for N in [int(a) for a in sys.argv[1:]] or [128, 512]:
        d, sd = _tridiag(N, 7, "spd")
        sd = np.append(sd, 0.0)
        reps = max(5, 200000 // (N * N))
        ev, perm = np.zeros(N), np.zeros(N, np.int32)
        counts, ns = np.zeros(3, np.int32), np.zeros(1)
        out = []
        for rnd in range(3):
            for fused in (0, 1):
                assert lib().kg_debug_host_chase(N, _vp(d), _vp(sd), fused, reps, _vp(ev), _vp(perm), None, 0,
                                                 _vp(counts), _vp(ns)) == 0
                out.append((fused, ns[0] / 1e3, ns[0] / counts[1]))
        for f in (0, 1):
            best = min(o[1] for o in out if o[0] == f)
            per = min(o[2] for o in out if o[0] == f)
            print(f"N={N} fused={f} steps={counts[0]} rotations={counts[1]} best {best:.1f} us "
                  f"= {per:.2f} ns/rotation", flush=True)


if __name__ == "__main__":
    main()
