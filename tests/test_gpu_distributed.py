"""The korali::Engine "Distributed" conduit (korali_amd/engine/distributed.cpp,
replacing the reference's MPI conduit, distributed.cpp.base:13-278, for the
generation hot path): ranks launched by torch.distributed.run, each an engine
on its GPU, the population / chains sharded, the exchange steps collectives
issued by the engine itself (no Python in the loop).

On the one-GPU box: 2 and 4 ranks share the device over the Host transport
(TCP bootstrap); the RCCL transport runs with one rank (RCCL refuses two
ranks on one device).  Every rank's state must equal rank 0's bit for bit;
TMCMC must equal the unsharded run bit for bit; CMA-ES must reproduce the
unsharded run bit for bit with the exact covariance update (the default; at
the C4 shape over 4 generations too), and with MFMA its sort exactly and its
mean / covariance / sigma within the partial-sum tolerance
(include/korali_amd.h: shard sums in another order).  Use Gradient
Information runs sharded too: each rank evaluates its rows' gradients, the
engine all-gathers them.  CCMA-ES (Problem "Constraints") runs replicated, its
objective and constraint callbacks split over the ranks: bit-identical; so
does mTMCMC, its likelihood / gradient / Fisher evaluations split."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(tmp_path, ranks, solver, model, transport, cov):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tools", "distributed_check.py"),
           str(tmp_path), solver, model, transport, cov]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [json.load(open(tmp_path / f"rank{k}.json")) for k in range(ranks)]


def close(a, b, rtol):
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    return a.shape == b.shape and np.allclose(a, b, rtol=rtol, atol=rtol * max(1.0, np.abs(b).max()))


@pytest.mark.parametrize("ranks,solver,model,transport,cov", [
    (2, "cmaes", "builtin", "Host", "Exact"), (4, "cmaes", "host", "Host", "Exact"),
    (1, "cmaes", "builtin", "RCCL", "Exact"), (2, "cmaes", "c4", "Host", "Exact"),
    (2, "cmaes", "builtin", "Host", "MFMA"), (1, "cmaes", "builtin", "RCCL", "MFMA"),
    (2, "cmaes", "grad", "Host", "Exact"), (2, "cmaes", "grad", "Host", "MFMA"),
    (3, "cmaes", "ccmaes", "Host", "Exact"), (1, "cmaes", "ccmaes", "RCCL", "Exact"),
    (2, "tmcmc", "builtin", "Host", "-"), (3, "tmcmc", "host", "Host", "-"), (1, "tmcmc", "builtin", "RCCL", "-"),
    (3, "tmcmc", "mtmcmc", "Host", "-")])
def test_distributed_conduit(tmp_path, ranks, solver, model, transport, cov):
    res = launch(tmp_path, ranks, solver, model, transport, cov)
    for gens in {"c4": ("1", "4"), "mtmcmc": ("1", "3")}.get(model, ("1", "6")):
        for r in res[1:]:
            assert r[gens]["sharded"] == res[0][gens]["sharded"], gens  # replicated: bit-identical on every rank
        s, u = res[0][gens]["sharded"], res[0][gens]["unsharded"]
        assert s["Current Generation"] == u["Current Generation"] == int(gens)
        if solver == "tmcmc" or cov == "Exact":
            # TMCMC: exact gather + replicated processGeneration; CMA-ES exact:
            # the selected rows gathered, the reference's summation order
            assert s == u, gens
            continue
        assert s["Model Evaluation Count"] == u["Model Evaluation Count"]
        if gens == "1":  # same state in: each rank's rows sampled / evaluated as the unsharded run's
            assert s["Value Vector"] == u["Value Vector"]
            assert s["Sorting Index"] == u["Sorting Index"]
            assert s["Best Ever Value"] == u["Best Ever Value"]
        # MFMA: per-generation partial-sum rounding, carried 6 generations
        tol = 1e-12 if gens == "1" else 1e-7
        for k in ("Current Mean", "Covariance Matrix", "Sigma", "Evolution Path", "Conjugate Evolution Path"):
            assert close(s[k], u[k], tol), (gens, k)


def test_replicated_callback_failure_reaches_every_rank(tmp_path):
    """Distributed CCMA-ES (replicated handle, constraint callbacks split over
    the ranks): rank 1's constraint raises; rank 1 reports its own error and
    rank 0 one naming rank 1 -- after the gathers, so neither waits forever."""
    res = launch(tmp_path, 2, "cmaes", "ccmaes_fail", "Host", "Exact")
    assert res[1]["error"] and "on purpose on rank 1" in res[1]["error"]
    assert res[0]["error"] and "rank 1 failed" in res[0]["error"]
