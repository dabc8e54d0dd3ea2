"""Population sharding on one device: S ranks (gloo,
host-staged collectives) against the unsharded handle — fitness all-gather,
replicated sort and state bit-identical across ranks, own rows bit-exact.
Exact covariance mode (default): every generation's whole state equal to the
unsharded exact run with np.array_equal, the runs independent (no state
copied); MFMA mode: mean / covariance / σ within the partial-sum tolerance."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("ranks,N,lam,gens,obj,backend,variant,cov", [
    (2, 32, 256, 6, "rosenbrock", "gloo", "plain", "exact"),
    (4, 200, 1024, 4, "ackley", "gloo", "plain", "exact"),
    (3, 130, 768, 4, "rosenbrock", "gloo", "plain", "exact"),
    (1, 64, 512, 4, "rosenbrock", "nccl", "plain", "exact"),
    (2, 32, 256, 6, "rosenbrock", "gloo", "bounded", "exact"),
    (2, 32, 256, 6, "rosenbrock", "gloo", "mirrored", "exact"),
    (3, 24, 192, 6, "rosenbrock", "gloo", "discrete", "exact"),
    (2, 40, 256, 6, "ackley", "gloo", "diagonal", "exact"),
    (2, 32, 256, 6, "rosenbrock", "gloo", "plain", "mfma"),
    (4, 200, 1024, 3, "ackley", "gloo", "plain", "mfma"),
    (1, 64, 512, 4, "rosenbrock", "nccl", "plain", "mfma")])
def test_sharded_population_matches_unsharded(ranks, N, lam, gens, obj, backend, variant, cov):
    """gloo: several ranks on the one device, host-staged collectives;
    nccl: the RCCL zero-copy device transport (one rank: one device here).
    Variants bounded / mirrored / discrete / diagonal: every rank draws the
    whole population (the redraw walk, the +-z pairs and the discrete
    mutations are sequential over it) and evaluates and sums its own rows."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tools", "shard_check.py"),
           str(N), str(lam), str(gens), obj, backend, variant, cov]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "SHARD_CHECK PASS" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.parametrize("ranks,N,P,gens,mcl,burn,backend", [(2, 4, 600, 8, 1, 0, "gloo"), (3, 3, 500, 8, 3, 1, "gloo"),
                                                             (4, 32, 1024, 4, 2, 2, "gloo"),
                                                             (1, 8, 512, 5, 2, 1, "nccl")])
def test_sharded_tmcmc_matches_unsharded(ranks, N, P, gens, mcl, burn, backend):
    """Chain sharding: every rank's state bit-identical to
    the unsharded run after the MAX all-reduce of the exchange words."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.join(ROOT, "tools", "shard_check_tmcmc.py"), str(N), str(P), str(gens), str(mcl), str(burn), backend]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "SHARD_CHECK PASS" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
