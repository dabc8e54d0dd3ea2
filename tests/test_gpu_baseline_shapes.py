"""GPU parity at the BASELINE.json shapes themselves:

* C4 — CMA-ES, 512-dim negative Ackley, λ = 65536, μ = 32768, x0 = 2,
  σ0 = 1, seed 1337, exact covariance mode: two full generations against the
  oracle (the OpenMP checker build keeps every output's reference order);
* C3 — TMCMC, 32 variables with one shared U(-5, 5) prior, loglik
  -0.5|x|², P = 8192 chains, seed 1337, run until Korali's termination
  (previous annealing exponent 1): every generation against the oracle;
* the BTPE branch of gsl_ran_binomial inside the multinomial resampling
  (n p >= 14), counted on both sides and required to have run;
* λ = 65536 population sharding over 2 gloo ranks against the unsharded
  handle (tools/shard_check.py, the default Exact covariance mode: the
  selected rows all-gathered, the rank-μ chains split by covariance tile and
  returned through the MAX-bits all-reduce).

Bar: bit-exact (np.array_equal / ==) everywhere, the sharded run included.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import refcpu as R
from test_gpu_tmcmc import SCA_KEYS, VEC_KEYS, seeded_pair

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c4_shape_two_generations_bit_exact():
    from korali_amd.native import CmaesDevice
    N, lam, seed = 512, 65536, 1337
    o = R.CMAES(N, lam, 0)
    o["Initial Value"] = np.full(N, 2.0)
    o["Initial Standard Deviation"] = np.ones(N)
    R.lib().kr_rng_seed(o.rng(0).ptr, seed)
    R.lib().kr_rng_seed(o.rng(1).ptr, seed + 1)
    dev = CmaesDevice(N, lam, initial_value=np.full(N, 2.0), initial_std=np.ones(N), normal_seed=seed,
                      uniform_seed=seed + 1, cov_mode="exact")
    for g in (1, 2):
        o.generation(g, "ackley")
        dev.generation(g, "ackley")
        dev.synchronize()
        assert np.array_equal(dev["Sample Population"], o["Sample Population"]), g
        assert np.array_equal(dev["Value Vector"], o["Value Vector"]), g
        assert np.array_equal(dev.sorting_index(), o.sorting_index()), g
        for key in ("Current Mean", "Previous Mean", "Evolution Path", "Conjugate Evolution Path",
                    "Covariance Matrix", "Covariance Eigenvector Matrix", "Axis Lengths"):
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in ("Sigma", "Best Ever Value", "Current Best Value", "Conjugate Evolution Path L2 Norm"):
            assert dev[key][0] == o[key][0], (g, key)
    assert dev.get_rng(0) == o.rng(0).get_bytes()
    assert dev.get_rng(1) == o.rng(1).get_bytes()
    dev.close()


def run_tmcmc_pair(N, P, target_cov, seed=1337, max_gens=40):
    dev, o, ndist = seeded_pair(N, P, True, seed=seed, target_cov=target_cov)
    b0 = R.lib().kr_btpe_draws()
    gens = 0
    for g in range(1, max_gens + 1):
        dev.generation(g)
        o.generation(g)
        dev.synchronize()
        gens = g
        for key in VEC_KEYS:
            assert np.array_equal(dev[key], o[key]), (g, key)
        for key in SCA_KEYS:
            a, b = dev[key][0], o[key][0]
            assert a == b or (np.isnan(a) and np.isnan(b)), (g, key, a, b)
        # Korali's TMCMC terminates one generation after reaching exponent 1
        if o["Previous Annealing Exponent"][0] >= 1.0:
            break
    for which in range(3 + ndist):
        assert dev.get_rng(which).hex().upper() == o.rng(which).to_hex(), which
    btpe_dev = dev["BTPE Binomial Draws"][0]
    btpe_oracle = R.lib().kr_btpe_draws() - b0
    dev.close()
    return gens, btpe_dev, btpe_oracle


def test_c3_shape_run_to_completion_bit_exact():
    """The whole C3 run (12 generations): candidates, accept decisions,
    annealing exponents, CoV, log-evidence, multinomial selections (two of
    them by BTPE), leaders, mean, covariance, generator states."""
    gens, btpe_dev, btpe_oracle = run_tmcmc_pair(32, 8192, 1.0)
    assert gens >= 10
    assert btpe_dev == btpe_oracle


def test_tmcmc_btpe_branch_runs_and_matches_oracle():
    """A high target CoV makes the resampling weights peaked, so many
    conditional binomials have n p >= 14 and take GSL's BTPE branch.  The
    device run equals the oracle bit for bit and the branch provably ran
    (counted on both sides).  GSL parity of BTPE itself stays unpinned: no
    reference fixture reaches it."""
    gens, btpe_dev, btpe_oracle = run_tmcmc_pair(8, 4096, 5.0)
    assert btpe_dev == btpe_oracle
    assert btpe_dev >= 20, btpe_dev


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c4_population_sharded_over_two_ranks():
    """λ = 65536, N = 512, Ackley: 2 gloo ranks (host-staged collectives) on
    the one device against the unsharded handle on rank 0."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tools", "shard_check.py"),
           "512", "65536", "2", "ackley", "gloo"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "SHARD_CHECK PASS" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
