"""CPU tests of the Distributed conduit (korali_amd/engine/distributed.cpp):
the TCP bootstrap and the Host transport's collectives with 2 and 4 ranks
(separate processes, RANK / WORLD_SIZE / MASTER_* as torch.distributed.run
sets them), and the configuration errors raised before any device call."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import korali

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = r"""
import json, sys
import numpy as np
from korali_amd import libkorali
rank, n = int(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(100 + rank)
block = rng.standard_normal(n)
block[0] = -0.0 if rank % 2 else float(rank)  # signed zero: its bits are INT64_MIN
try:
    r = libkorali._collective_selftest(int(sys.argv[3]), block.tolist(), int(sys.argv[4]))
except Exception as e:
    print(json.dumps({"error": str(e)}))
    sys.exit(3)
print(json.dumps(r))
"""


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(world, n, fail_rank=-1):
    port = free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-c", RANK_SCRIPT, str(rank), str(n), "0", str(fail_rank)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for rank, p in enumerate(procs):
        o, e = p.communicate(timeout=120)
        assert p.returncode == (3 if rank == fail_rank else 0), e[-2000:]
        outs.append(__import__("json").loads(o.strip().splitlines()[-1]))
    return outs


def expected_blocks(world, n):
    blocks = []
    for rank in range(world):
        b = np.random.default_rng(100 + rank).standard_normal(n)
        b[0] = -0.0 if rank % 2 else float(rank)
        blocks.append(b)
    return blocks


@pytest.mark.parametrize("world,n", [(2, 37), (4, 1000)])
def test_host_transport_collectives(world, n):
    outs = run_ranks(world, n)
    blocks = expected_blocks(world, n)
    gathered = np.concatenate(blocks)
    summed = blocks[0].copy()
    for b in blocks[1:]:
        summed = summed + b  # rank order, as the root combines them
    maxed = np.max(np.stack([b.view(np.int64) for b in blocks]), axis=0).view(np.float64)
    for rank, o in enumerate(outs):
        assert o["rank"] == rank and o["world"] == world
        assert np.array_equal(np.array(o["gathered"]), gathered)
        assert np.array_equal(np.array(o["summed"]), summed)  # bit-identical on every rank
        assert np.array_equal(np.array(o["maxed"]).view(np.int64), maxed.view(np.int64))


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (3, 2), (3, 0)])
def test_rank_failure_reaches_every_rank(world, fail_rank):
    """A rank that fails tells the others over the abort channel (the
    watchdog that ends an RCCL rank's collectives with ncclCommAbort): every
    other rank sees the failure instead of waiting for it forever."""
    outs = run_ranks(world, 4, fail_rank)
    for rank, o in enumerate(outs):
        if rank == fail_rank:
            assert "failed on purpose" in o["error"]
        else:
            assert o["peer_failed"] is True


def cmaes_experiment():
    e = korali.Experiment()
    e["Problem"]["Type"] = "Optimization"
    e["Problem"]["Objective Kernel"] = "Negative Sphere"
    e["Variables"][0]["Name"] = "X"
    e["Variables"][0]["Initial Value"] = 0.0
    e["Variables"][0]["Initial Standard Deviation"] = 1.0
    e["Solver"]["Type"] = "Optimizer/CMAES"
    e["Solver"]["Population Size"] = 8
    e["File Output"]["Enabled"] = False
    e["Console Output"]["Verbosity"] = "Silent"
    return e


def distributed_engine(**keys):
    k = korali.Engine()
    k["Conduit"]["Type"] = "Distributed"
    k["Conduit"]["Transport"] = "Host"  # one rank: no sockets
    for key, v in keys.items():
        k["Conduit"][key.replace("_", " ")] = v
    return k


@pytest.mark.parametrize("keys,solver,msg", [
    ({"Ranks_Per_Worker": 2}, {}, "'Ranks Per Worker' must be 1"),
    ({"Transport": "MPI"}, {}, "'Transport' must be 'RCCL' or 'Host'"),
    ({}, {"Covariance Update": "Cholesky"}, "'Covariance Update' must be 'Exact' or 'MFMA'"),
])
def test_distributed_configuration_errors(monkeypatch, keys, solver, msg):
    for v in ("RANK", "WORLD_SIZE"):
        monkeypatch.delenv(v, raising=False)
    e = cmaes_experiment()
    for key, v in solver.items():
        e["Solver"][key] = v
    with pytest.raises(korali.KoraliError, match=msg):
        distributed_engine(**keys).run(e)


def test_distributed_rejects_vracer(monkeypatch):
    for v in ("RANK", "WORLD_SIZE"):
        monkeypatch.delenv(v, raising=False)
    e = korali.Experiment()
    e["Problem"]["Type"] = "Reinforcement Learning / Continuous"
    e["Solver"]["Type"] = "Agent / Continuous / VRACER"
    e["File Output"]["Enabled"] = False
    with pytest.raises(korali.KoraliError, match="independent replicas"):
        distributed_engine().run(e)


def test_inconsistent_rank_environment(monkeypatch):
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(korali.KoraliError, match="RANK / WORLD_SIZE"):
        distributed_engine().run(cmaes_experiment())
