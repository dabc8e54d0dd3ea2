"""Host logic of population sharding (korali_amd/sharded.py) on CPU with a
world-size-2 gloo group: shard ranges, the host-transport all-gather of
fitness shards and the sum all-reduce of partials."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from korali_amd.sharded import allgather_shards, allreduce_max_bits, allreduce_sum, shard_range


def test_shard_range_partitions_population():
    lam, world = 65536, 8
    rows = [shard_range(lam, world, r) for r in range(world)]
    assert rows[0][0] == 0 and rows[-1][1] == lam
    assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
    with pytest.raises(ValueError):
        shard_range(1000, 3, 0)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lam = 12
    r0, r1 = shard_range(lam, world, rank)
    F = np.arange(lam, dtype=np.float64) * 1.5 - 3.0
    got = allgather_shards(dist, F[r0:r1], world)
    part = np.full(5, float(rank + 1)) * np.array([1.0, 0.5, 0.25, 1e-300, -2.0])
    red = allreduce_sum(dist, part)
    q.put((rank, np.array_equal(got, F), red.tolist()))
    dist.destroy_process_group()


def test_host_transport_collectives_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res)
    expect = (1.0 + 2.0) * np.array([1.0, 0.5, 0.25, 1e-300, -2.0])
    for _, _, red in res:
        assert red == expect.tolist()


def _max_worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    vals = np.array([-0.0, 0.0, np.inf, -np.inf, np.nan, 1e-310, -3.5, 2.0 ** 60, -1e300, 7.0, -0.0, 5.0])
    own = np.arange(vals.size) % world == rank
    bits = vals.view(np.int64).copy()
    bits[~own] = np.iinfo(np.int64).min      # INT64_MIN = bits of -0.0
    got = allreduce_max_bits(dist, bits.view(np.float64))
    q.put((rank, got.view(np.int64).tolist() == vals.view(np.int64).tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_max_bits_allreduce_gathers_exact_patterns(world):
    """TMCMC chain sharding's exchange (kg_tmcmc_process_partial/finalize):
    owners' IEEE bit patterns (incl. -0.0, NaN, subnormals) survive a MAX
    all-reduce over the int64 view with INT64_MIN elsewhere."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_max_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res)
