"""Population-sharded CMA-ES and chain-sharded TMCMC
(§8 f2) over torch.distributed.

One process per GPU; every rank holds the replicated solver state (mean, C,
B, D, paths, σ, generator states) in its own kg_cmaes_t handle created with
shard_rank / shard_count.  Per generation (CMAES::runGeneration,
CMAES.cpp.base:186-231):

  1. eigendecomposition — replicated (deterministic kernels: identical bits);
  2. the mt19937 polar stream is counted whole on every rank (its positions
     are global), but each rank materialises and transforms only the normals
     of its rows [r λ/S, (r+1) λ/S) and evaluates only those candidates;
  3. all-gather of the per-candidate fitnesses (λ doubles) — the one
     exchange the selection needs;
  4. replicated sort (identical sorting index everywhere, bit-exact);
  5. the update, in the handle's covariance mode:
     * "exact" (default): each rank packs the selected rows it owns
       (ascending selection rank) and one all-gather hands every rank all μ
       selected rows; mean and paths are then summed in the reference's
       order on every rank (CMAES.cpp.base:603-609), the rank-μ chains of
       the covariance's lower triangle are split by output entry across the
       ranks, each in the reference's order (:690-718), and one MAX
       all-reduce over their 64-bit patterns assembles the covariance.  Every
       rank's state is bit-identical to the unsharded run;
     * "mfma": each rank sums the mean and rank-μ terms of the selected rows
       it owns, one sum all-reduce of those partials (2N + N(N+16)/2
       doubles) — the sums in another order (≤1e-12 relative).

The collectives go through torch.distributed: backend "nccl" is RCCL over
xGMI on ROCm, and the tensors alias the handle's device buffers (zero copy,
ordered on the handle's HIP stream).  transport="host" stages the buffers
through host memory instead, for the gloo backend (several ranks on one
device, CPU-only process groups).
"""
import numpy as np

from .native import CmaesDevice, TmcmcDevice


class _DeviceArray:
    """__cuda_array_interface__ view of a device buffer (torch.as_tensor
    wraps it without copying)."""

    def __init__(self, ptr, n, typestr="<f8"):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def shard_range(lam, world, rank):
    """Rows [r0, r1) of the population owned by `rank` (λ % world == 0)."""
    if lam % world:
        raise ValueError(f"Population Size {lam} is not divisible by {world} ranks")
    per = lam // world
    return rank * per, (rank + 1) * per


def allgather_shards(dist, local, world, group=None):
    """Host transport: concatenate every rank's equal-size shard in rank
    order (numpy in, numpy out)."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(local))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts).numpy()


def allreduce_max_bits(dist, arr, group=None):
    """Host transport: element-wise MAX over ranks of the 64-bit patterns of a
    float64 array (int64 view).  With non-owned entries set to INT64_MIN (the
    bits of -0.0) this gathers every owner's exact bits."""
    import torch
    bits = np.ascontiguousarray(arr, dtype=np.float64).view(np.int64).copy()
    t = torch.from_numpy(bits)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.numpy().view(np.float64)


def allreduce_sum(dist, arr, group=None):
    """Host transport: element-wise sum over ranks (numpy in, numpy out)."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64).copy())
    dist.all_reduce(t, group=group)
    return t.numpy()


class ShardedCmaes:
    """CMA-ES generation loop with the population split across the ranks of
    a torch.distributed group (one kg_cmaes_t per rank)."""

    def __init__(self, N, lam, dist, group=None, device=0, transport="device", **cmaes_kw):
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.N, self.lam = int(N), int(lam)
        self.r0, self.r1 = shard_range(self.lam, self.world, self.rank)
        cmaes_kw.setdefault("cov_mode", "exact")
        self.exact = str(cmaes_kw["cov_mode"]).lower() == "exact"
        self.dev = CmaesDevice(N, lam, shard_rank=self.rank, shard_count=self.world, device=device, **cmaes_kw)
        self.transport = transport
        if transport == "device":
            import torch
            dv = torch.device("cuda", device)

            def view(name, typestr="<f8"):
                return torch.as_tensor(_DeviceArray(self.dev.device_ptr(name), self.dev.field_size(name), typestr),
                                       device=dv)

            self._F = view("Value Vector")
            if self.exact:
                self._R = view("Shard Rows") if self.dev.field_size("Shard Rows") else None
                self._C = view("Shard Covariance", "<i8")
            else:
                self._P = view("Shard Partials")
            self._stream = torch.cuda.ExternalStream(self.dev.stream(), device=dv)
        elif transport != "host":
            raise ValueError("transport must be 'device' or 'host'")

    def _exchange_fitness(self):
        if self.transport == "device":
            import torch
            with torch.cuda.stream(self._stream):
                self.dist.all_gather_into_tensor(self._F, self._F[self.r0:self.r1].clone(), group=self.group)
        else:
            F = self.dev["Value Vector"]
            self.dev["Value Vector"] = allgather_shards(self.dist, F[self.r0:self.r1], self.world, self.group)

    def _exchange_rows(self):
        n = self.dev.shard_row_count()  # doubles per rank block (0: every rank holds the population)
        if n == 0 or self.world == 1:
            return
        if self.transport == "device":
            import torch
            with torch.cuda.stream(self._stream):
                blk = self._R[self.rank * n:(self.rank + 1) * n].clone()
                self.dist.all_gather_into_tensor(self._R[:self.world * n], blk, group=self.group)
        else:
            R = self.dev.get_prefix("Shard Rows", self.world * n)
            self.dev["Shard Rows"] = allgather_shards(self.dist, R[self.rank * n:(self.rank + 1) * n], self.world,
                                                      self.group)

    def _gather_covariance(self):
        if self.world == 1:
            return
        if self.transport == "device":
            import torch
            with torch.cuda.stream(self._stream):
                self.dist.all_reduce(self._C, op=self.dist.ReduceOp.MAX, group=self.group)
        else:
            self.dev["Shard Covariance"] = allreduce_max_bits(self.dist, self.dev["Shard Covariance"], self.group)

    def _reduce_partials(self):
        if self.transport == "device":
            import torch
            with torch.cuda.stream(self._stream):
                self.dist.all_reduce(self._P, group=self.group)
        else:
            self.dev["Shard Partials"] = allreduce_sum(self.dist, self.dev["Shard Partials"], self.group)

    def generation(self, generation, objective):
        d = self.dev
        if generation == 1:
            d.initialize()
        d.sample()
        d.evaluate(objective)
        self._exchange_fitness()
        d.update_partial(generation)
        if self.exact:
            self._exchange_rows()
            d.update_rows(generation)
            self._gather_covariance()
        else:
            self._reduce_partials()
        d.update_finalize(generation)

    def synchronize(self):
        self.dev.synchronize()

    def close(self):
        self.dev.close()


class ShardedTmcmc:
    """TMCMC generation loop with the started chains split across the ranks
    of a torch.distributed group (one kg_tmcmc_t per rank, state
    replicated).  Per generation (TMCMC::runGeneration, TMCMC.cpp.base:
    107-157): Cholesky replicated; each rank draws, evaluates and steps only
    its contiguous share of the chains (the Multivariate / Uniform streams are
    counted whole, so positions are global); one MAX all-reduce over the
    int64 bits of the "Shard Exchange" buffer gathers the database, leader and
    candidate rows and accepted counts exactly; processGeneration (annealing
    search, multinomial resampling, weighted mean / covariance, leader
    expansion) then runs replicated, so every rank holds the unsharded run's
    state bit for bit."""

    def __init__(self, N, P, dist, group=None, device=0, transport="device", **tmcmc_kw):
        self.dist, self.group = dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.dev = TmcmcDevice(N, P, shard_rank=self.rank, shard_count=self.world, device=device, **tmcmc_kw)
        self.transport = transport
        if transport == "device":
            import torch
            dv = torch.device("cuda", device)
            n = self.dev.field_size("Shard Exchange")
            self._X = torch.as_tensor(_DeviceArray(self.dev.device_ptr("Shard Exchange"), n, "<i8"), device=dv)
            self._stream = torch.cuda.ExternalStream(self.dev.stream(), device=dv)
        elif transport != "host":
            raise ValueError("transport must be 'device' or 'host'")

    def _exchange(self):
        if self.world == 1:
            return
        if self.transport == "device":
            import torch
            with torch.cuda.stream(self._stream):
                self.dist.all_reduce(self._X, op=self.dist.ReduceOp.MAX, group=self.group)
        else:
            self.dev["Shard Exchange"] = allreduce_max_bits(self.dist, self.dev["Shard Exchange"], self.group)

    def generation(self, generation):
        d = self.dev
        d.prepare(generation)
        d.evaluate()
        d.process_partial(generation)
        self._exchange()
        d.process_finalize(generation)

    def synchronize(self):
        self.dev.synchronize()

    def close(self):
        self.dev.close()
