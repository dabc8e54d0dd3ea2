"""Population-sharding check (run under torch.distributed.run, gloo, any
number of ranks on one device): S ranks run a sharded CMA-ES; rank 0 also
runs the unsharded handle from the same seed and compares every generation.
Exit code 0 = pass.  Used by tests/test_gpu_shard.py.

    shard_check.py N lambda generations objective gloo|nccl variant [exact|mfma]

exact (default): the exact-order sharded update; the sharded run must equal
the unsharded exact run (the reference's trajectory, which the unsharded
handle reproduces bit for bit, tests/test_gpu_cmaes.py) in every compared
field with np.array_equal, generation after generation, with no state
copied between them.  mfma: per-shard partial sums; each generation is
compared at the partial-sum tolerance and the sharded ranks then continue
from the unsharded state (the two summation orders drift apart by rounding,
which a run carries forward)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch.distributed as dist

from korali_amd.native import CmaesDevice
from korali_amd.sharded import ShardedCmaes


def main():
    N, lam, gens = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    obj = sys.argv[4] if len(sys.argv) > 4 else "rosenbrock"
    backend = sys.argv[5] if len(sys.argv) > 5 else "gloo"
    # sampling variant: plain (rows sharded), or one of the configurations
    # every rank draws whole (finite bounds with redraws, Mirrored Sampling,
    # discrete variables, diagonal covariance)
    variant = sys.argv[6] if len(sys.argv) > 6 else "plain"
    cov = sys.argv[7] if len(sys.argv) > 7 else "exact"
    if backend == "nccl":
        # RCCL with the zero-copy device transport (one rank per device)
        import torch
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    kw = dict(initial_value=np.full(N, 1.0), initial_std=np.full(N, 0.7), normal_seed=4321, uniform_seed=4322)
    if variant == "bounded":  # ~1 in 6 draws of the first generations infeasible at N = 32
        kw.update(lower_bound=np.full(N, -1.5), upper_bound=np.full(N, 3.0))
    elif variant == "mirrored":
        kw.update(mirrored=True)
    elif variant == "discrete":
        kw.update(granularity=np.where(np.arange(N) % 3 == 0, 0.25, 0.0), lower_bound=np.full(N, -4.0),
                  upper_bound=np.full(N, 4.0))
    elif variant == "diagonal":
        kw.update(diagonal=True)
    elif variant != "plain":
        raise SystemExit(f"unknown variant {variant}")
    sh = ShardedCmaes(N, lam, dist, device=0, transport="device" if backend == "nccl" else "host", cov_mode=cov, **kw)
    ref = CmaesDevice(N, lam, cov_mode=cov, **kw) if rank == 0 else None
    ok = True
    for g in range(1, gens + 1):
        sh.generation(g, obj)
        sh.synchronize()
        # replicated state is bit-identical on every rank
        state = np.concatenate([sh.dev[k] for k in ("Current Mean", "Covariance Matrix", "Sigma",
                                                    "Conjugate Evolution Path", "Evolution Path")])
        states = [None] * world
        dist.all_gather_object(states, state.tobytes())
        if rank == 0:
            if any(s != states[0] for s in states):
                print(f"gen {g}: replicated state differs between ranks", flush=True)
                ok = False
            ref.generation(g, obj)
            ref.synchronize()
            X = ref["Sample Population"].reshape(lam, N)
            r0, r1 = sh.r0, sh.r1
            if not np.array_equal(sh.dev["Sample Population"].reshape(lam, N)[r0:r1], X[r0:r1]):
                print(f"gen {g}: own rows differ from the unsharded population", flush=True)
                ok = False
            if not np.array_equal(sh.dev["Value Vector"], ref["Value Vector"]):
                print(f"gen {g}: gathered fitness differs", flush=True)
                ok = False
            if not np.array_equal(sh.dev.sorting_index(), ref.sorting_index()):
                print(f"gen {g}: sorting index differs", flush=True)
                ok = False
            if sh.dev["Infeasible Sample Count"][0] != ref["Infeasible Sample Count"][0]:
                print(f"gen {g}: infeasible sample count differs", flush=True)
                ok = False
            if cov == "exact":
                for k in ("Current Mean", "Covariance Matrix", "Sigma", "Evolution Path", "Conjugate Evolution Path",
                          "Best Ever Variables", "Best Ever Value", "Current Best Variables", "Axis Lengths",
                          "Covariance Eigenvector Matrix", "Mean Update"):
                    if not np.array_equal(sh.dev[k], ref[k]):
                        print(f"gen {g}: {k} differs from the unsharded exact run", flush=True)
                        ok = False
                for which in (0, 1):
                    if sh.dev.get_rng(which) != ref.get_rng(which):
                        print(f"gen {g}: generator {which} state differs", flush=True)
                        ok = False
                st = None  # no state is copied: the runs proceed independently
            else:
                for k, tol in (("Current Mean", 1e-12), ("Covariance Matrix", 1e-11), ("Sigma", 1e-12),
                               ("Best Ever Variables", 0.0)):
                    a, b = sh.dev[k], ref[k]
                    rel = np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)
                    if rel > tol:
                        print(f"gen {g}: {k} rel diff {rel:.3e} > {tol}", flush=True)
                        ok = False
                # teacher-force: continue from the unsharded state on every rank
                st = {k: ref[k] for k in ("Current Mean", "Covariance Matrix", "Sigma", "Evolution Path",
                                          "Conjugate Evolution Path", "Best Ever Variables", "Best Ever Value")}
        else:
            st = None
        box = [st]
        dist.broadcast_object_list(box, src=0)
        for k, v in (box[0] or {}).items():
            sh.dev[k] = v
    flag = [ok]
    dist.broadcast_object_list(flag, src=0)
    if rank == 0:
        print("SHARD_CHECK", "PASS" if flag[0] else "FAIL", flush=True)
    sh.close()
    if ref is not None:
        ref.close()
    dist.destroy_process_group()
    sys.exit(0 if flag[0] else 1)


if __name__ == "__main__":
    main()
