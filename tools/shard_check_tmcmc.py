"""Chain-sharding check for TMCMC (run under torch.distributed.run; gloo with
any number of ranks on one device, or nccl with one rank per device): S
ranks run a sharded TMCMC; rank 0 also runs the unsharded handle from the
same seeds and compares every generation bit for bit.  Exit code 0 = pass.
Used by tests/test_gpu_shard.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch.distributed as dist

from korali_amd.native import TmcmcDevice
from korali_amd.sharded import ShardedTmcmc

KEYS = ("Chain Candidates", "Chain Candidates LogLikelihoods", "Chain Candidates LogPriors", "Chain Leaders",
        "Chain Leaders LogLikelihoods", "Chain Leaders LogPriors", "Chain Lengths", "Mean Theta", "Covariance Matrix",
        "Sample Database", "Sample LogLikelihood Database", "Sample LogPrior Database", "Num Selections",
        "Annealing Exponent", "Previous Annealing Exponent", "LogEvidence", "Coefficient Of Variation",
        "Max Loglikelihood", "Chain Count", "Accepted Samples Count", "Proposals Acceptance Rate",
        "Selection Acceptance Rate", "Model Evaluation Count", "Current Burn In")


def main():
    N, P, gens = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    mcl, burn = int(sys.argv[4]), int(sys.argv[5])
    backend = sys.argv[6] if len(sys.argv) > 6 else "gloo"
    if backend == "nccl":
        import torch
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    kw = dict(prior_min=[-5.0] * N, prior_max=[5.0] * N, prior_seeds=[77], prior_distribution=[0] * N,
              multinomial_seed=78, multivariate_seed=79, uniform_seed=80, max_chain_length=mcl, default_burn_in=burn)
    sh = ShardedTmcmc(N, P, dist, device=0, transport="device" if backend == "nccl" else "host", **kw)
    ref = TmcmcDevice(N, P, **kw) if rank == 0 else None
    ref2 = TmcmcDevice(N, P, **kw) if rank == 0 and os.environ.get("KORALI_AMD_SHARD_REF2") else None
    ok = True
    prev_nc = P
    for g in range(1, gens + 1):
        sh.generation(g)
        sh.synchronize()
        state = b"".join(np.asarray(sh.dev[k]).tobytes() for k in KEYS)
        states = [None] * world
        dist.all_gather_object(states, state)
        if rank == 0:
            if any(s != states[0] for s in states):
                print(f"gen {g}: replicated state differs between ranks", flush=True)
                ok = False
            ref.generation(g)
            ref.synchronize()
            for k in KEYS:
                a, b = sh.dev[k], ref[k]
                if a.tobytes() != b.tobytes():
                    print(f"gen {g}: {k} differs from the unsharded run", flush=True)
                    if k in ("Chain Candidates", "Sample Database", "Chain Leaders"):
                        ra, rb = np.asarray(a).reshape(P, -1), np.asarray(b).reshape(P, -1)
                        rows = np.nonzero((ra != rb).any(axis=1))[0]
                        print(f"   rows {rows[:12].tolist()} ({len(rows)}) of {P}; chain count before {prev_nc}", flush=True)
                    ok = False
            if ref2 is not None:
                ref2.generation(g)
                ref2.synchronize()
                for k in KEYS:
                    if ref2[k].tobytes() != ref[k].tobytes():
                        print(f"gen {g}: {k}: unsharded runs disagree", flush=True)
                    if ref2[k].tobytes() != sh.dev[k].tobytes():
                        print(f"gen {g}: {k}: sharded differs from the second unsharded run", flush=True)
            for which in range(4):
                if sh.dev.get_rng(which) != ref.get_rng(which):
                    print(f"gen {g}: generator {which} state differs", flush=True)
                    ok = False
        prev_nc = int(sh.dev["Chain Count"][0])
        if sh.dev["Previous Annealing Exponent"][0] >= 1.0:
            break
    flag = [ok]
    dist.broadcast_object_list(flag, src=0)
    if rank == 0:
        print("SHARD_CHECK", "PASS" if flag[0] else "FAIL", flush=True)
    sh.close()
    for r in (ref, ref2):
        if r is not None:
            r.close()
    dist.destroy_process_group()
    sys.exit(0 if flag[0] else 1)


if __name__ == "__main__":
    main()
