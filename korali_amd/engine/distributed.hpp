// distributed.hpp — the "Distributed" conduit of korali_amd: population /
// chain sharding across the processes of one node, one process per GPU.
//
// Replaces, for the generation hot path, the reference's MPI engine/worker
// farm (source/modules/conduit/distributed/distributed.cpp.base:13-278,
// JSON samples over MPI_Send / MPI_Recv to worker teams).  Here every rank is
// an engine holding the replicated solver state on its own GPU; the solver's
// exchange steps are collectives on device buffers:
//   CMA-ES: all-gather of the λ fitnesses, sum all-reduce of the mean /
//           rank-μ partials (kg_cmaes_update_partial / _finalize);
//   TMCMC:  MAX all-reduce over the 64-bit patterns of the chain exchange
//           buffer (kg_tmcmc_process_partial / _finalize).
// Transports:
//   RCCL — ncclAllGather / ncclAllReduce on the handle's HIP stream over
//          xGMI (librccl.so loaded at run time; the engine links only the
//          C-ABI);
//   Host — buffers staged through host memory and exchanged over the TCP
//          bootstrap connections (several ranks on one GPU; CPU tests).
// Rendezvous as torch.distributed.run sets it up: RANK, WORLD_SIZE,
// MASTER_ADDR, MASTER_PORT (the bootstrap listens on MASTER_PORT + 1, or on
// the conduit's "Bootstrap Port").
#pragma once

#include <cstddef>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace korali {

// one solver buffer as the C-ABI exposes it
struct SolverBuffer {
  std::function<void *()> devicePtr;                 // device address (RCCL)
  std::function<void *()> stream;                    // the handle's HIP stream (RCCL)
  std::function<void(void *, size_t)> get, set;      // host copies (Host transport; bytes)
};

class Collective {
 public:
  virtual ~Collective() {}
  int rank = 0, world = 1;
  virtual std::string transport() const = 0;
  // in place: the buffer holds world * count doubles, this rank's block at [rank count, (rank+1) count)
  virtual void allGather(const SolverBuffer &b, size_t count) = 0;
  // in place on host memory: buf holds world * count doubles (small
  // per-sample results, e.g. CCMA-ES constraint values), over the bootstrap
  virtual void allGatherHost(double *buf, size_t count) = 0;
  // element-wise sum of n doubles
  virtual void allReduceSum(const SolverBuffer &b, size_t n) = 0;
  // element-wise MAX of n int64 (the bit patterns of doubles; exact gather)
  virtual void allReduceMaxI64(const SolverBuffer &b, size_t n) = 0;
  virtual void barrier() = 0;
  // another rank failed (its abort reached this rank's watchdog)
  virtual bool failed() const { return false; }
};

// rank / world from the environment (RANK, WORLD_SIZE); the TCP bootstrap on
// MASTER_ADDR:port; transport "RCCL" or "Host"
std::unique_ptr<Collective> makeCollective(const std::string &transport, int port);

}  // namespace korali
