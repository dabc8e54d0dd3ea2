// kg_host_tridiag.hpp — GSL symmtd_decomp on the host core (see
// kg_host_tridiag.cpp for the operation order and why it runs there).
#pragma once

namespace kg {

// One parallel phase of the multi-threaded tridiagonalisation (thread t of P
// takes column blocks t, t + P, ... and row blocks t, t + P, ...; see
// kg_host_tridiag.cpp).
struct HtMtJob {
  int kind = 0;  // 0: one Householder step's pass, 1: load C into the blocks
  int N = 0, P = 1, o = 0;
  int syr2 = 0, symv = 0;  // apply the pending rank-2 update / form this step's column and row sums
  int nextCol = 0;         // the owner of column o copies it (after the update) to nextcol
  double **colblk = nullptr, **rowblk = nullptr;
  const double *v = nullptr, *t1 = nullptr, *pv = nullptr, *px = nullptr, *npv = nullptr, *npx = nullptr;
  double *colsum = nullptr, *rowsum = nullptr, *nextcol = nullptr;
  const double *C = nullptr;
  int ldc = 0;
};

struct HostTridiagPool;

struct HostTridiag {
  int N = 0;
  double *mem = nullptr, **row = nullptr;  // row r of the lower triangle (64-byte aligned)
  double *v[2] = {nullptr, nullptr}, *x[2] = {nullptr, nullptr}, *nv = nullptr, *nx = nullptr, *colb = nullptr,
         *t1 = nullptr;
  // threads (the calling one included): 1 = the single-core pass; more =
  // the blocked two-copy pass over a pool of pinned helper threads
  int threads = 1;
  HostTridiagPool *pool = nullptr;
  int init(int N);
  void release();
  ~HostTridiag() { release(); }
  // helpers stop sleeping and spin, ready for the next run (called ahead of
  // it, e.g. while the covariance is still on its way)
  void wake();
  // C: row-major, row stride ldc, lower triangle read (CMAES::eigen mirrors it).
  // H: row i (i < N - 2) = column i below the diagonal after the step
  //    (H[i][0] = β = sd[i], H[i][r] = the reflector's v_r, r >= 1; GSL's A);
  // tau[i], i < N - 2; d[0..N), sd[0..N-1): the tridiagonal.
  void run(const double *C, int ldc, double *H, double *tau, double *d, double *sd);
};

}  // namespace kg
