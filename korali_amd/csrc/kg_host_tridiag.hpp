// kg_host_tridiag.hpp — GSL symmtd_decomp on the host core (see
// kg_host_tridiag.cpp for the operation order and why it runs there).
#pragma once

namespace kg {

struct HostTridiag {
  int N = 0;
  double *mem = nullptr, **row = nullptr;  // row r of the lower triangle (64-byte aligned)
  double *v[2] = {nullptr, nullptr}, *x[2] = {nullptr, nullptr}, *nv = nullptr, *nx = nullptr, *colb = nullptr,
         *t1 = nullptr;
  int init(int N);
  void release();
  ~HostTridiag() { release(); }
  // C: row-major, row stride ldc, lower triangle read (CMAES::eigen mirrors it).
  // H: row i (i < N - 2) = column i below the diagonal after the step
  //    (H[i][0] = β = sd[i], H[i][r] = the reflector's v_r, r >= 1; GSL's A);
  // tau[i], i < N - 2; d[0..N), sd[0..N-1): the tridiagonal.
  void run(const double *C, int ldc, double *H, double *tau, double *d, double *sd);
};

}  // namespace kg
