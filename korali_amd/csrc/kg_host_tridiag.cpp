// kg_host_tridiag.cpp — phase A of CMAES::eigen (CMAES.cpp.base:896-938:
// gsl_eigen_symmv → gsl_linalg_symmtd_decomp, GSL 2.6 linalg/symmtd.c with
// gslcblas dnrm2 / dsymv / ddot / daxpy / dsyr2) on one host core.
//
// Why the host core: the decomposition's arithmetic order is fixed by the
// bit-exactness contract (the eigenvector signs steer the next population),
// so each Householder step is three ordered FP64 chains (dnrm2, the dsymv row
// sums, x·v) plus a dozen dependent scalar operations (hypot, τ, 1/s).  On
// gfx950 a dependent FP64 add costs 14 shader cycles and a workgroup barrier
// ~1 µs; the one-workgroup kernel (k_tridiag_sq) measured 0.43 ms at N = 128,
// two thirds of it per-step fixed latency (profiles/r5/eigen_trace_c2.txt).
// A host core adds in 3-4 cycles at ~5 GHz and keeps eight ordered chains in
// flight per AVX-512 instruction, so the same operations in the same order
// take tens of µs.  The device keeps every stage whose work is parallel (the
// unpack of Q, the rotation replay, the draw, the update).
//
// Operation order (pinned by oracle/refcpu.c symmtd_decomp, which reproduces
// the reference's 99 committed eigensystems bit for bit):
//   householder_transform: dnrm2 of v[1..n-1] (gslcblas scaled ssq, in
//     order), β = -sign(α)·hypot(α, ‖x‖) (fdlibm), τ = (β-α)/β, v *= 1/(α-β);
//   dsymv (RowMajor, Lower, alpha τ): x[c] = Σ_{r = n-1 .. c} (τ v_r) m_rc
//     (descending r, the diagonal last), + τ·Σ_{k<c} v_k m_ck (ascending k);
//   xv = Σ x_r v_r (ascending), α' = -(τ/2)·xv, x += α' v;
//   dsyr2 (Lower, alpha -1): m_rj += (-v_r) x_j + (-x_r) v_j.
// Vectorisation never reorders an element's operations: SIMD lanes are
// different output elements.
//
// Layout and schedule: the lower triangle only, row r at a 64-byte aligned
// offset (length rounded up to 8), so the active submatrix fits the core's
// L1 after the first steps.  Step i's dsyr2 is deferred and fused into step
// i+1's dsymv: one descending pass over rows of 8 per step reads each 8x8
// tile once, applies the pending rank-2 update, adds the tile's rows to the
// column sums x (descending r, per column) and, after an in-register
// transpose, to the eight rows' dot chains (ascending k, per row).  Only
// column i+1, which the next Householder vector needs first, is updated
// ahead of the pass.
//
// Compiled by the host compiler (g++) with -ffp-contract=off (no FMA), -O3.
// The body (kg_host_tridiag_body.inc) is compiled three times, for AVX-512F,
// AVX2 and baseline SSE2, and the widest the core supports is called
// (KORALI_AMD_HOST_TRIDIAG_ISA = avx512 | avx2 | sse2 forces one).  No
// variant uses FMA, so all three produce the same bits.
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "kg_host_tridiag.hpp"

#define KGI __attribute__((always_inline)) inline

// KG_HT_PHASES (tools/host_tridiag_phases.cpp): time-stamp counters per phase
// into kg_ht_phases[]: 0 the copy of C, 1 column i with the pending update,
// 2 dnrm2, 3 the Householder scalars and v, 4 the fused row pass, 5 x.v and w
#ifdef KG_HT_PHASES
#include <x86intrin.h>
extern unsigned long long kg_ht_phases[8];
#define KG_HT_T(v) const unsigned long long v = __rdtsc()
#define KG_HT_ACC(k, v) kg_ht_phases[k] += __rdtsc() - (v)
#else
#define KG_HT_T(v)
#define KG_HT_ACC(k, v)
#endif

namespace kg {

namespace ht_avx512 {
#pragma GCC push_options
#pragma GCC target("avx512f")
#include "kg_host_tridiag_body.inc"
#pragma GCC pop_options
}  // namespace ht_avx512

namespace ht_avx2 {
#pragma GCC push_options
#pragma GCC target("avx2")
#include "kg_host_tridiag_body.inc"
#pragma GCC pop_options
}  // namespace ht_avx2

namespace ht_sse2 {
#include "kg_host_tridiag_body.inc"
}  // namespace ht_sse2

namespace {
typedef void (*TridiagFn)(HostTridiag &, const double *, int, double *, double *, double *, double *);
TridiagFn pick_isa() {
  const char *e = std::getenv("KORALI_AMD_HOST_TRIDIAG_ISA");
  const bool has512 = __builtin_cpu_supports("avx512f"), has2 = __builtin_cpu_supports("avx2");
  if (e && !std::strcmp(e, "sse2")) return ht_sse2::tridiag_run;
  if (e && !std::strcmp(e, "avx2") && has2) return ht_avx2::tridiag_run;
  if (has512 && !(e && !std::strcmp(e, "avx2"))) return ht_avx512::tridiag_run;
  return has2 ? ht_avx2::tridiag_run : ht_sse2::tridiag_run;
}
}  // namespace

int HostTridiag::init(int N_) {
  release();
  N = N_;
  const int R = (N + 7) & ~7;  // rows incl. zero padding up to a whole block
  const int L = R + 16;
  size_t tot = 0;
  for (int r = 0; r < R; r++) tot += (size_t)((r + 8) & ~7);
  const size_t vec = (size_t)L, nvec = 8;
  mem = (double *)std::aligned_alloc(64, (tot + nvec * vec) * sizeof(double));
  row = (double **)std::malloc(sizeof(double *) * (R > 0 ? R : 1));
  if (!mem || !row) {
    release();
    return 1;
  }
  std::memset(mem, 0, (tot + nvec * vec) * sizeof(double));
  size_t off = 0;
  for (int r = 0; r < R; r++) {
    row[r] = mem + off;
    off += (size_t)((r + 8) & ~7);
  }
  double *p = mem + tot;
  v[0] = p;
  v[1] = p + vec;
  x[0] = p + 2 * vec;
  x[1] = p + 3 * vec;
  nv = p + 4 * vec;
  nx = p + 5 * vec;
  colb = p + 6 * vec;
  t1 = p + 7 * vec;
  return 0;
}

void HostTridiag::release() {
  std::free(mem);
  std::free(row);
  mem = nullptr;
  row = nullptr;
}

void HostTridiag::run(const double *C, int ldc, double *H, double *tau, double *d, double *sd) {
  if (N == 1) {
    d[0] = C[0];
    return;
  }
  static const TridiagFn fn = pick_isa();
  fn(*this, C, ldc, H, tau, d, sd);
}

}  // namespace kg
