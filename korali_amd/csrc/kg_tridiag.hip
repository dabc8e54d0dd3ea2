// kg_tridiag.hip — GSL-order Householder tridiagonalisation of one N <= 128
// symmetric matrix in ONE workgroup, built on the hand-scheduled chains of
// kg_chains.hpp.
//
// Replaces phase A of CMAES::eigen (CMAES.cpp.base:896-938 ->
// gsl_eigen_symmv -> gsl_linalg_symmtd_decomp).  The operation order is
// gslcblas's: dnrm2's scaled ssq recurrence, dsymv's
// descending column walk plus its ascending t2 walk, ddot, daxpy, dsyr2.
// Every one of those sums is a chain of dependent FP64 adds whose order is
// fixed by the bit-exactness contract, so a Householder step costs about
// three chains of length n = N-1-i; the kernel's job is to run those chains
// at the add latency and to keep everything else off the critical path:
//
//   A  wave 0: the pivot row (held in registers since the previous step)
//      is staged for dnrm2 (DPP prefix maximum, one division per element,
//      rescale flags as ballots), the ssq chain runs (kc_nrm2), then the
//      Householder scalars and v, tau v are written; waves 1-3, 5-7 meanwhile
//      apply the previous step's rank-2 update to the trailing block.
//   E  dsymv: four waves, one SIMD each — waves 0/1 the descending chains
//      of rows j < 64 / j >= 64, waves 2/3 the ascending t2 chains
//      (kc_lock_desc / kc_lock_asc, lockstep over zero-padded columns of
//      the strictly-upper storage, so no lane masks).
//   X  wave 0: x = acc + tau t2, the xv chain (kc_add), alpha, x += alpha v,
//      and the NEXT pivot row's rank-2 update straight into its registers.
//   M  waves 1-3, 5-7: rank-2 update of rows i+2.. (upper triangle + diagonal).
//
// Three workgroup barriers per step (after A, after E, after X).  Layout:
// the strictly upper triangle with row stride 130 (conflict-free row and
// column walks; 16 zero rows below the matrix absorb the ascending chains'
// read-ahead), the diagonal and all vectors padded by 16 zeros each side.
#include "kg_chains.hpp"

namespace kg {

constexpr int SQ_TPB = 512;  // 8 waves: <= 256 VGPRs each (the chains' scratch is v[192:255])
constexpr int SQ_LDA = 130;  // row stride for every N <= 128 (ds_read offsets are immediates);
                             // 130: 16-byte row reads of 64 lanes hit every bank equally
constexpr int SQ_VP = 16;    // zero padding before / after each vector (chain read-ahead)

// (even: every vector starts 16-byte aligned, for the chains' ds_read_b128 pairs)
__host__ __device__ inline size_t sq_vec(int N) { return ((size_t)N + 2 * SQ_VP + 1) & ~(size_t)1; }
__host__ __device__ inline size_t sq_lds_doubles(int N) {
  // M (N+16 rows) | dg | va[2] | tva[2] | xa | xd 128 | t2 128 | sv 160 | scal 16
  return (size_t)(N + 16) * SQ_LDA + 6 * sq_vec(N) + 128 + 128 + 160 + 16;
}
bool sq_fits(int N) { return N >= 3 && N <= 128 && sq_lds_doubles(N) * sizeof(double) <= 160 * 1024; }

__device__ __forceinline__ unsigned lds_addr(const double *p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) double *)p;
}
// a wave-uniform 64-bit value into scalar registers
__device__ __forceinline__ unsigned long long rfl64(unsigned long long x) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)x);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(x >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// hdsd / hflag (optional): the host chase's copy of d | sd, written with
// system-scope stores as the values are final (sd_i at step i, d at the
// end), then the flag = seq (what k_publish_dsd does after the kernel, one
// launch earlier on the critical path)
__device__ __forceinline__ void st_sys_d(double *p, double v) {
  __hip_atomic_store((unsigned long long *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
// kDpp: the two scalar chains (dnrm2's ssq, xv) run on register-held
// elements through DPP broadcasts (kc_nrm2_dpp / kc_add_dpp: one VALU
// instruction per element, no LDS access inside the chain); otherwise they
// stream the staged elements from LDS (kc_nrm2 / kc_add)
template <bool kDpp>
__global__ void __launch_bounds__(SQ_TPB) k_tridiag_sq(int N, const double *__restrict__ C, double *gH,
                                                       double *tauOut, double *dOut, double *sdOut,
                                                       unsigned long long *trace, double *hdsd,
                                                       unsigned long long *hflag, unsigned long long seq) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, nt = blockDim.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar control flow
  constexpr int lda = SQ_LDA;
  const int VS = (int)sq_vec(N);
  double *M = smem;  // strictly upper triangle, row r at r * lda; rows N .. N+15 zero
  double *vb = M + (size_t)(N + 16) * lda;
  double *dg = vb + SQ_VP;
  // v (v_0 = 1) and tau v by column, double-buffered across steps: buffer p
  // at vb + (1 + p) VS / vb + (3 + p) VS (plain offsets, not a pointer table,
  // so every access stays an LDS instruction)
  double *xa = vb + (size_t)5 * VS + SQ_VP;                                      // x after daxpy
  double *xd = vb + (size_t)6 * VS;  // descending chain + diagonal term, by j (rows j >= 64)
  double *t2 = xd + 128;             // ascending chains, by j
  double *sv = t2 + 128;             // 160: chain staging (dnrm2 addends, xv products)
  double *scal = sv + 160;
  const bool tr = trace && tid == 0;
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tm = tr ? __builtin_amdgcn_s_memtime() : 0;
  // (per-step phase times of the last launch at trace[32 + 8 i + k], for
  // the fixed / per-element split of every phase)
#define SQ_MARK(k)                                                \
  if (tr) {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    tacc[k] += t_ - tm;                                           \
    trace[32 + 8 * (size_t)i + (k)] = t_ - tm;                    \
    tm = t_;                                                      \
  }
  for (size_t idx = tid; idx < sq_lds_doubles(N); idx += nt) smem[idx] = 0.0;
  __syncthreads();
  // symmetrise from the lower triangle (CMAES.cpp.base:908-913); eight
  // loads in flight per thread
  for (int idx0 = tid; idx0 < N * N; idx0 += 8 * nt) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = idx0 + u * nt, r = idx / N, c = idx - r * N;
      v[u] = (idx < N * N && c >= r) ? C[(size_t)c * N + r] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = idx0 + u * nt, r = idx / N, c = idx - r * N;
      if (idx < N * N) {
        if (c > r) M[(size_t)r * lda + c] = v[u];
        else if (c == r) dg[r] = v[u];
      }
    }
  }
  __syncthreads();
  // wave 0 holds the pivot row: alpha = M[i][i+1], x_e = M[i][i+2+e] (e = lane, 64 + lane)
  double alpha = 0.0, R0 = 0.0, R1 = 0.0;
  if (wid == 0) {
    alpha = M[1];
    R0 = (2 + lane < N) ? M[2 + lane] : 0.0;
    R1 = (66 + lane < N) ? M[66 + lane] : 0.0;
  }
  for (int i = 0; i + 2 < N; i++) {
    const int n = N - i - 1, m = n - 1, par = i & 1;
    double *va = vb + (size_t)(1 + par) * VS + SQ_VP, *tva = vb + (size_t)(3 + par) * VS + SQ_VP;
    // ---- A (wave 0): dnrm2 of x, the Householder scalars, v and tau v
    if (wid == 0) {
      // zeros are skipped by dnrm2; the first nonzero element's rescale,
      // ssq = 1 + 1 (0/a)^2 = 1, is staged as the no-op addend +0.0
      const double a0 = lane < m ? fabs(R0) : 0.0;
      double pm0, pm1, carry;
      unsigned long long k0, k1 = 0;
      if (kDpp) {
        // both 64-element halves straight-line (the two quotients' division
        // sequences interleave); the chain's operands staged twice: c = t
        // (t = (a/b)^2) or 1.0 at a new running maximum, a = t (t = b/a) there
        // or 1.0 (kc_nrm2_dpp8: a half holding a rescale runs ssq = (ssq a) a + c
        // on all its elements, exact for both kinds)
        const double a1 = lane + 64 < m ? fabs(R1) : 0.0;
        wave_prefix_max2_nonneg(a0, a1, pm0, pm1);
        const double c0 = readlane_d(pm0, 63);
        const double b0 = dpp_d<0x138, 0xf>(pm0);             // running max before element lane (lane 0: 0.0)
        const double b1 = fmax(dpp_d<0x138, 0xf>(pm1), c0);  // running max before element 64 + lane
        const bool z0 = a0 != 0.0 && b0 != 0.0, n0 = z0 && b0 < a0;  // n: a new running maximum
        const bool z1 = a1 != 0.0 && b1 != 0.0, n1 = z1 && b1 < a1;
        const double q0 = (z0 ? (n0 ? b0 : a0) : 0.0) / (z0 ? (n0 ? a0 : b0) : 1.0);
        const double q1 = (z1 ? (n1 ? b1 : a1) : 0.0) / (z1 ? (n1 ? a1 : b1) : 1.0);
        k0 = __ballot(n0);
        k1 = __ballot(n1);
        sv[lane] = n0 ? 1.0 : q0 * q0;  // elements >= m: +0.0 (no-ops of the chain)
        sv[64 + lane] = n1 ? 1.0 : q1 * q1;
        t2[lane] = n0 ? q0 : 1.0;  // (t2 is free until this step's E phase)
        t2[64 + lane] = n1 ? q1 : 1.0;
        carry = fmax(c0, readlane_d(pm1, 63));
      } else if (m > 64) {  // uniform: both 64-element halves
        const double a1 = lane + 64 < m ? fabs(R1) : 0.0;
        wave_prefix_max2_nonneg(a0, a1, pm0, pm1);
        const double c0 = readlane_d(pm0, 63);
        const double b1 = fmax(dpp_d<0x138, 0xf>(pm1), c0);  // running max before element 64 + lane
        const bool z1 = a1 != 0.0 && b1 != 0.0, n1 = z1 && b1 < a1;
        const double q1 = (z1 ? (n1 ? b1 : a1) : 0.0) / (z1 ? (n1 ? a1 : b1) : 1.0);
        k1 = __ballot(n1);
        sv[64 + lane] = n1 ? q1 : q1 * q1;
        carry = fmax(c0, readlane_d(pm1, 63));
      } else {
        pm0 = wave_prefix_max_nonneg(a0);
        carry = readlane_d(pm0, 63);
      }
      if (!kDpp) {
        const double b0 = dpp_d<0x138, 0xf>(pm0);  // running max before element lane (lane 0: 0.0)
        const bool z0 = a0 != 0.0 && b0 != 0.0, n0 = z0 && b0 < a0;  // n: a new running maximum
        const double q0 = (z0 ? (n0 ? b0 : a0) : 0.0) / (z0 ? (n0 ? a0 : b0) : 1.0);
        k0 = __ballot(n0);
        sv[lane] = n0 ? q0 : q0 * q0;  // elements >= m: +0.0 (no-ops of the chain)
      }
      SQ_MARK(0)
      double ssq;
      if (kDpp) {
        double qa[8], qc[8];  // element 16 k + j in lane j of every row of q[k]
#pragma unroll
        for (int k = 0; k < 8; k++) qc[k] = sv[16 * k + (lane & 15)], qa[k] = t2[16 * k + (lane & 15)];
        ssq = chains::kc_nrm2_dpp8(1.0, qa, qc, __builtin_amdgcn_readfirstlane((unsigned)(m + 15) >> 4), k0, k1);
      } else {
        ssq = chains::kc_nrm2(1.0, lds_addr(sv), __builtin_amdgcn_readfirstlane((unsigned)(m + 15) >> 4), k0, k1);
      }
      const double xnorm = (m == 1) ? fabs(readlane_d(R0, 0)) : carry * sqrt(ssq);
      SQ_MARK(1)
      double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
      int branch = 0;
      if (xnorm != 0) {
        beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fast(alpha, xnorm);
        const double sgap = alpha - beta;
        const bool big = fabs(sgap) > DMIN;
        tau_i = (beta - alpha) / beta;
        f1 = (big ? 1.0 : EPS) / sgap;  // v[1:] *= 1/s, or EPS/s then 1/EPS (householder.c)
        f2 = big ? 1.0 : 1.0 / EPS;
        branch = big ? 1 : 2;
      }
      const double v0out = branch ? beta : alpha;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int e = lane + 64 * h;
        if (h == 1 && m <= 64) break;  // uniform
        if (e < m) {
          double t = h ? R1 : R0;
          if (branch != 0) {
            t = t * f1;
            if (branch == 2) t = t * f2;
          }
          gH[(size_t)i * N + 1 + e] = t;
          va[i + 2 + e] = t;
          tva[i + 2 + e] = tau_i * t;
        }
      }
      if (lane == 0) {
        gH[(size_t)i * N] = v0out;
        va[i] = 0.0;  // (the ascending walk may start one column early, at an even column)
        va[i + 1] = 1.0;
        tva[i + 1] = tau_i * 1.0;
        scal[0] = tau_i;
        tauOut[i] = tau_i;
        sdOut[i] = v0out;
        if (hdsd) st_sys_d(hdsd + N + i, v0out);
      }
      SQ_MARK(2)
    }
    __syncthreads();
    SQ_MARK(3)
    const double tau_i = scal[0];
    if (tau_i == 0.0) {  // no update this step (uniform): the next pivot row is current in LDS
      if (wid == 0) {
        const double *row = M + (size_t)(i + 1) * lda;
        alpha = row[i + 2];
        R0 = (i + 3 + lane < N) ? row[i + 3 + lane] : 0.0;
        R1 = (i + 67 + lane < N) ? row[i + 67 + lane] : 0.0;
      }
      continue;
    }
    // ---- E: dsymv chains (row r = i+1+j; lanes past the block walk zero row N)
    double xdj = 0.0;
    if (wid < 4) {
      const int h = wid & 1, j = lane + 64 * h;
      const bool valid = j < n;
      const int r = valid ? i + 1 + j : N;
      if (wid < 2) {
        // columns c = N-1 down to r+1 (lockstep from N-1 to i+2+64h), then the
        // diagonal term; with N odd the walk starts at the zero column N, so
        // that every pair it reads is 16-byte aligned
        const int T = n - 1 - 64 * h, top = N | 1, Tw = T + (top - (N - 1));
        const unsigned nb = __builtin_amdgcn_readfirstlane(T > 0 ? (unsigned)(Tw + 7) >> 3 : 0u);
        // (w as broadcast LDS pairs: the DPP-broadcast form kc_lock_desc_dpp measured
        // 28.5 against 23.1 cycles per element with four chain waves, profiles/r5)
        const double acc =
            chains::kc_lock_desc(0.0, lds_addr(tva + (top - 7)), lds_addr(M + (size_t)r * lda + (top - 7)), nb);
        if (valid) {
          xdj = acc + tva[r] * dg[r];
          if (h) xd[j] = xdj;
        }
      } else {
        // columns c = i+1 up to r-1 (lockstep up to the wave's largest row);
        // from the even column c0 (c0 = i: v_i = 0 this step, a +-0 no-op
        // product), so that every w pair is 16-byte aligned
        const int T = (64 * h < n) ? min(n, 64 * h + 64) - 1 : 0, c0 = (i + 1) & ~1, Tw = T + (i + 1 - c0);
        const unsigned nb = __builtin_amdgcn_readfirstlane(T > 0 ? (unsigned)(Tw + 7) >> 3 : 0u);
        const double acc =
            chains::kc_lock_asc<SQ_LDA * 8>(0.0, lds_addr(va + c0), lds_addr(M + (size_t)c0 * lda + r), nb);
        if (valid) t2[j] = acc;
      }
    }
    SQ_MARK(4)
    __syncthreads();
    SQ_MARK(5)
    // ---- X (wave 0): x = acc + tau t2, xv, alpha = -(tau/2) xv, x += alpha v,
    // and the next pivot row (i+1) with this step's rank-2 update
    if (wid == 0) {
      const int r1 = i + 1;
      const double *row1 = M + (size_t)r1 * lda;
      // operands of the next pivot row that do not depend on x (read early)
      const int ca = i + 3 + lane, cb = i + 67 + lane;
      const double ma = ca < N ? row1[ca] : 0.0, mb = cb < N ? row1[cb] : 0.0, malpha = row1[i + 2];
      const double vca = va[ca], vcb = va[cb], valpha = va[i + 2], dgr1 = dg[r1];
      const bool two = n > 64;  // uniform: a second 64-row half
      double x0 = 0.0, x1 = 0.0, v0 = 0.0, v1 = 0.0;
      if (lane < n) {
        x0 = xdj + tau_i * t2[lane];
        v0 = va[r1 + lane];
      }
      sv[lane] = x0 * v0;  // +0.0 past the block
      if (two) {
        if (lane + 64 < n) {
          x1 = xd[64 + lane] + tau_i * t2[64 + lane];
          v1 = va[r1 + 64 + lane];
        }
        sv[64 + lane] = x1 * v1;
      }
      double xv;
      if (kDpp) {
        double q[8];
#pragma unroll
        for (int k = 0; k < 8; k++) q[k] = sv[16 * k + (lane & 15)];
        xv = chains::kc_add_dpp(0.0, q, __builtin_amdgcn_readfirstlane((unsigned)(n + 15) >> 4));
      } else {
        xv = chains::kc_add(0.0, lds_addr(sv), __builtin_amdgcn_readfirstlane((unsigned)(n + 15) >> 4));
      }
      const double als = -(tau_i / 2.0) * xv;
      const double xf0 = x0 + als * v0, xf1 = x1 + als * v1;  // (+0.0 past the block)
      if (lane < n) xa[r1 + lane] = xf0;  // (for the M phase's waves)
      if (two && lane + 64 < n) xa[r1 + 64 + lane] = xf1;
      // dsyr2 (alpha = -1) on row r1: m += (-v_r1) x_c + (-x_r1) v_c, v_r1 = 1;
      // x_c of the columns c = i+3+lane (+64) from the registers two lanes up
      // (DPP wave shifts), not through LDS
      const double xr1 = readlane_d(xf0, 0), xf1_0 = readlane_d(xf1, 0), xf1_1 = readlane_d(xf1, 1);
      const double xs0 = dpp_d<0x130, 0xf>(dpp_d<0x130, 0xf>(xf0));  // wave_shl:1 twice: x_(lane+2)
      const double xs1 = dpp_d<0x130, 0xf>(dpp_d<0x130, 0xf>(xf1));
      const double xc0 = lane == 62 ? xf1_0 : (lane == 63 ? xf1_1 : xs0);
      const double nvr = -1.0 * 1.0, nxr = -1.0 * xr1;
      alpha = malpha + (nvr * readlane_d(xf0, 1) + nxr * valpha);
      R0 = ca < N ? ma + (nvr * xc0 + nxr * vca) : 0.0;
      R1 = (n > 65 && cb < N) ? mb + (nvr * xs1 + nxr * vcb) : 0.0;  // (next step's x_e, e >= 64)
      if (lane == 0) dg[r1] = dgr1 + (nvr * xr1 + nxr * 1.0);
    }
    SQ_MARK(6)
    __syncthreads();
    SQ_MARK(7)
    // ---- M (waves 1-3, 5-7; wave 4 shares wave 0's SIMD and stays idle):
    // rank-2 update of rows i+2.. (upper triangle) and their diagonal
    if (wid != 0 && wid != 4) {
      const int wk = wid < 4 ? wid - 1 : wid - 2;  // 0..5
      // lane = columns c0, c0 + 64 (fixed), rows r = i+2+wk, +6, ...: the
      // next row's operands are loaded while the current row is updated
      // (a lane whose column is on/below the diagonal or past N stores into
      // a dump slot instead of being masked off, no exec-mask branches: row
      // i, which nothing reads after this step's A phase)
      const int c0 = i + 3 + lane, c1 = c0 + 64;
      const double xc0 = xa[c0], vc0 = va[c0], xc1 = xa[c1], vc1 = va[c1];
      const unsigned dump0 = lds_addr(M + (size_t)i * lda + lane), dump1 = dump0 + 64 * 8;
      const int r0 = i + 2 + wk;
      if (r0 < N) {
        const double *vr = va + r0, *xr = xa + r0;
        double *row = M + (size_t)r0 * lda;
        // operands of row r + 6 are loaded before row r is stored (raw: the
        // negations happen at use, so no load is waited for in its own iteration)
        double v_ = vr[0], x_ = xr[0], m0 = row[c0], m1 = row[c1];
#pragma unroll 2
        for (int r = r0; r < N; r += 6) {
          vr += 6, xr += 6;
          double *rown = row + 6 * lda;  // (rows up to N+5 exist: the zero rows)
          const double vn = vr[0], xn = xr[0], m0n = rown[c0], m1n = rown[c1];
          const double nv = -1.0 * v_, nx = -1.0 * x_;
          const unsigned a0 = (c0 > r && c0 < N) ? lds_addr(row + c0) : dump0;
          const unsigned a1 = (c1 > r && c1 < N) ? lds_addr(row + c1) : dump1;
          *(__attribute__((address_space(3))) double *)(size_t)a0 = m0 + (nv * xc0 + nx * vc0);
          *(__attribute__((address_space(3))) double *)(size_t)a1 = m1 + (nv * xc1 + nx * vc1);
          v_ = vn, x_ = xn, m0 = m0n, m1 = m1n, row = rown;
        }
      }
      const int qd = wk * 64 + lane;
      if (qd < n - 1) {
        const int r = i + 2 + qd;
        const double nvr = -1.0 * va[r], nxr = -1.0 * xa[r];
        dg[r] += nvr * xa[r] + nxr * va[r];
      }
    }
  }
  __syncthreads();
#undef SQ_MARK
  if (tr)
    for (int k = 0; k < 8; k++) trace[8 + k] += tacc[k];
  for (int r = tid; r < N; r += nt) {
    dOut[r] = dg[r];
    if (hdsd) st_sys_d(hdsd + r, dg[r]);
  }
  if (tid == 0) {
    sdOut[N - 2] = alpha;
    if (hdsd) {
      st_sys_d(hdsd + N + (N - 2), alpha);
      st_sys_d(hdsd + N + (N - 1), 0.0);  // (never read by the chase)
    }
  }
  if (hdsd) {
    __syncthreads();
    if (tid == 0) {
      __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: the values before the flag
      __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ------------------------------------------------------------------------
// Phase A for 128 < N (the matrix no longer fits one CU's LDS): rows spread
// over the workgroups (row r on workgroup r % P, full symmetric rows in LDS
// so both dsymv chains of a row are local to its owner), ONE in-launch
// hand-off per Householder step (every owner publishes its x_r, every
// workgroup gathers x; the next pivot row is published one step ahead by its
// owner), everything else of the step recomputed redundantly by every
// workgroup with identical operands.  Compared with k_tridiag_mw (same
// decomposition) the step's chains run on the kg_chains.hpp primitives:
//   dnrm2: staged by all eight waves (64-element chunks, DPP prefix maxima,
//          chunk maxima exchanged through LDS), the ssq chain on wave 0
//          (kc_nrm2, 128 elements per call);
//   dsymv: products staged zero-padded per row (descending and ascending
//          arrays), one wave per chain (kc_add_desc / kc_add);
//   xv:    kc_add over the staged products;
//   x += alpha v is not stored: the rank-2 update recomputes x_f = x + alpha v
//          per operand (the same rounded value every time).
constexpr int MW2_TPB = 512;
constexpr int MW2_PAD = 32;  // zero padding on each side of a staged product row
__host__ __device__ inline size_t mw2_ps(int N) { return (size_t)N + 2 * MW2_PAD; }
__host__ __device__ inline size_t mw2_lds_doubles(int N, int RW) {
  // M | Pd | Pa | prow (+16) | nrow | vloc | tv | xl | sv (+64) | scal, accb, t2b, mskb, cmx (16 each) | sa (+64)
  return (size_t)RW * (N + 1) + 2 * (size_t)RW * mw2_ps(N) + (N + 16) + 4 * (size_t)N + (N + 64) + 5 * 16 + (N + 64);
}
// rows per workgroup chosen at init for the device's co-resident capacity, by N
// (0: the default); every handle of one N on this device arrives at the same value
static int g_mw2_rw[1025];
int mw2_rows(int N) {
  int rw = (N <= 1024 && g_mw2_rw[N] > 0) ? g_mw2_rw[N] : (N + 255) / 256;
  if (const char *e = getenv("KORALI_AMD_TMW_ROWS")) rw = atoi(e);
  if (rw < 1) rw = 1;
  while (rw > 1 && mw2_lds_doubles(N, rw) * sizeof(double) > 150 * 1024) rw--;
  return rw;
}
int mw2_groups(int N) { return (N + mw2_rows(N) - 1) / mw2_rows(N); }
size_t mw2_lds_bytes(int N) { return mw2_lds_doubles(N, mw2_rows(N)) * sizeof(double); }
bool mw2_fits(int N) { return N > 16 && N <= 1024 && mw2_lds_doubles(N, mw2_rows(N)) * sizeof(double) <= 150 * 1024; }

// kDpp: the ssq and xv chains on register-held elements (kc_nrm2_dpp /
// kc_add_dpp, 128 elements per call), as k_tridiag_sq<true>
template <bool kDpp>
__global__ void __launch_bounds__(MW2_TPB) k_tridiag_mw2(int N, const double *__restrict__ C, double *gH,
                                                         double *tauOut, double *dOut, double *sdOut,
                                                         unsigned long long *comm, unsigned int *errors,
                                                         unsigned long long *trace) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, nt = blockDim.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar control flow
  const int P = gridDim.x, g = blockIdx.x, RW = (N + P - 1) / P, lda = N + 1, PS = (int)mw2_ps(N);
  double *M = smem;                            // local row k = global row g + k P
  double *Pd = M + (size_t)RW * lda + MW2_PAD;  // descending products of local row k at Pd + k PS, by column
  double *Pa = Pd + (size_t)RW * PS;            // ascending products
  double *prow = Pa - MW2_PAD + (size_t)RW * PS;  // current pivot row, by column
  double *nrow = prow + N + 16;                 // next pivot row as published
  double *vloc = nrow + N;                      // v (v_0 = 1), by offset q = c - i - 1
  double *tv = vloc + N;                        // tau v
  double *xl = tv + N;                          // x (before daxpy)
  double *sv = xl + N;                          // chain staging (N + 64)
  double *scal = sv + N + 64;
  double *accb = scal + 16, *t2b = accb + 16;
  unsigned long long *mskb = (unsigned long long *)(t2b + 16);
  double *cmx = (double *)(mskb + 16);
  double *sa = cmx + 16;  // kDpp: the ssq chain's second operand (kc_nrm2_dpp8)
  unsigned long long *gx = comm, *grow = comm + 2 * (size_t)N * N, *abortw = comm + 4 * (size_t)N * N;
  const int writer = (N - 1) % P;  // owns row N-1: runs every step, writes the per-step outputs

  for (size_t idx = tid; idx < mw2_lds_doubles(N, RW); idx += nt) smem[idx] = 0.0;
  __syncthreads();
  for (int idx = tid; idx < RW * N; idx += nt) {
    const int k = idx / N, c = idx % N, r = g + k * P;
    if (r < N) M[(size_t)k * lda + c] = (c <= r) ? C[(size_t)r * N + c] : C[(size_t)c * N + r];
  }
  for (int c = tid; c < N; c += nt) {
    prow[c] = C[(size_t)c * N];                        // row 0 (symmetrised: column 0)
    nrow[c] = (c >= 1) ? C[(size_t)c * N + 1] : C[1];  // row 1 before any update
  }
  const int maxRow = g + ((N - 1 - g) / P) * P;  // largest row owned
  const bool tr = trace && g == writer && tid == 0;
  unsigned long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tm = tr ? __builtin_amdgcn_s_memtime() : 0;
#define MW2_MARK(k)                                               \
  if (tr) {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    tacc[k] += t_ - tm;                                           \
    tm = t_;                                                      \
  }
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    if (maxRow < i) break;  // no active rows left (never the writer)
    const int n = N - i - 1, m = n - 1;
    const unsigned tag = (unsigned)i + 1u;
    unsigned long long *gxp = gx + (size_t)i * 2 * N, *growp = grow + (size_t)i * 2 * N;
    // owner of row i+1 publishes it (state after step i-1) for step i's end
    if (i >= 1 && i + 4 <= N && (i + 1) % P == g) {
      const double *row = M + (size_t)((i + 1) / P) * lda;
      for (int c = i + 2 + tid; c < N; c += nt) put_granule_dbl(growp + 2 * c, tag, row[c]);
    }
    // ---- dnrm2 staging of x_e = prow[i+2+e], e < m, over 64-element chunks:
    // chunk k on wave k % 8; chunk maxima through LDS; elements up to the
    // next multiple of 16 past m staged as +0.0
    const int nch = (m + 63) >> 6;
    double pmk[2], ak[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int k = wid + 8 * u, e = 64 * k + lane;
      ak[u] = (k < nch && e < m) ? fabs(prow[i + 2 + e]) : 0.0;
      pmk[u] = wave_prefix_max_nonneg(ak[u]);
      if (k < nch && lane == 63) cmx[k] = pmk[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int k = wid + 8 * u;
      if (k < nch) {  // uniform
        double carry = 0.0;
        for (int k2 = 0; k2 < k; k2++) carry = fmax(carry, cmx[k2]);
        const double a = ak[u], b = fmax(dpp_d<0x138, 0xf>(pmk[u]), carry);
        const bool z = a != 0.0 && b != 0.0, nf = z && b < a;  // (first nonzero: no-op +0.0)
        const double qv = (z ? (nf ? b : a) : 0.0) / (z ? (nf ? a : b) : 1.0);
        const unsigned long long bm = __ballot(nf);
        if (kDpp) {  // c = t or 1.0 at a new running maximum, a = t there or 1.0 (as k_tridiag_sq)
          sv[64 * k + lane] = nf ? 1.0 : qv * qv;
          sa[64 * k + lane] = nf ? qv : 1.0;
        } else {
          sv[64 * k + lane] = nf ? qv : qv * qv;
        }
        if (lane == 0) mskb[k] = bm;
      }
    }
    MW2_MARK(0)
    __syncthreads();
    MW2_MARK(1)
    // ---- wave 0: the ssq chain and the Householder scalars (every lane)
    if (wid == 0) {
      double scale = 0.0;
      for (int k = 0; k < nch; k++) scale = fmax(scale, cmx[k]);
      double ssq = 1.0;
      const int G = (m + 15) >> 4;
      for (int b = 0; 8 * b < G; b++) {
        const unsigned gb = __builtin_amdgcn_readfirstlane((unsigned)min(8, G - 8 * b));
        const unsigned long long k0 = mskb[2 * b], k1 = (2 * b + 1 < nch) ? mskb[2 * b + 1] : 0ULL;
        if (kDpp) {
          double qa[8], qc[8];
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const int e = min(128 * b + 16 * k + (lane & 15), N + 63);  // (past 16 gb: unused)
            qc[k] = sv[e];
            qa[k] = sa[e];
          }
          ssq = chains::kc_nrm2_dpp8(ssq, qa, qc, gb, rfl64(k0), rfl64(k1));
        } else {
          ssq = chains::kc_nrm2(ssq, lds_addr(sv + 128 * b), gb, rfl64(k0), rfl64(k1));
        }
      }
      const double alpha = prow[i + 1];
      const double xnorm = (m == 1) ? fabs(prow[i + 2]) : scale * sqrt(ssq);
      MW2_MARK(2)
      double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
      int branch = 0;
      if (xnorm != 0) {
        beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fast(alpha, xnorm);
        const double sgap = alpha - beta;
        const bool big = fabs(sgap) > DMIN;
        tau_i = (beta - alpha) / beta;
        f1 = (big ? 1.0 : EPS) / sgap;
        f2 = big ? 1.0 : 1.0 / EPS;
        branch = big ? 1 : 2;
      }
      if (lane == 0) {
        scal[0] = tau_i;
        scal[1] = f1;
        scal[2] = f2;
        scal[3] = branch ? beta : alpha;  // v_0 after householder_transform
        scal[4] = (double)branch;
        if (g == writer) {
          tauOut[i] = tau_i;
          sdOut[i] = scal[3];
        }
      }
    }
    __syncthreads();
    MW2_MARK(3)
    const double tau_i = scal[0];
    const int branch = (int)scal[4];
    const double f1 = scal[1], f2 = scal[2];
    // v and tau v (q = c - i - 1); with tau != 0 also the dsymv products of
    // the owned rows, v recomputed inline (the same rounded values)
    for (int q = tid; q < n; q += nt) {
      double t = prow[i + 1 + q];
      if (q > 0 && branch != 0) {
        t = t * f1;
        if (branch == 2) t = t * f2;
      }
      if (g == writer) gH[(size_t)i * N + q] = (q == 0) ? scal[3] : t;
      vloc[q] = (q == 0) ? 1.0 : t;
      tv[q] = tau_i * ((q == 0) ? 1.0 : t);
    }
    if (tau_i != 0.0) {
      // Pd[k][c] = tau v_c m[r][c] for c > r, Pa[k][c] = v_c m[r][c] for i < c < r, +0.0 elsewhere
      // in [i-14, N+16) (the chains' zero padding)
      const int c0 = i - 14, span = N + 16 - c0;
      for (int k = 0; k < RW; k++) {
        const int r = g + k * P;
        if (r <= i || r >= N) continue;  // uniform
        const double *mr = M + (size_t)k * lda;
        double *pd = Pd + (size_t)k * PS, *pa = Pa + (size_t)k * PS;
        for (int o = tid; o < span; o += nt) {
          const int c = c0 + o;
          double dv = 0.0, av = 0.0;
          if (c > i && c < N) {
            double t = prow[c];  // v_q, q = c - i - 1 (recomputed as above)
            if (c > i + 1 && branch != 0) {
              t = t * f1;
              if (branch == 2) t = t * f2;
            }
            if (c == i + 1) t = 1.0;
            const double mv = mr[c];
            if (c > r) dv = (tau_i * t) * mv;
            else if (c < r) av = t * mv;
          }
          pd[c] = dv;
          pa[c] = av;
        }
      }
    }
    __syncthreads();
    MW2_MARK(4)
    if (tau_i != 0.0) {
      // ---- dsymv chains: one wave per chain (descending / ascending of each owned row)
      for (int ch = wid; ch < 2 * RW; ch += 8) {
        const int k = ch < RW ? ch : ch - RW, r = g + k * P;
        if (r <= i || r >= N) continue;  // uniform
        if (ch < RW) {
          // columns c = N-1 down to r+1, then the diagonal term
          const unsigned G = __builtin_amdgcn_readfirstlane((unsigned)(N - 1 - r + 15) >> 4);
          double acc = 0.0;
          if (kDpp) {
            // 128 staged products per block into registers (element e = column
            // N-1-e in lane e % 16 of q[e / 16 % 8]), then the DPP chain
            const double *pd = Pd + (size_t)k * PS;
            for (unsigned b = 0; 8 * b < G; b++) {
              double q[8];
#pragma unroll
              for (int kk = 0; kk < 8; kk++) q[kk] = pd[max(N - 1 - (int)(128 * b) - 16 * kk - (lane & 15), -MW2_PAD)];
              acc = chains::kc_add_dpp(acc, q, __builtin_amdgcn_readfirstlane(min(8u, G - 8 * b)));
            }
          } else {
            acc = chains::kc_add_desc(0.0, lds_addr(Pd + (size_t)k * PS + (N - 16)), G);
          }
          if (lane == 0) accb[k] = acc + tv[r - i - 1] * M[(size_t)k * lda + r];
        } else {
          // columns c = i+1 up to r-1
          const unsigned G = __builtin_amdgcn_readfirstlane((unsigned)(r - i - 1 + 15) >> 4);
          double acc = 0.0;
          if (kDpp) {
            const double *pa = Pa + (size_t)k * PS;
            for (unsigned b = 0; 8 * b < G; b++) {
              double q[8];
#pragma unroll
              for (int kk = 0; kk < 8; kk++) q[kk] = pa[min(i + 1 + (int)(128 * b) + 16 * kk + (lane & 15), N + MW2_PAD - 1)];
              acc = chains::kc_add_dpp(acc, q, __builtin_amdgcn_readfirstlane(min(8u, G - 8 * b)));
            }
          } else {
            acc = chains::kc_add(0.0, lds_addr(Pa + (size_t)k * PS + (i + 1)), G);
          }
          if (lane == 0) t2b[k] = acc;
        }
      }
      __syncthreads();
      if (tid < RW) {
        const int r = g + tid * P;
        if (r > i && r < N) put_granule_dbl(gxp + 2 * (r - i - 1), tag, accb[tid] + tau_i * t2b[tid]);
      }
      MW2_MARK(5)
      {
        // x of this step and, in the same sweep, the next pivot row as published
        const int nb = (i >= 1 && i + 3 < N) ? n - 1 : 0;
        const bool ok = poll_granule_dbls(gxp, n, xl, growp + 2 * (i + 2), nb, nrow + i + 2, tag, abortw, errors);
        if (__syncthreads_or(!ok)) return;
      }
      MW2_MARK(6)
      // ---- xv = sum x_q v_q (ordered chain over staged products); alpha = -(tau/2) xv
      for (int q = tid; q < n + 16; q += nt) sv[q] = q < n ? xl[q] * vloc[q] : 0.0;
      __syncthreads();
      if (wid == 0) {
        const unsigned G = __builtin_amdgcn_readfirstlane((unsigned)(n + 15) >> 4);
        double xv = 0.0;
        if (kDpp) {
          for (unsigned b = 0; 8 * b < G; b++) {
            double q[8];
#pragma unroll
            for (int k = 0; k < 8; k++) q[k] = sv[min((int)(128 * b) + 16 * k + (lane & 15), N + 63)];
            xv = chains::kc_add_dpp(xv, q, __builtin_amdgcn_readfirstlane(min(8u, G - 8 * b)));
          }
        } else {
          xv = chains::kc_add(0.0, lds_addr(sv), G);
        }
        if (lane == 0) scal[5] = -(tau_i / 2.0) * xv;
      }
      __syncthreads();
      MW2_MARK(7)
    }
    const double als = scal[5];
    // x_f(q) = x_q + alpha v_q (gsl_blas_daxpy), recomputed per use
    auto xf = [&](int q) { return xl[q] + als * vloc[q]; };
    // ---- next pivot row (i+1): as published (or from C at i = 0), plus this step's rank-2 update
    if (i + 3 < N) {
      if (i >= 1 && tau_i == 0.0) {  // (with tau != 0 it came with x)
        const bool ok = poll_granule_dbls(growp + 2 * (i + 2), n - 1, nrow + i + 2, growp, 0, nrow, tag, abortw,
                                          errors);
        if (__syncthreads_or(!ok)) return;
      }
      MW2_MARK(8)
      const double x0f = (tau_i != 0.0) ? xf(0) : 0.0;
      for (int c = i + 2 + tid; c < N; c += nt) {
        double t = nrow[c];
        if (tau_i != 0.0) {
          const int a = c - i - 1;
          const double tmp1 = -1.0 * vloc[a], tmp2 = -1.0 * xf(a);
          t += tmp1 * x0f + tmp2 * vloc[0];
        }
        prow[c] = t;
      }
    }
    // ---- dsyr2 (alpha = -1) on the owned active rows, both triangles
    if (tau_i != 0.0)
      for (int k = 0; k < RW; k++) {
        const int r = g + k * P;
        if (r <= i || r >= N) continue;  // uniform
        const int jr = r - i - 1;
        double *row = M + (size_t)k * lda + i + 1;
        const double vr = vloc[jr], xr = xf(jr);
        for (int jj = tid; jj < n; jj += nt) {
          const bool up = jr > jj;  // (a, b) = (max, min)
          const double va_ = up ? vr : vloc[jj], xa_ = up ? xr : xf(jj);
          const double vb_ = up ? vloc[jj] : vr, xb_ = up ? xf(jj) : xr;
          const double tmp1 = -1.0 * va_, tmp2 = -1.0 * xa_;
          row[jj] += tmp1 * xb_ + tmp2 * vb_;
        }
      }
    __syncthreads();
    MW2_MARK(9)
  }
#undef MW2_MARK
  if (tr)
    for (int k = 0; k < 10; k++) trace[16 + k] += tacc[k];
  for (int k = tid; k < RW; k += nt) {
    const int r = g + k * P;
    if (r < N) {
      dOut[r] = M[(size_t)k * lda + r];
      if (r == N - 2) sdOut[r] = M[(size_t)k * lda + r + 1];
    }
  }
}

}  // namespace kg
