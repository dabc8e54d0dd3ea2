// kg_cmaes.hip — CMA-ES generation on the MI355X (CMAES.cpp.base, see
// include/korali_amd.h for the per-entry-point reference map).
//
// HBM layout per handle (all FP64, row-major as the reference's vectors):
//   X   λ x N   sample population        Z   (λ+R) x N  polar normals
//   C,B N x N   covariance / eigenvectors D,mean,prevMean,pc,ps  N
//   F   λ       fitness                  idx λ  sorting index (uint32)
//   w   μ       recombination weights    sc  scalar block (σ, counters, ...)
// One HIP stream per handle; a generation is a fixed kernel sequence with no
// host synchronisation (device-side error flags are read at sync points).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/korali_amd.h"
#include "kg_common.hpp"
#include "kg_chains.hpp"
#include "kg_eigen.hpp"
#include "kg_rng.hpp"
#include <chrono>

namespace kg {


struct CmaesScalars {
  double sigma, trace, effectiveMu, cumulativeCovariance, sigmaCumulationFactor, dampFactor, chiSquareNumber;
  double psNorm, bestEverValue, previousBestEverValue, previousBestValue, currentBestValue;
  double currentMinStd, currentMaxStd, maxDiagC, minDiagC, minEig, maxEig;
  double infeasibleSampleCount, bestValidSample, modelEvaluationCount, hsig, eigenFailures;
  double ccov1, ccovmu;
  unsigned int errors, bestFlag;  // bestFlag: best-ever improved this generation
  unsigned int rmuOutOfRange;     // k_rankmu_prep: some rank-mu factor outside the Markstein range
  // discrete variables (CMAES.cpp.base:34, :106-107, :834-859)
  double nME, nDM, chiDM;  // Number Masking Matrix Entries, Number Of Discrete Mutations, Chi Square Number DM
  // CCMA-ES (CMAES.cpp.base:147, :724-731, :812-819)
  double gsr;              // Global Success Rate
  double resampledCount;   // Resampled Parameter Count (handleConstraints' redraws)
  // hsig's (1 - c_sigma)^(2 (1 + gen)) (:656), correctly rounded, formed by
  // k_sigma one generation ahead in a spare wave (the double-double pow is
  // ~5 us of one lane); valid for generation hsigPowGen and c_sigma hsigPowCs
  double hsigPow, hsigPowCs, hsigPowGen;
};

__device__ inline double hsig_pow(const CmaesScalars *sc, double cs, unsigned long long gen) {
  if (sc->hsigPowGen == (double)gen && sc->hsigPowCs == cs) return sc->hsigPow;
  return pow_cr(1. - cs, 2.0 * (1.0 + (double)gen));
}

// Bound on |z| of a GSL polar normal: z = y sqrt(-2 ln r2 / r2) with |y| <=
// sqrt(r2) and r2 >= 2^-62 (x, y are multiples of 2^-31), so |z| <=
// sqrt(124 ln 2) = 9.27.  A draw x = m + sigma B (D o z) then satisfies |x_d|
// <= |m|_inf + sigma * ZMAX * N * max D (|B_de| <= 1), which kg_cmaes_sample
// compares with DBL_MAX before taking the no-redraw path.
constexpr double KG_DRAW_ZMAX = 10.0;
constexpr double KG_DRAW_GUARD_LIMIT = 1e300;

// ----------------------------------------------------------------- init
// setInitialConfiguration (CMAES.cpp.base:14-184), initMuWeights (:233-284),
// initCovariance (:286-313); initial values/stds resolved on the host.
// full = 0: only initMuWeights + initCovariance, as checkMeanAndSetRegime
// does on leaving CCMA-ES's viability regime (:341-345; initCovariance sets
// the diagonals of C and B and keeps their other entries, as written);
// constrained: the constrained sigma cumulation factor (:270-273)
__global__ void __launch_bounds__(256) k_init(int N, int lam, int mu, int muType, double initialSigmaCumulationFactor,
                                              double initialDampFactor, double initialCumulativeCovariance,
                                              const double *__restrict__ iv, const double *__restrict__ istd,
                                              double *w, double *C, double *B, double *D, double *mean,
                                              double *prevMean, double *pc, double *ps, CmaesScalars *sc, int full,
                                              int constrained) {
  __shared__ double s1s2[2];
  const int tid = threadIdx.x;
  for (int i = tid; i < mu; i += blockDim.x) {
    double v;
    if (muType == KG_MU_LINEAR)
      v = (double)(mu - i);
    else if (muType == KG_MU_EQUAL || muType == KG_MU_PROPORTIONAL)
      v = 1.;
    else {
      const double a = (double)mu, b = 0.5 * (double)lam;
      v = log_cr((a > b ? a : b) + 0.5) - log_cr(i + 1.);
    }
    w[i] = v;
  }
  if (full) {
    for (int i = tid; i < N * N; i += blockDim.x) {
      C[i] = 0.0;
      B[i] = 0.0;
    }
    for (int i = tid; i < N; i += blockDim.x) {
      pc[i] = 0.0;
      ps[i] = 0.0;
      mean[i] = iv[i];
      prevMean[i] = iv[i];
    }
  }
  __syncthreads();
  if (tid == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < mu; i++) {
      s1 += w[i];
      s2 += w[i] * w[i];
    }
    s1s2[0] = s1;
    s1s2[1] = s2;
  }
  __syncthreads();
  for (int i = tid; i < mu; i += blockDim.x) w[i] /= s1s2[0];
  if (tid == 0) {
    const double Nd = (double)N;
    if (full) {
      sc->bestEverValue = -INFINITY;
      sc->previousBestEverValue = sc->bestEverValue;
      sc->previousBestValue = sc->bestEverValue;
      sc->currentBestValue = sc->bestEverValue;
      sc->chiSquareNumber = sqrt(Nd) * (1. - 1. / (4. * N) + 1. / (21. * N * N));
      sc->chiDM = sqrt(Nd) * (1. - 1. / (4. * N) + 1. / (21. * N * N));  // :34
      sc->nME = 0.0;
      sc->nDM = 0.0;
      sc->bestValidSample = constrained ? -1.0 : 0.0;
      sc->gsr = constrained ? 0.5 : -1.0;
      sc->resampledCount = 0.0;
    }
    const double effMu = s1s2[0] * s1s2[0] / s1s2[1];
    sc->effectiveMu = effMu;
    if ((initialCumulativeCovariance <= 0) || (initialCumulativeCovariance > 1))
      sc->cumulativeCovariance = (4.0 + effMu / (1.0 * N)) / (N + 4.0 + 2.0 * effMu / (1.0 * N));
    else
      sc->cumulativeCovariance = initialCumulativeCovariance;
    double cs = initialSigmaCumulationFactor;
    if (cs <= 0 || cs >= 1)
      cs = constrained ? sqrt(effMu) / (sqrt(effMu) + sqrt(Nd)) : (effMu + 2.0) / (N + effMu + 3.0);
    sc->sigmaCumulationFactor = cs;
    double ds = initialDampFactor;
    if (ds <= 0.0) {
      const double t = sqrt((effMu - 1.0) / (N + 1.0)) - 1;
      ds = (1.0 + 2 * (0.0 > t ? 0.0 : t)) + cs;
    }
    sc->dampFactor = ds;
    // initCovariance
    double trace = 0.0;
    for (int i = 0; i < N; ++i) trace += istd[i] * istd[i];
    sc->trace = trace;
    sc->sigma = sqrt(trace / N);
    for (int i = 0; i < N; ++i) {
      B[i * N + i] = 1.0;
      double v = istd[i] * sqrt(N / trace);
      D[i] = v;
      C[i * N + i] = v * v;
    }
    double mn = D[0], mx = D[0];
    for (int i = 1; i < N; i++) {
      if (D[i] < mn) mn = D[i];
      if (D[i] > mx) mx = D[i];
    }
    sc->minEig = mn * mn;
    sc->maxEig = mx * mx;
    double maxd = C[0], mind = C[0];
    for (int i = 1; i < N; ++i)
      if (maxd < C[i * N + i]) maxd = C[i * N + i];
    for (int i = 1; i < N; ++i)
      if (mind > C[i * N + i]) mind = C[i * N + i];
    sc->maxDiagC = maxd;
    sc->minDiagC = mind;
    if (full) {
      sc->infeasibleSampleCount = 0;
      sc->psNorm = 0.0;
      sc->currentMinStd = INFINITY;
      sc->currentMaxStd = -INFINITY;
      sc->hsigPowGen = -1.0;
    }
  }
}

// ------------------------------------------------------------ transform
// sampleSingle (CMAES.cpp.base:494-545): x = m + σ B (D∘z), the B·aux sum in
// the reference's order (e = 0..N-1 from 0.0, separate multiply and add);
// isSampleFeasible (optimizer.cpp.base:5-14) folded into the epilogue.
constexpr int TR_BK = 32, TR_XCD = 8;
// Tiles of BM rows x BN columns, (BM/8) x (BN/32) outputs per thread (rows
// ty PR + p, columns tx PC + q), K in chunks of TR_BK staged through LDS; the
// next chunk's global loads are issued into registers before the current
// chunk is summed, so their latency hides behind it.  XCD-aware order: the
// hardware deals workgroup b to XCD b % 8, so the column tiles of one row
// tile go to consecutive workgroups of ONE XCD — its Z rows come from HBM
// once and from that XCD's L2 for the other column tiles (row-major order
// sends each column tile of a row tile to a different XCD and fetches the
// row tile N / BN times).  The grid is padded to whole groups of 8 row
// tiles; surplus workgroups exit.
template <int BM, int BN>
inline unsigned tr_grid(int rows, int N) {
  const int nbm = (rows + BM - 1) / BM, nbn = (N + BN - 1) / BN;
  return (unsigned)(((nbm + TR_XCD - 1) / TR_XCD) * TR_XCD * nbn);
}
template <int BM, int BN>
__global__ void __launch_bounds__(256) k_transform(int N, int rows, int diagonal, const double *__restrict__ Z,
                                                   const double *__restrict__ B, const double *__restrict__ D,
                                                   const double *__restrict__ mean, CmaesScalars *__restrict__ sc,
                                                   const double *__restrict__ lb, const double *__restrict__ ub,
                                                   double *__restrict__ X, double *__restrict__ BDZ,
                                                   int *__restrict__ infeas, int no_reserve, int mirrored) {
  constexpr int PR = BM / 8, PC = BN / 32, ZL = BM * TR_BK / 256, BL = BN * TR_BK / 256;
  // rows padded by 2 doubles: 16-B aligned, so a thread's PR contiguous rows
  // and PC contiguous columns come in 16-B reads (ds_read_b128: 256 B per
  // LDS clock, where the paired ds_read2_b64 moves 128)
  __shared__ __attribute__((aligned(16))) double Za[TR_BK][BM + 2];
  __shared__ __attribute__((aligned(16))) double Bt[TR_BK][BN + 2];
  const int tid = threadIdx.x;
  const int nbn = (N + BN - 1) / BN;
  const int xcd = blockIdx.x % TR_XCD, j = blockIdx.x / TR_XCD;
  const int rt = (j / nbn) * TR_XCD + xcd, ct = j % nbn;
  const int i0 = rt * BM, d0 = ct * BN;
  if (i0 >= rows) return;
  const int tx = tid & 31, ty = tid >> 5;
  const double sigma = sc->sigma;
  double acc[PR][PC];
#pragma unroll
  for (int p = 0; p < PR; p++)
#pragma unroll
    for (int q = 0; q < PC; q++) acc[p][q] = 0.0;
  if (!diagonal) {
    double zr[ZL], br[BL];
    // element r of this thread's share: flat index tid + 256 r, K fastest
    // (coalesced along rows of Z and B)
    auto load = [&](int k0) {
#pragma unroll
      for (int r = 0; r < ZL; r++) {
        const int q = tid + 256 * r, c = q / TR_BK, e = k0 + q % TR_BK, i = i0 + c;
        double z = 0.0;
        if (i < rows && e < N) {
          // Mirrored Sampling (:461-491): rows 2j and 2j+1 take z_j and -z_j
          z = Z[(size_t)(mirrored ? (i >> 1) : i) * N + e];
          if (mirrored && (i & 1)) z = -z;
          z = D[e] * z;
        }
        zr[r] = z;
      }
#pragma unroll
      for (int r = 0; r < BL; r++) {
        const int q = tid + 256 * r, dd = q / TR_BK, e = k0 + q % TR_BK, d = d0 + dd;
        br[r] = (d < N && e < N) ? B[(size_t)d * N + e] : 0.0;
      }
    };
    auto store = [&]() {
#pragma unroll
      for (int r = 0; r < ZL; r++) {
        const int q = tid + 256 * r;
        Za[q % TR_BK][q / TR_BK] = zr[r];
      }
#pragma unroll
      for (int r = 0; r < BL; r++) {
        const int q = tid + 256 * r;
        Bt[q % TR_BK][q / TR_BK] = br[r];
      }
    };
    load(0);
    store();
    __syncthreads();
    for (int k0 = 0; k0 < N; k0 += TR_BK) {
      const bool more = k0 + TR_BK < N;
      if (more) load(k0 + TR_BK);
      const int kmax = (N - k0) < TR_BK ? (N - k0) : TR_BK;
      // operands of step kk + 1 are read from LDS while step kk is summed
      double a0[PR], b0[PC], a1[PR], b1[PC];
      auto fetch = [&](double *a, double *b, int kk) {
#pragma unroll
        for (int q = 0; q < PC; q += 2) {
          const double2 v = *(const double2 *)&Bt[kk][tx * PC + q];
          b[q] = v.x, b[q + 1] = v.y;
        }
#pragma unroll
        for (int p = 0; p < PR; p += 2) {
          const double2 v = *(const double2 *)&Za[kk][ty * PR + p];
          a[p] = v.x, a[p + 1] = v.y;
        }
      };
      // products formed in groups of 8 before their adds: independent
      // multiplies in flight instead of a mul -> add pair through one
      // temporary (issue-bound at one wave-op per ~8 cycles per wave)
      auto madd = [&](const double *a, const double *b) {
        static_assert((PR * PC) % 8 == 0, "8-product groups");
#pragma unroll
        for (int g = 0; g < PR * PC; g += 8) {
          double t[8];
#pragma unroll
          for (int u = 0; u < 8; u++) t[u] = b[(g + u) % PC] * a[(g + u) / PC];
#pragma unroll
          for (int u = 0; u < 8; u++) acc[(g + u) / PC][(g + u) % PC] += t[u];
        }
      };
      fetch(a0, b0, 0);
      if (kmax == TR_BK) {
        // whole chunk, no conditions in the loop: the waits before each
        // product group cover only the reads it consumes (lgkmcnt(n), n > 0)
#pragma unroll 1
        for (int kk = 0; kk < TR_BK - 2; kk += 2) {
          fetch(a1, b1, kk + 1);
          madd(a0, b0);
          fetch(a0, b0, kk + 2);
          madd(a1, b1);
        }
        fetch(a1, b1, TR_BK - 1);
        madd(a0, b0);
        madd(a1, b1);
      } else {
#pragma unroll 1
        for (int kk = 0; kk < kmax; kk++) {
          fetch(a0, b0, kk);
          madd(a0, b0);
        }
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int p = 0; p < PR; p++) {
    const int i = i0 + ty * PR + p;
    if (i >= rows) continue;
    int bad = 0;
#pragma unroll
    for (int q = 0; q < PC; q++) {
      const int d = d0 + tx * PC + q;
      if (d >= N) continue;
      double zd = 0.0;
      if (diagonal) {
        zd = Z[(size_t)(mirrored ? (i >> 1) : i) * N + d];
        if (mirrored && (i & 1)) zd = -zd;
      }
      const double bdz = diagonal ? D[d] * zd : acc[p][q];
      const double x = mean[d] + sigma * bdz;
      X[(size_t)i * N + d] = x;
      if (BDZ) BDZ[(size_t)i * N + d] = bdz;
      if (!isfinite(x) || x < lb[d] || x > ub[d]) bad = 1;
    }
    if (bad) {
      // no_reserve: all bounds infinite and the overflow guard of
      // kg_cmaes_sample proved every draw of this generation finite, so a bad
      // row is an internal inconsistency, not a redraw
      if (no_reserve)
        atomicOr(&sc->errors, KG_ERR_DRAW_GUARD);
      else
        atomicOr(&infeas[i], 1);
    }
  }
}

// The same transform with the B operand in SCALAR registers (round 4).
// k_transform's 4 x 2 register tile reads 3 x 16 B of LDS per lane for 16
// FP64 instructions: at four waves per CU that is 192 B per LDS clock against
// 128 available, so it runs at half its VALU peak.  Here a lane owns ONE
// sample row i and a wave C columns d: per k it loads its (D o z)[i][k] from a
// k-major copy (one coalesced 512-B wave load), and B[d][k] for its C columns
// is wave-uniform, so it arrives through s_load into SGPRs and feeds v_mul_f64
// as the scalar operand: no LDS traffic and no per-lane B fetch inside the K
// loop.  k_prescale_t forms D o z (sign-flipped for the odd rows of Mirrored
// Sampling), transposed, in one pass; the sum over k stays the reference's
// sequential order from 0.0 with a separate multiply and add (bit-identical
// to k_transform).  The tile goes out through LDS as coalesced row segments.
constexpr int PS_T = 64;
__global__ void __launch_bounds__(256) k_prescale_t(int N, int rows, int ldz, const double *__restrict__ Z,
                                                    const double *__restrict__ D, int mirrored,
                                                    double *__restrict__ dzT) {
  __shared__ double t[PS_T][PS_T + 1];
  const int i0 = blockIdx.x * PS_T, k0 = blockIdx.y * PS_T, tid = threadIdx.x;
#pragma unroll 4
  for (int r = 0; r < PS_T * PS_T / 256; r++) {
    const int q = tid + 256 * r, ii = q / PS_T, kk = q % PS_T, i = i0 + ii, k = k0 + kk;
    double z = 0.0;
    if (i < rows && k < N) {
      z = Z[(size_t)(mirrored ? (i >> 1) : i) * N + k];
      if (mirrored && (i & 1)) z = -z;
      z = D[k] * z;
    }
    t[ii][kk] = z;
  }
  __syncthreads();
#pragma unroll 4
  for (int r = 0; r < PS_T * PS_T / 256; r++) {
    const int q = tid + 256 * r, kk = q / PS_T, ii = q % PS_T, k = k0 + kk;
    if (k < N) dzT[(size_t)k * ldz + i0 + ii] = t[ii][kk];  // (rows past `rows`: +0.0)
  }
}
inline int sc_ldz(size_t rows) { return (int)((rows + 127) / 128 * 128); }
// RPL sample rows per lane (64 RPL per wave): each B value a wave reads
// through the scalar cache serves RPL rows
template <int C, int RPL>
inline unsigned trs_grid(int rows, int N) {
  const int nrt = (rows + 64 * RPL - 1) / (64 * RPL), ncg = (N + 4 * C - 1) / (4 * C);
  return (unsigned)(((nrt + TR_XCD - 1) / TR_XCD) * TR_XCD * ncg);
}
// default: the scalar-operand form from N = 256 up (C4: 1.55 against 1.70 ms
// per generation), the LDS-tiled one below (C2: 0.023 against 0.037 ms: too
// few 64-row tiles to fill the device, plus the prescale pass)
inline int transform_width(int N) {  // (read per handle: tests switch it per case)
  const char *e = getenv("KORALI_AMD_TRANSFORM_SC");
  if (!e || !*e) return N >= 256 ? 82 : 0;
  const int v = atoi(e);
  return (v == 8 || v == 16 || v == 82) ? v : 0;  // 82: C = 8 columns, 2 rows per lane
}
template <int C, int RPL>
__global__ void __launch_bounds__(256) k_transform_sc(int N, int rows, int ldz, const double *__restrict__ dzT,
                                                      const double *__restrict__ B, const double *__restrict__ mean,
                                                      CmaesScalars *__restrict__ sc, const double *__restrict__ lb,
                                                      const double *__restrict__ ub, double *__restrict__ X,
                                                      double *__restrict__ BDZ, int *__restrict__ infeas,
                                                      int no_reserve) {
  constexpr int WC = 4 * C, TR = 64 * RPL;  // columns (4 waves x C) and rows per workgroup
  __shared__ double so[TR][WC + 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order (as k_transform): the column groups of one row tile run
  // on one XCD, so its (D o z) rows come from HBM once
  const int ncg = (N + WC - 1) / WC;
  const int xcd = blockIdx.x % TR_XCD, j = blockIdx.x / TR_XCD;
  const int rt = (j / ncg) * TR_XCD + xcd, cg = j % ncg;
  const int i0 = rt * TR;
  if (i0 >= rows) return;
  const int d0 = cg * WC + w * C;
  const double *Bc[C];
#pragma unroll
  for (int c = 0; c < C; c++) Bc[c] = B + (size_t)min(d0 + c, N - 1) * N;  // (columns past N: discarded)
  double acc[RPL][C];
#pragma unroll
  for (int p = 0; p < RPL; p++)
#pragma unroll
    for (int c = 0; c < C; c++) acc[p][c] = 0.0;
  const double *zp = dzT + i0 + lane;
  auto step = [&](const double *z, int k) {  // z[p]: row i0 + 64 p + lane
    double t[RPL][C];
#pragma unroll
    for (int c = 0; c < C; c++) {
      const double b = Bc[c][k];
#pragma unroll
      for (int p = 0; p < RPL; p++) t[p][c] = b * z[p];
    }
#pragma unroll
    for (int p = 0; p < RPL; p++)
#pragma unroll
      for (int c = 0; c < C; c++) acc[p][c] += t[p][c];
  };
  // groups of 4 k, the next group's z loads in flight while this one is
  // summed (two register sets in turn: a copy between them would wait for
  // the loads).  Loads past the last group are clamped to row N - 1 rather
  // than branched around (a branch makes the compiler wait for them early).
  const int N4 = N & ~3;
  double za[4][RPL], zb[4][RPL];
  auto load4 = [&](double (*z)[RPL], int k) {
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int p = 0; p < RPL; p++) z[u][p] = zp[(size_t)min(k + u, N - 1) * ldz + 64 * p];
  };
  if (N4) load4(za, 0);
  int k = 0;
  for (; k + 8 <= N4; k += 8) {
    load4(zb, k + 4);
    // (compiler-only fences: B's scalar loads of a group are not hoisted
    // into the previous one, which ran out of SGPRs and spilled them at RPL 2)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < 4; u++) step(za[u], k + u);
    load4(za, k + 8);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < 4; u++) step(zb[u], k + 4 + u);
  }
  if (k < N4) {  // one group left (already in za)
#pragma unroll
    for (int u = 0; u < 4; u++) step(za[u], k + u);
  }
  for (int k = N4; k < N; k++) {
    double z[RPL];
#pragma unroll
    for (int p = 0; p < RPL; p++) z[p] = zp[(size_t)k * ldz + 64 * p];
    step(z, k);
  }
#pragma unroll
  for (int p = 0; p < RPL; p++)
#pragma unroll
    for (int c = 0; c < C; c++) so[64 * p + lane][w * C + c] = acc[p][c];
  __syncthreads();
  const double sigma = sc->sigma;
  for (int q = tid; q < TR * WC; q += 256) {
    const int r = q / WC, cc = q % WC, i = i0 + r, d = cg * WC + cc;
    if (i >= rows || d >= N) continue;
    const double bdz = so[r][cc];
    const double x = mean[d] + sigma * bdz;
    X[(size_t)i * N + d] = x;
    if (BDZ) BDZ[(size_t)i * N + d] = bdz;
    if (!isfinite(x) || x < lb[d] || x > ub[d]) {
      if (no_reserve)
        atomicOr(&sc->errors, KG_ERR_DRAW_GUARD);
      else
        atomicOr(&infeas[i], 1);
    }
  }
}

// resampling (prepareGeneration :443-460): candidate i takes the next block
// whose draw is feasible, or any block once the global infeasible counter
// reaches Max Infeasible Resamplings.  Sequential (one thread): runs only
// when some bound is finite (or the overflow guard tripped).  One ROUND
// walks the blocks transformed so far: candidates [i0, *iEnd) are assigned;
// when the blocks run out first, *iEnd < lam and the host transforms the
// next blocks of the stream (kg_cmaes_sample) and walks on from *iEnd with
// the same infeasible count, so the reference's unbounded do/while loop is
// followed for any number of redraws.
__global__ void k_select(int lam, int i0, int blocks, double maxRes, const int *__restrict__ infeas,
                         int *__restrict__ assign, unsigned long long *__restrict__ used, int *__restrict__ iEnd,
                         CmaesScalars *sc) {
  if (threadIdx.x != 0) return;
  double count = sc->infeasibleSampleCount;
  int j = 0, i = i0;
  for (; i < lam; i++) {
    bool taken = false;
    while (j < blocks) {
      const int feasible = infeas[j] ? 0 : 1;
      if (!feasible) count += 1;
      const int jj = j++;
      if (feasible || !(count < maxRes)) {
        assign[i] = jj;
        taken = true;
        break;
      }
    }
    if (!taken) break;  // blocks exhausted: candidate i continues in the next round
  }
  sc->infeasibleSampleCount = count;
  *used = (unsigned long long)j;
  *iEnd = i;
}

// Mirrored Sampling's resampling (:461-491): pair p takes the next block j
// (rows 2j, 2j+1) of which either draw is feasible; each infeasible draw
// counts.  Rounds as in k_select (i0, *iEnd are sample indices, even).
__global__ void k_select_mirrored(int lam, int i0, int blocks, double maxRes, const int *__restrict__ infeas,
                                  int *__restrict__ assign, unsigned long long *__restrict__ used,
                                  int *__restrict__ iEnd, CmaesScalars *sc) {
  if (threadIdx.x != 0) return;
  double count = sc->infeasibleSampleCount;
  int j = 0, i = i0;
  for (; i < lam; i += 2) {
    bool taken = false;
    while (j < blocks) {
      const int ok1 = infeas[2 * j] ? 0 : 1;
      if (!ok1) count += 1;
      const int ok2 = infeas[2 * j + 1] ? 0 : 1;
      if (!ok2) count += 1;
      const int jj = j++;
      if (ok1 || ok2 || !(count < maxRes)) {
        assign[i] = 2 * jj;
        assign[i + 1] = 2 * jj + 1;
        taken = true;
        break;
      }
    }
    if (!taken) break;
  }
  sc->infeasibleSampleCount = count;
  *used = (unsigned long long)j;
  *iEnd = i;
}

// the rows a round assigned, candidates [i0, *iEnd)
__global__ void k_gather_rows(int N, int i0, const int *__restrict__ iEnd, const int *__restrict__ assign,
                              const double *__restrict__ Xall, double *__restrict__ X,
                              const double *__restrict__ BDZall, double *__restrict__ BDZ) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = i0 + (int)(t / N), d = (int)(t % N);
  if (i >= *iEnd) return;
  X[(size_t)i * N + d] = Xall[(size_t)assign[i] * N + d];
  if (BDZ) BDZ[(size_t)i * N + d] = BDZall[(size_t)assign[i] * N + d];
}

// ------------------------------------------------------------ objective
// examples/optimization/stochastic/_model/model.py: negative_rosenbrock
// (:23-34), negative_ackley (:37-62), negative_sphere; sequential in d.
// 64 candidates per workgroup: all 256 threads load a 64 x 32 tile of the
// population (coalesced, 8 independent loads each) and, for Ackley, evaluate
// its cosines in parallel; the candidates' sums (sequential in d, the
// reference's order) then run on one wave.
constexpr int OB_C = 64, OB_D = 32;
__global__ void __launch_bounds__(256) k_objective(int N, int lam, int obj, const double *__restrict__ X,
                                                   double *__restrict__ F, CmaesScalars *sc, double addEvals) {
  if (blockIdx.x == 0 && threadIdx.x == 0) sc->modelEvaluationCount += addEvals;  // (was k_add_evals)
  __shared__ double tile[OB_C][OB_D + 1];
  __shared__ double ctile[OB_C][OB_D + 1];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * OB_C;
  const int i = c0 + tid;
  double r0 = 0.0, r1 = 0.0, prev = 0.0;
  const double cc = 2. * 3.141592653589793;
  for (int d0 = 0; d0 < N; d0 += OB_D) {
    const int dn = (N - d0) < OB_D ? (N - d0) : OB_D;
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int e = tid + 256 * u, row = e >> 5, col = e & 31, ii = c0 + row;
      v[u] = (ii < lam && col < dn) ? X[(size_t)ii * N + d0 + col] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int e = tid + 256 * u, row = e >> 5, col = e & 31;
      tile[row][col] = v[u];
      if (obj == KG_OBJ_NEGATIVE_ACKLEY) ctile[row][col] = cos_cr(cc * v[u]);
    }
    __syncthreads();
    if (tid < OB_C && i < lam) {
      for (int dd = 0; dd < dn; dd++) {
        const double x = tile[tid][dd];
        const int d = d0 + dd;
        if (obj == KG_OBJ_NEGATIVE_ROSENBROCK) {
          if (d > 0) {
            const double tt = x - prev * prev;
            const double u = 1 - prev;
            r0 += 100 * (tt * tt) + u * u;
          }
          prev = x;
        } else if (obj == KG_OBJ_NEGATIVE_ACKLEY) {
          r0 += x * x;
          r1 += ctile[tid][dd];
        } else {
          r0 += x * x;
        }
      }
    }
    __syncthreads();
  }
  if (tid >= OB_C || i >= lam) return;
  double f;
  if (obj == KG_OBJ_NEGATIVE_ROSENBROCK)
    f = -r0;
  else if (obj == KG_OBJ_NEGATIVE_ACKLEY) {
    const double s1 = r0 / (double)N, s2 = r1 / (double)N;
    const double e1 = 20. * exp_cr(-0.2 * sqrt(s1));
    const double e2 = exp_cr(s2);
    f = e1 + e2 - 20. - 2.718281828459045;
  } else
    f = -0.5 * r0;
  F[i] = f;
  if (!isfinite(f)) atomicOr(&sc->errors, KG_ERR_NONFINITE_F);
}

// The same objectives for N <= 128 with each row's ordered sum split from
// its terms: the 64 rows' X block is loaded with every load in flight at
// once; waves 1-3 form the terms of 32-column chunks (Rosenbrock's
// 100 (x_d - x_{d-1}^2)^2 + (1 - x_{d-1})^2, Ackley's x^2 and cos 2 pi x,
// the sphere's x^2) into LDS while wave 0 adds the previous chunk's terms
// in order, one add per term (k_objective's single wave formed and added
// every term itself, issue-bound at ~8 instructions per term).
constexpr int OB2_R = 64, OB2_NC = 32;  // rows per workgroup; columns per chunk
__host__ __device__ inline size_t ob2_lds_bytes(int N) {
  return ((size_t)OB2_R * (N + 1) + 2 * 2 * (size_t)OB2_R * (OB2_NC + 1)) * sizeof(double);
}
__global__ void __launch_bounds__(256) k_objective2(int N, int lam, int obj, const double *__restrict__ X,
                                                    double *__restrict__ F, CmaesScalars *sc, double addEvals) {
  extern __shared__ __attribute__((aligned(16))) double ob2[];
  if (blockIdx.x == 0 && threadIdx.x == 0) sc->modelEvaluationCount += addEvals;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ld = N + 1, c0 = blockIdx.x * OB2_R;
  double *Xs = ob2;                                   // [row][d], row stride N + 1
  double *Ta = Xs + (size_t)OB2_R * ld;               // [2][row][OB2_NC + 1] first terms
  double *Tb = Ta + 2 * (size_t)OB2_R * (OB2_NC + 1);  // [2][row][OB2_NC + 1] Ackley's cos terms
  const int tot = OB2_R * N;
  for (int q0 = tid; q0 < tot; q0 += 32 * 256) {  // N <= 128: one pass, 32 loads in flight per thread
    double v[32];
#pragma unroll
    for (int u = 0; u < 32; u++) {
      const int q = q0 + u * 256, r = q / N, d = q - r * N;
      v[u] = (q < tot && c0 + r < lam) ? X[(size_t)(c0 + r) * N + d] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 32; u++) {
      const int q = q0 + u * 256, r = q / N, d = q - r * N;
      if (q < tot) Xs[(size_t)r * ld + d] = v[u];
    }
  }
  __syncthreads();
  const int nch = (N + OB2_NC - 1) / OB2_NC;
  const double cc = 2. * 3.141592653589793;
  // producers: terms of chunk ch into buffer ch & 1 (row = lane, columns over waves 1-3)
  auto form = [&](int ch) {
    const int b = ch & 1, d0 = ch * OB2_NC, dn = min(OB2_NC, N - d0);
    double *ta = Ta + (size_t)b * OB2_R * (OB2_NC + 1) + (size_t)lane * (OB2_NC + 1);
    double *tb = Tb + (size_t)b * OB2_R * (OB2_NC + 1) + (size_t)lane * (OB2_NC + 1);
    const double *xr = Xs + (size_t)lane * ld;
    if (obj != KG_OBJ_NEGATIVE_ACKLEY) {  // every operand of the wave's columns read first, then the terms
      constexpr int PU = (OB2_NC + 2) / 3;
      double xs[PU], xp[PU];
#pragma unroll
      for (int u = 0; u < PU; u++) {
        const int dd = wid - 1 + 3 * u, d = d0 + dd;
        xs[u] = dd < dn ? xr[d] : 0.0;
        xp[u] = (dd < dn && d > 0) ? xr[d - 1] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < PU; u++) {
        const int dd = wid - 1 + 3 * u, d = d0 + dd;
        if (dd >= dn) break;
        const double x = xs[u];
        if (obj == KG_OBJ_NEGATIVE_ROSENBROCK) {
          if (d > 0) {
            const double prev = xp[u];
            const double tt = x - prev * prev;
            const double uu = 1 - prev;
            ta[dd] = 100 * (tt * tt) + uu * uu;
          }
        } else {
          ta[dd] = x * x;
        }
      }
      return;
    }
    for (int dd = wid - 1; dd < dn; dd += 3) {
      const int d = d0 + dd;
      const double x = xr[d];
      if (obj == KG_OBJ_NEGATIVE_ROSENBROCK) {
        if (d > 0) {
          const double prev = xr[d - 1];
          const double tt = x - prev * prev;
          const double u = 1 - prev;
          ta[dd] = 100 * (tt * tt) + u * u;
        }
      } else if (obj == KG_OBJ_NEGATIVE_ACKLEY) {
        ta[dd] = x * x;
        tb[dd] = cos_cr(cc * x);
      } else {
        ta[dd] = x * x;
      }
    }
  };
  if (wid > 0) form(0);
  __syncthreads();
  double r0 = 0.0, r1 = 0.0;
  for (int ch = 0; ch < nch; ch++) {
    if (wid == 0) {
      const int b = ch & 1, d0 = ch * OB2_NC, dn = min(OB2_NC, N - d0);
      const double *ta = Ta + (size_t)b * OB2_R * (OB2_NC + 1) + (size_t)lane * (OB2_NC + 1);
      const double *tb = Tb + (size_t)b * OB2_R * (OB2_NC + 1) + (size_t)lane * (OB2_NC + 1);
      if (obj == KG_OBJ_NEGATIVE_ROSENBROCK) {
        // eight terms read before their adds (one LDS round trip per eight,
        // the adds in column order as before)
        int dd = d0 == 0 ? 1 : 0;
        for (; dd + 8 <= dn; dd += 8) {
          double t[8];
#pragma unroll
          for (int u = 0; u < 8; u++) t[u] = ta[dd + u];
#pragma unroll
          for (int u = 0; u < 8; u++) r0 += t[u];
        }
        for (; dd < dn; dd++) r0 += ta[dd];
      } else if (obj == KG_OBJ_NEGATIVE_ACKLEY) {
        for (int dd = 0; dd < dn; dd++) {
          r0 += ta[dd];
          r1 += tb[dd];
        }
      } else {
        for (int dd = 0; dd < dn; dd++) r0 += ta[dd];
      }
    } else if (ch + 1 < nch) {
      form(ch + 1);
    }
    __syncthreads();
  }
  const int i = c0 + lane;
  if (wid != 0 || i >= lam) return;
  double f;
  if (obj == KG_OBJ_NEGATIVE_ROSENBROCK)
    f = -r0;
  else if (obj == KG_OBJ_NEGATIVE_ACKLEY) {
    const double s1 = r0 / (double)N, s2 = r1 / (double)N;
    const double e1 = 20. * exp_cr(-0.2 * sqrt(s1));
    const double e2 = exp_cr(s2);
    f = e1 + e2 - 20. - 2.718281828459045;
  } else
    f = -0.5 * r0;
  F[i] = f;
  if (!isfinite(f)) atomicOr(&sc->errors, KG_ERR_NONFINITE_F);
}

// ----------------------------------------------------------------- sort
// sort_index (CMAES.cpp.base:940-950): descending F; ties by index (the
// reference's std::sort leaves tie order unspecified).  Bitonic network:
// chunks of SORT_CHUNK in LDS, wider strides in global passes.
constexpr int SORT_CHUNK = 2048;
__device__ inline bool before(double ka, unsigned ia, double kb, unsigned ib) {
  return (ka > kb) || (ka == kb && ia < ib);
}

__global__ void __launch_bounds__(1024) k_sort_init(int lam, int P2, const double *__restrict__ F, double *key,
                                                    unsigned *val) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P2) return;
  key[i] = (i < lam) ? F[i] : -INFINITY;
  val[i] = (i < lam) ? (unsigned)i : 0xffffffffu;
}

// local stages: for k in [kmin..kmax] (kmax <= SORT_CHUNK), or one k with all
// j < SORT_CHUNK when kfixed > 0
__global__ void __launch_bounds__(1024) k_sort_local(int P2, int kfixed, double *key, unsigned *val) {
  __shared__ double sk[SORT_CHUNK];
  __shared__ unsigned sv[SORT_CHUNK];
  const int base = blockIdx.x * SORT_CHUNK;
  for (int q = threadIdx.x; q < SORT_CHUNK; q += blockDim.x) {
    sk[q] = key[base + q];
    sv[q] = val[base + q];
  }
  __syncthreads();
  const int kstart = kfixed ? kfixed : 2, kend = kfixed ? kfixed : SORT_CHUNK;
  for (int k = kstart; k <= kend; k <<= 1) {
    const int jstart = kfixed ? SORT_CHUNK / 2 : k / 2;
    for (int j = jstart; j > 0; j >>= 1) {
      for (int q = threadIdx.x; q < SORT_CHUNK; q += blockDim.x) {
        const int l = q ^ j;
        if (l > q) {
          const int gi = base + q;
          const bool asc = ((gi & k) == 0);
          const double ka = sk[q], kb = sk[l];
          const unsigned ia = sv[q], ib = sv[l];
          const bool sw = asc ? before(kb, ib, ka, ia) : before(ka, ia, kb, ib);
          if (sw) {
            sk[q] = kb;
            sk[l] = ka;
            sv[q] = ib;
            sv[l] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int q = threadIdx.x; q < SORT_CHUNK; q += blockDim.x) {
    key[base + q] = sk[q];
    val[base + q] = sv[q];
  }
}

__global__ void k_sort_global(int P2, int k, int j, double *key, unsigned *val) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P2) return;
  const int l = q ^ j;
  if (l <= q) return;
  const bool asc = ((q & k) == 0);
  const double ka = key[q], kb = key[l];
  const unsigned ia = val[q], ib = val[l];
  const bool sw = asc ? before(kb, ib, ka, ia) : before(ka, ia, kb, ib);
  if (sw) {
    key[q] = kb;
    key[l] = ka;
    val[q] = ib;
    val[l] = ia;
  }
}

// small λ (< SORT_CHUNK): one block sorts everything
__global__ void __launch_bounds__(1024) k_sort_small(int lam, int P2, const double *__restrict__ F, unsigned *out) {
  __shared__ double sk[SORT_CHUNK];
  __shared__ unsigned sv[SORT_CHUNK];
  for (int q = threadIdx.x; q < P2; q += blockDim.x) {
    sk[q] = (q < lam) ? F[q] : -INFINITY;
    sv[q] = (q < lam) ? (unsigned)q : 0xffffffffu;
  }
  __syncthreads();
  for (int k = 2; k <= P2; k <<= 1) {
    for (int j = k / 2; j > 0; j >>= 1) {
      for (int q = threadIdx.x; q < P2; q += blockDim.x) {
        const int l = q ^ j;
        if (l > q) {
          const bool asc = ((q & k) == 0);
          const double ka = sk[q], kb = sk[l];
          const unsigned ia = sv[q], ib = sv[l];
          const bool sw = asc ? before(kb, ib, ka, ia) : before(ka, ia, kb, ib);
          if (sw) {
            sk[q] = kb;
            sk[l] = ka;
            sv[q] = ib;
            sv[l] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int q = threadIdx.x; q < lam; q += blockDim.x) out[q] = sv[q];
}

// Rank sort for populations up to RANK_MAX: rank(i) = #{j : j before i}
// (descending F, ties by index — the same total order as the bitonic
// network), every key against every key in parallel: workgroup b ranks keys
// 16b..16b+15, its 16 thread groups each scanning one sixteenth of the
// population (LDS broadcast reads).  One launch instead of the bitonic
// network's many.
constexpr int RANK_MAX = 16384;
__global__ void __launch_bounds__(256) k_rank_sort(int lam, const double *__restrict__ F, unsigned *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double rk[];
  __shared__ unsigned part[16][17];
  for (int q0 = threadIdx.x; q0 < lam; q0 += 8 * blockDim.x) {  // eight loads in flight per thread
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = (q0 + u * (int)blockDim.x < lam) ? F[q0 + u * blockDim.x] : 0.0;
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q0 + u * (int)blockDim.x < lam) rk[q0 + u * blockDim.x] = v[u];
  }
  __syncthreads();
  const int li = threadIdx.x & 15, p = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + li;
  const double ki = (i < lam) ? rk[i] : 0.0;
  const int per = (lam + 15) / 16, j0 = p * per, j1 = min(lam, j0 + per);
  unsigned c = 0;
  int j = j0;
  // eight keys read before their compares (one LDS round trip per eight:
  // the one-key loop waited on every read, ~11 of its 21 us at lambda = 4096)
  for (; j + 8 <= j1; j += 8) {
    double kj[8];
#pragma unroll
    for (int u = 0; u < 8; u++) kj[u] = rk[j + u];
#pragma unroll
    for (int u = 0; u < 8; u++) c += (kj[u] > ki || (kj[u] == ki && j + u < i)) ? 1u : 0u;
  }
  for (; j < j1; j++) {
    const double kj = rk[j];
    c += (kj > ki || (kj == ki && j < i)) ? 1u : 0u;
  }
  part[p][li] = c;
  __syncthreads();
  if (threadIdx.x < 16 && i < lam) {
    unsigned r = 0;
    for (int q = 0; q < 16; q++) r += part[q][threadIdx.x];
    out[r] = (unsigned)i;
  }
}

// ------------------------------------------------ discrete variables
// prepareGeneration's sampling loop with Granularity (CMAES.cpp.base:443-458,
// sampleSingle :515-544, discretize :861-867) over the transformed rows
// Xall (every normal row of the stream, in order): sample i takes rows until
// one is feasible after its discrete mutation and rounding, exactly as the
// reference redraws; the mutation's uniforms come from U (the Uniform
// Generator's next words, peeked) in the reference's order, *uUsed of them
// consumed.  One workgroup, one sample at a time (the uniform walk is
// sequential); the rounded point is rounded once more as the evaluation does
// (:208).  Discrete problems are small (the reference example: N = 10,
// lambda = 8), so the O(lambda) barriers are not on a hot path.
__device__ __forceinline__ double discretize1(double x, double g) { return g != 0.0 ? round(x / g) * g : x; }
__global__ void __launch_bounds__(256) k_discrete_select(int N, int lam, int i0start, int blocks, int mirrored,
                                                         double maxRes, const double *__restrict__ Xall,
                                                         const double *__restrict__ BDZall, double *__restrict__ X,
                                                         double *__restrict__ BDZ, const double *__restrict__ lb,
                                                         const double *__restrict__ ub,
                                                         const double *__restrict__ gran,
                                                         const double *__restrict__ mask,
                                                         const double *__restrict__ best, const double *__restrict__ U,
                                                         unsigned long long ucap, unsigned long long *uUsed,
                                                         unsigned long long *used, int *__restrict__ iEnd,
                                                         CmaesScalars *sc) {
  extern __shared__ double xs[];  // 2 N: the unit's samples (one, or a mirrored pair)
  __shared__ int infeas[2];
  __shared__ int overflow;  // the attempt needed more peeked uniforms than U holds
  const int tid = threadIdx.x, per = mirrored ? 2 : 1;
  const double nDM = sc->nDM, nME = sc->nME;
  double count = sc->infeasibleSampleCount;
  int j = 0, i0 = i0start;
  unsigned long long u = 0;
  auto uni = [&]() {  // next uniform (thread 0)
    const double v = u < ucap ? U[u] : 0.0;
    u++;
    return v;
  };
  // a round ends at an attempt boundary: when the transformed blocks run out
  // or an attempt would read past the peeked uniforms (it is then undone and
  // redone in the next round from the stream position where it started)
  bool stop = false, outOfUniforms = false;
  for (; i0 < lam && !stop; i0 += per) {
    for (;;) {
      if (j >= blocks) {
        stop = true;
        break;
      }
      const int blk = j;
      const unsigned long long u0 = u;
      for (int q = tid; q < per * N; q += blockDim.x) xs[q] = Xall[((size_t)blk * per) * N + q];
      if (tid < 2) infeas[tid] = 0;
      if (tid == 0) overflow = 0;
      __syncthreads();
      if (tid == 0) {
        for (int s = 0; s < per; s++) {  // sampleSingle(i0 + s) in order (:472-473)
          const int i = i0 + s;
          double *x = xs + (size_t)s * N;
          if ((double)(i + 1) < nDM) {
            const double p_geom = pow_cr(0.7, 1.0 / nME);
            size_t select = (size_t)floor(uni() * nME);
            for (int d = 0; d < N; ++d)
              if ((mask[d] == 1.0) && (select-- == 0)) {
                double dm = 1.0;
                while (uni() > p_geom) dm += 1.0;
                dm *= gran[d];
                if (uni() > 0.5) dm *= -1.0;
                x[d] += dm;
              }
          } else if ((double)(i + 1) == nDM) {
            for (int d = 0; d < N; ++d)
              if (gran[d] != 0.0) x[d] += round(best[d] / gran[d]) * gran[d] - x[d];
          }
        }
        if (u > ucap) {
          overflow = 1;
          u = u0;
        }
      }
      __syncthreads();
      if (overflow) {
        stop = outOfUniforms = true;
        break;
      }
      for (int q = tid; q < per * N; q += blockDim.x) {
        const int d = q % N;
        const double x = discretize1(xs[q], gran[d]);
        xs[q] = x;
        if (!isfinite(x) || x < lb[d] || x > ub[d]) infeas[q / N] = 1;  // (benign race: every writer stores 1)
      }
      __syncthreads();
      bool anyOk = false;
      for (int s = 0; s < per; s++) {
        if (infeas[s]) count += 1;
        else anyOk = true;
      }
      j++;
      if (anyOk || !(count < maxRes)) {
        for (int q = tid; q < per * N; q += blockDim.x) {
          const int d = q % N;
          X[(size_t)i0 * N + q] = discretize1(xs[q], gran[d]);  // :208 before evaluation
          if (BDZ) BDZ[(size_t)i0 * N + q] = BDZall[((size_t)blk * per) * N + q];
        }
        __syncthreads();
        break;
      }
      __syncthreads();
    }
    if (stop) break;
  }
  if (tid == 0) {
    sc->infeasibleSampleCount = count;
    *used = (unsigned long long)j;
    *uUsed = u;
    iEnd[0] = i0 < lam ? i0 : lam;
    iEnd[1] = outOfUniforms ? 1 : 0;  // the host peeks a larger window before the next round
  }
}

// updateDiscreteMutationMatrix (:834-859), after adaptC with the old sigma
__global__ void k_discrete_masks(int N, int lam, const double *__restrict__ gran, const double *__restrict__ C,
                                 double *mask, double *maskSigma, CmaesScalars *sc) {
  if (threadIdx.x != 0) return;
  const double sigma = sc->sigma, cs = sc->sigmaCumulationFactor;
  double entries = (double)(N + 1);
  for (int d = 0; d < N; ++d) maskSigma[d] = 1.0;
  for (int d = 0; d < N; ++d)
    if (sigma * sqrt(C[(size_t)d * N + d]) / sqrt(cs) < 0.2 * gran[d]) {
      maskSigma[d] = 0.0;
      entries -= 1.0;
    }
  sc->chiDM = sqrt(entries) * (1. - 1. / (4. * entries) + 1. / (21. * entries * entries));
  double nme = 0.0;
  for (int d = 0; d < N; ++d) {
    mask[d] = 0.0;
    if (2.0 * sigma * sqrt(C[(size_t)d * N + d]) < gran[d]) {
      mask[d] = 1.0;
      nme += 1.0;
    }
  }
  sc->nME = nme;
  const double a = round((double)lam / 10.0 + nme + 1), b = floor((double)lam / 2.0) - 1;
  sc->nDM = a < b ? a : b;
}

__global__ void k_copy_idx(int lam, const unsigned *__restrict__ val, unsigned *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < lam) out[i] = val[i];
}

// --------------------------------------------------------------- update
// updateDistribution :547-609 (best bookkeeping, proportional weights)
// viol (CCMA-ES outside the viability regime): the best valid sample is the
// LAST sample in sorted order without constraint violations (:551-558, as
// written)
__global__ void __launch_bounds__(256) k_update_best(int N, int mu, int muType, unsigned long long gen,
                                                     const double *__restrict__ X, const double *__restrict__ F,
                                                     const unsigned *__restrict__ idx, double *w,
                                                     double *currBestVars, double *bestEverVars, CmaesScalars *sc,
                                                     const int *__restrict__ viol, int lam) {
  __shared__ int flag;
  __shared__ unsigned bestIdx;
  const int tid = threadIdx.x;
  if (tid == 0) {
    unsigned b = idx[0];
    if (viol) {
      long best = -1;
      for (int i = 0; i < lam; i++)
        if (viol[idx[i]] == 0) best = (long)idx[i];
      if (best < 0) sc->errors |= KG_ERR_CONSTRAINT;  // the reference reads _valueVector[-1]
      else b = (unsigned)best;
    }
    bestIdx = b;
  }
  __syncthreads();
  const unsigned i0 = bestIdx;
  if (tid == 0) {
    sc->bestValidSample = (double)i0;
    sc->previousBestValue = sc->currentBestValue;
    sc->currentBestValue = F[i0];
    flag = (sc->currentBestValue > sc->bestEverValue || gen == 1) ? 1 : 0;
    sc->bestFlag = (unsigned)flag;
    sc->rmuOutOfRange = 0u;  // set again by this generation's k_rankmu_prep
    if (flag) {
      sc->previousBestEverValue = sc->bestEverValue;
      sc->bestEverValue = sc->currentBestValue;
    }
    if (muType == KG_MU_PROPORTIONAL) {
      double valueSum = 0.;
      for (int i = 0; i < mu; ++i) {
        const double value = F[idx[i]];
        w[i] = value;
        valueSum += value;
      }
      for (int i = 0; i < mu; ++i) w[i] /= valueSum;
    }
  }
  __syncthreads();
  if (!X) return;  // population shards: the best row arrives through the partials
  for (int d = tid; d < N; d += blockDim.x) {
    const double v = X[(size_t)i0 * N + d];
    currBestVars[d] = v;
    if (flag) bestEverVars[d] = v;
  }
}

// gather the μ selected rows into Y (contiguous; shared by mean and adaptC)
__global__ void __launch_bounds__(256) k_gather_selected(int N, int mu, const double *__restrict__ X,
                                                         const unsigned *__restrict__ idx, double *__restrict__ Y,
                                                         const double *__restrict__ mean,
                                                         double *__restrict__ prevMean) {
  const int i = blockIdx.x;
  const size_t src = (size_t)idx[i] * N;
  for (int d = threadIdx.x; d < N; d += blockDim.x) Y[(size_t)i * N + d] = X[src + d];
  // m_prev (updateDistribution :603): read by k_mean and, concurrently, by
  // the rank-mu sum on the second stream
  if (i == 0)
    for (int d = threadIdx.x; d < N; d += blockDim.x) prevMean[d] = mean[d];
}

// ------------------------------------------------ exact rank-mu (adaptC)
// The reference adds, for every lower-triangle element (d, e) and k < mu in
// order (CMAES.cpp.base:700-707),
//   c += ccovmu * w_k * (x_kd - m_d) * (x_ke - m_e) / sigma^2
// = fl(fl(T_kd * Yc_ke) / s2)  with  Yc_kd = fl(x_kd - m_d),
//   T_kd = fl(fl(ccovmu w_k) Yc_kd),  s2 = fl(sigma sigma).
// k_rankmu_prep forms Yc (k-major, the e side) and T (transposed, d-major,
// the d side) once; k_adaptC_exact2 then spends per term one product, the
// Markstein-corrected quotient  q0 = p y, r = fma(-q0, s2, p),
// q = fma(r, y, q0)  (y = fl(1/s2); q == fl(p / s2) exactly whenever p and
// s2 stay far from underflow / overflow, Markstein's theorem) and the
// ordered add.  The range condition is checked here on every factor
// (exponents within +-450, nonzero, finite; then |p| in [2^-900, 2^900]);
// if any factor leaves it the generation uses true division throughout.
constexpr int RP_T = 32;
__device__ inline bool rmu_in_range(double v) {
  const int ex = (int)((__double_as_longlong(v) >> 52) & 0x7ff) - 1023;  // zero / subnormal: -1023
  return ex >= -450 && ex <= 450;
}
__global__ void __launch_bounds__(256) k_rankmu_prep(int N, int mu, const double *__restrict__ Y,
                                                     const double *__restrict__ w,
                                                     const double *__restrict__ prevMean,
                                                     CmaesScalars *sc, double *__restrict__ Yc,
                                                     double *__restrict__ Tt) {
  __shared__ double tile[RP_T][RP_T + 1];
  const int k0 = blockIdx.x * RP_T, d0 = blockIdx.y * RP_T;
  const int tx = threadIdx.x % RP_T, ty = threadIdx.x / RP_T;  // 32 x 8
  // c_mu from mu_eff with k_paths' formula (CMAES.cpp.base:693-694)
  const double effMu = sc->effectiveMu, ca = N + 1.3, cb = N + 2.0;
  const double ccov1 = 2.0 / (ca * ca + effMu);
  double ccovmu = 2.0 * (effMu - 2. + 1. / effMu) / (cb * cb + effMu);
  if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
  bool ok = true;
  for (int r = ty; r < RP_T; r += 8) {
    const int k = k0 + r, d = d0 + tx;
    double t = 0.0;
    if (k < mu && d < N) {
      const double yc = Y[(size_t)k * N + d] - prevMean[d];
      Yc[(size_t)k * N + d] = yc;
      t = (ccovmu * w[k]) * yc;
      ok = ok && rmu_in_range(yc) && rmu_in_range(t);
    }
    tile[r][tx] = t;
  }
  __syncthreads();
  for (int r = ty; r < RP_T; r += 8) {
    const int d = d0 + r, k = k0 + tx;
    if (d < N && k < mu) Tt[(size_t)d * mu + k] = tile[tx][r];
  }
  if (__syncthreads_or(!ok) && threadIdx.x == 0) atomicOr(&sc->rmuOutOfRange, 1u);
}

// k_update_best + k_gather_selected + k_rankmu_prep in one launch (the plain
// exact-mode update: no constraints, weights fixed at initialisation): tile
// (k0, d0) of the selected rows is read straight from the population through
// the sorting index into Y, Yc and T; workgroup (0, 0) also does the best
// bookkeeping, and the workgroups of the first row tile copy m into m_prev.
// m_prev is read by nothing in this launch (the factors take m itself, equal
// to m_prev until k_mean3 writes m).  The out-of-range flag is cleared by the
// previous update's k_sigma (or k_init), not here: a clear inside this launch
// could land after another workgroup's set.
__global__ void __launch_bounds__(256) k_select_prep(int N, int mu, unsigned long long gen,
                                                     const double *__restrict__ X, const double *__restrict__ F,
                                                     const unsigned *__restrict__ idx, const double *__restrict__ w,
                                                     const double *__restrict__ mean, double *__restrict__ prevMean,
                                                     double *__restrict__ Y, double *__restrict__ currBestVars,
                                                     double *__restrict__ bestEverVars, CmaesScalars *sc,
                                                     double *__restrict__ Yc, double *__restrict__ Tt) {
  __shared__ double tile[RP_T][RP_T + 1];
  __shared__ unsigned sidx[RP_T];
  const int k0 = blockIdx.x * RP_T, d0 = blockIdx.y * RP_T;
  const int tx = threadIdx.x % RP_T, ty = threadIdx.x / RP_T;  // 32 x 8
  if (threadIdx.x < RP_T) sidx[threadIdx.x] = (k0 + (int)threadIdx.x < mu) ? idx[k0 + threadIdx.x] : 0u;
  const double effMu = sc->effectiveMu, ca = N + 1.3, cb = N + 2.0;
  const double ccov1 = 2.0 / (ca * ca + effMu);
  double ccovmu = 2.0 * (effMu - 2. + 1. / effMu) / (cb * cb + effMu);
  if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
  __syncthreads();
  bool ok = true;
  double xv[RP_T / 8];
#pragma unroll
  for (int u = 0; u < RP_T / 8; u++) {  // every row's load in flight before the first use
    const int r = ty + 8 * u, k = k0 + r, d = d0 + tx;
    xv[u] = (k < mu && d < N) ? X[(size_t)sidx[r] * N + d] : 0.0;
  }
  const double md = d0 + tx < N ? mean[d0 + tx] : 0.0;
#pragma unroll
  for (int u = 0; u < RP_T / 8; u++) {
    const int r = ty + 8 * u, k = k0 + r, d = d0 + tx;
    double t = 0.0;
    if (k < mu && d < N) {
      Y[(size_t)k * N + d] = xv[u];
      const double yc = xv[u] - md;
      Yc[(size_t)k * N + d] = yc;
      t = (ccovmu * w[k]) * yc;
      ok = ok && rmu_in_range(yc) && rmu_in_range(t);
    }
    tile[r][tx] = t;
  }
  if (k0 == 0 && ty == 0 && d0 + tx < N) prevMean[d0 + tx] = md;
  __syncthreads();
  for (int r = ty; r < RP_T; r += 8) {
    const int d = d0 + r, k = k0 + tx;
    if (d < N && k < mu) Tt[(size_t)d * mu + k] = tile[tx][r];
  }
  if (__syncthreads_or(!ok) && threadIdx.x == 0) atomicOr(&sc->rmuOutOfRange, 1u);
  if (blockIdx.x || blockIdx.y) return;
  // updateDistribution's best bookkeeping (:547-560), as k_update_best
  __shared__ int flag;
  if (threadIdx.x == 0) {
    const unsigned i0 = sidx[0];
    sc->bestValidSample = (double)i0;
    sc->previousBestValue = sc->currentBestValue;
    sc->currentBestValue = F[i0];
    flag = (sc->currentBestValue > sc->bestEverValue || gen == 1) ? 1 : 0;
    sc->bestFlag = (unsigned)flag;
    if (flag) {
      sc->previousBestEverValue = sc->bestEverValue;
      sc->bestEverValue = sc->currentBestValue;
    }
  }
  __syncthreads();
  const unsigned i0 = sidx[0];
  for (int d = threadIdx.x; d < N; d += blockDim.x) {
    const double v = X[(size_t)i0 * N + d];
    currBestVars[d] = v;
    if (flag) bestEverVars[d] = v;
  }
}

// one wave per row d (4 rows per workgroup), one lane per column e (64
// columns per workgroup).  Per chunk of AX_K k: the workgroup stages the
// Yc rows of its 64 columns and the T values of its 4 rows in LDS (the next
// chunk's global loads are in flight while the current chunk is summed);
// each lane then runs its ordered chain reading Yc[k][lane] and the
// wave-uniform T[k][d] (broadcast) from LDS.
constexpr int AX_K = 64, AX_B = 16;
template <bool kMarkstein>
__device__ __forceinline__ double rankmu_term(double c, double t, double yc, double s2, double y) {
  const double p = t * yc;
  double q;
  if (kMarkstein) {
    const double q0 = p * y;
    const double r = __builtin_fma(-q0, s2, p);
    q = __builtin_fma(r, y, q0);
  } else {
    q = p / s2;
  }
  return c + q;
}
template <bool kMarkstein>
__device__ __forceinline__ double rankmu_quot(double t, double yc, double s2, double y) {
  const double p = t * yc;
  if (kMarkstein) {
    const double q0 = p * y;
    const double r = __builtin_fma(-q0, s2, p);
    return __builtin_fma(r, y, q0);
  }
  return p / s2;
}
template <bool kMarkstein>
__device__ __forceinline__ double rankmu_chunk(double c, const double *__restrict__ ys, const double *__restrict__ ts,
                                               int cnt, double s2, double y) {
  if (cnt == AX_K) {
    // operands of the next 16 terms are read from LDS while the current 16
    // quotients (independent) are formed and added in order
    double ya[AX_B], ta[AX_B], yb[AX_B], tb[AX_B];
#pragma unroll
    for (int u = 0; u < AX_B; u++) {
      ya[u] = ys[u * 64];
      ta[u] = ts[u];
    }
#pragma unroll
    for (int j = 0; j < AX_K / AX_B; j += 2) {
#pragma unroll
      for (int u = 0; u < AX_B; u++) {
        yb[u] = ys[((j + 1) * AX_B + u) * 64];
        tb[u] = ts[(j + 1) * AX_B + u];
      }
      double q[AX_B];
#pragma unroll
      for (int u = 0; u < AX_B; u++) q[u] = rankmu_quot<kMarkstein>(ta[u], ya[u], s2, y);
#pragma unroll
      for (int u = 0; u < AX_B; u++) c += q[u];
      if (j + 2 < AX_K / AX_B) {
#pragma unroll
        for (int u = 0; u < AX_B; u++) {
          ya[u] = ys[((j + 2) * AX_B + u) * 64];
          ta[u] = ts[(j + 2) * AX_B + u];
        }
      }
#pragma unroll
      for (int u = 0; u < AX_B; u++) q[u] = rankmu_quot<kMarkstein>(tb[u], yb[u], s2, y);
#pragma unroll
      for (int u = 0; u < AX_B; u++) c += q[u];
    }
  } else {
    for (int u = 0; u < cnt; u++) c = rankmu_term<kMarkstein>(c, ts[u], ys[u * 64], s2, y);
  }
  return c;
}
template <bool kMarkstein>
__device__ __forceinline__ double rankmu_rows(double c, const double *__restrict__ Yc, const double *__restrict__ Tt,
                                              int N, int mu, int d0, int e0, int wid, int lane, double s2, double y,
                                              double (*Ys)[AX_K][64], double (*Ts)[4][AX_K]) {
  const int tid = threadIdx.x;
  // staging: thread t loads Yc[k0 + t/16 + 16 j][e0 + 4 (t%16) .. +3] for
  // j < 4 (16-B vector loads), and T[d0 + t/64][k0 + t%64]
  const int kr = tid >> 4, ec = (tid & 15) * 4;
  double2 yv[4][2];
  double tv = 0.0;
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int k = k0 + kr + 16 * j;
      const double *src = Yc + (size_t)(k < mu ? k : mu - 1) * N + e0 + ec;  // clamped rows are never summed
      if ((N & 1) == 0 && e0 + ec + 3 < N) {  // 16-B aligned rows
        yv[j][0] = *(const double2 *)src;
        yv[j][1] = *(const double2 *)(src + 2);
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) ((double *)&yv[j][0])[q] = (e0 + ec + q < N) ? src[q] : 0.0;
      }
    }
    const int dr = d0 + (tid >> 6), kk = k0 + (tid & 63);
    tv = (dr < N && kk < mu) ? Tt[(size_t)dr * mu + kk] : 0.0;
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      double *dst = &Ys[buf][kr + 16 * j][ec];
      *(double2 *)dst = yv[j][0];
      *(double2 *)(dst + 2) = yv[j][1];
    }
    Ts[buf][tid >> 6][tid & 63] = tv;
  };
  load(0);
  store(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < mu; k0 += AX_K) {
    const bool more = k0 + AX_K < mu;
    if (more) load(k0 + AX_K);  // in flight during the chunk below
    c = rankmu_chunk<kMarkstein>(c, &Ys[buf][0][lane], &Ts[buf][wid][0], min(AX_K, mu - k0), s2, y);
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  return c;
}

__global__ void __launch_bounds__(256) k_adaptC_exact2(int N, int mu, int diagonal, const double *__restrict__ Yc,
                                                       const double *__restrict__ Tt,
                                                       const double *__restrict__ pc, double *C,
                                                       const CmaesScalars *__restrict__ sc) {
  __shared__ __attribute__((aligned(16))) double Ys[2][AX_K][64];
  __shared__ double Ts[2][4][AX_K];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d0 = blockIdx.x * 4, e0 = blockIdx.y * 64;
  if (e0 > d0 + 3) return;  // workgroup-uniform: entirely above the diagonal
  const int d = d0 + wid, e = e0 + lane;
  const bool active = d < N && e < N && e <= d && (!diagonal || e == d);
  const double ccov1 = sc->ccov1, ccovmu = sc->ccovmu, cc = sc->cumulativeCovariance;
  const int hsig = (int)sc->hsig;
  const double s2 = sc->sigma * sc->sigma;
  double c = 0.0;
  if (active) {
    const double Cde = C[(size_t)d * N + e];
    c = (1 - ccov1 - ccovmu) * Cde + ccov1 * (pc[d] * pc[e] + (1 - hsig) * cc * (2. - cc) * Cde);
  }
  const int ex = (int)((__double_as_longlong(s2) >> 52) & 0x7ff) - 1023;
  if (__builtin_amdgcn_readfirstlane((int)(sc->rmuOutOfRange == 0u && ex >= -100 && ex <= 100)))
    c = rankmu_rows<true>(c, Yc, Tt, N, mu, d0, e0, wid, lane, s2, 1.0 / s2, Ys, Ts);
  else
    c = rankmu_rows<false>(c, Yc, Tt, N, mu, d0, e0, wid, lane, s2, 0.0, Ys, Ts);
  if (active) {
    C[(size_t)d * N + e] = c;
    if (e < d) C[(size_t)e * N + d] = c;
  }
}

// The same ordered sums with the chain split from its operands.  One
// workgroup per 4-row x 16-column tile of the lower triangle: wave 0 runs the
// 64 chains (one per lane, kc_add over quotients staged in LDS, one dependent
// add per term), waves 1..AX3_P form the next 64 quotients of every chain
// (Yc / T loads one chunk ahead, the Markstein quotient) meanwhile.  A single
// wave forming its own quotients issues five FP64 operations per term and is
// issue-bound well above the add latency; here the add chain is the bound.
// Tiles of 16-column block cb run on XCD cb % 8 (workgroup slot s -> XCD s % 8),
// so a column block of Yc is fetched from HBM into one L2.
// A workgroup barrier that orders LDS only: __syncthreads' release fence
// waits for every outstanding global load too (s_waitcnt vmcnt(0)), which
// would expose the prefetches issued for later chunks at every round
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n s_barrier" ::: "memory"); }
// row stride 73: odd (two-way bank pairs at most for the consumer's per-lane
// rows) and >= 70, so every producer slot p + 7 u (u < 10) stores without a
// branch (slots 64..69 are never summed)
constexpr int AX3_P = 7, AX3_K = 64, AX3_S = 73;  // producers, chunk, LDS row stride
__device__ __forceinline__ int ax3_tiles_in(int N, int cb) {  // row blocks of column block cb
  const int R = (N + 3) / 4, lo = 4 * cb;
  return R > lo ? R - lo : 0;
}
int ax3_slots(int N) {
  int mx = 0;
  for (int x = 0; x < 8; x++) {
    int cnt = 0;
    for (int cb = x; 16 * cb < N; cb += 8) cnt += std::max(0, (N + 3) / 4 - 4 * cb);
    mx = std::max(mx, cnt);
  }
  return 8 * mx;
}
template <bool kMarkstein>
__device__ __forceinline__ double ax3_run(double c, const double *__restrict__ Yc, const double *__restrict__ Tt,
                                          int N, int mu, int d0, int e0, int wid, int lane, double s2, double y,
                                          double (*Q)[64 * AX3_S + 16]) {
  const int r = lane >> 4, cc = lane & 15, d = d0 + r, e = e0 + cc;
  const bool rowok = d < N, colok = e < N;
  constexpr int KP = (AX3_K + AX3_P - 1) / AX3_P;  // quotients per producer lane per chunk
  double yA[KP], tA[KP], yB[KP], tB[KP];
  const int p = wid - 1;
  auto load = [&](int k0, double(&yv)[KP], double(&tv)[KP]) {
#pragma unroll
    for (int u = 0; u < KP; u++) {
      const int kl = p + AX3_P * u, k = k0 + kl;
      const bool ok = kl < AX3_K && k < mu;
      yv[u] = (ok && colok) ? Yc[(size_t)k * N + e] : 0.0;
      tv[u] = (ok && rowok) ? Tt[(size_t)d * mu + k] : 0.0;
    }
  };
  auto store = [&](int buf, const double(&yv)[KP], const double(&tv)[KP]) {
#pragma unroll
    for (int u = 0; u < KP; u++) {
      const int kl = p + AX3_P * u;
      Q[buf][lane * AX3_S + kl] = rankmu_quot<kMarkstein>(tv[u], yv[u], s2, y);
    }
  };
  auto chain = [&](int k0, int buf) {
    const int cnt = min(AX3_K, mu - k0), g = cnt >> 4;
    const double *row = &Q[buf][lane * AX3_S];
    c = chains::kc_add(c, lds_addr(row), __builtin_amdgcn_readfirstlane((unsigned)g));
    for (int u = 16 * g; u < cnt; u++) c += row[u];
  };
  // producers: in the round where wave 0 sums chunk k, the loads of chunk
  // k+2 are issued first, then chunk k+1's quotients are formed from the
  // registers its loads filled one round earlier (two register sets in
  // turn).  Producer and consumer waves run separate loops with the same
  // barrier count, so the compiler keeps each register set in place.
  if (wid > 0) {
    load(0, yA, tA);
    load(AX3_K, yB, tB);
    store(0, yA, tA);
    lds_barrier();
    for (int k0 = 0; k0 < mu; k0 += 2 * AX3_K) {
      load(k0 + 2 * AX3_K, yA, tA);  // (rows past mu load zeros)
      if (k0 + AX3_K < mu) store(1, yB, tB);
      lds_barrier();
      if (k0 + AX3_K >= mu) break;
      load(k0 + 3 * AX3_K, yB, tB);
      if (k0 + 2 * AX3_K < mu) store(0, yA, tA);
      lds_barrier();
    }
  } else {
    lds_barrier();
    for (int k0 = 0; k0 < mu; k0 += 2 * AX3_K) {
      chain(k0, 0);
      lds_barrier();
      if (k0 + AX3_K >= mu) break;
      chain(k0 + AX3_K, 1);
      lds_barrier();
    }
  }
  return c;
}
__global__ void __launch_bounds__(64 * (AX3_P + 1)) k_adaptC_exact3(int N, int mu, int diagonal,
                                                                    const double *__restrict__ Yc,
                                                                    const double *__restrict__ Tt,
                                                                    const double *__restrict__ pc, double *C,
                                                                    const CmaesScalars *__restrict__ sc) {
  __shared__ __attribute__((aligned(16))) double Q[2][64 * AX3_S + 16];
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  // slot -> (column block, row block)
  const int x = blockIdx.x & 7;
  int j = blockIdx.x >> 3, cb = x, rb = -1;
  for (; 16 * cb < N; cb += 8) {
    const int t = ax3_tiles_in(N, cb);
    if (j < t) {
      rb = 4 * cb + j;
      break;
    }
    j -= t;
  }
  if (rb < 0) return;  // workgroup-uniform: past this XCD's tiles
  const int d0 = 4 * rb, e0 = 16 * cb;
  const int d = d0 + (lane >> 4), e = e0 + (lane & 15);
  const bool active = wid == 0 && d < N && e < N && e <= d && (!diagonal || e == d);
  const double ccov1 = sc->ccov1, ccovmu = sc->ccovmu, cc = sc->cumulativeCovariance;
  const int hsig = (int)sc->hsig;
  const double s2 = sc->sigma * sc->sigma;
  double c = 0.0;
  if (active) {
    const double Cde = C[(size_t)d * N + e];
    c = (1 - ccov1 - ccovmu) * Cde + ccov1 * (pc[d] * pc[e] + (1 - hsig) * cc * (2. - cc) * Cde);
  }
  const int ex = (int)((__double_as_longlong(s2) >> 52) & 0x7ff) - 1023;
  if (__builtin_amdgcn_readfirstlane((int)(sc->rmuOutOfRange == 0u && ex >= -100 && ex <= 100)))
    c = ax3_run<true>(c, Yc, Tt, N, mu, d0, e0, wid, lane, s2, 1.0 / s2, Q);
  else
    c = ax3_run<false>(c, Yc, Tt, N, mu, d0, e0, wid, lane, s2, 0.0, Q);
  if (active) {
    C[(size_t)d * N + e] = c;
    if (e < d) C[(size_t)e * N + d] = c;
  }
}

// adaptC's exact rank-mu sums on ROW chains (round 4): every 16-lane row owns
// one element (d, e) of the lower triangle and runs its ordered chain
// c += fl(fl(T_kd Yc_ke) / s2) with kc_row16 (lane j of the row forms the
// quotient of term 16 g + j: one product + the Markstein quotient, then one
// DPP-broadcast add per term).  Workgroup = a 4 (d) x AR_TC (e) tile, one
// wave per 4 elements: wave w takes d0 + w / (AR_TC/4) and columns
// e0 + 4 (w % (AR_TC/4)) + row.  T rows and the Yc columns of the tile are
// staged through LDS in chunks of AR_K terms (transposed to term-contiguous
// rows), the next chunk's loads in flight.
// (AR_K = 256: a chunk's sums cover the next chunk's load latency; 128-term
// chunks left the kernel latency-bound, 34 us at C2)
// Round 6: AR_TC = 4 (4-wave workgroups; 8 before, the same 30.3 vs 30.4 us
// at C2).  What sets C2's 30 us is issue: one DPP-broadcast FP64 add per term
// for 4 elements + a quarter of a quotient, ~2 500 instructions per wave and
// 2 064 waves on 1 024 SIMDs.  Measured round 6 (profiles/r6/README.md): the
// next group's quotient interleaved into the adds (31.96 us), and quad chains
// (4 lanes per element, 32-bit quad_perm moves + plain adds, 46.9 us) do not
// beat it -- every split of 8 256 chains of 2 048 ordered terms over lanes
// leaves the busiest SIMD about 8 000 FP64 instructions.
#ifndef KG_AR_TC
#define KG_AR_TC 4
#endif
constexpr int AR_TC = KG_AR_TC, AR_NT = 64 * AR_TC, AR_K = 256, AR_KS = AR_K + 2, AR_TU = 4 * AR_K / AR_NT,
              AR_YU = AR_TC * AR_K / AR_NT;
static_assert(AR_TC == 4 || AR_TC == 8, "4 x 4 or 4 x 8 tiles");
__host__ __device__ inline int ar_row_blocks(int N) { return (N + 3) / 4; }
__host__ __device__ inline int ar_col_blocks_upto(int rb) { return (4 * rb + 3) / AR_TC + 1; }  // e0 <= d0 + 3
int ar_tiles(int N) {
  int t = 0;
  for (int rb = 0; rb < ar_row_blocks(N); rb++) t += std::min(ar_col_blocks_upto(rb), (N + AR_TC - 1) / AR_TC);
  return t;
}
template <bool kMarkstein>
__device__ __forceinline__ double ar_run(double acc, int N, int mu, int d0, int e0, int dl, int el,
                                         const double *__restrict__ Yc, const double *__restrict__ Tt, double s2,
                                         double (*Ts)[4][AR_KS], double (*Ys)[AR_TC][AR_KS]) {
  const int tid = threadIdx.x, j = tid & 15;
  const double y = kMarkstein ? 1.0 / s2 : 0.0;
  // staging: T rows d0..d0+3 (4 x AR_K) and Yc[k][e0..e0+AR_TC-1] (AR_K x AR_TC)
  double tv[AR_TU], yv[AR_YU];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < AR_TU; u++) {
      const int q = tid + AR_NT * u, r = q / AR_K;
      int kq = q % AR_K;
      asm volatile("" : "+v"(kq));  // (an opaque value: no SDWA byte-select form of `q % 256` in its uses)
      const int k = k0 + kq;
      tv[u] = (d0 + r < N && k < mu) ? Tt[(size_t)(d0 + r) * mu + k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < AR_YU; u++) {
      const int q = tid + AR_NT * u, k = k0 + q / AR_TC, c = q % AR_TC;
      yv[u] = (k < mu && e0 + c < N) ? Yc[(size_t)k * N + e0 + c] : 0.0;
    }
  };
  auto store = [&](int b) {
#pragma unroll
    for (int u = 0; u < AR_TU; u++) {
      const int q = tid + AR_NT * u;
      int kq = q % AR_K;
      asm volatile("" : "+v"(kq));
      Ts[b][q / AR_K][kq] = tv[u];
    }
#pragma unroll
    for (int u = 0; u < AR_YU; u++) {
      const int q = tid + AR_NT * u;
      Ys[b][q % AR_TC][q / AR_TC] = yv[u];
    }
  };
  load(0);
  store(0);
  __syncthreads();
  for (int k0 = 0, b = 0; k0 < mu; k0 += AR_K, b ^= 1) {
    const bool more = k0 + AR_K < mu;
    if (more) load(k0 + AR_K);
    const int gn = (min(AR_K, mu - k0) + 15) >> 4;  // (the tail's terms are 0 * 0 / s2 = +0.0)
    for (int g = 0; g < gn; g++) {
      const double pr = Ts[b][dl][16 * g + j] * Ys[b][el][16 * g + j];
      double q;
      if (kMarkstein) {
        const double q0 = pr * y;
        const double r = __builtin_fma(-q0, s2, pr);
        q = __builtin_fma(r, y, q0);
      } else {
        q = pr / s2;
      }
      acc = chains::kc_row16(acc, q);
    }
    if (more) store(b ^ 1);
    __syncthreads();
  }
  return acc;
}
// tbase: the first tile of this launch (a population-sharded rank computes
// its share [tbase, tbase + gridDim.x) of the tiles); pack != nullptr: the
// lower-triangle results go to pack[d (d + 1) / 2 + e] (the sharded
// exchange buffer, "Shard Covariance") instead of C, entries that adaptC
// leaves unchanged (diagonal covariance) with their old value
__global__ void __launch_bounds__(AR_NT) k_adaptC_row(int N, int mu, int diagonal, const double *__restrict__ Yc,
                                                    const double *__restrict__ Tt, const double *__restrict__ pc,
                                                    double *C, const CmaesScalars *__restrict__ sc, int tbase,
                                                    double *__restrict__ pack) {
  __shared__ double Ts[2][4][AR_KS];
  __shared__ double Ys[2][AR_TC][AR_KS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row = lane >> 4, j = lane & 15;
  // tile index -> (row block, column block), row blocks in order
  int t = blockIdx.x + tbase, rb = 0;
  const int ncb = (N + AR_TC - 1) / AR_TC;
  for (;; rb++) {
    const int c = min(ar_col_blocks_upto(rb), ncb);
    if (t < c) break;
    t -= c;
  }
  const int d0 = 4 * rb, e0 = AR_TC * t;
  const int dl = wid / (AR_TC / 4), el = 4 * (wid % (AR_TC / 4)) + row;
  const int d = d0 + dl, e = e0 + el;
  const bool active = d < N && e < N && e <= d && (!diagonal || e == d);
  const double ccov1 = sc->ccov1, ccovmu = sc->ccovmu, cc = sc->cumulativeCovariance;
  const int hsig = (int)sc->hsig;
  const double s2 = sc->sigma * sc->sigma;
  double acc = 0.0;
  if (active) {
    const double Cde = C[(size_t)d * N + e];
    acc = (1 - ccov1 - ccovmu) * Cde + ccov1 * (pc[d] * pc[e] + (1 - hsig) * cc * (2. - cc) * Cde);
  }
  const int ex = (int)((__double_as_longlong(s2) >> 52) & 0x7ff) - 1023;
  if (__builtin_amdgcn_readfirstlane((int)(sc->rmuOutOfRange == 0u && ex >= -100 && ex <= 100)))
    acc = ar_run<true>(acc, N, mu, d0, e0, dl, el, Yc, Tt, s2, Ts, Ys);
  else
    acc = ar_run<false>(acc, N, mu, d0, e0, dl, el, Yc, Tt, s2, Ts, Ys);
  if (pack) {
    if (j == 0 && d < N && e <= d) pack[(size_t)d * (d + 1) / 2 + e] = active ? acc : C[(size_t)d * N + e];
    return;
  }
  if (active && j == 0) {
    C[(size_t)d * N + e] = acc;
    if (e < d) C[(size_t)e * N + d] = acc;
  }
}

// adaptC's exact rank-mu sums on LANE chains (round 5): every lane owns one
// element (d, e) of the lower triangle and runs its whole ordered chain
// c += fl(fl(T_kd Yc_ke) / s2) itself -- the same terms, quotients and
// order as k_adaptC_row, so the same bits.  A workgroup is a 16 x 16 tile
// (d0 + t/16, e0 + t%16) of the lower triangle; T rows and Yc columns are
// staged through LDS 64 terms at a time, the next chunk's loads in flight.
// Per term a wave issues five instructions for 64 elements (the row form: 20
// for 4 elements x 16 terms, its quotients shared out by 16 DPP-broadcast
// adds), and a tile reads 32 operand streams for 256 elements (the row form:
// 12 for 32): C4's 131 328 chains of 32 768 terms are issue-bound instead of
// chain-latency-bound, and the tiles re-read a third of the operands.
// Round 6: both staged operands are held term-contiguous ([row][term], rows
// padded to 66 doubles so the 16 rows a ds_read_b128 lane group touches start
// in distinct bank quads) and read two terms per ds_read_b128: 4 LDS-array
// cycles per wave and term instead of 8 for the [term][row] images, whose
// paired reads the compiler merged into ds_read2_b64 (8 cycles per pair).
// At C4 the busiest CUs hold three tiles (528 tiles on 256 CUs), so the LDS
// array, not the FP64 issue, had set the kernel's time.
#ifndef KG_AL_K
#define KG_AL_K 64
#endif
constexpr int AL_T = 16, AL_K = KG_AL_K, AL_KP = AL_K + 2;  // (64-term chunks: 34 KB of LDS, four workgroups per CU)
static_assert(AL_K % 2 == 0, "two terms per ds_read_b128");
__host__ __device__ inline int al_blocks(int N) { return (N + AL_T - 1) / AL_T; }
int al_tiles(int N) { return al_blocks(N) * (al_blocks(N) + 1) / 2; }
template <bool kMarkstein>
__device__ __forceinline__ void al_run(int N, int mu, int diagonal, const double *__restrict__ Yc,
                                       const double *__restrict__ Tt, const double *__restrict__ pc, double *C,
                                       const CmaesScalars *__restrict__ sc, int tbase, double *__restrict__ pack,
                                       double (*Ts)[AL_T][AL_KP], double (*Ys)[AL_T][AL_KP]) {
  const int tid = threadIdx.x, dl = tid >> 4, el = tid & 15;
  // tile -> (row block bd, column block be <= bd), row blocks in order (an
  // XCD-grouped order measured the same at C4, round 5: 1.97 vs 1.99 ms)
  int t = blockIdx.x + tbase, bd = 0;
  while (t > bd) t -= ++bd;
  const int d0 = AL_T * bd, e0 = AL_T * t;
  const int d = d0 + dl, e = e0 + el;
  const bool active = d < N && e <= d && (!diagonal || e == d);
  const double ccov1 = sc->ccov1, ccovmu = sc->ccovmu, cc = sc->cumulativeCovariance;
  const int hsig = (int)sc->hsig;
  const double s2 = sc->sigma * sc->sigma, y = kMarkstein ? 1.0 / s2 : 0.0;
  double acc = 0.0;
  if (active) {
    const double Cde = C[(size_t)d * N + e];
    acc = (1 - ccov1 - ccovmu) * Cde + ccov1 * (pc[d] * pc[e] + (1 - hsig) * cc * (2. - cc) * Cde);
  }
  // staging: T rows d0..d0+15 and Yc[k][e0..e0+15], both as [row][term]
  constexpr int U = AL_T * AL_K / 256;  // 4 values of each per thread
  double tv[U], yv[U];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = tid + 256 * u, r = q / AL_K, kq = q % AL_K, k = k0 + kq;
      tv[u] = (d0 + r < N && k < mu) ? Tt[(size_t)(d0 + r) * mu + k] : 0.0;
      const int kk = k0 + (q >> 4), c = q & 15;
      yv[u] = (kk < mu && e0 + c < N) ? Yc[(size_t)kk * N + e0 + c] : 0.0;
    }
  };
  auto store = [&](int b) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = tid + 256 * u;
      Ts[b][q / AL_K][q % AL_K] = tv[u];
      Ys[b][q & 15][q >> 4] = yv[u];
    }
  };
  auto quot = [&](double pr) __attribute__((always_inline)) {
    if (kMarkstein) {
      const double q0 = pr * y;
      const double r = __builtin_fma(-q0, s2, pr);
      return __builtin_fma(r, y, q0);
    }
    return pr / s2;
  };
  load(0);
  store(0);
  __syncthreads();
  for (int k0 = 0, b = 0; k0 < mu; k0 += AL_K, b ^= 1) {
    const bool more = k0 + AL_K < mu;
    if (more) load(k0 + AL_K);
    const int kn = min(AL_K, mu - k0);
    const double2 *tr = reinterpret_cast<const double2 *>(&Ts[b][dl][0]);
    const double2 *yr = reinterpret_cast<const double2 *>(&Ys[b][el][0]);
    int k = 0;
    // the next 8 terms' reads issued before this 8's adds (the index clamped
    // into the row on the last pass): two or three waves per SIMD do not
    // cover an LDS round trip per group
    double2 tp[4], yp[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      tp[u] = tr[u];
      yp[u] = yr[u];
    }
    for (; k + 8 <= kn; k += 8) {
      double q[8];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        q[2 * u] = quot(tp[u].x * yp[u].x);
        q[2 * u + 1] = quot(tp[u].y * yp[u].y);
      }
      const int nk = min(k + 8, AL_K - 8);
#pragma unroll
      for (int u = 0; u < 4; u++) {
        tp[u] = tr[nk / 2 + u];
        yp[u] = yr[nk / 2 + u];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) acc += q[u];
    }
    for (; k < kn; k++) acc += quot(Ts[b][dl][k] * Ys[b][el][k]);
    if (more) store(b ^ 1);
    __syncthreads();
  }
  if (pack) {
    if (d < N && e <= d) pack[(size_t)d * (d + 1) / 2 + e] = active ? acc : C[(size_t)d * N + e];
    return;
  }
  if (active) {
    C[(size_t)d * N + e] = acc;
    if (e < d) C[(size_t)e * N + d] = acc;
  }
}
__global__ void __launch_bounds__(256) k_adaptC_lane(int N, int mu, int diagonal, const double *__restrict__ Yc,
                                                     const double *__restrict__ Tt, const double *__restrict__ pc,
                                                     double *C, const CmaesScalars *__restrict__ sc, int tbase,
                                                     double *__restrict__ pack) {
  __shared__ __attribute__((aligned(16))) double Ts[2][AL_T][AL_KP], Ys[2][AL_T][AL_KP];  // [d - d0][term] / [e - e0][term]
  // Markstein quotients when every factor is in range (as k_adaptC_row)
  const double s2 = sc->sigma * sc->sigma;
  const int ex = (int)((__double_as_longlong(s2) >> 52) & 0x7ff) - 1023;
  if (__builtin_amdgcn_readfirstlane((int)(sc->rmuOutOfRange == 0u && ex >= -100 && ex <= 100)))
    al_run<true>(N, mu, diagonal, Yc, Tt, pc, C, sc, tbase, pack, Ts, Ys);
  else
    al_run<false>(N, mu, diagonal, Yc, Tt, pc, C, sc, tbase, pack, Ts, Ys);
}

// mean :603-609 and mean update :623-624.  The sum over the μ selected rows
// is sequential per d (the reference's order); a workgroup owns MN_D columns:
// all its threads stream the products w_i Y[i][d] into LDS, 256 rows at a
// time (next chunk loaded while the current one is summed), and MN_D lanes
// of wave 0 add them in order (an add-only chain at the FP64 add latency).
constexpr int MN_D = 8, MN_R = 256;
// the gradient-informed mean step (CMAES.cpp.base:611-621), after k_mean:
// mean_d += ((w_i step) / sqrt(N)) g_(i),d in selection order, then the
// mean update again
__global__ void k_mean_gradient(int N, int mu, double step, const double *__restrict__ G,
                                const unsigned *__restrict__ idx, const double *__restrict__ w, double *mean,
                                const double *__restrict__ prevMean, double *meanUpdate,
                                const CmaesScalars *__restrict__ sc) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= N) return;
  const double rn = sqrt((double)N);
  double acc = mean[d];
  for (int i = 0; i < mu; i++) acc += w[i] * step / rn * G[(size_t)idx[i] * N + d];
  mean[d] = acc;
  meanUpdate[d] = (acc - prevMean[d]) / sc->sigma;
}

__global__ void __launch_bounds__(256) k_mean(int N, int mu, const double *__restrict__ Y,
                                              const double *__restrict__ w, double *mean, double *prevMean,
                                              double *meanUpdate, const CmaesScalars *__restrict__ sc) {
  __shared__ double buf[2][MN_R][MN_D + 1];
  const int tid = threadIdx.x;
  const int d0 = blockIdx.x * MN_D;
  const int nd = (N - d0) < MN_D ? (N - d0) : MN_D;
  const int nchunks = (mu + MN_R - 1) / MN_R;
  double v[8];
  auto fetch = [&](int chunk) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int e = tid + 256 * u, r = e >> 3, c = e & 7, i = chunk * MN_R + r;
      v[u] = (i < mu && c < nd) ? w[i] * Y[(size_t)i * N + d0 + c] : 0.0;
    }
  };
  auto put = [&](int b) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int e = tid + 256 * u;
      buf[b][e >> 3][e & 7] = v[u];
    }
  };
  fetch(0);
  put(0);
  __syncthreads();
  double acc = 0.;
  for (int ch = 0; ch < nchunks; ch++) {
    if (ch + 1 < nchunks) fetch(ch + 1);
    if (tid < nd) {
      const int rn = (mu - ch * MN_R) < MN_R ? (mu - ch * MN_R) : MN_R;
      const double(*bb)[MN_D + 1] = buf[ch & 1];
      int r = 0;
      for (; r + 8 <= rn; r += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) t[u] = bb[r + u][tid];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += t[u];
      }
      for (; r < rn; r++) acc += bb[r][tid];
    }
    if (ch + 1 < nchunks) put((ch + 1) & 1);
    __syncthreads();
  }
  if (tid < nd) {
    const int d = d0 + tid;
    const double prev = prevMean[d];  // copied by k_gather_selected
    mean[d] = acc;
    meanUpdate[d] = (acc - prev) / sc->sigma;
  }
}

// k_mean on the chain primitive: lane c of wave 0 adds w_i y_(i),d0+c in
// selection order (kc_add: ~15 cycles per product); waves 1-3 stage the next
// MN2_R products of the 8 dimensions into the other half of a double-buffered
// LDS ring (transposed: dimension-major, zero past mu) while the chain runs.
constexpr int MN2_R = 1024, MN2_RS = MN2_R + 32;  // rows per chunk; row stride (the chain reads up to 31 ahead)
size_t mean2_lds_bytes() { return 2 * (size_t)MN_D * MN2_RS * sizeof(double); }
__global__ void __launch_bounds__(256) k_mean2(int N, int mu, const double *__restrict__ Y,
                                               const double *__restrict__ w, double *mean, double *prevMean,
                                               double *meanUpdate, const CmaesScalars *__restrict__ sc) {
  extern __shared__ __attribute__((aligned(16))) double pbuf[];  // [2][MN_D][MN2_RS]
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int d0 = blockIdx.x * MN_D;
  const int nd = (N - d0) < MN_D ? (N - d0) : MN_D;
  const int nchunks = (mu + MN2_R - 1) / MN2_R;
  // eight products' loads in flight per thread (one at a time, each round
  // trip to L2/HBM would be exposed: the staging, not the chain, was the bound)
  auto stage = [&](int chunk, int t0, int nt) {
    double *b = pbuf + (size_t)(chunk & 1) * MN_D * MN2_RS;
    for (int e0 = t0; e0 < MN_D * MN2_R; e0 += 8 * nt) {
      double wv[8], yv[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int e = e0 + u * nt, r = e >> 3, c = e & 7, i = chunk * MN2_R + r;
        const bool ok = e < MN_D * MN2_R && i < mu && c < nd;
        wv[u] = ok ? w[i] : 0.0;
        yv[u] = ok ? Y[(size_t)i * N + d0 + c] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int e = e0 + u * nt, r = e >> 3, c = e & 7;
        if (e < MN_D * MN2_R) b[(size_t)c * MN2_RS + r] = wv[u] * yv[u];
      }
    }
  };
  stage(0, tid, 256);
  __syncthreads();
  double acc = 0.0;
  const int c = lane < nd ? lane : 0;
  for (int ch = 0; ch < nchunks; ch++) {
    if (wid == 0) {
      const int rn = min(MN2_R, mu - ch * MN2_R);
      const double *b = pbuf + (size_t)(ch & 1) * MN_D * MN2_RS + (size_t)c * MN2_RS;
      acc = chains::kc_add(acc, lds_addr(b), __builtin_amdgcn_readfirstlane((unsigned)(rn + 15) >> 4));
    } else if (ch + 1 < nchunks) {
      stage(ch + 1, tid - 64, 192);
    }
    __syncthreads();
  }
  if (wid == 0 && lane < nd) {
    const int d = d0 + lane;
    const double prev = prevMean[d];  // copied by k_gather_selected
    mean[d] = acc;
    meanUpdate[d] = (acc - prev) / sc->sigma;
  }
}

// k_mean on ROW chains (round 4): every 16-lane row of a wave owns one
// dimension d and runs its ordered chain mean_d = sum_i w_i y_(i),d with
// kc_row16 (one v_fmac_f64 DPP broadcast per element: lane j of the row holds
// the product of element 16 g + j); four chains per wave, sixteen per
// workgroup.  The selected rows are staged through LDS in chunks of MR_K
// (coalesced 16-dimension row segments in, dimension-major out), the next
// chunk's loads in flight while the current one is summed.
// (MR_K = 256: one chunk's sum, 256 x ~9 cycles, covers the next chunk's
// load latency, which 128-term chunks did not: 20 us at C2)
constexpr int MR_K = 256, MR_KS = MR_K + 2, MR_U = MR_K * 16 / 256;
__global__ void __launch_bounds__(256) k_mean3(int N, int mu, const double *__restrict__ Y,
                                               const double *__restrict__ w, double *mean,
                                               const double *__restrict__ prevMean, double *meanUpdate,
                                               const CmaesScalars *__restrict__ sc) {
  __shared__ double ys[2][16][MR_KS];
  __shared__ double ws[2][MR_K];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row = lane >> 4, j = lane & 15, dl = 4 * wid + row;
  const int d0 = blockIdx.x * 16;
  const int nch = (mu + MR_K - 1) / MR_K;
  // the epilogue's operands, read now rather than after the chain
  const double pmd = (j == 0 && d0 + dl < N) ? prevMean[d0 + dl] : 0.0, sig = sc->sigma;
  // chunk loads: 256 threads x MR_U values of the (MR_K x 16) block, + w
  double ld[MR_U], wl = 0.0;
  auto load = [&](int ch) {
#pragma unroll
    for (int u = 0; u < MR_U; u++) {
      const int q = tid + 256 * u, k = q >> 4, c = q & 15, i = ch * MR_K + k;
      ld[u] = (i < mu && d0 + c < N) ? Y[(size_t)i * N + d0 + c] : 0.0;
    }
    const int i = ch * MR_K + tid;
    wl = (tid < MR_K && i < mu) ? w[i] : 0.0;
  };
  auto store = [&](int b) {
#pragma unroll
    for (int u = 0; u < MR_U; u++) {
      const int q = tid + 256 * u, k = q >> 4, c = q & 15;
      ys[b][c][k] = ld[u];
    }
    if (tid < MR_K) ws[b][tid] = wl;
  };
  load(0);
  store(0);
  __syncthreads();
  double acc = 0.0;
  for (int ch = 0; ch < nch; ch++) {
    const int b = ch & 1;
    if (ch + 1 < nch) load(ch + 1);
    const int gn = min(MR_K, mu - ch * MR_K + 15) >> 4;  // groups of 16 (the tail is zero-padded)
    // (a software-pipelined form -- group g + 1's product and g + 2's LDS
    // reads issued right after group g's adds -- measured slower here and in
    // k_adaptC_row, round 6: 50.0 / 40.9 against 48.0 / 36.3 us)
    for (int g = 0; g < gn; g++) {
      const double q = ws[b][16 * g + j] * ys[b][dl][16 * g + j];  // the product, rounded, then added
      acc = chains::kc_row16(acc, q);
    }
    if (ch + 1 < nch) store(b ^ 1);
    __syncthreads();
  }
  const int d = d0 + dl;
  if (j == 0 && d < N) {
    mean[d] = acc;
    meanUpdate[d] = (acc - pmd) / sig;  // (prevMean: copied by k_gather_selected / k_select_prep)
  }
}

// evolution paths for N <= 128 on ROW chains (round 4): one 1024-thread
// workgroup, 64 row chains per layer (16 waves x 4 rows; two passes at
// N = 128).  Every B value the two layers read is loaded at the start
// (layer 1: columns of B, layer 2: rows), so the only waits between them
// are the workgroup barriers.
constexpr int PR_T = 1024;
__global__ void __launch_bounds__(PR_T) k_paths3(int N, unsigned long long gen, const double *__restrict__ B,
                                                 const double *__restrict__ D, const double *__restrict__ meanUpdate,
                                                 double *auxBDZ, double *ps, double *pc, CmaesScalars *sc) {
  __shared__ double mu_s[128 + 16], aux_s[128 + 16], pn_s[128 + 16];
  __shared__ int hs;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row = lane >> 4, j = lane & 15;
  const double cs = sc->sigmaCumulationFactor, effMu = sc->effectiveMu, cc = sc->cumulativeCovariance;
  // every other operand read up front with B (one round of loads, not one per phase)
  const double chi = sc->chiSquareNumber, hpGen = sc->hsigPowGen, hpCs = sc->hsigPowCs, hp = sc->hsigPow;
  const double pcq = tid < N ? pc[tid] : 0.0, muq = tid < N ? meanUpdate[tid] : 0.0;
  double Dd[2], psd[2];
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const int d = 64 * p + 4 * wid + row;
    Dd[p] = (j == 0 && d < N) ? D[d] : 1.0;
    psd[p] = (j == 0 && d < N) ? ps[d] : 0.0;
  }
  const int G = (N + 15) >> 4;  // groups of 16 along e
  // chains of this lane's rows: d = 64 p + 4 wid + row, p = 0, 1
  double b1[2][8], b2[2][8];
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const int d = 64 * p + 4 * wid + row;
#pragma unroll
    for (int g = 0; g < 8; g++) {
      const int e = 16 * g + j;
      const bool ok = d < N && e < N;
      b1[p][g] = ok ? B[(size_t)e * N + d] : 0.0;  // B[e][d]: aux = D^-1 B^T mu   (:627-636)
      b2[p][g] = ok ? B[(size_t)d * N + e] : 0.0;  // B[d][e]: B aux               (:641-651)
    }
  }
  for (int q = tid; q < 128 + 16; q += PR_T) {
    mu_s[q] = q < N ? meanUpdate[q] : 0.0;
    pn_s[q] = 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const int d = 64 * p + 4 * wid + row;
    if (64 * p + 4 * wid >= N) break;  // (wave-uniform)
    double acc = 0.0;
#pragma unroll
    for (int g = 0; g < 8; g++)
      if (g < G) acc = chains::kc_row16(acc, b1[p][g] * mu_s[16 * g + j]);
    if (j == 0 && d < N) {
      const double a = acc / Dd[p];
      aux_s[d] = a;
      auxBDZ[d] = a;
    }
  }
  if (tid >= N && tid < 128 + 16) aux_s[tid] = 0.0;
  __syncthreads();
  const double fac = sqrt(cs * (2. - cs) * effMu);
#pragma unroll
  for (int p = 0; p < 2; p++) {
    const int d = 64 * p + 4 * wid + row;
    if (64 * p + 4 * wid >= N) break;
    double acc = 0.0;
#pragma unroll
    for (int g = 0; g < 8; g++)
      if (g < G) acc = chains::kc_row16(acc, b2[p][g] * aux_s[16 * g + j]);
    if (j == 0 && d < N) {
      const double pv = (1. - cs) * psd[p] + fac * acc;
      ps[d] = pv;
      pn_s[d] = pv * pv;  // std::pow(x, 2.0) == x*x (CR)
    }
  }
  __syncthreads();
  if (wid == 0) {
    double q[8];
#pragma unroll
    for (int k = 0; k < 8; k++) q[k] = pn_s[16 * k + (lane & 15)];
    const double nrm2 = chains::kc_add_dpp(0.0, q, __builtin_amdgcn_readfirstlane((unsigned)G));
    if (lane == 0) {
      const double nrm = sqrt(nrm2);
      sc->psNorm = nrm;
      const double hpw = (hpGen == (double)gen && hpCs == cs) ? hp : pow_cr(1. - cs, 2.0 * (1.0 + (double)gen));
      const int hsig = (1.4 + 2.0 / (N + 1) > nrm / sqrt(1. - hpw) / chi);
      hs = hsig;
      sc->hsig = hsig;
      const double a = N + 1.3, b = N + 2.0;
      const double ccov1 = 2.0 / (a * a + effMu);
      double ccovmu = 2.0 * (effMu - 2. + 1. / effMu) / (b * b + effMu);
      if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
      sc->ccov1 = ccov1;
      sc->ccovmu = ccovmu;
    }
  }
  __syncthreads();
  const double fac2 = sqrt(cc * (2. - cc) * effMu);
  if (tid < N) pc[tid] = (1. - cc) * pcq + hs * fac2 * muq;  // (N <= 128 < PR_T)
}

// evolution paths for N <= 128 (full covariance): B staged once in LDS (row
// stride 129: column and row walks both conflict-free), the two ordered
// matrix-vector chains and the |p_sigma| chain on the chain primitives.
constexpr int PA2_LD = 129;
// (the vectors start 16-byte aligned: kc_lock_asc reads w in pairs)
__host__ __device__ inline size_t paths2_vec(int N) { return ((size_t)N + 33) & ~(size_t)1; }
__host__ __device__ inline size_t paths2_bs(int N) { return ((size_t)(N + 16) * PA2_LD + 1) & ~(size_t)1; }
size_t paths2_lds_bytes(int N) { return (paths2_bs(N) + 3 * paths2_vec(N)) * sizeof(double); }
__global__ void __launch_bounds__(256) k_paths2(int N, unsigned long long gen, const double *__restrict__ B,
                                                const double *__restrict__ D, const double *__restrict__ meanUpdate,
                                                double *auxBDZ, double *ps, double *pc, CmaesScalars *sc) {
  extern __shared__ __attribute__((aligned(16))) double psm[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  double *Bs = psm;                                // (N+16) x 129, zero padded
  double *sv = Bs + paths2_bs(N);                  // mean update, zero past N
  double *aux = sv + paths2_vec(N);                // D^-1 B^T (mean update), zero past N
  double *pn = aux + paths2_vec(N);                // p_sigma squares, zero past N
  __shared__ int hs;
  const double cs = sc->sigmaCumulationFactor, effMu = sc->effectiveMu, cc = sc->cumulativeCovariance;
  // eight loads in flight per thread (one at a time, the L2 round trips were the kernel's time)
  for (int q0 = tid; q0 < (N + 16) * PA2_LD; q0 += 8 * 256) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = q0 + u * 256, e = q / PA2_LD, d = q - e * PA2_LD;
      v[u] = (q < (N + 16) * PA2_LD && e < N && d < N) ? B[(size_t)e * N + d] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = q0 + u * 256;
      if (q < (N + 16) * PA2_LD) Bs[q] = v[u];
    }
  }
  for (int q = tid; q < 3 * (int)paths2_vec(N); q += 256) sv[q] = (q < N) ? meanUpdate[q] : 0.0;
  __syncthreads();
  const unsigned nb = __builtin_amdgcn_readfirstlane((unsigned)(N + 7) >> 3);
  const int d = lane + 64 * (wid & 1);  // waves 0-1: rows d < 128
  // aux[d] = (sum_e B[e][d] mu[e]) / D[d]   (CMAES.cpp.base:627-636)
  if (wid < 2) {
    const double a1 = chains::kc_lock_asc<PA2_LD * 8>(0.0, lds_addr(sv), lds_addr(Bs + d), nb);
    if (d < N) {
      const double a = a1 / D[d];
      aux[d] = a;
      auxBDZ[d] = a;
    }
  }
  __syncthreads();
  // p_sigma = (1-c_s) p_sigma + sqrt(c_s (2-c_s) mu_eff) sum_e B[d][e] aux[e]   (:641-656)
  const double fac = sqrt(cs * (2. - cs) * effMu);
  if (wid < 2) {
    const double sum = chains::kc_lock_asc<8>(0.0, lds_addr(aux), lds_addr(Bs + (size_t)d * PA2_LD), nb);
    if (d < N) {
      const double p = (1. - cs) * ps[d] + fac * sum;
      ps[d] = p;
      pn[d] = p * p;  // std::pow(x, 2.0) == x*x (CR)
    }
  }
  __syncthreads();
  if (wid == 0) {
    const double nrm2 = chains::kc_add(0.0, lds_addr(pn), __builtin_amdgcn_readfirstlane((unsigned)(N + 15) >> 4));
    if (lane == 0) {
      const double nrm = sqrt(nrm2);
      sc->psNorm = nrm;
      const int hsig = (1.4 + 2.0 / (N + 1) > nrm / sqrt(1. - hsig_pow(sc, cs, gen)) /
                                                   sc->chiSquareNumber);
      hs = hsig;
      sc->hsig = hsig;
      const double a = N + 1.3, b = N + 2.0;
      const double ccov1 = 2.0 / (a * a + effMu);
      double ccovmu = 2.0 * (effMu - 2. + 1. / effMu) / (b * b + effMu);
      if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
      sc->ccov1 = ccov1;
      sc->ccovmu = ccovmu;
    }
  }
  __syncthreads();
  const double fac2 = sqrt(cc * (2. - cc) * effMu);
  for (int q = tid; q < N; q += 256) pc[q] = (1. - cc) * pc[q] + hs * fac2 * meanUpdate[q];
}

// evolution paths :626-662 (+ the adaptC constants :693-694).  Both
// matrix-vector products keep the reference's sequential e-order per output;
// B is staged through LDS in column chunks so row sweeps stay coalesced.
constexpr int PA_EC = 16;
__global__ void __launch_bounds__(1024) k_paths(int N, int diagonal, unsigned long long gen,
                                                const double *__restrict__ B, const double *__restrict__ D,
                                                const double *__restrict__ meanUpdate, double *auxBDZ, double *ps,
                                                double *pc, CmaesScalars *sc) {
  extern __shared__ __attribute__((aligned(16))) double psm[];
  double *tile = psm;                       // N x (PA_EC+1)
  double *sv = psm + (size_t)N * (PA_EC + 1);  // N: mean update, then aux, then ps
  __shared__ int hs;
  const int tid = threadIdx.x;
  const double cs = sc->sigmaCumulationFactor, effMu = sc->effectiveMu, cc = sc->cumulativeCovariance;
  for (int d = tid; d < N; d += blockDim.x) sv[d] = meanUpdate[d];
  __syncthreads();
  // aux[d] = (sum_e B[e][d] mu[e]) / D[d]   (column sweep: coalesced)
  double a1 = 0.0;
  if (tid < N) {
    if (diagonal)
      a1 = sv[tid];
    else
      for (int e = 0; e < N; ++e) a1 += B[(size_t)e * N + tid] * sv[e];
    a1 = a1 / D[tid];
  }
  __syncthreads();
  if (tid < N) {
    sv[tid] = a1;
    auxBDZ[tid] = a1;
  }
  __syncthreads();
  // sum_e B[d][e] aux[e]   (row sweep through LDS chunks)
  double sum = 0.0;
  if (diagonal) {
    if (tid < N) sum = sv[tid];
  } else {
    for (int e0 = 0; e0 < N; e0 += PA_EC) {
      const int en = (N - e0) < PA_EC ? (N - e0) : PA_EC;
      for (int q = tid; q < N * PA_EC; q += blockDim.x) {
        const int d = q / PA_EC, ee = q % PA_EC;
        tile[d * (PA_EC + 1) + ee] = (ee < en) ? B[(size_t)d * N + e0 + ee] : 0.0;
      }
      __syncthreads();
      if (tid < N)
        for (int ee = 0; ee < en; ++ee) sum += tile[tid * (PA_EC + 1) + ee] * sv[e0 + ee];
      __syncthreads();
    }
  }
  const double fac = sqrt(cs * (2. - cs) * effMu);
  if (tid < N) {
    const double p = (1. - cs) * ps[tid] + fac * sum;
    ps[tid] = p;
    tile[tid] = p;
  }
  __syncthreads();
  if (tid == 0) {
    double nrm = 0.0;
    for (int d = 0; d < N; ++d) nrm += tile[d] * tile[d];  // std::pow(x, 2.0) == x*x (CR)
    nrm = sqrt(nrm);
    sc->psNorm = nrm;
    const int hsig = (1.4 + 2.0 / (N + 1) > nrm / sqrt(1. - hsig_pow(sc, cs, gen)) /
                                                 sc->chiSquareNumber);
    hs = hsig;
    sc->hsig = hsig;
    const double a = N + 1.3, b = N + 2.0;
    const double ccov1 = 2.0 / (a * a + effMu);
    double ccovmu = 2.0 * (effMu - 2. + 1. / effMu) / (b * b + effMu);
    if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
    sc->ccov1 = ccov1;
    sc->ccovmu = ccovmu;
  }
  __syncthreads();
  const double fac2 = sqrt(cc * (2. - cc) * effMu);
  for (int d = tid; d < N; d += blockDim.x) pc[d] = (1. - cc) * pc[d] + hs * fac2 * meanUpdate[d];
}

// adaptC :690-707, exact: one thread per lower-triangle element, the rank-μ
// sum sequential over k exactly as the reference evaluates it.
constexpr int AC_T = 16, AC_K = 64;
__device__ inline void tri_tile(int t, int &td, int &te) {
  int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) / 2.0);
  while ((r + 1) * (r + 2) / 2 <= t) r++;
  while (r * (r + 1) / 2 > t) r--;
  td = r;
  te = t - r * (r + 1) / 2;
}

__global__ void __launch_bounds__(256) k_adaptC_exact(int N, int mu, int diagonal, const double *__restrict__ X,
                                                      const unsigned *__restrict__ idx, const double *__restrict__ w,
                                                      const double *__restrict__ prevMean,
                                                      const double *__restrict__ pc, double *C,
                                                      const CmaesScalars *__restrict__ sc) {
  __shared__ double Yd[AC_K][AC_T], Ye[AC_K][AC_T], cw[AC_K];
  int td, te;
  tri_tile(blockIdx.x, td, te);
  const int tid = threadIdx.x, ty = tid / AC_T, tx = tid % AC_T;
  const int d = td * AC_T + ty, e = te * AC_T + tx;
  const bool active = (d < N && e < N && e <= d && (!diagonal || e == d));
  const double ccov1 = sc->ccov1, ccovmu = sc->ccovmu, cc = sc->cumulativeCovariance;
  const int hsig = (int)sc->hsig;
  const double sigmasquare = sc->sigma * sc->sigma;
  double c = 0.0;
  if (active) {
    const double Cde = C[(size_t)d * N + e];
    c = (1 - ccov1 - ccovmu) * Cde + ccov1 * (pc[d] * pc[e] + (1 - hsig) * cc * (2. - cc) * Cde);
  }
  for (int k0 = 0; k0 < mu; k0 += AC_K) {
    const int kn = (mu - k0) < AC_K ? (mu - k0) : AC_K;
    for (int q = tid; q < AC_K * AC_T; q += 256) {
      const int kk = q / AC_T, cidx = q % AC_T;
      double yd = 0.0, ye = 0.0;
      if (kk < kn) {
        const size_t row = (size_t)(k0 + kk) * N;  // Y row k = X[idx[k]]
        const int dd = td * AC_T + cidx, ee = te * AC_T + cidx;
        if (dd < N) yd = X[row + dd] - prevMean[dd];
        if (ee < N) ye = X[row + ee] - prevMean[ee];
      }
      Yd[kk][cidx] = yd;
      Ye[kk][cidx] = ye;
    }
    for (int q = tid; q < kn; q += 256) cw[q] = ccovmu * w[k0 + q];
    __syncthreads();
    if (active)
      for (int kk = 0; kk < kn; kk++) c += cw[kk] * Yd[kk][ty] * Ye[kk][tx] / sigmasquare;
    __syncthreads();
  }
  if (active) {
    C[(size_t)d * N + e] = c;
    if (e < d) C[(size_t)e * N + d] = c;
  }
}

// adaptC with the rank-μ sum on the FP64 matrix cores (the "MFMA"
// covariance mode): Σ_k ŷ_k y_kᵀ over the lower 64x64 tiles of C, Ŷ_k =
// (cμ w_k / σ²) y_k, y_k = x_sel(k) - m_prev.  One 256-thread workgroup per
// (64x64 tile, K-slice); each wave owns a 32x32 quarter as 2x2
// v_mfma_f64_16x16x4f64 accumulators fed from LDS.  The slice's rows are
// staged 32 at a time (centred and scaled while staging, coalesced 16-B
// loads prefetched into registers one chunk ahead).  Workgroup ids are
// dealt to the 8 XCDs round-robin, so all tiles of one K-slice are given
// ids of one XCD: the slice's rows come from HBM once into that XCD's L2
// and are re-read there by the slice's tiles.  Partial sums go to
// part[slice][16x16 tile] for k_adaptC_combine / k_part_reduce, which add
// the slices and the base terms in a fixed order (deterministic).
// SHARD: rows are the rank's owned selected rows (count on the device),
// weights w[kidx[j]], scale 1/σ² (cμ applied after the all-reduce).
typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int RT_T = 64, RT_KC = 32, RT_LD = RT_T + 16;  // LDS row stride: the 4 k-rows of a fragment in 2 bank halves

inline int rankmu_grid(int N, int kslices) {
  const int nt = (N + RT_T - 1) / RT_T;
  return nt * (nt + 1) / 2 * kslices;
}

inline int rankmu_kslices(int N, int rows) {
  const int nt = (N + RT_T - 1) / RT_T, ntiles = nt * (nt + 1) / 2;
  // >= 256 rows per slice: the partial tiles written stay well below the rows read
  int want = (1024 + 8 * ntiles - 1) / (8 * ntiles), cap = rows / (8 * 256);
  if (cap < 1) cap = 1;
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  return 8 * want;
}

template <bool SHARD>
__global__ void __launch_bounds__(256) k_rankmu_tile(int N, int rowsIn, const int *__restrict__ rowsp, int kslices,
                                                     const double *__restrict__ Y, const int *__restrict__ kidx,
                                                     const double *__restrict__ w, const double *__restrict__ pm,
                                                     const CmaesScalars *__restrict__ sc, double *__restrict__ part) {
  __shared__ double As[RT_KC][RT_LD], Bs[RT_KC][RT_LD];
  const int nt = (N + RT_T - 1) / RT_T, ntiles = nt * (nt + 1) / 2;
  const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
  const int slice = xcd + 8 * (local / ntiles);
  int td, te;
  tri_tile(local % ntiles, td, te);
  const bool diagTile = td == te;
  double scale;
  if (SHARD) {
    scale = 1.0 / (sc->sigma * sc->sigma);
  } else {
    // c_mu from mu_eff with k_paths' formula (CMAES.cpp.base:693-694): this
    // kernel runs concurrently with k_paths, which stores the same value
    const double effMu = sc->effectiveMu, ca = N + 1.3, cb = N + 2.0;
    const double ccov1 = 2.0 / (ca * ca + effMu);
    double ccovmu = 2.0 * (effMu - 2. + 1. / effMu) / (cb * cb + effMu);
    if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
    scale = ccovmu / (sc->sigma * sc->sigma);
  }
  const int rows = SHARD ? *rowsp : rowsIn;
  const int per = (((rows + kslices - 1) / kslices) + 3) & ~3;
  const int kbeg = slice * per, kend = (kbeg + per) < rows ? (kbeg + per) : rows;
  // staging role: rows r0 + 8q (q < 4) of a chunk, columns 2c, 2c+1 of the tile
  const int t = threadIdx.x, sr = t >> 5, c2 = 2 * (t & 31);
  const int colA = td * RT_T + c2, colB = te * RT_T + c2;
  const bool evenN = (N & 1) == 0;
  const double pa0 = colA < N ? pm[colA] : 0.0, pa1 = colA + 1 < N ? pm[colA + 1] : 0.0;
  const double pb0 = colB < N ? pm[colB] : 0.0, pb1 = colB + 1 < N ? pm[colB + 1] : 0.0;
  double ra[4][2], rb[4][2], rs[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int k = k0 + sr + 8 * q;
      ra[q][0] = ra[q][1] = rb[q][0] = rb[q][1] = 0.0;
      rs[q] = 0.0;
      if (k < kend) {
        rs[q] = scale * w[SHARD ? kidx[k] : k];
        const double *row = Y + (size_t)k * N;
        if (evenN) {
          if (colA < N) {
            const double2 v = *reinterpret_cast<const double2 *>(row + colA);
            ra[q][0] = v.x, ra[q][1] = v.y;
          }
          if (!diagTile && colB < N) {
            const double2 v = *reinterpret_cast<const double2 *>(row + colB);
            rb[q][0] = v.x, rb[q][1] = v.y;
          }
        } else {
          if (colA < N) ra[q][0] = row[colA];
          if (colA + 1 < N) ra[q][1] = row[colA + 1];
          if (!diagTile && colB < N) rb[q][0] = row[colB];
          if (!diagTile && colB + 1 < N) rb[q][1] = row[colB + 1];
        }
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int r = sr + 8 * q;
      // rows past the slice end have rs = 0: their ŷ is 0 and y finite
      const double a0 = ra[q][0] - pa0, a1 = ra[q][1] - pa1;
      const double b0 = diagTile ? a0 : rb[q][0] - pb0, b1 = diagTile ? a1 : rb[q][1] - pb1;
      *reinterpret_cast<double2 *>(&As[r][c2]) = make_double2(rs[q] * a0, rs[q] * a1);
      *reinterpret_cast<double2 *>(&Bs[r][c2]) = make_double2(b0, b1);
    }
  };
  const int lane = t & 63, wave = t >> 6, wr = wave >> 1, wc = wave & 1, li = lane & 15, lk = lane >> 4;
  const bool computes = !(diagTile && wc > wr);  // the upper quarter of a diagonal tile is not needed
  dbl4 acc00 = {0, 0, 0, 0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += RT_KC) {
    __syncthreads();  // the previous chunk's fragments are read
    stage();
    __syncthreads();
    if (k0 + RT_KC < kend) load(k0 + RT_KC);  // in flight during this chunk's MFMAs
    if (computes) {
#pragma unroll
      for (int kk = 0; kk < RT_KC; kk += 4) {
        const double a0 = As[kk + lk][wr * 32 + li], a1 = As[kk + lk][wr * 32 + 16 + li];
        const double b0 = Bs[kk + lk][wc * 32 + li], b1 = Bs[kk + lk][wc * 32 + 16 + li];
        acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc11, 0, 0, 0);
      }
    }
  }
  if (!computes) return;
  // C/D layout: col = lane & 15, row = (lane >> 4) + 4 r; 16x16 tiles of the
  // lower triangle indexed TD (TD + 1) / 2 + TE
  const int nt16 = (N + 15) / 16, ntiles16 = nt16 * (nt16 + 1) / 2;
  const dbl4 *accs[4] = {&acc00, &acc01, &acc10, &acc11};
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const int TD = td * 4 + wr * 2 + (b >> 1), TE = te * 4 + wc * 2 + (b & 1);
    if (TE > TD || TD >= nt16) continue;
    double *out = part + ((size_t)slice * ntiles16 + (size_t)TD * (TD + 1) / 2 + TE) * 256;
#pragma unroll
    for (int r = 0; r < 4; r++) out[(lk + 4 * r) * 16 + li] = (*accs[b])[r];
  }
}

__global__ void __launch_bounds__(256) k_adaptC_combine(int N, int kslices, int ntiles, int diagonal,
                                                        const double *__restrict__ part,
                                                        const double *__restrict__ pc, double *C,
                                                        const CmaesScalars *__restrict__ sc, int scaleByCcovmu) {
  int td, te;
  tri_tile(blockIdx.x, td, te);
  const int tid = threadIdx.x, ty = tid / 16, tx = tid % 16;
  const int d = td * 16 + ty, e = te * 16 + tx;
  if (!(d < N && e < N && e <= d && (!diagonal || e == d))) return;
  const double ccov1 = sc->ccov1, ccovmu = sc->ccovmu, cc = sc->cumulativeCovariance;
  const int hsig = (int)sc->hsig;
  const double Cde = C[(size_t)d * N + e];
  double c = (1 - ccov1 - ccovmu) * Cde + ccov1 * (pc[d] * pc[e] + (1 - hsig) * cc * (2. - cc) * Cde);
  double s = 0.0;
  for (int sl = 0; sl < kslices; sl++) s += part[((size_t)sl * ntiles + blockIdx.x) * 256 + ty * 16 + tx];
  c += scaleByCcovmu ? ccovmu * s : s;
  C[(size_t)d * N + e] = c;
  if (e < d) C[(size_t)e * N + d] = c;
}

// ------------------------------------------------------ population shards
// ranks own rows [r0, r1) of the population.  After the
// fitness all-gather every rank sorts the whole vector (identical index);
// each then sums mean and rank-μ terms over the selected rows it owns, the
// caller sum-all-reduces the partials, and every rank finishes the update.

// selected positions k < mu with idx[k] in [r0, r1), ascending k
__global__ void __launch_bounds__(1024) k_shard_select(int mu, int r0, int r1, const unsigned *__restrict__ idx,
                                                       int *__restrict__ kidx, int *__restrict__ cnt) {
  __shared__ int wtot[16];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int base = 0; base < mu; base += 1024) {
    const int k = base + threadIdx.x;
    const int own = (k < mu && (int)idx[k] >= r0 && (int)idx[k] < r1) ? 1 : 0;
    const unsigned long long bal = __ballot(own);
    const int before = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wtot[wid] = __popcll(bal);
    __syncthreads();
    int woff = carry;
    for (int q = 0; q < wid; q++) woff += wtot[q];
    if (own) kidx[woff + before] = k;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int q = 0; q < 16; q++) carry += wtot[q];
    __syncthreads();
  }
  if (threadIdx.x == 0) *cnt = carry;
}

__global__ void __launch_bounds__(128) k_gather_owned(int N, const double *__restrict__ X,
                                                      const unsigned *__restrict__ idx, const int *__restrict__ kidx,
                                                      const int *__restrict__ cnt, double *__restrict__ Y) {
  const int j = blockIdx.x;
  if (j >= *cnt) return;
  const size_t src = (size_t)idx[kidx[j]] * N;
  for (int d = threadIdx.x; d < N; d += blockDim.x) Y[(size_t)j * N + d] = X[src + d];
}

// part[d] = sum_j w[kidx[j]] Y[j][d] (ascending k); part[N + d] = best row
// if this rank owns it, else 0
__global__ void __launch_bounds__(64) k_shard_mean(int N, int r0, int r1, const int *__restrict__ cntp,
                                                   const double *__restrict__ Y, const double *__restrict__ w,
                                                   const int *__restrict__ kidx, const double *__restrict__ X,
                                                   const unsigned *__restrict__ idx, double *__restrict__ part) {
  const int d = blockIdx.x * 64 + threadIdx.x;
  if (d >= N) return;
  const int cnt = *cntp;
  double acc = 0.;
  int j = 0;
  for (; j + 16 <= cnt; j += 16) {
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) v[q] = w[kidx[j + q]] * Y[(size_t)(j + q) * N + d];
#pragma unroll
    for (int q = 0; q < 16; q++) acc += v[q];
  }
  for (; j < cnt; j++) acc += w[kidx[j]] * Y[(size_t)j * N + d];
  part[d] = acc;
  const int i0 = (int)idx[0];
  part[N + d] = (i0 >= r0 && i0 < r1) ? X[(size_t)i0 * N + d] : 0.0;
}

__global__ void __launch_bounds__(256) k_part_reduce(int kslices, int ntiles, const double *__restrict__ slices,
                                                     double *__restrict__ out) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
  for (int sl = 0; sl < kslices; sl++) s += slices[(size_t)sl * ntiles * 256 + t];
  out[t] = s;
}

// after the all-reduce: mean (:603-609, :623-624) and best variables
__global__ void __launch_bounds__(256) k_shard_finalize(int N, const double *__restrict__ part, double *mean,
                                                        double *prevMean, double *meanUpdate, double *currBestVars,
                                                        double *bestEverVars, const CmaesScalars *__restrict__ sc) {
  const int d = blockIdx.x * 256 + threadIdx.x;
  if (d >= N) return;
  const double acc = part[d], prev = mean[d];
  prevMean[d] = prev;
  mean[d] = acc;
  meanUpdate[d] = (acc - prev) / sc->sigma;
  const double v = part[N + d];
  currBestVars[d] = v;
  if (sc->bestFlag) bestEverVars[d] = v;
}

// ---- the exact-order sharded update (cov_mode EXACT).  The reference sums
// mean and rank-mu over the selected rows in selection order
// (CMAES.cpp.base:603-609, :690-718); partial sums per shard would reorder
// them.  Instead every rank receives all mu selected rows: rank o packs the
// selected rows it owns, ascending selection rank, into block o of the
// exchange buffer ("Shard Rows", blocks of maxcnt rows), the caller
// all-gathers the blocks, and every rank unpacks Y in selection order.  Which
// rank owns selection k, and where in its block row k sits, follow from the
// replicated sorting index alone (owner = idx[k] / (lambda / S)).
constexpr int SHARD_MAX = 64;
// pos[k] = position of selection k in its owner's block; cnt[o] = rows owner
// o packs; cnt[S] = their maximum (the block size, in rows)
__global__ void __launch_bounds__(1024) k_shard_positions(int mu, int per, int S, const unsigned *__restrict__ idx,
                                                          int *__restrict__ pos, int *__restrict__ cnt) {
  __shared__ int wtot[16][SHARD_MAX];
  __shared__ int carry[SHARD_MAX];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid < S) carry[tid] = 0;
  __syncthreads();
  for (int base = 0; base < mu; base += 1024) {
    const int k = base + tid;
    const int o = k < mu ? (int)(idx[k] / (unsigned)per) : -1;
    int before = 0;
    for (int q = 0; q < S; q++) {
      const unsigned long long bal = __ballot(o == q);
      if (o == q) before = __popcll(bal & ((1ULL << lane) - 1ULL));
      if (lane == 0) wtot[wid][q] = __popcll(bal);
    }
    __syncthreads();
    if (o >= 0) {
      int off = carry[o];
      for (int w = 0; w < wid; w++) off += wtot[w][o];
      pos[k] = off + before;
    }
    __syncthreads();
    if (tid < S)
      for (int w = 0; w < 16; w++) carry[tid] += wtot[w][tid];
    __syncthreads();
  }
  if (tid < S) cnt[tid] = carry[tid];
  __syncthreads();
  if (tid == 0) {
    int m = 0;
    for (int q = 0; q < S; q++) m = max(m, carry[q]);
    cnt[S] = m;
  }
}

// this rank's selected rows into its block of the exchange buffer
__global__ void __launch_bounds__(128) k_shard_pack(int N, int rank, int per, int S, const unsigned *__restrict__ idx,
                                                    const int *__restrict__ pos, const int *__restrict__ cnt,
                                                    const double *__restrict__ X, double *__restrict__ rows) {
  const int k = blockIdx.x;
  const unsigned i = idx[k];
  if ((int)(i / (unsigned)per) != rank) return;
  const size_t dst = ((size_t)rank * cnt[S] + pos[k]) * N;
  for (int d = threadIdx.x; d < N; d += blockDim.x) rows[dst + d] = X[(size_t)i * N + d];
}

// Y in selection order from the gathered blocks (rows == nullptr: every rank
// holds the whole population in X); m_prev; the best variables (row 0)
__global__ void __launch_bounds__(128) k_shard_unpack(int N, int per, int S, const unsigned *__restrict__ idx,
                                                      const int *__restrict__ pos, const int *__restrict__ cnt,
                                                      const double *__restrict__ rows, const double *__restrict__ X,
                                                      double *__restrict__ Y, const double *__restrict__ mean,
                                                      double *__restrict__ prevMean, double *__restrict__ currBestVars,
                                                      double *__restrict__ bestEverVars,
                                                      const CmaesScalars *__restrict__ sc) {
  const int k = blockIdx.x;
  const unsigned i = idx[k];
  const double *src = rows ? rows + ((size_t)(i / (unsigned)per) * cnt[S] + pos[k]) * N : X + (size_t)i * N;
  for (int d = threadIdx.x; d < N; d += blockDim.x) Y[(size_t)k * N + d] = src[d];
  if (k == 0) {
    const bool flag = sc->bestFlag != 0u;
    for (int d = threadIdx.x; d < N; d += blockDim.x) {
      prevMean[d] = mean[d];
      const double v = src[d];
      currBestVars[d] = v;
      if (flag) bestEverVars[d] = v;
    }
  }
}

// INT64_MIN (the bits of -0.0) everywhere: the MAX all-reduce of the int64
// view then returns every entry's owner's exact bits
__global__ void k_fill_min_i64(size_t n, long long *__restrict__ p) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (long long)0x8000000000000000ULL;
}

// the gathered lower triangle back into the symmetric C
__global__ void __launch_bounds__(256) k_shard_cov_unpack(int N, const double *__restrict__ pack, double *C) {
  const int d = blockIdx.x;
  const double *row = pack + (size_t)d * (d + 1) / 2;
  for (int e = threadIdx.x; e <= d; e += blockDim.x) {
    const double v = row[e];
    C[(size_t)d * N + e] = v;
    C[(size_t)e * N + d] = v;
  }
}

// adaptC diag extrema :709-717, updateSigma :720-761, numericalErrorTreatment
// :763-772, min/max standard deviation :679-687.  (The reference's max/min
// diagonal scan uses "else if"; a new maximum can never be a new minimum, so
// plain extrema are identical.)
}  // namespace kg
// what Experiment::run's termination check reads after every generation
// (engine.cpp CmaesModule::checkTermination), in one host-coherent record
struct TermSummary {
  double f[KG_TERMINATION_FIELDS];
  // overflow guard of the next draw (kg_cmaes_sample): |m|_inf + sigma * ZMAX
  // * N * sqrt(a bound on the next axis lengths' max square); NaN if any
  // input is not finite
  double guard;
  unsigned int errors, pad;
  unsigned long long seq;  // written last (system-scope release)
};
namespace kg {

// (the same publication protocol as kg_eigen.hip k_publish_dsd: relaxed
// system-scope stores of the payload, release fence, release store of seq)
__device__ void summary_store(const CmaesScalars *sc, const StreamState *a, const StreamState *b, TermSummary *out,
                              unsigned long long seq, double guard) {
  const double f[KG_TERMINATION_FIELDS] = {sc->modelEvaluationCount, sc->infeasibleSampleCount, sc->maxEig,
                                           sc->minEig, sc->currentMinStd, sc->currentMaxStd, sc->bestEverValue,
                                           sc->currentBestValue, sc->previousBestValue};
  for (int i = 0; i < KG_TERMINATION_FIELDS; i++)
    __hip_atomic_store((unsigned long long *)&out->f[i], (unsigned long long)__double_as_longlong(f[i]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store((unsigned long long *)&out->guard, (unsigned long long)__double_as_longlong(guard),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&out->errors, sc->errors | a->errors | b->errors, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __atomic_thread_fence(__ATOMIC_RELEASE);
  __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// updateSigma (+ the termination record: one launch fewer per generation)
__global__ void __launch_bounds__(256) k_sigma(int N, int mu, int isSigmaBounded, const double *__restrict__ C,
                                               const double *__restrict__ F, const unsigned *__restrict__ idx,
                                               const double *__restrict__ minStdUpdate, CmaesScalars *sc,
                                               const StreamState *stA, const StreamState *stB, TermSummary *out,
                                               unsigned long long seq, const double *__restrict__ maskSigma,
                                               const double *__restrict__ ps, const double *__restrict__ mean,
                                               int muCfg, int viability, double tsr, double gslr,
                                               unsigned long long nextGen) {
  __shared__ double ssig;
  __shared__ int viol;
  __shared__ double red[4][6];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    const double cs = sc->sigmaCumulationFactor, ds = sc->dampFactor;
    double sigma = sc->sigma;
    if (viability) {  // CCMA-ES viability regime (:724-731)
      const double gsr = (1 - gslr) * sc->gsr;
      sc->gsr = gsr;
      sigma *= exp_cr((gsr - (tsr / (1.0 - tsr)) * (1 - gsr)) / ds);
    } else if (maskSigma) {  // discrete variables (:729-735)
      double pathL2 = 0.0;
      for (int d = 0; d < N; ++d) pathL2 += maskSigma[d] * ps[d] * ps[d];
      sigma *= exp_cr(cs / ds * (sqrt(pathL2) / sc->chiDM - 1.));
    } else
      sigma *= exp_cr(cs / ds * (sc->psNorm / sc->chiSquareNumber - 1.));
    // (the configured _muValue; the index uses the current mu, :743)
    if (muCfg > 1 && sc->currentBestValue == F[idx[mu - 1]]) sigma *= exp_cr(0.2 + cs / ds);
    const double ub = sqrt(sc->trace / N);
    if (sigma > ub && isSigmaBounded) sigma = ub;
    ssig = sigma;
    viol = 0;
  }
  if (tid == 64) {  // (wave 1, beside wave 0's sigma update: the next generation's hsig power)
    const double cs = sc->sigmaCumulationFactor;
    sc->hsigPow = pow_cr(1. - cs, 2.0 * (1.0 + (double)nextGen));
    sc->hsigPowCs = cs;
    sc->hsigPowGen = (double)nextGen;
  }
  __syncthreads();
  for (int d = tid; d < N; d += blockDim.x)
    if (ssig * sqrt(C[(size_t)d * N + d]) < minStdUpdate[d]) viol = 1;
  __syncthreads();
  if (viol && tid == 0) {
    const double cs = sc->sigmaCumulationFactor, ds = sc->dampFactor;
    double sigma = ssig;
    for (int d = 0; d < N; ++d) {
      const double cdd = C[(size_t)d * N + d];
      if (sigma * sqrt(cdd) < minStdUpdate[d]) sigma = (minStdUpdate[d]) / sqrt(cdd) * exp_cr(0.05 + cs / ds);
    }
    ssig = sigma;
  }
  __syncthreads();
  const double sigma = ssig;
  double mxd = -INFINITY, mnd = INFINITY, mns = INFINITY, mxs = -INFINITY;
  // overflow guard inputs: |m|_inf and the trace of C (NaN-propagating sums)
  double mabs = 0.0, tr = 0.0;
  for (int d = tid; d < N; d += blockDim.x) {
    const double cdd = C[(size_t)d * N + d];
    mxd = fmax(mxd, cdd);
    mnd = fmin(mnd, cdd);
    const double s = sigma * sqrt(cdd);
    mns = fmin(mns, s);
    mxs = fmax(mxs, s);
    mabs += fabs(mean[d]);
    tr += fabs(cdd);
  }
  for (int off = 32; off > 0; off >>= 1) {
    mxd = fmax(mxd, __shfl_xor(mxd, off, 64));
    mnd = fmin(mnd, __shfl_xor(mnd, off, 64));
    mns = fmin(mns, __shfl_xor(mns, off, 64));
    mxs = fmax(mxs, __shfl_xor(mxs, off, 64));
    mabs += __shfl_xor(mabs, off, 64);
    tr += __shfl_xor(tr, off, 64);
  }
  if (lane == 0) {
    red[wid][0] = mxd;
    red[wid][1] = mnd;
    red[wid][2] = mns;
    red[wid][3] = mxs;
    red[wid][4] = mabs;
    red[wid][5] = tr;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; w++) {
      mxd = fmax(mxd, red[w][0]);
      mnd = fmin(mnd, red[w][1]);
      mns = fmin(mns, red[w][2]);
      mxs = fmax(mxs, red[w][3]);
      mabs += red[w][4];
      tr += red[w][5];
    }
    sc->maxDiagC = mxd;
    sc->minDiagC = mnd;
    sc->sigma = sigma;
    sc->rmuOutOfRange = 0u;  // (read by this update's adaptC; the next k_select_prep may set it)
    sc->currentMinStd = mns;
    sc->currentMaxStd = mxs;
    // next draw: the axis lengths come from C's eigenvalues (each <= trace
    // for the PSD update, 1% slack for rounding) or stay the current ones
    // (a rejected decomposition keeps them, max square = maxEig)
    const double d2 = fmax(1.01 * tr, sc->maxEig);
    const double guard = mabs + sigma * KG_DRAW_ZMAX * (double)N * sqrt(d2);
    summary_store(sc, stA, stB, out, seq, (isfinite(mabs) && isfinite(tr) && isfinite(sigma) && isfinite(sc->maxEig)) ? guard : NAN);
  }
}

// ------------------------------------------------------------- CCMA-ES
// handleConstraints' covariance correction (:779-804): auxC = C, then for
// every (violating sample i, constraint c with its viability indicator set)
// pair in the reference's order: the constraint normal's running
// approximation v_c = (1 - beta) v_c + beta BDZ_i, v2 = |v_c|^2 (sequential),
// and auxC -= (cmaf cmaf v_c,d v_c,e) / (v2 cnt_i cnt_i) elementwise.
__global__ void __launch_bounds__(256) k_ccm_adapt(int N, int npairs, const int *__restrict__ pi,
                                                   const int *__restrict__ pc_, const double *__restrict__ pcnt,
                                                   const double *__restrict__ BDZ, double *__restrict__ V, double beta,
                                                   double cmaf, const double *__restrict__ C, double *__restrict__ auxC) {
  __shared__ double v2s;
  const int tid = threadIdx.x;
  for (int q = tid; q < N * N; q += blockDim.x) auxC[q] = C[q];
  for (int p = 0; p < npairs; p++) {
    const int i = pi[p];
    double *v = V + (size_t)pc_[p] * N;
    __syncthreads();
    for (int d = tid; d < N; d += blockDim.x) v[d] = (1.0 - beta) * v[d] + beta * BDZ[(size_t)i * N + d];
    __syncthreads();
    if (tid == 0) {
      double v2 = 0;
      for (int d = 0; d < N; ++d) v2 += v[d] * v[d];
      v2s = v2;
    }
    __syncthreads();
    const double den = v2s * pcnt[p] * pcnt[p];
    for (int q = tid; q < N * N; q += blockDim.x) {
      const int d = q / N, e = q % N;
      auxC[q] = auxC[q] - ((cmaf * cmaf * v[d] * v[e]) / den);
    }
  }
}

// handleConstraints' redraws (:806-822) over one round of transformed
// blocks: list entry k (a violating sample, in index order) takes blocks
// until one is feasible or the Resampled Parameter Count (+1 per draw, every
// draw) reaches Max Infeasible Resamplings; entries [k0, *kEnd) are assigned
// (the rest continue in the next round, as k_select)
__global__ void k_select_list(int nlist, int k0, int blocks, double maxRes, const int *__restrict__ infeas,
                              int *__restrict__ assign, unsigned long long *__restrict__ used,
                              int *__restrict__ kEnd, CmaesScalars *sc) {
  if (threadIdx.x != 0) return;
  double count = sc->resampledCount;
  int j = 0, k = k0;
  for (; k < nlist; k++) {
    bool taken = false;
    while (j < blocks) {
      count += 1;
      const int feasible = infeas[j] ? 0 : 1;
      const int jj = j++;
      if (feasible || !(count < maxRes)) {
        assign[k] = jj;
        taken = true;
        break;
      }
    }
    if (!taken) break;
  }
  sc->resampledCount = count;
  *used = (unsigned long long)j;
  kEnd[0] = k;
}

__global__ void k_gather_list(int N, int k0, const int *__restrict__ kEnd, const int *__restrict__ list,
                              const int *__restrict__ assign, const double *__restrict__ Xall, double *__restrict__ X,
                              const double *__restrict__ BDZall, double *__restrict__ BDZ) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = k0 + (int)(t / N), d = (int)(t % N);
  if (k >= *kEnd) return;
  const size_t dst = (size_t)list[k] * N + d, src = (size_t)assign[k] * N + d;
  X[dst] = Xall[src];
  BDZ[dst] = BDZall[src];
}

__global__ void k_add_evals(CmaesScalars *sc, double n) {
  if (threadIdx.x == 0) sc->modelEvaluationCount += n;
}

}  // namespace kg

// ===================================================================== ABI
using namespace kg;


struct kg_cmaes_s {
  kg_cmaes_cfg cfg;
  int N = 0, lam = 0, mu = 0, R = 0;  // lam / mu: the CURRENT population and mu (CCMA-ES regimes)
  int lamCfg = 0, muCfg = 0, lamMax = 0, muMax = 0;  // configured; allocated (max over the regimes)
  // CCMA-ES (cfg.constraint_count > 0): host-side constraint bookkeeping
  // (CMAES.cpp.base:350-437), device-side covariance correction / redraws
  size_t nc = 0;
  bool viability = false;  // Is Viability Regime
  kg_constraint_fn cfn = nullptr;
  void *cctx = nullptr;
  std::vector<double> cEval, cInd, cCnt, vBounds, bestCEval;  // [c][i] nc x lamMax, (i), (c)
  double cEvalCount = 0, adaptCount = 0, maxViolCount = 0;
  double *V = nullptr, *auxC = nullptr;  // normal approximations (nc x N), corrected covariance
  int *violDev = nullptr, *pairI = nullptr, *pairC = nullptr, *listDev = nullptr;
  double *pairCnt = nullptr;
  bool finiteBounds = false;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // the rank-mu sum, concurrent with the mean and the paths
  hipEvent_t evY = nullptr, evC = nullptr;
  double *mean = nullptr, *prevMean = nullptr, *C = nullptr, *B = nullptr, *D = nullptr, *pc = nullptr,
         *ps = nullptr, *w = nullptr, *X = nullptr, *Xall = nullptr, *BDZ = nullptr, *BDZall = nullptr,
         *F = nullptr, *Z = nullptr, *bestEverVars = nullptr, *currBestVars = nullptr, *meanUpdate = nullptr,
         *auxBDZ = nullptr;
  double *lb = nullptr, *ub = nullptr, *iv = nullptr, *istd = nullptr, *minstd = nullptr;
  unsigned *idx = nullptr;
  double *sortKey = nullptr;
  unsigned *sortVal = nullptr;
  CmaesScalars *sc = nullptr;
  double *covPart = nullptr, *Y = nullptr;
  double *Yc = nullptr, *Tt = nullptr;  // exact rank-mu factors (k_rankmu_prep)
  double *dzT = nullptr;                // k_transform_sc: D o z, k-major (ldz rows per k)
  size_t dzTRows = 0;
  int trW = 0;                          // k_transform_sc columns per wave (0: k_transform)
  EigenSolver eig;
  int *infeas = nullptr, *assign = nullptr;
  int *selEnd = nullptr;  // a resampling round's end: [next unassigned sample, uniform window exhausted]
  unsigned long long *blockEnd = nullptr, *usedBlocks = nullptr;
  // state set by the caller (initialize, set_field) since the last update:
  // the termination record's overflow guard does not describe it
  bool stateDirty = true;
  size_t resamplingRounds = 0;  // rounds beyond the first (diagnostics: "Resampling Rounds")
  bool mirrored = false;  // "Mirrored Sampling": blocks of N normals feed two rows
  double *G = nullptr;    // samples' gradients (use_gradients)
  // discrete variables: Granularity, Masking Matrix (Sigma), the peeked
  // uniforms of the discrete mutations and how many were used
  bool hasDiscrete = false;
  double *gran = nullptr, *mask = nullptr, *maskSigma = nullptr, *ubuf = nullptr, *dzero = nullptr;
  unsigned long long *uused = nullptr;
  size_t ucap = 0;
  size_t blocks = 0;      // normal blocks drawn per generation (λ or λ/2, + the reserve R)
  int kslices = 8;  // rank-mu K-slices (rankmu_kslices), a multiple of the 8 XCDs
  // population shards
  int shards = 1, shardRank = 0, r0 = 0, r1 = 0;
  bool replSample = false;  // sharded, but every rank draws the whole population (kg_cmaes_create)
  int *kidx = nullptr, *shardCnt = nullptr;
  double *part = nullptr;  // "Shard Partials": mean (N), best row (N), rank-mu tiles
  // exact-order sharded update (cov_mode EXACT): selected-row exchange blocks
  // ("Shard Rows", S blocks of up to rowsCap rows), the positions / counts of
  // the blocks, and this rank's share of the new covariance ("Shard Covariance",
  // the packed lower triangle)
  int *shardPos = nullptr, *shardCounts = nullptr;
  double *rows = nullptr, *covPack = nullptr;
  size_t rowsCap = 0;
  int rowBlock = -1;  // rows per block of the current generation's exchange (host copy; -1: not yet known)
  unsigned long long *eigTrace = nullptr;  // KORALI_AMD_TRACE_EIGEN: s_memtime per phase
  // termination scalars + error flags of the last update, written by the
  // device into host-coherent memory (kg_cmaes_wait_termination_fields)
  TermSummary *summary = nullptr, *summaryDev = nullptr;
  unsigned long long updates = 0;
  bool sampleBegun = false;  // kg_cmaes_begin_sample enqueued the next draw's first half
  MtStream normal, uniform;
  // profiling
  bool profile = false;
  std::vector<std::tuple<std::string, hipEvent_t, hipEvent_t>> pending;
  std::map<std::string, hipEvent_t> openMarks;  // kg_cmaes_profile_mark begun, not ended
  std::map<std::string, std::pair<double, size_t>> prof;
};

namespace {

struct Stage {
  kg_cmaes_s *h;
  std::string name;
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s;
  Stage(kg_cmaes_s *h_, const char *n, hipStream_t on = nullptr) : h(h_), name(n), s(on ? on : h_->stream) {
    if (h->profile) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, s);
    }
  }
  ~Stage() {
    if (h->profile) {
      (void)hipEventRecord(b, s);
      h->pending.emplace_back(name, a, b);
    }
  }
};

// eigensolver stage profiling: device stages by events, host stages by clock
void eig_prof(void *ctx, const char *stage, int phase) {
  auto *h = (kg_cmaes_s *)ctx;
  if (!h->profile) return;
  static thread_local hipEvent_t a;
  static thread_local std::chrono::steady_clock::time_point t0;
  if (phase == 0) {
    (void)hipEventCreate(&a);
    (void)hipEventRecord(a, h->stream);
  } else if (phase == 1) {
    hipEvent_t b;
    (void)hipEventCreate(&b);
    (void)hipEventRecord(b, h->stream);
    h->pending.emplace_back(stage, a, b);
  } else if (phase == 2) {
    t0 = std::chrono::steady_clock::now();
  } else {
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    auto &p = h->prof[stage];
    p.first += ms;
    p.second += 1;
  }
}

// KORALI_AMD_RUN_PHASES=1: kg_cmaes_create's phases on stderr
struct CreateClock {
  bool on = getenv("KORALI_AMD_RUN_PHASES") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string text;
  void mark(const char *phase) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    char b[96];
    snprintf(b, sizeof(b), " %s=%.3fms", phase, std::chrono::duration<double, std::milli>(n - t).count());
    text += b;
    t = n;
  }
  ~CreateClock() {
    if (on) fprintf(stderr, "[korali_amd cmaes create]%s\n", text.c_str());
  }
};

template <typename T>
int dalloc(T **p, size_t n, bool wait = true) {
  if (n == 0) n = 1;
  KG_HIP(dev_alloc(p, n * sizeof(T)));
  if (wait ? zero_fill(*p, n * sizeof(T)) : zero_fill_async(*p, n * sizeof(T))) return 1;
  return 0;
}
// kg_cmaes_create's buffers: zero fills queued on the null stream, waited for
// once after the last one
template <typename T>
int dalloc_q(T **p, size_t n) {
  return dalloc(p, n, false);
}

void gsl_seed_state(uint64_t seed, unsigned char *out5000) {
  uint64_t mt[624];
  uint64_t s = seed & 0xffffffffULL;
  if (s == 0) s = 4357;
  mt[0] = s;
  for (int i = 1; i < 624; i++) mt[i] = (1812433253ULL * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint64_t)i) & 0xffffffffULL;
  memset(out5000, 0, 5000);
  memcpy(out5000, mt, sizeof(mt));
  int32_t mti = 624;
  memcpy(out5000 + 624 * 8, &mti, 4);
}

__global__ void k_collect_errors(CmaesScalars *sc, const StreamState *a, const StreamState *b) {
  sc->errors |= a->errors | b->errors;
}

int check_errors(kg_cmaes_s *h) {
  // one read: the generators' flags are folded into the scalar block first
  unsigned int e = 0;
  hipLaunchKernelGGL(k_collect_errors, dim3(1), dim3(1), 0, h->stream, h->sc, h->normal.state(), h->uniform.state());
  KG_HIP(hipGetLastError());
  KG_HIP(hipMemcpyAsync(&e, &h->sc->errors, sizeof(e), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  if (e == 0) return 0;
  std::string m = "korali_amd CMA-ES device error:";
  if (e & KG_ERR_NONFINITE_F) m += " Non finite value of function evaluation detected.";
  if (e & KG_ERR_RNG_UNDERRUN) m += " RNG stream underrun.";
  if (e & KG_ERR_DRAW_GUARD) m += " A draw the overflow guard proved finite was not (internal error).";
  if (e & KG_ERR_ZERO_LIST) m += " Too many zero mt19937 words pending.";
  if (e & KG_ERR_EIGEN) m += " Eigen decomposition did not converge.";
  if (e & KG_ERR_SYNC_TIMEOUT) m += " An in-launch workgroup hand-off timed out.";
  set_error(m);
  return 1;
}

struct FieldRef {
  double *dev;
  size_t n;
};

bool field_ref(kg_cmaes_s *h, const std::string &k, FieldRef &r) {
  const size_t N = h->N, L = h->lam;
#define VEC(key, ptr, n) \
  if (k == key) {        \
    r = {ptr, n};        \
    return true;         \
  }
  VEC("Current Mean", h->mean, N)
  VEC("Previous Mean", h->prevMean, N)
  VEC("Covariance Matrix", h->C, N * N)
  VEC("Covariance Eigenvector Matrix", h->B, N * N)
  VEC("Axis Lengths", h->D, N)
  VEC("Evolution Path", h->pc, N)
  VEC("Conjugate Evolution Path", h->ps, N)
  VEC("Mu Weights", h->w, (size_t)h->mu)
  VEC("Sample Population", h->X, L * N)
  VEC("Value Vector", h->F, L)
  VEC("Best Ever Variables", h->bestEverVars, N)
  VEC("Current Best Variables", h->currBestVars, N)
  VEC("Mean Update", h->meanUpdate, N)
  VEC("Auxiliar BDZ Matrix", h->auxBDZ, N)
  VEC("Lower Bound", h->lb, N)
  VEC("Upper Bound", h->ub, N)
  VEC("Initial Value", h->iv, N)
  VEC("Initial Standard Deviation", h->istd, N)
  VEC("Minimum Standard Deviation Update", h->minstd, N)
  VEC("Granularity", h->gran, N)
  VEC("Masking Matrix", h->mask, N)
  VEC("Masking Matrix Sigma", h->maskSigma, N)
  if (h->BDZ) VEC("BDZ Matrix", h->BDZ, L * N)
  if (h->G) VEC("Gradients", h->G, L * N)
  if (h->part) {
    const size_t nt = (N + 15) / 16;
    VEC("Shard Partials", h->part, 2 * N + nt * (nt + 1) / 2 * 256)
  }
  if (h->rows) VEC("Shard Rows", h->rows, (size_t)h->shards * h->rowsCap * N)
  if (h->covPack) VEC("Shard Covariance", h->covPack, N * (N + 1) / 2)
#define SCA(key, fld) VEC(key, &h->sc->fld, 1)
  SCA("Sigma", sigma)
  SCA("Trace", trace)
  SCA("Effective Mu", effectiveMu)
  SCA("Cumulative Covariance", cumulativeCovariance)
  SCA("Sigma Cumulation Factor", sigmaCumulationFactor)
  SCA("Damp Factor", dampFactor)
  SCA("Chi Square Number", chiSquareNumber)
  SCA("Conjugate Evolution Path L2 Norm", psNorm)
  SCA("Best Ever Value", bestEverValue)
  SCA("Previous Best Ever Value", previousBestEverValue)
  SCA("Previous Best Value", previousBestValue)
  SCA("Current Best Value", currentBestValue)
  SCA("Current Min Standard Deviation", currentMinStd)
  SCA("Current Max Standard Deviation", currentMaxStd)
  SCA("Maximum Diagonal Covariance Matrix Element", maxDiagC)
  SCA("Minimum Diagonal Covariance Matrix Element", minDiagC)
  SCA("Minimum Covariance Eigenvalue", minEig)
  SCA("Maximum Covariance Eigenvalue", maxEig)
  SCA("Infeasible Sample Count", infeasibleSampleCount)
  SCA("Best Valid Sample", bestValidSample)
  SCA("Model Evaluation Count", modelEvaluationCount)
  SCA("Hsig", hsig)
  SCA("Eigen Failures", eigenFailures)
  SCA("Number Masking Matrix Entries", nME)
  SCA("Number Of Discrete Mutations", nDM)
  SCA("Chi Square Number Discrete Mutations", chiDM)
  SCA("Global Success Rate", gsr)
  SCA("Resampled Parameter Count", resampledCount)
  if (h->nc) VEC("Normal Constraint Approximation", h->V, h->nc * N)
#undef SCA
#undef VEC
  return false;
}

// the current population and mu (CCMA-ES switches them between regimes):
// blocks drawn per generation, the unsharded evaluation range, and the block
// count the no-reserve path consumes (λ, or λ/2 when mirrored)
int set_current(kg_cmaes_s *h, int lam, int mu) {
  h->lam = lam;
  h->mu = mu;
  h->blocks = (h->mirrored ? (size_t)lam / 2 : (size_t)lam) + h->R;
  if (h->shards == 1) {
    h->r0 = 0;
    h->r1 = lam;
  }
  const unsigned long long used = (unsigned long long)(h->mirrored ? lam / 2 : lam);
  KG_HIP(hipMemcpy(h->usedBlocks, &used, sizeof(used), hipMemcpyHostToDevice));
  return 0;
}

}  // namespace

extern "C" {

int kg_cmaes_create(const kg_cmaes_cfg *cfg, kg_cmaes_t *out) {
  KG_CHECK(cfg && out, "kg_cmaes_create: null argument");
  KG_CHECK(cfg->variable_count >= 1, "'Variable Count' must be >= 1");
  KG_CHECK(cfg->population_size > 1, "'Population Size' must be larger 1.");  // CMAES.cpp.base:26
  KG_CHECK(!cfg->mirrored_sampling || cfg->population_size % 2 == 0,
           "Mirrored Sampling can only be applied with an even Sample Population");  // CMAES.cpp.base:91
  KG_CHECK(!cfg->use_gradients || cfg->gradient_step_size > 0.0,
           "Gradient Step Size must be larger than 0.0");  // CMAES.cpp.base:86
  KG_CHECK(cfg->variable_count <= 960, "device path supports up to 960 variables");
  KG_CHECK(cfg->mu_type >= 0 && cfg->mu_type <= 3,
           "Invalid setting of Mu Type (Linear, Equal, Logarithmic, or Proportional accepted).");
  KG_HIP(hipSetDevice(cfg->device));
  upload_dd_tables();
  if (cfg->constraint_count > 0) {  // CCMA-ES checks (CMAES.cpp.base:86-95, :134-141)
    KG_CHECK(!cfg->mirrored_sampling, "Mirrored Sampling not applicable to problems with constraints");
    KG_CHECK(cfg->shard_count <= 1, "constrained CMA-ES runs unsharded");
    KG_CHECK(cfg->viability_population_size >= 1, "'Viability Population Size' must be >= 1");
    KG_CHECK(cfg->global_success_learning_rate > 0.0 && cfg->global_success_learning_rate <= 1.0,
             "Invalid Global Success Learning Rate, must be greater than 0.0 and less than 1.0");
    KG_CHECK(cfg->target_success_rate > 0.0 && cfg->target_success_rate <= 1.0,
             "Invalid Target Success Rate, must be greater than 0.0 and less than 1.0");
    KG_CHECK(cfg->covariance_matrix_adaption_strength > 0.0, "Invalid Adaption Size, must be greater than 0.0");
    if (cfg->granularity)
      for (size_t i = 0; i < cfg->variable_count; i++)
        KG_CHECK(cfg->granularity[i] == 0.0, "constrained CMA-ES with discrete variables is not on the device path");
  }
  auto *h = new kg_cmaes_s();
  h->cfg = *cfg;
  const int N = (int)cfg->variable_count;
  h->N = N;
  h->lamCfg = (int)cfg->population_size;
  h->muCfg = (int)(cfg->mu_value ? cfg->mu_value : cfg->population_size / 2);
  KG_CHECK(h->muCfg >= 1 && h->muCfg <= h->lamCfg, "'Mu Value' must be in [1, Population Size]");
  h->nc = cfg->constraint_count;
  h->lamMax = h->lamCfg;
  h->muMax = h->muCfg;
  if (h->nc) {
    const int lv = (int)cfg->viability_population_size;
    const int mv = (int)(cfg->viability_mu_value ? cfg->viability_mu_value : cfg->viability_population_size / 2);
    KG_CHECK(mv >= 1 && mv <= lv, "'Viability Mu Value' must be in [1, Viability Population Size]");
    h->lamMax = std::max(h->lamMax, lv);
    h->muMax = std::max(h->muMax, mv);
    h->cfg.store_bdz = 1;  // the correction reads the samples' BDZ rows
  }
  h->lam = h->lamCfg;
  h->mu = h->muCfg;
  // allocations below hold the larger regime
  const int L = h->lamMax;
  std::vector<double> lb(N, -INFINITY), ub(N, INFINITY), iv(N, NAN), istd(N, NAN), minstd(N, 0.0);
  for (int i = 0; i < N; i++) {
    if (cfg->lower_bound) lb[i] = cfg->lower_bound[i];
    if (cfg->upper_bound) ub[i] = cfg->upper_bound[i];
    if (cfg->initial_value) iv[i] = cfg->initial_value[i];
    if (cfg->initial_std) istd[i] = cfg->initial_std[i];
    if (cfg->min_std_update) minstd[i] = cfg->min_std_update[i];
    if (std::isfinite(lb[i]) || std::isfinite(ub[i])) h->finiteBounds = true;
    // CMAES.cpp.base:111-126
    if (!std::isfinite(iv[i])) {
      if (!std::isfinite(lb[i]) || !std::isfinite(ub[i])) {
        set_error("'Initial Value' of variable " + std::to_string(i) +
                  " not defined, and cannot be inferred because variable bounds are not finite.");
        delete h;
        return 1;
      }
      iv[i] = (ub[i] + lb[i]) * 0.5;
    }
    if (!std::isfinite(istd[i])) {
      if (!std::isfinite(lb[i]) || !std::isfinite(ub[i])) {
        set_error("Initial Standard Deviation of variable " + std::to_string(i) +
                  " not defined, and cannot be inferred because variable bounds are not finite.");
        delete h;
        return 1;
      }
      istd[i] = (ub[i] - lb[i]) * 0.3;
    }
  }
  std::vector<double> gran(N, 0.0);
  for (int i = 0; i < N; i++) {
    if (cfg->granularity) gran[i] = cfg->granularity[i];
    if (gran[i] < 0.0) {  // CMAES.cpp.base:48
      set_error("Negative granularity for variable " + std::to_string(i) + ".");
      delete h;
      return 1;
    }
    if (gran[i] > 0.0) h->hasDiscrete = true;
  }
  // a reserve of transformed rows for resampling: finite bounds, or discrete
  // variables (a rounded or mutated sample may leave the bounds or not)
  h->R = (h->finiteBounds || h->hasDiscrete) ? std::max(256, L / 4) : 0;
  h->shards = cfg->shard_count > 1 ? cfg->shard_count : 1;
  h->shardRank = h->shards > 1 ? cfg->shard_rank : 0;
  if (h->shards > 1 && (L % h->shards != 0 || cfg->shard_rank < 0 || cfg->shard_rank >= h->shards ||
                        h->shards > SHARD_MAX)) {
    set_error("population sharding needs Population Size divisible by the shard count, "
              "0 <= shard_rank < shard_count and at most " + std::to_string(SHARD_MAX) + " shards");
    delete h;
    return 1;
  }
  CreateClock clk;
  h->r0 = h->shardRank * (L / h->shards);
  h->r1 = h->r0 + L / h->shards;
  h->mirrored = cfg->mirrored_sampling != 0;
  // a population whose draw is not "row i = block i" (the redraw walk of
  // finite bounds and discrete variables, the +-z pairs of Mirrored Sampling)
  // or that has no B (diagonal covariance) is drawn and transformed whole on
  // every rank, each rank evaluating and summing its own rows
  h->replSample = h->shards > 1 &&
                  (h->finiteBounds || h->hasDiscrete || h->mirrored || cfg->diagonal_covariance);
  h->trW = transform_width(N);
  h->blocks = (h->mirrored ? (size_t)L / 2 : (size_t)L) + h->R;
  const size_t rows = (size_t)L + h->R;
  const size_t xrows = h->mirrored ? 2 * h->blocks : rows;  // transformed rows (Xall, infeasibility flags)
  int rc = 0;
  rc |= dalloc_q(&h->mean, N) | dalloc_q(&h->prevMean, N) | dalloc_q(&h->C, (size_t)N * N) | dalloc_q(&h->B, (size_t)N * N);
  rc |= dalloc_q(&h->D, N) | dalloc_q(&h->pc, N) | dalloc_q(&h->ps, N) | dalloc_q(&h->w, h->muMax);
  rc |= dalloc_q(&h->X, (size_t)L * N) | dalloc_q(&h->F, L) | dalloc_q(&h->Z, rows * N);
  rc |= dalloc_q(&h->bestEverVars, N) | dalloc_q(&h->currBestVars, N) | dalloc_q(&h->meanUpdate, N) | dalloc_q(&h->auxBDZ, N);
  rc |= dalloc_q(&h->lb, N) | dalloc_q(&h->ub, N) | dalloc_q(&h->iv, N) | dalloc_q(&h->istd, N) | dalloc_q(&h->minstd, N);
  rc |= dalloc_q(&h->Y, (size_t)h->muMax * N);
  if (cfg->cov_mode != KG_COV_MFMA) rc |= dalloc_q(&h->Yc, (size_t)h->muMax * N) | dalloc_q(&h->Tt, (size_t)h->muMax * N);
  rc |= dalloc_q(&h->idx, L) | dalloc_q(&h->sc, 1);
  rc |= dalloc_q(&h->infeas, xrows) | dalloc_q(&h->assign, L) | dalloc_q(&h->blockEnd, rows) | dalloc_q(&h->usedBlocks, 1);
  rc |= dalloc_q(&h->selEnd, 2);
  if (h->cfg.store_bdz) rc |= dalloc_q(&h->BDZ, (size_t)L * N);
  if (cfg->use_gradients) rc |= dalloc_q(&h->G, (size_t)L * N);
  rc |= dalloc_q(&h->gran, N) | dalloc_q(&h->mask, N) | dalloc_q(&h->maskSigma, N);
  if (h->hasDiscrete) {
    h->ucap = 16 * (size_t)L + 1024;  // the mutations' uniforms per generation: ~2-4 per mutated sample
    rc |= dalloc_q(&h->ubuf, h->ucap) | dalloc_q(&h->uused, 1);
  }
  if (h->R) {
    rc |= dalloc_q(&h->Xall, xrows * N);
    if (h->cfg.store_bdz) rc |= dalloc_q(&h->BDZall, xrows * N);
  }
  size_t P2 = 1;
  while (P2 < (size_t)L) P2 <<= 1;
  if (P2 < SORT_CHUNK) P2 = SORT_CHUNK;
  rc |= dalloc_q(&h->sortKey, P2) | dalloc_q(&h->sortVal, P2);
  const int nt = (N + 15) / 16;
  h->kslices = rankmu_kslices(N, h->muMax);
  rc |= dalloc_q(&h->covPart, (size_t)h->kslices * (nt * (nt + 1) / 2) * 256);
  if (h->nc) {
    rc |= dalloc_q(&h->V, h->nc * (size_t)N) | dalloc_q(&h->auxC, (size_t)N * N) | dalloc_q(&h->violDev, L);
    rc |= dalloc_q(&h->pairI, h->nc * (size_t)L) | dalloc_q(&h->pairC, h->nc * (size_t)L) |
          dalloc_q(&h->pairCnt, h->nc * (size_t)L) | dalloc_q(&h->listDev, L);
    h->cEval.assign(h->nc * (size_t)L, 0.0);
    h->cInd.assign(h->nc * (size_t)L, 0.0);
    h->cCnt.assign(L, 0.0);
    h->vBounds.assign(h->nc, 0.0);
    h->bestCEval.assign(h->nc, 0.0);
  }
  rc |= dalloc_q(&h->kidx, h->muMax) | dalloc_q(&h->shardCnt, 1) | dalloc_q(&h->part, 2 * (size_t)N + (size_t)(nt * (nt + 1) / 2) * 256);
  if (cfg->shard_count >= 1 && cfg->cov_mode != KG_COV_MFMA) {
    // a rank owns lambda / S rows, so it packs at most min(mu, lambda / S)
    // selected ones; whole-population ranks (replSample) exchange no rows
    h->rowsCap = h->replSample ? 0 : (size_t)std::min(h->muMax, L / h->shards);
    rc |= dalloc_q(&h->shardPos, h->muMax) | dalloc_q(&h->shardCounts, h->shards + 1) |
          dalloc_q(&h->covPack, (size_t)N * (N + 1) / 2);
    if (h->rowsCap) rc |= dalloc_q(&h->rows, (size_t)h->shards * h->rowsCap * N);
  }
  if (!rc && hipStreamSynchronize(nullptr) != hipSuccess) {
    set_error("kg_cmaes_create: zero fills of the device buffers failed");
    rc = 1;
  }
  if (rc) {
    delete h;
    return 1;
  }
  clk.mark("buffers");
  if (getenv("KORALI_AMD_TRACE_EIGEN")) rc |= dalloc(&h->eigTrace, 32 + 8 * (size_t)std::max(N, 128));
  if (host_alloc(&h->summary, sizeof(TermSummary), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void **)&h->summaryDev, h->summary, 0) != hipSuccess) {
    delete h;
    KG_CHECK(false, "hipHostMalloc of the termination summary failed");
  }
  memset(h->summary, 0, sizeof(TermSummary));
  if (L <= RANK_MAX && (size_t)L * sizeof(double) > 64 * 1024)
    KG_HIP(allow_dynamic_lds((const void *)k_rank_sort, (int)((size_t)L * sizeof(double))));
  {
    const size_t pbytes = ((size_t)N * (PA_EC + 1) + N) * sizeof(double);
    if (pbytes > 64 * 1024)
      KG_HIP(allow_dynamic_lds((const void *)k_paths, (int)pbytes));
    KG_HIP(allow_dynamic_lds((const void *)k_mean2, (int)mean2_lds_bytes()));
    if (N <= 128)
      KG_HIP(allow_dynamic_lds((const void *)k_objective2, (int)ob2_lds_bytes(N)));
    if (N <= 128)
      KG_HIP(allow_dynamic_lds((const void *)k_paths2, (int)paths2_lds_bytes(N)));
  }
  if (rc) {
    delete h;
    return 1;
  }
  KG_HIP(stream_acquire(&h->stream));
  KG_HIP(stream_acquire(&h->stream2));
  KG_HIP(hipEventCreateWithFlags(&h->evY, hipEventDisableTiming));
  KG_HIP(hipEventCreateWithFlags(&h->evC, hipEventDisableTiming));
  {
    const char *ev = getenv("KORALI_AMD_EIGEN_CHASE");
    bool hostChase = !cfg->eigen_device_chase;
    if (ev && std::string(ev) == "device") hostChase = false;
    if (ev && std::string(ev) == "host") hostChase = true;
    if (h->eig.init(N, hostChase)) {
      delete h;
      return 1;
    }
  }
  clk.mark("eigen");
  if (set_current(h, h->lamCfg, h->muCfg)) return 1;
  KG_HIP(hipMemcpy(h->lb, lb.data(), N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->ub, ub.data(), N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->iv, iv.data(), N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->istd, istd.data(), N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->minstd, minstd.data(), N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->gran, gran.data(), N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemset(h->mask, 0, N * sizeof(double)));
  KG_HIP(hipMemset(h->maskSigma, 0, N * sizeof(double)));
  const size_t words = h->normal.words_for_normals(rows * N);
  if (h->normal.init(3 * words + 4096) || h->uniform.init(std::max<size_t>(1 << 16, 2 * h->ucap + 4096))) {
    delete h;
    return 1;
  }
  clk.mark("rng_init");
  unsigned char st[5000];
  gsl_seed_state(cfg->normal_seed, st);
  if (h->normal.import_gsl(st, h->stream)) return 1;
  clk.mark("normal_seed");
  gsl_seed_state(cfg->uniform_seed, st);
  if (h->uniform.import_gsl(st, h->stream)) return 1;
  clk.mark("uniform_seed");
  *out = h;
  return 0;
}

int kg_cmaes_destroy(kg_cmaes_t h) {
  if (!h) return 0;
  // every stream drained before the blocks go back to the cache
  (void)hipStreamSynchronize(h->stream);
  if (h->stream2) (void)hipStreamSynchronize(h->stream2);
  h->eig.drain();
  h->normal.drain();
  h->uniform.drain();
  if (h->summary) host_release(h->summary);
  for (void *p : {(void *)h->mean, (void *)h->prevMean, (void *)h->C, (void *)h->B, (void *)h->D, (void *)h->pc,
                  (void *)h->ps, (void *)h->w, (void *)h->X, (void *)h->Xall, (void *)h->BDZ, (void *)h->BDZall,
                  (void *)h->F, (void *)h->Z, (void *)h->bestEverVars, (void *)h->currBestVars,
                  (void *)h->meanUpdate, (void *)h->auxBDZ, (void *)h->lb, (void *)h->ub, (void *)h->iv,
                  (void *)h->istd, (void *)h->minstd, (void *)h->idx, (void *)h->sortKey, (void *)h->sortVal,
                  (void *)h->sc, (void *)h->covPart, (void *)h->infeas,
                  (void *)h->assign, (void *)h->blockEnd, (void *)h->usedBlocks, (void *)h->Y, (void *)h->Yc, (void *)h->Tt,
                  (void *)h->eigTrace, (void *)h->kidx, (void *)h->shardCnt, (void *)h->part, (void *)h->G,
                  (void *)h->gran, (void *)h->mask, (void *)h->maskSigma, (void *)h->ubuf, (void *)h->uused,
                  (void *)h->selEnd, (void *)h->V, (void *)h->auxC, (void *)h->violDev, (void *)h->pairI,
                  (void *)h->pairC, (void *)h->pairCnt, (void *)h->listDev, (void *)h->dzT, (void *)h->shardPos,
                  (void *)h->shardCounts, (void *)h->rows, (void *)h->covPack})
    if (p) dev_release(p);
  for (auto &t : h->pending) {
    (void)hipEventDestroy(std::get<1>(t));
    (void)hipEventDestroy(std::get<2>(t));
  }
  for (auto &m : h->openMarks) (void)hipEventDestroy(m.second);
  if (h->stream2) {
    (void)hipStreamSynchronize(h->stream2);
    stream_release(h->stream2);
  }
  if (h->evY) (void)hipEventDestroy(h->evY);
  if (h->evC) (void)hipEventDestroy(h->evC);
  stream_release(h->stream);
  delete h;
  return 0;
}

int kg_cmaes_initialize(kg_cmaes_t h) {
  Stage st(h, "init");
  h->stateDirty = true;
  // setInitialConfiguration (:54-66, :132-170): CCMA-ES starts in the viability regime
  h->viability = h->nc > 0;
  if (h->viability) {
    const int lv = (int)h->cfg.viability_population_size;
    const int mv = (int)(h->cfg.viability_mu_value ? h->cfg.viability_mu_value : h->cfg.viability_population_size / 2);
    if (set_current(h, lv, mv)) return 1;
    std::fill(h->cEval.begin(), h->cEval.end(), 0.0);
    std::fill(h->cInd.begin(), h->cInd.end(), 0.0);
    std::fill(h->cCnt.begin(), h->cCnt.end(), 0.0);
    std::fill(h->vBounds.begin(), h->vBounds.end(), 0.0);
    std::fill(h->bestCEval.begin(), h->bestCEval.end(), 0.0);
    h->cEvalCount = h->adaptCount = h->maxViolCount = 0.0;
    KG_HIP(hipMemsetAsync(h->V, 0, h->nc * (size_t)h->N * sizeof(double), h->stream));
  } else if (set_current(h, h->lamCfg, h->muCfg)) {
    return 1;
  }
  hipLaunchKernelGGL(k_init, dim3(1), dim3(256), 0, h->stream, h->N, h->lam, h->mu, h->cfg.mu_type,
                     h->cfg.initial_sigma_cumulation_factor, h->cfg.initial_damp_factor,
                     h->cfg.initial_cumulative_covariance, h->iv, h->istd, h->w, h->C, h->B, h->D, h->mean,
                     h->prevMean, h->pc, h->ps, h->sc, 1, h->nc > 0 ? 1 : 0);
  KG_HIP(hipGetLastError());
  return 0;
}

static int cmaes_eigen(kg_cmaes_t h) {
  Stage st(h, "eigen");
  h->eig.trace = h->eigTrace;
  return h->eig.run(h->C, h->cfg.diagonal_covariance, h->B, h->D, &h->sc->minEig, &h->sc->maxEig,
                    &h->sc->eigenFailures, &h->sc->errors, h->stream, eig_prof, h);
}

static int cmaes_draw_begin(kg_cmaes_t h) {
  const int N = h->N;
  const size_t rows = h->blocks;
  if (h->normal.prefetch(rows * N, h->stream)) return 1;  // overlaps the eigensolver
  // the polar pass reads only the generator stream: it runs on the
  // producer's side stream too, concurrently with the eigensolver
  const bool shard = h->shards > 1 && !h->replSample;
  return h->normal.polar_normals(h->Z, rows * N, N, h->blockEnd, h->normal.side_stream(),
                                 shard ? (size_t)h->r0 * N : 0, shard ? (size_t)h->r1 * N : (size_t)-1);
}

int kg_cmaes_begin_sample(kg_cmaes_t h) {
  if (h->sampleBegun) return 0;
  if (h->nc) return 0;  // CCMA-ES: the regime check may reset C before the next draw
  if (cmaes_draw_begin(h)) return 1;
  h->eig.trace = h->eigTrace;
  if (h->eig.run_begin(h->C, h->cfg.diagonal_covariance, h->B, h->D, &h->sc->minEig, &h->sc->maxEig,
                       &h->sc->eigenFailures, &h->sc->errors, h->stream, eig_prof, h))
    return 1;
  h->sampleBegun = true;
  return 0;
}

// x = m + sigma B (D o z) for `rows` rows into Xo / Bo (+ infeasibility flags):
// k_transform_sc (scalar-operand B, KORALI_AMD_TRANSFORM_SC = 8 | 16 columns
// per wave; 16 spills SGPRs) or k_transform (LDS-tiled, KORALI_AMD_TRANSFORM_SC = 0); the
// diagonal covariance always takes k_transform's epilogue-only path
static int cmaes_transform(kg_cmaes_t h, size_t rows, double *Xo, double *Bo, int no_reserve, int mirrored) {
  const int N = h->N, W = h->cfg.diagonal_covariance ? 0 : h->trW;
  if (rows == 0) return 0;
  if (W == 0) {
    hipLaunchKernelGGL((k_transform<32, 64>), dim3(tr_grid<32, 64>((int)rows, N)), dim3(256), 0, h->stream, N,
                       (int)rows, h->cfg.diagonal_covariance, h->Z, h->B, h->D, h->mean, h->sc, h->lb, h->ub, Xo, Bo,
                       h->infeas, no_reserve, mirrored);
    KG_HIP(hipGetLastError());
    return 0;
  }
  const int ldz = sc_ldz(rows);
  if ((size_t)ldz > h->dzTRows) {
    if (h->dzT) dev_release(h->dzT, h->stream);
    h->dzT = nullptr;
    h->dzTRows = 0;
    if (dalloc(&h->dzT, (size_t)ldz * N)) return 1;
    h->dzTRows = (size_t)ldz;
  }
  hipLaunchKernelGGL(k_prescale_t, dim3((unsigned)(ldz / PS_T), (unsigned)((N + PS_T - 1) / PS_T)), dim3(256), 0,
                     h->stream, N, (int)rows, ldz, h->Z, h->D, mirrored, h->dzT);
  KG_HIP(hipGetLastError());
  if (W == 82)
    hipLaunchKernelGGL((k_transform_sc<8, 2>), dim3(trs_grid<8, 2>((int)rows, N)), dim3(256), 0, h->stream, N,
                       (int)rows, ldz, h->dzT, h->B, h->mean, h->sc, h->lb, h->ub, Xo, Bo, h->infeas, no_reserve);
  else if (W == 8)
    hipLaunchKernelGGL((k_transform_sc<8, 1>), dim3(trs_grid<8, 1>((int)rows, N)), dim3(256), 0, h->stream, N,
                       (int)rows, ldz, h->dzT, h->B, h->mean, h->sc, h->lb, h->ub, Xo, Bo, h->infeas, no_reserve);
  else
    hipLaunchKernelGGL((k_transform_sc<16, 1>), dim3(trs_grid<16, 1>((int)rows, N)), dim3(256), 0, h->stream, N,
                       (int)rows, ldz, h->dzT, h->B, h->mean, h->sc, h->lb, h->ub, Xo, Bo, h->infeas, no_reserve);
  KG_HIP(hipGetLastError());
  return 0;
}

// Overflow guard of a generation without finite bounds (and no discrete
// variables): the reference redraws a sample only when it is not finite
// (optimizer.cpp.base:5-14), which needs |m| + sigma |B (D o z)| to overflow.
// *finite = every draw of this generation is provably finite (|z| <=
// KG_DRAW_ZMAX), so the population is the first lambda blocks of the stream.
// The bound comes from the last update's termination record (host-coherent,
// already written when the host chase returns) or, when the caller set the
// state since (initialize, set_field), from the state itself.
static int draw_guard(kg_cmaes_t h, bool *finite, bool *stateFinite = nullptr) {
  double G = NAN;
  if (!stateFinite && !h->stateDirty && h->updates > 0) {
    const unsigned long long want = h->updates;
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(&h->summary->seq, __ATOMIC_ACQUIRE) < want) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
        KG_HIP(hipStreamSynchronize(h->stream));
        if (check_errors(h)) return 1;
        KG_CHECK(false, "termination summary never arrived");
      }
    }
    G = h->summary->guard;
  } else {
    const int N = h->N;
    std::vector<double> m(N), D(N);
    double sigma = 0.0;
    KG_HIP(hipMemcpyAsync(m.data(), h->mean, N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipMemcpyAsync(D.data(), h->D, N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipMemcpyAsync(&sigma, &h->sc->sigma, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    double ma = 0.0, dm = 0.0;
    bool ok = std::isfinite(sigma);
    for (int d = 0; d < N; d++) {
      ok = ok && std::isfinite(m[d]) && std::isfinite(D[d]);
      ma += std::fabs(m[d]);
      dm = std::max(dm, std::fabs(D[d]));
    }
    if (ok) G = ma + sigma * KG_DRAW_ZMAX * (double)N * dm;
    if (stateFinite) *stateFinite = ok;
  }
  *finite = G < KG_DRAW_GUARD_LIMIT;  // false for NaN
  return 0;
}

// buffers of the redraw path for a handle created without a reserve
static int ensure_redraw_buffers(kg_cmaes_t h) {
  if (h->Xall) return 0;
  const size_t xrows = h->mirrored ? 2 * (size_t)(h->lamMax / 2) : (size_t)h->lamMax;  // (no reserve: R = 0)
  if (dalloc(&h->Xall, xrows * h->N)) return 1;
  if (h->cfg.store_bdz && dalloc(&h->BDZall, xrows * h->N)) return 1;
  return 0;
}

// prepareGeneration's redraw loops (CMAES.cpp.base:443-491) in rounds: each
// round transforms the next `blocks` blocks of the Normal stream (the first
// round's were drawn beside the eigensolver), walks them in the reference's
// order from the first unassigned sample, and consumes exactly the blocks the
// walk used.  When a round runs out of blocks, the next one continues the
// stream where it stopped, so any number of infeasible draws is followed.
static int cmaes_resample(kg_cmaes_t h) {
  const int N = h->N, L = h->lam;
  const size_t nb = h->blocks, xr = h->mirrored ? 2 * nb : nb;
  int i0 = 0;
  for (int round = 0;; round++) {
    if (round > 0) {
      h->resamplingRounds++;
      Stage st(h, "rng_polar");
      if (h->normal.polar_normals(h->Z, nb * N, N, h->blockEnd, h->stream)) return 1;
    }
    {
      Stage st(h, "transform");
      KG_HIP(hipMemsetAsync(h->infeas, 0, xr * sizeof(int), h->stream));
      if (cmaes_transform(h, xr, h->Xall, h->BDZall, 0, h->mirrored ? 1 : 0)) return 1;
      if (h->hasDiscrete) {
        if (h->uniform.peek_uniforms(h->ubuf, h->ucap, h->stream)) return 1;
        hipLaunchKernelGGL(k_discrete_select, dim3(1), dim3(256), 2 * N * sizeof(double), h->stream, N, L, i0, (int)nb,
                           h->mirrored ? 1 : 0, h->cfg.max_infeasible_resamplings, h->Xall, h->BDZall, h->X, h->BDZ,
                           h->lb, h->ub, h->gran, h->mask, h->bestEverVars, h->ubuf, (unsigned long long)h->ucap,
                           h->uused, h->usedBlocks, h->selEnd, h->sc);
        KG_HIP(hipGetLastError());
        if (h->uniform.consume_words_dev(h->uused, h->stream)) return 1;
      } else {
        if (h->mirrored)
          hipLaunchKernelGGL(k_select_mirrored, dim3(1), dim3(64), 0, h->stream, L, i0, (int)nb,
                             h->cfg.max_infeasible_resamplings, h->infeas, h->assign, h->usedBlocks, h->selEnd, h->sc);
        else
          hipLaunchKernelGGL(k_select, dim3(1), dim3(64), 0, h->stream, L, i0, (int)nb,
                             h->cfg.max_infeasible_resamplings, h->infeas, h->assign, h->usedBlocks, h->selEnd, h->sc);
        KG_HIP(hipGetLastError());
        const size_t tot = (size_t)(L - i0) * N;
        hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, N, i0,
                           (const int *)h->selEnd, h->assign, h->Xall, h->X, h->BDZall, h->BDZ);
        KG_HIP(hipGetLastError());
      }
    }
    {
      Stage st(h, "rng_consume");
      if (h->normal.consume_normals_dev(h->usedBlocks, N, h->blockEnd, h->stream)) return 1;
    }
    int se[2] = {0, 0};
    KG_HIP(hipMemcpyAsync(se, h->selEnd, sizeof(se), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    if (se[0] >= L) break;
    if (se[0] == i0) {
      // a round without progress: either the peeked uniforms were too few
      // for one attempt (discrete mutations), or no draw of a whole round
      // was feasible.  The reference keeps redrawing; a distribution that is
      // not finite would make it redraw forever, which is reported instead.
      if (se[1]) {
        const size_t cap = 2 * h->ucap;
        KG_CHECK(cap + 4096 <= h->uniform.capacity_words() / 2,
                 "discrete mutations need more uniforms per sample than the device window holds");
        double *nb2 = nullptr;
        if (dalloc(&nb2, cap)) return 1;
        dev_release(h->ubuf, h->stream);
        h->ubuf = nb2;
        h->ucap = cap;
      } else {
        bool fin = false, stateFinite = false;
        if (draw_guard(h, &fin, &stateFinite)) return 1;
        KG_CHECK(stateFinite, "the sampling distribution (mean, sigma, axis lengths) is not finite: every draw is "
                              "infeasible and the reference would redraw forever");
      }
    }
    i0 = se[0];
  }
  if (!h->R) {
    // a handle without a reserve consumes exactly its lambda blocks otherwise
    const unsigned long long used = (unsigned long long)nb;
    KG_HIP(hipMemcpyAsync(h->usedBlocks, &used, sizeof(used), hipMemcpyHostToDevice, h->stream));
  }
  return 0;
}

int kg_cmaes_sample(kg_cmaes_t h) {
  const int N = h->N;
  if (!h->sampleBegun && cmaes_draw_begin(h)) return 1;
  h->sampleBegun = false;
  if (cmaes_eigen(h)) return 1;
  {
    Stage st(h, "rng_polar");  // what of the producer + polar pass the eigensolver did not hide
    if (h->normal.join(h->stream)) return 1;
  }
  bool redraw = h->R > 0;
  if (!redraw) {
    bool finite = false;
    if (draw_guard(h, &finite)) return 1;
    if (!finite) {
      KG_CHECK(h->shards == 1 || h->replSample,
               "a population-sharded handle cannot redraw non-finite samples (overflow guard tripped)");
      if (ensure_redraw_buffers(h)) return 1;
      redraw = true;
    }
  }
  if (redraw) return cmaes_resample(h);
  {
    Stage st(h, "transform");
    // no redraw possible: the population is the first lambda blocks; a shard
    // transforms its own rows only
    const int t0 = h->replSample ? 0 : h->r0, t1 = h->replSample ? h->lam : h->r1;
    const size_t trows = (size_t)(t1 - t0);
    double *xo = h->X + (size_t)t0 * N;
    double *bo = h->BDZ ? h->BDZ + (size_t)t0 * N : nullptr;
    // 32 x 64 tiles, 4 x 2 outputs per thread: larger register tiles drop the
    // kernel to 2 waves per SIMD and measured slower at C4 (1.96 / 2.25 ms
    // for 32 x 128 / 64 x 64 against 1.73 ms)
    if (cmaes_transform(h, trows, xo, bo, 1, h->mirrored ? 1 : 0)) return 1;
  }
  {
    Stage st(h, "rng_consume");
    if (h->normal.consume_normals_dev(h->usedBlocks, N, h->blockEnd, h->stream)) return 1;
  }
  return 0;
}

int kg_cmaes_eval_builtin(kg_cmaes_t h, int objective) {
  KG_CHECK(objective >= 0 && objective <= 2, "unknown builtin objective");
  Stage st(h, "objective");
  const int rows = h->r1 - h->r0;
  if (h->N <= 128)
    hipLaunchKernelGGL(k_objective2, dim3((rows + OB2_R - 1) / OB2_R), dim3(256), ob2_lds_bytes(h->N), h->stream,
                       h->N, rows, objective, h->X + (size_t)h->r0 * h->N, h->F + h->r0, h->sc, (double)h->lam);
  else
    hipLaunchKernelGGL(k_objective, dim3((rows + OB_C - 1) / OB_C), dim3(256), 0, h->stream, h->N, rows, objective,
                       h->X + (size_t)h->r0 * h->N, h->F + h->r0, h->sc, (double)h->lam);
  KG_HIP(hipGetLastError());
  return 0;
}

int kg_cmaes_get_candidates(kg_cmaes_t h, double *X, size_t ld) {
  const size_t N = h->N;
  if (ld == 0) ld = N;
  KG_HIP(hipMemcpy2DAsync(X, ld * sizeof(double), h->X, N * sizeof(double), N * sizeof(double), h->lam,
                          hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

static int cmaes_upload_fitness(kg_cmaes_t h, const double *F, bool allow_neg_inf) {
  for (int i = 0; i < h->lam; i++)
    KG_CHECK(std::isfinite(F[i]) || (allow_neg_inf && F[i] == -INFINITY),
             "Non finite value of function evaluation detected: " + std::to_string(F[i]));
  KG_HIP(hipMemcpyAsync(h->F, F, h->lam * sizeof(double), hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(k_add_evals, dim3(1), dim3(1), 0, h->stream, h->sc, (double)h->lam);
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_cmaes_set_fitness(kg_cmaes_t h, const double *F) { return cmaes_upload_fitness(h, F, false); }

int kg_cmaes_set_log_posterior(kg_cmaes_t h, const double *F) { return cmaes_upload_fitness(h, F, true); }

int kg_cmaes_set_gradients(kg_cmaes_t h, const double *G) {
  KG_CHECK(h->G, "kg_cmaes_set_gradients: the handle was created without use_gradients");
  KG_CHECK(G, "kg_cmaes_set_gradients: null argument");
  KG_HIP(hipMemcpyAsync(h->G, G, (size_t)h->lam * h->N * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));  // G may be a caller's temporary
  return 0;
}

static int cmaes_sort(kg_cmaes_t h) {
  const int L = h->lam;
  {
    Stage st(h, "sort");
    int P2 = 1;
    while (P2 < L) P2 <<= 1;
    if (L <= RANK_MAX && L > 256) {
      hipLaunchKernelGGL(k_rank_sort, dim3((L + 15) / 16), dim3(256), (size_t)L * sizeof(double), h->stream, L, h->F,
                         h->idx);
    } else if (P2 <= SORT_CHUNK) {
      hipLaunchKernelGGL(k_sort_small, dim3(1), dim3(1024), 0, h->stream, L, P2, h->F, h->idx);
    } else {
      hipLaunchKernelGGL(k_sort_init, dim3((P2 + 1023) / 1024), dim3(1024), 0, h->stream, L, P2, h->F, h->sortKey,
                         h->sortVal);
      hipLaunchKernelGGL(k_sort_local, dim3(P2 / SORT_CHUNK), dim3(1024), 0, h->stream, P2, 0, h->sortKey,
                         h->sortVal);
      for (int k = 2 * SORT_CHUNK; k <= P2; k <<= 1) {
        for (int j = k / 2; j >= SORT_CHUNK; j >>= 1)
          hipLaunchKernelGGL(k_sort_global, dim3((P2 + 255) / 256), dim3(256), 0, h->stream, P2, k, j, h->sortKey,
                             h->sortVal);
        hipLaunchKernelGGL(k_sort_local, dim3(P2 / SORT_CHUNK), dim3(1024), 0, h->stream, P2, k, h->sortKey,
                           h->sortVal);
      }
      hipLaunchKernelGGL(k_copy_idx, dim3((L + 255) / 256), dim3(256), 0, h->stream, L, h->sortVal, h->idx);
    }
    KG_HIP(hipGetLastError());
  }
  return 0;
}

static int cmaes_sigma(kg_cmaes_t h, size_t gen) {
  const int N = h->N, mu = h->mu;
  {
    Stage st(h, "sigma");
    if (h->hasDiscrete)
      hipLaunchKernelGGL(k_discrete_masks, dim3(1), dim3(64), 0, h->stream, N, h->lam, h->gran, h->C, h->mask,
                         h->maskSigma, h->sc);
    hipLaunchKernelGGL(k_sigma, dim3(1), dim3(256), 0, h->stream, N, mu, h->cfg.is_sigma_bounded, h->C, h->F, h->idx,
                       h->minstd, h->sc, h->normal.state(), h->uniform.state(), h->summaryDev, ++h->updates,
                       h->hasDiscrete ? h->maskSigma : (const double *)nullptr, h->ps, h->mean, h->muCfg,
                       h->viability ? 1 : 0, h->cfg.target_success_rate, h->cfg.global_success_learning_rate,
                       (unsigned long long)(gen + 1));
    h->stateDirty = false;  // the record's guard describes the next draw
    KG_HIP(hipGetLastError());
  }
  return 0;
}


// KORALI_AMD_ROWCHAINS=0: the round-3 lockstep-lane mean / paths kernels (A/B)
// the exact rank-mu sums on lane chains (k_adaptC_lane) from N = 256 up:
// measured round 5 (gpurun_out/r5z) C4 (N = 512) 3.75 -> 2.14 ms per
// generation, C2 (N = 128: 36 tiles, a third of the chip) 0.036 -> 0.060 ms,
// so C2 keeps the row chains (KORALI_AMD_ADAPTC_LANE_MIN moves the switch)
static bool lane_chains(int N) {
  static const int from = [] {
    const char *e = getenv("KORALI_AMD_ADAPTC_LANE_MIN");
    return e && *e ? atoi(e) : 256;
  }();
  return N >= from;
}
static bool row_chains() {
  static const bool on = [] {
    const char *e = getenv("KORALI_AMD_ROWCHAINS");
    return !(e && *e == '0');
  }();
  return on;
}

static int cmaes_paths(kg_cmaes_t h, size_t generation) {
  const int N = h->N;
  if (N <= 128 && !h->cfg.diagonal_covariance && row_chains()) {
    hipLaunchKernelGGL(k_paths3, dim3(1), dim3(PR_T), 0, h->stream, N, (unsigned long long)generation, h->B, h->D,
                       h->meanUpdate, h->auxBDZ, h->ps, h->pc, h->sc);
    KG_HIP(hipGetLastError());
    return 0;
  }
  if (N <= 128 && !h->cfg.diagonal_covariance) {
    hipLaunchKernelGGL(k_paths2, dim3(1), dim3(256), paths2_lds_bytes(N), h->stream, N, (unsigned long long)generation,
                       h->B, h->D, h->meanUpdate, h->auxBDZ, h->ps, h->pc, h->sc);
    KG_HIP(hipGetLastError());
    return 0;
  }
  const size_t pbytes = ((size_t)N * (PA_EC + 1) + N) * sizeof(double);
  hipLaunchKernelGGL(k_paths, dim3(1), dim3(N <= 1024 ? ((N + 63) / 64) * 64 : 1024), pbytes, h->stream, N,
                     h->cfg.diagonal_covariance, (unsigned long long)generation, h->B, h->D, h->meanUpdate,
                     h->auxBDZ, h->ps, h->pc, h->sc);
  KG_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ CCMA-ES
// The constraint stages of CMAES::runGeneration (CMAES.cpp.base:190-196).
// Constraint values are host callbacks (the reference's per-sample Python /
// C++ functions); their bookkeeping (violation counts, indicators, viability
// boundaries) is O(lambda x constraints) and stays on this host thread; the
// covariance correction, its eigendecomposition and the redraws run on the
// device.

// constraint values of rows `ids` of X (device) or of the mean
static int ccm_eval(kg_cmaes_t h, const std::vector<size_t> &ids, bool mean, std::vector<double> &out) {
  KG_CHECK(h->cfn, "constraints configured but kg_cmaes_set_constraints was not called");
  const size_t N = h->N, rows = mean ? 1 : ids.size();
  std::vector<double> X(rows * N);
  if (mean) {
    KG_HIP(hipMemcpyAsync(X.data(), h->mean, N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  } else {
    for (size_t r = 0; r < rows; r++)
      KG_HIP(hipMemcpyAsync(X.data() + r * N, h->X + ids[r] * N, N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  }
  KG_HIP(hipStreamSynchronize(h->stream));
  out.assign(rows * h->nc, 0.0);
  std::vector<size_t> mid(1, (size_t)-1);
  if (h->cfn(X.data(), rows, N, mean ? mid.data() : ids.data(), out.data(), h->cctx) != 0) {
    set_error("constraint evaluation failed");
    return 1;
  }
  for (size_t q = 0; q < out.size(); q++)
    KG_CHECK(std::isfinite(out[q]), "Non finite value of constraint evaluation " + std::to_string(q % h->nc) +
                                        " detected: " + std::to_string(out[q]));
  h->cEvalCount += (double)rows;
  return 0;
}

// checkMeanAndSetRegime (:315-348)
static int ccm_check_mean(kg_cmaes_t h) {
  if (!h->viability) return 0;
  std::vector<double> ev;
  if (ccm_eval(h, {}, true, ev)) return 1;
  for (size_t c = 0; c < h->nc; c++)
    if (ev[c] > 0.0) return 0;
  h->viability = false;
  std::fill(h->vBounds.begin(), h->vBounds.end(), 0.0);
  if (set_current(h, h->lamCfg, h->muCfg)) return 1;
  hipLaunchKernelGGL(k_init, dim3(1), dim3(256), 0, h->stream, h->N, h->lam, h->mu, h->cfg.mu_type,
                     h->cfg.initial_sigma_cumulation_factor, h->cfg.initial_damp_factor,
                     h->cfg.initial_cumulative_covariance, h->iv, h->istd, h->w, h->C, h->B, h->D, h->mean,
                     h->prevMean, h->pc, h->ps, h->sc, 0, 1);
  KG_HIP(hipGetLastError());
  h->stateDirty = true;
  return 0;
}

// updateConstraints (:350-387)
static int ccm_update_constraints(kg_cmaes_t h, size_t generation) {
  const size_t L = h->lam, S = h->lamMax, nc = h->nc;
  std::vector<size_t> ids(L);
  for (size_t i = 0; i < L; i++) ids[i] = i;
  std::vector<double> ev;
  if (ccm_eval(h, ids, false, ev)) return 1;
  for (size_t i = 0; i < L; i++) {
    h->cCnt[i] = 0;
    for (size_t c = 0; c < nc; c++) h->cEval[c * S + i] = ev[i * nc + c];
  }
  h->maxViolCount = 0;
  for (size_t c = 0; c < nc; c++) {
    double maxviolation = 0.0;
    for (size_t i = 0; i < L; ++i) {
      const double e = h->cEval[c * S + i];
      if (e > maxviolation) maxviolation = e;
      if (generation == 1 && h->viability) h->vBounds[c] = maxviolation;
      if (e > h->vBounds[c] + 1e-12) h->cCnt[i] += 1;
      if (h->cCnt[i] > h->maxViolCount) h->maxViolCount = h->cCnt[i];
    }
  }
  return 0;
}

// redraw the listed samples (handleConstraints :806-822) in rounds of the
// Normal stream, as cmaes_resample
static int ccm_redraw(kg_cmaes_t h, const std::vector<int> &list) {
  const int N = h->N, nl = (int)list.size();
  if (ensure_redraw_buffers(h)) return 1;  // (unbounded variables: no reserve rows yet)
  const size_t nb = h->blocks;
  KG_HIP(hipMemcpyAsync(h->listDev, list.data(), nl * sizeof(int), hipMemcpyHostToDevice, h->stream));
  int k0 = 0;
  for (;;) {
    if (h->normal.polar_normals(h->Z, nb * N, N, h->blockEnd, h->stream)) return 1;
    KG_HIP(hipMemsetAsync(h->infeas, 0, nb * sizeof(int), h->stream));
    if (cmaes_transform(h, nb, h->Xall, h->BDZall, 0, 0)) return 1;
    hipLaunchKernelGGL(k_select_list, dim3(1), dim3(64), 0, h->stream, nl, k0, (int)nb,
                       h->cfg.max_infeasible_resamplings, h->infeas, h->assign, h->usedBlocks, h->selEnd, h->sc);
    const size_t tot = (size_t)(nl - k0) * N;
    hipLaunchKernelGGL(k_gather_list, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, N, k0,
                       (const int *)h->selEnd, (const int *)h->listDev, h->assign, h->Xall, h->X, h->BDZall, h->BDZ);
    KG_HIP(hipGetLastError());
    if (h->normal.consume_normals_dev(h->usedBlocks, N, h->blockEnd, h->stream)) return 1;
    int se[2] = {0, 0};
    KG_HIP(hipMemcpyAsync(se, h->selEnd, sizeof(se), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    if (se[0] >= nl) break;
    k0 = se[0];
  }
  return 0;
}

// handleConstraints (:774-832) + reEvaluateConstraints (:389-422)
static int ccm_handle_constraints(kg_cmaes_t h) {
  const int N = h->N;
  const size_t L = h->lam, S = h->lamMax, nc = h->nc;
  const double beta = 1.0 / (2.0 + N), cmaf = h->cfg.covariance_matrix_adaption_strength / (N + 2.);
  while (h->maxViolCount > 0) {
    // the (sample, constraint) pairs in the reference's order; the loop
    // returns at the pair that takes the count past the maximum
    std::vector<int> pi, pc;
    std::vector<double> pcnt;
    bool truncated = false;
    for (size_t i = 0; i < L && !truncated; ++i)
      if (h->cCnt[i] > 0)
        for (size_t c = 0; c < nc; c++)
          if (h->cInd[c * S + i] != 0) {
            h->adaptCount += 1;
            if (h->adaptCount > h->cfg.max_covariance_matrix_corrections) {
              truncated = true;
              break;
            }
            pi.push_back((int)i);
            pc.push_back((int)c);
            pcnt.push_back(h->cCnt[i]);
          }
    const int np = (int)pi.size();
    if (np) {
      KG_HIP(hipMemcpyAsync(h->pairI, pi.data(), np * sizeof(int), hipMemcpyHostToDevice, h->stream));
      KG_HIP(hipMemcpyAsync(h->pairC, pc.data(), np * sizeof(int), hipMemcpyHostToDevice, h->stream));
      KG_HIP(hipMemcpyAsync(h->pairCnt, pcnt.data(), np * sizeof(double), hipMemcpyHostToDevice, h->stream));
    }
    hipLaunchKernelGGL(k_ccm_adapt, dim3(1), dim3(256), 0, h->stream, N, np, h->pairI, h->pairC, h->pairCnt, h->BDZ,
                       h->V, beta, cmaf, h->C, h->auxC);
    KG_HIP(hipGetLastError());
    KG_HIP(hipStreamSynchronize(h->stream));  // (the pair vectors are temporaries)
    if (truncated) return 0;                  // "max adaptions reached" (:787-791)
    // updateEigensystem(auxC)
    if (h->eig.run(h->auxC, h->cfg.diagonal_covariance, h->B, h->D, &h->sc->minEig, &h->sc->maxEig,
                   &h->sc->eigenFailures, &h->sc->errors, h->stream, eig_prof, h))
      return 1;
    std::vector<int> list;
    for (size_t i = 0; i < L; ++i)
      if (h->cCnt[i] > 0) list.push_back((int)i);
    if (ccm_redraw(h, list)) return 1;
    // reEvaluateConstraints
    std::vector<size_t> ids(list.begin(), list.end());
    std::vector<double> ev;
    if (ccm_eval(h, ids, false, ev)) return 1;
    h->maxViolCount = 0;
    for (size_t r = 0; r < ids.size(); r++) {
      const size_t i = ids[r];
      h->cCnt[i] = 0;
      for (size_t c = 0; c < nc; c++) {
        h->cEval[c * S + i] = ev[r * nc + c];
        if (ev[r * nc + c] > h->vBounds[c] + 1e-12) {
          h->cInd[c * S + i] = 1;
          h->cCnt[i] += 1;
        } else {
          h->cInd[c * S + i] = 0;
        }
      }
      if (h->cCnt[i] > h->maxViolCount) h->maxViolCount = h->cCnt[i];
    }
  }
  return 0;
}

// after updateDistribution: updateViabilityBoundaries (:424-437; the sigma
// step does not read them) and the best constraint values (:576-579)
static int ccm_after_update(kg_cmaes_t h) {
  const size_t L = h->lam, S = h->lamMax, nc = h->nc;
  std::vector<unsigned> idx(L);
  CmaesScalars hs;
  KG_HIP(hipMemcpyAsync(idx.data(), h->idx, L * sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipMemcpyAsync(&hs, h->sc, sizeof(hs), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  if (hs.errors & KG_ERR_CONSTRAINT) return check_errors(h);
  if (hs.bestFlag)
    for (size_t c = 0; c < nc; c++) h->bestCEval[c] = h->cEval[c * S + (size_t)hs.bestValidSample];
  if (h->viability)
    for (size_t c = 0; c < nc; c++) {
      double maxviolation = 0.0;
      for (int i = 0; i < h->mu; ++i)
        if (h->cEval[c * S + idx[i]] > maxviolation) maxviolation = h->cEval[c * S + idx[i]];
      const double t = 0.5 * (maxviolation + h->vBounds[c]);
      const double mn = (t < h->vBounds[c]) ? t : h->vBounds[c];  // std::min
      h->vBounds[c] = (0.0 < mn) ? mn : 0.0;                     // std::max(0.0, .)
    }
  return 0;
}

// C is final once the covariance update has run (k_sigma and the
// termination record only read it): with the tridiagonalisation on the host
// core, the next eigendecomposition's hand-off (k_publish_c) goes ahead of
// k_sigma, so the host starts on C while sigma and the record are computed.
// (CCMA-ES may still reset C in ccm_after_update; KORALI_AMD_EARLY_PUBLISH=0
// restores the order publish-after-sigma.)
static int early_publish(kg_cmaes_t h) {
  static const bool early = [] {
    const char *e = getenv("KORALI_AMD_EARLY_PUBLISH");
    return !(e && *e == '0');
  }();
  if (!early || h->nc || !h->eig.host_tridiag() || h->cfg.diagonal_covariance) return 0;
  h->eig.trace = h->eigTrace;
  return h->eig.run_begin(h->C, 0, h->B, h->D, &h->sc->minEig, &h->sc->maxEig, &h->sc->eigenFailures, &h->sc->errors,
                          h->stream, eig_prof, h);
}

int kg_cmaes_update(kg_cmaes_t h, size_t generation) {
  KG_CHECK(h->shards == 1, "a population-sharded handle updates through kg_cmaes_update_partial / _finalize");
  const int N = h->N, mu = h->mu;
  if (cmaes_sort(h)) return 1;
  {
    Stage st(h, "mean_paths");
    const bool ccm = h->nc > 0 && !h->viability;  // the best VALID sample (:551-558)
    if (ccm) {
      std::vector<int> viol(h->lam);
      for (int i = 0; i < h->lam; i++) viol[i] = h->cCnt[i] > 0 ? 1 : 0;
      KG_HIP(hipMemcpyAsync(h->violDev, viol.data(), h->lam * sizeof(int), hipMemcpyHostToDevice, h->stream));
      KG_HIP(hipStreamSynchronize(h->stream));  // (viol is a temporary)
    }
    // one launch for the best bookkeeping, the gather and the exact factors
    // when nothing between them needs a grid-wide order (no constraints, no
    // proportional weights, a k_sigma already cleared the range flag;
    // KORALI_AMD_FUSED_SELECT=0: the three kernels)
    static const bool fusedSel = [] {
      const char *e = getenv("KORALI_AMD_FUSED_SELECT");
      return !(e && *e == '0');
    }();
    const bool fused = fusedSel && !ccm && h->nc == 0 && h->cfg.mu_type != KG_MU_PROPORTIONAL &&
                       h->cfg.cov_mode != KG_COV_MFMA && h->updates > 0;
    if (fused) {
      hipLaunchKernelGGL(k_select_prep, dim3((mu + RP_T - 1) / RP_T, (N + RP_T - 1) / RP_T), dim3(256), 0, h->stream,
                         N, mu, (unsigned long long)generation, h->X, h->F, h->idx, h->w, h->mean, h->prevMean, h->Y,
                         h->currBestVars, h->bestEverVars, h->sc, h->Yc, h->Tt);
      KG_HIP(hipGetLastError());
    } else {
    hipLaunchKernelGGL(k_update_best, dim3(1), dim3(256), 0, h->stream, N, mu, h->cfg.mu_type,
                       (unsigned long long)generation, h->X, h->F, h->idx, h->w, h->currBestVars, h->bestEverVars,
                       h->sc, ccm ? (const int *)h->violDev : (const int *)nullptr, h->lam);
    hipLaunchKernelGGL(k_gather_selected, dim3(mu), dim3(128), 0, h->stream, N, mu, h->X, h->idx, h->Y, h->mean,
                       h->prevMean);
    }
    // the rank-mu sum (MFMA) needs only Y, the weights and m_prev: it runs on
    // the second stream while the mean and the evolution paths are computed.
    // The exact mode's factors (k_rankmu_prep, ~6 us) run in line: the two
    // cross-queue waits of a second stream cost more (~7 us each, kernel trace)
    if (h->cfg.cov_mode == KG_COV_MFMA) {
      KG_HIP(hipEventRecord(h->evY, h->stream));
      KG_HIP(hipStreamWaitEvent(h->stream2, h->evY, 0));
      Stage st(h, "rankmu_mfma", h->stream2);
      hipLaunchKernelGGL(k_rankmu_tile<false>, dim3(rankmu_grid(N, h->kslices)), dim3(256), 0, h->stream2, N, mu,
                         (const int *)nullptr, h->kslices, h->Y, (const int *)nullptr, h->w, h->prevMean, h->sc,
                         h->covPart);
      KG_HIP(hipGetLastError());
      KG_HIP(hipEventRecord(h->evC, h->stream2));
    } else if (!fused) {
      hipLaunchKernelGGL(k_rankmu_prep, dim3((mu + RP_T - 1) / RP_T, (N + RP_T - 1) / RP_T), dim3(256), 0,
                         h->stream, N, mu, h->Y, h->w, h->prevMean, h->sc, h->Yc, h->Tt);
      KG_HIP(hipGetLastError());
    }
    if (row_chains())
      hipLaunchKernelGGL(k_mean3, dim3((N + 15) / 16), dim3(256), 0, h->stream, N, mu, h->Y, h->w, h->mean,
                         h->prevMean, h->meanUpdate, h->sc);
    else
      hipLaunchKernelGGL(k_mean2, dim3((N + MN_D - 1) / MN_D), dim3(256), mean2_lds_bytes(), h->stream, N, mu,
                         h->Y, h->w, h->mean, h->prevMean, h->meanUpdate, h->sc);
    if (h->G)
      hipLaunchKernelGGL(k_mean_gradient, dim3((N + 63) / 64), dim3(64), 0, h->stream, N, mu, h->cfg.gradient_step_size,
                         h->G, h->idx, h->w, h->mean, h->prevMean, h->meanUpdate, h->sc);
    if (cmaes_paths(h, generation)) return 1;
  }
  {
    Stage st(h, "covariance");
    const int nt = (N + 15) / 16, ntiles = nt * (nt + 1) / 2;
    if (h->cfg.cov_mode == KG_COV_MFMA) {
      KG_HIP(hipStreamWaitEvent(h->stream, h->evC, 0));
      hipLaunchKernelGGL(k_adaptC_combine, dim3(ntiles), dim3(256), 0, h->stream, N, h->kslices, ntiles,
                         h->cfg.diagonal_covariance, h->covPart, h->pc, h->C, h->sc, 0);
    } else {
      static const bool old2 = getenv("KORALI_AMD_ADAPTC2") != nullptr;  // A/B switch
      if (!old2 && lane_chains(N)) {
        hipLaunchKernelGGL(k_adaptC_lane, dim3(al_tiles(N)), dim3(256), 0, h->stream, N, mu,
                           h->cfg.diagonal_covariance, h->Yc, h->Tt, h->pc, h->C, h->sc, 0, (double *)nullptr);
      } else if (!old2 && row_chains()) {
        // Markstein quotients when every factor is in range (k_rankmu_prep's
        // flag, read on the device: the kernel picks the branch per launch)
        hipLaunchKernelGGL(k_adaptC_row, dim3(ar_tiles(N)), dim3(AR_NT), 0, h->stream, N, mu,
                           h->cfg.diagonal_covariance, h->Yc, h->Tt, h->pc, h->C, h->sc, 0, (double *)nullptr);
      } else if (old2)
        hipLaunchKernelGGL(k_adaptC_exact2, dim3((N + 3) / 4, (N + 63) / 64), dim3(256), 0, h->stream, N, mu,
                           h->cfg.diagonal_covariance, h->Yc, h->Tt, h->pc, h->C, h->sc);
      else
        hipLaunchKernelGGL(k_adaptC_exact3, dim3(ax3_slots(N)), dim3(64 * (AX3_P + 1)), 0, h->stream, N, mu,
                           h->cfg.diagonal_covariance, h->Yc, h->Tt, h->pc, h->C, h->sc);
    }
    KG_HIP(hipGetLastError());
  }
  if (early_publish(h)) return 1;
  if (cmaes_sigma(h, generation)) return 1;  // (k_sigma also publishes the termination record)
  return h->nc ? ccm_after_update(h) : 0;
}

int kg_cmaes_update_partial(kg_cmaes_t h, size_t generation) {
  const int N = h->N, mu = h->mu;
  if (cmaes_sort(h)) return 1;
  if (h->covPack) {
    // exact order: best bookkeeping, then this rank's selected rows into its
    // exchange block
    Stage st(h, "mean_paths");
    const int per = h->lam / h->shards;
    hipLaunchKernelGGL(k_update_best, dim3(1), dim3(256), 0, h->stream, N, mu, h->cfg.mu_type,
                       (unsigned long long)generation, (const double *)nullptr, h->F, h->idx, h->w, h->currBestVars,
                       h->bestEverVars, h->sc, (const int *)nullptr, h->lam);
    if (h->rows) {
      hipLaunchKernelGGL(k_shard_positions, dim3(1), dim3(1024), 0, h->stream, mu, per, h->shards, h->idx, h->shardPos,
                         h->shardCounts);
      hipLaunchKernelGGL(k_shard_pack, dim3(mu), dim3(128), 0, h->stream, N, h->shardRank, per, h->shards, h->idx,
                         h->shardPos, h->shardCounts, h->X, h->rows);
    }
    KG_HIP(hipGetLastError());
    h->rowBlock = -1;
    return 0;
  }
  {
    Stage st(h, "mean_paths");
    hipLaunchKernelGGL(k_update_best, dim3(1), dim3(256), 0, h->stream, N, mu, h->cfg.mu_type,
                       (unsigned long long)generation, (const double *)nullptr, h->F, h->idx, h->w, h->currBestVars,
                       h->bestEverVars, h->sc, (const int *)nullptr, h->lam);
    hipLaunchKernelGGL(k_shard_select, dim3(1), dim3(1024), 0, h->stream, mu, h->r0, h->r1, h->idx, h->kidx,
                       h->shardCnt);
    hipLaunchKernelGGL(k_gather_owned, dim3(mu), dim3(128), 0, h->stream, N, h->X, h->idx, h->kidx, h->shardCnt, h->Y);
    hipLaunchKernelGGL(k_shard_mean, dim3((N + 63) / 64), dim3(64), 0, h->stream, N, h->r0, h->r1, h->shardCnt, h->Y,
                       h->w, h->kidx, h->X, h->idx, h->part);
    KG_HIP(hipGetLastError());
  }
  {
    Stage st(h, "covariance");
    const int nt = (N + 15) / 16, ntiles = nt * (nt + 1) / 2;
    hipLaunchKernelGGL(k_rankmu_tile<true>, dim3(rankmu_grid(N, h->kslices)), dim3(256), 0, h->stream, N, 0,
                       h->shardCnt, h->kslices, h->Y, h->kidx, h->w, h->mean, h->sc, h->covPart);  // mean not yet advanced
    hipLaunchKernelGGL(k_part_reduce, dim3(ntiles), dim3(256), 0, h->stream, h->kslices, ntiles, h->covPart,
                       h->part + 2 * (size_t)N);
    KG_HIP(hipGetLastError());
  }
  return 0;
}

int kg_cmaes_shard_row_count(kg_cmaes_t h, size_t *count) {
  KG_CHECK(h->covPack, "kg_cmaes_shard_row_count: the handle is not sharded in the exact covariance mode");
  KG_CHECK(count, "kg_cmaes_shard_row_count: null argument");
  if (!h->rows) {
    h->rowBlock = 0;  // every rank holds the whole population: nothing to exchange
  } else {
    int m = 0;
    KG_HIP(hipMemcpyAsync(&m, h->shardCounts + h->shards, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    KG_CHECK(m >= 0 && (size_t)m <= h->rowsCap, "shard row count out of range (internal error)");
    h->rowBlock = m;
  }
  *count = (size_t)h->rowBlock * h->N;
  return 0;
}

int kg_cmaes_update_rows(kg_cmaes_t h, size_t generation) {
  KG_CHECK(h->covPack, "kg_cmaes_update_rows: the handle is not sharded in the exact covariance mode");
  KG_CHECK(h->rowBlock >= 0, "kg_cmaes_update_rows before kg_cmaes_shard_row_count");
  const int N = h->N, mu = h->mu;
  const int per = h->lam / h->shards;
  {
    Stage st(h, "mean_paths");
    hipLaunchKernelGGL(k_shard_unpack, dim3(mu), dim3(128), 0, h->stream, N, per, h->shards, h->idx, h->shardPos,
                       h->shardCounts, (const double *)h->rows, h->X, h->Y, h->mean, h->prevMean, h->currBestVars,
                       h->bestEverVars, h->sc);
    hipLaunchKernelGGL(k_rankmu_prep, dim3((mu + RP_T - 1) / RP_T, (N + RP_T - 1) / RP_T), dim3(256), 0, h->stream, N,
                       mu, h->Y, h->w, h->prevMean, h->sc, h->Yc, h->Tt);
    if (row_chains())
      hipLaunchKernelGGL(k_mean3, dim3((N + 15) / 16), dim3(256), 0, h->stream, N, mu, h->Y, h->w, h->mean,
                         h->prevMean, h->meanUpdate, h->sc);
    else
      hipLaunchKernelGGL(k_mean2, dim3((N + MN_D - 1) / MN_D), dim3(256), mean2_lds_bytes(), h->stream, N, mu, h->Y,
                         h->w, h->mean, h->prevMean, h->meanUpdate, h->sc);
    if (h->G)  // every rank holds the whole population's gradients (the caller's all-gather)
      hipLaunchKernelGGL(k_mean_gradient, dim3((N + 63) / 64), dim3(64), 0, h->stream, N, mu, h->cfg.gradient_step_size,
                         h->G, h->idx, h->w, h->mean, h->prevMean, h->meanUpdate, h->sc);
    KG_HIP(hipGetLastError());
    if (cmaes_paths(h, generation)) return 1;
  }
  {
    // this rank's contiguous share of the covariance tiles, each element's
    // chain in the reference's order
    Stage st(h, "covariance");
    const size_t npk = (size_t)N * (N + 1) / 2;
    hipLaunchKernelGGL(k_fill_min_i64, dim3((unsigned)std::min<size_t>((npk + 255) / 256, 1024)), dim3(256), 0,
                       h->stream, npk, (long long *)h->covPack);
    const bool lane = lane_chains(N);
    const int nt = lane ? al_tiles(N) : ar_tiles(N);
    const int t0 = (int)((long long)nt * h->shardRank / h->shards), t1 = (int)((long long)nt * (h->shardRank + 1) / h->shards);
    if (t1 > t0 && lane)
      hipLaunchKernelGGL(k_adaptC_lane, dim3(t1 - t0), dim3(256), 0, h->stream, N, mu, h->cfg.diagonal_covariance,
                         h->Yc, h->Tt, h->pc, h->C, h->sc, t0, h->covPack);
    else if (t1 > t0)
      hipLaunchKernelGGL(k_adaptC_row, dim3(t1 - t0), dim3(AR_NT), 0, h->stream, N, mu, h->cfg.diagonal_covariance, h->Yc,
                         h->Tt, h->pc, h->C, h->sc, t0, h->covPack);
    KG_HIP(hipGetLastError());
  }
  h->rowBlock = -1;
  return 0;
}

int kg_cmaes_update_finalize(kg_cmaes_t h, size_t generation) {
  const int N = h->N;
  if (h->covPack) {
    Stage st(h, "covariance");
    hipLaunchKernelGGL(k_shard_cov_unpack, dim3(N), dim3(256), 0, h->stream, N, (const double *)h->covPack, h->C);
    KG_HIP(hipGetLastError());
    if (early_publish(h)) return 1;
    return cmaes_sigma(h, generation);
  }
  {
    Stage st(h, "mean_paths");
    hipLaunchKernelGGL(k_shard_finalize, dim3((N + 255) / 256), dim3(256), 0, h->stream, N, h->part, h->mean,
                       h->prevMean, h->meanUpdate, h->currBestVars, h->bestEverVars, h->sc);
    if (h->G)
      hipLaunchKernelGGL(k_mean_gradient, dim3((N + 63) / 64), dim3(64), 0, h->stream, N, h->mu,
                         h->cfg.gradient_step_size, h->G, h->idx, h->w, h->mean, h->prevMean, h->meanUpdate, h->sc);
    KG_HIP(hipGetLastError());
    if (cmaes_paths(h, generation)) return 1;
  }
  {
    Stage st(h, "covariance");
    const int nt = (N + 15) / 16, ntiles = nt * (nt + 1) / 2;
    hipLaunchKernelGGL(k_adaptC_combine, dim3(ntiles), dim3(256), 0, h->stream, N, 1, ntiles,
                       h->cfg.diagonal_covariance, h->part + 2 * (size_t)N, h->pc, h->C, h->sc, 1);
    KG_HIP(hipGetLastError());
  }
  return cmaes_sigma(h, generation);  // (k_sigma also publishes the termination record, as after kg_cmaes_update)
}

int kg_cmaes_generation(kg_cmaes_t h, size_t generation, int objective) {
  KG_CHECK(h->shards == 1, "a population-sharded generation needs the caller's collectives between its stages");
  if (generation == 1 && kg_cmaes_initialize(h)) return 1;
  if (kg_cmaes_sample(h)) return 1;
  if (kg_cmaes_eval_builtin(h, objective)) return 1;
  return kg_cmaes_update(h, generation);
}

int kg_cmaes_wait_termination_fields(kg_cmaes_t h, double *out) {
  // the record of the last kg_cmaes_update; spin on host-coherent memory
  // (microseconds) instead of synchronising the stream, which may already
  // hold the next generation's first half (kg_cmaes_begin_sample)
  const unsigned long long want = h->updates;
  KG_CHECK(want > 0, "kg_cmaes_wait_termination_fields before any kg_cmaes_update");
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(&h->summary->seq, __ATOMIC_ACQUIRE) < want) {
    __builtin_ia32_pause();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
      KG_HIP(hipStreamSynchronize(h->stream));  // surfaces a device fault, if any
      if (check_errors(h)) return 1;
      KG_CHECK(false, "termination summary never arrived");
    }
  }
  if (h->summary->errors) {
    KG_HIP(hipStreamSynchronize(h->stream));
    return check_errors(h);
  }
  for (int i = 0; i < KG_TERMINATION_FIELDS; i++) out[i] = h->summary->f[i];
  return 0;
}

int kg_cmaes_synchronize(kg_cmaes_t h) {
  KG_HIP(hipStreamSynchronize(h->stream));
  if (h->eigTrace) {
    unsigned long long t[32];
    KG_HIP(hipMemcpy(t, h->eigTrace, sizeof(t), hipMemcpyDeviceToHost));
    int steps = 0, rots = 0;
    h->eig.last_counts(steps, rots);
    fprintf(stderr,
            "[korali_amd tridiag trace, cumulative s_memtime ticks] nrm2 %llu dsymv %llu xv %llu dsyr2 %llu; last QR: "
            "%d steps, %d rotations\n[korali_amd apply trace] groups %llu time-units %llu steps %llu ticks %llu\n"
            "[korali_amd multi-workgroup tridiag, writer wg] dnrm2 %llu householder %llu dsymv-stage %llu dsymv-chain "
            "%llu x-gather %llu xv-stage %llu xv-chain %llu alpha %llu pivot-poll %llu update %llu\n"
            "[korali_amd streamed apply] batches %llu steps-before-chase-done %llu ticks-to-first-batch %llu\n"
            "[korali_amd one-workgroup tridiag] householder %llu barrier %llu dsymv %llu xv %llu x-update %llu "
            "pivot-update %llu chain-w0 %llu chain-w3 %llu (A: dnrm2 %llu [of which pre-chain %llu] scalars %llu)\n",
            t[0], t[1], t[2], t[3], steps, rots, t[4], t[5], t[6], t[7], t[16], t[17], t[18], t[19], t[20], t[21],
            t[22], t[23], t[24], t[25], t[26], t[27], t[28], t[8], t[9], t[10], t[11], t[12], t[13], t[14], t[15], t[29], t[31], t[30]);
    fprintf(stderr,
            "[korali_amd sq tridiag, wave 0] staging %llu nrm2-chain %llu scalars+v %llu wait-A %llu dsymv %llu "
            "wait-E %llu xv+pivot %llu wait-X %llu\n",
            t[8], t[9], t[10], t[11], t[12], t[13], t[14], t[15]);
    fprintf(stderr,
            "[korali_amd mw2 tridiag, writer wg] staging %llu barrier %llu nrm2-chain %llu scalars %llu products %llu "
            "dsymv-chains %llu x-gather %llu xv %llu poll %llu update %llu\n",
            t[16], t[17], t[18], t[19], t[20], t[21], t[22], t[23], t[24], t[25]);
    // the one-workgroup kernel's last launch, step by step: every phase's
    // ticks fitted as a + b n over the steps (n = N-1-i, the chain length)
    if (h->eig.tridiag_kind() == 4) {
      const int steps = h->N - 2;
      std::vector<unsigned long long> ps(8 * (size_t)steps);
      KG_HIP(hipMemcpy(ps.data(), h->eigTrace + 32, ps.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      static const char *nm[8] = {"staging", "nrm2-chain", "scalars+v", "wait-A", "dsymv", "wait-E", "xv+pivot", "wait-X"};
      std::string line = "[korali_amd sq tridiag per step, ticks = a + b n]";
      for (int k = 0; k < 8; k++) {
        double sx = 0, sy = 0, sxx = 0, sxy = 0;
        for (int i = 0; i < steps; i++) {
          const double x = h->N - 1 - i, y = (double)ps[8 * (size_t)i + k];
          sx += x, sy += y, sxx += x * x, sxy += x * y;
        }
        const double b = (steps * sxy - sx * sy) / (steps * sxx - sx * sx), a = (sy - b * sx) / steps;
        char buf[96];
        snprintf(buf, sizeof(buf), " %s a=%.0f b=%.1f", nm[k], a, b);
        line += buf;
      }
      fprintf(stderr, "%s\n", line.c_str());
      for (int i = 0; i < steps; i += 25) {
        fprintf(stderr, "[korali_amd sq tridiag step %d, n=%d]", i, h->N - 1 - i);
        for (int k = 0; k < 8; k++) fprintf(stderr, " %llu", ps[8 * (size_t)i + k]);
        fprintf(stderr, "\n");
      }
    }
  }
  return check_errors(h);
}

// CCMA-ES state kept on the host (CMAES.config internal settings)
struct HostField {
  double *p;
  size_t n;
  bool writable;
};
static bool host_field(kg_cmaes_t h, const std::string &k, HostField &f, double &tmp) {
  if (!h->nc) return false;
  const size_t S = h->lamMax;
  if (k == "Constraint Evaluations") f = {h->cEval.data(), h->nc * S, true};
  else if (k == "Viability Indicator") f = {h->cInd.data(), h->nc * S, true};
  else if (k == "Sample Constraint Violation Counts") f = {h->cCnt.data(), S, true};
  else if (k == "Viability Boundaries") f = {h->vBounds.data(), h->nc, true};
  else if (k == "Best Constraint Evaluations") f = {h->bestCEval.data(), h->nc, true};
  else if (k == "Constraint Evaluation Count") f = {&h->cEvalCount, 1, true};
  else if (k == "Covariance Matrix Adaptation Count") f = {&h->adaptCount, 1, true};
  else if (k == "Max Constraint Violation Count") f = {&h->maxViolCount, 1, true};
  else if (k == "Is Viability Regime") {
    tmp = h->viability ? 1.0 : 0.0;
    f = {&tmp, 1, true};
  } else if (k == "Current Population Size") {
    tmp = h->lam;
    f = {&tmp, 1, false};
  } else if (k == "Current Mu Value") {
    tmp = h->mu;
    f = {&tmp, 1, false};
  } else if (k == "Covariance Matrix Adaption Factor") {
    tmp = h->cfg.covariance_matrix_adaption_strength / (h->N + 2.);
    f = {&tmp, 1, false};
  } else if (k == "Normal Vector Learning Rate") {
    tmp = 1.0 / (2.0 + h->N);
    f = {&tmp, 1, false};
  } else
    return false;
  return true;
}

int kg_cmaes_field_size(kg_cmaes_t h, const char *name, size_t *n) {
  HostField hf;
  double tmp = 0;
  if (host_field(h, name, hf, tmp)) {
    *n = hf.n;
    return 0;
  }
  FieldRef r;
  KG_CHECK(field_ref(h, name, r), std::string("unknown CMA-ES field: ") + name);
  *n = r.n;
  return 0;
}

int kg_cmaes_get_field(kg_cmaes_t h, const char *name, double *out, size_t n) {
  HostField hf;
  double tmp = 0;
  if (host_field(h, name, hf, tmp)) {
    KG_CHECK(n == hf.n, std::string("size mismatch for field ") + name);
    memcpy(out, hf.p, n * sizeof(double));
    return 0;
  }
  FieldRef r;
  KG_CHECK(field_ref(h, name, r), std::string("unknown CMA-ES field: ") + name);
  KG_CHECK(n == r.n || (n < r.n && std::string(name) == "Shard Rows"),  // (exchange blocks: a prefix)
           std::string("size mismatch for field ") + name);
  KG_HIP(hipMemcpyAsync(out, r.dev, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_cmaes_set_field(kg_cmaes_t h, const char *name, const double *in, size_t n) {
  HostField hf;
  double tmp = 0;
  if (host_field(h, name, hf, tmp)) {
    KG_CHECK(n == hf.n, std::string("size mismatch for field ") + name);
    KG_CHECK(hf.writable, std::string("read-only field ") + name);
    if (std::string(name) == "Is Viability Regime") {  // (resume) the regime's sizes follow
      h->viability = in[0] != 0.0;
      const int lv = (int)h->cfg.viability_population_size;
      const int mv = (int)(h->cfg.viability_mu_value ? h->cfg.viability_mu_value : h->cfg.viability_population_size / 2);
      return h->viability ? set_current(h, lv, mv) : set_current(h, h->lamCfg, h->muCfg);
    }
    memcpy(hf.p, in, n * sizeof(double));
    return 0;
  }
  FieldRef r;
  KG_CHECK(field_ref(h, name, r), std::string("unknown CMA-ES field: ") + name);
  KG_CHECK(n == r.n || (n < r.n && std::string(name) == "Shard Rows"), std::string("size mismatch for field ") + name);
  KG_HIP(hipMemcpyAsync(r.dev, in, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  h->stateDirty = true;
  h->eig.invalidate();  // a decomposition issued ahead (kg_cmaes_update / _begin_sample) saw the old state
  return 0;
}

int kg_cmaes_get_fields(kg_cmaes_t h, const char *const *names, size_t count, double *out) {
  // one copy of the scalar block serves every scalar name
  CmaesScalars hs;
  KG_HIP(hipMemcpyAsync(&hs, h->sc, sizeof(hs), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  for (size_t i = 0; i < count; i++) {
    HostField hf;
    double tmp = 0;
    if (host_field(h, names[i], hf, tmp)) {
      KG_CHECK(hf.n == 1, std::string("kg_cmaes_get_fields: not a scalar field: ") + names[i]);
      out[i] = *hf.p;
      continue;
    }
    FieldRef r;
    KG_CHECK(field_ref(h, names[i], r), std::string("unknown CMA-ES field: ") + names[i]);
    const char *base = (const char *)h->sc;
    const char *p = (const char *)r.dev;
    if (r.n == 1 && p >= base && p < base + sizeof(CmaesScalars)) {
      memcpy(&out[i], (const char *)&hs + (p - base), sizeof(double));
    } else {
      KG_CHECK(r.n == 1, std::string("kg_cmaes_get_fields: not a scalar field: ") + names[i]);
      KG_HIP(hipMemcpy(&out[i], r.dev, sizeof(double), hipMemcpyDeviceToHost));
    }
  }
  return 0;
}

int kg_cmaes_get_sorting_index(kg_cmaes_t h, uint64_t *out) {
  std::vector<unsigned> t(h->lam);
  KG_HIP(hipMemcpyAsync(t.data(), h->idx, h->lam * sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  for (int i = 0; i < h->lam; i++) out[i] = t[i];
  return 0;
}

int kg_cmaes_get_rng(kg_cmaes_t h, int which, void *state5000) {
  KG_CHECK(which == 0 || which == 1, "rng index must be 0 (Normal) or 1 (Uniform)");
  return (which == 0 ? h->normal : h->uniform).export_gsl(state5000, h->stream);
}

int kg_cmaes_set_rng(kg_cmaes_t h, int which, const void *state5000) {
  KG_CHECK(which == 0 || which == 1, "rng index must be 0 (Normal) or 1 (Uniform)");
  return (which == 0 ? h->normal : h->uniform).import_gsl(state5000, h->stream);
}

int kg_cmaes_device_ptr(kg_cmaes_t h, const char *name, void **ptr) {
  FieldRef r;
  KG_CHECK(field_ref(h, name, r), std::string("unknown CMA-ES field: ") + name);
  *ptr = r.dev;
  return 0;
}

int kg_cmaes_stream(kg_cmaes_t h, void **stream) {
  *stream = (void *)h->stream;
  return 0;
}

int kg_cmaes_set_constraints(kg_cmaes_t h, kg_constraint_fn fn, void *ctx) {
  KG_CHECK(h->nc > 0, "kg_cmaes_set_constraints: the handle was created with constraint_count = 0");
  h->cfn = fn;
  h->cctx = ctx;
  return 0;
}

int kg_cmaes_prepare_constrained(kg_cmaes_t h, size_t generation) {
  if (h->nc && ccm_check_mean(h)) return 1;
  if (kg_cmaes_sample(h)) return 1;
  if (!h->nc) return 0;
  if (ccm_update_constraints(h, generation)) return 1;
  return ccm_handle_constraints(h);
}

int kg_cmaes_population_size(kg_cmaes_t h, size_t *lambda, size_t *mu) {
  if (lambda) *lambda = (size_t)h->lam;
  if (mu) *mu = (size_t)h->mu;
  return 0;
}

int kg_cmaes_profile(kg_cmaes_t h, int enable) {
  h->profile = enable != 0;
  return 0;
}

int kg_cmaes_profile_mark(kg_cmaes_t h, const char *stage, int phase) {
  if (!h || !stage || (phase != 0 && phase != 1)) return 1;
  hipEvent_t e;
  KG_HIP(hipEventCreate(&e));
  KG_HIP(hipEventRecord(e, h->stream));
  if (phase == 0) {
    auto it = h->openMarks.find(stage);
    if (it != h->openMarks.end()) (void)hipEventDestroy(it->second);
    h->openMarks[stage] = e;
    return 0;
  }
  auto it = h->openMarks.find(stage);
  if (it == h->openMarks.end()) {
    (void)hipEventDestroy(e);
    return 1;
  }
  h->pending.emplace_back(stage, it->second, e);
  h->openMarks.erase(it);
  return 0;
}

int kg_cmaes_profile_read(kg_cmaes_t h, const char *stage, double *ms_total, size_t *count) {
  KG_HIP(hipStreamSynchronize(h->stream));
  for (auto &t : h->pending) {
    float ms = 0.f;
    KG_HIP(hipEventElapsedTime(&ms, std::get<1>(t), std::get<2>(t)));
    auto &p = h->prof[std::get<0>(t)];
    p.first += ms;
    p.second += 1;
    (void)hipEventDestroy(std::get<1>(t));
    (void)hipEventDestroy(std::get<2>(t));
  }
  h->pending.clear();
  auto it = h->prof.find(stage);
  if (it == h->prof.end()) {
    *ms_total = 0;
    *count = 0;
  } else {
    *ms_total = it->second.first;
    *count = it->second.second;
    h->prof.erase(it);
  }
  return 0;
}

}  // extern "C"
