// kg_tmcmc.hip — TMCMC generation (TMCMC::runGeneration, TMCMC.cpp.base:107-157)
// on the device, Version "TMCMC" with any Max Chain Length / Burn In / Per
// Generation Burn In.
//
// Work split (same rationale as the eigensolver):
//   device — Cholesky of the proposal covariance, P x N polar normals from the
//            Multivariate generator, the dtrmv + leader shift of every chain,
//            uniform-prior log-densities + builtin Gaussian log-likelihood,
//            Metropolis accept (one Uniform draw per chain), all P-sized
//            exponentials of the annealing search and of the importance
//            weights, the weighted mean / covariance (P-long ordered sums,
//            one lane per output element) and the leader expansion.
//   host   — the strictly serial scalar recurrences the reference evaluates
//            in x87 80-bit arithmetic or with data-dependent RNG consumption:
//            the nmsimplex search over the squared CoV difference (gsl_stats
//            mean / sd_m keep `long double` running sums), the P-long
//            accumulate of the weights, and gsl_ran_multinomial's chain of
//            conditional binomials on the Multinomial generator.  A host core
//            runs those chains ~8x faster than one GPU lane.
// Results are identical to the reference's (tests/test_gpu_tmcmc.py).
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <condition_variable>
#include <string>
#include <thread>
#include <utility>
#include <tuple>
#include <vector>

#include "../../include/korali_amd.h"
#include "kg_common.hpp"
#include "kg_mtmcmc.hpp"
#include "kg_rng.hpp"

namespace kg {
namespace {

constexpr int TM_MAX_N = 120;  // LDS-resident Cholesky (N x (N+1) doubles)
constexpr int CV_MAX_PTS = 8;  // speculative points per annealing-search batch

// values produced on the device, read back at the processGeneration sync
struct TmDev {
  double maxLoglikelihood;  // processGeneration :371-377 (first element wins, NaN only if first)
  double llmaxCv;           // gsl_stats_max of the database log-likelihoods (NaN if any)
  double lwmax;             // max log-weight :286-293 (NaN if any)
  unsigned int accepted;    // processCandidate :241
  unsigned int errors;
};

struct CvPoints {
  double x[CV_MAX_PTS];
};

// ------------------------------------------------------------ Cholesky
// gsl_linalg_cholesky_decomp (GSL 2.6 linalg/cholesky.c, Level-2 form, with
// gslcblas dgemv order: temp = sum_i x[i] A[r][i] from 0, y += alpha*temp),
// called in place on the covariance (TMCMC.cpp.base:205-213).  With
// gsl_set_error_handler_off (engine.cpp:30) a non-positive pivot returns
// early and leaves the partially factored matrix, which the reference then
// uses as it is: mirrored here.
__global__ void __launch_bounds__(256) k_tm_cholesky(int N, const double *__restrict__ cov, double *__restrict__ L,
                                                     TmDev *dev) {
  extern __shared__ double A[];  // N x (N+1)
  __shared__ double f;
  __shared__ int failed;
  const int S = N + 1;
  for (int e = threadIdx.x; e < N * N; e += blockDim.x) A[(e / N) * S + e % N] = cov[e];
  if (threadIdx.x == 0) failed = 0;
  __syncthreads();
  for (int j = 0; j < N; j++) {
    if (j > 0) {
      for (int r = j + threadIdx.x; r < N; r += blockDim.x) {
        double temp = 0.0;
        for (int i = 0; i < j; i++) temp += A[j * S + i] * A[r * S + i];
        A[r * S + j] += -1.0 * temp;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      double ajj = A[j * S + j];
      if (ajj <= 0.0) {
        failed = 1;
      } else {
        ajj = sqrt(ajj);
        f = 1.0 / ajj;
      }
    }
    __syncthreads();
    if (failed) break;
    for (int r = j + threadIdx.x; r < N; r += blockDim.x) A[r * S + j] *= f;
    __syncthreads();
  }
  if (!failed) {  // gsl_matrix_transpose_tricpy: upper = lower^T
    for (int e = threadIdx.x; e < N * N; e += blockDim.x) {
      const int i = e / N, j = e % N;
      if (i < j) A[i * S + j] = A[j * S + i];
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < N * N; e += blockDim.x) L[e] = A[(e / N) * S + e % N];
  (void)dev;
}

// --------------------------------------------------------- candidates
// Step schedule of chain c in one generation (host-computed prefix sums over
// the chains in chain order, the Sequential conduit's completion order):
// S steps (Chain Lengths[c] + Current Burn In), its first Uniform draw u0,
// its first row z0 of the extra Multivariate normals (one row per candidate
// after the first), its first database entry db0.
struct ChainSched {
  unsigned S, u0, z0, db0;
};

// generateCandidate :560-566 -> gsl_ran_multivariate_gaussian (normals from
// the polar pass, dtrmv Lower/NoTrans/NonUnit in gslcblas order, + zero mean)
// then + leader.  One thread per (chain, i): x_i = (sum_{j<i} z_j L_ij) + z_i L_ii.
// kRound: the candidate after step s of chain c (only chains with S > s;
// normal row z0 + s - 1), which then becomes pending; otherwise row c for
// every chain (prepareGeneration :222-225).
// Chains [c_lo, c_hi) (a shard's own chains); Z holds the rows from c_lo
// (prepare) or from extra-normal row zbase (kRound).
template <bool kRound>
__global__ void __launch_bounds__(256) k_tm_draw(int N, int c_lo, int P, const double *__restrict__ Z,
                                                 const double *__restrict__ Lg, const double *__restrict__ leaders,
                                                 double *__restrict__ cand, const ChainSched *__restrict__ sch,
                                                 int s, unsigned zbase, unsigned char *__restrict__ pend) {
  extern __shared__ double sm[];
  const int S = N + 1;
  double *Ls = sm;            // N x (N+1)
  double *zs = sm + N * S;    // CB x N
  const int CB = max(1, 256 / N);
  const int c0 = c_lo + blockIdx.x * CB;
  for (int e = threadIdx.x; e < N * N; e += blockDim.x) Ls[(e / N) * S + e % N] = Lg[e];
  for (int e = threadIdx.x; e < CB * N; e += blockDim.x) {
    const int c = c0 + e / N;
    double z = 0.0;
    if (c < P) {
      if (!kRound)
        z = Z[(size_t)(c - c_lo) * N + e % N];
      else if ((int)sch[c].S > s)
        z = Z[((size_t)sch[c].z0 + s - 1 - zbase) * N + e % N];
    }
    zs[e] = z;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < CB * N; e += blockDim.x) {
    const int cl = e / N, i = e % N, c = c0 + cl;
    if (c >= P) continue;
    if (kRound) {
      const bool more = (int)sch[c].S > s;
      if (i == 0) pend[c] = more ? 1 : 0;
      if (!more) continue;
    }
    const double *z = zs + cl * N;
    const double *Li = Ls + i * S;
    double temp = 0.0;
    for (int j = 0; j < i; j++) temp += z[j] * Li[j];
    double x = temp + z[i] * Li[i];
    x = x + 0.0;  // gsl_vector_add(result, mu), mu = 0
    x += leaders[(size_t)c * N + i];
    cand[(size_t)c * N + i] = x;
  }
}

// generation 1: candidate d of chain c from its prior's generator
// (TMCMC.cpp.base:216-221, Uniform::getRandomNumber = gsl_ran_flat,
// univariate/uniform/uniform.cpp.base:30-36): a*(1-u) + b*u.  Variables with
// a Normal prior (vkind 1) take the host's sequential draw nrm (tm_normal_priors).
__global__ void k_tm_prior(int N, int P, const double *__restrict__ U, const unsigned long long *__restrict__ uoff,
                           const int *__restrict__ ustride, const double *__restrict__ pmin,
                           const double *__restrict__ pmax, const int *__restrict__ vkind,
                           const double *__restrict__ nrm, double *__restrict__ cand) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const int c = (int)(e / N), d = (int)(e % N);
  if (vkind[d]) {
    cand[e] = nrm[e];
    return;
  }
  const double u = U[uoff[d] + (size_t)c * ustride[d]];
  cand[e] = pmin[d] * (1 - u) + pmax[d] * u;
}

// Bayesian::evaluate (bayesian.cpp.base:24-84): logPrior = sum of the
// variables' prior log-densities in variable order — Uniform: -log(b-a)
// inside, -inf outside (uniform.cpp.base:38-44); Normal: logNormalization -
// 0.5 d d, d = (x - mean) / sd (normal.cpp.base:17-21; pmin / pmax hold mean
// and sd);
// -inf prior -> loglik -inf without evaluating the model; otherwise the
// builtin Gaussian loglik -0.5*sum x^2 (samplers/mean/model/model.py:32-37).
__global__ void k_tm_evaluate(int N, int P, int lik, const double *__restrict__ cand,
                              const double *__restrict__ negLogWidth, const double *__restrict__ pmin,
                              const double *__restrict__ pmax, const int *__restrict__ vkind,
                              double *__restrict__ candLL, double *__restrict__ candLP,
                              const unsigned char *__restrict__ pend) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P || !pend[c]) return;
  const double *x = cand + (size_t)c * N;
  double lp = 0.0;
  for (int d = 0; d < N; d++) {
    const double a = pmin[d], b = pmax[d], c = negLogWidth[d];
    switch (vkind[d]) {
      case KG_PRIOR_NORMAL: {
        const double z = (x[d] - a) / b;
        lp += c - 0.5 * z * z;
        break;
      }
      case KG_PRIOR_EXPONENTIAL: {  // exponential.cpp.base: -log(mean) - (x - location) / mean
        const double y = x[d] - a;
        lp += y < 0 ? -INFINITY : c - y / b;
        break;
      }
      case KG_PRIOR_LAPLACE:  // laplace.cpp.base: aux - |x - mean| / width
        lp += c - fabs(x[d] - a) / b;
        break;
      case KG_PRIOR_CAUCHY: {  // cauchy.cpp.base: aux - log(1 + (x - loc)^2 / scale^2)
        const double y = x[d] - a;
        lp += c - log_cr(1. + y * y / (b * b));
        break;
      }
      case KG_PRIOR_LOGNORMAL: {  // logNormal.cpp.base: aux - log x - 0.5 d^2, d = (log x - mu) / sigma
        if (x[d] <= 0) {
          lp += -INFINITY;
        } else {
          const double lx = log_cr(x[d]), z = (lx - a) / b;
          lp += c - lx - 0.5 * z * z;
        }
        break;
      }
      default:
        lp += (x[d] >= a && x[d] <= b) ? c : -INFINITY;
    }
  }
  candLP[c] = lp;
  double ll = -INFINITY;
  if (!(isinf(lp) && lp < 0)) {
    if (lik < 0) return;  // prior only: the host evaluates the likelihood model
    double ss = 0.0;
    for (int d = 0; d < N; d++) ss += x[d] * x[d];
    ll = -0.5 * ss;
  }
  candLL[c] = ll;
}

// host-evaluated log-prior / log-likelihood of the pending chains
__global__ void k_tm_set_pending(int P, const unsigned char *__restrict__ pend, const double *__restrict__ lp,
                                 const double *__restrict__ ll, double *__restrict__ candLP,
                                 double *__restrict__ candLL) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P || !pend[c]) return;
  candLP[c] = lp[c];
  candLL[c] = ll[c];
}

// started chains c in [lo, hi) (this shard's) are pending their first
// evaluation (runGeneration :114-130)
__global__ void k_tm_pend_init(int P, int lo, int hi, unsigned char *__restrict__ pend) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < P) pend[c] = (c >= lo && c < hi) ? 1 : 0;
}

// each variable's log-density constant (the distributions' updateDistribution
// / getLogDensity): Uniform -log(b - a); Normal and LogNormal -0.5 log(2 pi)
// - log(sd); Exponential -log(mean); Laplace -log(2 width); Cauchy
// -log(scale pi)
__global__ void k_tm_neglogwidth(int N, const double *__restrict__ pmin, const double *__restrict__ pmax,
                                 const int *__restrict__ vkind, double *__restrict__ out) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= N) return;
  const double pi = 3.14159265358979323846, b = pmax[d];
  switch (vkind[d]) {
    case KG_PRIOR_NORMAL:
    case KG_PRIOR_LOGNORMAL: out[d] = -0.5 * log_cr(2 * pi) - log_cr(b); break;
    case KG_PRIOR_EXPONENTIAL: out[d] = -log_cr(b); break;
    case KG_PRIOR_LAPLACE: out[d] = -log_cr(2. * b); break;
    case KG_PRIOR_CAUCHY: out[d] = -log_cr(b * pi); break;
    default: out[d] = -log_cr(b - pmin[d]);
  }
}

// processCandidate + calculateAcceptanceProbability + updateDatabase
// (:229-252, :611-633): P = exp((ll_c - ll_l) rho + (lp_c - lp_l)) if both
// candidate values are finite, else 0; one Uniform draw per chain (always);
// accept if P > U or generation 1.  Chain c's database entry is its leader.
// mTMCMC (:634-677, `mode` non-null): chains with mode[c] = 1 (leader and
// candidate without errors) add the proposal log-density ratio extra[c] =
// log q(leader | candidate) - log q(candidate | leader), formed on the host.
__global__ void k_tm_accept(int c_lo, int P, int gen1, double rho, const double *__restrict__ U,
                            const double *__restrict__ candLL, const double *__restrict__ candLP,
                            double *__restrict__ leadLL, double *__restrict__ leadLP, double *__restrict__ dbLL,
                            double *__restrict__ dbLP, unsigned char *__restrict__ acc, TmDev *dev,
                            const double *__restrict__ extra, const unsigned char *__restrict__ mode) {
  const int c = c_lo + blockIdx.x * blockDim.x + threadIdx.x;
  bool a = false;
  if (c < P) {
    double p = 0.0;
    const double lpc = candLP[c], llc = candLL[c];
    if (isfinite(lpc) && isfinite(llc)) {
      if (mode && mode[c])
        p = exp_cr((llc - leadLL[c]) * rho + extra[c] + (lpc - leadLP[c]));
      else
        p = exp_cr((llc - leadLL[c]) * rho + (lpc - leadLP[c]));
    }
    a = (p > U[c]) || gen1;
    acc[c] = a ? 1 : 0;
    if (a) {
      leadLL[c] = llc;
      leadLP[c] = lpc;
    }
    dbLL[c] = leadLL[c];
    dbLP[c] = leadLP[c];
  }
  const unsigned long long m = __ballot(a);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&dev->accepted, (unsigned int)__popcll(m));
}

__global__ void k_tm_copy_rows(int N, int c_lo, int P, const unsigned char *__restrict__ acc,
                               const double *__restrict__ cand, double *__restrict__ leaders, double *__restrict__ db) {
  const size_t e = (size_t)c_lo * N + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const int c = (int)(e / N);
  double v = leaders[e];
  if (acc[c]) {
    v = cand[e];
    leaders[e] = v;
  }
  db[e] = v;
}

// step s (1-based) of every chain with S >= s (runGeneration :132-143 +
// processCandidate :229-252): one Uniform (u0 + s - 1), accept if P > U or
// generation 1, counted and entered into the database only past the burn-in
// B (entry db0 + s - B - 1).
__global__ void k_tm_round_accept(int c_lo, int nc, int s, int B, int gen1, double rho,
                                  const ChainSched *__restrict__ sch, const double *__restrict__ U,
                                  const double *__restrict__ candLL, const double *__restrict__ candLP,
                                  double *__restrict__ leadLL, double *__restrict__ leadLP, double *__restrict__ dbLL,
                                  double *__restrict__ dbLP, unsigned char *__restrict__ acc, TmDev *dev) {
  const int c = c_lo + blockIdx.x * blockDim.x + threadIdx.x;
  bool counted = false;
  if (c < nc) {
    const ChainSched q = sch[c];
    if ((int)q.S >= s) {
      double p = 0.0;
      const double lpc = candLP[c], llc = candLL[c];
      if (isfinite(lpc) && isfinite(llc)) p = exp_cr((llc - leadLL[c]) * rho + (lpc - leadLP[c]));
      const bool a = (p > U[(size_t)q.u0 + s - 1]) || gen1;
      acc[c] = a ? 1 : 0;
      if (a) {
        leadLL[c] = llc;
        leadLP[c] = lpc;
      }
      if (s > B) {
        const size_t k = (size_t)q.db0 + s - B - 1;
        dbLL[k] = leadLL[c];
        dbLP[k] = leadLP[c];
        counted = a;
      }
    }
  }
  const unsigned long long m = __ballot(counted);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&dev->accepted, (unsigned int)__popcll(m));
}

__global__ void k_tm_round_rows(int N, int c_lo, int nc, int s, int B, const ChainSched *__restrict__ sch,
                                const unsigned char *__restrict__ acc, const double *__restrict__ cand,
                                double *__restrict__ leaders, double *__restrict__ db) {
  const size_t e = (size_t)c_lo * N + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)nc * N) return;
  const int c = (int)(e / N);
  const ChainSched q = sch[c];
  if ((int)q.S < s) return;
  double v = leaders[e];
  if (acc[c]) {
    v = cand[e];
    leaders[e] = v;
  }
  if (s > B) db[((size_t)q.db0 + s - B - 1) * N + e % N] = v;
}

// first-index maximum of a_i = v_i * scale (scale applied when use_scale),
// with both of the reference's NaN conventions:
//   out_any  : NaN if any a_i is NaN (gsl_stats_max / the :286-293 loop)
//   out_first: NaN only if a_0 is NaN, NaNs elsewhere skipped (:371-377)
struct MaxAcc {
  double v;
  int idx;  // -1: empty
};
__device__ inline MaxAcc max_comb(MaxAcc a, MaxAcc b) {
  if (a.idx < 0) return b;
  if (b.idx < 0) return a;
  if (b.v > a.v) return b;
  if (a.v > b.v) return a;
  return a.idx <= b.idx ? a : b;
}
__global__ void __launch_bounds__(1024) k_tm_max(int P, const double *__restrict__ v, double scale, int use_scale,
                                                 double *out_any, double *out_first) {
  __shared__ MaxAcc wacc[16];
  __shared__ int wnan[16];
  MaxAcc m{0.0, -1};
  int anyNan = 0;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const double a = use_scale ? v[i] * scale : v[i];
    if (a != a) {
      anyNan = 1;
      continue;
    }
    m = max_comb(m, MaxAcc{a, i});
  }
  for (int off = 32; off > 0; off >>= 1) {
    MaxAcc o{__shfl_down(m.v, off, 64), __shfl_down(m.idx, off, 64)};
    m = max_comb(m, o);
    anyNan |= __shfl_down(anyNan, off, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    wacc[wid] = m;
    wnan[wid] = anyNan;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MaxAcc t{0.0, -1};
    int n = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
      t = max_comb(t, wacc[w]);
      n |= wnan[w];
    }
    const double a0 = use_scale ? v[0] * scale : v[0];
    if (out_any) *out_any = n ? NAN : t.v;
    if (out_first) *out_first = (a0 != a0) ? NAN : t.v;
  }
}

// calculateSquaredCVDifference :683-703 for a batch of search points.
// Grid (CV_BLOCKS, npts): every block takes a slice of the P exponentials
//   E_k[i] = exp((ll_i - ll_max) (x_k - rho))           (kept for the exact tail)
// and accumulates d = E - 1 (exact for E in [1/2, 1]: the shift keeps the
// variance free of cancellation when the weights are nearly uniform) as
// double-double sums of d and d^2; the last block of point k to finish
// forms cv_k = sd(E_k) / mean(E_k).  cv is invariant to the normalisation
// w = E / sum(E), so cv_k is the reference's coefficient of variation up to
// the reference's own rounding; `ratio` = max(E)/mean(E) feeds the host's
// bound on that rounding.
struct CvOut {
  double cv2, cv, ratio;
  int flag;  // non-finite / degenerate: the host evaluates exactly
  int pad;
};
struct CvPart {
  double s_hi, s_lo, q_hi, q_lo, mx;
  int bad, pad;
};
constexpr int CV_BLOCKS = 32;
constexpr int CV_TPB = 256;
__device__ inline dd dd_shfl_down(dd a, int off) { return dd{__shfl_down(a.hi, off, 64), __shfl_down(a.lo, off, 64)}; }
__global__ void __launch_bounds__(CV_TPB) k_tm_cv_part(int P, const double *__restrict__ ll,
                                                       const TmDev *__restrict__ dev, double rho, CvPoints pts,
                                                       CvPart *__restrict__ part) {
  __shared__ dd sh_s[CV_TPB / 64], sh_q[CV_TPB / 64];
  __shared__ double sh_m[CV_TPB / 64];
  __shared__ int sh_b[CV_TPB / 64];
  const int k = blockIdx.y, b = blockIdx.x;
  const double x = pts.x[k], llmax = dev->llmaxCv;
  dd s{0.0, 0.0}, q{0.0, 0.0};
  double mx = 0.0;
  int bad = 0;
  for (int i = b * CV_TPB + threadIdx.x; i < P; i += CV_BLOCKS * CV_TPB) {
    const double e = exp_cr((ll[i] - llmax) * (x - rho));
    if (!isfinite(e)) bad = 1;
    const double d = e - 1.0;
    s = dd_add(s, dd{d, 0.0});
    q = dd_add(q, dd_tp(d, d));
    mx = e > mx ? e : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    s = dd_add(s, dd_shfl_down(s, off));
    q = dd_add(q, dd_shfl_down(q, off));
    mx = fmax(mx, __shfl_down(mx, off, 64));
    bad |= __shfl_down(bad, off, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sh_s[wid] = s;
    sh_q[wid] = q;
    sh_m[wid] = mx;
    sh_b[wid] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < CV_TPB / 64; w++) {
      s = dd_add(s, sh_s[w]);
      q = dd_add(q, sh_q[w]);
      mx = fmax(mx, sh_m[w]);
      bad |= sh_b[w];
    }
    part[k * CV_BLOCKS + b] = CvPart{s.hi, s.lo, q.hi, q.lo, mx, bad, 0};
  }
}

// one wave per point: combine the partials, form cv, and publish it to
// host-coherent memory as 16-byte {value, sequence} records (each record
// one PCIe write: the host sees the value once it sees the sequence, no
// fence needed)
__global__ void __launch_bounds__(64) k_tm_cv_final(int P, double target, const CvPart *__restrict__ part,
                                                    double2 *__restrict__ rec, unsigned long long seq) {
  const int k = blockIdx.x, j = threadIdx.x;
  dd S{0.0, 0.0}, Q{0.0, 0.0};
  double M = 0.0;
  int B = 0;
  if (j < CV_BLOCKS) {
    const CvPart p = part[k * CV_BLOCKS + j];
    S = dd{p.s_hi, p.s_lo};
    Q = dd{p.q_hi, p.q_lo};
    M = p.mx;
    B = p.bad;
  }
  for (int off = 32; off > 0; off >>= 1) {
    S = dd_add(S, dd_shfl_down(S, off));
    Q = dd_add(Q, dd_shfl_down(Q, off));
    M = fmax(M, __shfl_down(M, off, 64));
    B |= __shfl_down(B, off, 64);
  }
  if (j != 0) return;
  const dd Pd{(double)P, 0.0};
  const dd dmean = dd_div(S, Pd);                      // mean(d)
  dd ss = dd_add(Q, dd_mul(dd{-S.hi, -S.lo}, dmean));  // sum (d - mean d)^2
  const double var = (ss.hi + ss.lo) / (double)(P - 1);
  const dd mean = dd_add(dmean, dd{1.0, 0.0});
  const double meand = mean.hi + mean.lo;
  const double cv = sqrt(var > 0.0 ? var : 0.0) / meand;
  double c = cv - target;
  c *= c;
  const double ratio = M / meand;
  const int flag = (B || !isfinite(c) || !(meand > 0.0) || !isfinite(ratio) || var < 0.0) ? 1 : 0;
  typedef double d2v __attribute__((ext_vector_type(2)));
  const double sq = __longlong_as_double((long long)seq);
  d2v *r = (d2v *)(rec + 4 * k);
  __builtin_nontemporal_store(d2v{c, sq}, r + 0);  // one 16-byte store each
  __builtin_nontemporal_store(d2v{cv, sq}, r + 1);
  __builtin_nontemporal_store(d2v{ratio, sq}, r + 2);
  __builtin_nontemporal_store(d2v{(double)flag, sq}, r + 3);
}

// the exponentials of one search point, for the host's exact tail
__global__ void k_tm_cv_exp(int P, const double *__restrict__ ll, const TmDev *__restrict__ dev, double rho, double x,
                            double *__restrict__ E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < P) E[i] = exp_cr((ll[i] - dev->llmaxCv) * (x - rho));
}

// minSearch :712-779 on the device: the whole one-dimensional nmsimplex
// loop (the host's min_search below, comparison for comparison) in one
// cooperative launch.  Workgroup 0 runs the simplex; NM_W worker
// workgroups hold P/NM_W log-likelihoods each in LDS and evaluate the
// points of a round (every possible next point of an iteration, as the
// host's batches) as double-double sums of d = E - 1 with the device exp
// (<= 1 ulp; its error joins the bound as 16 u max/mean).  A round is one
// agent-scope release/acquire broadcast of the points and one fan-in of
// per-worker partial records, which the controller adds in a fixed tree
// (deterministic).  Comparisons are decided on the same rigorous
// intervals as the host path, so each one equals the comparison of the
// reference's values.  Values the intervals cannot separate (or
// degenerate ones) need the reference's exact value, which only the host
// forms (x87 long double recurrences, cv2_tail): the search then stops
// with status 1 and names the points; the host evaluates them and
// relaunches with the values in `tab`, where every later evaluation of
// those points finds them, so the search replays identically up to that
// comparison and then decides it exactly, as the host path does.  On
// success the final simplex and the iteration count are left for the
// exact stored minimum (k_tm_nm_exp): one round trip per generation
// instead of one per iteration.
constexpr int NM_TAB = 8, NM_PTS = 8, NM_W = 64, NM_TPB = 256, NM_LDS = 4096;
struct NmTab {
  double x[NM_TAB], y[NM_TAB];
  int n;
};
struct NmOut {
  double X[2], y[2], need[2];
  long long iters;
  int status, lo, nneed, loExact;  // status 0 done, 1 exact values needed, 2 no progress (the host searches)
  int loBad;                        // Ylo's interval is void (degenerate value): only its exact value decides
  double loEps;                     // |Ylo - exact| <= loEps otherwise
  unsigned evals, rounds;
  // phase times (s_memrealtime, 100 MHz ticks): controller publish+wait,
  // combine, simplex logic; worker 1 wait, evaluate, reduce+publish
  unsigned long long tc[3], tw[3];
};
struct NmPart {
  double s_hi, s_lo, q_hi, q_lo, mx, flags;  // flags: bit 0 non-finite, bit 1 some argument != 0
};
struct NmSync {
  double x[NM_PTS];
  unsigned long long n, quit;
  unsigned long long seq;         // round published by the controller
  unsigned long long done[NM_W];  // round each worker has published
  NmPart part[NM_W][NM_PTS];
  NmPart part2[2][NM_W][NM_PTS];  // k_tm_nm_sym: by round parity
};
struct NmVal {
  double x, y, eps;
  int exact;
};
constexpr unsigned long long NM_SPIN_LIMIT = 1ull << 24;
// c ? a : b field by field (a select of whole structs is lowered through
// their addresses, which puts the simplex's values in scratch memory)
__device__ __forceinline__ NmVal nm_sel(bool c, const NmVal &a, const NmVal &b) {
  return NmVal{c ? a.x : b.x, c ? a.y : b.y, c ? a.eps : b.eps, c ? a.exact : b.exact};
}

// Hand-offs between the controller and the workers (MI355X_MICROARCH.md,
// inter-workgroup visibility, the sc1 form): every handed-off byte is
// stored and loaded with agent-scope relaxed atomics (global_store/load
// sc1, write-through / L1-bypassing), every storing wave drains its stores
// (vmcnt(0)) before a workgroup barrier, then one lane stores the flag
// (sc1); the consumer polls the flag with sc1 loads and loads the bytes
// with sc1 loads after its poll matched (other waves behind a barrier).
// No L2 write-back or invalidate per round.
__device__ inline unsigned long long nm_ld(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double nm_ldd(const double *p) {
  return __longlong_as_double((long long)nm_ld((const unsigned long long *)p));
}
__device__ inline void nm_st(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void nm_std(double *p, double v) { nm_st((unsigned long long *)p, (unsigned long long)__double_as_longlong(v)); }
__device__ inline void nm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ inline NmPart nm_part_add(NmPart a, NmPart b) {
  const dd s = dd_add(dd{a.s_hi, a.s_lo}, dd{b.s_hi, b.s_lo}), q = dd_add(dd{a.q_hi, a.q_lo}, dd{b.q_hi, b.q_lo});
  const int f = (int)a.flags | (int)b.flags;
  return NmPart{s.hi, s.lo, q.hi, q.lo, fmax(a.mx, b.mx), (double)f};
}
// down-shift within 32-lane segments
__device__ inline NmPart nm_part_shfl32(NmPart a, int off) {
  return NmPart{__shfl_down(a.s_hi, off, 32), __shfl_down(a.s_lo, off, 32), __shfl_down(a.q_hi, off, 32),
                __shfl_down(a.q_lo, off, 32), __shfl_down(a.mx, off, 32), __shfl_down(a.flags, off, 32)};
}
__device__ inline NmPart nm_part_ld(const NmPart *p) {
  const double *d = (const double *)p;
  return NmPart{nm_ldd(d), nm_ldd(d + 1), nm_ldd(d + 2), nm_ldd(d + 3), nm_ldd(d + 4), nm_ldd(d + 5)};
}
__device__ inline void nm_part_st(NmPart *p, const NmPart &v) {
  double *d = (double *)p;
  nm_std(d, v.s_hi);
  nm_std(d + 1, v.s_lo);
  nm_std(d + 2, v.q_hi);
  nm_std(d + 3, v.q_lo);
  nm_std(d + 4, v.mx);
  nm_std(d + 5, v.flags);
}

// minSearch's one-dimensional nmsimplex loop (:712-779; the host's
// min_search below, comparison for comparison) over values that
// run_round(pts, n) leaves in val[] / spts[] / sbn (it returns true when a
// hand-off timed out).  Shared by the controller of k_tm_nm_search and every
// workgroup of k_tm_nm_sym, which all run it on identical values.
template <class RunRound>
__device__ __forceinline__ void nm_drive(const NmTab &tab, const NmVal *val, const double *spts, const int &sbn,
                                         RunRound &run_round, double &X0, double &X1, NmVal &Y0, NmVal &Y1,
                                         long long &iter, int &lo, int &status, int &nneed, double &need0,
                                         double &need1) {
  auto request = [&](const NmVal &v) __attribute__((always_inline)) {
    // branch-free (keeps need0 / need1 in registers)
    const bool first = !v.exact && nneed == 0;
    const bool second = !v.exact && nneed == 1 && __double_as_longlong(v.x) != __double_as_longlong(need0);
    need0 = first ? v.x : need0;
    need1 = second ? v.x : need1;
    nneed += (first || second) ? 1 : 0;
    status = 1;
  };
  // the value at x; `slot` is where the round's batch put x (checked)
  auto get = [&](double x, NmVal &v, int slot) __attribute__((always_inline)) {
    bool found = false;
    if (tab.n > 0) {
#pragma unroll
      for (int t = 0; t < NM_TAB; t++)
        if (!found && t < tab.n && __double_as_longlong(tab.x[t]) == __double_as_longlong(x)) {
          v = NmVal{x, tab.y[t], 0.0, 1};
          found = true;
        }
      if (found) return;
    }
    if (slot < sbn && __double_as_longlong(spts[slot]) == __double_as_longlong(x)) {
      v = val[slot];
      found = true;
    }
    for (int k = 0; !found && k < sbn; k++)
      if (__double_as_longlong(spts[k]) == __double_as_longlong(x)) {
        v = val[k];
        found = true;
        break;
      }
    if (!found) {
      double one[NM_PTS] = {x, 0, 0, 0, 0, 0, 0, 0};
      if (run_round(one, 1)) status = 2;
      v = val[0];
    }
    if (v.exact < 0) {  // degenerate: the host's exact value decides
      v.exact = 0;
      request(v);
    }
  };
  // a < b (or a <= b): exact values compare exactly, others on their
  // intervals; undecidable -> request the inexact operands
  auto cmp = [&](const NmVal &a, const NmVal &b, bool orEqual) __attribute__((always_inline)) -> bool {
    if (a.exact && b.exact) return orEqual ? a.y <= b.y : a.y < b.y;
    if (a.y + a.eps < b.y - b.eps) return true;
    if (a.y - a.eps > b.y + b.eps) return false;
    request(a);
    request(b);
    return false;
  };
  const int MaxIter = 1000;
  const double Tol = 1e-12;
  {
    const double p2[NM_PTS] = {X0, X1, 0, 0, 0, 0, 0, 0};
    if (run_round(p2, 2)) status = 2;
    get(X0, Y0, 0);
    if (!status) get(X1, Y1, 1);
  }
  while (status == 0) {
    iter++;
    int hi = 0;
    lo = 0;
    if (cmp(Y1, Y0, false)) {
      lo = 1;
    } else {
      if (status) break;
      if (cmp(Y0, Y1, false)) hi = 1;
    }
    if (status) break;
    const double Xhi = hi ? X1 : X0, Xlo = lo ? X1 : X0;
    const double mp = hi ? X0 : X1;
    const double xc = mp - (-1.0) * (mp - Xhi);
    {
      // every point this iteration may evaluate (the host's batch)
      double pts[NM_PTS] = {0, 0, 0, 0, 0, 0, 0, 0};
      int np = 0;
      pts[np++] = xc;
      pts[np++] = mp - (-2.0) * (mp - Xhi);
      pts[np++] = mp - 0.5 * (mp - Xhi);
      pts[np++] = mp - 0.5 * (mp - xc);
      // shrink towards lo, with and without X[hi] = xc (1-D: the vertex != lo)
      const double Xo = lo ? X0 : X1;  // the vertex that is not lo
      const double XoR = (hi == lo) ? Xo : xc, XloR = (hi == lo) ? xc : Xlo;
      pts[np++] = 0.5 * (Xo + Xlo);
      pts[np++] = 0.5 * (XoR + XloR);
      if (run_round(pts, np)) status = 2;
      if (status) break;
    }
    NmVal v;
    get(xc, v, 0);
    if (status) break;
    const NmVal Ylo = nm_sel(lo, Y1, Y0);
    const bool better = cmp(v, Ylo, false);
    if (status) break;
    if (better) {
      NmVal v2;
      const double xc2 = mp - (-2.0) * (mp - Xhi);
      get(xc2, v2, 1);
      if (status) break;
      const bool b2 = cmp(v2, Ylo, false);
      if (status) break;
      const double nx = b2 ? xc2 : xc;
      const NmVal ny = nm_sel(b2, v2, v);
      if (hi) X1 = nx, Y1 = ny;
      else X0 = nx, Y0 = ny;
    } else {
      const bool worse = cmp(Y0, v, false);  // Y[s_hi], s_hi = 0
      if (status) break;
      if (worse) {
        const bool r1 = cmp(v, nm_sel(hi, Y1, Y0), true);
        if (status) break;
        if (r1) {
          if (hi) X1 = xc, Y1 = v;
          else X0 = xc, Y0 = v;
        }
        NmVal v2;
        const double xh = hi ? X1 : X0;
        const double xc2 = mp - 0.5 * (mp - xh);
        get(xc2, v2, r1 ? 3 : 2);
        if (status) break;
        const bool r2 = cmp(v2, nm_sel(hi, Y1, Y0), true);
        if (status) break;
        if (r2) {
          if (hi) X1 = xc2, Y1 = v2;
          else X0 = xc2, Y0 = v2;
        } else {
          // X[i] = 0.5 (X[i] + X[lo]) for i != lo
          if (lo == 0) {
            X1 = 0.5 * (X1 + X0);
            get(X1, Y1, r1 ? 5 : 4);
          } else {
            X0 = 0.5 * (X0 + X1);
            get(X0, Y0, r1 ? 5 : 4);
          }
          if (status) break;
        }
      } else {
        if (hi) X1 = xc, Y1 = v;
        else X0 = xc, Y0 = v;
      }
    }
    const bool r = cmp(Y1, Y0, false);
    if (status) break;
    lo = r ? 1 : 0;
    const double center = (X0 + X1) / 2;
    double ssz = 0.0;
    ssz += fabs(X0 - center);
    ssz += fabs(X1 - center);
    if (!(ssz / 2.0 < Tol) && iter < MaxIter) continue;
    break;
  }
}

__global__ void __launch_bounds__(NM_TPB) k_tm_nm_search(int P, const double *__restrict__ ll,
                                                          const TmDev *__restrict__ dev, double rho, double target,
                                                          NmTab tab, NmSync *__restrict__ S, NmOut *__restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = tid >> 5, sub = tid & 31;  // point / segment lane of the 32-wide reductions
  const double llmax = dev->llmaxCv;
  if (blockIdx.x > 0) {
    // ------------------------------------------------------------ worker
    __shared__ double sll[NM_LDS];
    __shared__ double sx[NM_PTS];
    __shared__ int sn, squit;
    __shared__ NmPart red[NM_PTS][NM_TPB];
    const int w = blockIdx.x - 1, chunk = (P + NM_W - 1) / NM_W;
    const int i0 = w * chunk < P ? w * chunk : P, i1 = (w + 1) * chunk < P ? (w + 1) * chunk : P;
    const bool inLds = chunk <= NM_LDS;
    if (inLds)
      for (int i = i0 + tid; i < i1; i += NM_TPB) sll[i - i0] = ll[i];
    unsigned long long tw0 = 0, tw1 = 0, tw2 = 0;
    for (unsigned long long round = 1;; round++) {
      const unsigned long long ta = __builtin_amdgcn_s_memrealtime();
      if (tid == 0) {
        unsigned long long spins = 0;
        while (nm_ld(&S->seq) < round && ++spins < NM_SPIN_LIMIT) __builtin_amdgcn_s_sleep(1);
        if (spins >= NM_SPIN_LIMIT) {
          squit = 1;
        } else {
          squit = (int)nm_ld(&S->quit);
          sn = (int)nm_ld(&S->n);
          for (int k = 0; k < NM_PTS; k++) sx[k] = nm_ldd(&S->x[k]);
        }
      }
      __syncthreads();
      if (squit) {
        if (tid == 0 && w == 0) out->tw[0] = tw0, out->tw[1] = tw1, out->tw[2] = tw2;
        return;
      }
      const unsigned long long tb = __builtin_amdgcn_s_memrealtime();
      const int n = sn;
      NmPart acc[NM_PTS];
#pragma unroll
      for (int k = 0; k < NM_PTS; k++) acc[k] = NmPart{0, 0, 0, 0, 0, 0};
      int fl[NM_PTS];
#pragma unroll
      for (int k = 0; k < NM_PTS; k++) fl[k] = 0;
      for (int i = i0 + tid; i < i1; i += NM_TPB) {
        const double a = (inLds ? sll[i - i0] : ll[i]) - llmax;
#pragma unroll
        for (int k = 0; k < NM_PTS; k++) {
          if (k < n) {
            const double arg = a * (sx[k] - rho);
            const double e = exp(arg);
            fl[k] |= (!isfinite(e) ? 1 : 0) | (arg != 0.0 ? 2 : 0);
            const double d = e - 1.0;
            const dd s2 = dd_add(dd{acc[k].s_hi, acc[k].s_lo}, dd{d, 0.0});
            const dd q2 = dd_add(dd{acc[k].q_hi, acc[k].q_lo}, dd_tp(d, d));
            acc[k].s_hi = s2.hi, acc[k].s_lo = s2.lo, acc[k].q_hi = q2.hi, acc[k].q_lo = q2.lo;
            acc[k].mx = e > acc[k].mx ? e : acc[k].mx;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < NM_PTS; k++) {
        acc[k].flags = (double)fl[k];
        if (k < n) red[k][tid] = acc[k];
      }
      __syncthreads();
      const unsigned long long tcomp = __builtin_amdgcn_s_memrealtime();
      // point grp: 8 serial adds per segment lane, then a 32-lane tree
      if (grp < n) {
        NmPart v = red[grp][sub];
        for (int j = 1; j < NM_TPB / 32; j++) v = nm_part_add(v, red[grp][sub + 32 * j]);
        for (int off = 16; off > 0; off >>= 1) v = nm_part_add(v, nm_part_shfl32(v, off));
        if (sub == 0) nm_part_st(&S->part[w][grp], v);
        nm_drain();
      }
      __syncthreads();  // every storing wave has drained its stores
      if (tid == 0) nm_st(&S->done[w], round);
      const unsigned long long te = __builtin_amdgcn_s_memrealtime();
      tw0 += tb - ta;
      tw1 += tcomp - tb;
      tw2 += te - tcomp;
    }
  }
  // -------------------------------------------------------------- controller
  __shared__ NmVal val[NM_PTS];
  __shared__ double spts[NM_PTS];
  __shared__ int sfail;
  unsigned long long round = 0;
  unsigned evals = 0;
  // the last round's points and values stay in LDS (spts, val, sbn) until
  // the next round
  __shared__ int sbn;
  // one round over pts[0..n): broadcast, fan-in, fixed-order combine
  unsigned long long tc0 = 0, tc1 = 0, tc2 = 0, tlast = __builtin_amdgcn_s_memrealtime();
  const dd invP = dd_div(dd{1.0, 0.0}, dd{(double)P, 0.0});
  auto run_round = [&](const double *pts, int n) __attribute__((always_inline)) {
    const unsigned long long ra = __builtin_amdgcn_s_memrealtime();
    tc2 += ra - tlast;
    round++;
    evals += n;
    __syncthreads();  // every thread has read the previous round's spts / val
    if (tid == 0) {
#pragma unroll
      for (int k = 0; k < NM_PTS; k++) {
        const double x = k < n ? pts[k] : 0.0;
        nm_std(&S->x[k], x);
        spts[k] = x;
      }
      nm_st(&S->n, (unsigned long long)n);
      nm_st(&S->quit, 0ull);
      sbn = n;
      nm_drain();
      nm_st(&S->seq, round);
    }
    if (wid == 0) {
      unsigned long long spins = 0;
      for (;;) {
        const bool ok = nm_ld(&S->done[lane]) >= round;  // NM_W == 64: one lane per worker
        if (__all(ok)) break;
        if (++spins >= NM_SPIN_LIMIT) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) sfail = spins >= NM_SPIN_LIMIT;
    }
    __syncthreads();
    const unsigned long long rb = __builtin_amdgcn_s_memrealtime();
    // point grp over the 64 workers' records: 2 per segment lane, then a 32-lane tree
    if (grp < n) {
      const int k = grp;
      NmPart v = nm_part_add(nm_part_ld(&S->part[sub][k]), nm_part_ld(&S->part[sub + 32][k]));
      for (int off = 16; off > 0; off >>= 1) v = nm_part_add(v, nm_part_shfl32(v, off));
      if (sub == 0) {
        const dd Sd{v.s_hi, v.s_lo}, Qd{v.q_hi, v.q_lo};
        const dd dmean = dd_mul(Sd, invP);
        const dd ss = dd_add(Qd, dd_mul(dd{-Sd.hi, -Sd.lo}, dmean));
        const double var = (ss.hi + ss.lo) / (double)(P - 1);
        const dd mean = dd_add(dmean, dd{1.0, 0.0});
        const double meand = mean.hi + mean.lo;
        const double cv = sqrt(var > 0.0 ? var : 0.0) / meand;
        double c = cv - target;
        c *= c;
        const double ratio = v.mx / meand;
        // CvSearch::get's bound, plus 16 u max/mean for the device exp
        const double u = 1.1102230246251565e-16, acv = fabs(cv);
        const double dc = 1e-13 * acv + 32.0 * u * ratio + 4.0 * u * u / (acv > 1e-300 ? acv : 1e-300);
        const double eps = 2.0 * fabs(cv - target) * dc + dc * dc + 4.0 * u * fabs(c) + 1e-300;
        // every argument exactly 0: every E is exactly 1 and cv2_tail gives target^2
        const int vf = (int)v.flags;
        const bool allOne = vf == 0 && P > 1;
        const bool bad = (vf & 1) || !isfinite(c) || !(meand > 0.0) || !isfinite(ratio) || var < 0.0 ||
                         !isfinite(eps);
        const double x = spts[k];
        val[k] = allOne ? NmVal{x, target * target, 0.0, 1} : NmVal{x, c, eps, bad ? -1 : 0};
      }
    }
    __syncthreads();
    tlast = __builtin_amdgcn_s_memrealtime();
    tc0 += rb - ra;
    tc1 += tlast - rb;
    return sfail != 0;
  };
  double X0 = rho, X1 = rho + 1e-8;  // (GSL step 1e-8)
  NmVal Y0{}, Y1{};
  long long iter = 0;
  int lo = 0, status = 0, nneed = 0;
  double need0 = 0.0, need1 = 0.0;
  nm_drive(tab, val, spts, sbn, run_round, X0, X1, Y0, Y1, iter, lo, status, nneed, need0, need1);
  if (tid == 0) {
    nm_st(&S->quit, 1ull);
    nm_drain();
    nm_st(&S->seq, round + 1);  // workers leave
    const NmVal Ylo = nm_sel(lo, Y1, Y0);
    out->X[0] = X0;
    out->X[1] = X1;
    out->y[0] = Y0.y;
    out->y[1] = Y1.y;
    out->need[0] = need0;
    out->need[1] = need1;
    out->iters = iter;
    out->status = status;
    out->lo = lo;
    out->nneed = nneed;
    out->loExact = status ? 0 : Ylo.exact;
    out->loBad = Ylo.exact < 0;
    out->loEps = Ylo.eps;
    out->evals = evals;
    out->rounds = (unsigned)round;
    out->tc[0] = tc0;
    out->tc[1] = tc1;
    out->tc[2] = tc2 + (__builtin_amdgcn_s_memrealtime() - tlast);
  }
}

// The same search with NO controller (round 4): NM_W symmetric workgroups,
// each holding P/NM_W log-likelihoods in LDS.  A round is ONE hand-off:
// every workgroup evaluates the round's points on its slice, publishes its
// partial records (by round parity) and its round flag, waits for every
// other flag, adds all NM_W records in the fixed tree order, and runs the
// simplex logic (nm_drive) itself on those identical values, so every
// workgroup decides the same next points without a broadcast.  (The
// controller form pays two hand-offs per round: points out, partials in.)
// Results equal k_tm_nm_search's: the same partials, the same combine, the
// same logic.
//
// NMW (16, 32 or 64) workgroups: enough that each thread evaluates about one
// log-likelihood per point (P / 256 of them), no more -- every extra
// workgroup is one more arrival to wait for and one more record to add.
template <int NMW>
__global__ void __launch_bounds__(NM_TPB) k_tm_nm_sym(int P, const double *__restrict__ ll,
                                                       const TmDev *__restrict__ dev, double rho, double target,
                                                       NmTab tab, NmSync *__restrict__ S, NmOut *__restrict__ out) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = tid >> 5, sub = tid & 31;  // point / segment lane of the 32-wide reductions
  const double llmax = dev->llmaxCv;
  __shared__ double sll[NM_LDS];
  __shared__ NmPart red[NM_PTS][NM_TPB];
  __shared__ NmVal val[NM_PTS];
  __shared__ double spts[NM_PTS];
  __shared__ int sfail, sbn;
  const unsigned long long tk0 = __builtin_amdgcn_s_memrealtime();
  const int w = blockIdx.x, chunk = (P + NMW - 1) / NMW;
  const int i0 = w * chunk < P ? w * chunk : P, i1 = (w + 1) * chunk < P ? (w + 1) * chunk : P;
  const bool inLds = chunk <= NM_LDS;
  if (inLds)
    for (int i = i0 + tid; i < i1; i += NM_TPB) sll[i - i0] = ll[i];
  unsigned long long round = 0;
  unsigned evals = 0;
  unsigned long long tEval = 0, tWait = 0, tComb = 0, tRest = 0, tlast = __builtin_amdgcn_s_memrealtime(), tFirst = 0;
  const dd invP = dd_div(dd{1.0, 0.0}, dd{(double)P, 0.0});
  auto run_round = [&](const double *pts, int n) __attribute__((always_inline)) {
    const unsigned long long ra = __builtin_amdgcn_s_memrealtime();
    tRest += ra - tlast;
    if (round == 0) tFirst = ra;
    round++;
    evals += n;
    __syncthreads();  // every thread has read the previous round's spts / val (and sll is loaded)
    if (tid < NM_PTS) {  // (static indices: pts stays in registers, not in scratch)
      double x = 0.0;
#pragma unroll
      for (int k = 0; k < NM_PTS; k++)
        if (k == tid && k < n) x = pts[k];
      spts[tid] = x;
    }
    if (tid == 0) sbn = n;
    // ---- this workgroup's slice (as k_tm_nm_search's workers)
    NmPart acc[NM_PTS];
#pragma unroll
    for (int k = 0; k < NM_PTS; k++) acc[k] = NmPart{0, 0, 0, 0, 0, 0};
    int fl[NM_PTS];
#pragma unroll
    for (int k = 0; k < NM_PTS; k++) fl[k] = 0;
    for (int i = i0 + tid; i < i1; i += NM_TPB) {
      const double a = (inLds ? sll[i - i0] : ll[i]) - llmax;
#pragma unroll
      for (int k = 0; k < NM_PTS; k++) {
        if (k < n) {
          const double arg = a * (pts[k] - rho);
          const double e = exp(arg);
          fl[k] |= (!isfinite(e) ? 1 : 0) | (arg != 0.0 ? 2 : 0);
          const double d = e - 1.0;
          const dd s2 = dd_add(dd{acc[k].s_hi, acc[k].s_lo}, dd{d, 0.0});
          const dd q2 = dd_add(dd{acc[k].q_hi, acc[k].q_lo}, dd_tp(d, d));
          acc[k].s_hi = s2.hi, acc[k].s_lo = s2.lo, acc[k].q_hi = q2.hi, acc[k].q_lo = q2.lo;
          acc[k].mx = e > acc[k].mx ? e : acc[k].mx;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NM_PTS; k++) {
      acc[k].flags = (double)fl[k];
      if (k < n) red[k][tid] = acc[k];
    }
    __syncthreads();
    NmPart *mine = S->part2[round & 1][w];
    if (grp < n) {
      NmPart v = red[grp][sub];
      for (int j = 1; j < NM_TPB / 32; j++) v = nm_part_add(v, red[grp][sub + 32 * j]);
      for (int off = 16; off > 0; off >>= 1) v = nm_part_add(v, nm_part_shfl32(v, off));
      if (sub == 0) nm_part_st(&mine[grp], v);
      nm_drain();
    }
    __syncthreads();  // every storing wave has drained its stores
    if (tid == 0) nm_st(&S->done[w], round);
    const unsigned long long rb = __builtin_amdgcn_s_memrealtime();
    // ---- every workgroup's records of this round
    if (wid == 0) {
      unsigned long long spins = 0;
      for (;;) {
        const bool ok = lane >= NMW || nm_ld(&S->done[lane]) >= round;  // one lane per workgroup
        if (__all(ok)) break;
        if (++spins >= NM_SPIN_LIMIT) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) sfail = spins >= NM_SPIN_LIMIT;
    }
    __syncthreads();
    const unsigned long long rc = __builtin_amdgcn_s_memrealtime();
    if (grp < n) {
      const int k = grp;
      NmPart v = NmPart{0, 0, 0, 0, 0, 0};  // (an exact identity of nm_part_add)
      if (NMW == 64)
        v = nm_part_add(nm_part_ld(&S->part2[round & 1][sub][k]), nm_part_ld(&S->part2[round & 1][sub + 32][k]));
      else if (sub < NMW)
        v = nm_part_ld(&S->part2[round & 1][sub][k]);
      for (int off = 16; off > 0; off >>= 1) v = nm_part_add(v, nm_part_shfl32(v, off));
      if (sub == 0) {
        const dd Sd{v.s_hi, v.s_lo}, Qd{v.q_hi, v.q_lo};
        const dd dmean = dd_mul(Sd, invP);
        const dd ss = dd_add(Qd, dd_mul(dd{-Sd.hi, -Sd.lo}, dmean));
        const double var = (ss.hi + ss.lo) / (double)(P - 1);
        const dd mean = dd_add(dmean, dd{1.0, 0.0});
        const double meand = mean.hi + mean.lo;
        const double cv = sqrt(var > 0.0 ? var : 0.0) / meand;
        double c = cv - target;
        c *= c;
        const double ratio = v.mx / meand;
        const double u = 1.1102230246251565e-16, acv = fabs(cv);
        const double dc = 1e-13 * acv + 32.0 * u * ratio + 4.0 * u * u / (acv > 1e-300 ? acv : 1e-300);
        const double eps = 2.0 * fabs(cv - target) * dc + dc * dc + 4.0 * u * fabs(c) + 1e-300;
        const int vf = (int)v.flags;
        const bool allOne = vf == 0 && P > 1;
        const bool bad = (vf & 1) || !isfinite(c) || !(meand > 0.0) || !isfinite(ratio) || var < 0.0 ||
                         !isfinite(eps);
        const double x = spts[k];
        val[k] = allOne ? NmVal{x, target * target, 0.0, 1} : NmVal{x, c, eps, bad ? -1 : 0};
      }
    }
    __syncthreads();
    tlast = __builtin_amdgcn_s_memrealtime();
    tEval += rb - ra;
    tWait += rc - rb;
    tComb += tlast - rc;
    return sfail != 0;
  };
  double X0 = rho, X1 = rho + 1e-8;  // (GSL step 1e-8)
  NmVal Y0{}, Y1{};
  long long iter = 0;
  int lo = 0, status = 0, nneed = 0;
  double need0 = 0.0, need1 = 0.0;
  nm_drive(tab, val, spts, sbn, run_round, X0, X1, Y0, Y1, iter, lo, status, nneed, need0, need1);
  if (w == 0 && tid == 0) {
    const NmVal Ylo = nm_sel(lo, Y1, Y0);
    out->X[0] = X0;
    out->X[1] = X1;
    out->y[0] = Y0.y;
    out->y[1] = Y1.y;
    out->need[0] = need0;
    out->need[1] = need1;
    out->iters = iter;
    out->status = status;
    out->lo = lo;
    out->nneed = nneed;
    out->loExact = status ? 0 : Ylo.exact;
    out->loBad = Ylo.exact < 0;
    out->loEps = Ylo.eps;
    out->evals = evals;
    out->rounds = (unsigned)round;
    // (phases: hand-off wait, simplex logic, evaluation + publish)
    out->tc[0] = tWait;
    out->tc[1] = tRest + (__builtin_amdgcn_s_memrealtime() - tlast);
    out->tc[2] = tEval;
    // (workgroup 0: whole kernel, its prologue before the first round, the
    // combine of every round's records)
    out->tw[0] = __builtin_amdgcn_s_memrealtime() - tk0;
    out->tw[1] = tFirst - tk0;
    out->tw[2] = tComb;
  }
}

// the exponentials (exp_cr, k_tm_cv_exp's values) of the points whose
// exact value the host forms next: X[lo] after a finished search, the
// requested points after status 1
__global__ void k_tm_nm_exp(int P, const double *__restrict__ ll, const TmDev *__restrict__ dev, double rho,
                            const NmOut *__restrict__ o, double *__restrict__ E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
  if (i >= P) return;
  const int nE = o->status == 1 ? o->nneed : (o->status == 0 && !o->loExact ? 1 : 0);
  if (j >= nE) return;
  const double x = o->status == 1 ? o->need[j] : o->X[o->lo];
  E[(size_t)j * P + i] = exp_cr((ll[i] - dev->llmaxCv) * (x - rho));
}

// processGeneration :284-296: w_i = exp(ll_i (rho - rho_prev) - max)
__global__ void k_tm_lw_exp(int P, const double *__restrict__ ll, double drho, const TmDev *__restrict__ dev,
                            double *__restrict__ E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  E[i] = exp_cr(ll[i] * drho - dev->lwmax);
}

// processGeneration :318-329, the weighted mean and covariance of the
// database, each output element one ordered P-long sum (the reference's
// order, so the result is bit-identical):
//   mean_i = sum_j db[j][i] w_j
//   cov_ij = covScaling * s / (1 - sum w^2),  s = sum_k w_k (x_ki - m_i)(x_kj - m_j),  j >= i
// The factors of every term are formed first by fully parallel kernels,
// in the reference's operand order (left to right, identical roundings):
//   mean: T[k][i]  = db[k][i] * w_k
//   cov : WD[k][i] = w_k * (db[k][i] - m_i),  D[k][i] = db[k][i] - m_i
// (cov term = WD[k][i] * D[k][j]).  The ordered sums then use one lane per
// output element in wave 0 of each workgroup; three more waves stream the
// factor rows into a double-buffered LDS tile (16-byte loads, all in flight
// at once), the computing wave reads the next terms while adding the
// current ones, and its dependent add chain (14 cycles per add on gfx950,
// tools/ubench_chain.hip) is the cost.
__global__ void k_tm_factors_mean(int N, int P, const double *__restrict__ db, const double *__restrict__ w,
                                  double *__restrict__ T) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < (size_t)P * N) T[e] = db[e] * w[e / N];
}
__global__ void k_tm_factors_cov(int N, int P, const double *__restrict__ db, const double *__restrict__ w,
                                 const double *__restrict__ mean, double *__restrict__ WD, double *__restrict__ D) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const double d = db[e] - mean[e % N];
  WD[e] = w[e / N] * d;
  D[e] = d;
}

constexpr int WS_TPB = 256, WS_LANES = 64, WS_MAXV = 16;  // 16 x 16-byte loads per thread per array
__host__ __device__ inline int ws_rows(int N, bool cov) {
  const int r = (WS_TPB * WS_MAXV * 2 / (cov ? 2 * N : N)) & ~7;
  return r < 8 ? 8 : (r > 256 ? 256 : r);
}
__host__ __device__ inline size_t ws_lds_bytes(int N, bool cov) {
  return 2 * (size_t)ws_rows(N, cov) * N * (cov ? 2 : 1) * sizeof(double);
}
template <bool COV>
__global__ void __launch_bounds__(WS_TPB) k_tm_wsum(int N, int P, const double *__restrict__ A,
                                                    const double *__restrict__ B, const int2 *__restrict__ pairs,
                                                    int nout, double scaling, double denom,
                                                    double *__restrict__ out) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  extern __shared__ double sm[];
  const int rows = ws_rows(N, COV);
  const int tile = rows * N;              // even: rows is a multiple of 8
  const int buf = COV ? 2 * tile : tile;  // one buffer: A tile, then B tile
  const int nchunks = (P + rows - 1) / rows;
  const int tid = threadIdx.x, oidx = blockIdx.x * WS_LANES + tid;
  const bool active = tid < WS_LANES && oidx < nout;
  int pi = 0, pj = 0;
  if (active) {
    if (COV) {
      const int2 ij = pairs[oidx];
      pi = ij.x;
      pj = ij.y;
    } else {
      pi = oidx;
    }
  }
  d2v ra[WS_MAXV], rb[WS_MAXV];
  int lim = 0;
  // branch-free 16-byte loads (clamped pair index, zeroed past the end; the
  // factor arrays carry 2 doubles of padding)
  auto fetch = [&](int c) {
    const int r0 = c * rows, nk = min(rows, P - r0);
    const d2v *a = (const d2v *)(A + (size_t)r0 * N), *b = (const d2v *)(B + (size_t)r0 * N);
    lim = nk * N;
    const int lastp = (lim - 1) >> 1;
#pragma unroll
    for (int v = 0; v < WS_MAXV; v++) {
      if (v * WS_TPB * 2 < tile) {  // uniform
        const int pidx = min(tid + v * WS_TPB, lastp);
        ra[v] = a[pidx];
        if (COV) rb[v] = b[pidx];
      }
    }
  };
  auto store = [&](double *dst) {
#pragma unroll
    for (int v = 0; v < WS_MAXV; v++) {
      const int e = 2 * (tid + v * WS_TPB);
      if (e < tile) {
        d2v x = ra[v];
        x.x = e < lim ? x.x : 0.0;
        x.y = e + 1 < lim ? x.y : 0.0;
        *(d2v *)(dst + e) = x;
        if (COV) {
          d2v y = rb[v];
          y.x = e < lim ? y.x : 0.0;
          y.y = e + 1 < lim ? y.y : 0.0;
          *(d2v *)(dst + tile + e) = y;
        }
      }
    }
  };
  fetch(0);
  store(sm);
  __syncthreads();
  double acc = 0.0;
  for (int c = 0; c < nchunks; c++) {
    if (c + 1 < nchunks) fetch(c + 1);
    const double *cur = sm + (c & 1) * buf;
    const int nk = min(rows, P - c * rows);
    if (active) {
      // software-pipelined: the next 8 terms are read while the current 8
      // are added, so the LDS latency stays off the add chain
      const double *Ta = cur, *Tb = cur + tile;
      auto term = [&](int r) { return COV ? Ta[r * N + pi] * Tb[r * N + pj] : Ta[r * N + pi]; };
      int r = 0;
      if (nk >= 16) {
        double ta[8], tb[8];
#pragma unroll
        for (int q = 0; q < 8; q++) ta[q] = term(q);
        for (; r + 16 <= nk; r += 16) {
#pragma unroll
          for (int q = 0; q < 8; q++) tb[q] = term(r + 8 + q);
#pragma unroll
          for (int q = 0; q < 8; q++) acc += ta[q];
          const int rn = min(r + 16, nk - 8);  // clamped prefetch, recomputed below if unused
#pragma unroll
          for (int q = 0; q < 8; q++) ta[q] = term(rn + q);
#pragma unroll
          for (int q = 0; q < 8; q++) acc += tb[q];
        }
      }
      for (; r < nk; r++) acc += term(r);
    }
    if (c + 1 < nchunks) store(sm + ((c + 1) & 1) * buf);
    __syncthreads();
  }
  if (!active) return;
  if (COV) {
    const double v = scaling * acc / denom;
    out[pi * N + pj] = v;
    out[pj * N + pi] = v;
  } else {
    out[pi] = acc;
  }
}

// The same ordered sums on ROW chains (round 4, the default): one 16-lane
// row per output element keeps the accumulator and adds its 16 lanes' terms
// through DPP row_newbcast operands of v_fmac_f64 (chains::kc_row16, one
// VALU instruction per term, ~8 cycles instead of the ~14 of a dependent
// v_add_f64 plus the LDS reads).  The factors are stored TRANSPOSED, one
// Pp-long row per variable (Pp = P rounded up to WR_D * 16, the pad is
// +0.0: acc starts at +0.0 and can never be -0.0, so adding +0.0 is a
// no-op), so a row's 16 lanes read 128 contiguous bytes; each lane keeps
// WR_D loads in flight (registers, no LDS, no barriers).
constexpr int WR_D = 32;
inline int wr_pitch(int P) { return (P + 16 * WR_D - 1) / (16 * WR_D) * (16 * WR_D); }
__global__ void k_tm_factors_mean_t(int N, int P, int Pp, const double *__restrict__ db,
                                    const double *__restrict__ w, double *__restrict__ TT) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)N * Pp) return;
  const int i = (int)(e / Pp), k = (int)(e % Pp);
  TT[e] = k < P ? db[(size_t)k * N + i] * w[k] : 0.0;
}
__global__ void k_tm_factors_cov_t(int N, int P, int Pp, const double *__restrict__ db, const double *__restrict__ w,
                                   const double *__restrict__ mean, double *__restrict__ WDT,
                                   double *__restrict__ DT) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)N * Pp) return;
  const int i = (int)(e / Pp), k = (int)(e % Pp);
  double wd = 0.0, d = 0.0;
  if (k < P) {
    d = db[(size_t)k * N + i] - mean[i];
    wd = w[k] * d;
  }
  WDT[e] = wd;
  DT[e] = d;
}
// One slot: wait for its loads (issued WR_D slots ago: every later load is
// one of this lane's own), form the term, 16 row-chain steps, reload the
// slot from the next group.  The loads are issued inside the asm so the
// compiler's conservative waits cannot drain the queue (it otherwise waits
// for every load at the loop head).
#define WR_FMAC16 \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"  \
  "v_fmac_f64 %[acc], %[t], %[one] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"  \

template <int S>
__device__ __forceinline__ void wr_slot_cov(double &acc, double &qa, double &qb, const double *an, const double *bn,
                                            double one) {
  double t;
  asm volatile(
      "s_waitcnt vmcnt(%[w])\n"
      "v_mul_f64 %[t], %[qa], %[qb]\n"
      "s_nop 1\n" WR_FMAC16
      "global_load_dwordx2 %[qa], %[pa], off offset:%[off]\n"
      "global_load_dwordx2 %[qb], %[pb], off offset:%[off]\n"
      : [acc] "+&v"(acc), [qa] "+&v"(qa), [qb] "+&v"(qb), [t] "=&v"(t)
      : [pa] "v"(an), [pb] "v"(bn), [one] "v"(one), [off] "i"(S * 128), [w] "i"(2 * WR_D - 2));
}
template <int S>
__device__ __forceinline__ void wr_slot_mean(double &acc, double &qa, const double *an, double one) {
  asm volatile(
      "s_waitcnt vmcnt(%[w])\n"
      "s_nop 1\n" WR_FMAC16
      "global_load_dwordx2 %[t], %[pa], off offset:%[off]\n"
      : [acc] "+&v"(acc), [t] "+&v"(qa)
      : [pa] "v"(an), [one] "v"(one), [off] "i"(S * 128), [w] "i"(WR_D - 1));
}
template <bool COV, int... S>
__device__ __forceinline__ void wr_group(double &acc, double (&qa)[WR_D], double (&qb)[WR_D], const double *an,
                                         const double *bn, double one, std::integer_sequence<int, S...>) {
  if (COV)
    (wr_slot_cov<S>(acc, qa[S], qb[S], an, bn, one), ...);
  else
    (wr_slot_mean<S>(acc, qa[S], an, one), ...);
}
template <int S>
__device__ __forceinline__ void wr_load_cov(double &qa, double &qb, const double *a, const double *b) {
  asm volatile(
      "global_load_dwordx2 %[qa], %[pa], off offset:%[off]\n"
      "global_load_dwordx2 %[qb], %[pb], off offset:%[off]\n"
      : [qa] "=&v"(qa), [qb] "=&v"(qb)
      : [pa] "v"(a), [pb] "v"(b), [off] "i"(S * 128));
}
template <int S>
__device__ __forceinline__ void wr_load_mean(double &qa, const double *a) {
  asm volatile("global_load_dwordx2 %[qa], %[pa], off offset:%[off]\n" : [qa] "=&v"(qa) : [pa] "v"(a), [off] "i"(S * 128));
}
template <bool COV, int... S>
__device__ __forceinline__ void wr_prologue(double (&qa)[WR_D], double (&qb)[WR_D], const double *a, const double *b,
                                            std::integer_sequence<int, S...>) {
  if (COV)
    (wr_load_cov<S>(qa[S], qb[S], a, b), ...);
  else
    (wr_load_mean<S>(qa[S], a), ...);
}
template <bool COV>
__global__ void __launch_bounds__(64) k_tm_wsum_rows(int N, int Pp, const double *__restrict__ A,
                                                     const double *__restrict__ B, const int2 *__restrict__ pairs,
                                                     int nout, double scaling, double denom,
                                                     double *__restrict__ out) {
  const int lane = threadIdx.x, l = lane & 15;
  const int o = blockIdx.x * 4 + (lane >> 4);
  const int oc = o < nout ? o : nout - 1;  // (a row past the end recomputes the last element, unused)
  int pi = oc, pj = 0;
  if (COV) {
    const int2 ij = pairs[oc];
    pi = ij.x;
    pj = ij.y;
  }
  const double *a = A + (size_t)pi * Pp + l;
  const double *b = B + (size_t)pj * Pp + l;
  const int ns = Pp >> 4;  // 16-term slots, a multiple of WR_D
  const double one = 1.0;
  double qa[WR_D], qb[WR_D];
  wr_prologue<COV>(qa, qb, a, b, std::make_integer_sequence<int, WR_D>{});
  double acc = 0.0;
  for (int g = 0; g < ns; g += WR_D) {
    const int nx = g + WR_D < ns ? g + WR_D : g;  // the last group reloads itself (unused)
    wr_group<COV>(acc, qa, qb, a + (size_t)nx * 16, b + (size_t)nx * 16, one,
                  std::make_integer_sequence<int, WR_D>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (o >= nout || l != 0) return;
  if (COV) {
    const double v = scaling * acc / denom;
    out[pi * N + pj] = v;
    out[pj * N + pi] = v;
  } else {
    out[pi] = acc;
  }
}

// leader expansion :331-360: leader j < count = database entry src[j] with
// chain length len[j]; chain lengths past count are 0 and those leaders keep
// their previous rows (std::fill of _chainLengths, :329)
__global__ void k_tm_expand(int N, int P, int count, const unsigned *__restrict__ src,
                            const double *__restrict__ len, const double *__restrict__ db,
                            const double *__restrict__ dbLL, const double *__restrict__ dbLP,
                            double *__restrict__ leaders, double *__restrict__ leadLL, double *__restrict__ leadLP,
                            double *__restrict__ chainLen) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const int j = (int)(e / N), d = (int)(e % N);
  if (j >= count) {
    if (d == 0) chainLen[j] = 0.0;
    return;
  }
  const unsigned s = src[j];
  leaders[e] = db[(size_t)s * N + d];
  if (d == 0) {
    leadLL[j] = dbLL[s];
    leadLP[j] = dbLP[s];
    chainLen[j] = len[j];
  }
}

__global__ void k_tm_fill(double *p, size_t n, double v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// ------------------------------------------------------- chain sharding
// After its chains finished, a shard's rows of the database, leaders and
// candidates (+ log-likelihoods / log-priors) and its accepted count travel
// in one buffer of 64-bit words: own entries carry their IEEE bits, all
// others INT64_MIN (the bits of -0.0).  A MAX all-reduce over the int64 view
// then yields every owner's exact bits (max(INT64_MIN, x) = x for every
// pattern x, including -0.0 itself), so the replicated state stays
// bit-identical to the unsharded run.
constexpr int XS_SECTIONS = 10;
struct XchSec {
  double *p;          // device array
  unsigned long long off, n;  // offset in the exchange buffer, words
  unsigned long long lo, hi;  // owned words [lo, hi) of the array
};
struct XchMap {
  XchSec s[XS_SECTIONS];
  int ns;
};

__global__ void k_tm_pack(XchMap m, unsigned long long total, long long *__restrict__ xch,
                          const TmDev *__restrict__ dev, int rank) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  long long v = LLONG_MIN;
  int k = 0;
  while (k + 1 < m.ns && i >= m.s[k + 1].off) k++;
  const XchSec q = m.s[k];
  const unsigned long long j = i - q.off;
  if (q.p) {
    if (j >= q.lo && j < q.hi) v = __double_as_longlong(q.p[j]);
  } else if ((int)j == rank) {
    v = (long long)dev->accepted;  // accepted-count slots, one per rank
  }
  xch[i] = v;
}

__global__ void k_tm_unpack(XchMap m, unsigned long long total, const long long *__restrict__ xch, TmDev *dev,
                            int world) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int k = 0;
  while (k + 1 < m.ns && i >= m.s[k + 1].off) k++;
  const XchSec q = m.s[k];
  const unsigned long long j = i - q.off;
  if (q.p) {
    q.p[j] = __longlong_as_double(xch[i]);
  } else if (j == 0) {
    unsigned long long a = 0;
    for (int r = 0; r < world; r++) a += (unsigned long long)xch[i + r];
    dev->accepted = (unsigned int)a;
  }
}

// ------------------------------------------------------------ host side
// GSL mt19937 (rng/mt.c) for the Multinomial generator, whose consumption is
// data-dependent and runs with the multinomial on the host.
struct HostMt {
  uint32_t mt[MT_N];
  int mti = MT_N;
  void seed(uint64_t s) {
    s &= 0xffffffffULL;
    if (s == 0) s = 4357;
    mt[0] = (uint32_t)s;
    for (int i = 1; i < MT_N; i++) mt[i] = (uint32_t)(1812433253UL * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i);
    mti = MT_N;
  }
  uint32_t get() {
    if (mti >= MT_N) refill();
    return mt_temper(mt[mti++]);
  }
  // the block regeneration in GSL's three ranges (no index wrap inside the
  // loops: the multinomial's walk draws ~P words per generation on the
  // host's critical path)
  void refill() {
    int k = 0;
    for (; k < MT_N - MT_M; k++) mt[k] = mt_next(mt[k], mt[k + 1], mt[k + MT_M]);
    for (; k < MT_N - 1; k++) mt[k] = mt_next(mt[k], mt[k + 1], mt[k + MT_M - MT_N]);
    mt[MT_N - 1] = mt_next(mt[MT_N - 1], mt[0], mt[MT_M - 1]);
    mti = 0;
  }
  double uniform() { return get() / 4294967296.0; }
  void save(unsigned char *b) const {
    memset(b, 0, 5000);
    for (int i = 0; i < MT_N; i++) {
      const uint64_t v = mt[i];
      memcpy(b + 8 * i, &v, 8);
    }
    const int32_t m = mti;
    memcpy(b + 8 * MT_N, &m, 4);
  }
  int load(const unsigned char *b) {
    int32_t m;
    memcpy(&m, b + 8 * MT_N, 4);
    KG_CHECK(m >= 0 && m <= MT_N, "invalid mt19937 state (mti out of range)");
    for (int i = 0; i < MT_N; i++) {
      uint64_t v;
      memcpy(&v, b + 8 * i, 8);
      mt[i] = (uint32_t)v;
    }
    mti = m;
    return 0;
  }
};

// gsl_ran_binomial (GSL 2.6 randist/binomial_tpe.c): inversion below
// n*p = 14, BTPE (Kachitvichyanukul & Schmeiser) above.
double pow_uint(double x, unsigned n) {
  double v = 1.0;
  do {
    if (n & 1) v *= x;
    n >>= 1;
    x *= x;
  } while (n);
  return v;
}

double btpe_tail(double y1) {
  const double y2 = y1 * y1;
  return (13860.0 - (462.0 - (132.0 - (99.0 - 140.0 / y2) / y2) / y2) / y2) / y1 / 166320.0;
}

unsigned binomial(HostMt &r, double p, unsigned n, double *btpeDraws) {
  if (n == 0) return 0;
  bool flip = false;
  if (p > 0.5) {
    p = 1.0 - p;
    flip = true;
  }
  const double q = 1 - p, s = p / q, np = n * p;
  int ix = 0;
  if (np < 14) {
    const double f0 = pow_uint(q, n);
    for (;;) {
      double f = f0, u = r.uniform();
      bool done = false;
      for (ix = 0; ix <= 110; ++ix) {
        if (u < f) {
          done = true;
          break;
        }
        u -= f;
        f *= s * (n - ix) / (ix + 1);
      }
      if (done) break;
    }
  } else {
    *btpeDraws += 1.0;  // diagnostics: draws that took the BTPE branch
    const double ffm = np + p;
    const int m = (int)ffm;
    const double fm = m, xm = fm + 0.5, npq = np * q;
    const double p1 = floor(2.195 * sqrt(npq) - 4.6 * q) + 0.5;
    const double xl = xm - p1, xr = xm + p1;
    const double c = 0.134 + 20.5 / (15.3 + fm);
    const double p2 = p1 * (1.0 + c + c);
    const double al = (ffm - xl) / (ffm - xl * p);
    const double lambda_l = al * (1.0 + 0.5 * al);
    const double ar = (xr - ffm) / (xr * q);
    const double lambda_r = ar * (1.0 + 0.5 * ar);
    const double p3 = p2 + c / lambda_l, p4 = p3 + c / lambda_r;
    for (;;) {
      const double u = r.uniform() * p4;
      double v = r.uniform();
      if (u <= p1) {
        ix = (int)(xm - p1 * v + u);
        break;
      } else if (u <= p2) {
        const double x = xl + (u - p1) / c;
        v = v * c + 1.0 - fabs(x - xm) / p1;
        if (v > 1.0 || v <= 0) continue;
        ix = (int)x;
      } else if (u <= p3) {
        ix = (int)(xl + host_log_cr(v) / lambda_l);
        if (ix < 0) continue;
        v = v * ((u - p2) * lambda_l);
      } else {
        ix = (int)(xr - host_log_cr(v) / lambda_r);
        if (ix > (double)n) continue;
        v = v * ((u - p3) * lambda_r);
      }
      const int k = abs(ix - m);
      double var, accept;
      if (k <= 20) {
        const double g = (n + 1) * s;
        double f = 1.0;
        var = v;
        if (m < ix) {
          for (int i = m + 1; i <= ix; i++) f *= (g / i - s);
        } else if (m > ix) {
          for (int i = ix + 1; i <= m; i++) f /= (g / i - s);
        }
        accept = f;
      } else {
        var = host_log_cr(v);
        if (k < npq / 2 - 1) {
          const double amaxp = k / npq * ((k * (k / 3.0 + 0.625) + (1.0 / 6.0)) / npq + 0.5);
          const double ynorm = -(k * k / (2.0 * npq));
          if (var < ynorm - amaxp) break;
          if (var > ynorm + amaxp) continue;
        }
        const double x1 = ix + 1.0, w1 = n - ix + 1.0, f1 = fm + 1.0, z1 = n + 1.0 - fm;
        accept = xm * host_log_cr(f1 / x1) + (n - m + 0.5) * host_log_cr(z1 / w1) +
                 (ix - m) * host_log_cr(w1 * p / (x1 * q)) + btpe_tail(f1) + btpe_tail(z1) - btpe_tail(x1) -
                 btpe_tail(w1);
      }
      if (var <= accept) break;
    }
  }
  return flip ? (n - ix) : (unsigned)ix;
}

// gsl_ran_multinomial (randist/multinomial.c), Multinomial::getSelections
// (specific/multinomial/multinomial.cpp.base:7-10)
void multinomial(HostMt &r, size_t K, unsigned N, const double *p, unsigned *n, double *btpeDraws) {
  double norm = 0.0, sum_p = 0.0;
  unsigned sum_n = 0;
  for (size_t k = 0; k < K; k++) norm += p[k];
  for (size_t k = 0; k < K; k++) {
    n[k] = p[k] > 0.0 ? binomial(r, p[k] / (norm - sum_p), N - sum_n, btpeDraws) : 0;
    sum_p += p[k];
    sum_n += n[k];
  }
}

// multinomial() with the inversion's comparisons decided on certified
// intervals (round 4).  gsl_ran_binomial's inversion compares the uniform
// with f0 = pow_uint(q, n) and its successors f_(ix+1) = f_ix s (n - ix) /
// (ix + 1), subtracting each from u: only the OUTCOME of those comparisons
// matters (the counts and the stream position), not the values.  Here f0 is
// exp(n log q), within d0 = (n + 128) 2^-50 + |n log q| 2^-51 of pow_uint's
// value relative (pow_uint's squarings: <= n 2^-53; log and exp: <= 1 ulp
// each), and the successors and u carry running bounds; a comparison whose
// intervals straddle goes through the exact loop from the same uniform, so
// the result is the reference's bit for bit (KORALI_AMD_TM_MULTINOMIAL=exact:
// the exact form everywhere; tests/test_multinomial_cpu.py compares both
// with the oracle).  The walk's dependent chain loses pow_uint's squarings,
// its branches, and the division per step.
static double g_inv1[112];
static const bool g_inv1_init = [] {
  for (int i = 0; i < 112; i++) g_inv1[i] = 1.0 / (i + 1);
  return true;
}();
unsigned binomial_inv_exact(HostMt &r, double u, double q, double s, bool flip, unsigned n) {
  const double f0 = pow_uint(q, n);
  int ix = 0;
  for (;;) {
    double f = f0;
    bool done = false;
    for (ix = 0; ix <= 110; ++ix) {
      if (u < f) {
        done = true;
        break;
      }
      u -= f;
      f *= s * (n - ix) / (ix + 1);
    }
    if (done) break;
    u = r.uniform();
  }
  return flip ? (n - ix) : (unsigned)ix;
}
unsigned binomial_inv_interval(HostMt &r, double q, double lq, double s, bool flip, unsigned n) {
  const double u0 = r.uniform();
  const double z = (double)n * lq;
  double F = exp(z);
  if (F > 1e-280) {
    double d = (n + 128.0) * 8.881784197001252e-16 + fabs(z) * 4.440892098500626e-16;  // |F - f| <= d f
    double U = u0, E = 0.0;                                                            // |U - u| <= E
    for (int ix = 0; ix <= 110; ++ix) {
      const double lo = F * (1.0 - 2.0 * d), hi = F * (1.0 + 2.0 * d);
      if (U + E < lo) return flip ? (n - ix) : (unsigned)ix;  // u < f certainly
      if (!(U - E >= hi)) break;                               // straddles (or NaN): the exact loop
      const double U1 = U - F;
      E = E + 2.0 * d * F + 2.220446049250313e-16 * (fabs(U1) + fabs(U)) + 1e-300;
      U = U1;
      F = F * (s * (double)(n - ix)) * g_inv1[ix];
      d = d + 6.661338147750939e-16;  // this step's roundings, both forms
    }
  }
  return binomial_inv_exact(r, u0, q, s, flip, n);
}
void multinomial_interval(HostMt &r, size_t K, unsigned N, const double *p, unsigned *n, double *btpeDraws,
                          std::vector<double> &scratch) {
  scratch.resize(4 * K);
  double *po = scratch.data(), *qf = po + K, *sf = po + 2 * K, *lq = po + 3 * K;
  double norm = 0.0, sum_p = 0.0;
  for (size_t k = 0; k < K; k++) norm += p[k];
  // the conditional probabilities do not depend on the draws: formed first
  for (size_t k = 0; k < K; k++) {
    const double pk = p[k] / (norm - sum_p);
    sum_p += p[k];
    const double pf = pk > 0.5 ? 1.0 - pk : pk;
    po[k] = pk;
    qf[k] = 1 - pf;
    sf[k] = pf / qf[k];
    lq[k] = log(qf[k]);
  }
  unsigned sum_n = 0;
  size_t k = 0;
  for (; k < K && sum_n < N; k++) {  // (past sum_n == N every binomial is 0 without a draw)
    const unsigned m = N - sum_n;
    unsigned v = 0;
    if (p[k] > 0.0) {
      const bool flip = po[k] > 0.5;
      const double pf = flip ? 1.0 - po[k] : po[k];
      if (m * pf < 14)
        v = binomial_inv_interval(r, qf[k], lq[k], sf[k], flip, m);
      else
        v = binomial(r, po[k], m, btpeDraws);
    }
    n[k] = v;
    sum_n += v;
  }
  for (; k < K; k++) n[k] = 0;
}

// the serial tail of calculateSquaredCVDifference :683-703 on one search
// point's exponentials: std::accumulate, normalisation, gsl_stats_mean and
// gsl_stats_sd_m with their `long double` running recurrences.
double cv2_tail(const double *E, size_t n, double target, double *w) {
  double sum = 0.0;
  for (size_t i = 0; i < n; i++) sum += E[i];
  for (size_t i = 0; i < n; i++) w[i] = E[i] / sum;
  long double lm = 0;
  for (size_t i = 0; i < n; i++) lm += (w[i] - lm) / (i + 1);
  const double mean = (double)lm;
  long double lv = 0;
  for (size_t i = 0; i < n; i++) {
    const long double delta = (w[i] - mean);
    lv += (delta * delta - lv) / (i + 1);
  }
  const double var = (double)lv;
  const double sd = sqrt(var * ((double)n / (double)(n - 1)));
  double c = (sd / mean) - target;
  c *= c;
  if (!std::isfinite(c)) return -DBL_MAX;  // 'Lowest'
  return c;
}

// cv2_tail of the search's stored minimum on a host worker thread: once the
// device's interval has decided that minimum against the 1e-12 tolerance,
// its exact value only feeds the reported coefficient of variation, so the
// x87 recurrences (~180 us at P = 8192) overlap the weights and the
// multinomial instead of preceding them
class HostTail {
 public:
  ~HostTail() {
    if (!th_.joinable()) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void start(const double *E, size_t n, double target) {
    if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    std::lock_guard<std::mutex> lk(mu_);
    E_ = E;
    n_ = n;
    target_ = target;
    w_.resize(n);
    busy_ = true;
    cv_.notify_all();
  }
  bool busy() {
    std::lock_guard<std::mutex> lk(mu_);
    return busy_;
  }
  double wait() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !busy_; });
    return y_;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return quit_ || busy_; });
      if (quit_) return;
      const double *E = E_;
      const size_t n = n_;
      const double t = target_;
      lk.unlock();
      const double y = cv2_tail(E, n, t, w_.data());
      lk.lock();
      y_ = y;
      busy_ = false;
      cv_.notify_all();
    }
  }
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  const double *E_ = nullptr;
  size_t n_ = 0;
  double target_ = 0, y_ = 0;
  bool busy_ = false, quit_ = false;
  std::vector<double> w_;
};

}  // namespace
}  // namespace kg

using namespace kg;

struct kg_tmcmc_s {
  // mTMCMC (cfg.version == 1): per-chain errors / gradients / proposal
  // covariances of leaders (L), candidates (C) and database entries (D) on
  // the host (kg_mtmcmc.hpp), the acceptance's proposal-density ratio and
  // its mode on the device
  bool mt = false;
  std::vector<double> mtLE, mtCE, mtDE, mtLG, mtCG, mtDG, mtLC, mtCC, mtDC, mtUpper, mtLower;
  std::vector<double> mtCand, mtLead, mtExtra;
  std::vector<unsigned char> mtMode;
  double *mtExtraDev = nullptr;
  unsigned char *mtModeDev = nullptr;
  double numCovarianceCorrections = 0;
  kg_tmcmc_cfg cfg;
  int N = 0, P = 0, ndist = 0;
  hipStream_t stream = nullptr;
  // device state
  double *leaders = nullptr, *leadLL = nullptr, *leadLP = nullptr, *cand = nullptr, *candLL = nullptr,
         *candLP = nullptr, *chainLen = nullptr, *mean = nullptr, *cov = nullptr, *chol = nullptr, *db = nullptr,
         *dbLL = nullptr, *dbLP = nullptr, *numSel = nullptr, *pmin = nullptr, *pmax = nullptr,
         *negLogWidth = nullptr, *Z = nullptr, *U = nullptr, *Uprior = nullptr, *E = nullptr, *w = nullptr;
  unsigned long long *uoff = nullptr;
  int2 *pairs = nullptr;
  bool wsumLds = false, exactMultinomial = false;  // KORALI_AMD_TM_MULTINOMIAL=exact
  std::vector<double> mnScratch;
  double *fA = nullptr, *fB = nullptr;  // term factors of the ordered sums (P x N + 2, or N x wr_pitch(P))    // upper-triangle (i, j), j >= i, row-major
  int *ustride = nullptr;
  int *vkind = nullptr;         // per variable: 0 Uniform prior, 1 Normal (pmin / pmax = mean / sd)
  double *priorNrm = nullptr;   // generation 1: the Normal priors' draws (P x N, host-made)
  std::vector<int> hkind;
  unsigned *src = nullptr;
  unsigned char *acc = nullptr, *pend = nullptr;
  TmDev *dev = nullptr;
  // chain steps (Max Chain Length > 1 / burn-in): per-chain schedule, the
  // generation's Uniform draws and its extra Multivariate normals
  ChainSched *sch = nullptr, *hSch = nullptr;
  double *Zx = nullptr, *dLen = nullptr, *hLenD = nullptr;
  size_t capU = 0, capZx = 0;
  // pinned host staging
  double *hE = nullptr, *hW = nullptr, *hNsel = nullptr;
  // the deferred exact minimum (HostTail): hEtail holds its exponentials
  // (swapped with hE), tailPending until kg_tmcmc_process_finalize collects it
  double *hEtail = nullptr;
  HostTail tail;
  bool tailPending = false, deferTail = true;
  // the next generation's first-step normals (P x N, one rank) formed on the
  // multivariate side stream during the host multinomial; prepare consumes
  bool zAhead = false, zAheadOn = true;  // KORALI_AMD_TM_NORMALS_AHEAD=0: off  // KORALI_AMD_TM_DEFER_TAIL=0: form it before going on
  double tailDeferred = 0;
  void *hCv = nullptr;                       // CvOut[CV_MAX_PTS + 1] (host)
  double2 *hRec = nullptr, *dRec = nullptr;  // 4 x CV_MAX_PTS+1 records, host-coherent (+ device alias)
  unsigned long long cvSeq = 0;
  void *cvPart = nullptr;                  // CvPart[(CV_MAX_PTS + 1) * CV_BLOCKS]
  bool exactSearch = false;                // KORALI_AMD_TMCMC_EXACT_SEARCH=1: every cv2 on the host
  bool hostSearch = false;                 // KORALI_AMD_TMCMC_HOST_SEARCH=1: simplex loop on the host (min_search)
  NmOut *dNm = nullptr, *hNm = nullptr;    // k_tm_nm_search result (device, pinned host)
  NmSync *nmSync = nullptr;                // its controller / worker hand-off records
  size_t nmRelaunches = 0, nmFallbacks = 0, nmEvals = 0, nmRounds = 0;
  double nmTime[6] = {0, 0, 0, 0, 0, 0};  // ms: controller wait, combine, logic; worker wait, evaluate, reduce
  size_t exactEvals = 0;
  unsigned *hSrc = nullptr;
  TmDev *hDev = nullptr;
  std::vector<double> wtmp;
  std::vector<unsigned> nsel;
  std::vector<double> perGenBurnIn;  // "Per Generation Burn In"
  std::vector<unsigned> hLen;        // host mirror of "Chain Lengths"
  int step = 0, maxSteps = 1;        // chain steps done / needed this generation
  size_t pendingCount = 0;           // own chains whose candidate awaits evaluation
  // chain sharding: this rank's started chains [ca, cb), the rows it owns of
  // candidates / leaders [ca, cbp) (the last rank also owns the chains that
  // were not started), its database entries [dba, dbb), its first extra
  // normal row zbase
  int rank = 0, world = 1;
  size_t ca = 0, cb = 0, cbp = 0, dba = 0, dbb = 0, zbase = 0;
  long long *xch = nullptr;  // "Shard Exchange" (sharded handles only)
  size_t xchWords = 0;
  bool rounds = false;               // this generation needs the general step schedule
  // per-distribution prior layout
  std::vector<int> distOf;           // variable -> distribution
  std::vector<size_t> distVars;      // variables per distribution
  std::vector<size_t> distOffset;    // offset of the distribution's draws in Uprior
  std::vector<int> distKind;         // 0 Uniform, 1 Normal
  // RNGs
  HostMt multinomialRng;
  MtStream multivariate, uniform;
  std::vector<MtStream *> priorRng;
  // scalars (TMCMC.config internal settings)
  double annealingExponent = 0, previousAnnealingExponent = 0, logEvidence = 0, coefficientOfVariation = 0,
         maxLoglikelihood = -INFINITY, chainCount = 0, acceptedSamplesCount = 0, proposalsAcceptanceRate = 0,
         selectionAcceptanceRate = 0, dbCount = 0, modelEvaluationCount = 0, minSearchIterations = 0,
         currentBurnIn = 0;
  double exactEvalsD = 0;
  double nmRelaunchesD = 0, nmEvalsD = 0, nmRoundsD = 0, nmFallbacksD = 0;  // diagnostics: device-search relaunches after host-exact values  // diagnostics: host-exact cv2 evaluations so far
  double btpeDraws = 0;    // diagnostics: multinomial binomials drawn by BTPE (n p >= 14)
  bool devPending = false;  // accepted count / maxLoglikelihood not yet read back
  // profiling
  bool profile = false;
  std::vector<std::tuple<std::string, hipEvent_t, hipEvent_t>> pending;
  std::map<std::string, std::pair<double, size_t>> prof;
};

namespace {

struct TmStage {
  kg_tmcmc_s *h;
  std::string name;
  hipEvent_t a = nullptr, b = nullptr;
  TmStage(kg_tmcmc_s *h_, const char *n) : h(h_), name(n) {
    if (h->profile) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, h->stream);
    }
  }
  ~TmStage() {
    if (h->profile) {
      (void)hipEventRecord(b, h->stream);
      h->pending.emplace_back(name, a, b);
    }
  }
};

struct HostClock {
  kg_tmcmc_s *h;
  const char *name;
  std::chrono::steady_clock::time_point t0;
  HostClock(kg_tmcmc_s *h_, const char *n) : h(h_), name(n), t0(std::chrono::steady_clock::now()) {}
  ~HostClock() {
    if (!h->profile) return;
    auto &p = h->prof[name];
    p.first += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    p.second += 1;
  }
};

template <typename T>
int tdalloc(T **p, size_t n) {
  if (n == 0) n = 1;
  KG_HIP(dev_alloc(p, n * sizeof(T)));
  if (zero_fill(*p, n * sizeof(T))) return 1;
  return 0;
}

void seed_state(uint64_t seed, unsigned char *out5000) {
  HostMt m;
  m.seed(seed);
  m.save(out5000);
}

inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

int tm_sync_dev(kg_tmcmc_s *h) {
  KG_HIP(hipStreamSynchronize(h->stream));
  if (h->devPending) {
    h->acceptedSamplesCount = (double)h->hDev->accepted;
    h->maxLoglikelihood = h->hDev->maxLoglikelihood;
    h->devPending = false;
  }
  return 0;
}

// calculateSquaredCVDifference at the annealing search's points.  The
// device returns cv2 for a whole batch of points from double-double sums; the
// reference's own value differs from that by its rounding (std::accumulate,
// the divisions by the sum, and the x87 `long double` gsl_stats recurrences),
// bounded below.  Every comparison the simplex makes is decided on these
// intervals when they are disjoint; otherwise both operands are evaluated
// exactly as the reference does (cv2_tail on the host) and compared.  Values
// that are stored (the minimum, the CoV) are always exact.  The simplex path
// and every stored value are therefore the reference's.
struct YV {
  double y = 0, eps = 0, x = 0;
  bool exact = false;
};

struct CvSearch {
  kg_tmcmc_s *h;
  double exponent, target;
  bool exactOnly = false;
  double xs[CV_MAX_PTS];
  int n = 0;
  double spareX = 0;  // the point whose E / CvOut sit in the spare slot
  bool spareValid = false;
  size_t exactEvals = 0;
  int launch(const double *pts, int npts, int slot0);
  int batch(const double *pts, int npts);
  int slot_of(double x, bool needOut);
  int exact(YV &v);
  int get(double x, YV &v);
  int lt(YV &a, YV &b, bool &r);
  int le(YV &a, YV &b, bool &r);
};

int CvSearch::launch(const double *pts, int npts, int slot0) {
  CvPoints cp{};
  for (int k = 0; k < npts; k++) cp.x[k] = pts[k];
  const unsigned long long seq = ++h->cvSeq;
  hipLaunchKernelGGL(k_tm_cv_part, dim3(CV_BLOCKS, npts), dim3(CV_TPB), 0, h->stream, h->P, h->dbLL, h->dev, exponent,
                     cp, (CvPart *)h->cvPart + slot0 * CV_BLOCKS);
  hipLaunchKernelGGL(k_tm_cv_final, dim3(npts), dim3(64), 0, h->stream, h->P, target,
                     (const CvPart *)h->cvPart + slot0 * CV_BLOCKS, h->dRec + 4 * slot0, seq);
  KG_HIP(hipGetLastError());
  // wait on the results themselves (zero-copy), not on the stream
  const auto t0 = std::chrono::steady_clock::now();
  CvOut *res = (CvOut *)h->hCv;
  for (int k = 0; k < npts; k++) {
    volatile const unsigned long long *r = (volatile const unsigned long long *)(h->hRec + 4 * (slot0 + k));
    unsigned spins = 0;
    for (;;) {
      bool ready = true;
      for (int f = 0; f < 4; f++)
        if (r[2 * f + 1] != seq) ready = false;
      if (ready) break;
      if (++spins % 4096 == 0) {
        const hipError_t e = hipStreamQuery(h->stream);
        if (e != hipSuccess && e != hipErrorNotReady) KG_HIP(e);
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
          set_error("kg_tmcmc: annealing-search kernel did not complete");
          return 1;
        }
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    CvOut &o = res[slot0 + k];
    double v[4];
    for (int f = 0; f < 4; f++) {
      const unsigned long long bits = r[2 * f];
      memcpy(&v[f], &bits, sizeof(double));
    }
    o.cv2 = v[0];
    o.cv = v[1];
    o.ratio = v[2];
    o.flag = v[3] != 0.0 ? 1 : 0;
  }
  return 0;
}

int CvSearch::batch(const double *pts, int npts) {
  n = std::min(npts, CV_MAX_PTS);
  for (int k = 0; k < n; k++) xs[k] = pts[k];
  return launch(pts, n, 0);
}

// slot holding x's exponentials and CvOut (evaluating x into the spare slot
// if it is not in the current batch); -1 on error
int CvSearch::slot_of(double x, bool) {
  for (int k = 0; k < n; k++)
    if (memcmp(&xs[k], &x, sizeof(double)) == 0) return k;
  if (spareValid && memcmp(&spareX, &x, sizeof(double)) == 0) return CV_MAX_PTS;
  if (launch(&x, 1, CV_MAX_PTS)) return -1;
  spareX = x;
  spareValid = true;
  return CV_MAX_PTS;
}

// the reference's value at v.x, bit for bit
int CvSearch::exact(YV &v) {
  if (v.exact) return 0;
  hipLaunchKernelGGL(k_tm_cv_exp, dim3(nblk(h->P, 256)), dim3(256), 0, h->stream, h->P, h->dbLL, h->dev, exponent,
                     v.x, h->E);
  KG_HIP(hipGetLastError());
  KG_HIP(hipMemcpyAsync(h->hE, h->E, (size_t)h->P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  v.y = cv2_tail(h->hE, h->P, target, h->wtmp.data());
  v.eps = 0;
  v.exact = true;
  exactEvals++;
  return 0;
}

int CvSearch::get(double x, YV &v) {
  const int slot = slot_of(x, true);
  if (slot < 0) return 1;
  const CvOut &o = ((const CvOut *)h->hCv)[slot];
  v.x = x;
  v.exact = false;
  if (exactOnly || o.flag) return exact(v);
  // |cv_ref - cv| <= dc: 1e-13 relative for the long
  // double recurrences and final roundings (worst case ~2^-64 (3P + 10
  // max/mean) + 4u ~ 2e-15 at P = 8192), 16u*max/mean for the rounding of
  // each w_i = E_i / sum (worst case u*max/mean), 4u^2/cv second order
  const double u = 1.1102230246251565e-16;
  const double cv = fabs(o.cv);
  const double dc = 1e-13 * cv + 16.0 * u * o.ratio + 4.0 * u * u / (cv > 1e-300 ? cv : 1e-300);
  v.y = o.cv2;
  v.eps = 2.0 * fabs(o.cv - target) * dc + dc * dc + 4.0 * u * fabs(o.cv2) + 1e-300;
  if (!std::isfinite(v.eps)) return exact(v);
  return 0;
}

int CvSearch::lt(YV &a, YV &b, bool &r) {
  if (!(a.exact && b.exact)) {
    if (a.y + a.eps < b.y - b.eps) {
      r = true;
      return 0;
    }
    if (a.y - a.eps > b.y + b.eps) {
      r = false;
      return 0;
    }
    if (exact(a) || exact(b)) return 1;
  }
  r = a.y < b.y;
  return 0;
}

int CvSearch::le(YV &a, YV &b, bool &r) {
  if (!(a.exact && b.exact)) {
    if (a.y + a.eps < b.y - b.eps) {
      r = true;
      return 0;
    }
    if (a.y - a.eps > b.y + b.eps) {
      r = false;
      return 0;
    }
    if (exact(a) || exact(b)) return 1;
  }
  r = a.y <= b.y;
  return 0;
}

double simplex_size(const double X[2]) {
  const double center = (X[0] + X[1]) / 2;
  double ss = 0.0;
  ss += fabs(X[0] - center);
  ss += fabs(X[1] - center);
  return ss / 2.0;
}

#define TRY(call) \
  do {            \
    if (call) return 1; \
  } while (0)

// minSearch :712-779: gsl_multimin_fminimizer_nmsimplex (v1) in one
// dimension, x0 = exponent, step 1e-8, size tolerance 1e-12, <= 1000
// iterations.  Each iteration's possible next points (reflection,
// expansion, both contractions, both contract-by-best outcomes) are
// evaluated on the device in one batch.  cv2 is never non-finite (the
// reference maps that to 'Lowest'), so its isfinite() tests always pass.
int min_search(kg_tmcmc_s *h, double exponent, double objCov, double &xmin, double &fmin, size_t &iters) {
  const size_t MaxIter = 1000;
  const double Tol = 1e-12, Step = 1e-8;
  CvSearch cv{h, exponent, objCov};
  cv.exactOnly = h->exactSearch;
  double X[2] = {exponent, exponent + Step};
  YV Y[2];
  TRY(cv.batch(X, 2));
  TRY(cv.get(X[0], Y[0]));
  TRY(cv.get(X[1], Y[1]));
  size_t lo = 0, iter = 0;
  bool r;
  int status;
  do {
    iter++;
    size_t hi = 0, s_hi = 0;
    lo = 0;
    TRY(cv.lt(Y[1], Y[0], r));
    if (r) {
      lo = 1;
    } else {
      TRY(cv.lt(Y[0], Y[1], r));
      if (r) hi = 1;  // s_hi stays 0
    }
    const double mp = X[1 - hi];
    const double xc = mp - (-1.0) * (mp - X[hi]);
    {
      double pts[CV_MAX_PTS];
      int np = 0;
      pts[np++] = xc;
      pts[np++] = mp - (-2.0) * (mp - X[hi]);
      pts[np++] = mp - 0.5 * (mp - X[hi]);
      pts[np++] = mp - 0.5 * (mp - xc);
      for (int var = 0; var < 2; var++) {
        double Xv[2] = {X[0], X[1]};
        if (var) Xv[hi] = xc;
        for (size_t i = 0; i < 2; i++)
          if (i != lo) pts[np++] = 0.5 * (Xv[i] + Xv[lo]);
      }
      TRY(cv.batch(pts, np));
    }
    YV v;
    TRY(cv.get(xc, v));
    TRY(cv.lt(v, Y[lo], r));
    if (r) {
      YV v2;
      const double xc2 = mp - (-2.0) * (mp - X[hi]);
      TRY(cv.get(xc2, v2));
      TRY(cv.lt(v2, Y[lo], r));
      if (r) {
        X[hi] = xc2;
        Y[hi] = v2;
      } else {
        X[hi] = xc;
        Y[hi] = v;
      }
    } else {
      TRY(cv.lt(Y[s_hi], v, r));
      if (r) {
        TRY(cv.le(v, Y[hi], r));
        if (r) {
          X[hi] = xc;
          Y[hi] = v;
        }
        YV v2;
        const double xc2 = mp - 0.5 * (mp - X[hi]);
        TRY(cv.get(xc2, v2));
        TRY(cv.le(v2, Y[hi], r));
        if (r) {
          X[hi] = xc2;
          Y[hi] = v2;
        } else {
          for (size_t i = 0; i < 2; i++)
            if (i != lo) {
              X[i] = 0.5 * (X[i] + X[lo]);
              TRY(cv.get(X[i], Y[i]));
            }
        }
      } else {
        X[hi] = xc;
        Y[hi] = v;
      }
    }
    // gsl_vector_min_index
    TRY(cv.lt(Y[1], Y[0], r));
    lo = r ? 1 : 0;
    status = (simplex_size(X) < Tol) ? 0 : 1;
  } while (status == 1 && iter < MaxIter);
  TRY(cv.exact(Y[lo]));
  fmin = 0;
  xmin = 0.0;
  if (Y[lo].y <= Tol) {
    fmin = Y[lo].y;
    xmin = X[lo];
  }
  if (xmin >= 1.0) {
    YV one;
    one.x = 1.0;
    TRY(cv.exact(one));
    fmin = one.y;
    xmin = 1.0;
  }
  iters = iter;
  h->exactEvals += cv.exactEvals;
  return 0;
}

// minSearch with the simplex loop on the device (k_tm_nm_search): one
// launch and one round trip per generation, plus one per comparison the
// intervals could not decide (the host forms those values exactly and
// relaunches).  Equal to min_search result for result.
int cv2_exact(kg_tmcmc_s *h, double exponent, double x, double &y);

int min_search_device(kg_tmcmc_s *h, double exponent, double objCov, double &xmin, double &fmin, size_t &iters) {
  const double Tol = 1e-12;
  const int P = h->P;
  if (h->tailPending) {  // (a previous finalize that failed before collecting it)
    (void)h->tail.wait();
    h->tailPending = false;
  }
  NmTab tab{};
  for (;;) {
    KG_HIP(hipMemsetAsync(h->nmSync, 0, sizeof(NmSync), h->stream));
    int Pa = P;
    const double *llp = h->dbLL;
    const TmDev *devp = h->dev;
    double rho = exponent, tgt = objCov;
    NmSync *syncp = h->nmSync;
    NmOut *outp = h->dNm;
    void *args[] = {&Pa, (void *)&llp, (void *)&devp, &rho, &tgt, &tab, &syncp, &outp};
    // the controller and its workers must be co-resident: launch_resident
    // checks the capacity (or fails rather than under-schedules) and, for
    // this per-generation 65-workgroup grid, launches it on the handle's
    // stream instead of ROCm's cooperative queue (kg_common.hpp)
    // (KORALI_AMD_NM_SYM=0: the controller form, two hand-offs per round)
    const char *symEnv = getenv("KORALI_AMD_NM_SYM");  // (read per search: tests switch it)
    const bool sym = !(symEnv && *symEnv == '0');
    // symmetric workgroups: about one log-likelihood per thread and point
    // (KORALI_AMD_NM_W = 16 | 32 | 64 forces a count)
    int nmw = 16;
    while (nmw < NM_W && (size_t)nmw * NM_TPB < (size_t)P) nmw *= 2;
    if (const char *e = getenv("KORALI_AMD_NM_W")) {
      const int v = atoi(e);
      if (v == 16 || v == 32 || v == 64) nmw = v;
    }
    const void *symFn = nmw == 16 ? (const void *)k_tm_nm_sym<16>
                        : nmw == 32 ? (const void *)k_tm_nm_sym<32> : (const void *)k_tm_nm_sym<64>;
    if (launch_resident(sym ? symFn : (const void *)k_tm_nm_search, dim3(sym ? nmw : 1 + NM_W),
                        dim3(NM_TPB), args, 0, h->stream,
                        /*prefer_plain=*/true) !=
        hipSuccess) {
      (void)hipGetLastError();
      h->nmFallbacks++;
      return min_search(h, exponent, objCov, xmin, fmin, iters);
    }
    hipLaunchKernelGGL(k_tm_nm_exp, dim3(nblk(P, 256), 2), dim3(256), 0, h->stream, P, h->dbLL, h->dev, exponent,
                       h->dNm, h->E);
    KG_HIP(hipGetLastError());
    KG_HIP(hipMemcpyAsync(h->hNm, h->dNm, sizeof(NmOut), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipMemcpyAsync(h->hE, h->E, (size_t)P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    const NmOut o = *h->hNm;
    h->nmEvals += o.evals;
    h->nmRounds += o.rounds;
    for (int q = 0; q < 3; q++) h->nmTime[q] += o.tc[q] * 1e-5, h->nmTime[3 + q] += o.tw[q] * 1e-5;  // ms
    if (o.status == 0) {
      double ylo = o.y[o.lo];
      bool deferred = false;
      if (!o.loExact) {
        // the interval decides ylo <= Tol unless it straddles Tol: above, the
        // minimum is rejected (fmin = 0, xmin = 0) and its exact value is never
        // used; below, xmin is known and the exact value (only fmin, for the
        // coefficient of variation) is formed on the host worker meanwhile
        const bool ok = !o.loBad && std::isfinite(o.loEps);
        if (ok && ylo - o.loEps > Tol) {
          ylo = INFINITY;
        } else if (ok && ylo + o.loEps <= Tol && o.X[o.lo] < 1.0 && h->deferTail) {
          std::swap(h->hE, h->hEtail);
          h->tail.start(h->hEtail, P, objCov);
          h->tailPending = true;
          h->exactEvals++;
          h->tailDeferred++;
          deferred = true;
        } else {
          ylo = cv2_tail(h->hE, P, objCov, h->wtmp.data());
          h->exactEvals++;
        }
      }
      fmin = 0;
      xmin = 0.0;
      if (deferred) {
        fmin = NAN;  // (collected by kg_tmcmc_process_finalize)
        xmin = o.X[o.lo];
      } else if (ylo <= Tol) {
        fmin = ylo;
        xmin = o.X[o.lo];
      }
      if (xmin >= 1.0) {
        double y1 = 0;
        if (cv2_exact(h, exponent, 1.0, y1)) return 1;
        fmin = y1;
        xmin = 1.0;
      }
      iters = (size_t)o.iters;
      return 0;
    }
    if (o.status != 1 || o.nneed < 1 || tab.n + o.nneed > NM_TAB) {  // the host search decides
      h->nmFallbacks++;
      return min_search(h, exponent, objCov, xmin, fmin, iters);
    }
    if (o.nneed > 1) KG_HIP(hipMemcpy(h->hE + P, h->E + P, (size_t)P * sizeof(double), hipMemcpyDeviceToHost));
    for (int j = 0; j < o.nneed; j++) {
      tab.x[tab.n] = o.need[j];
      tab.y[tab.n] = cv2_tail(h->hE + (size_t)j * P, P, objCov, h->wtmp.data());
      tab.n++;
      h->exactEvals++;
    }
    h->nmRelaunches++;
  }
}

// the reference's squared CoV difference at x, exactly
int cv2_exact(kg_tmcmc_s *h, double exponent, double x, double &y) {
  CvSearch cv{h, exponent, h->cfg.target_cov};
  YV v;
  v.x = x;
  if (cv.exact(v)) return 1;
  y = v.y;
  return 0;
}

int tm_initialize(kg_tmcmc_s *h) {
  // setInitialConfiguration :92-104
  h->annealingExponent = 0.0;
  h->logEvidence = 0.0;
  h->coefficientOfVariation = 0.0;
  h->maxLoglikelihood = -INFINITY;
  h->chainCount = h->P;
  hipLaunchKernelGGL(k_tm_fill, dim3(nblk(h->P, 256)), dim3(256), 0, h->stream, h->chainLen, (size_t)h->P, 1.0);
  KG_HIP(hipGetLastError());
  h->hLen.assign(h->P, 1u);
  return 0;
}

// setBurnIn :781-789
double tm_burn_in(const kg_tmcmc_s *h, size_t gen) {
  if (gen <= 1) return 0.0;
  if (gen - 2 < h->perGenBurnIn.size()) return h->perGenBurnIn[gen - 2];
  return h->cfg.default_burn_in;
}

template <typename T>
int tm_ensure(T **p, size_t &cap, size_t n) {
  if (n <= cap) return 0;
  if (*p) {
    KG_HIP(hipDeviceSynchronize());  // (a cached block is reused at once: no kernel may still use it)
    dev_release(*p);
  }
  *p = nullptr;
  cap = 0;
  if (tdalloc(p, n)) return 1;
  cap = n;
  return 0;
}

// The first step of every chain needs no Uniform index bookkeeping when all
// chains run exactly one step (Max Chain Length 1 selections, no burn-in):
// chain c draws Uniform c and writes database entry c.  Otherwise the step
// schedule (prefix sums in chain order) is built here and uploaded.
int tm_schedule(kg_tmcmc_s *h) {
  const size_t nc = (size_t)h->chainCount, B = (size_t)h->currentBurnIn, P = h->P;
  KG_CHECK(nc <= P && h->hLen.size() == P, "inconsistent Chain Count / Chain Lengths");
  h->rounds = !(B == 0 && nc == P);
  h->step = 0;
  h->maxSteps = 1;
  if (h->mt) {
    // mTMCMC (Max Chain Length 1): the WAITANY loop of runGeneration
    // (:112-144) re-evaluates every chain's unchanged candidate 1 + Burn In
    // times, and processCandidate runs once per chain after it (:146-155),
    // so a burn-in only repeats the evaluations (the last one is kept) and
    // the evaluation count; the step itself is the burn-in-free one
    KG_CHECK(nc == P, "mTMCMC: every chain runs one step (Max Chain Length 1)");
    h->rounds = false;
    h->maxSteps = 1 + (int)B;
  }
  if (!h->rounds) {
    h->dba = h->ca;
    h->dbb = h->cb;
    return 0;
  }
  size_t u = 0, z = 0, db = 0;
  for (size_t c = 0; c < nc; c++) {
    const size_t S = h->hLen[c] + B;
    KG_CHECK(S >= 1, "a started chain has zero steps (Chain Lengths 0 with Burn In 0)");
    h->hSch[c] = ChainSched{(unsigned)S, (unsigned)u, (unsigned)z, (unsigned)db};
    u += S;
    z += S - 1;
    db += h->hLen[c];
    h->maxSteps = std::max(h->maxSteps, (int)S);
  }
  KG_CHECK(db == P, "the chain lengths of the started chains must sum to the population size");
  KG_CHECK(u < (1ull << 32) && z < (1ull << 32), "chain schedule exceeds 32-bit indexing");
  auto at = [&](size_t c, int f) -> size_t {  // prefix sums at chain c (c == nc: totals)
    if (c < nc) return f == 0 ? h->hSch[c].z0 : h->hSch[c].db0;
    return f == 0 ? z : db;
  };
  h->zbase = at(h->ca, 0);
  const size_t zend = at(h->cb, 0);
  h->dba = at(h->ca, 1);
  h->dbb = at(h->cb, 1);
  KG_HIP(hipMemcpyAsync(h->sch, h->hSch, nc * sizeof(ChainSched), hipMemcpyHostToDevice, h->stream));
  // the generation's Uniform draws (one per step, chain-major) and its extra
  // candidates' normals (after prepareGeneration's P x N); a shard counts
  // the whole stream but materialises only its chains' rows
  if (tm_ensure(&h->U, h->capU, u)) return 1;
  if (h->uniform.uniforms(h->U, u, h->stream)) return 1;
  const size_t M = z * (size_t)h->N;
  if (M) {
    if (tm_ensure(&h->Zx, h->capZx, std::max<size_t>(1, (zend - h->zbase) * h->N))) return 1;
    TmStage st(h, "rng_polar");
    if (h->multivariate.polar_normals(h->Zx, M, h->N, nullptr, h->stream, h->zbase * h->N, zend * h->N)) return 1;
    if (h->multivariate.consume_normals(M, h->N, nullptr, h->stream)) return 1;
  }
  return 0;
}

// this rank's share of the started chains (contiguous, in chain order)
void tm_shard_ranges(kg_tmcmc_s *h) {
  const size_t nc = (size_t)h->chainCount, W = h->world, r = h->rank;
  h->ca = nc * r / W;
  h->cb = nc * (r + 1) / W;
  h->cbp = (r + 1 == W) ? (size_t)h->P : h->cb;
}

XchMap tm_xch_map(kg_tmcmc_s *h, size_t &total) {
  const size_t N = h->N, P = h->P;
  XchMap m{};
  unsigned long long off = 0;
  auto add = [&](double *p, size_t n, size_t lo, size_t hi) {
    m.s[m.ns++] = XchSec{p, off, n, lo, hi};
    off += n;
  };
  add(h->db, P * N, h->dba * N, h->dbb * N);
  add(h->dbLL, P, h->dba, h->dbb);
  add(h->dbLP, P, h->dba, h->dbb);
  add(h->leaders, P * N, h->ca * N, h->cbp * N);
  add(h->leadLL, P, h->ca, h->cbp);
  add(h->leadLP, P, h->ca, h->cbp);
  add(h->cand, P * N, h->ca * N, h->cbp * N);
  add(h->candLL, P, h->ca, h->cbp);
  add(h->candLP, P, h->ca, h->cbp);
  add(nullptr, (size_t)h->world, 0, 0);
  total = off;
  return m;
}

struct TmField {
  double *dev;   // device vector, or nullptr for a host scalar
  double *host;  // host scalar (or host array of n)
  size_t n;
};

bool tm_field(kg_tmcmc_s *h, const std::string &k, TmField &r) {
  const size_t N = h->N, P = h->P;
#define VEC(key, ptr, n)       \
  if (k == key) {              \
    r = {ptr, nullptr, n};     \
    return true;               \
  }
#define SCA(key, var)          \
  if (k == key) {              \
    r = {nullptr, &h->var, 1}; \
    return true;               \
  }
  VEC("Prior Minimum", h->pmin, N)
  VEC("Prior Maximum", h->pmax, N)
  VEC("Chain Leaders", h->leaders, P * N)
  VEC("Chain Leaders LogLikelihoods", h->leadLL, P)
  VEC("Chain Leaders LogPriors", h->leadLP, P)
  VEC("Chain Candidates", h->cand, P * N)
  VEC("Chain Candidates LogLikelihoods", h->candLL, P)
  VEC("Chain Candidates LogPriors", h->candLP, P)
  VEC("Chain Lengths", h->chainLen, P)
  VEC("Mean Theta", h->mean, N)
  VEC("Covariance Matrix", h->cov, N * N)
  VEC("Cholesky Factor", h->chol, N * N)
  VEC("Sample Database", h->db, P * N)
  VEC("Sample LogLikelihood Database", h->dbLL, P)
  VEC("Sample LogPrior Database", h->dbLP, P)
  VEC("Num Selections", h->numSel, P)
  if (k == "Shard Exchange" && h->xch) {
    r = {(double *)h->xch, nullptr, h->xchWords};
    return true;
  }
  SCA("Annealing Exponent", annealingExponent)
  SCA("Previous Annealing Exponent", previousAnnealingExponent)
  SCA("LogEvidence", logEvidence)
  SCA("Coefficient Of Variation", coefficientOfVariation)
  SCA("Max Loglikelihood", maxLoglikelihood)
  SCA("Chain Count", chainCount)
  SCA("Accepted Samples Count", acceptedSamplesCount)
  SCA("Proposals Acceptance Rate", proposalsAcceptanceRate)
  SCA("Selection Acceptance Rate", selectionAcceptanceRate)
  SCA("Database Entries", dbCount)
  SCA("Model Evaluation Count", modelEvaluationCount)
  SCA("Min Search Iterations", minSearchIterations)
  SCA("Current Burn In", currentBurnIn)
  SCA("Exact Search Evaluations", exactEvalsD)
  SCA("Deferred Search Evaluations", tailDeferred)
  SCA("Device Search Relaunches", nmRelaunchesD)
  SCA("Device Search Evaluations", nmEvalsD)
  SCA("Device Search Rounds", nmRoundsD)
  SCA("Num Covariance Corrections", numCovarianceCorrections)
  if (h->mt) {
    const std::pair<const char *, std::vector<double> *> mtf[] = {
        {"Chain Leaders Errors", &h->mtLE},         {"Chain Candidates Errors", &h->mtCE},
        {"Sample Error Database", &h->mtDE},        {"Chain Leaders Gradients", &h->mtLG},
        {"Chain Candidates Gradients", &h->mtCG},   {"Sample Gradient Database", &h->mtDG},
        {"Chain Leaders Covariance", &h->mtLC},     {"Chain Candidates Covariance", &h->mtCC},
        {"Sample Covariances Database", &h->mtDC},  {"Upper Extended Boundaries", &h->mtUpper},
        {"Lower Extended Boundaries", &h->mtLower}};
    for (const auto &f : mtf)
      if (k == f.first) {
        r = {nullptr, f.second->data(), f.second->size()};
        return true;
      }
  }
  if (k == "Device Search Phase Times") {  // ms: controller wait, combine, logic; worker wait, evaluate, reduce
    r = {nullptr, h->nmTime, 6};
    return true;
  }
  SCA("Device Search Fallbacks", nmFallbacksD)
  SCA("BTPE Binomial Draws", btpeDraws)
#undef VEC
#undef SCA
  return false;
}

}  // namespace

extern "C" {

int kg_tmcmc_create(const kg_tmcmc_cfg *cfg, kg_tmcmc_t *out) {
  KG_CHECK(cfg && out, "kg_tmcmc_create: null argument");
  KG_CHECK(cfg->variable_count >= 1 && cfg->variable_count <= (size_t)TM_MAX_N,
           "device TMCMC path supports 1..120 variables");
  KG_CHECK(cfg->population_size >= 2, "TMCMC 'Population Size' must be at least 2");
  KG_CHECK(cfg->max_chain_length >= 1.0 && cfg->max_chain_length == floor(cfg->max_chain_length),
           "Max Chain Length must be a positive integer");
  KG_CHECK(cfg->default_burn_in >= 0.0 && cfg->default_burn_in == floor(cfg->default_burn_in),
           "Burn In must be a non-negative integer");
  for (size_t k = 0; k < cfg->per_generation_burn_in_count; k++)
    KG_CHECK(cfg->per_generation_burn_in && cfg->per_generation_burn_in[k] >= 0.0 &&
                 cfg->per_generation_burn_in[k] == floor(cfg->per_generation_burn_in[k]),
             "Per Generation Burn In entries must be non-negative integers");
  KG_CHECK(cfg->covariance_scaling > 0.0, "Covariance Scaling must be larger 0.0");  // TMCMC.cpp.base:28
  KG_CHECK(cfg->prior_min && cfg->prior_max, "prior_min / prior_max are required");
  KG_CHECK(cfg->likelihood == KG_LIK_GAUSSIAN, "unknown builtin likelihood");
  KG_CHECK(cfg->version == 0 || cfg->version == 1, "TMCMC 'Version' must be TMCMC or mTMCMC");
  if (cfg->version == 1) {  // TMCMC.cpp.base:48-55
    KG_CHECK(cfg->max_chain_length == 1.0,
             "Current version of 'mTMCMC' supports only 'Max Chain Length' of 1 (BASIS).");
    KG_CHECK(cfg->step_size >= 0.0, "Step Size lower than 0.0");
    KG_CHECK(cfg->domain_extension_factor >= 0.0, "Domain Extension Factor lower than 0.0");
    KG_CHECK(cfg->shard_count <= 1, "mTMCMC runs unsharded");
    KG_CHECK(cfg->variable_count <= 128, "mTMCMC: at most 128 variables");
    for (size_t d = 0; cfg->prior_kind && d < cfg->variable_count; d++)  // TMCMC.cpp.base:76-77
      KG_CHECK(cfg->prior_kind[d] == 0, "Only 'Univariate/Uniform' priors allowed (mTMCMC)");
  }
  for (size_t d = 0; cfg->prior_kind && d < cfg->variable_count; d++) {
    KG_CHECK(cfg->prior_kind[d] >= KG_PRIOR_UNIFORM && cfg->prior_kind[d] <= KG_PRIOR_LOGNORMAL,
             "prior_kind entries must be KG_PRIOR_UNIFORM .. KG_PRIOR_LOGNORMAL");
    // the distributions' updateDistribution checks (exponential.cpp.base has none)
    KG_CHECK(cfg->prior_kind[d] == KG_PRIOR_UNIFORM || cfg->prior_kind[d] == KG_PRIOR_EXPONENTIAL ||
                 cfg->prior_max[d] > 0.0,
             "Incorrect scale parameter (Standard Deviation / Width / Scale / Sigma) of a prior distribution");
  }
  KG_HIP(hipSetDevice(cfg->device));
  upload_dd_tables();
  auto *h = new kg_tmcmc_s();
  h->cfg = *cfg;
  h->cfg.per_generation_burn_in = nullptr;
  h->world = cfg->shard_count > 1 ? cfg->shard_count : 1;
  h->rank = h->world > 1 ? cfg->shard_rank : 0;
  if (h->rank < 0 || h->rank >= h->world) {
    delete h;
    KG_CHECK(false, "shard_rank out of range");
  }
  if (cfg->per_generation_burn_in_count)
    h->perGenBurnIn.assign(cfg->per_generation_burn_in, cfg->per_generation_burn_in + cfg->per_generation_burn_in_count);
  double maxBurn = cfg->default_burn_in;
  for (double b : h->perGenBurnIn) maxBurn = std::max(maxBurn, b);
  const int N = (int)cfg->variable_count, P = (int)cfg->population_size;
  h->N = N;
  h->P = P;
  h->distOf.resize(N);
  int nd = (int)cfg->distribution_count;
  for (int d = 0; d < N; d++) {
    h->distOf[d] = cfg->prior_distribution ? cfg->prior_distribution[d] : d;
    if (h->distOf[d] < 0) {
      delete h;
      KG_CHECK(false, "negative prior distribution index");
    }
    nd = std::max(nd, h->distOf[d] + 1);
  }
  if (nd == 0) nd = N;
  h->ndist = nd;
  h->distVars.assign(nd, 0);
  h->distKind.assign(nd, -1);
  h->hkind.assign(N, 0);
  for (int d = 0; d < N; d++) {
    const int k = cfg->prior_kind ? cfg->prior_kind[d] : 0;
    h->hkind[d] = k;
    if (h->distKind[h->distOf[d]] >= 0 && h->distKind[h->distOf[d]] != k) {
      delete h;
      KG_CHECK(false, "variables sharing a prior distribution must share its kind");
    }
    h->distKind[h->distOf[d]] = k;
  }
  for (int &k : h->distKind) k = std::max(k, 0);
  std::vector<unsigned long long> uoff(N);
  std::vector<int> ustride(N);
  std::vector<size_t> rank(N);
  for (int d = 0; d < N; d++) rank[d] = h->distVars[h->distOf[d]]++;
  h->distOffset.assign(nd, 0);
  size_t acc = 0;
  for (int k = 0; k < nd; k++) {
    h->distOffset[k] = acc;
    acc += h->distVars[k] * (size_t)P;
  }
  for (int d = 0; d < N; d++) {
    uoff[d] = h->distOffset[h->distOf[d]] + rank[d];
    ustride[d] = (int)h->distVars[h->distOf[d]];
  }
  const size_t PN = (size_t)P * N;
  int rc = 0;
  rc |= tdalloc(&h->leaders, PN) | tdalloc(&h->leadLL, P) | tdalloc(&h->leadLP, P) | tdalloc(&h->cand, PN);
  rc |= tdalloc(&h->candLL, P) | tdalloc(&h->candLP, P) | tdalloc(&h->chainLen, P) | tdalloc(&h->mean, N);
  rc |= tdalloc(&h->cov, (size_t)N * N) | tdalloc(&h->chol, (size_t)N * N) | tdalloc(&h->db, PN);
  rc |= tdalloc(&h->dbLL, P) | tdalloc(&h->dbLP, P) | tdalloc(&h->numSel, P) | tdalloc(&h->pmin, N);
  rc |= tdalloc(&h->pmax, N) | tdalloc(&h->negLogWidth, N) | tdalloc(&h->Z, PN) | tdalloc(&h->U, P);
  h->capU = P;
  rc |= tdalloc(&h->Uprior, PN) | tdalloc(&h->E, (size_t)(CV_MAX_PTS + 1) * P) | tdalloc(&h->w, P);
  rc |= tdalloc(&h->uoff, N) | tdalloc(&h->ustride, N) | tdalloc(&h->src, P) | tdalloc(&h->acc, P);
  rc |= tdalloc(&h->vkind, N);
  for (int k : h->hkind)
    if (k) {
      rc |= tdalloc(&h->priorNrm, PN);
      break;
    }
  rc |= tdalloc(&h->pend, P) | tdalloc(&h->sch, P) | tdalloc(&h->dLen, P);
  h->xchWords = 3 * (PN + 2 * (size_t)P) + h->world;
  if (cfg->shard_count >= 1) rc |= tdalloc(&h->xch, h->xchWords);  // explicitly sharded (even one rank)
  rc |= tdalloc(&h->dev, 1) | tdalloc(&h->pairs, N * (N + 1) / 2);
  {  // (LDS form: P x N + 2; row form: N x wr_pitch(P))
    const size_t nf = std::max(PN + 2, (size_t)N * wr_pitch(P));
    rc |= tdalloc(&h->fA, nf) | tdalloc(&h->fB, nf);
  }
  rc |= tdalloc((char **)&h->cvPart, (CV_MAX_PTS + 1) * CV_BLOCKS * sizeof(CvPart));
  rc |= tdalloc((char **)&h->dNm, sizeof(NmOut)) | tdalloc((char **)&h->nmSync, sizeof(NmSync));
  if (rc) {
    delete h;
    return 1;
  }
  KG_HIP(host_alloc(&h->hE, 2 * (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hEtail, 2 * (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hNm, sizeof(NmOut), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hW, (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hNsel, (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hSrc, (size_t)P * sizeof(unsigned), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hSch, (size_t)P * sizeof(ChainSched), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hLenD, (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hDev, sizeof(TmDev), hipHostMallocDefault));
  KG_HIP(host_alloc(&h->hCv, (CV_MAX_PTS + 1) * sizeof(CvOut), hipHostMallocDefault));
  KG_HIP(host_alloc((void **)&h->hRec, 4 * (CV_MAX_PTS + 1) * sizeof(double2),
                       hipHostMallocCoherent | hipHostMallocMapped));
  memset(h->hRec, 0, 4 * (CV_MAX_PTS + 1) * sizeof(double2));
  KG_HIP(hipHostGetDevicePointer((void **)&h->dRec, h->hRec, 0));
  {
    const char *ev = getenv("KORALI_AMD_TMCMC_EXACT_SEARCH");
    h->exactSearch = ev && ev[0] == '1';
    const char *hs = getenv("KORALI_AMD_TMCMC_HOST_SEARCH");
    h->hostSearch = hs && hs[0] == '1';
    const char *ws = getenv("KORALI_AMD_TM_WSUM");  // "lds": the round-2 LDS-tile sums
    h->wsumLds = ws && strcmp(ws, "lds") == 0;
    const char *dt = getenv("KORALI_AMD_TM_DEFER_TAIL");
    h->deferTail = !(dt && dt[0] == '0');
    const char *em = getenv("KORALI_AMD_TM_MULTINOMIAL");
    h->exactMultinomial = em && strcmp(em, "exact") == 0;
    const char *za = getenv("KORALI_AMD_TM_NORMALS_AHEAD");
    h->zAheadOn = !(za && za[0] == '0');
  }
  h->wtmp.resize(P);
  h->nsel.resize(P);
  KG_HIP(stream_acquire(&h->stream));
  KG_HIP(hipMemcpy(h->pmin, cfg->prior_min, N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->pmax, cfg->prior_max, N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->uoff, uoff.data(), N * sizeof(unsigned long long), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->ustride, ustride.data(), N * sizeof(int), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->vkind, h->hkind.data(), N * sizeof(int), hipMemcpyHostToDevice));
  {
    std::vector<int2> pr;
    for (int i = 0; i < N; i++)
      for (int j = i; j < N; j++) pr.push_back(make_int2(i, j));
    KG_HIP(hipMemcpy(h->pairs, pr.data(), pr.size() * sizeof(int2), hipMemcpyHostToDevice));
  }
  {
    KG_HIP(allow_dynamic_lds((const void *)k_tm_wsum<false>, (int)ws_lds_bytes(N, false)));
    KG_HIP(allow_dynamic_lds((const void *)k_tm_wsum<true>, (int)ws_lds_bytes(N, true)));
    const size_t lbytes = (size_t)N * (N + 1) * sizeof(double) + (size_t)std::max(1, 256 / N) * N * sizeof(double);
    if (lbytes > 64 * 1024) {
      KG_HIP(allow_dynamic_lds((const void *)k_tm_draw<false>, (int)lbytes));
      KG_HIP(allow_dynamic_lds((const void *)k_tm_draw<true>, (int)lbytes));
      KG_HIP(allow_dynamic_lds((const void *)k_tm_cholesky, (int)((size_t)N * (N + 1) * sizeof(double))));
    }

  }
  hipLaunchKernelGGL(k_tm_neglogwidth, dim3(nblk(N, 64)), dim3(64), 0, h->stream, N, h->pmin, h->pmax, h->vkind,
                     h->negLogWidth);
  KG_HIP(hipGetLastError());
  // per generation: P x N normals for prepareGeneration and up to
  // P (1 + burn-in) x N for the chains' later steps; one Uniform per step
  const size_t steps = (size_t)P * (size_t)(1.0 + maxBurn);
  if (h->multivariate.init(3 * h->multivariate.words_for_normals(PN + steps * N) + 4096) ||
      h->uniform.init(4 * steps + 4096)) {
    delete h;
    return 1;
  }
  unsigned char st[5000];
  seed_state(cfg->multivariate_seed, st);
  if (h->multivariate.import_gsl(st, h->stream)) return 1;
  seed_state(cfg->uniform_seed, st);
  if (h->uniform.import_gsl(st, h->stream)) return 1;
  h->multinomialRng.seed(cfg->multinomial_seed);
  h->priorRng.resize(nd);
  for (int k = 0; k < nd; k++) {
    h->priorRng[k] = new MtStream();
    if (h->priorRng[k]->init((h->distKind[k] ? 1 : 2 * h->distVars[k] * (size_t)P) + 4096)) return 1;
    seed_state(cfg->prior_seeds ? cfg->prior_seeds[k] : 0, st);
    if (h->priorRng[k]->import_gsl(st, h->stream)) return 1;
  }
  h->chainCount = P;
  h->hLen.assign(P, 1u);
  if (cfg->version == 1) {
    // TMCMC.cpp.base:57-82: errors start at -1; extended prior boundaries
    h->mt = true;
    const size_t PN = (size_t)P * N, PNN = PN * N;
    h->mtLE.assign(P, -1.0);
    h->mtCE.assign(P, -1.0);
    h->mtDE.assign(P, -1.0);
    h->mtLG.assign(PN, 0.0);
    h->mtCG.assign(PN, 0.0);
    h->mtDG.assign(PN, 0.0);
    h->mtLC.assign(PNN, 0.0);
    h->mtCC.assign(PNN, 0.0);
    h->mtDC.assign(PNN, 0.0);
    h->mtUpper.resize(N);
    h->mtLower.resize(N);
    for (int d = 0; d < N; d++) {
      const double width = cfg->prior_max[d] - cfg->prior_min[d];
      h->mtUpper[d] = cfg->prior_max[d] + width * cfg->domain_extension_factor;
      h->mtLower[d] = cfg->prior_min[d] - width * cfg->domain_extension_factor;
    }
    h->mtCand.assign(PN, 0.0);
    h->mtLead.assign(PN, 0.0);
    h->mtExtra.assign(P, 0.0);
    h->mtMode.assign(P, 0);
    if (tdalloc(&h->mtExtraDev, P) || tdalloc(&h->mtModeDev, P)) return 1;
  }
  *out = h;
  return 0;
}

int kg_tmcmc_destroy(kg_tmcmc_t h) {
  if (!h) return 0;
  (void)hipStreamSynchronize(h->stream);
  if (h->tailPending) (void)h->tail.wait();

  for (void *p : {(void *)h->leaders, (void *)h->leadLL, (void *)h->leadLP, (void *)h->cand, (void *)h->candLL,
                  (void *)h->candLP, (void *)h->chainLen, (void *)h->mean, (void *)h->cov, (void *)h->chol,
                  (void *)h->db, (void *)h->dbLL, (void *)h->dbLP, (void *)h->numSel, (void *)h->pmin,
                  (void *)h->pmax, (void *)h->negLogWidth, (void *)h->Z, (void *)h->U, (void *)h->Uprior,
                  (void *)h->E, (void *)h->w, (void *)h->uoff, (void *)h->ustride, (void *)h->src, (void *)h->acc,
                  (void *)h->dev, h->cvPart, (void *)h->pairs, (void *)h->pend, (void *)h->sch, (void *)h->Zx,
                  (void *)h->dLen, (void *)h->xch, (void *)h->vkind, (void *)h->priorNrm,
                  (void *)h->fA, (void *)h->fB, (void *)h->dNm, (void *)h->nmSync, (void *)h->mtExtraDev,
                  (void *)h->mtModeDev})
    if (p) dev_release(p);
  for (void *p : {(void *)h->hE, (void *)h->hEtail, (void *)h->hW, (void *)h->hNsel, (void *)h->hSrc, (void *)h->hDev, h->hCv, (void *)h->hRec,
                  (void *)h->hSch, (void *)h->hLenD, (void *)h->hNm})
    if (p) host_release(p);
  for (auto *r : h->priorRng) delete r;
  for (auto &t : h->pending) {
    (void)hipEventDestroy(std::get<1>(t));
    (void)hipEventDestroy(std::get<2>(t));
  }
  stream_release(h->stream);
  delete h;
  return 0;
}

// generateCandidate, mTMCMC branch (TMCMC.cpp.base:567-608), every chain in
// order: a leader without errors proposes from N(leader, step Sigma_l) plus
// the drift (step/2) Sigma_l g_l (a failed Cholesky draws nothing and keeps
// the old candidate); a leader with errors from N(leader, Sigma).  The
// Multivariate normals are drawn on the device (exact stream positions:
// N per drawing chain), the N x N per-chain algebra on the host.
static int tm_mt_candidates(kg_tmcmc_s *h) {
  const int N = h->N, P = h->P;
  const size_t NN = (size_t)N * N, PN = (size_t)P * N;
  std::vector<double> Lg(NN), S((size_t)P * NN), z;
  std::vector<unsigned char> draws(P);
  KG_HIP(hipMemcpyAsync(Lg.data(), h->chol, NN * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipMemcpyAsync(h->mtLead.data(), h->leaders, PN * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipMemcpyAsync(h->mtCand.data(), h->cand, PN * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  size_t M = 0;
  for (int c = 0; c < P; c++) {
    if (h->mtLE[c] == 0.0) {
      double *Sc = S.data() + (size_t)c * NN;
      for (size_t k = 0; k < NN; k++) Sc[k] = h->mtLC[(size_t)c * NN + k] * h->cfg.step_size;
      draws[c] = mt::cholesky(N, Sc) ? 1 : 0;
    } else {
      draws[c] = 1;
    }
    if (draws[c]) M += N;
  }
  if (M) {
    TmStage st(h, "rng_polar");
    if (h->multivariate.polar_normals(h->Z, M, N, nullptr, h->stream)) return 1;
    if (h->multivariate.consume_normals(M, N, nullptr, h->stream)) return 1;
    if (h->multivariate.prefetch(PN, h->stream)) return 1;
    z.resize(M);
    KG_HIP(hipMemcpyAsync(z.data(), h->Z, M * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  }
  KG_HIP(hipStreamSynchronize(h->stream));
  TmStage st(h, "draw");
  size_t k = 0;
  const double alpha = 0.5 * h->cfg.step_size;
  for (int c = 0; c < P; c++) {
    double *x = h->mtCand.data() + (size_t)c * N;
    const double *lead = h->mtLead.data() + (size_t)c * N;
    if (h->mtLE[c] == 0.0) {
      if (!draws[c]) continue;
      for (int d = 0; d < N; d++) x[d] = z[k + d];
      k += N;
      mt::dtrmv_lower(N, S.data() + (size_t)c * NN, x);
      for (int d = 0; d < N; d++) x[d] = x[d] + lead[d];  // gsl_vector_add(result, mu = leader)
      mt::dgemv_add(N, alpha, h->mtLC.data() + (size_t)c * NN, h->mtLG.data() + (size_t)c * N, x);
    } else {
      for (int d = 0; d < N; d++) x[d] = z[k + d];
      k += N;
      mt::dtrmv_lower(N, Lg.data(), x);
      for (int d = 0; d < N; d++) x[d] = x[d] + lead[d];
    }
  }
  KG_HIP(hipMemcpyAsync(h->cand, h->mtCand.data(), PN * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// generation 1, non-Uniform priors (getRandomNumber of Normal = mean +
// gsl_ran_gaussian(sd), normal.cpp.base:30-33; Exponential location +
// gsl_ran_exponential(mean); Laplace mean + gsl_ran_laplace(width); Cauchy
// location + gsl_ran_cauchy(scale); LogNormal gsl_ran_lognormal(mu, sigma) --
// GSL 2.6 randist): rejection loops make a draw's word count data-dependent,
// and a distribution shared by several variables interleaves them
// sample-major (TMCMC.cpp.base:215-221), so the P x (its variables) draws
// run on the host from the distribution's exported generator, which then
// continues from where they left it.  Once per run.
static int tm_normal_priors(kg_tmcmc_t h) {
  const int N = h->N, P = h->P;
  std::vector<double> mean(N), sd(N), out((size_t)P * N, 0.0);
  KG_HIP(hipMemcpyAsync(mean.data(), h->pmin, N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipMemcpyAsync(sd.data(), h->pmax, N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  unsigned char st[5000];
  for (int k = 0; k < h->ndist; k++) {
    if (!h->distKind[k] || !h->distVars[k]) continue;
    HostMt g;
    if (h->priorRng[k]->export_gsl(st, h->stream) || g.load(st)) return 1;
    auto upos = [&]() {
      double u;
      do u = g.uniform();
      while (u == 0.0);
      return u;
    };
    const double pi = 3.14159265358979323846;
    for (int i = 0; i < P; i++)
      for (int d = 0; d < N; d++) {
        if (h->distOf[d] != k) continue;
        const double a = mean[d], b = sd[d];
        double v = 0.0;
        switch (h->distKind[k]) {
          case KG_PRIOR_NORMAL: {
            double x, y, r2;
            do {
              x = -1 + 2 * upos();
              y = -1 + 2 * upos();
              r2 = x * x + y * y;
            } while (r2 > 1.0 || r2 == 0);
            v = a + b * y * std::sqrt(-2.0 * host_log_cr(r2) / r2);
            break;
          }
          case KG_PRIOR_EXPONENTIAL: {
            const double u = g.uniform();
            v = a + -b * std::log1p(-u);
            break;
          }
          case KG_PRIOR_LAPLACE: {
            double u;
            do u = 2 * g.uniform() - 1.0;
            while (u == 0.0);
            v = a + (u < 0 ? b * host_log_cr(-u) : -b * host_log_cr(u));
            break;
          }
          case KG_PRIOR_CAUCHY: {
            double u;
            do u = g.uniform();
            while (u == 0.5);
            v = a + b * std::tan(pi * u);
            break;
          }
          case KG_PRIOR_LOGNORMAL: {
            double x, y, r2;
            do {
              x = -1 + 2 * g.uniform();
              y = -1 + 2 * g.uniform();
              r2 = x * x + y * y;
            } while (r2 > 1.0 || r2 == 0);
            const double normal = x * std::sqrt(-2.0 * host_log_cr(r2) / r2);
            v = std::exp(b * normal + a);
            break;
          }
        }
        out[(size_t)i * N + d] = v;
      }
    g.save(st);
    if (h->priorRng[k]->import_gsl(st, h->stream)) return 1;
  }
  KG_HIP(hipMemcpyAsync(h->priorNrm, out.data(), out.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_prepare(kg_tmcmc_t h, size_t generation) {
  const int N = h->N, P = h->P;
  const size_t PN = (size_t)P * N;
  if (h->zAhead) {
    // the normals formed ahead (during the last multinomial) are complete
    // before this generation's producer is queued behind them on the side
    // stream; a new run (generation 1) does not use them
    if (h->multivariate.join(h->stream)) return 1;
    if (generation == 1) h->zAhead = false;
  }
  if (generation == 1 && tm_initialize(h)) return 1;
  if (tm_sync_dev(h)) return 1;
  // prepareGeneration :161-170
  h->currentBurnIn = tm_burn_in(h, generation);
  tm_shard_ranges(h);

  h->acceptedSamplesCount = 0;
  h->maxLoglikelihood = -INFINITY;
  h->dbCount = 0;
  KG_HIP(hipMemsetAsync(h->dev, 0, sizeof(TmDev), h->stream));
  if (generation > 1 && h->multivariate.prefetch(PN, h->stream)) return 1;
  {
    TmStage st(h, "cholesky");
    hipLaunchKernelGGL(k_tm_cholesky, dim3(1), dim3(256), (size_t)N * (N + 1) * sizeof(double), h->stream, N, h->cov,
                       h->chol, h->dev);
    KG_HIP(hipGetLastError());
  }
  if (h->mt) {
    // prepareGeneration :174-200: this generation's candidates start
    // without errors (generation 1: -1), the leaders' proposals and
    // gradients re-annealed
    const double fc = h->previousAnnealingExponent / h->annealingExponent;
    const double fg = h->annealingExponent / h->previousAnnealingExponent;
    h->numCovarianceCorrections = 0;
    for (int c = 0; c < P; c++) h->mtCE[c] = generation > 1 ? 0.0 : -1.0;
    for (double &v : h->mtLC) v *= fc;
    for (double &v : h->mtLG) v *= fg;
    std::fill(h->mtMode.begin(), h->mtMode.end(), (unsigned char)0);
    KG_HIP(hipMemsetAsync(h->mtModeDev, 0, (size_t)P, h->stream));
  }
  if (generation == 1) {
    TmStage st(h, "prior_draw");
    if (h->priorNrm && tm_normal_priors(h)) return 1;
    for (int k = 0; k < h->ndist; k++)
      if (h->distVars[k] && !h->distKind[k] &&
          h->priorRng[k]->uniforms(h->Uprior + h->distOffset[k], h->distVars[k] * (size_t)P, h->stream))
        return 1;
    hipLaunchKernelGGL(k_tm_prior, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, h->Uprior, h->uoff, h->ustride,
                       h->pmin, h->pmax, h->vkind, h->priorNrm, h->cand);
    KG_HIP(hipGetLastError());
  } else if (h->mt) {
    if (tm_mt_candidates(h)) return 1;
  } else {
    {
      TmStage st(h, "rng_polar");
      if (h->zAhead && h->world == 1) {  // formed during the last generation's multinomial (joined above)
      } else if (h->multivariate.polar_normals(h->Z, PN, N, nullptr, h->stream, h->ca * N, h->cbp * N)) {
        return 1;
      }
      h->zAhead = false;
      if (h->multivariate.consume_normals(PN, N, nullptr, h->stream)) return 1;
      // the next generation's words are produced on the side stream while
      // this generation's search runs on the host
      if (h->multivariate.prefetch(PN, h->stream)) return 1;
    }
    TmStage st(h, "draw");
    const int CB = std::max(1, 256 / N);
    const size_t lbytes = (size_t)N * (N + 1) * sizeof(double) + (size_t)CB * N * sizeof(double);
    if (h->cbp > h->ca)
      hipLaunchKernelGGL(k_tm_draw<false>, dim3(nblk(h->cbp - h->ca, CB)), dim3(256), lbytes, h->stream, N, (int)h->ca,
                         (int)h->cbp, h->Z, h->chol, h->leaders, h->cand, (const ChainSched *)nullptr, 0, 0u,
                         (unsigned char *)nullptr);
    KG_HIP(hipGetLastError());
  }
  // started chains (c < Chain Count) begin with their prepared candidate
  // (:114-130); _modelEvaluationCount++ per started sample (:127)
  hipLaunchKernelGGL(k_tm_pend_init, dim3(nblk(P, 256)), dim3(256), 0, h->stream, P, (int)h->ca, (int)h->cb,
                     h->pend);
  KG_HIP(hipGetLastError());
  h->pendingCount = h->cb - h->ca;
  h->modelEvaluationCount += h->chainCount;
  return tm_schedule(h);
}

int kg_tmcmc_evaluate(kg_tmcmc_t h) {
  TmStage st(h, "evaluate");
  hipLaunchKernelGGL(k_tm_evaluate, dim3(nblk(h->P, 128)), dim3(128), 0, h->stream, h->N, h->P, h->cfg.likelihood,
                     h->cand, h->negLogWidth, h->pmin, h->pmax, h->vkind, h->candLL, h->candLP, h->pend);
  KG_HIP(hipGetLastError());
  return 0;
}

int kg_tmcmc_evaluate_prior(kg_tmcmc_t h) {
  TmStage st(h, "evaluate");
  hipLaunchKernelGGL(k_tm_evaluate, dim3(nblk(h->P, 128)), dim3(128), 0, h->stream, h->N, h->P, -1, h->cand,
                     h->negLogWidth, h->pmin, h->pmax, h->vkind, h->candLL, h->candLP, h->pend);
  KG_HIP(hipGetLastError());
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_get_pending(kg_tmcmc_t h, unsigned char *mask) {
  KG_HIP(hipMemcpyAsync(mask, h->pend, (size_t)h->P, hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_get_candidates(kg_tmcmc_t h, double *X, size_t ld) {
  const size_t N = h->N;
  if (ld == 0) ld = N;
  KG_HIP(hipMemcpy2DAsync(X, ld * sizeof(double), h->cand, N * sizeof(double), N * sizeof(double), h->P,
                          hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_set_evaluations(kg_tmcmc_t h, const double *log_prior, const double *log_likelihood) {
  const size_t P = h->P;
  KG_HIP(hipMemcpyAsync(h->E, log_prior, P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->E + P, log_likelihood, P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(k_tm_set_pending, dim3(nblk(P, 256)), dim3(256), 0, h->stream, (int)P, h->pend, h->E, h->E + P,
                     h->candLP, h->candLL);
  KG_HIP(hipGetLastError());
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_set_gradients(kg_tmcmc_t h, const double *grad, const double *fisher) {
  KG_CHECK(h->mt, "kg_tmcmc_set_gradients: the handle is not mTMCMC");
  KG_CHECK(grad && fisher, "kg_tmcmc_set_gradients: null argument");
  const int N = h->N, P = h->P;
  const size_t NN = (size_t)N * N;
  std::vector<double> lp(P), ll(P);
  KG_HIP(hipMemcpyAsync(lp.data(), h->candLP, P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipMemcpyAsync(ll.data(), h->candLL, P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  const double rho = h->annealingExponent, chi2inv = mt::chi2inv_068(N);
  const int chains = (int)h->chainCount;
  // calculateGradients :383-403
  for (int c = 0; c < chains; c++) {
    if (!(std::isfinite(lp[c]) && std::isfinite(ll[c]))) continue;
    for (int d = 0; d < N; d++) h->mtCG[(size_t)c * N + d] = grad[(size_t)c * N + d] * rho;
  }
  // calculateProposals :405-558
  std::vector<double> F(NN), Finv(NN), E(NN), ev(N), c0(N), c1(N);
  std::vector<size_t> perm(N);
  for (int c = 0; c < chains; c++) {
    if (!(std::isfinite(lp[c]) && std::isfinite(ll[c]))) continue;
    const double *cand = h->mtCand.data() + (size_t)c * N;
    double *CC = h->mtCC.data() + (size_t)c * NN;
    for (size_t k = 0; k < NN; k++) CC[k] = 0.0;
    for (size_t k = 0; k < NN; k++) F[k] = fisher[(size_t)c * NN + k] * rho;
    mt::lu_decomp(N, F.data(), perm.data());
    mt::lu_invert(N, F.data(), perm.data(), Finv.data());
    mt::symmv_unsorted(N, Finv.data(), ev.data(), E.data());
    bool correction = false;
    for (int d = 0; d < N; d++) {
      double scale = std::sqrt(ev[d] * chi2inv);
      const double before = scale;
      for (int e = 0; e < N; e++) c0[e] = cand[e] + (1.0 * scale) * E[(size_t)e * N + d];
      for (int e = 0; e < N; e++) c1[e] = cand[e] + (-1.0 * scale) * E[(size_t)e * N + d];
      for (int e = 0; e < N; e++) {
        const double up = h->mtUpper[e] - cand[e], lo = cand[e] - h->mtLower[e];
        const double inv = 1.0 / E[(size_t)e * N + d];
        double v;
        if (c0[e] - h->mtUpper[e] > 0.) {
          v = std::fabs(inv * up);
          scale = (v < scale) ? v : scale;
        }
        if (h->mtLower[e] - c0[e] > 0.) {
          v = std::fabs(inv * lo);
          scale = (v < scale) ? v : scale;
        }
        if (c1[e] - h->mtUpper[e] > 0.) {
          v = std::fabs(inv * up);
          scale = (v < scale) ? v : scale;
        }
        if (h->mtLower[e] - c1[e] > 0.) {
          v = std::fabs(inv * lo);
          scale = (v < scale) ? v : scale;
        }
      }
      ev[d] = scale * scale / chi2inv;
      if (before != scale) correction = true;
    }
    if (correction) h->numCovarianceCorrections += 1;
    for (int d = 0; d < N; d++) {
      const double f = std::sqrt(ev[d]);
      for (int e = 0; e < N; e++) E[(size_t)e * N + d] *= f;
    }
    for (int i = 0; i < N; i++)  // gslcblas dgemm NoTrans / Trans, alpha 1, beta 0
      for (int j = 0; j < N; j++) {
        double temp = 0.0;
        for (int q = 0; q < N; q++) temp += E[(size_t)i * N + q] * E[(size_t)j * N + q];
        CC[(size_t)i * N + j] = 0.0 + 1.0 * temp;
      }
  }
  // calculateAcceptanceProbability :634-673: the proposal log-density ratio
  // of chains whose leader and candidate have no errors
  std::vector<double> mL(N), mC(N), L(NN);
  const double alpha = 0.5 * h->cfg.step_size;
  for (int c = 0; c < chains; c++) {
    h->mtMode[c] = (h->mtLE[c] == 0.0 && h->mtCE[c] == 0.0) ? 1 : 0;
    h->mtExtra[c] = 0.0;
    if (!h->mtMode[c] || !(std::isfinite(lp[c]) && std::isfinite(ll[c]))) continue;
    const double *LC = h->mtLC.data() + (size_t)c * NN;
    const double *lead = h->mtLead.data() + (size_t)c * N, *cand = h->mtCand.data() + (size_t)c * N;
    for (int d = 0; d < N; d++) mL[d] = lead[d], mC[d] = cand[d];
    mt::dgemv_add(N, alpha, LC, h->mtLG.data() + (size_t)c * N, mL.data());
    mt::dgemv_add(N, alpha, LC, h->mtCG.data() + (size_t)c * N, mC.data());
    for (size_t k = 0; k < NN; k++) L[k] = LC[k] * h->cfg.step_size;
    (void)mt::cholesky(N, L.data());  // gsl_linalg_cholesky_decomp1; failure leaves the partial factor
    const double lpC = mt::mvn_log_pdf(N, cand, mL.data(), L.data());
    const double lpL = mt::mvn_log_pdf(N, lead, mC.data(), L.data());
    h->mtExtra[c] = lpL - lpC;
  }
  KG_HIP(hipMemcpyAsync(h->mtExtraDev, h->mtExtra.data(), P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->mtModeDev, h->mtMode.data(), (size_t)P, hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_advance(kg_tmcmc_t h, size_t generation, size_t *pending) {
  const int N = h->N, P = h->P;
  KG_CHECK(h->step < h->maxSteps, "kg_tmcmc_advance: every chain has finished this generation");
  const int s = ++h->step;
  if (!h->rounds && h->mt && s < h->maxSteps) {
    // mTMCMC burn-in: the same candidates are evaluated again (tm_schedule)
    h->pendingCount = (size_t)(h->cb - h->ca);
    h->modelEvaluationCount += (double)h->chainCount;  // the re-started samples (:127)
    if (pending) *pending = h->pendingCount;
    return 0;
  }
  if (!h->rounds) {
    // every chain runs one step: Uniform c, database entry c
    TmStage st(h, "accept");
    if (h->uniform.uniforms(h->U, P, h->stream)) return 1;
    const int a = (int)h->ca, b = (int)h->cb;
    if (b > a) {
      hipLaunchKernelGGL(k_tm_accept, dim3(nblk(b - a, 256)), dim3(256), 0, h->stream, a, b, generation == 1 ? 1 : 0,
                         h->annealingExponent, h->U, h->candLL, h->candLP, h->leadLL, h->leadLP, h->dbLL, h->dbLP,
                         h->acc, h->dev, h->mt ? h->mtExtraDev : (const double *)nullptr,
                         h->mt ? h->mtModeDev : (const unsigned char *)nullptr);
      hipLaunchKernelGGL(k_tm_copy_rows, dim3(nblk((size_t)(b - a) * N, 256)), dim3(256), 0, h->stream, N, a, b,
                         h->acc, h->cand, h->leaders, h->db);
      KG_HIP(hipGetLastError());
      if (h->mt) {
        // processCandidate :239-244 and updateDatabase :617-622 for the
        // errors / gradients / proposals (chain c's entry is c)
        const size_t NN = (size_t)N * N;
        std::vector<unsigned char> acc(P);
        KG_HIP(hipMemcpyAsync(acc.data(), h->acc, (size_t)P, hipMemcpyDeviceToHost, h->stream));
        KG_HIP(hipStreamSynchronize(h->stream));
        for (int c = a; c < b; c++) {
          if (acc[c]) {
            h->mtLE[c] = h->mtCE[c];
            std::copy_n(h->mtCG.begin() + (size_t)c * N, N, h->mtLG.begin() + (size_t)c * N);
            std::copy_n(h->mtCC.begin() + (size_t)c * NN, NN, h->mtLC.begin() + (size_t)c * NN);
          }
          h->mtDE[c] = h->mtLE[c];
          std::copy_n(h->mtLG.begin() + (size_t)c * N, N, h->mtDG.begin() + (size_t)c * N);
          std::copy_n(h->mtLC.begin() + (size_t)c * NN, NN, h->mtDC.begin() + (size_t)c * NN);
        }
      }
    }
    h->pendingCount = 0;
    h->step = h->maxSteps;
  } else {
    const int a = (int)h->ca, b = (int)h->cb, B = (int)h->currentBurnIn;
    if (b > a) {
      TmStage st(h, "accept");
      hipLaunchKernelGGL(k_tm_round_accept, dim3(nblk(b - a, 256)), dim3(256), 0, h->stream, a, b, s, B,
                         generation == 1 ? 1 : 0, h->annealingExponent, h->sch, h->U, h->candLL, h->candLP,
                         h->leadLL, h->leadLP, h->dbLL, h->dbLP, h->acc, h->dev);
      hipLaunchKernelGGL(k_tm_round_rows, dim3(nblk((size_t)(b - a) * N, 256)), dim3(256), 0, h->stream, N, a, b, s,
                         B, h->sch, h->acc, h->cand, h->leaders, h->db);
      KG_HIP(hipGetLastError());
    }
    size_t more = 0, mine = 0;
    for (int c = 0; c < (int)h->chainCount; c++)
      if ((int)h->hSch[c].S > s) {
        more++;
        mine += (c >= a && c < b);
      }
    if (mine) {
      TmStage st(h, "draw");
      const int CB = std::max(1, 256 / N);
      const size_t lbytes = (size_t)N * (N + 1) * sizeof(double) + (size_t)CB * N * sizeof(double);
      hipLaunchKernelGGL(k_tm_draw<true>, dim3(nblk(b - a, CB)), dim3(256), lbytes, h->stream, N, a, b, h->Zx,
                         h->chol, h->leaders, h->cand, h->sch, s, (unsigned)h->zbase, h->pend);
      KG_HIP(hipGetLastError());
    } else {
      hipLaunchKernelGGL(k_tm_pend_init, dim3(nblk(P, 256)), dim3(256), 0, h->stream, P, 0, 0, h->pend);
      KG_HIP(hipGetLastError());
    }
    h->pendingCount = mine;
    h->modelEvaluationCount += (double)more;  // the next step's started samples (:127)
    if (s >= h->maxSteps) h->step = h->maxSteps;
  }
  if (pending) *pending = h->pendingCount;
  return 0;
}

int kg_tmcmc_process_partial(kg_tmcmc_t h, size_t generation) {
  // the chains' remaining steps with the builtin likelihood
  while (h->step < h->maxSteps) {
    size_t more = 0;
    if (kg_tmcmc_advance(h, generation, &more)) return 1;
    if (more && kg_tmcmc_evaluate(h)) return 1;
  }
  if (h->xch) {
    size_t total = 0;
    const XchMap m = tm_xch_map(h, total);
    hipLaunchKernelGGL(k_tm_pack, dim3(nblk(total, 256)), dim3(256), 0, h->stream, m, (unsigned long long)total,
                       h->xch, h->dev, h->rank);
    KG_HIP(hipGetLastError());
  }
  return 0;
}

int kg_tmcmc_process_finalize(kg_tmcmc_t h, size_t generation) {
  (void)generation;
  const int N = h->N, P = h->P;
  const size_t PN = (size_t)P * N;
  KG_CHECK(h->step >= h->maxSteps, "kg_tmcmc_process_finalize: chains have steps left (call process_partial)");
  if (h->xch) {
    size_t total = 0;
    const XchMap m = tm_xch_map(h, total);
    hipLaunchKernelGGL(k_tm_unpack, dim3(nblk(total, 256)), dim3(256), 0, h->stream, m, (unsigned long long)total,
                       h->xch, h->dev, h->world);
    KG_HIP(hipGetLastError());
  }
  {
    TmStage st(h, "accept");
    hipLaunchKernelGGL(k_tm_max, dim3(1), dim3(1024), 0, h->stream, P, h->dbLL, 1.0, 0, &h->dev->llmaxCv,
                       &h->dev->maxLoglikelihood);
    KG_HIP(hipGetLastError());
    KG_HIP(hipMemcpyAsync(h->hDev, h->dev, sizeof(TmDev), hipMemcpyDeviceToHost, h->stream));
    h->devPending = true;
  }
  h->dbCount = P;
  // ---------------------------------------------- processGeneration :254-381
  double xmin = 0, fmin = 0;
  size_t iters = 0;
  {
    HostClock hc(h, "min_search");
    const bool onHost = h->exactSearch || h->hostSearch;
    if ((onHost ? min_search : min_search_device)(h, h->annealingExponent, h->cfg.target_cov, xmin, fmin, iters))
      return 1;
  }
  if (tm_sync_dev(h)) return 1;
  h->minSearchIterations = (double)iters;
  h->exactEvalsD = (double)h->exactEvals;
  h->nmRelaunchesD = (double)h->nmRelaunches;
  h->nmEvalsD = (double)h->nmEvals;
  h->nmRoundsD = (double)h->nmRounds;
  h->nmFallbacksD = (double)h->nmFallbacks;
  h->previousAnnealingExponent = h->annealingExponent;
  bool cvFromTail = false;
  {
    const double pe = h->previousAnnealingExponent;
    double y = 0;
    if (xmin > pe + h->cfg.max_annealing_exponent_update) {
      h->annealingExponent = pe + h->cfg.max_annealing_exponent_update;
      if (cv2_exact(h, pe, h->annealingExponent, y)) return 1;
      h->coefficientOfVariation = sqrt(y) + h->cfg.target_cov;
    } else if (xmin < 1.0 && xmin < pe + h->cfg.min_annealing_exponent_update) {
      h->annealingExponent = pe + h->cfg.min_annealing_exponent_update;
      if (cv2_exact(h, pe, h->annealingExponent, y)) return 1;
      h->coefficientOfVariation = sqrt(y) + h->cfg.target_cov;
    } else {
      h->annealingExponent = xmin;
      // (a deferred fmin: collected at the end of this function)
      if (!h->tailPending) h->coefficientOfVariation = sqrt(fmin) + h->cfg.target_cov;
      cvFromTail = h->tailPending;
    }
  }
  const double drho = h->annealingExponent - h->previousAnnealingExponent;
  {
    TmStage st(h, "weights");
    hipLaunchKernelGGL(k_tm_max, dim3(1), dim3(1024), 0, h->stream, P, h->dbLL, drho, 1, &h->dev->lwmax,
                       (double *)nullptr);
    hipLaunchKernelGGL(k_tm_lw_exp, dim3(nblk(P, 256)), dim3(256), 0, h->stream, P, h->dbLL, drho, h->dev, h->E);
    KG_HIP(hipGetLastError());
    // the next generation's first-step normals do not depend on the
    // selections (every one of the P chains draws N at its first step, one
    // rank): form them on the side stream while the host runs the
    // multinomial (the stream position only advances in prepare, so an
    // experiment that ends here is unaffected)
    h->zAhead = false;
    if (!h->mt && h->world == 1 && h->zAheadOn)
      h->zAhead = h->multivariate.polar_normals_ahead(h->Z, PN, N, h->stream) == 0;
    KG_HIP(hipMemcpyAsync(h->hE, h->E, (size_t)P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipMemcpyAsync(h->hDev, h->dev, sizeof(TmDev), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
  }
  size_t zeroCount = 0, leaderId = 0, total = 0;
  double sumw2 = 0.0;
  {
    HostClock hc(h, "multinomial");
    double *wt = h->hW;
    const double lwmax = h->hDev->lwmax;
    double sw = 0.0;
    for (int i = 0; i < P; i++) sw += h->hE[i];
    for (int i = 0; i < P; i++) wt[i] = h->hE[i] / sw;
    h->logEvidence += host_log_cr(sw) + lwmax - host_log_cr((double)P);
    if (h->exactMultinomial)
      multinomial(h->multinomialRng, P, (unsigned)P, wt, h->nsel.data(), &h->btpeDraws);
    else
      multinomial_interval(h->multinomialRng, P, (unsigned)P, wt, h->nsel.data(), &h->btpeDraws, h->mnScratch);
    for (int i = 0; i < P; i++) h->hNsel[i] = h->nsel[i];
    for (int i = 0; i < P; i++) wt[i] = wt[i] * h->nsel[i];
    sw = 0.0;
    for (int i = 0; i < P; i++) sw += wt[i];
    for (int i = 0; i < P; i++) wt[i] = wt[i] / sw;
    for (int i = 0; i < P; i++) sumw2 += wt[i] * wt[i];
    // leaders and chain lengths :329-360 ("uniform splitting" of selections
    // above Max Chain Length)
    const unsigned mcl = (unsigned)h->cfg.max_chain_length;
    for (int i = 0; i < P; i++) {
      unsigned n = h->nsel[i];
      if (n == 0) zeroCount++;
      while (n > 0) {
        const unsigned len = n > mcl ? mcl - (n % mcl != 0 ? 1u : 0u) : n;
        h->hSrc[leaderId] = (unsigned)i;
        h->hLenD[leaderId] = (double)len;
        h->hLen[leaderId] = len;
        n -= len;
        total += len;
        leaderId++;
      }
    }
    for (size_t j = leaderId; j < (size_t)P; j++) h->hLen[j] = 0;
    if (h->mt) {
      // :339-344 leaders take their entry's errors / gradients / proposals;
      // :362-372 then anneal them
      const size_t NN = (size_t)N * N;
      for (size_t j = 0; j < leaderId; j++) {
        const size_t i = h->hSrc[j];
        h->mtLE[j] = h->mtDE[i];
        std::copy_n(h->mtDG.begin() + i * N, N, h->mtLG.begin() + j * N);
        std::copy_n(h->mtDC.begin() + i * NN, NN, h->mtLC.begin() + j * NN);
      }
      if (h->previousAnnealingExponent > 0.0) {
        const double f = h->annealingExponent / h->previousAnnealingExponent;
        for (int i = 0; i < P; i++) {
          if (h->mtLE[i] != 0.0) continue;
          for (int d = 0; d < N; d++) h->mtLG[(size_t)i * N + d] *= f;
          for (size_t q = 0; q < NN; q++) h->mtLC[(size_t)i * NN + q] *= f;
        }
      }
    }
  }
  KG_CHECK(total == (size_t)P, "multinomial selections do not sum to the population size");
  KG_HIP(hipMemcpyAsync(h->w, h->hW, (size_t)P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->numSel, h->hNsel, (size_t)P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->src, h->hSrc, leaderId * sizeof(unsigned), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->dLen, h->hLenD, leaderId * sizeof(double), hipMemcpyHostToDevice, h->stream));
  {
    TmStage st(h, "mean_cov");
    const int npairs = N * (N + 1) / 2;
    if (h->wsumLds) {
      hipLaunchKernelGGL(k_tm_factors_mean, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, h->db, h->w, h->fA);
      hipLaunchKernelGGL(k_tm_wsum<false>, dim3(nblk(N, WS_LANES)), dim3(WS_TPB), ws_lds_bytes(N, false), h->stream,
                         N, P, h->fA, h->fA, h->pairs, N, 0.0, 1.0, h->mean);
      hipLaunchKernelGGL(k_tm_factors_cov, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, h->db, h->w, h->mean,
                         h->fA, h->fB);
      hipLaunchKernelGGL(k_tm_wsum<true>, dim3(nblk(npairs, WS_LANES)), dim3(WS_TPB), ws_lds_bytes(N, true),
                         h->stream, N, P, h->fA, h->fB, h->pairs, npairs, h->cfg.covariance_scaling, 1.0 - sumw2,
                         h->cov);
    } else {
      const int Pp = wr_pitch(P);
      const size_t NP = (size_t)N * Pp;
      hipLaunchKernelGGL(k_tm_factors_mean_t, dim3(nblk(NP, 256)), dim3(256), 0, h->stream, N, P, Pp, h->db, h->w,
                         h->fA);
      hipLaunchKernelGGL(k_tm_wsum_rows<false>, dim3((N + 3) / 4), dim3(64), 0, h->stream, N, Pp, h->fA, h->fA,
                         h->pairs, N, 0.0, 1.0, h->mean);
      hipLaunchKernelGGL(k_tm_factors_cov_t, dim3(nblk(NP, 256)), dim3(256), 0, h->stream, N, P, Pp, h->db, h->w,
                         h->mean, h->fA, h->fB);
      hipLaunchKernelGGL(k_tm_wsum_rows<true>, dim3((npairs + 3) / 4), dim3(64), 0, h->stream, N, Pp, h->fA, h->fB,
                         h->pairs, npairs, h->cfg.covariance_scaling, 1.0 - sumw2, h->cov);
    }
    KG_HIP(hipGetLastError());
  }
  {
    TmStage st(h, "expand");
    hipLaunchKernelGGL(k_tm_expand, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, (int)leaderId, h->src,
                       h->dLen, h->db, h->dbLL, h->dbLP, h->leaders, h->leadLL, h->leadLP, h->chainLen);
    KG_HIP(hipGetLastError());
  }
  h->proposalsAcceptanceRate = (1.0 * h->acceptedSamplesCount) / P;
  h->selectionAcceptanceRate = (1.0 * (P - zeroCount)) / P;
  h->chainCount = (double)leaderId;
  if (h->tailPending) {
    const double y = h->tail.wait();
    h->tailPending = false;
    if (cvFromTail) h->coefficientOfVariation = sqrt(y) + h->cfg.target_cov;
  }
  // the pinned staging buffers are reused by the next generation's search,
  // which synchronises the stream before touching them
  return 0;
}

int kg_tmcmc_process(kg_tmcmc_t h, size_t generation) {
  KG_CHECK(h->world == 1, "sharded TMCMC over several ranks: call process_partial, all-reduce 'Shard Exchange', process_finalize");
  if (kg_tmcmc_process_partial(h, generation)) return 1;
  return kg_tmcmc_process_finalize(h, generation);
}

int kg_tmcmc_generation(kg_tmcmc_t h, size_t generation) {
  KG_CHECK(!h->mt, "mTMCMC needs the problem's gradients: evaluate on the host (kg_tmcmc_set_evaluations, "
                   "kg_tmcmc_set_gradients)");
  if (kg_tmcmc_prepare(h, generation)) return 1;
  if (kg_tmcmc_evaluate(h)) return 1;
  return kg_tmcmc_process(h, generation);
}

int kg_tmcmc_synchronize(kg_tmcmc_t h) { return tm_sync_dev(h); }

int kg_tmcmc_field_size(kg_tmcmc_t h, const char *name, size_t *n) {
  TmField r;
  KG_CHECK(tm_field(h, name, r), std::string("unknown TMCMC field: ") + name);
  *n = r.n;
  return 0;
}

int kg_tmcmc_get_field(kg_tmcmc_t h, const char *name, double *out, size_t n) {
  TmField r;
  KG_CHECK(tm_field(h, name, r), std::string("unknown TMCMC field: ") + name);
  KG_CHECK(n == r.n, std::string("size mismatch for field ") + name);
  if (tm_sync_dev(h)) return 1;
  if (r.host) {
    for (size_t q = 0; q < n; q++) out[q] = r.host[q];
    return 0;
  }
  KG_HIP(hipMemcpyAsync(out, r.dev, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_tmcmc_set_field(kg_tmcmc_t h, const char *name, const double *in, size_t n) {
  TmField r;
  KG_CHECK(tm_field(h, name, r), std::string("unknown TMCMC field: ") + name);
  KG_CHECK(n == r.n, std::string("size mismatch for field ") + name);
  if (tm_sync_dev(h)) return 1;
  if (r.host) {
    for (size_t q = 0; q < n; q++) r.host[q] = in[q];
    return 0;
  }
  KG_HIP(hipMemcpyAsync(r.dev, in, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  if (r.dev == h->chainLen)
    for (size_t c = 0; c < n; c++) {
      KG_CHECK(in[c] >= 0 && in[c] == floor(in[c]), "Chain Lengths must be non-negative integers");
      h->hLen[c] = (unsigned)in[c];
    }
  if (r.dev == h->pmin || r.dev == h->pmax) {
    hipLaunchKernelGGL(k_tm_neglogwidth, dim3(nblk(h->N, 64)), dim3(64), 0, h->stream, h->N, h->pmin, h->pmax, h->vkind,
                       h->negLogWidth);
    KG_HIP(hipGetLastError());
  }
  return 0;
}

int kg_tmcmc_get_rng(kg_tmcmc_t h, int which, void *state5000) {
  KG_CHECK(which >= 0 && which < 3 + h->ndist, "rng index out of range");
  if (tm_sync_dev(h)) return 1;
  if (which == 0) {
    h->multinomialRng.save((unsigned char *)state5000);
    return 0;
  }
  MtStream &m = which == 1 ? h->multivariate : which == 2 ? h->uniform : *h->priorRng[which - 3];
  return m.export_gsl(state5000, h->stream);
}

int kg_tmcmc_set_rng(kg_tmcmc_t h, int which, const void *state5000) {
  KG_CHECK(which >= 0 && which < 3 + h->ndist, "rng index out of range");
  if (tm_sync_dev(h)) return 1;
  if (which == 0) return h->multinomialRng.load((const unsigned char *)state5000);
  MtStream &m = which == 1 ? h->multivariate : which == 2 ? h->uniform : *h->priorRng[which - 3];
  if (which == 1 && h->zAhead) {  // the normals formed ahead are from the replaced state
    if (m.join(h->stream)) return 1;
    h->zAhead = false;
  }
  return m.import_gsl(state5000, h->stream);
}

int kg_tmcmc_device_ptr(kg_tmcmc_t h, const char *name, void **ptr) {
  TmField r;
  KG_CHECK(tm_field(h, name, r) && r.dev, std::string("unknown TMCMC device field: ") + name);
  *ptr = r.dev;
  return 0;
}

int kg_tmcmc_stream(kg_tmcmc_t h, void **stream) {
  *stream = (void *)h->stream;
  return 0;
}

int kg_tmcmc_profile(kg_tmcmc_t h, int enable) {
  h->profile = enable != 0;
  return 0;
}

int kg_tmcmc_profile_read(kg_tmcmc_t h, const char *stage, double *ms_total, size_t *count) {
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

// host-only check of the multinomial forms (no device call): `reps`
// consecutive K-category draws of N from one generator seeded with `seed`
// (GSL mt19937 seeding), exact form into n_exact, interval form into
// n_interval (reps * K each)
int kg_debug_multinomial(uint64_t seed, size_t K, unsigned N, const double *p, size_t reps, unsigned *n_exact,
                         unsigned *n_interval) {
  KG_CHECK(K > 0 && p && n_exact && n_interval, "kg_debug_multinomial: bad arguments");
  kg::HostMt a, b;
  a.seed(seed);
  b.seed(seed);
  double bt = 0;
  std::vector<double> scratch;
  for (size_t r = 0; r < reps; r++) {
    kg::multinomial(a, K, N, p, n_exact + r * K, &bt);
    kg::multinomial_interval(b, K, N, p, n_interval + r * K, &bt, scratch);
  }
  return 0;
}
