// kg_tmcmc.hip — TMCMC generation (TMCMC::runGeneration, TMCMC.cpp.base:107-157)
// on the device, Version "TMCMC", Max Chain Length 1, Burn In 0 (the C3
// configuration).
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
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/korali_amd.h"
#include "kg_common.hpp"
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
// generateCandidate :560-566 -> gsl_ran_multivariate_gaussian (normals from
// the polar pass, dtrmv Lower/NoTrans/NonUnit in gslcblas order, + zero mean)
// then + leader.  One thread per (chain, i): x_i = (sum_{j<i} z_j L_ij) + z_i L_ii.
__global__ void __launch_bounds__(256) k_tm_draw(int N, int P, const double *__restrict__ Z,
                                                 const double *__restrict__ Lg, const double *__restrict__ leaders,
                                                 double *__restrict__ cand) {
  extern __shared__ double sm[];
  const int S = N + 1;
  double *Ls = sm;            // N x (N+1)
  double *zs = sm + N * S;    // CB x N
  const int CB = max(1, 256 / N);
  const int c0 = blockIdx.x * CB;
  for (int e = threadIdx.x; e < N * N; e += blockDim.x) Ls[(e / N) * S + e % N] = Lg[e];
  for (int e = threadIdx.x; e < CB * N; e += blockDim.x) {
    const int c = c0 + e / N;
    zs[e] = c < P ? Z[(size_t)c * N + e % N] : 0.0;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < CB * N; e += blockDim.x) {
    const int cl = e / N, i = e % N, c = c0 + cl;
    if (c >= P) continue;
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
// univariate/uniform/uniform.cpp.base:30-36): a*(1-u) + b*u.
__global__ void k_tm_prior(int N, int P, const double *__restrict__ U, const unsigned long long *__restrict__ uoff,
                           const int *__restrict__ ustride, const double *__restrict__ pmin,
                           const double *__restrict__ pmax, double *__restrict__ cand) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const int c = (int)(e / N), d = (int)(e % N);
  const double u = U[uoff[d] + (size_t)c * ustride[d]];
  cand[e] = pmin[d] * (1 - u) + pmax[d] * u;
}

// Bayesian::evaluate (bayesian.cpp.base:24-84): logPrior = sum of uniform
// log-densities (-log(b-a) inside, -inf outside; uniform.cpp.base:38-44);
// -inf prior -> loglik -inf without evaluating the model; otherwise the
// builtin Gaussian loglik -0.5*sum x^2 (samplers/mean/model/model.py:32-37).
__global__ void k_tm_evaluate(int N, int P, int lik, const double *__restrict__ cand,
                              const double *__restrict__ negLogWidth, const double *__restrict__ pmin,
                              const double *__restrict__ pmax, double *__restrict__ candLL,
                              double *__restrict__ candLP) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P) return;
  const double *x = cand + (size_t)c * N;
  double lp = 0.0;
  for (int d = 0; d < N; d++) lp += (x[d] >= pmin[d] && x[d] <= pmax[d]) ? negLogWidth[d] : -INFINITY;
  candLP[c] = lp;
  double ll = -INFINITY;
  if (!(isinf(lp) && lp < 0)) {
    double ss = 0.0;
    for (int d = 0; d < N; d++) ss += x[d] * x[d];
    ll = -0.5 * ss;
    (void)lik;
  }
  candLL[c] = ll;
}

__global__ void k_tm_neglogwidth(int N, const double *__restrict__ pmin, const double *__restrict__ pmax,
                                 double *__restrict__ out) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < N) out[d] = -log_cr(pmax[d] - pmin[d]);
}

// processCandidate + calculateAcceptanceProbability + updateDatabase
// (:229-252, :611-633): P = exp((ll_c - ll_l) rho + (lp_c - lp_l)) if both
// candidate values are finite, else 0; one Uniform draw per chain (always);
// accept if P > U or generation 1.  Chain c's database entry is its leader.
__global__ void k_tm_accept(int P, int gen1, double rho, const double *__restrict__ U,
                            const double *__restrict__ candLL, const double *__restrict__ candLP,
                            double *__restrict__ leadLL, double *__restrict__ leadLP, double *__restrict__ dbLL,
                            double *__restrict__ dbLP, unsigned char *__restrict__ acc, TmDev *dev) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  bool a = false;
  if (c < P) {
    double p = 0.0;
    const double lpc = candLP[c], llc = candLL[c];
    if (isfinite(lpc) && isfinite(llc)) p = exp_cr((llc - leadLL[c]) * rho + (lpc - leadLP[c]));
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

__global__ void k_tm_copy_rows(int N, int P, const unsigned char *__restrict__ acc, const double *__restrict__ cand,
                               double *__restrict__ leaders, double *__restrict__ db) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const int c = (int)(e / N);
  double v = leaders[e];
  if (acc[c]) {
    v = cand[e];
    leaders[e] = v;
  }
  db[e] = v;
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

// calculateSquaredCVDifference :683-703, the parallel part: for each search
// point x_k, E_k[i] = exp((ll_i - ll_max) * (x_k - rho)).
__global__ void k_tm_cv_exp(int P, int npts, const double *__restrict__ ll, const TmDev *__restrict__ dev, double rho,
                            CvPoints pts, double *__restrict__ E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (i >= P || k >= npts) return;
  const double llmax = dev->llmaxCv;
  E[(size_t)k * P + i] = exp_cr((ll[i] - llmax) * (pts.x[k] - rho));
}

// processGeneration :284-296: w_i = exp(ll_i (rho - rho_prev) - max)
__global__ void k_tm_lw_exp(int P, const double *__restrict__ ll, double drho, const TmDev *__restrict__ dev,
                            double *__restrict__ E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  E[i] = exp_cr(ll[i] * drho - dev->lwmax);
}

// processGeneration :318-322: meanTheta_i = sum_j db[j][i] w_j, sequential in j
__global__ void __launch_bounds__(64) k_tm_mean(int N, int P, const double *__restrict__ db,
                                                const double *__restrict__ w, double *__restrict__ mean) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double m = 0;
  int j = 0;
  for (; j + 8 <= P; j += 8) {
    double v[8], ww[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      v[q] = db[(size_t)(j + q) * N + i];
      ww[q] = w[j + q];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) m += v[q] * ww[q];
  }
  for (; j < P; j++) m += db[(size_t)j * N + i] * w[j];
  mean[i] = m;
}

// processGeneration :324-329: cov_ij = covScaling * s / (1 - sum w^2),
// s = sum_k w_k (x_ki - m_i)(x_kj - m_j) sequential in k, j >= i; one lane
// per (i, j) pair, database rows staged through LDS.
constexpr int COV_ROWS = 64;
__global__ void __launch_bounds__(256) k_tm_cov(int N, int P, const double *__restrict__ db,
                                                const double *__restrict__ w, const double *__restrict__ mean,
                                                double scaling, double denom, double *__restrict__ cov) {
  extern __shared__ double rows[];  // COV_ROWS x N, then COV_ROWS weights
  double *ws = rows + COV_ROWS * N;
  const int npairs = N * (N + 1) / 2;
  const int pidx = blockIdx.x * blockDim.x + threadIdx.x;
  int pi = 0, pj = 0;
  const bool active = pidx < npairs;
  if (active) {  // pidx -> (i, j), row-major over the upper triangle
    int rem = pidx, i = 0;
    while (rem >= N - i) {
      rem -= N - i;
      i++;
    }
    pi = i;
    pj = i + rem;
  }
  const double mi = active ? mean[pi] : 0.0, mj = active ? mean[pj] : 0.0;
  double s = 0.0;
  for (int k0 = 0; k0 < P; k0 += COV_ROWS) {
    const int nk = min(COV_ROWS, P - k0);
    __syncthreads();
    for (int e = threadIdx.x; e < nk * N; e += blockDim.x) rows[e] = db[(size_t)k0 * N + e];
    for (int e = threadIdx.x; e < nk; e += blockDim.x) ws[e] = w[k0 + e];
    __syncthreads();
    if (active)
      for (int k = 0; k < nk; k++) s += ws[k] * (rows[k * N + pi] - mi) * (rows[k * N + pj] - mj);
  }
  if (active) {
    const double v = scaling * s / denom;
    cov[pi * N + pj] = v;
    cov[pj * N + pi] = v;
  }
}

// leader expansion :331-360 with Max Chain Length 1: leader j = database
// entry src[j], chain length 1
__global__ void k_tm_expand(int N, int P, const unsigned *__restrict__ src, const double *__restrict__ db,
                            const double *__restrict__ dbLL, const double *__restrict__ dbLP,
                            double *__restrict__ leaders, double *__restrict__ leadLL, double *__restrict__ leadLP,
                            double *__restrict__ chainLen) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)P * N) return;
  const int j = (int)(e / N), d = (int)(e % N);
  const unsigned s = src[j];
  leaders[e] = db[(size_t)s * N + d];
  if (d == 0) {
    leadLL[j] = dbLL[s];
    leadLP[j] = dbLP[s];
    chainLen[j] = 1.0;
  }
}

__global__ void k_tm_fill(double *p, size_t n, double v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
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
    if (mti >= MT_N) {
      for (int k = 0; k < MT_N; k++) mt[k] = mt_next(mt[k], mt[(k + 1) % MT_N], mt[(k + MT_M) % MT_N]);
      mti = 0;
    }
    return mt_temper(mt[mti++]);
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

unsigned binomial(HostMt &r, double p, unsigned n) {
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
void multinomial(HostMt &r, size_t K, unsigned N, const double *p, unsigned *n) {
  double norm = 0.0, sum_p = 0.0;
  unsigned sum_n = 0;
  for (size_t k = 0; k < K; k++) norm += p[k];
  for (size_t k = 0; k < K; k++) {
    n[k] = p[k] > 0.0 ? binomial(r, p[k] / (norm - sum_p), N - sum_n) : 0;
    sum_p += p[k];
    sum_n += n[k];
  }
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

}  // namespace
}  // namespace kg

using namespace kg;

struct kg_tmcmc_s {
  kg_tmcmc_cfg cfg;
  int N = 0, P = 0, ndist = 0;
  hipStream_t stream = nullptr;
  // device state
  double *leaders = nullptr, *leadLL = nullptr, *leadLP = nullptr, *cand = nullptr, *candLL = nullptr,
         *candLP = nullptr, *chainLen = nullptr, *mean = nullptr, *cov = nullptr, *chol = nullptr, *db = nullptr,
         *dbLL = nullptr, *dbLP = nullptr, *numSel = nullptr, *pmin = nullptr, *pmax = nullptr,
         *negLogWidth = nullptr, *Z = nullptr, *U = nullptr, *Uprior = nullptr, *E = nullptr, *w = nullptr;
  unsigned long long *uoff = nullptr;
  int *ustride = nullptr;
  unsigned *src = nullptr;
  unsigned char *acc = nullptr;
  TmDev *dev = nullptr;
  // pinned host staging
  double *hE = nullptr, *hW = nullptr, *hNsel = nullptr;
  unsigned *hSrc = nullptr;
  TmDev *hDev = nullptr;
  std::vector<double> wtmp;
  std::vector<unsigned> nsel;
  // per-distribution prior layout
  std::vector<int> distOf;           // variable -> distribution
  std::vector<size_t> distVars;      // variables per distribution
  std::vector<size_t> distOffset;    // offset of the distribution's draws in Uprior
  // RNGs
  HostMt multinomialRng;
  MtStream multivariate, uniform;
  std::vector<MtStream *> priorRng;
  // scalars (TMCMC.config internal settings)
  double annealingExponent = 0, previousAnnealingExponent = 0, logEvidence = 0, coefficientOfVariation = 0,
         maxLoglikelihood = -INFINITY, chainCount = 0, acceptedSamplesCount = 0, proposalsAcceptanceRate = 0,
         selectionAcceptanceRate = 0, dbCount = 0, modelEvaluationCount = 0, minSearchIterations = 0;
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
  KG_HIP(hipMalloc(p, n * sizeof(T)));
  KG_HIP(hipMemset(*p, 0, n * sizeof(T)));
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

// evaluates calculateSquaredCVDifference at batches of search points: the
// exponentials on the device, the serial tail on the host
struct CvSearch {
  kg_tmcmc_s *h;
  double exponent, target;
  double xs[CV_MAX_PTS];
  int n = 0;
  int batch(const double *pts, int npts) {
    CvPoints cp{};
    n = std::min(npts, CV_MAX_PTS);
    for (int k = 0; k < n; k++) cp.x[k] = xs[k] = pts[k];
    const int P = h->P;
    hipLaunchKernelGGL(k_tm_cv_exp, dim3(nblk(P, 256), n), dim3(256), 0, h->stream, P, n, h->dbLL, h->dev, exponent,
                       cp, h->E);
    KG_HIP(hipGetLastError());
    KG_HIP(hipMemcpyAsync(h->hE, h->E, (size_t)n * P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    return 0;
  }
  // f(x); rc != 0 on a HIP error
  double eval(double x, int &rc) {
    for (int k = 0; k < n; k++)
      if (memcmp(&xs[k], &x, sizeof(double)) == 0) return cv2_tail(h->hE + (size_t)k * h->P, h->P, target, h->wtmp.data());
    rc |= batch(&x, 1);
    return cv2_tail(h->hE, h->P, target, h->wtmp.data());
  }
};

double simplex_size(const double X[2]) {
  const double center = (X[0] + X[1]) / 2;
  double ss = 0.0;
  ss += fabs(X[0] - center);
  ss += fabs(X[1] - center);
  return ss / 2.0;
}

// minSearch :712-779: gsl_multimin_fminimizer_nmsimplex (v1) in one
// dimension, x0 = exponent, step 1e-8, size tolerance 1e-12, <= 1000
// iterations; each iteration's possible next points are evaluated on the
// device in one batch.
int min_search(kg_tmcmc_s *h, double exponent, double objCov, double &xmin, double &fmin, size_t &iters) {
  const size_t MaxIter = 1000;
  const double Tol = 1e-12, Step = 1e-8;
  CvSearch cv{h, exponent, objCov};
  int rc = 0;
  double X[2] = {exponent, exponent + Step}, Y[2];
  if (cv.batch(X, 2)) return 1;
  Y[0] = cv.eval(X[0], rc);
  Y[1] = cv.eval(X[1], rc);
  double xbest = X[0], fval = 0.0, size;
  size_t iter = 0;
  int status;
  do {
    iter++;
    size_t hi = 0, s_hi = 0, lo = 0;
    double dhi = Y[0], ds_hi = Y[0], dlo = Y[0];
    {
      const double val = Y[1];
      if (val < dlo) {
        dlo = val;
        lo = 1;
      } else if (val > dhi) {
        ds_hi = dhi;
        s_hi = hi;
        dhi = val;
        hi = 1;
      } else if (val > ds_hi) {
        ds_hi = val;
        s_hi = 1;
      }
    }
    const double mp = X[1 - hi];
    const double xc = mp - (-1.0) * (mp - X[hi]);
    // speculative batch: reflection, expansion, both contractions and both
    // contract-by-best outcomes
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
      if (cv.batch(pts, np)) return 1;
    }
    double val = cv.eval(xc, rc);
    if (std::isfinite(val) && val < Y[lo]) {
      const double xc2 = mp - (-2.0) * (mp - X[hi]);
      const double val2 = cv.eval(xc2, rc);
      if (std::isfinite(val2) && val2 < Y[lo]) {
        X[hi] = xc2;
        Y[hi] = val2;
      } else {
        X[hi] = xc;
        Y[hi] = val;
      }
    } else if (!std::isfinite(val) || val > Y[s_hi]) {
      if (std::isfinite(val) && val <= Y[hi]) {
        X[hi] = xc;
        Y[hi] = val;
      }
      const double xc2 = mp - 0.5 * (mp - X[hi]);
      const double val2 = cv.eval(xc2, rc);
      if (std::isfinite(val2) && val2 <= Y[hi]) {
        X[hi] = xc2;
        Y[hi] = val2;
      } else {
        for (size_t i = 0; i < 2; i++)
          if (i != lo) {
            X[i] = 0.5 * (X[i] + X[lo]);
            Y[i] = cv.eval(X[i], rc);
          }
      }
    } else {
      X[hi] = xc;
      Y[hi] = val;
    }
    // gsl_vector_min_index (NaN wins)
    lo = 0;
    {
      double mn = Y[0];
      for (size_t i = 0; i < 2; i++) {
        if (Y[i] < mn) {
          mn = Y[i];
          lo = i;
        }
        if (Y[i] != Y[i]) {
          lo = i;
          break;
        }
      }
    }
    xbest = X[lo];
    fval = Y[lo];
    size = simplex_size(X);
    status = (size < Tol) ? 0 : 1;
  } while (status == 1 && iter < MaxIter && rc == 0);
  if (rc) return 1;
  fmin = 0;
  xmin = 0.0;
  if (fval <= Tol) {
    fmin = fval;
    xmin = xbest;
  }
  if (xmin >= 1.0) {
    fmin = cv.eval(1.0, rc);
    xmin = 1.0;
  }
  iters = iter;
  return rc;
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
  return 0;
}

struct TmField {
  double *dev;   // device vector, or nullptr for a host scalar
  double *host;  // host scalar
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
  KG_CHECK(cfg->max_chain_length == 1.0, "device TMCMC path supports 'Max Chain Length' 1 only");
  KG_CHECK(cfg->default_burn_in == 0.0, "device TMCMC path supports 'Default Burn In' 0 only");
  KG_CHECK(cfg->covariance_scaling > 0.0, "Covariance Scaling must be larger 0.0");  // TMCMC.cpp.base:28
  KG_CHECK(cfg->prior_min && cfg->prior_max, "prior_min / prior_max are required");
  KG_CHECK(cfg->likelihood == KG_LIK_GAUSSIAN, "unknown builtin likelihood");
  KG_HIP(hipSetDevice(cfg->device));
  upload_dd_tables();
  auto *h = new kg_tmcmc_s();
  h->cfg = *cfg;
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
  rc |= tdalloc(&h->Uprior, PN) | tdalloc(&h->E, (size_t)CV_MAX_PTS * P) | tdalloc(&h->w, P);
  rc |= tdalloc(&h->uoff, N) | tdalloc(&h->ustride, N) | tdalloc(&h->src, P) | tdalloc(&h->acc, P);
  rc |= tdalloc(&h->dev, 1);
  if (rc) {
    delete h;
    return 1;
  }
  KG_HIP(hipHostMalloc(&h->hE, (size_t)CV_MAX_PTS * P * sizeof(double), hipHostMallocDefault));
  KG_HIP(hipHostMalloc(&h->hW, (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(hipHostMalloc(&h->hNsel, (size_t)P * sizeof(double), hipHostMallocDefault));
  KG_HIP(hipHostMalloc(&h->hSrc, (size_t)P * sizeof(unsigned), hipHostMallocDefault));
  KG_HIP(hipHostMalloc(&h->hDev, sizeof(TmDev), hipHostMallocDefault));
  h->wtmp.resize(P);
  h->nsel.resize(P);
  KG_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  KG_HIP(hipMemcpy(h->pmin, cfg->prior_min, N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->pmax, cfg->prior_max, N * sizeof(double), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->uoff, uoff.data(), N * sizeof(unsigned long long), hipMemcpyHostToDevice));
  KG_HIP(hipMemcpy(h->ustride, ustride.data(), N * sizeof(int), hipMemcpyHostToDevice));
  {
    const size_t lbytes = (size_t)N * (N + 1) * sizeof(double) + (size_t)std::max(1, 256 / N) * N * sizeof(double);
    if (lbytes > 64 * 1024) {
      KG_HIP(hipFuncSetAttribute((const void *)k_tm_draw, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lbytes));
      KG_HIP(hipFuncSetAttribute((const void *)k_tm_cholesky, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)((size_t)N * (N + 1) * sizeof(double))));
    }
  }
  hipLaunchKernelGGL(k_tm_neglogwidth, dim3(nblk(N, 64)), dim3(64), 0, h->stream, N, h->pmin, h->pmax, h->negLogWidth);
  KG_HIP(hipGetLastError());
  if (h->multivariate.init(3 * h->multivariate.words_for_normals(PN) + 4096) || h->uniform.init(4 * (size_t)P + 4096)) {
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
    if (h->priorRng[k]->init(2 * h->distVars[k] * (size_t)P + 4096)) return 1;
    seed_state(cfg->prior_seeds ? cfg->prior_seeds[k] : 0, st);
    if (h->priorRng[k]->import_gsl(st, h->stream)) return 1;
  }
  h->chainCount = P;
  *out = h;
  return 0;
}

int kg_tmcmc_destroy(kg_tmcmc_t h) {
  if (!h) return 0;
  (void)hipStreamSynchronize(h->stream);
  for (void *p : {(void *)h->leaders, (void *)h->leadLL, (void *)h->leadLP, (void *)h->cand, (void *)h->candLL,
                  (void *)h->candLP, (void *)h->chainLen, (void *)h->mean, (void *)h->cov, (void *)h->chol,
                  (void *)h->db, (void *)h->dbLL, (void *)h->dbLP, (void *)h->numSel, (void *)h->pmin,
                  (void *)h->pmax, (void *)h->negLogWidth, (void *)h->Z, (void *)h->U, (void *)h->Uprior,
                  (void *)h->E, (void *)h->w, (void *)h->uoff, (void *)h->ustride, (void *)h->src, (void *)h->acc,
                  (void *)h->dev})
    if (p) (void)hipFree(p);
  for (void *p : {(void *)h->hE, (void *)h->hW, (void *)h->hNsel, (void *)h->hSrc, (void *)h->hDev})
    if (p) (void)hipHostFree(p);
  for (auto *r : h->priorRng) delete r;
  for (auto &t : h->pending) {
    (void)hipEventDestroy(std::get<1>(t));
    (void)hipEventDestroy(std::get<2>(t));
  }
  (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int kg_tmcmc_prepare(kg_tmcmc_t h, size_t generation) {
  const int N = h->N, P = h->P;
  const size_t PN = (size_t)P * N;
  if (generation == 1 && tm_initialize(h)) return 1;
  if (tm_sync_dev(h)) return 1;
  // prepareGeneration :161-170
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
  if (generation == 1) {
    TmStage st(h, "prior_draw");
    for (int k = 0; k < h->ndist; k++)
      if (h->distVars[k] && h->priorRng[k]->uniforms(h->Uprior + h->distOffset[k], h->distVars[k] * (size_t)P, h->stream))
        return 1;
    hipLaunchKernelGGL(k_tm_prior, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, h->Uprior, h->uoff, h->ustride,
                       h->pmin, h->pmax, h->cand);
    KG_HIP(hipGetLastError());
  } else {
    {
      TmStage st(h, "rng_polar");
      if (h->multivariate.polar_normals(h->Z, PN, N, nullptr, h->stream)) return 1;
      if (h->multivariate.consume_normals(PN, N, nullptr, h->stream)) return 1;
    }
    TmStage st(h, "draw");
    const int CB = std::max(1, 256 / N);
    const size_t lbytes = (size_t)N * (N + 1) * sizeof(double) + (size_t)CB * N * sizeof(double);
    hipLaunchKernelGGL(k_tm_draw, dim3(nblk(P, CB)), dim3(256), lbytes, h->stream, N, P, h->Z, h->chol, h->leaders,
                       h->cand);
    KG_HIP(hipGetLastError());
  }
  return 0;
}

int kg_tmcmc_evaluate(kg_tmcmc_t h) {
  TmStage st(h, "evaluate");
  hipLaunchKernelGGL(k_tm_evaluate, dim3(nblk(h->P, 128)), dim3(128), 0, h->stream, h->N, h->P, h->cfg.likelihood,
                     h->cand, h->negLogWidth, h->pmin, h->pmax, h->candLL, h->candLP);
  KG_HIP(hipGetLastError());
  h->modelEvaluationCount += h->P;
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
  KG_HIP(hipMemcpyAsync(h->candLP, log_prior, h->P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->candLL, log_likelihood, h->P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  h->modelEvaluationCount += h->P;
  return 0;
}

int kg_tmcmc_process(kg_tmcmc_t h, size_t generation) {
  const int N = h->N, P = h->P;
  const size_t PN = (size_t)P * N;
  {
    TmStage st(h, "accept");
    if (h->uniform.uniforms(h->U, P, h->stream)) return 1;
    hipLaunchKernelGGL(k_tm_accept, dim3(nblk(P, 256)), dim3(256), 0, h->stream, P, generation == 1 ? 1 : 0,
                       h->annealingExponent, h->U, h->candLL, h->candLP, h->leadLL, h->leadLP, h->dbLL, h->dbLP,
                       h->acc, h->dev);
    hipLaunchKernelGGL(k_tm_copy_rows, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, h->acc, h->cand,
                       h->leaders, h->db);
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
    if (min_search(h, h->annealingExponent, h->cfg.target_cov, xmin, fmin, iters)) return 1;
  }
  if (tm_sync_dev(h)) return 1;
  h->minSearchIterations = (double)iters;
  h->previousAnnealingExponent = h->annealingExponent;
  {
    CvSearch cv{h, h->previousAnnealingExponent, h->cfg.target_cov};
    int rc = 0;
    if (xmin > h->previousAnnealingExponent + h->cfg.max_annealing_exponent_update) {
      h->annealingExponent = h->previousAnnealingExponent + h->cfg.max_annealing_exponent_update;
      h->coefficientOfVariation = sqrt(cv.eval(h->annealingExponent, rc)) + h->cfg.target_cov;
    } else if (xmin < 1.0 && xmin < h->previousAnnealingExponent + h->cfg.min_annealing_exponent_update) {
      h->annealingExponent = h->previousAnnealingExponent + h->cfg.min_annealing_exponent_update;
      h->coefficientOfVariation = sqrt(cv.eval(h->annealingExponent, rc)) + h->cfg.target_cov;
    } else {
      h->annealingExponent = xmin;
      h->coefficientOfVariation = sqrt(fmin) + h->cfg.target_cov;
    }
    if (rc) return 1;
  }
  const double drho = h->annealingExponent - h->previousAnnealingExponent;
  {
    TmStage st(h, "weights");
    hipLaunchKernelGGL(k_tm_max, dim3(1), dim3(1024), 0, h->stream, P, h->dbLL, drho, 1, &h->dev->lwmax,
                       (double *)nullptr);
    hipLaunchKernelGGL(k_tm_lw_exp, dim3(nblk(P, 256)), dim3(256), 0, h->stream, P, h->dbLL, drho, h->dev, h->E);
    KG_HIP(hipGetLastError());
    KG_HIP(hipMemcpyAsync(h->hE, h->E, (size_t)P * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipMemcpyAsync(h->hDev, h->dev, sizeof(TmDev), hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
  }
  size_t zeroCount = 0, leaderId = 0;
  double sumw2 = 0.0;
  {
    HostClock hc(h, "multinomial");
    double *wt = h->hW;
    const double lwmax = h->hDev->lwmax;
    double sw = 0.0;
    for (int i = 0; i < P; i++) sw += h->hE[i];
    for (int i = 0; i < P; i++) wt[i] = h->hE[i] / sw;
    h->logEvidence += host_log_cr(sw) + lwmax - host_log_cr((double)P);
    multinomial(h->multinomialRng, P, (unsigned)P, wt, h->nsel.data());
    for (int i = 0; i < P; i++) h->hNsel[i] = h->nsel[i];
    for (int i = 0; i < P; i++) wt[i] = wt[i] * h->nsel[i];
    sw = 0.0;
    for (int i = 0; i < P; i++) sw += wt[i];
    for (int i = 0; i < P; i++) wt[i] = wt[i] / sw;
    for (int i = 0; i < P; i++) sumw2 += wt[i] * wt[i];
    for (int i = 0; i < P; i++) {
      if (h->nsel[i] == 0) zeroCount++;
      for (unsigned t = 0; t < h->nsel[i]; t++) h->hSrc[leaderId++] = (unsigned)i;
    }
  }
  KG_CHECK(leaderId == (size_t)P, "multinomial selections do not sum to the population size");
  KG_HIP(hipMemcpyAsync(h->w, h->hW, (size_t)P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->numSel, h->hNsel, (size_t)P * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->src, h->hSrc, (size_t)P * sizeof(unsigned), hipMemcpyHostToDevice, h->stream));
  {
    TmStage st(h, "mean_cov");
    hipLaunchKernelGGL(k_tm_mean, dim3(nblk(N, 64)), dim3(64), 0, h->stream, N, P, h->db, h->w, h->mean);
    const int npairs = N * (N + 1) / 2;
    const size_t cbytes = (size_t)COV_ROWS * N * sizeof(double) + COV_ROWS * sizeof(double);
    hipLaunchKernelGGL(k_tm_cov, dim3(nblk(npairs, 256)), dim3(256), cbytes, h->stream, N, P, h->db, h->w, h->mean,
                       h->cfg.covariance_scaling, 1.0 - sumw2, h->cov);
    KG_HIP(hipGetLastError());
  }
  {
    TmStage st(h, "expand");
    hipLaunchKernelGGL(k_tm_expand, dim3(nblk(PN, 256)), dim3(256), 0, h->stream, N, P, h->src, h->db, h->dbLL,
                       h->dbLP, h->leaders, h->leadLL, h->leadLP, h->chainLen);
    KG_HIP(hipGetLastError());
  }
  h->proposalsAcceptanceRate = (1.0 * h->acceptedSamplesCount) / P;
  h->selectionAcceptanceRate = (1.0 * (P - zeroCount)) / P;
  h->chainCount = (double)leaderId;
  // the pinned staging buffers are reused by the next generation's search,
  // which synchronises the stream before touching them
  return 0;
}

int kg_tmcmc_generation(kg_tmcmc_t h, size_t generation) {
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
    *out = *r.host;
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
    *r.host = *in;
    return 0;
  }
  KG_HIP(hipMemcpyAsync(r.dev, in, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  if (r.dev == h->pmin || r.dev == h->pmax) {
    hipLaunchKernelGGL(k_tm_neglogwidth, dim3(nblk(h->N, 64)), dim3(64), 0, h->stream, h->N, h->pmin, h->pmax,
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
  return m.import_gsl(state5000, h->stream);
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
