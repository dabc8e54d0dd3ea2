/*
 * refcpu.c — CPU ORACLE (test infrastructure only; see refcpu.h header).
 *
 * Every function cites the reference file:line (paths relative to the
 * reference root) or the GSL 2.6 / gslcblas routine whose published
 * algorithm it restates.  GSL itself is not present in the reference tree
 * (subprojects/gsl.wrap pins release-2-6); the restatements follow SURVEY.md
 * Appendix A and were pinned against the reference's committed generation
 * files (tests/golden/).
 */
#include "refcpu.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Threads for the data-parallel loops of the checker (OpenMP build only).
 * Every parallel loop computes independent outputs, each with the
 * reference's own operation order, so results do not depend on the thread
 * count; the CPU-baseline timing sets 1 (the reference is single-threaded). */
void kr_set_threads(int n)
{
#ifdef _OPENMP
  omp_set_num_threads(n < 1 ? 1 : n);
#else
  (void)n;
#endif
}

#define KR_DBL_EPSILON 2.2204460492503131e-16
#define KR_DBL_MIN 2.2250738585072014e-308


/* ======================================================================
 * Correctly-rounded log / exp / pow (double-double evaluation).
 *
 * The reference's committed fixtures were produced on a host whose libm
 * log is correctly rounded (glibc < 2.28 IBM Accurate Mathematical
 * Library): with a CR log the oracle reproduces all 99 fixture populations
 * bit-exactly, with this image's glibc 2.35 log (< 0.52 ulp, not CR) 9 of
 * 99 generations differ by 1 ulp in one normal.  The oracle therefore
 * evaluates every log/exp the reference path calls in double-double
 * (~2^-100 relative) and rounds once.
 * ==================================================================== */
typedef struct
{
  double hi, lo;
} dd_t;

static inline dd_t dd_quick_two_sum(double a, double b)
{
  dd_t r;
  r.hi = a + b;
  r.lo = b - (r.hi - a);
  return r;
}
static inline dd_t dd_two_sum(double a, double b)
{
  dd_t r;
  double bb;
  r.hi = a + b;
  bb = r.hi - a;
  r.lo = (a - (r.hi - bb)) + (b - bb);
  return r;
}
static inline void dd_split(double a, double *h, double *l)
{
  const double t = 134217729.0 * a; /* 2^27 + 1 */
  *h = t - (t - a);
  *l = a - *h;
}
static inline dd_t dd_two_prod(double a, double b)
{
  dd_t r;
  double ah, al, bh, bl;
  r.hi = a * b;
  dd_split(a, &ah, &al);
  dd_split(b, &bh, &bl);
  r.lo = ((ah * bh - r.hi) + ah * bl + al * bh) + al * bl;
  return r;
}
static inline dd_t dd_add(dd_t a, dd_t b)
{
  dd_t s = dd_two_sum(a.hi, b.hi), t = dd_two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = dd_quick_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return dd_quick_two_sum(s.hi, s.lo);
}
static inline dd_t dd_mul(dd_t a, dd_t b)
{
  dd_t p = dd_two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return dd_quick_two_sum(p.hi, p.lo);
}
static inline dd_t dd_mul_d(dd_t a, double b)
{
  dd_t p = dd_two_prod(a.hi, b);
  p.lo += a.lo * b;
  return dd_quick_two_sum(p.hi, p.lo);
}
static inline dd_t dd_div(dd_t a, dd_t b)
{
  double q1 = a.hi / b.hi, q2, q3;
  dd_t r = dd_add(a, dd_mul_d(b, -q1));
  q2 = r.hi / b.hi;
  r = dd_add(r, dd_mul_d(b, -q2));
  q3 = r.hi / b.hi;
  r = dd_quick_two_sum(q1, q2);
  return dd_add(r, (dd_t){q3, 0.0});
}
static inline dd_t dd_from(double a) { return (dd_t){a, 0.0}; }

static const dd_t DD_LN2 = {6.93147180559945286227e-01, 2.31904681384629955842e-17};

/* 1/(2j+1), j = 0..21, as double-doubles (the series coefficients of
 * dd_log, computed once at load by the same dd_div) */
static dd_t dd_log_inv_odd[22];
__attribute__((constructor)) static void dd_log_init(void)
{
  int j;
  for (j = 0; j < 22; j++) dd_log_inv_odd[j] = dd_div(dd_from(1.0), dd_from(2.0 * j + 1.0));
}

/* log(x) for finite x > 0 as a double-double: x = m 2^k, m in
 * [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m-1)/(m+1). */
static dd_t dd_log(double x)
{
  int k = 0, j;
  double m = frexp(x, &k); /* x = m 2^k, m in [0.5, 1) */
  dd_t s, z, p;
  if (m < 0.70710678118654752440)
  {
    m *= 2.0;
    k -= 1;
  }
  s = dd_div(dd_from(m - 1.0), dd_two_sum(m, 1.0));
  z = dd_mul(s, s);
  p = dd_log_inv_odd[21];
  for (j = 20; j >= 0; j--) p = dd_add(dd_mul(p, z), dd_log_inv_odd[j]);
  p = dd_mul(dd_mul_d(s, 2.0), p);
  return dd_add(dd_mul_d(DD_LN2, (double)k), p);
}

/* KR_LIBM_TIMING: timing-only build (librefcpu_libm.so) that calls the
 * system libm instead of the correctly-rounded evaluations, i.e. runs at the
 * speed the reference itself would on this host.  Not bit-exact; used only
 * as the conservative CPU baseline in bench.py. */
double kr_log_cr(double x)
{
#ifdef KR_LIBM_TIMING
  return log(x);
#endif
  if (!(x > 0.0) || isinf(x)) return log(x);
  if (x == 1.0) return 0.0;
  if (x < 2.2250738585072014e-308) return kr_log_cr(x * 18014398509481984.0) - 37.42994775023704; /* rare */
  {
    dd_t r = dd_log(x);
    return r.hi + r.lo;
  }
}

/* exp of a double-double argument: e^a = 2^k e^r, r = (a - k ln2)/256 */
static dd_t dd_exp(dd_t a)
{
  const double kd = floor(a.hi / DD_LN2.hi + 0.5);
  dd_t r = dd_add(a, dd_mul_d(DD_LN2, -kd)), t, p;
  int j;
  r = dd_mul_d(r, 1.0 / 256.0);
  /* Taylor to 14 terms for |r| < 1.4e-3 */
  p = dd_from(1.0);
  t = dd_from(1.0);
  for (j = 14; j >= 1; j--) p = dd_add(dd_from(1.0), dd_div(dd_mul(p, r), dd_from((double)j)));
  (void)t;
  for (j = 0; j < 8; j++) p = dd_mul(p, p);
  p.hi = ldexp(p.hi, (int)kd);
  p.lo = ldexp(p.lo, (int)kd);
  return p;
}

double kr_exp_cr(double x)
{
#ifdef KR_LIBM_TIMING
  return exp(x);
#endif
  if (isnan(x)) return x;
  if (x > 709.0 || x < -708.0) return exp(x); /* out of the dd range: libm */
  if (x == 0.0) return 1.0;
  {
    dd_t r = dd_exp(dd_from(x));
    return r.hi + r.lo;
  }
}

double kr_pow_cr(double x, double y)
{
#ifdef KR_LIBM_TIMING
  return pow(x, y);
#endif
  if (y == 2.0) return x * x;
  if (!(x > 0.0) || isinf(x) || isinf(y) || isnan(y)) return pow(x, y);
  {
    dd_t l = dd_mul_d(dd_log(x), y);
    if (l.hi > 709.0 || l.hi < -708.0) return pow(x, y);
    l = dd_exp(l);
    return l.hi + l.lo;
  }
}

/* Correctly-rounded cos for the Ackley objective (model.py:37-62 calls
 * np.cos; the platform libm / SIMD cos is not correctly rounded, so both
 * the oracle and the device pin the CR value).  Cody-Waite reduction by a
 * triple-double pi/2 with exact products, then the Taylor series of cos or
 * sin of r (|r| <= pi/4) in double-double, rounded once.  Same operation
 * sequence as korali_amd/csrc/kg_common.hpp cos_cr. */
static const double KR_CH[15] = {0x1p+0, -0x1p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
  -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45,
  -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62, -0x1.0ce396db7f853p-70, 0x1.f2cf01972f578p-80,
  -0x1.88e85fc6a4e5ap-89, 0x1.0a18a2635085dp-98};
static const double KR_CL[15] = {0.0, 0.0, 0x1.5555555555555p-59, 0x1.f49f49f49f49fp-65, 0x1.a01a01a01a01ap-76,
  -0x1.cbbc05b4fa99ap-76, -0x1.2aec959e14c06p-83, -0x1.05d6f8a2efd1fp-92, 0x1.1d8656b0ee8cbp-101,
  -0x1.eec01221a8b0bp-107, 0x1.ea72b4afe3c2fp-120, 0x1.aebcdbd20331cp-124, -0x1.9ada5fcc1ab14p-135,
  0x1.71c37ebd16540p-143, 0x1.b9e2e28e1aa54p-153};
static const double KR_SH[15] = {0x1p+0, -0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
  0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41,
  0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66, -0x1.761b41316381ap-75,
  0x1.3f3ccdd165fa9p-84, -0x1.d1ab1c2dccea3p-94, 0x1.259f98b4358adp-103};
static const double KR_SL[15] = {0.0, -0x1.5555555555555p-57, 0x1.1111111111111p-63, -0x1.a01a01a01a01ap-73,
  -0x1.c154f8ddc6c00p-73, 0x1.c062e06d1f209p-80, 0x1.f28e0cc748ebep-87, -0x1.1d8656b0ee8cbp-97,
  0x1.ac981465ddc6cp-103, -0x1.2650f61dbdcb4p-112, -0x1.d043ae40c4647p-120, 0x1.3423c7d91404fp-130,
  -0x1.58ddadf344487p-139, -0x1.054d0c78aea14p-149, 0x1.eaf8c39dd9bc5p-157};

double kr_cos_cr(double x)
{
#ifdef KR_LIBM_TIMING
  return cos(x);
#endif
  const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
  const double INV_PIO2 = 0x1.45f306dc9c883p-1;
  double kd, v;
  dd_t t1, t2, r, z, p;
  int q, odd, j;
  if (!(fabs(x) < 1073741824.0)) return cos(x);
  kd = floor(x * INV_PIO2 + 0.5);
  t1 = dd_two_prod(kd, P1);
  t2 = dd_two_prod(kd, P2);
  r = dd_add(dd_from(x), (dd_t){-t1.hi, -t1.lo});
  r = dd_add(r, (dd_t){-t2.hi, -t2.lo});
  r = dd_add(r, (dd_t){-(kd * P3), 0.0});
  q = (int)((long long)kd & 3);
  odd = q & 1;
  z = dd_mul(r, r);
  p = odd ? (dd_t){KR_SH[14], KR_SL[14]} : (dd_t){KR_CH[14], KR_CL[14]};
  for (j = 13; j >= 0; j--)
    p = dd_add(dd_mul(p, z), odd ? (dd_t){KR_SH[j], KR_SL[j]} : (dd_t){KR_CH[j], KR_CL[j]});
  p = dd_mul(p, odd ? r : dd_from(1.0));
  v = p.hi + p.lo;
  return (q == 1 || q == 2) ? -v : v;
}

/* ======================================================================
 * mt19937, GSL semantics (rng/mt.c, 2002 seeding)
 * Korali: distribution.cpp.base:32-62 (gsl_rng_alloc(gsl_rng_default))
 * ==================================================================== */
#define MT_N 624
#define MT_M 397
#define MT_UPPER 0x80000000UL
#define MT_LOWER 0x7fffffffUL

void kr_rng_seed(kr_rng *r, uint64_t s)
{
  int i;
  if (s == 0) s = 4357;
  r->mt[0] = s & 0xffffffffUL;
  for (i = 1; i < MT_N; i++)
  {
    r->mt[i] = (1812433253UL * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint64_t)i);
    r->mt[i] &= 0xffffffffUL;
  }
  r->mti = i;
  r->pad = 0;
}

static inline uint64_t mt_magic(uint64_t y) { return (y & 1) ? 0x9908b0dfUL : 0UL; }

uint32_t kr_rng_get(kr_rng *r)
{
  uint64_t k;
  uint64_t *const mt = r->mt;
  if (r->mti >= MT_N)
  {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++)
    {
      uint64_t y = (mt[kk] & MT_UPPER) | (mt[kk + 1] & MT_LOWER);
      mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mt_magic(y);
    }
    for (; kk < MT_N - 1; kk++)
    {
      uint64_t y = (mt[kk] & MT_UPPER) | (mt[kk + 1] & MT_LOWER);
      mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mt_magic(y);
    }
    {
      uint64_t y = (mt[MT_N - 1] & MT_UPPER) | (mt[0] & MT_LOWER);
      mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mt_magic(y);
    }
    r->mti = 0;
  }
  k = mt[r->mti];
  k ^= (k >> 11);
  k ^= (k << 7) & 0x9d2c5680UL;
  k ^= (k << 15) & 0xefc60000UL;
  k ^= (k >> 18);
  r->mti++;
  return (uint32_t)(k & 0xffffffffUL);
}

double kr_rng_uniform(kr_rng *r) { return kr_rng_get(r) / 4294967296.0; }

double kr_rng_uniform_pos(kr_rng *r)
{
  double x;
  do x = kr_rng_uniform(r);
  while (x == 0);
  return x;
}

/* n draws of 0 + gsl_ran_gaussian(r, 1.0) in stream order: the accept /
 * reject loop consumes the generator serially, the log / sqrt of each
 * accepted pair (the same expression as kr_ran_gaussian) run in parallel */
void kr_ran_gaussian_n(kr_rng *r, size_t n, double *out)
{
  double *r2v = (double *)malloc(sizeof(double) * n);
  long i;
  size_t k;
  for (k = 0; k < n; k++)
  {
    double x, y, r2;
    do
    {
      x = -1 + 2 * kr_rng_uniform_pos(r);
      y = -1 + 2 * kr_rng_uniform_pos(r);
      r2 = x * x + y * y;
    } while (r2 > 1.0 || r2 == 0);
    out[k] = y;
    r2v[k] = r2;
  }
#pragma omp parallel for schedule(static)
  for (i = 0; i < (long)n; i++) out[i] = 0.0 + 1.0 * out[i] * sqrt(-2.0 * kr_log_cr(r2v[i]) / r2v[i]);
  free(r2v);
}

/* gsl_ran_gaussian (randist/gauss.c, polar Box-Muller); Korali
 * univariate/normal/normal.cpp.base:32-35 */
double kr_ran_gaussian(kr_rng *r, double sigma)
{
  double x, y, r2;
  do
  {
    x = -1 + 2 * kr_rng_uniform_pos(r);
    y = -1 + 2 * kr_rng_uniform_pos(r);
    r2 = x * x + y * y;
  } while (r2 > 1.0 || r2 == 0);
  return sigma * y * sqrt(-2.0 * kr_log_cr(r2) / r2);
}

/* GSL 2.6 randist samplers behind the other univariate priors
 * (exponential.c, laplace.c, cauchy.c, lognormal.c; Korali
 * univariate/{exponential,laplace,cauchy,logNormal}/*.cpp.base getRandomNumber).
 * log1p, tan and exp are the host libm's (as the device library's host
 * draws); log is the correctly rounded one, as everywhere in this file. */
double kr_ran_exponential(kr_rng *r, double mu)
{
  double u = kr_rng_uniform(r);
  return -mu * log1p(-u);
}

double kr_ran_laplace(kr_rng *r, double a)
{
  double u;
  do
  {
    u = 2 * kr_rng_uniform(r) - 1.0;
  } while (u == 0.0);
  if (u < 0) return a * kr_log_cr(-u);
  return -a * kr_log_cr(u);
}

double kr_ran_cauchy(kr_rng *r, double a)
{
  double u;
  do
  {
    u = kr_rng_uniform(r);
  } while (u == 0.5);
  return a * tan(3.14159265358979323846 * u);
}

double kr_ran_lognormal(kr_rng *r, double zeta, double sigma)
{
  double u, v, r2, normal;
  do
  {
    u = -1 + 2 * kr_rng_uniform(r);
    v = -1 + 2 * kr_rng_uniform(r);
    r2 = u * u + v * v;
  } while (r2 > 1.0 || r2 == 0);
  normal = u * sqrt(-2.0 * kr_log_cr(r2) / r2);
  return exp(sigma * normal + zeta);
}

/* gsl_ran_flat; Korali univariate/uniform/uniform.cpp.base:30-36 */
double kr_ran_flat(kr_rng *r, double a, double b)
{
  double u = kr_rng_uniform(r);
  return a * (1 - u) + b * u;
}

static double pow_uint(double x, unsigned int n)
{
  double value = 1.0;
  do
  {
    if (n & 1) value *= x;
    n >>= 1;
    x *= x;
  } while (n);
  return value;
}

/* Stirling tail used by GSL's BTPE (randist/binomial_tpe.c) */
static double btpe_stirling(double y1)
{
  double y2 = y1 * y1;
  return (13860.0 - (462.0 - (132.0 - (99.0 - 140.0 / y2) / y2) / y2) / y2) / y1 / 166320.0;
}

/* gsl_ran_binomial (randist/binomial_tpe.c: inversion for n*p < 14, BTPE
 * otherwise).  The BTPE branch is restated from Kachitvichyanukul &
 * Schmeiser (1988) as GSL implements it; no reference fixture reaches it
 * (parity unpinned for that branch). */
static unsigned long long kr_btpe_count; /* draws that took the BTPE branch */
unsigned long long kr_btpe_draws(void) { return kr_btpe_count; }

unsigned int kr_ran_binomial(kr_rng *rng, double p, unsigned int n)
{
  int ix;
  int flipped = 0;
  double q, s, np;
  if (n == 0) return 0;
  if (p > 0.5)
  {
    p = 1.0 - p;
    flipped = 1;
  }
  q = 1 - p;
  s = p / q;
  np = n * p;
  if (np < 14)
  {
    double f0 = pow_uint(q, n);
    while (1)
    {
      double f = f0;
      double u = kr_rng_uniform(rng);
      for (ix = 0; ix <= 110; ++ix)
      {
        if (u < f) goto Finish;
        u -= f;
        f *= s * (n - ix) / (ix + 1);
      }
    }
  }
  else
  {
    int k;
    double ffm = np + p;
    int m = (int)ffm;
    double fm = m;
    double xm = fm + 0.5;
    double npq = np * q;
    double p1 = floor(2.195 * sqrt(npq) - 4.6 * q) + 0.5;
    double xl = xm - p1;
    double xr = xm + p1;
    double c = 0.134 + 20.5 / (15.3 + fm);
    double p2 = p1 * (1.0 + c + c);
    double al = (ffm - xl) / (ffm - xl * p);
    double lambda_l = al * (1.0 + 0.5 * al);
    double ar = (xr - ffm) / (xr * q);
    double lambda_r = ar * (1.0 + 0.5 * ar);
    double p3 = p2 + c / lambda_l;
    double p4 = p3 + c / lambda_r;
    double var, accept;
    double u, v;
    kr_btpe_count++;
  TryAgain:
    u = kr_rng_uniform(rng) * p4;
    v = kr_rng_uniform(rng);
    if (u <= p1)
    {
      ix = (int)(xm - p1 * v + u);
      goto Finish;
    }
    else if (u <= p2)
    {
      double x = xl + (u - p1) / c;
      v = v * c + 1.0 - fabs(x - xm) / p1;
      if (v > 1.0 || v <= 0) goto TryAgain;
      ix = (int)x;
    }
    else if (u <= p3)
    {
      ix = (int)(xl + kr_log_cr(v) / lambda_l);
      if (ix < 0) goto TryAgain;
      v = v * ((u - p2) * lambda_l);
    }
    else
    {
      ix = (int)(xr - kr_log_cr(v) / lambda_r);
      if (ix > (double)n) goto TryAgain;
      v = v * ((u - p3) * lambda_r);
    }
    k = abs(ix - m);
    if (k <= 20)
    {
      double g = (n + 1) * s;
      double f = 1.0;
      var = v;
      if (m < ix)
      {
        int i;
        for (i = m + 1; i <= ix; i++) f *= (g / i - s);
      }
      else if (m > ix)
      {
        int i;
        for (i = ix + 1; i <= m; i++) f /= (g / i - s);
      }
      accept = f;
    }
    else
    {
      var = kr_log_cr(v);
      if (k < npq / 2 - 1)
      {
        double amaxp = k / npq * ((k * (k / 3.0 + 0.625) + (1.0 / 6.0)) / npq + 0.5);
        double ynorm = -(k * k / (2.0 * npq));
        if (var < ynorm - amaxp) goto Finish;
        if (var > ynorm + amaxp) goto TryAgain;
      }
      {
        double x1 = ix + 1.0;
        double w1 = n - ix + 1.0;
        double f1 = fm + 1.0;
        double z1 = n + 1.0 - fm;
        accept = xm * kr_log_cr(f1 / x1) + (n - m + 0.5) * kr_log_cr(z1 / w1) + (ix - m) * kr_log_cr(w1 * p / (x1 * q)) + btpe_stirling(f1) + btpe_stirling(z1) - btpe_stirling(x1) - btpe_stirling(w1);
      }
    }
    if (var <= accept)
      goto Finish;
    else
      goto TryAgain;
  }
Finish:
  return (flipped) ? (n - ix) : (unsigned int)ix;
}

/* gsl_ran_multinomial (randist/multinomial.c); Korali
 * specific/multinomial/multinomial.cpp.base:7-10 */
void kr_ran_multinomial(kr_rng *r, size_t K, unsigned int N, const double *p, unsigned int *n)
{
  size_t k;
  double norm = 0.0;
  double sum_p = 0.0;
  unsigned int sum_n = 0;
  for (k = 0; k < K; k++) norm += p[k];
  for (k = 0; k < K; k++)
  {
    if (p[k] > 0.0)
      n[k] = kr_ran_binomial(r, p[k] / (norm - sum_p), N - sum_n);
    else
      n[k] = 0;
    sum_p += p[k];
    sum_n += n[k];
  }
}

/* ======================================================================
 * fdlibm __ieee754_hypot (glibc < 2.35 behaviour)
 * ==================================================================== */
static inline uint32_t hi_word(double x)
{
  uint64_t u;
  memcpy(&u, &x, 8);
  return (uint32_t)(u >> 32);
}
static inline uint32_t lo_word(double x)
{
  uint64_t u;
  memcpy(&u, &x, 8);
  return (uint32_t)u;
}
static inline double set_hi(double x, uint32_t h)
{
  uint64_t u;
  memcpy(&u, &x, 8);
  u = (u & 0xffffffffULL) | ((uint64_t)h << 32);
  memcpy(&x, &u, 8);
  return x;
}

double kr_hypot(double x, double y)
{
  double a, b, t1, t2, y1, y2, w;
  int32_t j, k, ha, hb;
  ha = (int32_t)(hi_word(x) & 0x7fffffff);
  hb = (int32_t)(hi_word(y) & 0x7fffffff);
  if (hb > ha)
  {
    a = y;
    b = x;
    j = ha;
    ha = hb;
    hb = j;
  }
  else
  {
    a = x;
    b = y;
  }
  a = set_hi(a, (uint32_t)ha);
  b = set_hi(b, (uint32_t)hb);
  if ((ha - hb) > 0x3c00000) return a + b;
  k = 0;
  if (ha > 0x5f300000)
  {
    if (ha >= 0x7ff00000)
    {
      uint32_t low;
      w = a + b;
      low = lo_word(a);
      if (((ha & 0xfffff) | low) == 0) w = a;
      low = lo_word(b);
      if (((hb ^ 0x7ff00000) | low) == 0) w = b;
      return w;
    }
    ha -= 0x25800000;
    hb -= 0x25800000;
    k += 600;
    a = set_hi(a, (uint32_t)ha);
    b = set_hi(b, (uint32_t)hb);
  }
  if (hb < 0x20b00000)
  {
    if (hb <= 0x000fffff)
    {
      uint32_t low = lo_word(b);
      if ((hb | low) == 0) return a;
      t1 = set_hi(0.0, 0x7fd00000);
      b *= t1;
      a *= t1;
      k -= 1022;
    }
    else
    {
      ha += 0x25800000;
      hb += 0x25800000;
      k -= 600;
      a = set_hi(a, (uint32_t)ha);
      b = set_hi(b, (uint32_t)hb);
    }
  }
  w = a - b;
  if (w > b)
  {
    t1 = set_hi(0.0, (uint32_t)ha);
    t2 = a - t1;
    w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
  }
  else
  {
    a = a + a;
    y1 = set_hi(0.0, (uint32_t)hb);
    y2 = b - y1;
    t1 = set_hi(0.0, (uint32_t)(ha + 0x00100000));
    t2 = a - t1;
    w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
  }
  if (k != 0)
  {
    t1 = set_hi(1.0, hi_word(1.0) + ((uint32_t)k << 20));
    return t1 * w;
  }
  return w;
}

/* gslcblas dnrm2 (blas/source_nrm2_r.h) */
double kr_dnrm2(size_t n, const double *X, size_t inc)
{
  double scale = 0.0, ssq = 1.0;
  size_t i;
  if (n == 0) return 0;
  if (n == 1) return fabs(X[0]);
  for (i = 0; i < n; i++)
  {
    const double x = X[i * inc];
    if (x != 0.0)
    {
      const double ax = fabs(x);
      if (scale < ax)
      {
        ssq = 1.0 + ssq * (scale / ax) * (scale / ax);
        scale = ax;
      }
      else
        ssq += (ax / scale) * (ax / scale);
    }
  }
  return scale * sqrt(ssq);
}

/* ======================================================================
 * gsl_eigen_symmv (eigen/symmv.c + qrstep.c, linalg/symmtd.c,
 * linalg/householder.c) + gsl_eigen_symmv_sort(ABS_ASC) (eigen/sort.c).
 * Called from CMAES::eigen, CMAES.cpp.base:896-938.
 * ==================================================================== */

/* gsl_linalg_householder_transform on v[0..n) with stride inc */
static double householder_transform(size_t n, double *v, size_t inc)
{
  double alpha, beta, tau, xnorm, s;
  size_t i;
  if (n == 1) return 0.0;
  xnorm = kr_dnrm2(n - 1, v + inc, inc);
  if (xnorm == 0) return 0.0;
  alpha = v[0];
  beta = -(alpha >= 0.0 ? 1.0 : -1.0) * kr_hypot(alpha, xnorm);
  tau = (beta - alpha) / beta;
  s = (alpha - beta);
  if (fabs(s) > KR_DBL_MIN)
  {
    const double f = 1.0 / s;
    for (i = 1; i < n; i++) v[i * inc] *= f;
  }
  else
  {
    const double f1 = KR_DBL_EPSILON / s, f2 = 1.0 / KR_DBL_EPSILON;
    for (i = 1; i < n; i++) v[i * inc] *= f1;
    for (i = 1; i < n; i++) v[i * inc] *= f2;
  }
  v[0] = beta;
  return tau;
}

/* gsl_linalg_symmtd_decomp; tau has n-1 entries (scratch x overlaps it) */
static void symmtd_decomp(size_t N, double *A, double *tau)
{
  size_t i, r, j;
  for (i = 0; i + 2 < N; i++)
  {
    const size_t n = N - (i + 1);
    double *v = A + (i + 1) * N + i; /* column i below the diagonal, stride N */
    double tau_i = householder_transform(n, v, N);
    if (tau_i != 0.0)
    {
      double *m = A + (i + 1) * N + (i + 1); /* submatrix, lda N */
      double *x = tau + i;                   /* length n */
      double ei = v[0];
      double xv, alpha;
      v[0] = 1.0;
      /* dsymv RowMajor Lower, alpha=tau_i, beta=0 */
      for (r = 0; r < n; r++) x[r] = 0.0;
      for (r = n; r > 0 && r--;)
      {
        double temp1 = tau_i * v[r * N];
        double temp2 = 0.0;
        x[r] += temp1 * m[r * N + r];
        for (j = 0; j < r; j++)
        {
          x[j] += temp1 * m[r * N + j];
          temp2 += v[j * N] * m[r * N + j];
        }
        x[r] += tau_i * temp2;
      }
      /* w = x - (tau/2)(x'v) v */
      xv = 0.0;
      for (r = 0; r < n; r++) xv += x[r] * v[r * N];
      alpha = -(tau_i / 2.0) * xv;
      for (r = 0; r < n; r++) x[r] += alpha * v[r * N];
      /* dsyr2 RowMajor Lower, alpha=-1: A -= v w' + w v' */
      for (r = 0; r < n; r++)
      {
        const double tmp1 = -1.0 * v[r * N];
        const double tmp2 = -1.0 * x[r];
        for (j = 0; j <= r; j++) m[r * N + j] += tmp1 * x[j] + tmp2 * v[j * N];
      }
      v[0] = ei;
    }
    tau[i] = tau_i;
  }
}

/* gsl_linalg_symmtd_decomp alone (checker of the device library's host
 * tridiagonalisation, kg_debug_host_tridiag); tau needs N - 1 entries */
void kr_symmtd_decomp(size_t N, double *A, double *tau) { symmtd_decomp(N, A, tau); }

/* gsl_linalg_householder_hm(tau, h (h0 := 1), Q[i+1:, i+1:]) */
static void householder_hm(size_t n, double tau, const double *h, size_t hinc, double *Q, size_t lda)
{
  size_t i, j;
  if (tau == 0.0) return;
  for (j = 0; j < n; j++)
  {
    double wj = Q[j];
    for (i = 1; i < n; i++) wj += Q[i * lda + j] * h[i * hinc];
    Q[j] = Q[j] - tau * wj;
    for (i = 1; i < n; i++) Q[i * lda + j] = Q[i * lda + j] - tau * h[i * hinc] * wj;
  }
}

static void chop_small_elements(size_t N, const double *d, double *sd)
{
  double d_i = d[0];
  size_t i;
  for (i = 0; i + 1 < N; i++)
  {
    double sd_i = sd[i];
    double d_ip1 = d[i + 1];
    if (fabs(sd_i) < KR_DBL_EPSILON * (fabs(d_i) + fabs(d_ip1))) sd[i] = 0.0;
    d_i = d_ip1;
  }
}

static double trailing_eigenvalue(size_t n, const double *d, const double *sd)
{
  double ta = d[n - 2];
  double tb = d[n - 1];
  double tab = sd[n - 2];
  double dt = (ta - tb) / 2.0;
  double mu;
  if (dt > 0)
    mu = tb - tab * (tab / (dt + kr_hypot(dt, tab)));
  else if (dt == 0)
    mu = tb - fabs(tab);
  else
    mu = tb + tab * (tab / ((-dt) + kr_hypot(dt, tab)));
  return mu;
}

static void create_givens(double a, double b, double *c, double *s)
{
  if (b == 0)
  {
    *c = 1;
    *s = 0;
  }
  else if (fabs(b) > fabs(a))
  {
    double t = -a / b;
    double s1 = 1.0 / sqrt(1 + t * t);
    *s = s1;
    *c = s1 * t;
  }
  else
  {
    double t = -b / a;
    double c1 = 1.0 / sqrt(1 + t * t);
    *c = c1;
    *s = c1 * t;
  }
}

static void qrstep(size_t n, double *d, double *sd, double *gc, double *gs)
{
  double x, z, ak, bk, zk, ap, bp, aq, bq;
  size_t k;
  double mu = trailing_eigenvalue(n, d, sd);
  if (KR_DBL_EPSILON * fabs(mu) > (fabs(d[0]) + fabs(sd[0]))) mu = 0;
  x = d[0] - mu;
  z = sd[0];
  ak = 0;
  bk = 0;
  zk = 0;
  ap = d[0];
  bp = sd[0];
  aq = d[1];
  if (n == 2)
  {
    double c, s;
    create_givens(x, z, &c, &s);
    gc[0] = c;
    gs[0] = s;
    {
      double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
      double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
      double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
      ak = ap1;
      bk = bp1;
      ap = aq1;
    }
    d[0] = ak;
    sd[0] = bk;
    d[1] = ap;
    return;
  }
  bq = sd[1];
  for (k = 0; k < n - 1; k++)
  {
    double c, s;
    create_givens(x, z, &c, &s);
    gc[k] = c;
    gs[k] = s;
    {
      double bk1 = c * bk - s * zk;
      double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
      double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
      double zp1 = -s * bq;
      double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
      double bq1 = c * bq;
      ak = ap1;
      bk = bp1;
      zk = zp1;
      ap = aq1;
      bp = bq1;
      if (k < n - 2) aq = d[k + 2];
      if (k < n - 3) bq = sd[k + 2];
      d[k] = ak;
      if (k > 0) sd[k - 1] = bk1;
      if (k < n - 2) sd[k + 1] = bp;
      x = bk;
      z = zk;
    }
  }
  d[k] = ap;
  sd[k - 1] = bk;
}

static size_t eigen_symmv(size_t N, double *A, double *eval, double *evec, int sort);
size_t kr_eigen_symmv(size_t N, double *A, double *eval, double *evec) { return eigen_symmv(N, A, eval, evec, 1); }
/* gsl_eigen_symmv without gsl_eigen_symmv_sort (TMCMC.cpp.base:468) */
size_t kr_eigen_symmv_unsorted(size_t N, double *A, double *eval, double *evec) { return eigen_symmv(N, A, eval, evec, 0); }

/* the QR loop of eigen_symmv alone (symmv.c main loop + qrstep) on a given
 * tridiagonal d / sd (both overwritten): the rotation sequence (c, s) in
 * order into cs (2 per rotation, up to maxRot) and the unsorted eigenvalues
 * in d; returns the rotation count (checker of the device library's host
 * chase, kg_debug_qr_chase) */
size_t kr_qr_chase(size_t N, double *d, double *sd, double *cs, size_t maxRot)
{
  double *gc = (double *)malloc(sizeof(double) * N), *gs = (double *)malloc(sizeof(double) * N);
  size_t b = N - 1, rot = 0;
  chop_small_elements(N, d, sd);
  while (b > 0)
  {
    size_t a, k;
    if (sd[b - 1] == 0.0 || isnan(sd[b - 1]))
    {
      b--;
      continue;
    }
    a = b - 1;
    while (a > 0)
    {
      if (sd[a - 1] == 0.0) break;
      a--;
    }
    qrstep(b - a + 1, d + a, sd + a, gc, gs);
    for (k = 0; k + 1 < b - a + 1 && rot < maxRot; k++, rot++)
    {
      cs[2 * rot] = gc[k];
      cs[2 * rot + 1] = gs[k];
    }
    chop_small_elements(b - a + 1, d + a, sd + a);
  }
  free(gc);
  free(gs);
  return rot;
}
static size_t eigen_symmv(size_t N, double *A, double *eval, double *evec, int sort)
{
  size_t i, steps = 0;
  double *d, *sd, *gc, *gs;
  if (N == 1)
  {
    eval[0] = A[0];
    evec[0] = 1.0;
    return 0;
  }
  d = (double *)malloc(sizeof(double) * N);
  sd = (double *)malloc(sizeof(double) * N);
  gc = (double *)malloc(sizeof(double) * N);
  gs = (double *)malloc(sizeof(double) * N);

  symmtd_decomp(N, A, sd); /* tau lives in sd (symmv.c) */
  /* symmtd_unpack: Q = I; apply H_i for i = N-3 .. 0 */
  memset(evec, 0, sizeof(double) * N * N);
  for (i = 0; i < N; i++) evec[i * N + i] = 1.0;
  for (i = N - 2; i-- > 0;)
  {
    const double *h = A + (i + 1) * N + i;
    householder_hm(N - (i + 1), sd[i], h, N, evec + (i + 1) * N + (i + 1), N);
  }
  for (i = 0; i < N; i++) d[i] = A[i * N + i];
  for (i = 0; i + 1 < N; i++) sd[i] = A[(i + 1) * N + i];

  chop_small_elements(N, d, sd);
  {
    size_t b = N - 1;
    while (b > 0)
    {
      size_t a;
      if (sd[b - 1] == 0.0 || isnan(sd[b - 1]))
      {
        b--;
        continue;
      }
      a = b - 1;
      while (a > 0)
      {
        if (sd[a - 1] == 0.0) break;
        a--;
      }
      {
        const size_t n_block = b - a + 1;
        size_t k, r;
        qrstep(n_block, d + a, sd + a, gc, gs);
        steps++;
        for (k = 0; k + 1 < n_block; k++)
        {
          const double c = gc[k], s = gs[k];
          for (r = 0; r < N; r++)
          {
            double qki = evec[r * N + a + k];
            double qkj = evec[r * N + a + k + 1];
            evec[r * N + a + k] = qki * c - qkj * s;
            evec[r * N + a + k + 1] = qki * s + qkj * c;
          }
        }
        chop_small_elements(n_block, d + a, sd + a);
      }
    }
  }
  for (i = 0; i < N; i++) eval[i] = d[i];

  /* gsl_eigen_symmv_sort(ABS_ASC): selection sort, strict < on |e| */
  for (i = 0; sort && i + 1 < N; i++)
  {
    size_t j, k = i;
    double ek = eval[i];
    for (j = i + 1; j < N; j++)
    {
      const double ej = eval[j];
      if (fabs(ej) < fabs(ek))
      {
        k = j;
        ek = ej;
      }
    }
    if (k != i)
    {
      size_t r;
      double t = eval[i];
      eval[i] = eval[k];
      eval[k] = t;
      for (r = 0; r < N; r++)
      {
        double q = evec[r * N + i];
        evec[r * N + i] = evec[r * N + k];
        evec[r * N + k] = q;
      }
    }
  }
  free(d);
  free(sd);
  free(gc);
  free(gs);
  return steps;
}

/* gsl_linalg_cholesky_decomp1 (linalg/cholesky.c, Level-2 form) with
 * gslcblas dgemv loop order; Korali TMCMC.cpp.base:205-213 */
int kr_cholesky(size_t N, double *A)
{
  size_t i, j, r;
  for (j = 0; j < N; ++j)
  {
    double ajj, f;
    if (j > 0)
    {
      for (r = j; r < N; r++)
      {
        double temp = 0.0;
        for (i = 0; i < j; i++) temp += A[j * N + i] * A[r * N + i];
        A[r * N + j] += -1.0 * temp;
      }
    }
    ajj = A[j * N + j];
    if (ajj <= 0.0) return 1;
    ajj = sqrt(ajj);
    f = 1.0 / ajj;
    for (r = j; r < N; r++) A[r * N + j] *= f;
  }
  for (j = 1; j < N; ++j)
    for (i = 0; i < j; ++i) A[i * N + j] = A[j * N + i];
  return 0;
}

/* gslcblas dtrmv RowMajor, Lower, NoTrans, NonUnit */
void kr_dtrmv_lower(size_t N, const double *L, double *X)
{
  size_t i, j;
  for (i = N; i > 0 && i--;)
  {
    double temp = 0.0;
    for (j = 0; j < i; j++) temp += X[j] * L[N * i + j];
    X[i] = temp + X[i] * L[N * i + i];
  }
}

/* gsl_stats_mean / gsl_stats_sd_m: long double running recurrences */
double kr_stats_mean(const double *x, size_t n)
{
  long double mean = 0;
  size_t i;
  for (i = 0; i < n; i++) mean += (x[i] - mean) / (i + 1);
  return (double)mean;
}

double kr_stats_sd_m(const double *x, size_t n, double mean)
{
  long double variance = 0;
  size_t i;
  double var_d;
  for (i = 0; i < n; i++)
  {
    const long double delta = (x[i] - mean);
    variance += (delta * delta - variance) / (i + 1);
  }
  var_d = (double)variance;
  return sqrt(var_d * ((double)n / (double)(n - 1)));
}

/* ======================================================================
 * Analytic objectives: examples/optimization/stochastic/_model/model.py
 * (negative_rosenbrock :23-34, negative_ackley :37-62, negative_sphere) and
 * tests/statistical/samplers/mean/model/model.py:32-37 (lgaussianxdCustom).
 * Squares are written x*x (the Python '**2').
 * ==================================================================== */
double kr_obj_negative_rosenbrock(const double *x, size_t n)
{
  double res = 0.;
  size_t i;
  for (i = 0; i + 1 < n; i++)
  {
    const double t = x[i + 1] - x[i] * x[i];
    const double u = 1 - x[i];
    res += 100 * (t * t) + u * u;
  }
  return -res;
}

double kr_obj_negative_ackley(const double *x, size_t n)
{
  const double a = 20., b = 0.2, c = 2. * 3.141592653589793;
  double sum1 = 0., sum2 = 0., r1, r2;
  size_t i;
  for (i = 0; i < n; i++)
  {
    sum1 += x[i] * x[i];
    sum2 += kr_cos_cr(c * x[i]);
  }
  sum1 /= (double)n;
  sum2 /= (double)n;
  r1 = a * kr_exp_cr(-b * sqrt(sum1));
  r2 = kr_exp_cr(sum2);
  return r1 + r2 - a - 2.718281828459045;
}

double kr_obj_negative_sphere(const double *x, size_t n)
{
  double res = 0.;
  size_t i;
  for (i = 0; i < n; i++) res += x[i] * x[i];
  return -0.5 * res;
}

double kr_loglik_gaussian(const double *x, size_t n)
{
  double ss = 0.0;
  size_t i;
  for (i = 0; i < n; i++) ss += x[i] * x[i];
  return -0.5 * ss;
}

/* ======================================================================
 * CMA-ES — source/modules/solver/optimizer/CMAES/CMAES.cpp.base
 * ==================================================================== */
struct kr_cmaes
{
  size_t N, lambda, mu;
  /* options (CMAES.config defaults) */
  int muType; /* 0 Logarithmic, 1 Linear, 2 Equal, 3 Proportional */
  double initialSigmaCumulationFactor, initialDampFactor, initialCumulativeCovariance;
  int isSigmaBounded, diagonal, mirrored;
  double maxInfeasibleResamplings;
  /* variables */
  double *lowerBound, *upperBound, *initialValue, *initialStd, *minStdUpdate;
  /* vectors */
  double *currentMean, *previousMean, *C, *B, *D, *pc, *ps, *muWeights;
  double *X, *BDZ, *F, *bestEverVariables, *currentBestVariables, *meanUpdate, *auxBDZ;
  double *auxAxisLengths, *auxEvec;
  size_t *sortingIndex;
  /* scalars */
  double sigma, trace, effectiveMu, cumulativeCovariance, sigmaCumulationFactor, dampFactor, chiSquareNumber;
  double psNorm, bestEverValue, previousBestEverValue, previousBestValue, currentBestValue;
  double currentMinStd, currentMaxStd, maxDiagC, minDiagC, minEig, maxEig;
  double infeasibleSampleCount, bestValidSample, modelEvaluationCount, hsig, eigenFailures;
  kr_rng normal, uniform;
  /* "Use Gradient Information" (CMAES.cpp.base:82-87, :611-621): the
   * samples' "Gradient" (lambda x N) and the step size */
  int useGradients;
  double gradientStepSize;
  double *gradients;
  /* discrete variables (CMAES.cpp.base:34, :44-50, :101-107, :515-544,
   * :834-867): Granularity per variable, the masking vectors and the
   * discrete-mutation bookkeeping */
  double *granularity, *maskingMatrix, *maskingMatrixSigma, *discreteMutations;
  double numberMaskingMatrixEntries, numberOfDiscreteMutations, chiSquareNumberDiscreteMutations;
  int hasDiscrete;
  /* configured Population Size / Mu Value; lambda / mu above are the
   * CURRENT ones (_currentPopulationSize / _currentMuValue), which differ
   * during CCMA-ES's viability regime */
  size_t populationSize, muValue, smax, mumax;
  /* CCMA-ES (Problem "Constraints"; CMAES.cpp.base:54-68, :132-170,
   * :315-437, :551-580, :724-731, :774-832) */
  int hasConstraints, isViabilityRegime;
  size_t nc, viabilityPopulationSize, viabilityMuValue;
  double maxCovarianceMatrixCorrections, targetSuccessRate, covarianceMatrixAdaptionStrength, globalSuccessLearningRate;
  double normalVectorLearningRate, covarianceMatrixAdaptionFactor, globalSuccessRate;
  double constraintEvaluationCount, covarianceMatrixAdaptationCount, maxConstraintViolationCount, resampledParameterCount;
  double *constraintEvaluations;  /* [c][i], nc x smax */
  double *viabilityIndicator;     /* [c][i] as 0 / 1 */
  double *sampleConstraintViolationCounts, *viabilityBoundaries, *normalConstraintApproximation;
  double *bestConstraintEvaluations, *auxC;
  kr_constraint_fn constraintFn;
  void *constraintCtx;
  int constraintError; /* the reference's out-of-range _bestValidSample (no valid sample) */
};

kr_cmaes *kr_cmaes_new(size_t N, size_t lambda, size_t mu)
{
  kr_cmaes *h = (kr_cmaes *)calloc(1, sizeof(kr_cmaes));
  size_t i;
  h->N = N;
  h->lambda = lambda;
  h->mu = mu == 0 ? lambda / 2 : mu; /* CMAES.cpp.base:27 */
  h->muType = 0;
  h->initialSigmaCumulationFactor = -1.0;
  h->initialDampFactor = -1.0;
  h->initialCumulativeCovariance = -1.0;
  h->maxInfeasibleResamplings = INFINITY;
#define AL(p, n) p = (double *)calloc((n), sizeof(double))
  AL(h->lowerBound, N);
  AL(h->upperBound, N);
  AL(h->initialValue, N);
  AL(h->initialStd, N);
  AL(h->minStdUpdate, N);
  for (i = 0; i < N; i++)
  {
    h->lowerBound[i] = -INFINITY;
    h->upperBound[i] = INFINITY;
    h->initialValue[i] = NAN;
    h->initialStd[i] = NAN;
  }
  AL(h->currentMean, N);
  AL(h->previousMean, N);
  AL(h->C, N * N);
  AL(h->B, N * N);
  AL(h->D, N);
  AL(h->pc, N);
  AL(h->ps, N);
  AL(h->muWeights, h->mu);
  AL(h->X, lambda * N);
  AL(h->BDZ, lambda * N);
  AL(h->F, lambda);
  AL(h->bestEverVariables, N);
  AL(h->currentBestVariables, N);
  AL(h->meanUpdate, N);
  AL(h->auxBDZ, N);
  AL(h->auxAxisLengths, N);
  AL(h->auxEvec, N * N);
  AL(h->granularity, N);
  AL(h->maskingMatrix, N);
  AL(h->maskingMatrixSigma, N);
  AL(h->discreteMutations, lambda * N);
#undef AL
  h->sortingIndex = (size_t *)calloc(lambda, sizeof(size_t));
  h->populationSize = h->smax = lambda;
  h->muValue = h->mumax = h->mu;
  kr_rng_seed(&h->normal, 0);
  kr_rng_seed(&h->uniform, 0);
  return h;
}

void kr_cmaes_free(kr_cmaes *h)
{
  if (!h) return;
  free(h->gradients);
  free(h->lowerBound);
  free(h->upperBound);
  free(h->initialValue);
  free(h->initialStd);
  free(h->minStdUpdate);
  free(h->currentMean);
  free(h->previousMean);
  free(h->C);
  free(h->B);
  free(h->D);
  free(h->pc);
  free(h->ps);
  free(h->muWeights);
  free(h->X);
  free(h->BDZ);
  free(h->F);
  free(h->bestEverVariables);
  free(h->currentBestVariables);
  free(h->meanUpdate);
  free(h->auxBDZ);
  free(h->auxAxisLengths);
  free(h->auxEvec);
  free(h->granularity);
  free(h->maskingMatrix);
  free(h->maskingMatrixSigma);
  free(h->discreteMutations);
  free(h->sortingIndex);
  free(h->constraintEvaluations);
  free(h->viabilityIndicator);
  free(h->sampleConstraintViolationCounts);
  free(h->viabilityBoundaries);
  free(h->normalConstraintApproximation);
  free(h->bestConstraintEvaluations);
  free(h->auxC);
  free(h);
}

/* Problem "Constraints" (nc functions, evaluated by fn in the reference's
 * order: sample.run(_constraints[c]) for c = 0..nc-1, optimization.cpp.base:
 * 11-24) and the CCMA-ES sizes (CMAES.cpp.base:25-30): every per-sample array
 * grows to max(Population Size, Viability Population Size) */
void kr_cmaes_set_constraints(kr_cmaes *h, size_t nc, size_t viabilityPopulationSize, size_t viabilityMuValue,
                              kr_constraint_fn fn, void *ctx)
{
  const size_t N = h->N;
  h->nc = nc;
  h->hasConstraints = nc > 0;
  h->constraintFn = fn;
  h->constraintCtx = ctx;
  h->viabilityPopulationSize = viabilityPopulationSize;
  h->viabilityMuValue = viabilityMuValue ? viabilityMuValue : viabilityPopulationSize / 2;
  h->smax = h->populationSize > viabilityPopulationSize ? h->populationSize : viabilityPopulationSize;
  h->mumax = h->muValue > h->viabilityMuValue ? h->muValue : h->viabilityMuValue;
#define RE(p, n) p = (double *)realloc(p, sizeof(double) * (n)), memset(p, 0, sizeof(double) * (n))
  RE(h->X, h->smax * N);
  RE(h->BDZ, h->smax * N);
  RE(h->F, h->smax);
  RE(h->discreteMutations, h->smax * N);
  RE(h->muWeights, h->mumax);
  RE(h->constraintEvaluations, nc * h->smax + 1);
  RE(h->viabilityIndicator, nc * h->smax + 1);
  RE(h->sampleConstraintViolationCounts, h->smax);
  RE(h->viabilityBoundaries, nc + 1);
  RE(h->normalConstraintApproximation, nc * N + 1);
  RE(h->bestConstraintEvaluations, nc + 1);
  RE(h->auxC, N * N);
#undef RE
  h->sortingIndex = (size_t *)realloc(h->sortingIndex, sizeof(size_t) * h->smax);
  if (h->gradients) h->gradients = (double *)realloc(h->gradients, sizeof(double) * h->smax * N);
  h->maxCovarianceMatrixCorrections = 1000000; /* CMAES.config defaults */
  h->targetSuccessRate = 0.1818;
  h->covarianceMatrixAdaptionStrength = 0.1;
  h->globalSuccessLearningRate = 0.2;
}

double *kr_cmaes_field(kr_cmaes *h, const char *name, size_t *len)
{
  const size_t N = h->N;
#define VEC(key, ptr, n)            \
  if (strcmp(name, key) == 0)       \
  {                                 \
    if (len) *len = (n);            \
    return ptr;                     \
  }
#define SCA(key, var) VEC(key, &h->var, 1)
  VEC("Lower Bound", h->lowerBound, N)
  VEC("Upper Bound", h->upperBound, N)
  VEC("Initial Value", h->initialValue, N)
  VEC("Initial Standard Deviation", h->initialStd, N)
  VEC("Minimum Standard Deviation Update", h->minStdUpdate, N)
  VEC("Current Mean", h->currentMean, N)
  VEC("Previous Mean", h->previousMean, N)
  VEC("Covariance Matrix", h->C, N * N)
  VEC("Covariance Eigenvector Matrix", h->B, N * N)
  VEC("Axis Lengths", h->D, N)
  VEC("Evolution Path", h->pc, N)
  VEC("Conjugate Evolution Path", h->ps, N)
  VEC("Mu Weights", h->muWeights, h->mu)
  VEC("Sample Population", h->X, h->lambda * N)
  VEC("BDZ Matrix", h->BDZ, h->lambda * N)
  VEC("Value Vector", h->F, h->lambda)
  if (h->gradients) VEC("Gradients", h->gradients, h->lambda * h->N)
  VEC("Best Ever Variables", h->bestEverVariables, N)
  VEC("Current Best Variables", h->currentBestVariables, N)
  VEC("Mean Update", h->meanUpdate, N)
  VEC("Auxiliar BDZ Matrix", h->auxBDZ, N)
  VEC("Granularity", h->granularity, N)
  VEC("Masking Matrix", h->maskingMatrix, N)
  VEC("Masking Matrix Sigma", h->maskingMatrixSigma, N)
  VEC("Discrete Mutations", h->discreteMutations, h->lambda * N)
  SCA("Number Masking Matrix Entries", numberMaskingMatrixEntries)
  SCA("Number Of Discrete Mutations", numberOfDiscreteMutations)
  SCA("Chi Square Number Discrete Mutations", chiSquareNumberDiscreteMutations)
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
  if (h->hasConstraints)
  {
    VEC("Constraint Evaluations", h->constraintEvaluations, h->nc * h->smax)
    VEC("Viability Indicator", h->viabilityIndicator, h->nc * h->smax)
    VEC("Sample Constraint Violation Counts", h->sampleConstraintViolationCounts, h->lambda)
    VEC("Viability Boundaries", h->viabilityBoundaries, h->nc)
    VEC("Normal Constraint Approximation", h->normalConstraintApproximation, h->nc * N)
    VEC("Best Constraint Evaluations", h->bestConstraintEvaluations, h->nc)
  }
  SCA("Global Success Rate", globalSuccessRate)
  SCA("Covariance Matrix Adaption Factor", covarianceMatrixAdaptionFactor)
  SCA("Normal Vector Learning Rate", normalVectorLearningRate)
  SCA("Constraint Evaluation Count", constraintEvaluationCount)
  SCA("Covariance Matrix Adaptation Count", covarianceMatrixAdaptationCount)
  SCA("Max Constraint Violation Count", maxConstraintViolationCount)
  SCA("Resampled Parameter Count", resampledParameterCount)
  SCA("Max Covariance Matrix Corrections", maxCovarianceMatrixCorrections)
  SCA("Target Success Rate", targetSuccessRate)
  SCA("Covariance Matrix Adaption Strength", covarianceMatrixAdaptionStrength)
  SCA("Global Success Learning Rate", globalSuccessLearningRate)
#undef VEC
#undef SCA
  if (len) *len = 0;
  return NULL;
}

size_t *kr_cmaes_sorting_index(kr_cmaes *h) { return h->sortingIndex; }
kr_rng *kr_cmaes_rng(kr_cmaes *h, int which) { return which == 0 ? &h->normal : &h->uniform; }

void kr_cmaes_set_option(kr_cmaes *h, const char *name, double v)
{
  if (strcmp(name, "Mu Type") == 0) h->muType = (int)v;
  else if (strcmp(name, "Initial Sigma Cumulation Factor") == 0) h->initialSigmaCumulationFactor = v;
  else if (strcmp(name, "Initial Damp Factor") == 0) h->initialDampFactor = v;
  else if (strcmp(name, "Initial Cumulative Covariance") == 0) h->initialCumulativeCovariance = v;
  else if (strcmp(name, "Is Sigma Bounded") == 0) h->isSigmaBounded = (int)v;
  else if (strcmp(name, "Diagonal Covariance") == 0) h->diagonal = (int)v;
  else if (strcmp(name, "Mirrored Sampling") == 0) h->mirrored = (int)v;
  else if (strcmp(name, "Use Gradient Information") == 0)
  {
    h->useGradients = (int)v;
    if (h->useGradients && !h->gradients) h->gradients = (double *)calloc(h->lambda * h->N, sizeof(double));
  }
  else if (strcmp(name, "Gradient Step Size") == 0) h->gradientStepSize = v;
  else if (strcmp(name, "Max Infeasible Resamplings") == 0) h->maxInfeasibleResamplings = v;
  else if (strcmp(name, "Max Covariance Matrix Corrections") == 0) h->maxCovarianceMatrixCorrections = v;
  else if (strcmp(name, "Target Success Rate") == 0) h->targetSuccessRate = v;
  else if (strcmp(name, "Covariance Matrix Adaption Strength") == 0) h->covarianceMatrixAdaptionStrength = v;
  else if (strcmp(name, "Global Success Learning Rate") == 0) h->globalSuccessLearningRate = v;
}

/* initMuWeights, CMAES.cpp.base:233-284 (unconstrained branch) */
static void cmaes_init_mu_weights(kr_cmaes *h, size_t numsamplesmu)
{
  size_t i;
  double s1 = 0.0, s2 = 0.0;
  const size_t N = h->N;
  for (i = 0; i < numsamplesmu; i++)
  {
    switch (h->muType)
    {
    case 1: h->muWeights[i] = (double)(numsamplesmu - i); break;
    case 2: h->muWeights[i] = 1.; break;
    case 3: h->muWeights[i] = 1.; break;
    default:
    {
      const double a = (double)numsamplesmu, b = 0.5 * (double)h->lambda;
      h->muWeights[i] = kr_log_cr((a > b ? a : b) + 0.5) - kr_log_cr(i + 1.);
    }
    }
  }
  for (i = 0; i < numsamplesmu; i++)
  {
    s1 += h->muWeights[i];
    s2 += h->muWeights[i] * h->muWeights[i];
  }
  h->effectiveMu = s1 * s1 / s2;
  for (i = 0; i < numsamplesmu; i++) h->muWeights[i] /= s1;

  if ((h->initialCumulativeCovariance <= 0) || (h->initialCumulativeCovariance > 1))
    h->cumulativeCovariance = (4.0 + h->effectiveMu / (1.0 * N)) / (N + 4.0 + 2.0 * h->effectiveMu / (1.0 * N));
  else
    h->cumulativeCovariance = h->initialCumulativeCovariance;

  h->sigmaCumulationFactor = h->initialSigmaCumulationFactor;
  if (h->sigmaCumulationFactor <= 0 || h->sigmaCumulationFactor >= 1)
  {
    if (h->hasConstraints) /* :270-273 */
      h->sigmaCumulationFactor = sqrt(h->effectiveMu) / (sqrt(h->effectiveMu) + sqrt((double)N));
    else
      h->sigmaCumulationFactor = (h->effectiveMu + 2.0) / (N + h->effectiveMu + 3.0);
  }

  h->dampFactor = h->initialDampFactor;
  if (h->dampFactor <= 0.0)
  {
    double t = sqrt((h->effectiveMu - 1.0) / (N + 1.0)) - 1;
    h->dampFactor = (1.0 + 2 * (0.0 > t ? 0.0 : t)) + h->sigmaCumulationFactor;
  }
}

/* initCovariance, CMAES.cpp.base:286-313 */
static void cmaes_init_covariance(kr_cmaes *h)
{
  const size_t N = h->N;
  size_t i;
  double mn, mx;
  h->trace = 0.0;
  for (i = 0; i < N; ++i) h->trace += h->initialStd[i] * h->initialStd[i];
  h->sigma = sqrt(h->trace / N);
  for (i = 0; i < N; ++i)
  {
    h->B[i * N + i] = 1.0;
    h->C[i * N + i] = h->D[i] = h->initialStd[i] * sqrt(N / h->trace);
    h->C[i * N + i] *= h->C[i * N + i];
  }
  mn = mx = h->D[0];
  for (i = 1; i < N; i++)
  {
    if (h->D[i] < mn) mn = h->D[i];
    if (h->D[i] > mx) mx = h->D[i];
  }
  h->minEig = mn * mn;
  h->maxEig = mx * mx;
  h->maxDiagC = h->C[0];
  for (i = 1; i < N; ++i)
    if (h->maxDiagC < h->C[i * N + i]) h->maxDiagC = h->C[i * N + i];
  h->minDiagC = h->C[0];
  for (i = 1; i < N; ++i)
    if (h->minDiagC > h->C[i * N + i]) h->minDiagC = h->C[i * N + i];
}

/* setInitialConfiguration, CMAES.cpp.base:14-184 (no constraints) */
void kr_cmaes_initialize(kr_cmaes *h)
{
  const size_t N = h->N;
  size_t i;
  /* :34, :44-50, :101-107 */
  h->chiSquareNumberDiscreteMutations = sqrt((double)N) * (1. - 1. / (4. * N) + 1. / (21. * N * N));
  h->hasDiscrete = 0;
  for (i = 0; i < N; i++)
    if (h->granularity[i] > 0.0) h->hasDiscrete = 1;
  memset(h->discreteMutations, 0, sizeof(double) * h->lambda * N);
  memset(h->maskingMatrix, 0, sizeof(double) * N);
  memset(h->maskingMatrixSigma, 0, sizeof(double) * N);
  h->numberMaskingMatrixEntries = 0;
  h->numberOfDiscreteMutations = 0;
  h->bestEverValue = -INFINITY;
  h->previousBestEverValue = h->bestEverValue;
  h->previousBestValue = h->bestEverValue;
  h->currentBestValue = h->bestEverValue;
  h->chiSquareNumber = sqrt((double)N) * (1. - 1. / (4. * N) + 1. / (21. * N * N));
  for (i = 0; i < N; ++i)
  {
    if (!isfinite(h->initialValue[i])) h->initialValue[i] = (h->upperBound[i] + h->lowerBound[i]) * 0.5;
    if (!isfinite(h->initialStd[i])) h->initialStd[i] = (h->upperBound[i] - h->lowerBound[i]) * 0.3;
  }
  h->bestValidSample = 0;
  memset(h->C, 0, sizeof(double) * N * N);
  memset(h->B, 0, sizeof(double) * N * N);
  /* :54-66 regime and current sizes; :132-165 constraint state */
  h->isViabilityRegime = h->hasConstraints;
  h->lambda = h->isViabilityRegime ? h->viabilityPopulationSize : h->populationSize;
  h->mu = h->isViabilityRegime ? h->viabilityMuValue : h->muValue;
  if (h->hasConstraints)
  {
    h->globalSuccessRate = 0.5;
    h->bestValidSample = -1;
    memset(h->constraintEvaluations, 0, sizeof(double) * h->nc * h->smax);
    memset(h->viabilityIndicator, 0, sizeof(double) * h->nc * h->smax);
    memset(h->sampleConstraintViolationCounts, 0, sizeof(double) * h->smax);
    memset(h->viabilityBoundaries, 0, sizeof(double) * h->nc);
    memset(h->normalConstraintApproximation, 0, sizeof(double) * h->nc * N);
    memset(h->bestConstraintEvaluations, 0, sizeof(double) * h->nc);
    h->normalVectorLearningRate = 1.0 / (2.0 + N);
    h->covarianceMatrixAdaptionFactor = h->covarianceMatrixAdaptionStrength / (N + 2.);
  }
  else
  {
    h->globalSuccessRate = -1.0;
    h->covarianceMatrixAdaptionFactor = -1.0;
  }
  h->covarianceMatrixAdaptationCount = 0;
  h->maxConstraintViolationCount = 0;
  h->resampledParameterCount = 0;
  cmaes_init_mu_weights(h, h->mu);
  cmaes_init_covariance(h);
  h->infeasibleSampleCount = 0;
  h->psNorm = 0.0;
  for (i = 0; i < N; i++) h->currentMean[i] = h->previousMean[i] = h->initialValue[i];
  h->currentMinStd = INFINITY;
  h->currentMaxStd = -INFINITY;
}

/* updateEigensystem(M), CMAES.cpp.base:869-890 (+ eigen :896-938) */
static void cmaes_update_eigensystem(kr_cmaes *h, const double *M)
{
  const size_t N = h->N;
  size_t i, j;
  double mn, mx;
  if (h->diagonal)
  {
    memset(h->auxEvec, 0, sizeof(double) * N * N);
    for (i = 0; i < N; ++i) h->auxEvec[i * N + i] = 1.;
    for (i = 0; i < N; ++i) h->auxAxisLengths[i] = M[i * N + i];
  }
  else
  {
    double *data = (double *)malloc(sizeof(double) * N * N);
    for (i = 0; i < N; i++)
      for (j = 0; j <= i; j++)
      {
        data[i * N + j] = M[i * N + j];
        data[j * N + i] = M[i * N + j];
      }
    kr_eigen_symmv(N, data, h->auxAxisLengths, h->auxEvec);
    free(data);
  }
  mn = mx = h->auxAxisLengths[0];
  for (i = 1; i < N; i++)
  {
    if (h->auxAxisLengths[i] < mn) mn = h->auxAxisLengths[i];
    if (h->auxAxisLengths[i] > mx) mx = h->auxAxisLengths[i];
  }
  if (mn <= 0.0)
  {
    h->eigenFailures += 1;
    return;
  }
  for (i = 0; i < N; i++) h->auxAxisLengths[i] = sqrt(h->auxAxisLengths[i]);
  h->minEig = mn;
  h->maxEig = mx;
  for (i = 0; i < N; i++) h->D[i] = h->auxAxisLengths[i];
  memcpy(h->B, h->auxEvec, sizeof(double) * N * N);
}

void kr_cmaes_eigen_only(kr_cmaes *h) { cmaes_update_eigensystem(h, h->C); }

/* discretize, CMAES.cpp.base:861-867 */
static void cmaes_discretize(const kr_cmaes *h, double *x)
{
  size_t d;
  for (d = 0; d < h->N; ++d)
    if (h->granularity[d] != 0.0) x[d] = round(x[d] / h->granularity[d]) * h->granularity[d];
}

/* sampleSingle, CMAES.cpp.base:494-545 */
static void cmaes_sample_single(kr_cmaes *h, size_t idx, const double *z)
{
  const size_t N = h->N;
  size_t d, e;
  double *bdz = h->BDZ + idx * N, *x = h->X + idx * N;
  for (d = 0; d < N; ++d)
  {
    if (h->diagonal)
    {
      bdz[d] = h->D[d] * z[d];
      x[d] = h->currentMean[d] + h->sigma * bdz[d];
    }
    else
      h->auxBDZ[d] = h->D[d] * z[d];
  }
  if (!h->diagonal)
    for (d = 0; d < N; ++d)
    {
      bdz[d] = 0.0;
      for (e = 0; e < N; ++e) bdz[d] += h->B[d * N + e] * h->auxBDZ[e];
      x[d] = h->currentMean[d] + h->sigma * bdz[d];
    }
  if (h->hasDiscrete)
  {
    /* :515-544: a geometric +-mutation of one masked variable for the first
     * numberOfDiscreteMutations - 1 samples, the best-ever point rounded for
     * the next one (uniforms from the solver's Uniform Generator) */
    if ((double)(idx + 1) < h->numberOfDiscreteMutations)
    {
      const double p_geom = kr_pow_cr(0.7, 1.0 / h->numberMaskingMatrixEntries);
      size_t select = (size_t)floor(kr_ran_flat(&h->uniform, 0.0, 1.0) * h->numberMaskingMatrixEntries);
      for (d = 0; d < N; ++d)
        if ((h->maskingMatrix[d] == 1.0) && (select-- == 0))
        {
          double dmutation = 1.0;
          while (kr_ran_flat(&h->uniform, 0.0, 1.0) > p_geom) dmutation += 1.0;
          dmutation *= h->granularity[d];
          if (kr_ran_flat(&h->uniform, 0.0, 1.0) > 0.5) dmutation *= -1.0;
          h->discreteMutations[idx * N + d] = dmutation;
          x[d] += dmutation;
        }
    }
    else if ((double)(idx + 1) == h->numberOfDiscreteMutations)
    {
      for (d = 0; d < N; ++d)
        if (h->granularity[d] != 0.0)
        {
          const double dmutation = round(h->bestEverVariables[d] / h->granularity[d]) * h->granularity[d] - x[d];
          h->discreteMutations[idx * N + d] = dmutation;
          x[d] += dmutation;
        }
    }
  }
}

/* Optimizer::isSampleFeasible, optimizer.cpp.base:5-14 */
static int cmaes_feasible(const kr_cmaes *h, const double *x)
{
  size_t d;
  for (d = 0; d < h->N; d++)
  {
    if (isfinite(x[d]) == 0) return 0;
    if (x[d] < h->lowerBound[d]) return 0;
    if (x[d] > h->upperBound[d]) return 0;
  }
  return 1;
}

/* x_i = m + sigma B (D o z_i) for samples [0, lambda) from normals drawn in
 * stream order beforehand (the loop of sampleSingle, CMAES.cpp.base:494-545,
 * per sample; samples are independent) */
static void cmaes_sample_all(kr_cmaes *h, const double *Z)
{
  const size_t N = h->N;
  long i;
#pragma omp parallel
  {
    double *aux = (double *)malloc(sizeof(double) * N);
#pragma omp for schedule(static)
    for (i = 0; i < (long)h->lambda; ++i)
    {
      const double *z = Z + (size_t)i * N;
      double *bdz = h->BDZ + (size_t)i * N, *x = h->X + (size_t)i * N;
      size_t d, e;
      for (d = 0; d < N; ++d)
      {
        if (h->diagonal)
        {
          bdz[d] = h->D[d] * z[d];
          x[d] = h->currentMean[d] + h->sigma * bdz[d];
        }
        else
          aux[d] = h->D[d] * z[d];
      }
      if (!h->diagonal)
        for (d = 0; d < N; ++d)
        {
          bdz[d] = 0.0;
          for (e = 0; e < N; ++e) bdz[d] += h->B[d * N + e] * aux[e];
          x[d] = h->currentMean[d] + h->sigma * bdz[d];
        }
    }
    free(aux);
  }
}

/* draw loop of prepareGeneration, CMAES.cpp.base:443-491 */
void kr_cmaes_sample_only(kr_cmaes *h)
{
  const size_t N = h->N;
  size_t i, d;
  double *r1 = (double *)malloc(sizeof(double) * N), *r2 = (double *)malloc(sizeof(double) * N);
  if (!h->mirrored)
  {
    /* fast form: draw every normal first (stream order), transform the
     * samples in parallel, then check feasibility in sample order; on the
     * first infeasible sample rewind the generator and replay the
     * reference's sequential resampling loop below */
    kr_rng saved = h->normal;
    double *Z = (double *)malloc(sizeof(double) * N * h->lambda);
    int all_ok = !h->hasDiscrete; /* discrete variables: the sequential loop below */
    kr_ran_gaussian_n(&h->normal, h->lambda * N, Z);
    cmaes_sample_all(h, Z);
    for (i = 0; i < h->lambda && all_ok; ++i) all_ok = cmaes_feasible(h, h->X + i * N);
    if (all_ok && !h->diagonal)
      for (d = 0; d < N; ++d) h->auxBDZ[d] = h->D[d] * Z[(h->lambda - 1) * N + d];
    free(Z);
    if (all_ok)
    {
      free(r1);
      free(r2);
      return;
    }
    h->normal = saved;
    for (i = 0; i < h->lambda; ++i)
    {
      int ok;
      do
      {
        for (d = 0; d < N; ++d) r1[d] = 0.0 + kr_ran_gaussian(&h->normal, 1.0);
        cmaes_sample_single(h, i, r1);
        if (h->hasDiscrete) cmaes_discretize(h, h->X + i * N);
        ok = cmaes_feasible(h, h->X + i * N);
        h->infeasibleSampleCount += ok ? 0 : 1;
      } while (ok == 0 && (h->infeasibleSampleCount < h->maxInfeasibleResamplings));
    }
  }
  else
  {
    for (i = 0; i < h->lambda; i += 2)
    {
      int ok;
      do
      {
        int ok1, ok2;
        for (d = 0; d < N; ++d)
        {
          r1[d] = 0.0 + kr_ran_gaussian(&h->normal, 1.0);
          r2[d] = -r1[d];
        }
        cmaes_sample_single(h, i, r1);
        cmaes_sample_single(h, i + 1, r2);
        if (h->hasDiscrete)
        {
          cmaes_discretize(h, h->X + i * N);
          cmaes_discretize(h, h->X + (i + 1) * N);
        }
        ok1 = cmaes_feasible(h, h->X + i * N);
        if (!ok1) h->infeasibleSampleCount++;
        ok2 = cmaes_feasible(h, h->X + (i + 1) * N);
        if (!ok2) h->infeasibleSampleCount++;
        ok = ok1 || ok2;
      } while (ok == 0 && (h->infeasibleSampleCount < h->maxInfeasibleResamplings));
    }
  }
  free(r1);
  free(r2);
}

void kr_cmaes_prepare(kr_cmaes *h)
{
  kr_cmaes_eigen_only(h);
  kr_cmaes_sample_only(h);
}

void kr_cmaes_evaluate(kr_cmaes *h, int objective)
{
  long i;
#pragma omp parallel for schedule(static)
  for (i = 0; i < (long)h->lambda; i++)
  {
    double *x = h->X + (size_t)i * h->N;
    double f;
    if (h->hasDiscrete) cmaes_discretize(h, x); /* :208 */
    if (objective == 0) f = kr_obj_negative_rosenbrock(x, h->N);
    else if (objective == 1) f = kr_obj_negative_ackley(x, h->N);
    else f = kr_obj_negative_sphere(x, h->N);
    h->F[i] = f;
  }
  h->modelEvaluationCount += (double)h->lambda;
}

/* sort_index, CMAES.cpp.base:940-950: std::sort descending.  Ties are
 * broken by index here (std::sort's tie order is unspecified; parity tests
 * compare tie groups as sets). */
static const double *g_sort_vec;
static int cmp_desc(const void *a, const void *b)
{
  const size_t i1 = *(const size_t *)a, i2 = *(const size_t *)b;
  const double v1 = g_sort_vec[i1], v2 = g_sort_vec[i2];
  if (v1 > v2) return -1;
  if (v1 < v2) return 1;
  return (i1 < i2) ? -1 : (i1 > i2);
}

/* updateDistribution, CMAES.cpp.base:547-688 + adaptC :690-718 +
 * updateSigma :720-761 + numericalErrorTreatment :763-772 */
void kr_cmaes_update(kr_cmaes *h, size_t gen)
{
  const size_t N = h->N, mu = h->mu;
  size_t i, d, e, k;
  int hsig;
  double ccov1, ccovmu, sigmasquare;
  for (i = 0; i < h->lambda; i++) h->sortingIndex[i] = i;
  g_sort_vec = h->F;
  qsort(h->sortingIndex, h->lambda, sizeof(size_t), cmp_desc);

  {
    /* :552-558: with constraints outside the viability regime, the LAST
     * sample in sorted order without violations (as written) */
    long best = (long)h->sortingIndex[0];
    if (h->hasConstraints && !h->isViabilityRegime)
    {
      best = -1;
      for (i = 0; i < h->lambda; i++)
        if (h->sampleConstraintViolationCounts[h->sortingIndex[i]] == 0) best = (long)h->sortingIndex[i];
      if (best < 0)
      {
        h->constraintError = 1; /* the reference indexes _valueVector[-1] */
        best = (long)h->sortingIndex[0];
      }
    }
    h->bestValidSample = (double)best;
    h->previousBestValue = h->currentBestValue;
    h->currentBestValue = h->F[best];
    for (d = 0; d < N; ++d) h->currentBestVariables[d] = h->X[(size_t)best * N + d];
    if (h->currentBestValue > h->bestEverValue || gen == 1)
    {
      h->previousBestEverValue = h->bestEverValue;
      h->bestEverValue = h->currentBestValue;
      for (d = 0; d < N; ++d) h->bestEverVariables[d] = h->currentBestVariables[d];
      if (h->hasConstraints)
        for (k = 0; k < h->nc; k++) h->bestConstraintEvaluations[k] = h->constraintEvaluations[k * h->smax + (size_t)best];
    }
  }
  if (h->muType == 3)
  {
    double valueSum = 0.;
    for (i = 0; i < mu; ++i)
    {
      const double value = h->F[h->sortingIndex[i]];
      h->muWeights[i] = value;
      valueSum += value;
    }
    for (i = 0; i < mu; ++i) h->muWeights[i] /= valueSum;
  }
  {
    long dd;
#pragma omp parallel for schedule(static)
    for (dd = 0; dd < (long)N; ++dd)
    {
      size_t ii;
      h->previousMean[dd] = h->currentMean[dd];
      h->currentMean[dd] = 0.;
      for (ii = 0; ii < mu; ++ii) h->currentMean[dd] += h->muWeights[ii] * h->X[h->sortingIndex[ii] * N + dd];
    }
  }
  if (h->useGradients)
  {
    /* :611-621 (its l2update is computed there but never used) */
    for (d = 0; d < N; ++d)
      for (i = 0; i < mu; ++i)
        h->currentMean[d] += h->muWeights[i] * h->gradientStepSize / sqrt((double)N) * h->gradients[h->sortingIndex[i] * N + d];
  }
  for (d = 0; d < N; ++d) h->meanUpdate[d] = (h->currentMean[d] - h->previousMean[d]) / h->sigma;
  for (d = 0; d < N; ++d)
  {
    double sum = 0.0;
    if (h->diagonal)
      sum = h->meanUpdate[d];
    else
      for (e = 0; e < N; ++e) sum += h->B[e * N + d] * h->meanUpdate[e];
    h->auxBDZ[d] = sum / h->D[d];
  }
  h->psNorm = 0.0;
  for (d = 0; d < N; ++d)
  {
    double sum = 0.0;
    if (h->diagonal)
      sum = h->auxBDZ[d];
    else
      for (e = 0; e < N; ++e) sum += h->B[d * N + e] * h->auxBDZ[e];
    h->ps[d] = (1. - h->sigmaCumulationFactor) * h->ps[d] + sqrt(h->sigmaCumulationFactor * (2. - h->sigmaCumulationFactor) * h->effectiveMu) * sum;
    h->psNorm += kr_pow_cr(h->ps[d], 2.0);
  }
  h->psNorm = sqrt(h->psNorm);
  hsig = (1.4 + 2.0 / (N + 1) > h->psNorm / sqrt(1. - kr_pow_cr(1. - h->sigmaCumulationFactor, 2.0 * (1.0 + gen))) / h->chiSquareNumber);
  h->hsig = hsig;
  for (d = 0; d < N; ++d)
    h->pc[d] = (1. - h->cumulativeCovariance) * h->pc[d] + hsig * sqrt(h->cumulativeCovariance * (2. - h->cumulativeCovariance) * h->effectiveMu) * h->meanUpdate[d];

  /* adaptC */
  ccov1 = 2.0 / (kr_pow_cr(N + 1.3, 2) + h->effectiveMu);
  ccovmu = 2.0 * (h->effectiveMu - 2. + 1. / h->effectiveMu) / (kr_pow_cr(N + 2.0, 2) + h->effectiveMu);
  if (1.0 - ccov1 < ccovmu) ccovmu = 1.0 - ccov1;
  sigmasquare = h->sigma * h->sigma;
  {
    /* every element (d, e <= d) is one sequential sum over k in the
     * reference's order; rows are independent */
    long dd;
#pragma omp parallel for schedule(dynamic, 4)
    for (dd = (long)N - 1; dd >= 0; --dd)
    {
      size_t ee, kk;
      const size_t d1 = (size_t)dd;
      for (ee = h->diagonal ? d1 : 0; ee <= d1; ++ee)
      {
        double c = (1 - ccov1 - ccovmu) * h->C[d1 * N + ee] + ccov1 * (h->pc[d1] * h->pc[ee] + (1 - hsig) * h->cumulativeCovariance * (2. - h->cumulativeCovariance) * h->C[d1 * N + ee]);
        for (kk = 0; kk < mu; ++kk)
        {
          const double *xk = h->X + h->sortingIndex[kk] * N;
          c += ccovmu * h->muWeights[kk] * (xk[d1] - h->previousMean[d1]) * (xk[ee] - h->previousMean[ee]) / sigmasquare;
        }
        h->C[d1 * N + ee] = c;
        if (ee < d1) h->C[ee * N + d1] = c;
      }
    }
  }
  h->maxDiagC = h->minDiagC = h->C[0];
  for (d = 1; d < N; ++d)
  {
    if (h->maxDiagC < h->C[d * N + d])
      h->maxDiagC = h->C[d * N + d];
    else if (h->minDiagC > h->C[d * N + d])
      h->minDiagC = h->C[d * N + d];
  }

  /* updateDiscreteMutationMatrix, :834-859 (after adaptC, with the old sigma) */
  if (h->hasDiscrete)
  {
    double entries = (double)(N + 1);
    for (d = 0; d < N; ++d) h->maskingMatrixSigma[d] = 1.0;
    for (d = 0; d < N; ++d)
      if (h->sigma * sqrt(h->C[d * N + d]) / sqrt(h->sigmaCumulationFactor) < 0.2 * h->granularity[d])
      {
        h->maskingMatrixSigma[d] = 0.0;
        entries -= 1.0;
      }
    h->chiSquareNumberDiscreteMutations = sqrt(entries) * (1. - 1. / (4. * entries) + 1. / (21. * entries * entries));
    h->numberMaskingMatrixEntries = 0;
    for (d = 0; d < N; ++d) h->maskingMatrix[d] = 0.0;
    for (d = 0; d < N; ++d)
      if (2.0 * h->sigma * sqrt(h->C[d * N + d]) < h->granularity[d])
      {
        h->maskingMatrix[d] = 1.0;
        h->numberMaskingMatrixEntries += 1.0;
      }
    {
      const double a = round((double)h->populationSize / 10.0 + h->numberMaskingMatrixEntries + 1),
                   b = floor((double)h->populationSize / 2.0) - 1;
      h->numberOfDiscreteMutations = a < b ? a : b;
    }
    memset(h->discreteMutations, 0, sizeof(double) * h->lambda * N);
  }

  /* updateViabilityBoundaries :424-437 (viability regime) */
  if (h->hasConstraints && h->isViabilityRegime)
    for (k = 0; k < h->nc; k++)
    {
      double maxviolation = 0.0, t;
      for (i = 0; i < mu; ++i)
        if (h->constraintEvaluations[k * h->smax + h->sortingIndex[i]] > maxviolation)
          maxviolation = h->constraintEvaluations[k * h->smax + h->sortingIndex[i]];
      t = 0.5 * (maxviolation + h->viabilityBoundaries[k]);
      t = (t < h->viabilityBoundaries[k]) ? t : h->viabilityBoundaries[k]; /* std::min(bound, t) */
      h->viabilityBoundaries[k] = (0.0 < t) ? t : 0.0;                    /* std::max(0.0, .) */
    }

  /* updateSigma :720-761 */
  if (h->hasConstraints && h->isViabilityRegime)
  {
    /* :724-731 */
    h->globalSuccessRate = (1 - h->globalSuccessLearningRate) * h->globalSuccessRate;
    h->sigma *= kr_exp_cr((h->globalSuccessRate - (h->targetSuccessRate / (1.0 - h->targetSuccessRate)) * (1 - h->globalSuccessRate)) /
                          h->dampFactor);
  }
  else if (h->hasDiscrete)
  {
    double pathL2 = 0.0;
    for (d = 0; d < N; ++d) pathL2 += h->maskingMatrixSigma[d] * h->ps[d] * h->ps[d];
    h->sigma *= kr_exp_cr(h->sigmaCumulationFactor / h->dampFactor * (sqrt(pathL2) / h->chiSquareNumberDiscreteMutations - 1.));
  }
  else
    h->sigma *= kr_exp_cr(h->sigmaCumulationFactor / h->dampFactor * (h->psNorm / h->chiSquareNumber - 1.));
  /* (_muValue: the configured one; the index uses the current mu) */
  if (h->muValue > 1 && h->currentBestValue == h->F[h->sortingIndex[mu - 1]])
    h->sigma *= kr_exp_cr(0.2 + h->sigmaCumulationFactor / h->dampFactor);
  {
    const double ub = sqrt(h->trace / N);
    if (h->sigma > ub && h->isSigmaBounded) h->sigma = ub;
  }
  /* numericalErrorTreatment */
  for (d = 0; d < N; ++d)
    if (h->sigma * sqrt(h->C[d * N + d]) < h->minStdUpdate[d])
      h->sigma = (h->minStdUpdate[d]) / sqrt(h->C[d * N + d]) * kr_exp_cr(0.05 + h->sigmaCumulationFactor / h->dampFactor);

  h->currentMinStd = INFINITY;
  h->currentMaxStd = -INFINITY;
  for (i = 0; i < N; ++i)
  {
    const double s = h->sigma * sqrt(h->C[i * N + i]);
    if (s < h->currentMinStd) h->currentMinStd = s;
    if (s > h->currentMaxStd) h->currentMaxStd = s;
  }
}

/* ---- CCMA-ES: the constraint stages of runGeneration (CMAES.cpp.base:186-196) */
static void cmaes_eval_constraints(kr_cmaes *h, const double *x, double *out)
{
  h->constraintFn(x, h->N, out, h->nc, h->constraintCtx);
  h->constraintEvaluationCount += 1;
}

/* checkMeanAndSetRegime, :315-348 */
void kr_cmaes_check_mean_and_set_regime(kr_cmaes *h)
{
  size_t c;
  double *ev;
  if (!h->isViabilityRegime) return;
  if (h->hasDiscrete) cmaes_discretize(h, h->currentMean);
  ev = (double *)malloc(sizeof(double) * (h->nc + 1));
  cmaes_eval_constraints(h, h->currentMean, ev);
  for (c = 0; c < h->nc; c++)
    if (ev[c] > 0.0)
    {
      free(ev);
      return;
    }
  free(ev);
  h->isViabilityRegime = 0;
  for (c = 0; c < h->nc; c++) h->viabilityBoundaries[c] = 0;
  h->lambda = h->populationSize;
  h->mu = h->muValue;
  cmaes_init_mu_weights(h, h->mu);
  cmaes_init_covariance(h);
}

/* updateConstraints, :350-387 */
void kr_cmaes_update_constraints(kr_cmaes *h, size_t gen)
{
  const size_t S = h->smax;
  size_t i, c;
  double *ev = (double *)malloc(sizeof(double) * (h->nc + 1));
  for (i = 0; i < h->lambda; i++)
  {
    h->sampleConstraintViolationCounts[i] = 0;
    if (h->hasDiscrete) cmaes_discretize(h, h->X + i * h->N);
    cmaes_eval_constraints(h, h->X + i * h->N, ev);
    for (c = 0; c < h->nc; c++) h->constraintEvaluations[c * S + i] = ev[c];
  }
  free(ev);
  h->maxConstraintViolationCount = 0;
  for (c = 0; c < h->nc; c++)
  {
    double maxviolation = 0.0;
    for (i = 0; i < h->lambda; ++i)
    {
      const double e = h->constraintEvaluations[c * S + i];
      if (e > maxviolation) maxviolation = e;
      if (gen == 1 && h->isViabilityRegime) h->viabilityBoundaries[c] = maxviolation;
      if (e > h->viabilityBoundaries[c] + 1e-12) h->sampleConstraintViolationCounts[i] += 1;
      if (h->sampleConstraintViolationCounts[i] > h->maxConstraintViolationCount)
        h->maxConstraintViolationCount = h->sampleConstraintViolationCounts[i];
    }
  }
}

/* reEvaluateConstraints, :389-422 */
static void cmaes_reevaluate_constraints(kr_cmaes *h)
{
  const size_t S = h->smax;
  size_t i, c;
  double *ev = (double *)malloc(sizeof(double) * (h->nc + 1));
  h->maxConstraintViolationCount = 0;
  for (i = 0; i < h->lambda; ++i)
    if (h->sampleConstraintViolationCounts[i] > 0)
    {
      if (h->hasDiscrete) cmaes_discretize(h, h->X + i * h->N);
      cmaes_eval_constraints(h, h->X + i * h->N, ev);
      h->sampleConstraintViolationCounts[i] = 0;
      for (c = 0; c < h->nc; c++)
      {
        h->constraintEvaluations[c * S + i] = ev[c];
        if (ev[c] > h->viabilityBoundaries[c] + 1e-12)
        {
          h->viabilityIndicator[c * S + i] = 1;
          h->sampleConstraintViolationCounts[i] += 1;
        }
        else
          h->viabilityIndicator[c * S + i] = 0;
      }
      if (h->sampleConstraintViolationCounts[i] > h->maxConstraintViolationCount)
        h->maxConstraintViolationCount = h->sampleConstraintViolationCounts[i];
    }
  free(ev);
}

/* handleConstraints, :774-832: shrink the covariance along the constraint
 * normals' running approximations, re-decompose it, redraw the violating
 * samples, re-evaluate them; until no sample violates.  (The viability
 * indicators read by the first pass are the last re-evaluation's, as in the
 * reference: updateConstraints does not set them.) */
void kr_cmaes_handle_constraints(kr_cmaes *h)
{
  const size_t N = h->N, S = h->smax;
  size_t i, c, d, e;
  double *r = (double *)malloc(sizeof(double) * N);
  while (h->maxConstraintViolationCount > 0)
  {
    memcpy(h->auxC, h->C, sizeof(double) * N * N);
    for (i = 0; i < h->lambda; ++i)
      if (h->sampleConstraintViolationCounts[i] > 0)
        for (c = 0; c < h->nc; c++)
          if (h->viabilityIndicator[c * S + i] != 0)
          {
            double v2 = 0, *v = h->normalConstraintApproximation + c * N;
            const double cnt = h->sampleConstraintViolationCounts[i];
            h->covarianceMatrixAdaptationCount += 1;
            if (h->covarianceMatrixAdaptationCount > h->maxCovarianceMatrixCorrections)
            {
              free(r);
              return;
            }
            for (d = 0; d < N; ++d)
            {
              v[d] = (1.0 - h->normalVectorLearningRate) * v[d] + h->normalVectorLearningRate * h->BDZ[i * N + d];
              v2 += v[d] * v[d];
            }
            for (d = 0; d < N; ++d)
              for (e = 0; e < N; ++e)
                h->auxC[d * N + e] = h->auxC[d * N + e] - ((h->covarianceMatrixAdaptionFactor * h->covarianceMatrixAdaptionFactor * v[d] * v[e]) /
                                                           (v2 * cnt * cnt));
          }
    cmaes_update_eigensystem(h, h->auxC);
    for (i = 0; i < h->lambda; ++i)
      if (h->sampleConstraintViolationCounts[i] > 0)
      {
        int ok;
        do
        {
          h->resampledParameterCount += 1;
          for (d = 0; d < N; ++d) r[d] = 0.0 + kr_ran_gaussian(&h->normal, 1.0);
          cmaes_sample_single(h, i, r);
          if (h->hasDiscrete) cmaes_discretize(h, h->X + i * N);
          ok = cmaes_feasible(h, h->X + i * N);
        } while (ok == 0 && h->resampledParameterCount < h->maxInfeasibleResamplings);
      }
    cmaes_reevaluate_constraints(h);
  }
  free(r);
}

int kr_cmaes_constraint_error(kr_cmaes *h) { return h->constraintError; }

/* runGeneration up to the objective (:188-196): regime, prepareGeneration,
 * updateConstraints + handleConstraints; the caller evaluates the objective
 * of samples [0, current lambda) and calls kr_cmaes_update */
void kr_cmaes_ccmaes_prepare(kr_cmaes *h, size_t gen)
{
  if (gen == 1) kr_cmaes_initialize(h);
  if (h->hasConstraints) kr_cmaes_check_mean_and_set_regime(h);
  kr_cmaes_prepare(h);
  if (h->hasConstraints)
  {
    kr_cmaes_update_constraints(h, gen);
    kr_cmaes_handle_constraints(h);
  }
}

void kr_cmaes_generation(kr_cmaes *h, size_t gen, int objective)
{
  if (gen == 1) kr_cmaes_initialize(h);
  kr_cmaes_prepare(h);
  kr_cmaes_evaluate(h, objective);
  kr_cmaes_update(h, gen);
}

/* ======================================================================
 * TMCMC — source/modules/solver/sampler/TMCMC/TMCMC.cpp.base
 * (Version "TMCMC", Sequential conduit: chains complete in chain order)
 * ==================================================================== */
struct kr_tmcmc
{
  size_t N, P;
  /* options */
  double maxChainLength, burnIn, targetCOV, covScaling, minAnnealingExponentUpdate, maxAnnealingExponentUpdate;
  double *perGenBurnIn; /* "Per Generation Burn In": entry k applies to generation k+2 */
  size_t perGenBurnInCount;
  double currentBurnIn;
  /* priors: uniform [priorMin, priorMax] per variable, RNG per variable */
  double *priorMin, *priorMax;
  kr_rng *priorRng;
  int *priorMap; /* variable -> prior distribution (shared distributions share an RNG) */
  int *priorKind; /* per variable: 0 Uniform [priorMin, priorMax], 1 Normal (mean, sd), 2 Exponential
                   * (location, mean), 3 Laplace (mean, width), 4 Cauchy (location, scale), 5 LogNormal
                   * (mu, sigma): priorMin / priorMax hold the two parameters */
  /* state */
  double *leaders, *leadersLL, *leadersLP, *candidates, *candidatesLL, *candidatesLP;
  double *chainLengths, *meanTheta, *cov, *chol;
  double *dbX, *dbLL, *dbLP; /* sample database (P entries when all chains finish) */
  double *numSelections;
  double annealingExponent, previousAnnealingExponent, logEvidence, coefficientOfVariation, maxLoglikelihood;
  double chainCount, acceptedSamplesCount, proposalsAcceptanceRate, selectionAcceptanceRate;
  double dbCount, modelEvaluationCount, minSearchIterations;
  kr_rng multinomial, multivariate, uniform;
  /* mTMCMC (TMCMC.cpp.base:48-83, :146-157, :174-200, :383-558, :567-609,
   * :634-681): errors / gradients / proposal covariances of the chain
   * leaders (L*), candidates (C*) and database (D*); errors held as doubles */
  double version, stepSize, domainExtensionFactor, numCovarianceCorrections;
  double *upperExt, *lowerExt;
  double *LE, *CE, *DE, *LG, *CG, *DG, *LC, *CC, *DC;
};

kr_tmcmc *kr_tmcmc_new(size_t N, size_t P)
{
  kr_tmcmc *h = (kr_tmcmc *)calloc(1, sizeof(kr_tmcmc));
  size_t i;
  h->N = N;
  h->P = P;
  h->maxChainLength = 1;
  h->burnIn = 0;
  h->targetCOV = 1.0;
  h->covScaling = 0.04;
  h->minAnnealingExponentUpdate = 1e-5;
  h->maxAnnealingExponentUpdate = 1.0;
#define AL(p, n) p = (double *)calloc((n), sizeof(double))
  AL(h->priorMin, N);
  AL(h->priorMax, N);
  AL(h->leaders, P * N);
  AL(h->leadersLL, P);
  AL(h->leadersLP, P);
  AL(h->candidates, P * N);
  AL(h->candidatesLL, P);
  AL(h->candidatesLP, P);
  AL(h->chainLengths, P);
  AL(h->meanTheta, N);
  AL(h->cov, N * N);
  AL(h->chol, N * N);
  AL(h->dbX, P * N);
  AL(h->dbLL, P);
  AL(h->dbLP, P);
  AL(h->numSelections, P);
#undef AL
  h->priorRng = (kr_rng *)calloc(N, sizeof(kr_rng));
  h->priorMap = (int *)calloc(N, sizeof(int));
  h->priorKind = (int *)calloc(N, sizeof(int));
  for (i = 0; i < N; i++)
  {
    h->priorMap[i] = (int)i;
    h->priorMin[i] = 0.0;
    h->priorMax[i] = 1.0;
    kr_rng_seed(&h->priorRng[i], 0);
  }
  kr_rng_seed(&h->multinomial, 0);
  kr_rng_seed(&h->multivariate, 0);
  kr_rng_seed(&h->uniform, 0);
  return h;
}

void kr_tmcmc_free(kr_tmcmc *h)
{
  if (!h) return;
  free(h->priorMin);
  free(h->priorMax);
  free(h->priorRng);
  free(h->priorMap);
  free(h->priorKind);
  free(h->leaders);
  free(h->leadersLL);
  free(h->leadersLP);
  free(h->candidates);
  free(h->candidatesLL);
  free(h->candidatesLP);
  free(h->chainLengths);
  free(h->meanTheta);
  free(h->cov);
  free(h->chol);
  free(h->dbX);
  free(h->dbLL);
  free(h->dbLP);
  free(h->numSelections);
  free(h->perGenBurnIn);
  free(h->upperExt);
  free(h->lowerExt);
  free(h->LE);
  free(h->CE);
  free(h->DE);
  free(h->LG);
  free(h->CG);
  free(h->DG);
  free(h->LC);
  free(h->CC);
  free(h->DC);
  free(h);
}

double *kr_tmcmc_field(kr_tmcmc *h, const char *name, size_t *len)
{
  const size_t N = h->N, P = h->P;
#define VEC(key, ptr, n)      \
  if (strcmp(name, key) == 0) \
  {                           \
    if (len) *len = (n);      \
    return ptr;               \
  }
#define SCA(key, var) VEC(key, &h->var, 1)
  VEC("Prior Minimum", h->priorMin, N)
  VEC("Prior Maximum", h->priorMax, N)
  VEC("Chain Leaders", h->leaders, P * N)
  VEC("Chain Leaders LogLikelihoods", h->leadersLL, P)
  VEC("Chain Leaders LogPriors", h->leadersLP, P)
  VEC("Chain Candidates", h->candidates, P * N)
  VEC("Chain Candidates LogLikelihoods", h->candidatesLL, P)
  VEC("Chain Candidates LogPriors", h->candidatesLP, P)
  VEC("Chain Lengths", h->chainLengths, P)
  VEC("Mean Theta", h->meanTheta, N)
  VEC("Covariance Matrix", h->cov, N * N)
  VEC("Cholesky Factor", h->chol, N * N)
  VEC("Sample Database", h->dbX, P * N)
  VEC("Sample LogLikelihood Database", h->dbLL, P)
  VEC("Sample LogPrior Database", h->dbLP, P)
  VEC("Num Selections", h->numSelections, P)
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
  SCA("Num Covariance Corrections", numCovarianceCorrections)
  if (h->LE)
  {
    VEC("Chain Leaders Errors", h->LE, P)
    VEC("Chain Candidates Errors", h->CE, P)
    VEC("Sample Error Database", h->DE, P)
    VEC("Chain Leaders Gradients", h->LG, P * N)
    VEC("Chain Candidates Gradients", h->CG, P * N)
    VEC("Sample Gradient Database", h->DG, P * N)
    VEC("Chain Leaders Covariance", h->LC, P * N * N)
    VEC("Chain Candidates Covariance", h->CC, P * N * N)
    VEC("Sample Covariances Database", h->DC, P * N * N)
    VEC("Upper Extended Boundaries", h->upperExt, N)
    VEC("Lower Extended Boundaries", h->lowerExt, N)
  }
#undef VEC
#undef SCA
  if (len) *len = 0;
  return NULL;
}

kr_rng *kr_tmcmc_rng(kr_tmcmc *h, int which)
{
  if (which == 0) return &h->multinomial;
  if (which == 1) return &h->multivariate;
  if (which == 2) return &h->uniform;
  return &h->priorRng[which - 3];
}

/* _variables[d]->_distributionIndex (TMCMC.cpp.base:218-220): variables
 * drawing from the same distribution object consume its one generator */
void kr_tmcmc_set_prior_map(kr_tmcmc *h, const int *map)
{
  size_t d;
  for (d = 0; d < h->N; d++) h->priorMap[d] = map[d];
}

/* the variables' prior kinds: 0 Univariate/Uniform, 1 Univariate/Normal
 * (univariate/normal/normal.cpp.base: Mean / Standard Deviation in
 * Prior Minimum / Prior Maximum) */
void kr_tmcmc_set_prior_kinds(kr_tmcmc *h, const int *kinds)
{
  size_t d;
  for (d = 0; d < h->N; d++) h->priorKind[d] = kinds[d];
}

void kr_tmcmc_set_option(kr_tmcmc *h, const char *name, double v)
{
  if (strcmp(name, "Max Chain Length") == 0) h->maxChainLength = v;
  else if (strcmp(name, "Default Burn In") == 0) h->burnIn = v;
  else if (strcmp(name, "Target Coefficient Of Variation") == 0) h->targetCOV = v;
  else if (strcmp(name, "Covariance Scaling") == 0) h->covScaling = v;
  else if (strcmp(name, "Min Annealing Exponent Update") == 0) h->minAnnealingExponentUpdate = v;
  else if (strcmp(name, "Max Annealing Exponent Update") == 0) h->maxAnnealingExponentUpdate = v;
  else if (strcmp(name, "Version") == 0) h->version = v; /* 0 TMCMC, 1 mTMCMC */
  else if (strcmp(name, "Step Size") == 0) h->stepSize = v;
  else if (strcmp(name, "Domain Extension Factor") == 0) h->domainExtensionFactor = v;
}

void kr_tmcmc_set_per_generation_burn_in(kr_tmcmc *h, const double *v, size_t n)
{
  free(h->perGenBurnIn);
  h->perGenBurnIn = (double *)calloc(n ? n : 1, sizeof(double));
  if (n) memcpy(h->perGenBurnIn, v, n * sizeof(double));
  h->perGenBurnInCount = n;
}

/* setBurnIn, TMCMC.cpp.base:781-789 */
static double tm_burn_in(const kr_tmcmc *h, size_t gen)
{
  if (gen <= 1) return 0.0;
  if (gen - 2 < h->perGenBurnInCount) return h->perGenBurnIn[gen - 2];
  return h->burnIn;
}

/* setInitialConfiguration, TMCMC.cpp.base:21-105 */
void kr_tmcmc_initialize(kr_tmcmc *h)
{
  size_t i;
  h->annealingExponent = 0.0;
  h->logEvidence = 0.0;
  h->coefficientOfVariation = 0.0;
  h->maxLoglikelihood = -INFINITY;
  h->chainCount = (double)h->P;
  for (i = 0; i < h->P; i++) h->chainLengths[i] = 1;
  if (h->version == 1.0 && !h->LE)
  {
    const size_t N = h->N, P = h->P;
#define AL(p, n) p = (double *)calloc((n), sizeof(double))
    AL(h->upperExt, N);
    AL(h->lowerExt, N);
    AL(h->LE, P);
    AL(h->CE, P);
    AL(h->DE, P);
    AL(h->LG, P * N);
    AL(h->CG, P * N);
    AL(h->DG, P * N);
    AL(h->LC, P * N * N);
    AL(h->CC, P * N * N);
    AL(h->DC, P * N * N);
#undef AL
    /* :57-59 errors start at -1; :76-82 extended boundaries */
    for (i = 0; i < P; i++) h->CE[i] = h->LE[i] = h->DE[i] = -1;
    for (i = 0; i < N; i++)
    {
      const double width = h->priorMax[i] - h->priorMin[i];
      h->upperExt[i] = h->priorMax[i] + width * h->domainExtensionFactor;
      h->lowerExt[i] = h->priorMin[i] - width * h->domainExtensionFactor;
    }
  }
  if (h->LE) h->numCovarianceCorrections = 0;
}

/* generateCandidate :560-566 -> multivariate::Normal::getRandomVector
 * (gsl_ran_multivariate_gaussian: N polar normals, dtrmv, + zero mean), then
 * + leader */
static void tm_generate_candidate(kr_tmcmc *h, size_t i)
{
  const size_t N = h->N;
  size_t d;
  double *x = h->candidates + i * N;
  for (d = 0; d < N; d++) x[d] = kr_ran_gaussian(&h->multivariate, 1.0);
  kr_dtrmv_lower(N, h->chol, x);
  for (d = 0; d < N; d++) x[d] = x[d] + 0.0;
  for (d = 0; d < N; d++) x[d] += h->leaders[i * N + d];
}

/* gslcblas dgemv RowMajor NoTrans, beta = 1: y_i += alpha (sum_j A_ij x_j) */
static void mt_dgemv_add(size_t N, double alpha, const double *A, const double *x, double *y)
{
  size_t i, j;
  for (i = 0; i < N; i++)
  {
    double temp = 0.0;
    for (j = 0; j < N; j++) temp += A[i * N + j] * x[j];
    y[i] += alpha * temp;
  }
}

/* generateCandidate, mTMCMC branch (:567-608): a leader without errors
 * proposes from N(leader + (step/2) Sigma_l g_l, step Sigma_l) (the mean
 * vector, then the drift added by dgemv); a failed Cholesky draws nothing
 * and leaves the candidate as it was; a leader with errors proposes from
 * N(leader, Sigma) with the population covariance. */
static void mt_generate_candidate(kr_tmcmc *h, size_t i)
{
  const size_t N = h->N;
  size_t d;
  double *x = h->candidates + i * N;
  if (h->LE[i] == 0)
  {
    double *S = (double *)malloc(sizeof(double) * N * N);
    for (d = 0; d < N * N; d++) S[d] = h->LC[i * N * N + d] * h->stepSize;
    if (kr_cholesky(N, S) == 0)
    {
      for (d = 0; d < N; d++) x[d] = kr_ran_gaussian(&h->multivariate, 1.0);
      kr_dtrmv_lower(N, S, x);
      for (d = 0; d < N; d++) x[d] = x[d] + h->leaders[i * N + d];
      mt_dgemv_add(N, 0.5 * h->stepSize, h->LC + i * N * N, h->LG + i * N, x);
    }
    free(S);
  }
  if (h->LE[i] != 0)
  {
    for (d = 0; d < N; d++) x[d] = kr_ran_gaussian(&h->multivariate, 1.0);
    kr_dtrmv_lower(N, h->chol, x);
    for (d = 0; d < N; d++) x[d] = x[d] + h->leaders[i * N + d];
  }
}

/* ---- mTMCMC linear algebra (GSL 2.6 is absent here: the Level-2 forms of
 * linalg/lu.c, linalg/luinv via LU_svx, randist/mvgauss.c, gslcblas
 * dtrsv / dgemm loop orders; parity with GSL itself is unpinned) ---- */

/* gsl_cdf_chisq_Pinv(0.68, N), N = 1..128 (tools/make_chi2_table.py) */
static const double MT_CHI2_068[128] = {
  0.988946481478023, 2.27886856637673, 3.505882355768179, 4.695422319122993,
  5.8608022596974125, 7.009169946950603, 8.144788668939585, 9.270418200246363,
  10.387958013319528, 11.498778181311328, 12.603903905356493, 13.704125276314006,
  14.800066067589455, 15.892228745155391, 16.98102499350416, 18.066797057367218,
  19.149833056062814, 20.230378223312684, 21.308643320753227, 22.38481104613223,
  23.459040989954513, 24.53147352253592, 25.602232880235793, 26.67142964341346,
  27.739162746301982, 28.805521122384825, 29.870585062847724, 30.934427346913328,
  31.997114189146984, 33.05870603866459, 34.119258257565306, 35.17882170015321,
  36.237443210107635, 37.29516604936419, 38.35203026982309, 39.40807303692524,
  40.46332891249609, 41.517830102949176, 42.571606677894444, 43.6246867633504,
  44.67709671307324, 45.728861260956485, 46.78000365699435, 47.83054578892401,
  48.880508291347134, 49.929910643870045, 50.97877125958297, 52.02710756501539,
  53.074936072549725, 54.122272446144436, 55.16913156110684, 56.215527558560616,
  57.26147389517232, 58.30698338863145, 59.35206825931891, 60.39674016854704,
  61.44101025370968, 62.48488916064193, 63.528387073455576, 64.57151374208671,
  65.61427850776624, 66.65669032660158, 67.69875779143783, 68.74048915214941,
  69.78189233449768, 70.82297495767644, 71.86374435065521, 72.90420756741935,
  73.9443714011968, 74.98424239775245, 76.0238268678238, 77.06313089876471,
  78.10216036545802, 79.14092094055236, 80.17941810407355, 81.21765715245671,
  82.2556432070412, 83.29338122206687, 84.33087599220691, 85.36813215966977,
  86.4051542208999, 87.44194653290452, 88.47851331923188, 89.51485867562381,
  90.55098657536443, 91.5869008743443, 92.62260531585866, 93.65810353515641,
  94.6933990637555, 95.72849533353936, 96.7633956806475, 97.79810334917329,
  98.83262149467973, 99.86695318754488, 100.90110141614619, 101.93506908989364,
  102.96885904212003, 104.00247403283672, 105.03591675136242, 106.06918981883199,
  107.10229579059188, 108.13523715848865, 109.1680163530559, 110.20063574560554,
  111.2330976502281, 112.26540432570714, 113.29755797735193, 114.32956075875305,
  115.36141477346426, 116.39312207661503, 117.4246846764566, 118.45610453584531,
  119.48738357366618, 120.5185236661994, 121.5495266484329, 122.58039431532332,
  123.6111284230079, 124.64173068996958, 125.67220279815764, 126.70254639406568,
  127.73276308976914, 128.76285446392407, 129.79282206272907, 130.82266740085166,
  131.85239196232124, 132.88199720138954, 133.91148454336053, 134.9408553853905,
};

double kr_chi2inv_068(size_t N) { return (N >= 1 && N <= 128) ? MT_CHI2_068[N - 1] : NAN; }

/* gsl_linalg_LU_decomp: partial pivoting, row operations, perm[] */
static void mt_lu_decomp(size_t N, double *A, size_t *perm)
{
  size_t i, j, k;
  for (i = 0; i < N; i++) perm[i] = i;
  for (j = 0; j + 1 < N; j++)
  {
    double ajj, max = fabs(A[j * N + j]);
    size_t ip = j;
    for (i = j + 1; i < N; i++)
    {
      const double aij = fabs(A[i * N + j]);
      if (aij > max)
      {
        max = aij;
        ip = i;
      }
    }
    if (ip != j)
    {
      size_t t;
      for (k = 0; k < N; k++)
      {
        const double q = A[j * N + k];
        A[j * N + k] = A[ip * N + k];
        A[ip * N + k] = q;
      }
      t = perm[j];
      perm[j] = perm[ip];
      perm[ip] = t;
    }
    ajj = A[j * N + j];
    if (ajj != 0.0)
      for (i = j + 1; i < N; i++)
      {
        const double aij = A[i * N + j] / ajj;
        A[i * N + j] = aij;
        for (k = j + 1; k < N; k++) A[i * N + k] = A[i * N + k] - aij * A[j * N + k];
      }
  }
}

/* gsl_linalg_LU_invert: identity columns through LU_svx (permute, dtrsv
 * Lower Unit, dtrsv Upper NonUnit) */
static void mt_lu_invert(size_t N, const double *LU, const size_t *perm, double *inv)
{
  size_t c, i, j;
  double *x = (double *)malloc(sizeof(double) * N), *y = (double *)malloc(sizeof(double) * N);
  for (c = 0; c < N; c++)
  {
    for (i = 0; i < N; i++) y[i] = (i == c) ? 1.0 : 0.0;
    for (i = 0; i < N; i++) x[i] = y[perm[i]]; /* gsl_permute_vector: v'_i = v_{p_i} */
    for (i = 1; i < N; i++)
    {
      double tmp = x[i];
      for (j = 0; j < i; j++) tmp -= LU[i * N + j] * x[j];
      x[i] = tmp;
    }
    x[N - 1] = x[N - 1] / LU[(N - 1) * N + (N - 1)];
    for (i = N - 1; i > 0 && i--;)
    {
      double tmp = x[i];
      for (j = i + 1; j < N; j++) tmp -= LU[i * N + j] * x[j];
      x[i] = tmp / LU[i * N + i];
    }
    for (i = 0; i < N; i++) inv[i * N + c] = x[i];
  }
  free(x);
  free(y);
}

/* gsl_ran_multivariate_gaussian_log_pdf with the lower Cholesky factor L */
static double mt_mvn_log_pdf(size_t N, const double *x, const double *mu, const double *L)
{
  size_t i, j;
  double quad = 0.0, logdet = 0.0;
  double *w = (double *)malloc(sizeof(double) * N);
  for (i = 0; i < N; i++) w[i] = x[i] - mu[i];
  w[0] = w[0] / L[0];
  for (i = 1; i < N; i++)
  {
    double tmp = w[i];
    for (j = 0; j < i; j++) tmp -= L[i * N + j] * w[j];
    w[i] = tmp / L[i * N + i];
  }
  for (i = 0; i < N; i++) quad += w[i] * w[i];
  for (i = 0; i < N; i++) logdet += kr_log_cr(L[i * N + i]);
  free(w);
  return -0.5 * quad - logdet - 0.5 * (double)N * kr_log_cr(2.0 * 3.14159265358979323846);
}

/* calculateGradients + calculateProposals (:383-558) for the chains whose
 * candidate has a finite log-prior and log-likelihood; grad (P x N) and
 * fim (P x N x N) are the problem's "logLikelihood Gradient" and "Fisher
 * Information" of every candidate (rows of other chains are not read). */
void kr_tmcmc_set_gradients(kr_tmcmc *h, const double *grad, const double *fim)
{
  const size_t N = h->N, NN = N * N;
  const double chi2inv = kr_chi2inv_068(N);
  double *F = (double *)malloc(sizeof(double) * NN), *Finv = (double *)malloc(sizeof(double) * NN);
  double *ev = (double *)malloc(sizeof(double) * N), *E = (double *)malloc(sizeof(double) * NN);
  double *c0 = (double *)malloc(sizeof(double) * N), *c1 = (double *)malloc(sizeof(double) * N);
  size_t *perm = (size_t *)malloc(sizeof(size_t) * N);
  size_t c, d, e, i, j, k;
  for (c = 0; c < (size_t)h->chainCount; c++)
  {
    if (!(isfinite(h->candidatesLP[c]) && isfinite(h->candidatesLL[c]))) continue;
    for (d = 0; d < N; d++) h->CG[c * N + d] = grad[c * N + d] * h->annealingExponent;
  }
  for (c = 0; c < (size_t)h->chainCount; c++)
  {
    const double *cand = h->candidates + c * N;
    double *CC = h->CC + c * NN;
    int correction = 0;
    if (!(isfinite(h->candidatesLP[c]) && isfinite(h->candidatesLL[c]))) continue;
    for (k = 0; k < NN; k++) CC[k] = 0.0;
    for (k = 0; k < NN; k++) F[k] = fim[c * NN + k] * h->annealingExponent;
    mt_lu_decomp(N, F, perm);
    mt_lu_invert(N, F, perm, Finv);
    /* gsl_eigen_symmv, unsorted */
    kr_eigen_symmv_unsorted(N, Finv, ev, E);
    for (d = 0; d < N; d++)
    {
      double scale = sqrt(ev[d] * chi2inv);
      const double before = scale;
      for (e = 0; e < N; e++) c0[e] = cand[e] + (1.0 * scale) * E[e * N + d];
      for (e = 0; e < N; e++) c1[e] = cand[e] + (-1.0 * scale) * E[e * N + d];
      for (e = 0; e < N; e++)
      {
        const double up = h->upperExt[e] - cand[e], lo = cand[e] - h->lowerExt[e];
        double len, v;
        len = c0[e] - h->upperExt[e];
        if (len > 0.)
        {
          v = fabs(1.0 / E[e * N + d] * up);
          scale = (v < scale) ? v : scale;
        }
        len = h->lowerExt[e] - c0[e];
        if (len > 0.)
        {
          v = fabs(1.0 / E[e * N + d] * lo);
          scale = (v < scale) ? v : scale;
        }
        len = c1[e] - h->upperExt[e];
        if (len > 0.)
        {
          v = fabs(1.0 / E[e * N + d] * up);
          scale = (v < scale) ? v : scale;
        }
        len = h->lowerExt[e] - c1[e];
        if (len > 0.)
        {
          v = fabs(1.0 / E[e * N + d] * lo);
          scale = (v < scale) ? v : scale;
        }
      }
      ev[d] = scale * scale / chi2inv;
      if (before != scale) correction = 1;
    }
    if (correction) h->numCovarianceCorrections += 1;
    for (d = 0; d < N; d++)
    {
      const double f = sqrt(ev[d]);
      for (e = 0; e < N; e++) E[e * N + d] *= f;
    }
    /* gslcblas dgemm RowMajor NoTrans/Trans, alpha 1, beta 0 */
    for (i = 0; i < N; i++)
      for (j = 0; j < N; j++)
      {
        double temp = 0.0;
        for (k = 0; k < N; k++) temp += E[i * N + k] * E[j * N + k];
        CC[i * N + j] = 0.0 + 1.0 * temp;
      }
  }
  free(F);
  free(Finv);
  free(ev);
  free(E);
  free(c0);
  free(c1);
  free(perm);
}

/* calculateAcceptanceProbability, mTMCMC branch (:634-677) */
static double mt_acceptance(kr_tmcmc *h, size_t c)
{
  const size_t N = h->N, NN = N * N;
  const double *LC = h->LC + c * NN;
  double *mL = (double *)malloc(sizeof(double) * N), *mC = (double *)malloc(sizeof(double) * N);
  double *L = (double *)malloc(sizeof(double) * NN);
  double lpC, lpL, P;
  size_t k;
  memcpy(mL, h->leaders + c * N, sizeof(double) * N);
  memcpy(mC, h->candidates + c * N, sizeof(double) * N);
  mt_dgemv_add(N, 0.5 * h->stepSize, LC, h->LG + c * N, mL);
  mt_dgemv_add(N, 0.5 * h->stepSize, LC, h->CG + c * N, mC);
  for (k = 0; k < NN; k++) L[k] = LC[k] * h->stepSize;
  kr_cholesky(N, L);
  lpC = mt_mvn_log_pdf(N, h->candidates + c * N, mL, L);
  lpL = mt_mvn_log_pdf(N, h->leaders + c * N, mC, L);
  P = kr_exp_cr((h->candidatesLL[c] - h->leadersLL[c]) * h->annealingExponent + (lpL - lpC) +
                (h->candidatesLP[c] - h->leadersLP[c]));
  free(mL);
  free(mC);
  free(L);
  return P;
}

/* prepareGeneration, TMCMC.cpp.base:159-227 (setBurnIn :781-789) */
void kr_tmcmc_prepare(kr_tmcmc *h, size_t gen)
{
  const size_t N = h->N;
  size_t i, d;
  h->currentBurnIn = tm_burn_in(h, gen);
  h->acceptedSamplesCount = 0;
  h->maxLoglikelihood = -INFINITY;
  h->dbCount = 0;
  if (h->LE)
  {
    /* :174-200: error flags of this generation's candidates, then the
     * leaders' proposals and gradients re-annealed */
    const double fc = h->previousAnnealingExponent / h->annealingExponent;
    const double fg = h->annealingExponent / h->previousAnnealingExponent;
    h->numCovarianceCorrections = 0;
    for (i = 0; i < h->P; i++) h->CE[i] = gen > 1 ? 0 : -1;
    for (i = 0; i < h->P; i++)
    {
      for (d = 0; d < N * N; d++) h->LC[i * N * N + d] *= fc;
      for (d = 0; d < N; d++) h->LG[i * N + d] *= fg;
    }
  }
  memcpy(h->chol, h->cov, sizeof(double) * N * N);
  kr_cholesky(N, h->chol);
  for (i = 0; i < h->P; i++)
  {
    if (gen == 1)
    {
      /* TMCMC.cpp.base:218-220: getRandomNumber of each variable's
       * distribution; Normal: mean + gsl_ran_gaussian(sd) (normal.cpp.base:30-33) */
      for (d = 0; d < N; d++)
      {
        kr_rng *g = &h->priorRng[h->priorMap[d]];
        const double a = h->priorMin[d], b = h->priorMax[d];
        double v;
        switch (h->priorKind[d])
        {
        case 1: v = a + kr_ran_gaussian(g, b); break;
        case 2: v = a + kr_ran_exponential(g, b); break;
        case 3: v = a + kr_ran_laplace(g, b); break;
        case 4: v = a + kr_ran_cauchy(g, b); break;
        case 5: v = kr_ran_lognormal(g, a, b); break;
        default: v = kr_ran_flat(g, a, b);
        }
        h->candidates[i * N + d] = v;
      }
    }
    else if (h->LE)
      mt_generate_candidate(h, i);
    else
      tm_generate_candidate(h, i);
  }
}

/* Bayesian::evaluate (bayesian.cpp.base:24-84): logPrior = sum of uniform
 * log-densities (uniform.cpp.base:38-44); -inf prior -> -inf loglik without
 * calling the model; else builtin Gaussian loglik (model.py:32-37). */
static void tm_evaluate_one(kr_tmcmc *h, size_t i)
{
  const size_t N = h->N;
  size_t d;
  const double *x = h->candidates + i * N;
  double lp = 0.0;
  for (d = 0; d < N; d++)
  {
    const double a = h->priorMin[d], b = h->priorMax[d], pi = 3.14159265358979323846;
    switch (h->priorKind[d])
    {
    case 1:
    { /* normal.cpp.base:17-21, :40-46 */
      const double logNorm = -0.5 * kr_log_cr(2 * pi) - kr_log_cr(b);
      const double z = (x[d] - a) / b;
      lp += logNorm - 0.5 * z * z;
      continue;
    }
    case 2:
    { /* exponential.cpp.base getLogDensity */
      const double y = x[d] - a;
      lp += y < 0 ? -INFINITY : -kr_log_cr(b) - y / b;
      continue;
    }
    case 3: /* laplace.cpp.base: aux = -log(2 width) */
      lp += -kr_log_cr(2. * b) - fabs(x[d] - a) / b;
      continue;
    case 4:
    { /* cauchy.cpp.base: aux = -log(scale pi) */
      const double y = x[d] - a;
      lp += -kr_log_cr(b * pi) - kr_log_cr(1. + y * y / (b * b));
      continue;
    }
    case 5:
    { /* logNormal.cpp.base: aux = -0.5 log(2 pi) - log(sigma) */
      if (x[d] <= 0)
      {
        lp += -INFINITY;
        continue;
      }
      const double aux = -0.5 * kr_log_cr(2 * pi) - kr_log_cr(b), lx = kr_log_cr(x[d]), z = (lx - a) / b;
      lp += aux - lx - 0.5 * z * z;
      continue;
    }
    default: break;
    }
    const double aux = -kr_log_cr(h->priorMax[d] - h->priorMin[d]);
    lp += (x[d] >= h->priorMin[d] && x[d] <= h->priorMax[d]) ? aux : -INFINITY;
  }
  h->candidatesLP[i] = lp;
  h->candidatesLL[i] = isinf(lp) && lp < 0 ? -INFINITY : kr_loglik_gaussian(x, N);
  h->modelEvaluationCount += 1;
}

/* the first step of every started chain (runGeneration :114-130 starts
 * chains c < Chain Count) */
void kr_tmcmc_evaluate(kr_tmcmc *h)
{
  size_t i;
  for (i = 0; i < (size_t)h->chainCount; i++) tm_evaluate_one(h, i);
}

/* runGeneration's WAITANY loop :112-144 with processCandidate +
 * calculateAcceptanceProbability + updateDatabase (:229-252, :611-633).
 * With the Sequential conduit the waitAny scan (conduit.cpp.base:180-210)
 * always hands the single worker to the lowest-index started sample, and a
 * finished chain is restarted before the next scan, so every step of chain
 * c completes before chain c+1's first: chain-major order.  Step s of chain
 * c (1-based, S = Chain Lengths[c] + Current Burn In steps): one Uniform,
 * accept if P > U or generation 1 (counted only past the burn-in), a new
 * candidate (N Multivariate normals) while s < S, a database entry past the
 * burn-in.  Step 1's candidate was evaluated by kr_tmcmc_evaluate. */
void kr_tmcmc_process_candidates(kr_tmcmc *h, size_t gen)
{
  const size_t N = h->N;
  const size_t B = (size_t)h->currentBurnIn;
  size_t c, s;
  for (c = 0; c < (size_t)h->chainCount; c++)
  {
    const size_t S = (size_t)h->chainLengths[c] + B;
    for (s = 1; s <= S; s++)
    {
      double P = 0.0, U;
      if (s > 1) tm_evaluate_one(h, c);
      if (isfinite(h->candidatesLP[c]) && isfinite(h->candidatesLL[c]))
      {
        if (h->LE && h->LE[c] == 0 && h->CE[c] == 0)
          P = mt_acceptance(h, c);
        else
          P = kr_exp_cr((h->candidatesLL[c] - h->leadersLL[c]) * h->annealingExponent + (h->candidatesLP[c] - h->leadersLP[c]));
      }
      U = kr_ran_flat(&h->uniform, 0.0, 1.0);
      if (P > U || gen == 1)
      {
        memcpy(h->leaders + c * N, h->candidates + c * N, sizeof(double) * N);
        h->leadersLP[c] = h->candidatesLP[c];
        h->leadersLL[c] = h->candidatesLL[c];
        if (h->LE)
        {
          h->LE[c] = h->CE[c];
          memcpy(h->LG + c * N, h->CG + c * N, sizeof(double) * N);
          memcpy(h->LC + c * N * N, h->CC + c * N * N, sizeof(double) * N * N);
        }
        if (s > B) h->acceptedSamplesCount++;
      }
      if (s < S) tm_generate_candidate(h, c);
      if (s > B && (size_t)h->dbCount < h->P) /* sum of chain lengths = P */
      {
        const size_t k = (size_t)h->dbCount;
        memcpy(h->dbX + k * N, h->leaders + c * N, sizeof(double) * N);
        h->dbLP[k] = h->leadersLP[c];
        h->dbLL[k] = h->leadersLL[c];
        if (h->LE)
        {
          h->DE[k] = h->LE[c];
          memcpy(h->DG + k * N, h->LG + c * N, sizeof(double) * N);
          memcpy(h->DC + k * N * N, h->LC + c * N * N, sizeof(double) * N * N);
        }
        h->dbCount += 1;
      }
    }
  }
}

/* calculateSquaredCVDifference, TMCMC.cpp.base:683-703 */
double kr_tmcmc_cv2(double x, const double *loglike, size_t Ns, double exponent, double targetCOV)
{
  double *weight = (double *)malloc(sizeof(double) * Ns);
  double loglike_max = loglike[0], sum_weight = 0.0, mean, sd, cov2;
  size_t i;
  for (i = 0; i < Ns; i++)
  {
    if (loglike[i] > loglike_max) loglike_max = loglike[i];
    if (isnan(loglike[i]))
    {
      loglike_max = loglike[i];
      break;
    }
  }
  for (i = 0; i < Ns; i++) weight[i] = kr_exp_cr((loglike[i] - loglike_max) * (x - exponent));
  for (i = 0; i < Ns; i++) sum_weight += weight[i];
  for (i = 0; i < Ns; i++) weight[i] = weight[i] / sum_weight;
  mean = kr_stats_mean(weight, Ns);
  sd = kr_stats_sd_m(weight, Ns, mean);
  free(weight);
  cov2 = (sd / mean) - targetCOV;
  cov2 *= cov2;
  if (!isfinite(cov2)) return -DBL_MAX; /* 'Lowest' */
  return cov2;
}

/* GSL nmsimplex (v1) in one dimension; minSearch TMCMC.cpp.base:712-779 */
typedef struct
{
  const double *ll;
  size_t Ns;
  double exponent, cov;
} nm_param;

static double nm_f(double x, const nm_param *p) { return kr_tmcmc_cv2(x, p->ll, p->Ns, p->exponent, p->cov); }

static double nm_size(const double X[2])
{
  const double center = (X[0] + X[1]) / 2;
  double ss = 0.0;
  ss += fabs(X[0] - center);
  ss += fabs(X[1] - center);
  return ss / 2.0;
}

size_t kr_tmcmc_minsearch(const double *loglike, size_t Ns, double exponent, double objCov, double *xmin, double *fmin)
{
  const size_t MaxIter = 1000;
  const double Tol = 1e-12, Step = 1e-8;
  nm_param p;
  double X[2], Y[2], size, fval = 0.0, xbest;
  size_t iter = 0;
  int status;
  p.ll = loglike;
  p.Ns = Ns;
  p.exponent = exponent;
  p.cov = objCov;
  X[0] = exponent;
  Y[0] = nm_f(X[0], &p);
  X[1] = exponent + Step;
  Y[1] = nm_f(X[1], &p);
  size = nm_size(X);
  xbest = X[0];
  do
  {
    size_t hi = 0, s_hi = 0, lo = 0, i;
    double dhi, ds_hi, dlo, val, val2, xc, xc2;
    iter++;
    dhi = ds_hi = dlo = Y[0];
    for (i = 1; i < 2; i++)
    {
      val = Y[i];
      if (val < dlo)
      {
        dlo = val;
        lo = i;
      }
      else if (val > dhi)
      {
        ds_hi = dhi;
        s_hi = hi;
        dhi = val;
        hi = i;
      }
      else if (val > ds_hi)
      {
        ds_hi = val;
        s_hi = i;
      }
    }
    {
      /* move_corner(-1, hi): mp = mean of other rows (one row here) */
      const double mp = (X[1 - hi]) / 1.0;
      xc = mp - (-1.0) * (mp - X[hi]);
      val = nm_f(xc, &p);
    }
    if (isfinite(val) && val < Y[lo])
    {
      const double mp = (X[1 - hi]) / 1.0;
      xc2 = mp - (-2.0) * (mp - X[hi]);
      val2 = nm_f(xc2, &p);
      if (isfinite(val2) && val2 < Y[lo])
      {
        X[hi] = xc2;
        Y[hi] = val2;
      }
      else
      {
        X[hi] = xc;
        Y[hi] = val;
      }
    }
    else if (!isfinite(val) || val > Y[s_hi])
    {
      if (isfinite(val) && val <= Y[hi])
      {
        X[hi] = xc;
        Y[hi] = val;
      }
      {
        const double mp = (X[1 - hi]) / 1.0;
        xc2 = mp - (0.5) * (mp - X[hi]);
        val2 = nm_f(xc2, &p);
      }
      if (isfinite(val2) && val2 <= Y[hi])
      {
        X[hi] = xc2;
        Y[hi] = val2;
      }
      else
      {
        /* contract_by_best(lo) */
        for (i = 0; i < 2; i++)
          if (i != lo)
          {
            X[i] = 0.5 * (X[i] + X[lo]);
            Y[i] = nm_f(X[i], &p);
          }
      }
    }
    else
    {
      X[hi] = xc;
      Y[hi] = val;
    }
    /* lo = gsl_vector_min_index(y1) */
    lo = 0;
    {
      double mn = Y[0];
      for (i = 0; i < 2; i++)
      {
        if (Y[i] < mn)
        {
          mn = Y[i];
          lo = i;
        }
        if (isnan(Y[i]))
        {
          lo = i;
          break;
        }
      }
    }
    xbest = X[lo];
    fval = Y[lo];
    size = nm_size(X);
    status = (size < Tol) ? 0 : 1;
  } while (status == 1 && iter < MaxIter);

  *fmin = 0;
  *xmin = 0.0;
  if (fval <= Tol)
  {
    *fmin = fval;
    *xmin = xbest;
  }
  if (*xmin >= 1.0)
  {
    *fmin = kr_tmcmc_cv2(1.0, loglike, Ns, exponent, objCov);
    *xmin = 1.0;
  }
  return iter;
}

/* processGeneration, TMCMC.cpp.base:254-381 */
void kr_tmcmc_process_generation(kr_tmcmc *h)
{
  const size_t N = h->N, P = h->P;
  size_t i, j, k;
  double fmin = 0, xmin = 0, loglikemax, sum_weight, sum_weight2;
  double *log_weight = (double *)malloc(sizeof(double) * P);
  double *weight = (double *)malloc(sizeof(double) * P);
  unsigned int *nsel = (unsigned int *)malloc(sizeof(unsigned int) * P);
  size_t leaderId = 0, zeroCount = 0;
  double *newLeaders = (double *)malloc(sizeof(double) * P * N);

  h->minSearchIterations = (double)kr_tmcmc_minsearch(h->dbLL, P, h->annealingExponent, h->targetCOV, &xmin, &fmin);
  h->previousAnnealingExponent = h->annealingExponent;
  if (xmin > h->previousAnnealingExponent + h->maxAnnealingExponentUpdate)
  {
    h->annealingExponent = h->previousAnnealingExponent + h->maxAnnealingExponentUpdate;
    h->coefficientOfVariation = sqrt(kr_tmcmc_cv2(h->annealingExponent, h->dbLL, P, h->previousAnnealingExponent, h->targetCOV)) + h->targetCOV;
  }
  else if (xmin < 1.0 && xmin < h->previousAnnealingExponent + h->minAnnealingExponentUpdate)
  {
    h->annealingExponent = h->previousAnnealingExponent + h->minAnnealingExponentUpdate;
    h->coefficientOfVariation = sqrt(kr_tmcmc_cv2(h->annealingExponent, h->dbLL, P, h->previousAnnealingExponent, h->targetCOV)) + h->targetCOV;
  }
  else
  {
    h->annealingExponent = xmin;
    h->coefficientOfVariation = sqrt(fmin) + h->targetCOV;
  }

  for (i = 0; i < P; i++) log_weight[i] = h->dbLL[i] * (h->annealingExponent - h->previousAnnealingExponent);
  loglikemax = log_weight[0];
  for (i = 0; i < P; i++)
  {
    if (log_weight[i] > loglikemax) loglikemax = log_weight[i];
    if (isnan(log_weight[i]))
    {
      loglikemax = log_weight[i];
      break;
    }
  }
  for (i = 0; i < P; i++) weight[i] = kr_exp_cr(log_weight[i] - loglikemax);
  sum_weight = 0.0;
  for (i = 0; i < P; i++) sum_weight += weight[i];
  for (i = 0; i < P; i++) weight[i] = weight[i] / sum_weight;
  h->logEvidence += kr_log_cr(sum_weight) + loglikemax - kr_log_cr((double)P);

  kr_ran_multinomial(&h->multinomial, P, (unsigned int)P, weight, nsel);
  for (i = 0; i < P; i++) h->numSelections[i] = nsel[i];

  for (i = 0; i < P; i++) weight[i] = weight[i] * nsel[i];
  sum_weight = 0.0;
  for (i = 0; i < P; i++) sum_weight += weight[i];
  for (i = 0; i < P; i++) weight[i] = weight[i] / sum_weight;
  sum_weight2 = 0.0;
  for (i = 0; i < P; i++) sum_weight2 += weight[i] * weight[i];

  for (i = 0; i < N; i++)
  {
    h->meanTheta[i] = 0;
    for (j = 0; j < P; j++) h->meanTheta[i] += h->dbX[j * N + i] * weight[j];
  }
  for (i = 0; i < N; i++)
    for (j = i; j < N; ++j)
    {
      double s = 0.0;
      for (k = 0; k < P; ++k) s += weight[k] * (h->dbX[k * N + i] - h->meanTheta[i]) * (h->dbX[k * N + j] - h->meanTheta[j]);
      h->cov[i * N + j] = h->cov[j * N + i] = h->covScaling * s / (1.0 - sum_weight2);
    }

  for (i = 0; i < P; i++) h->chainLengths[i] = 0;
  for (i = 0; i < P; i++)
  {
    if (nsel[i] == 0) zeroCount++;
    while (nsel[i] > 0)
    {
      size_t len;
      memcpy(newLeaders + leaderId * N, h->dbX + i * N, sizeof(double) * N);
      h->leadersLP[leaderId] = h->dbLP[i];
      h->leadersLL[leaderId] = h->dbLL[i];
      if (h->LE)
      {
        h->LE[leaderId] = h->DE[i];
        memcpy(h->LG + leaderId * N, h->DG + i * N, sizeof(double) * N);
        memcpy(h->LC + leaderId * N * N, h->DC + i * N * N, sizeof(double) * N * N);
      }
      if (nsel[i] > h->maxChainLength)
      {
        const size_t mcl = (size_t)h->maxChainLength;
        const size_t rest = (nsel[i] % mcl != 0);
        len = mcl - rest;
      }
      else
        len = nsel[i];
      h->chainLengths[leaderId] = (double)len;
      nsel[i] -= (unsigned int)len;
      leaderId++;
    }
  }
  memcpy(h->leaders, newLeaders, sizeof(double) * leaderId * N);
  /* :362-372 anneal the leaders' gradients and proposals */
  if (h->LE && h->previousAnnealingExponent > 0.0)
  {
    const double f = h->annealingExponent / h->previousAnnealingExponent;
    for (i = 0; i < P; i++)
    {
      if (h->LE[i] != 0) continue;
      for (j = 0; j < N; j++) h->LG[i * N + j] *= f;
      for (j = 0; j < N * N; j++) h->LC[i * N * N + j] *= f;
    }
  }
  h->proposalsAcceptanceRate = (1.0 * h->acceptedSamplesCount) / P;
  h->selectionAcceptanceRate = (1.0 * (P - zeroCount)) / P;
  h->maxLoglikelihood = h->dbLL[0];
  for (i = 1; i < P; i++)
    if (h->dbLL[i] > h->maxLoglikelihood) h->maxLoglikelihood = h->dbLL[i];
  h->chainCount = (double)leaderId;
  free(log_weight);
  free(weight);
  free(nsel);
  free(newLeaders);
}

void kr_tmcmc_generation(kr_tmcmc *h, size_t gen)
{
  if (gen == 1) kr_tmcmc_initialize(h);
  kr_tmcmc_prepare(h, gen);
  kr_tmcmc_evaluate(h);
  kr_tmcmc_process_candidates(h, gen);
  kr_tmcmc_process_generation(h);
}
