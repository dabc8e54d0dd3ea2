// kg_eigen.hip — GSL-faithful symmetric eigensolver on one CDNA4 workgroup.
//
// Replaces CMAES::updateEigensystem + CMAES::eigen (CMAES.cpp.base:869-938),
// i.e. gsl_eigen_symmv + gsl_eigen_symmv_sort(GSL_EIGEN_SORT_ABS_ASC).  The
// eigenvector SIGNS of LAPACK-style solvers differ from GSL in 2-6 columns
// per generation and every sign flip changes the next population, so this
// kernel replays GSL 2.6's exact arithmetic:
//
//   A  Householder tridiagonalisation (linalg/symmtd.c) with gslcblas
//      dnrm2 / dsymv / dsyr2 operation order; A lives in LDS (row stride
//      N+1: conflict-free column and row sweeps) when N <= 128.
//   B  symmtd_unpack: Q = prod H_i (householder_hm), Q kept transposed in
//      LDS, one column per thread.
//   C  implicit-shift QR (eigen/qrstep.c): the Givens chase is inherently
//      serial and runs on lane 0 of wave 0; the rotations of step t are
//      applied row-parallel by waves 1..15 while lane 0 chases step t+1
//      (double-buffered gc/gs, one barrier per QR step).
//   D  ABS_ASC selection sort (parallel arg-min per position) and the
//      updateEigensystem write-back (keep the old B, D if min eval <= 0).
//
// Every +,-,*,/,sqrt is IEEE correctly rounded on gfx950 and the file is
// compiled with -ffp-contract=off, so the result equals the oracle bit for
// bit.
#include <chrono>
#include <cstdlib>

#include "kg_eigen.hpp"
#include "kg_chains.hpp"

namespace kg {

namespace {

__device__ __attribute__((unused)) inline double readlane_d(double x, int l) {
  const long long v = __double_as_longlong(x);
  int lo = (int)(v & 0xffffffffLL), hi = (int)(v >> 32);
  lo = __builtin_amdgcn_readlane(lo, l);
  hi = __builtin_amdgcn_readlane(hi, l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__host__ __device__ inline uint32_t hiw(double x) { return (uint32_t)(__builtin_bit_cast(unsigned long long, x) >> 32); }
__host__ __device__ inline uint32_t low(double x) {
  return (uint32_t)(__builtin_bit_cast(unsigned long long, x) & 0xffffffffULL);
}
__host__ __device__ inline double sethi(double x, uint32_t h) {
  return __builtin_bit_cast(double, ((unsigned long long)h << 32) | (unsigned long long)low(x));
}

// fdlibm __ieee754_hypot (glibc < 2.35), SURVEY.md Appendix A
__host__ __device__ double hypot_fdlibm(double x, double y) {
  double a, b, t1, t2, y1, y2, w;
  int32_t j, k, ha, hb;
  ha = (int32_t)(hiw(x) & 0x7fffffff);
  hb = (int32_t)(hiw(y) & 0x7fffffff);
  if (hb > ha) {
    a = y;
    b = x;
    j = ha;
    ha = hb;
    hb = j;
  } else {
    a = x;
    b = y;
  }
  a = sethi(a, (uint32_t)ha);
  b = sethi(b, (uint32_t)hb);
  if ((ha - hb) > 0x3c00000) return a + b;
  k = 0;
  if (ha > 0x5f300000) {
    if (ha >= 0x7ff00000) {
      w = a + b;
      if (((ha & 0xfffff) | low(a)) == 0) w = a;
      if (((hb ^ 0x7ff00000) | low(b)) == 0) w = b;
      return w;
    }
    ha -= 0x25800000;
    hb -= 0x25800000;
    k += 600;
    a = sethi(a, (uint32_t)ha);
    b = sethi(b, (uint32_t)hb);
  }
  if (hb < 0x20b00000) {
    if (hb <= 0x000fffff) {
      if ((hb | (int32_t)low(b)) == 0) return a;
      t1 = sethi(0.0, 0x7fd00000);
      b *= t1;
      a *= t1;
      k -= 1022;
    } else {
      ha += 0x25800000;
      hb += 0x25800000;
      k -= 600;
      a = sethi(a, (uint32_t)ha);
      b = sethi(b, (uint32_t)hb);
    }
  }
  w = a - b;
  if (w > b) {
    t1 = sethi(0.0, (uint32_t)ha);
    t2 = a - t1;
    w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
  } else {
    a = a + a;
    y1 = sethi(0.0, (uint32_t)hb);
    y2 = b - y1;
    t1 = sethi(0.0, (uint32_t)(ha + 0x00100000));
    t2 = a - t1;
    w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
  }
  if (k != 0) {
    t1 = sethi(1.0, hiw(1.0) + ((uint32_t)k << 20));
    return t1 * w;
  }
  return w;
}

// hypot_fdlibm for the device's Householder step: the same arithmetic on
// fdlibm's common path (no range rescaling needed: both high words in
// [0x20b00000, 0x5f300000]) with both of its final formulas formed and one
// selected, so no divergent branches sit on the critical path; anything
// else falls back to hypot_fdlibm.
__device__ __forceinline__ double hypot_fast(double x, double y) {
  int32_t ha = (int32_t)(hiw(x) & 0x7fffffff), hb = (int32_t)(hiw(y) & 0x7fffffff);
  const bool sw = hb > ha;
  double a = sw ? y : x, b = sw ? x : y;
  const int32_t h1 = sw ? hb : ha, h2 = sw ? ha : hb;
  ha = h1;
  hb = h2;
  a = sethi(a, (uint32_t)ha);
  b = sethi(b, (uint32_t)hb);
  const bool common = (ha - hb) <= 0x3c00000 && ha <= 0x5f300000 && hb >= 0x20b00000;
  if (!__builtin_amdgcn_readfirstlane((int)common)) return hypot_fdlibm(x, y);
  const double w = a - b;
  // w > b
  const double t1a = sethi(0.0, (uint32_t)ha), t2a = a - t1a;
  const double ra = t1a * t1a - (b * (-b) - t2a * (a + t1a));
  // w <= b
  const double a2 = a + a, y1 = sethi(0.0, (uint32_t)hb), y2 = b - y1;
  const double t1b = sethi(0.0, (uint32_t)(ha + 0x00100000)), t2b = a2 - t1b;
  const double rb = t1b * y1 - (w * (-w) - (t1b * y2 + t2b * b));
  return sqrt(w > b ? ra : rb);
}

constexpr double EPS = 2.2204460492503131e-16;
constexpr double DMIN = 2.2250738585072014e-308;

__host__ __device__ inline void chop_small(int n, const double *d, double *sd) {
  double d_i = d[0];
  for (int i = 0; i + 1 < n; i++) {
    const double sd_i = sd[i], d_ip1 = d[i + 1];
    if (fabs(sd_i) < EPS * (fabs(d_i) + fabs(d_ip1))) sd[i] = 0.0;
    d_i = d_ip1;
  }
}

// gsl_linalg / eigen create_givens, branches as GSL writes them.  (A
// branch-free form -- operands selected before the one division -- was
// measured slower on the box's EPYC 9575F, round 5: chase 0.335-0.341 against
// 0.310-0.314 ms per C2 generation; the predictor follows these branches, a
// select puts the comparison on the critical chain.)
__host__ __device__ inline void create_givens(double a, double b, double &c, double &s) {
  if (b == 0) {
    c = 1;
    s = 0;
  } else if (fabs(b) > fabs(a)) {
    const double t = -a / b;
    const double s1 = 1.0 / sqrt(1 + t * t);
    s = s1;
    c = s1 * t;
  } else {
    const double t = -b / a;
    const double c1 = 1.0 / sqrt(1 + t * t);
    c = c1;
    s = c1 * t;
  }
}

// eigen/qrstep.c qrstep on d[0..n), sd[0..n-1)
__host__ __device__ void qrstep(int n, double *d, double *sd, double *gc, double *gs) {
  double x, z, ak, bk, zk, ap, bp, aq, bq;
  double mu;
  {
    const double ta = d[n - 2], tb = d[n - 1], tab = sd[n - 2];
    const double dt = (ta - tb) / 2.0;
    if (dt > 0)
      mu = tb - tab * (tab / (dt + hypot_fdlibm(dt, tab)));
    else if (dt == 0)
      mu = tb - fabs(tab);
    else
      mu = tb + tab * (tab / ((-dt) + hypot_fdlibm(dt, tab)));
  }
  if (EPS * fabs(mu) > (fabs(d[0]) + fabs(sd[0]))) mu = 0;
  x = d[0] - mu;
  z = sd[0];
  ak = 0;
  bk = 0;
  zk = 0;
  ap = d[0];
  bp = sd[0];
  aq = d[1];
  if (n == 2) {
    double c, s;
    create_givens(x, z, c, s);
    gc[0] = c;
    gs[0] = s;
    const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
    const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
    const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
    d[0] = ap1;
    sd[0] = bp1;
    d[1] = aq1;
    return;
  }
  bq = sd[1];
  // d[k+2], sd[k+2] read at step k were never written by this chase yet:
  // load them one step ahead so LDS latency stays off the critical path
  double dn = d[n - 1 < 2 ? n - 1 : 2], sdn = sd[n - 2 < 2 ? n - 2 : 2];
  int k;
  for (k = 0; k < n - 1; k++) {
    const double dpf = d[(k + 3 < n - 1) ? k + 3 : n - 1];  // unconditional loads (unused past the end)
    const double sdpf = sd[(k + 3 < n - 2) ? k + 3 : n - 2];
    double c, s;
    create_givens(x, z, c, s);
    gc[k] = c;
    gs[k] = s;
    const double bk1 = c * bk - s * zk;
    const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
    const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
    const double zp1 = -s * bq;
    const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
    const double bq1 = c * bq;
    ak = ap1;
    bk = bp1;
    zk = zp1;
    ap = aq1;
    bp = bq1;
    if (k < n - 2) aq = dn;
    if (k < n - 3) bq = sdn;
    dn = dpf;
    sdn = sdpf;
    d[k] = ak;
    if (k > 0) sd[k - 1] = bk1;
    if (k < n - 2) sd[k + 1] = bp;
    x = bk;
    z = zk;
  }
  d[k] = ap;
  sd[k - 1] = bk;
}

// qrstep with the chase's bookkeeping folded into the sweep: each rotation
// goes straight to the rotation record (cs: c, s pairs), and chop_small's
// test of index k-1 (|sd[k-1]| < eps (|d[k-1]| + |d[k]|)) runs at iteration
// k, when d[k-1], d[k] and sd[k-1] hold their final values of this step --
// the same values chop_small reads after the step, so the same zeros.  The
// sweep never reads sd[k-1] again after iteration k.  The tests sit off the
// rotation chain (the core runs them in the shadow of its divisions), where
// the separate pass and the copy were ~15% of the chase.
__host__ __device__ void qrstep_fused(int n, double *d, double *sd, double *cs) {
  double x, z, ak, bk, zk, ap, bp, aq, bq;
  double mu;
  {
    const double ta = d[n - 2], tb = d[n - 1], tab = sd[n - 2];
    const double dt = (ta - tb) / 2.0;
    if (dt > 0)
      mu = tb - tab * (tab / (dt + hypot_fdlibm(dt, tab)));
    else if (dt == 0)
      mu = tb - fabs(tab);
    else
      mu = tb + tab * (tab / ((-dt) + hypot_fdlibm(dt, tab)));
  }
  if (EPS * fabs(mu) > (fabs(d[0]) + fabs(sd[0]))) mu = 0;
  x = d[0] - mu;
  z = sd[0];
  ak = 0;
  bk = 0;
  zk = 0;
  ap = d[0];
  bp = sd[0];
  aq = d[1];
  if (n == 2) {
    double c, s;
    create_givens(x, z, c, s);
    cs[0] = c;
    cs[1] = s;
    const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
    const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
    const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
    d[0] = ap1;
    sd[0] = bp1;
    d[1] = aq1;
    if (fabs(bp1) < EPS * (fabs(ap1) + fabs(aq1))) sd[0] = 0.0;
    return;
  }
  bq = sd[1];
  double dn = d[n - 1 < 2 ? n - 1 : 2], sdn = sd[n - 2 < 2 ? n - 2 : 2];
  double dprev = 0.0;  // d[k - 1] as written at iteration k - 1
  int k;
  for (k = 0; k < n - 1; k++) {
    const double dpf = d[(k + 3 < n - 1) ? k + 3 : n - 1];
    const double sdpf = sd[(k + 3 < n - 2) ? k + 3 : n - 2];
    double c, s;
    create_givens(x, z, c, s);
    cs[2 * k] = c;
    cs[2 * k + 1] = s;
    const double bk1 = c * bk - s * zk;
    const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
    const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
    const double zp1 = -s * bq;
    const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
    const double bq1 = c * bq;
    ak = ap1;
    bk = bp1;
    zk = zp1;
    ap = aq1;
    bp = bq1;
    if (k < n - 2) aq = dn;
    if (k < n - 3) bq = sdn;
    dn = dpf;
    sdn = sdpf;
    d[k] = ak;
    if (k > 0) sd[k - 1] = (fabs(bk1) < EPS * (fabs(dprev) + fabs(ak))) ? 0.0 : bk1;
    if (k < n - 2) sd[k + 1] = bp;
    dprev = ak;
    x = bk;
    z = zk;
  }
  d[k] = ap;
  sd[k - 1] = (fabs(bk) < EPS * (fabs(dprev) + fabs(ap))) ? 0.0 : bk;
}

// DPP lane moves of a double (both halves; lanes without a source get 0.0)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_d(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(v & 0xffffffffLL), CTRL, ROWMASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), CTRL, ROWMASK, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// inclusive prefix max over the wave of values >= 0 (identity 0.0):
// row_shr 1/2/4/8 inside rows of 16, then row_bcast 15 / 31 across rows
__device__ __forceinline__ double wave_prefix_max_nonneg(double x) {
  x = fmax(x, dpp_d<0x111, 0xf>(x));
  x = fmax(x, dpp_d<0x112, 0xf>(x));
  x = fmax(x, dpp_d<0x114, 0xf>(x));
  x = fmax(x, dpp_d<0x118, 0xf>(x));
  x = fmax(x, dpp_d<0x142, 0xa>(x));
  x = fmax(x, dpp_d<0x143, 0xc>(x));
  return x;
}

// v_max_f64 without the canonicalising self-max the compiler adds to fmax
// (the operands here are |x| of finite values or 0.0, never NaN)
__device__ __forceinline__ double vmax_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// wave_prefix_max_nonneg of two independent vectors, level by level (the
// two dependency chains interleave)
__device__ __forceinline__ void wave_prefix_max2_nonneg(double x, double y, double &px, double &py) {
#define KG_PM2(CTRL, RM)                   \
  {                                        \
    const double dx = dpp_d<CTRL, RM>(x);  \
    const double dy = dpp_d<CTRL, RM>(y);  \
    x = vmax_f64(x, dx);                   \
    y = vmax_f64(y, dy);                   \
  }
  KG_PM2(0x111, 0xf)
  KG_PM2(0x112, 0xf)
  KG_PM2(0x114, 0xf)
  KG_PM2(0x118, 0xf)
  KG_PM2(0x142, 0xa)
  KG_PM2(0x143, 0xc)
#undef KG_PM2
  px = x;
  py = y;
}

// gslcblas dnrm2 of m elements x[k*stride], k < m, by one wave (every lane
// returns the result): scale = running max |x| (prefix max, lane-parallel),
// the addends (|x|/scale)^2 and rescale ratios staged in LDS (sv: m doubles,
// msk: ceil(m/64) words marking new-maximum elements), then the ssq
// recurrence in the reference's order with the next 8 addends loaded while
// the current 8 are added.  Zero elements add +0.0 (ssq >= 1: exact).
__device__ double dnrm2_wave(const double *x, int stride, int m, double *sv, unsigned long long *msk) {
  const int lane = threadIdx.x & 63;
  double carry = 0.0;
  const int m8 = (m + 7) & ~7;  // staged length: zero addends (exact) pad to whole batches
  for (int base = 0; base < m8; base += 64) {
    const int e = base + lane;
    const double a_ = fabs(x[(size_t)min(e, m - 1) * stride]);
    const double a = (e < m) ? a_ : 0.0;
    const double pm = wave_prefix_max_nonneg(a);  // DPP: no LDS round trips
    const double before = fmax(dpp_d<0x138, 0xf>(pm), carry);  // wave_shr:1, lane 0 gets 0.0
    int type = 0;
    double q = 0.0;
    if (e < m && a != 0.0) {
      if (before < a) {
        type = 1;
        q = before / a;
      } else {
        type = 2;
        q = a / before;
      }
    }
    const unsigned long long b1 = __ballot(type == 1);
    if (e < m8) sv[e] = (type == 1) ? q : ((type == 2) ? q * q : 0.0);
    if (lane == 0) msk[base >> 6] = b1;
    carry = fmax(carry, readlane_d(pm, 63));
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double ssq = 1.0;
  // one mask word per 64 (uniform, loaded once), values two batches deep
#define KG_NRM2_STEP8(T, BITS)                        \
  {                                                   \
    const unsigned bits_ = (BITS);                    \
    if (bits_ == 0) {                                 \
      _Pragma("unroll") for (int u = 0; u < 8; u++) ssq += T[u]; \
    } else {                                          \
      _Pragma("unroll") for (int u = 0; u < 8; u++) { \
        if ((bits_ >> u) & 1u)                        \
          ssq = 1.0 + ssq * T[u] * T[u];              \
        else                                          \
          ssq += T[u];                                \
      }                                               \
    }                                                 \
  }
  for (int c0 = 0; c0 < m8; c0 += 64) {
    const unsigned long long mw = msk[c0 >> 6];
    const int cn = (m8 - c0) < 64 ? (m8 - c0) : 64;
    double a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = sv[c0 + u];
    for (int e = 0; e < cn; e += 16) {
#pragma unroll
      for (int u = 0; u < 8; u++) b[u] = sv[c0 + e + 8 + u];
      KG_NRM2_STEP8(a, (unsigned)((mw >> e) & 0xffULL))
      if (e + 8 >= cn) break;
#pragma unroll
      for (int u = 0; u < 8; u++) a[u] = sv[c0 + e + 16 + u];
      KG_NRM2_STEP8(b, (unsigned)((mw >> (e + 8)) & 0xffULL))
    }
  }
#undef KG_NRM2_STEP8
  __builtin_amdgcn_wave_barrier();
  return (m == 1) ? fabs(x[0]) : carry * sqrt(ssq);
}

// dnrm2_wave for m <= 128 (the one-workgroup tridiagonalisation): both
// 64-element chunks are staged at once (independent DPP prefix maxima, one
// division per element — before / a for a new maximum, a / before otherwise —
// as a select of operands, no divergent branches), the rescale masks stay in
// scalar registers; the ordered ssq recurrence is dnrm2_wave's.
__device__ double dnrm2_wave128(const double *x, int m, double *sv) {
  const int lane = threadIdx.x & 63;
  const int m8 = (m + 7) & ~7;
  const int e0 = lane, e1 = lane + 64;
  const double r0 = fabs(x[min(e0, m - 1)]), r1 = fabs(x[min(e1, m - 1)]);
  const double a0 = e0 < m ? r0 : 0.0, a1 = e1 < m ? r1 : 0.0;
  const double pm0 = wave_prefix_max_nonneg(a0), pm1 = wave_prefix_max_nonneg(a1);
  const double c0 = readlane_d(pm0, 63);
  const double b0 = dpp_d<0x138, 0xf>(pm0);            // before, chunk 0 (lane 0: 0.0)
  const double b1 = fmax(dpp_d<0x138, 0xf>(pm1), c0);  // before, chunk 1
  const bool z0 = e0 < m && a0 != 0.0, z1 = e1 < m && a1 != 0.0;
  const bool n0 = z0 && b0 < a0, n1 = z1 && b1 < a1;
  const double q0 = (n0 ? b0 : a0) / (n0 ? a0 : b0), q1 = (n1 ? b1 : a1) / (n1 ? a1 : b1);
  const unsigned long long k0 = __ballot(n0), k1 = __ballot(n1);
  if (e0 < m8) sv[e0] = n0 ? q0 : (z0 ? q0 * q0 : 0.0);
  if (e1 < m8) sv[e1] = n1 ? q1 : (z1 ? q1 * q1 : 0.0);
  const double carry = fmax(c0, readlane_d(pm1, 63));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double ssq = 1.0;
#define KG_NRM2_STEP8(T, BITS)                        \
  {                                                   \
    const unsigned bits_ = (BITS);                    \
    if (bits_ == 0) {                                 \
      _Pragma("unroll") for (int u = 0; u < 8; u++) ssq += T[u]; \
    } else {                                          \
      _Pragma("unroll") for (int u = 0; u < 8; u++) { \
        if ((bits_ >> u) & 1u)                        \
          ssq = 1.0 + ssq * T[u] * T[u];              \
        else                                          \
          ssq += T[u];                                \
      }                                               \
    }                                                 \
  }
  for (int cb = 0; cb < m8; cb += 64) {
    const unsigned long long mw = cb ? k1 : k0;
    const int cn = (m8 - cb) < 64 ? (m8 - cb) : 64;
    double a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = sv[cb + u];
    for (int e = 0; e < cn; e += 16) {
#pragma unroll
      for (int u = 0; u < 8; u++) b[u] = sv[cb + e + 8 + u];
      KG_NRM2_STEP8(a, (unsigned)((mw >> e) & 0xffULL))
      if (e + 8 >= cn) break;
#pragma unroll
      for (int u = 0; u < 8; u++) a[u] = sv[cb + e + 16 + u];
      KG_NRM2_STEP8(b, (unsigned)((mw >> (e + 8)) & 0xffULL))
    }
  }
#undef KG_NRM2_STEP8
  __builtin_amdgcn_wave_barrier();
  return (m == 1) ? fabs(x[0]) : carry * sqrt(ssq);
}

}  // namespace

// Dynamic LDS: [matrix region N*(N+1) doubles if lds_mats] + vectors.
// Vectors (doubles): x N, d N, sd N, tau N, gc 2N, gs 2N, ev N, scal 16; ints
// perm N, misc 8.
// ------------------------------------------------------------------------
// Phase A: Householder tridiagonalisation (gsl_linalg_symmtd_decomp).
// Outputs: Householder vectors H (row i = column i of A below the
// diagonal), tau, diagonal d and sub-diagonal sd of the tridiagonal form.
template <bool kLds>
__global__ void __launch_bounds__(1024) k_tridiag(int N, const double *__restrict__ C, double *gA, double *gH,
                                                  double *tauOut, double *dOut, double *sdOut,
                                                  unsigned long long *trace) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wid = tid >> 6;
  const int lda = N + 1;
  double *M = kLds ? smem : gA;
  double *vb = kLds ? smem + (size_t)N * lda : smem;
  double *x = vb, *scal = vb + N;
  double *sv = vb + N + 16;  // staged addends of a serial chain (wave 0); t2 of dsymv
  double *tv = sv + (N > 64 ? N : 64) + 8;  // tau * v_r, contiguous (dsymv); sv padded for dnrm2_wave
  double *vv = tv + N;       // v_r with v_0 = 1, contiguous (dsymv)
  unsigned long long acc_t[4] = {0, 0, 0, 0}, tmark = 0;
#define KG_MARK() \
  if (trace && tid == 0) tmark = __builtin_amdgcn_s_memtime();
#define KG_ACC(k) \
  if (trace && tid == 0) acc_t[k] += __builtin_amdgcn_s_memtime() - tmark;

  // symmetrise from the lower triangle (CMAES.cpp.base:908-913)
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, j = idx % N;
    M[i * lda + j] = (j <= i) ? C[i * N + j] : C[j * N + i];
  }
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    const int n = N - i - 1;
    double *v = M + (size_t)(i + 1) * lda + i;        // stride lda
    double *m = M + (size_t)(i + 1) * lda + (i + 1);  // lda
    KG_MARK()
    if (wid == 0) {
      // gslcblas dnrm2 over v[1..n-1]
      const double xnorm = dnrm2_wave(v + lda, lda, n - 1, sv, (unsigned long long *)(scal + 8));
      if (lane == 0) {
        double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
        int branch = 0;
        if (xnorm != 0) {
          const double alpha = v[0];
          beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fdlibm(alpha, xnorm);
          tau_i = (beta - alpha) / beta;
          const double s = alpha - beta;
          if (fabs(s) > DMIN) {
            f1 = 1.0 / s;
            branch = 1;
          } else {
            f1 = EPS / s;
            f2 = 1.0 / EPS;
            branch = 2;
          }
        }
        scal[0] = tau_i;
        scal[1] = f1;
        scal[2] = f2;
        scal[3] = beta;
        scal[4] = (double)branch;
        tauOut[i] = tau_i;
      }
    }
    __syncthreads();
    KG_ACC(0)
    const double tau_i = scal[0];
    const int branch = (int)scal[4];
    if (branch != 0) {
      const double f1 = scal[1], f2 = scal[2];
      for (int r = 1 + tid; r < n; r += nt) {
        double t = v[(size_t)r * lda] * f1;
        if (branch == 2) t = t * f2;
        v[(size_t)r * lda] = t;
      }
      if (tid == 0) v[0] = scal[3];
    }
    __syncthreads();
    if (tau_i == 0.0) continue;
    KG_MARK()
    // x = tau * m * v (dsymv RowMajor Lower, beta = 0), v0 := 1
    for (int r = tid; r < n; r += nt) {
      const double vr = (r == 0) ? 1.0 : v[(size_t)r * lda];
      vv[r] = vr;
      tv[r] = tau_i * vr;
    }
    __syncthreads();
    // The two sequential chains of output j run on different waves (all four
    // SIMDs busy), products formed inline, 8 at a time, loads unconditional:
    //   acc_j: rows r = n-1 .. j+1 (descending) of (tau v_r) m[r][j]   (thread j)
    //   t2_j : cols q = 0 .. j-1 of v_q m[j][q]                        (thread 128 + j)
    // then x_j = (acc_j + (tau v_j) m[j][j]) + tau t2_j.
    double *t2b = sv;  // t2 of every j (sv holds max(N, 64) doubles)
    const int half = (nt / 2) & ~63;
    if (tid < half) {
      for (int j = tid; j < n; j += half) {
        const double *mc = m + j;
        // rows r = n-1 .. j+1 (descending)
        x[j] = ordered_sum(0.0, n - 1 - j, [&](int q) { return tv[n - 1 - q] * mc[(size_t)(n - 1 - q) * lda]; });
      }
    } else {
      for (int j = tid - half; j < n; j += nt - half) {
        const double *mj = m + (size_t)j * lda;
        t2b[j] = ordered_sum(0.0, j, [&](int q) { return vv[q] * mj[q]; });
      }
    }
    __syncthreads();
    for (int j = tid; j < n; j += nt) {
      double acc = x[j];
      acc += tv[j] * m[(size_t)j * lda + j];
      acc += tau_i * t2b[j];
      x[j] = acc;
    }
    __syncthreads();
    KG_ACC(1)
    KG_MARK()
    // xv = sum x[r] v[r] sequentially: products staged by all threads (tv is
    // free after dsymv), one ordered chain on wave 0; alpha = -(tau/2) xv
    for (int r = tid; r < n; r += nt) tv[r] = x[r] * vv[r];
    __syncthreads();
    if (wid == 0) {
      const double xv = ordered_sum(0.0, n, [&](int q) { return tv[q]; });
      if (lane == 0) scal[5] = -(tau_i / 2.0) * xv;
    }
    __syncthreads();
    {
      const double alpha = scal[5];
      for (int r = tid; r < n; r += nt) x[r] += alpha * ((r == 0) ? 1.0 : v[(size_t)r * lda]);
    }
    __syncthreads();
    KG_ACC(2)
    KG_MARK()
    // dsyr2 RowMajor Lower, alpha = -1
    for (int r = wid; r < n; r += (nt >> 6)) {
      const double vr = (r == 0) ? 1.0 : v[(size_t)r * lda];
      const double tmp1 = -1.0 * vr, tmp2 = -1.0 * x[r];
      for (int j = lane; j <= r; j += 64) {
        const double vj = (j == 0) ? 1.0 : v[(size_t)j * lda];
        m[(size_t)r * lda + j] += tmp1 * x[j] + tmp2 * vj;
      }
    }
    __syncthreads();
    KG_ACC(3)
  }
  // Householder vectors, diag / sub-diagonal
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, r = idx % N;
    if (i + 2 < N && r < N - i - 1) gH[(size_t)i * N + r] = M[(size_t)(i + 1 + r) * lda + i];
  }
  for (int i = tid; i < N; i += nt) {
    dOut[i] = M[(size_t)i * lda + i];
    if (i + 1 < N) sdOut[i] = M[(size_t)(i + 1) * lda + i];
  }
  if (trace && tid == 0)
    for (int k = 0; k < 4; k++) trace[k] += acc_t[k];
#undef KG_MARK
#undef KG_ACC
}

// Phase B: Q = H_0 ... H_{N-3} (gsl_linalg_symmtd_unpack via
// householder_hm), built transposed (Qt[col][row]) and stored to gQt.
template <bool kLds>
__global__ void __launch_bounds__(1024) k_unpack(int N, const double *__restrict__ gH,
                                                 const double *__restrict__ tau, double *gQt) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lda = N + 1;
  double *M = kLds ? smem : gQt;
  double *h = kLds ? smem + (size_t)N * lda : smem;
  for (int idx = tid; idx < N * lda; idx += nt) {
    const int c = idx / lda, r = idx % lda;
    M[idx] = (r < N && c == r) ? 1.0 : 0.0;
  }
  __syncthreads();
  double *wsh = h + N;  // w_j = col_j . h (phase 1 result)
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int i = N - 3; i >= 0; i--) {
    const double ti = tau[i];
    if (ti == 0.0) continue;  // householder_hm returns early
    const int n = N - (i + 1);
    for (int r = tid; r < n; r += nt) h[r] = gH[(size_t)i * N + r];
    __syncthreads();
    // phase 1: w_j = sum_r Q[i+1+r][i+1+j] h[r], one ordered chain per j
    for (int j = tid; j < n; j += nt) {
      const double *col = M + (size_t)(i + 1 + j) * lda + (i + 1);  // Q[i+1+r][i+1+j], r = 0..n-1
      wsh[j] = ordered_sum(col[0], n - 1, [&](int q) { return col[1 + q] * h[1 + q]; });
    }
    __syncthreads();
    // phase 2 (every wave): Q[.][j] -= tau h w_j, element-parallel
    for (int j = wid; j < n; j += nw) {
      double *col = M + (size_t)(i + 1 + j) * lda + (i + 1);
      const double wj = wsh[j];
      for (int r = lane; r < n; r += 64) col[r] = (r == 0) ? col[0] - ti * wj : col[r] - ti * h[r] * wj;
    }
    __syncthreads();
  }
  if (kLds)
    for (int idx = tid; idx < N * lda; idx += nt) gQt[idx] = M[idx];
}

// ------------------------------------------------------------------------
// Phase A for N > 128 (the matrix no longer fits one CU's LDS): many
// workgroups, each holding a few FULL rows of the symmetric matrix in LDS
// (rows round-robin, row r on workgroup r % P).  Symmetric storage makes
// every gslcblas chain of a row local to its owner:
//   dsymv  x_j = (sum_{c desc} (tau v_c) m[j][c] + (tau v_j) m[j][j]) + tau sum_{c asc} v_c m[j][c]
//          (column j of the lower triangle is row j of the upper one);
//   dsyr2  m[a][b] += (-v_a) x_b + (-x_a) v_b with a >= b, applied to both
//          (a,b) and (b,a), so the two copies stay bit-identical.
// One in-launch hand-off per Householder step (R2 granules, slots per step
// so nothing is ever overwritten within a launch): every owner publishes its
// x_j and every workgroup gathers the whole x.  Everything else of the step
// is recomputed redundantly by every workgroup with identical operands:
// xv and alpha, the next pivot row (its owner publishes it one step ahead,
// off the critical path; every workgroup applies the step's rank-2 update to
// it), its dnrm2 / Householder scalars and the scaled v.  Chains add
// products staged in LDS by all threads (an add-only chain runs at the
// FP64 add latency; tools/ubench_chain2.hip).
constexpr int TMW_TPB = 256;

__host__ __device__ inline size_t tmw_lds_doubles(int N, int RW) {
  return 2 * (size_t)RW * (N + 1) + 5 * (size_t)N + 4 * 16 + 32;  // +32: chain read-ahead slack
}
// rows per workgroup (<= 16): default spreads the rows over up to 256
// workgroups (measured: more workgroups, fewer rows each, is faster — C2
// 0.86 ms with 1 row vs 1.09 ms with 16; C4 7.4 ms with 2 vs 7.9 with 8);
// KORALI_AMD_TMW_ROWS overrides
int tmw_rows(int N) {
  int rw = (N + 255) / 256;
  if (const char *e = getenv("KORALI_AMD_TMW_ROWS")) rw = atoi(e);
  if (rw < 1) rw = 1;
  if (rw > 16) rw = 16;
  while (rw > 1 && tmw_lds_doubles(N, rw) * sizeof(double) > 150 * 1024) rw--;
  return rw;
}
int tmw_groups(int N) { return (N + tmw_rows(N) - 1) / tmw_rows(N); }
size_t tmw_lds_bytes(int N) { return tmw_lds_doubles(N, tmw_rows(N)) * sizeof(double); }
// comm buffer (u64 words): x granules [N][2N], pivot-row granules [N][2N],
// abort word (+ pad to 16 bytes)
size_t tmw_comm_words(int N) { return 4 * (size_t)N * N + 2; }

// Add-only ordered chains over values staged in LDS (one lane): the next 8
// values are loaded while the current 8 are added (two register sets, no
// copies), so LDS latency hides behind the 14-cycle dependent FP64 adds.
// They read up to 16 values past the end (ascending) or before the start
// (descending); those reads stay inside the kernel's LDS and are not added.
__device__ __forceinline__ double staged_chain(double acc, const double *p, int cnt) {
  double a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; u++) a[u] = p[u];
  int q = 0;
  for (; q + 16 <= cnt; q += 16) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = p[q + 8 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = p[q + 16 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += b[u];
  }
  if (q + 8 <= cnt) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = p[q + 8 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
    q += 8;
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + u < cnt) acc += b[u];
  } else {
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + u < cnt) acc += a[u];
  }
  return acc;
}
// acc + p[cnt-1] + p[cnt-2] + ... + p[0]
__device__ __forceinline__ double staged_chain_desc(double acc, const double *p, int cnt) {
  const double *e = p + cnt - 1;  // e[-j] = p[cnt-1-j]
  double a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; u++) a[u] = e[-u];
  int q = 0;
  for (; q + 16 <= cnt; q += 16) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = e[-(q + 8 + u)];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = e[-(q + 16 + u)];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += b[u];
  }
  if (q + 8 <= cnt) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = e[-(q + 8 + u)];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
    q += 8;
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + u < cnt) acc += b[u];
  } else {
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + u < cnt) acc += a[u];
  }
  return acc;
}

__global__ void __launch_bounds__(TMW_TPB) k_tridiag_mw(int N, const double *__restrict__ C, double *gH,
                                                        double *tauOut, double *dOut, double *sdOut,
                                                        unsigned long long *comm, unsigned int *errors,
                                                        unsigned long long *trace) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x;
  const int P = gridDim.x, g = blockIdx.x, RW = (N + P - 1) / P, lda = N + 1;
  double *M = smem;                         // local row k = global row g + k P
  double *Pr = M + (size_t)RW * lda;        // staged dsymv products, same shape
  double *prow = Pr + (size_t)RW * lda;     // current pivot row, indexed by column
  double *nrow = prow + N;                  // next pivot row as published (before this step's update)
  double *vloc = nrow + N;                  // v with v_0 = 1
  double *tv = vloc + N;                    // tau v; also dnrm2 / xv staging
  double *xl = tv + N;                      // x
  double *scal = xl + N;                    // 16 scalars
  double *accb = scal + 16;                 // 16: dsymv acc per local row
  double *t2b = accb + 16;                  // 16: dsymv t2 per local row
  unsigned long long *mskb = (unsigned long long *)(t2b + 16);  // 16: dnrm2 rescale masks
  unsigned long long *gx = comm, *grow = comm + 2 * (size_t)N * N, *abortw = comm + 4 * (size_t)N * N;
  const int writer = (N - 1) % P;  // owns row N-1: runs every step, writes the per-step outputs

  for (int idx = tid; idx < RW * N; idx += nt) {
    const int k = idx / N, c = idx % N, r = g + k * P;
    if (r < N) M[(size_t)k * lda + c] = (c <= r) ? C[(size_t)r * N + c] : C[(size_t)c * N + r];
  }
  for (int c = tid; c < N; c += nt) {
    prow[c] = C[(size_t)c * N];                             // row 0 (symmetrised: column 0)
    nrow[c] = (c >= 1) ? C[(size_t)c * N + 1] : C[1];       // row 1 before any update
  }
  const int maxRow = g + ((N - 1 - g) / P) * P;  // largest row owned
  const bool tr = trace && g == writer && tid == 0;
  unsigned long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tm = tr ? __builtin_amdgcn_s_memtime() : 0;
#define TMW_MARK(k)                                               \
  if (tr) {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    tacc[k] += t_ - tm;                                           \
    tm = t_;                                                      \
  }
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    if (maxRow < i) break;  // no active rows left (never the writer)
    const int n = N - i - 1;
    const unsigned tag = (unsigned)i + 1u;
    unsigned long long *gxp = gx + (size_t)i * 2 * N, *growp = grow + (size_t)i * 2 * N;
    // owner of row i+1 publishes it (state after step i-1) for step i's end
    if (i >= 1 && i + 4 <= N && (i + 1) % P == g) {
      const double *row = M + (size_t)((i + 1) / P) * lda;
      for (int c = i + 2 + tid; c < N; c += nt) put_granule_dbl(growp + 2 * c, tag, row[c]);
    }
    // ---- Householder vector of the pivot row i (redundant on every workgroup)
    const double *v = prow + i + 1;  // v[0] = alpha, v[1..n-1]
    if (wid == 0) {
      const double xnorm = dnrm2_wave(v + 1, 1, n - 1, tv, mskb);
      TMW_MARK(0)
      if (lane == 0) {
        double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
        int branch = 0;
        if (xnorm != 0) {
          const double alpha = v[0];
          beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fdlibm(alpha, xnorm);
          tau_i = (beta - alpha) / beta;
          const double s = alpha - beta;
          if (fabs(s) > DMIN) {
            f1 = 1.0 / s;
            branch = 1;
          } else {
            f1 = EPS / s;
            f2 = 1.0 / EPS;
            branch = 2;
          }
        }
        scal[0] = tau_i;
        scal[1] = f1;
        scal[2] = f2;
        scal[3] = branch ? beta : v[0];  // v_0 after householder_transform
        scal[4] = (double)branch;
        if (g == writer) {
          tauOut[i] = tau_i;
          sdOut[i] = scal[3];
        }
      }
    }
    __syncthreads();
    const double tau_i = scal[0];
    {
      const int branch = (int)scal[4];
      const double f1 = scal[1], f2 = scal[2];
      for (int r = tid; r < n; r += nt) {
        double t = v[r];
        if (r > 0 && branch != 0) {
          t = t * f1;
          if (branch == 2) t = t * f2;
        }
        if (g == writer) gH[(size_t)i * N + r] = (r == 0) ? scal[3] : t;
        vloc[r] = (r == 0) ? 1.0 : t;
        tv[r] = tau_i * ((r == 0) ? 1.0 : t);
      }
    }
    __syncthreads();
    TMW_MARK(1)
    if (tau_i != 0.0) {
      // ---- dsymv: products staged by all threads, then the row chains
      for (int k = 0; k < RW; k++) {
        const int r = g + k * P;
        if (r <= i || r >= N) continue;  // uniform
        for (int q = tid; q < n; q += nt) {
          const int c = i + 1 + q;
          Pr[(size_t)k * lda + c] = ((c > r) ? tv[q] : vloc[q]) * M[(size_t)k * lda + c];
        }
      }
      __syncthreads();
      TMW_MARK(2)
      if (wid < 2 && lane < RW) {
        const int r = g + lane * P;
        if (r > i && r < N) {
          const double *pr = Pr + (size_t)lane * lda;
          if (wid == 0)  // columns c = N-1 .. r+1, descending, then the diagonal
            accb[lane] = staged_chain_desc(0.0, pr + r + 1, N - 1 - r) + tv[r - i - 1] * M[(size_t)lane * lda + r];
          else  // columns c = i+1 .. r-1, ascending
            t2b[lane] = staged_chain(0.0, pr + i + 1, r - i - 1);
        }
      }
      __syncthreads();
      if (tid < RW) {
        const int r = g + tid * P;
        if (r > i && r < N) put_granule_dbl(gxp + 2 * (r - i - 1), tag, accb[tid] + tau_i * t2b[tid]);
      }
      TMW_MARK(3)
      {
        // x of this step and, in the same sweep, the next pivot row as published
        const int nb = (i >= 1 && i + 3 < N) ? n - 1 : 0;
        const bool ok = poll_granule_dbls(gxp, n, xl, growp + 2 * (i + 2), nb, nrow + i + 2, tag, abortw, errors);
        if (__syncthreads_or(!ok)) return;
      }
      TMW_MARK(4)
      // ---- xv = sum x_r v_r (products staged in tv, one ordered chain); alpha = -(tau/2) xv
      for (int r = tid; r < n; r += nt) tv[r] = xl[r] * vloc[r];
      __syncthreads();
      TMW_MARK(5)
      if (tid == 0) scal[5] = -(tau_i / 2.0) * staged_chain(0.0, tv, n);
      __syncthreads();
      TMW_MARK(6)
      {
        const double alpha = scal[5];
        for (int r = tid; r < n; r += nt) xl[r] += alpha * vloc[r];
      }
      __syncthreads();
      TMW_MARK(7)
    }
    // ---- next pivot row (i+1): as published (or from C at i = 0), plus this step's rank-2 update
    if (i + 3 < N) {
      if (i >= 1 && tau_i == 0.0) {  // (with tau != 0 it came with x)
        const bool ok = poll_granule_dbls(growp + 2 * (i + 2), n - 1, nrow + i + 2, growp, 0, nrow, tag, abortw,
                                          errors);
        if (__syncthreads_or(!ok)) return;
      }
      TMW_MARK(8)
      for (int c = i + 2 + tid; c < N; c += nt) {
        double t = nrow[c];
        if (tau_i != 0.0) {
          const int a = c - i - 1;
          const double tmp1 = -1.0 * vloc[a], tmp2 = -1.0 * xl[a];
          t += tmp1 * xl[0] + tmp2 * vloc[0];
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
        for (int jj = tid; jj < n; jj += nt) {
          const int a = jr > jj ? jr : jj, b = jr > jj ? jj : jr;
          const double tmp1 = -1.0 * vloc[a], tmp2 = -1.0 * xl[a];
          row[jj] += tmp1 * xl[b] + tmp2 * vloc[b];
        }
      }
    __syncthreads();
    TMW_MARK(9)
  }
#undef TMW_MARK
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

// ------------------------------------------------------------------------
// Phase A in ONE workgroup for N <= 128 (the full symmetric matrix in LDS,
// 132 KB at N = 128): no in-launch hand-offs at all.  Per Householder step i
// (n = N-i-1), with the same operations in the same order as k_tridiag_mw:
//   A  wave 0: dnrm2 of the pivot row, the Householder scalars (every lane
//      redundantly, no broadcast), the scaled v / tau v and the outputs;
//      waves 1..15 meanwhile finish the previous step's rank-2 update
//   E  dsymv: waves 0-1 run the descending chains, waves 2-3 the ascending
//      chains of rows i+1.., one SIMD each, products formed inline 8 ahead
//   G  x_j = acc_j + tau t2_j and the xv products (all threads)
//   I  wave 0: the xv chain, alpha
//   K  x += alpha v
//   M  rank-2 update of the trailing block: wave 0 updates the next pivot
//      row first and goes straight on to the next step's dnrm2 while waves
//      1..15 update rows i+2.. (the column below the pivot is never read
//      again and is skipped).  Its element formula needs no case split:
//        m[a][b] += (-v_a) x_b + (-x_a) v_b   (a >= b, dsyr2 Lower)
//      has the same two rounded products as (-v_b) x_a + (-x_b) v_a, so both
//      triangles get fl(m + fl(fl(-v_r x_c) + fl(-x_r v_c))) for row r.
// v is double-buffered across steps because A of step i+1 (wave 0) writes it
// while the rank-2 update of step i still reads it.
constexpr int T1_TPB = 1024;
__host__ __device__ inline size_t t1_lds_doubles(int N) {
  return (size_t)N * (N + 1) + 2 * (128 + (size_t)(N + 32)) + (N + 64) + 3 * (size_t)(N + 32) + 16 + 8;
}
bool t1_fits(int N) { return N >= 3 && N <= 128 && t1_lds_doubles(N) * sizeof(double) <= 160 * 1024; }

// acc = 0 + sum_{t < T} a[S t] b[S t] (S = -1 descending, +1 ascending), T
// wave-uniform; products of the next 8 formed while the current 8 are added,
// p / q swapping roles.  Callers align every lane's own chain to the end of
// the T steps: its leading steps read zero-padded operands (0 x finite =
// +-0.0, and a sum that starts at +0.0 is unchanged by adding +-0.0 under
// round-to-nearest), so no lane needs a mask.
template <int S>
__device__ __forceinline__ double padded_chain(const double *a, const double *b, int T_) {
  const int T = __builtin_amdgcn_readfirstlane(T_);
  double acc = 0.0;
  int t = 0;
  if (T >= 8) {
    double p[8], q[8];
#pragma unroll
    for (int u = 0; u < 8; u++) p[u] = a[S * u] * b[S * u];
    t = 8;
    for (; t + 16 <= T; t += 16) {
      const double *at = a + S * t, *bt = b + S * t;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        q[u] = at[S * u] * bt[S * u];
        acc += p[u];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        p[u] = at[S * (8 + u)] * bt[S * (8 + u)];
        acc += q[u];
      }
    }
    if (t + 8 <= T) {
      const double *at = a + S * t, *bt = b + S * t;
#pragma unroll
      for (int u = 0; u < 8; u++) {
        q[u] = at[S * u] * bt[S * u];
        acc += p[u];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) p[u] = q[u];
      t += 8;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc += p[u];
  }
  for (; t < T; t++) acc += a[S * t] * b[S * t];
  return acc;
}

__global__ void __launch_bounds__(T1_TPB) k_tridiag_1wg(int N, const double *__restrict__ C, double *gH,
                                                        double *tauOut, double *dOut, double *sdOut,
                                                        unsigned long long *trace, int xflags) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x;
  const int lda = N + 1, VS = N + 32;
  double *M = smem;                    // row r at r*lda; column N is a zero pad
  double *vbuf = M + (size_t)N * lda;  // v (v_0 = 1), two buffers (step parity),
                                       // each after 128 zeros
  double *tv = vbuf + 2 * (128 + VS);  // tau v, zeros from index n to n+63
  double *xl = tv + (N + 64);          // x
  double *t2b = xl + VS;               // ascending dsymv chains
  double *sv = t2b + VS;               // dnrm2 addends, then the xv products
  double *scal = sv + VS;              // 16 scalars
  unsigned long long *msk = (unsigned long long *)(scal + 16);  // dnrm2 rescale masks
  const bool tr = trace && tid == 0;
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tm = tr ? __builtin_amdgcn_s_memtime() : 0;
  if ((xflags & 1) && wid == 0) __builtin_amdgcn_s_setprio(3);
  if ((xflags & 4) && wid > 0 && wid < 4) __builtin_amdgcn_s_setprio(2);
#define T1_MARK(k)                                                \
  if (tr) {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    tacc[k] += t_ - tm;                                           \
    tm = t_;                                                      \
  }
  // zero everything first: the padded dsymv chains read the pad column, the
  // zeros around v / tau v and (past row N-1) the vectors, all finite
  for (size_t idx = tid; idx < t1_lds_doubles(N); idx += nt) smem[idx] = 0.0;
  __syncthreads();
  for (int idx = tid; idx < N * N; idx += nt) {
    const int r = idx / N, c = idx % N;
    M[(size_t)r * lda + c] = (c <= r) ? C[(size_t)r * N + c] : C[(size_t)c * N + r];
  }
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    const int n = N - i - 1;
    double *vloc = vbuf + 128 + (i & 1) * (128 + VS);
    // ---- A: Householder vector of pivot row i (wave 0; every lane holds the scalars)
    if (wid == 0) {
      const double *v = M + (size_t)i * lda + i + 1;  // v[0] = alpha, v[1..n-1]
      const double xnorm = dnrm2_wave128(v + 1, n - 1, sv);
      if (tr) {
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();
        tacc[6] += t_ - tm;
        tm = t_;
      }
      double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
      int branch = 0;
      if (xnorm != 0) {
        const double alpha = v[0];
        beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fdlibm(alpha, xnorm);
        tau_i = (beta - alpha) / beta;
        const double sgap = alpha - beta;
        if (fabs(sgap) > DMIN) {
          f1 = 1.0 / sgap;
          branch = 1;
        } else {
          f1 = EPS / sgap;
          f2 = 1.0 / EPS;
          branch = 2;
        }
      }
      const double v0out = branch ? beta : v[0];
      if (tr) {
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();
        tacc[7] += t_ - tm;
        tm = t_;
      }
      for (int r = lane; r < n; r += 64) {
        double t = v[r];
        if (r > 0 && branch != 0) {
          t = t * f1;
          if (branch == 2) t = t * f2;
        }
        gH[(size_t)i * N + r] = (r == 0) ? v0out : t;
        const double vr = (r == 0) ? 1.0 : t;
        vloc[r] = vr;
        tv[r] = tau_i * vr;
      }
      tv[n + lane] = 0.0;  // the descending chains' leading pad
      if (lane == 0) {
        scal[0] = tau_i;
        tauOut[i] = tau_i;
        sdOut[i] = v0out;
      }
    }
    T1_MARK(0)
    __syncthreads();
    T1_MARK(1)
    const double tau_i = scal[0];
    if (tau_i == 0.0) continue;  // no update this step (uniform)
    // ---- E: dsymv chains of rows r = i+1+j, every lane's chain aligned to
    // the end of its wave's T steps (leading steps read the zero pads)
    if (wid < 4) {
      const unsigned long long te0 = (trace && lane == 0) ? __builtin_amdgcn_s_memtime() : 0;
      const int j = lane + 64 * (wid & 1);
      const int r = i + 1 + (j < n ? j : n - 1);
      const double *row = M + (size_t)r * lda;
      const int lo = 64 * (wid & 1);                     // smallest j of this wave
      const int hi = min(n, lo + 64) - 1;                // largest active j
      if (wid < 2) {  // c = N-1 .. r+1 descending (n-1-j terms), then the diagonal
        const int sh = j - lo;
        const double acc = padded_chain<-1>(tv + (n - 1) + sh, row + (N - 1) + sh, n - 1 - lo);
        if (j < n) xl[j] = acc + tv[j] * row[r];
      } else {  // c = i+1 .. r-1 ascending (j terms)
        const int sh = j - hi;
        const double acc = padded_chain<1>(vloc + sh, row + i + 1 + sh, hi);
        if (j < n) t2b[j] = acc;
      }
      if (trace && lane == 0 && (wid == 0 || wid == 3)) {
        __builtin_amdgcn_s_waitcnt(0);
        trace[wid == 0 ? 14 : 15] += __builtin_amdgcn_s_memtime() - te0;  // one writer per slot
      }
    }
    __syncthreads();
    T1_MARK(2)
    // ---- G, I, K on wave 0 alone (two elements per lane, no block barriers):
    // x = acc + tau t2 and the xv products, the xv chain, alpha = -(tau/2) xv,
    // x += alpha v
    if (wid == 0) {
      for (int r = lane; r < n; r += 64) {
        const double x = xl[r] + tau_i * t2b[r];
        xl[r] = x;
        sv[r] = x * vloc[r];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const double alpha = -(tau_i / 2.0) * staged_chain(0.0, sv, n);
      T1_MARK(3)
      for (int r = lane; r < n; r += 64) xl[r] += alpha * vloc[r];
    }
    __syncthreads();
    T1_MARK(4)
    // ---- M: rank-2 update (both triangles), next pivot row first on wave 0
    if (wid == 0) {
      double *row = M + (size_t)(i + 1) * lda + i + 1;
      const double x0 = xl[0], v0 = vloc[0];
      for (int jj = lane; jj < n; jj += 64) {
        const double tmp1 = -1.0 * vloc[jj], tmp2 = -1.0 * xl[jj];
        row[jj] += tmp1 * x0 + tmp2 * v0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else if (n > 1) {
      // lane's columns jj = 1 + lane, 65 + lane (n <= 128)
      const int ja = 1 + lane, jb = 65 + lane;
      const double xa = ja < n ? xl[ja] : 0.0, va = ja < n ? vloc[ja] : 0.0;
      const double xb = jb < n ? xl[jb] : 0.0, vb = jb < n ? vloc[jb] : 0.0;
      for (int jr = wid; jr < n; jr += 15) {
        double *row = M + (size_t)(i + 1 + jr) * lda + i + 1;
        const double nvr = -1.0 * vloc[jr], nxr = -1.0 * xl[jr];
        if (ja < n) row[ja] += nvr * xa + nxr * va;
        if (jb < n) row[jb] += nvr * xb + nxr * vb;
      }
    }
    T1_MARK(5)
  }
  __syncthreads();
#undef T1_MARK
  if (tr) {
    for (int k = 0; k < 6; k++) trace[8 + k] += tacc[k];
    trace[29] += tacc[6];
    trace[30] += tacc[7];
  }
  for (int r = tid; r < N; r += nt) {
    dOut[r] = M[(size_t)r * lda + r];
    if (r == N - 2) sdOut[r] = M[(size_t)r * lda + r + 1];
  }
}

// ------------------------------------------------------------------------
// Phase A in ONE workgroup, version 2 (the default for N <= 128): the
// trailing block is stored as its STRICTLY UPPER triangle (zeros on and
// below the diagonal; the diagonal lives in its own vector).  Then every
// gslcblas dsymv chain walks a zero-padded sequence without any lane mask:
//   descending (rows r, lockstep over columns c = N-1, N-2, ...):
//     acc_r += tv_c M[r][c]   — M[r][c] = 0 for c <= r adds +-0.0 to an
//     accumulator that started at +0.0 and so is never -0.0: unchanged
//   ascending (c = i+1, i+2, ...): t2_r += v_c M[c][r]  (M[c][r] = m[r][c]
//     for c < r by symmetry, 0 for c >= r)
// and the rank-2 update touches only the upper triangle and the diagonal
// (half of the full symmetric update).  Both chain reads are conflict-free
// (a column walk over rows of stride N+1, a row walk over consecutive r);
// the vector operand is a broadcast.  dnrm2's ssq chain takes its rare
// rescaling steps (a new running maximum) through scalar branches, so the
// common step is one dependent add.  Operation order is the reference's
// throughout, so the result is bit-identical to
// k_tridiag_1wg and the oracle.
constexpr int T2_TPB = 1024, T2_VP = 16;  // T2_VP: pad before / after each vector (chain read-ahead)
__host__ __device__ inline size_t t2_vec(int N) { return (size_t)N + 2 * T2_VP; }
__host__ __device__ inline size_t t2_lds_doubles(int N) {
  // M | dg | vA[2] | tvA[2] | xA[2] | xd | t2 | sv (192) | scal
  return (size_t)N * (N + 1) + 9 * t2_vec(N) + 192 + 16;
}
bool t2_fits(int N) { return N >= 3 && N <= 128 && t2_lds_doubles(N) * sizeof(double) <= 160 * 1024; }

// s_waitcnt lgkmcnt(K) alone (vmcnt / expcnt left at their maxima).  An
// explicit wait satisfies the compiler's own wait insertion for every LDS
// load it covers, so a batch of adds that follows waits once, not per
// value (a wait per dependent add costs ~4 cycles of the ~8 of the add).
#define KG_WAIT_LGKM(K) __builtin_amdgcn_s_waitcnt(0xC07F | ((K) << 8))

// acc = 0 + sum_{t < T} w[S t] m[S t ms] in order (T wave-uniform); the next
// 8 steps' operands are read while the current 8 are multiplied and added
// (two register sets, roles alternating).  Scheduling barriers keep the
// read-ahead where it is written and one explicit wait per batch replaces
// the compiler's wait per operand (KG_WAIT_LGKM: the compiler still adds a
// wait for anything the explicit one does not cover, so the count only
// tunes speed, never correctness).  Reads run at most 8 steps past T (in
// bounds by the LDS layout) and are not added.
#define KG_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
template <int S>
__device__ __forceinline__ double lockstep_chain(const double *w, const double *m, int ms, int T_) {
  const int T = __builtin_amdgcn_readfirstlane(T_);
  double acc = 0.0;
  double wa[8], ma[8], wb[8], mb[8];
#pragma unroll
  for (int u = 0; u < 8; u++) {
    wa[u] = w[S * u];
    ma[u] = m[S * u * ms];
  }
  int t = 0;
  for (; t + 16 <= T; t += 16) {
    const double *wt = w + S * (t + 8), *mt = m + S * (t + 8) * ms;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      wb[u] = wt[S * u];
      mb[u] = mt[S * u * ms];
    }
    KG_SCHED_FENCE();
    KG_WAIT_LGKM(12);
#pragma unroll
    for (int u = 0; u < 8; u++) acc += wa[u] * ma[u];
    KG_SCHED_FENCE();
    wt = w + S * (t + 16);
    mt = m + S * (t + 16) * ms;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      wa[u] = wt[S * u];
      ma[u] = mt[S * u * ms];
    }
    KG_SCHED_FENCE();
    KG_WAIT_LGKM(12);
#pragma unroll
    for (int u = 0; u < 8; u++) acc += wb[u] * mb[u];
    KG_SCHED_FENCE();
  }
  if (t + 8 <= T) {
    const double *wt = w + S * (t + 8), *mt = m + S * (t + 8) * ms;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      wb[u] = wt[S * u];
      mb[u] = mt[S * u * ms];
    }
    KG_SCHED_FENCE();
    KG_WAIT_LGKM(12);
#pragma unroll
    for (int u = 0; u < 8; u++) acc += wa[u] * ma[u];
    t += 8;
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (t + u < T) acc += wb[u] * mb[u];
  } else {
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (t + u < T) acc += wa[u] * ma[u];
  }
  return acc;
}

// ordered add-only chain acc + x_0 + ... + x_{cnt-1} over values held one
// per lane (x_e in lane e of v0 for e < 64, of v1 for e >= 64; cnt <= 128),
// each read into scalar registers with v_readlane (no LDS traffic); every
// lane returns the sum
__device__ __forceinline__ double lane_sum(double acc, double v0, double v1, int cnt_) {
  const int cnt = __builtin_amdgcn_readfirstlane(cnt_);
  const long long b0 = __double_as_longlong(v0), b1 = __double_as_longlong(v1);
  const int l0 = (int)b0, h0 = (int)(b0 >> 32), l1 = (int)b1, h1 = (int)(b1 >> 32);
#define KG_LANE_STEP(L, H, E)                                                                        \
  acc += __longlong_as_double(((long long)__builtin_amdgcn_readlane(H, E) << 32) |                    \
                              (unsigned int)__builtin_amdgcn_readlane(L, E))
  int e = 0;
  for (; e + 8 <= min(cnt, 64); e += 8) {
#pragma unroll
    for (int u = 0; u < 8; u++) KG_LANE_STEP(l0, h0, e + u);
  }
  for (; e < min(cnt, 64); e++) KG_LANE_STEP(l0, h0, e);
  for (; e + 8 <= cnt; e += 8) {
#pragma unroll
    for (int u = 0; u < 8; u++) KG_LANE_STEP(l1, h1, e - 64 + u);
  }
  for (; e < cnt; e++) KG_LANE_STEP(l1, h1, e - 64);
#undef KG_LANE_STEP
  return acc;
}


// staged_sum reading pairs with 16-byte LDS loads (p 16-byte aligned): the
// next 8 values are in flight (4 loads) while the current 8 are added after
// ONE wait
__device__ __forceinline__ double staged_sum_v2(double acc, const double *p, int cnt_) {
  const int cnt = __builtin_amdgcn_readfirstlane(cnt_);
  const double2 *q2 = (const double2 *)p;
  double2 a[4], b[4];
#pragma unroll
  for (int u = 0; u < 4; u++) a[u] = q2[u];
  int q = 0;
  for (; q + 16 <= cnt; q += 16) {
#pragma unroll
    for (int u = 0; u < 4; u++) b[u] = q2[(q >> 1) + 4 + u];
    KG_WAIT_LGKM(4);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      acc += a[u].x;
      acc += a[u].y;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) a[u] = q2[(q >> 1) + 8 + u];
    KG_WAIT_LGKM(4);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      acc += b[u].x;
      acc += b[u].y;
    }
  }
  if (q + 8 <= cnt) {
#pragma unroll
    for (int u = 0; u < 4; u++) b[u] = q2[(q >> 1) + 4 + u];
    KG_WAIT_LGKM(4);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      acc += a[u].x;
      acc += a[u].y;
    }
    q += 8;
    KG_WAIT_LGKM(0);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (q + 2 * u < cnt) acc += b[u].x;
      if (q + 2 * u + 1 < cnt) acc += b[u].y;
    }
  } else {
    KG_WAIT_LGKM(0);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (q + 2 * u < cnt) acc += a[u].x;
      if (q + 2 * u + 1 < cnt) acc += a[u].y;
    }
  }
  return acc;
}

// acc + p[0] + ... + p[cnt-1] (p an LDS address, wave-uniform; 0 <= cnt
// <= 128) as ONE straight-line inline-assembly sequence: the next 8 values
// are in flight (8 ds_read_b64) while the current 8 are added after a
// single counted wait; the only branches are forward exits to the tail.
// (Compiled code waits before every add and hoists the loads next to their
// uses, ~15 cycles per element; a dependent FP64 add is 8.3, an LDS-fed
// add chain waiting once per 8 values 10.6 — tools/ubench_issue.hip.)
// Reads run up to 16 values past cnt (callers pad) and are not added.
__device__ __forceinline__ double lds_chain_add(double acc, const double *p, int cnt) {
  const unsigned va = (unsigned)(size_t)(const __attribute__((address_space(3))) double *)p;
  int rem = __builtin_amdgcn_readfirstlane(cnt);
  double a[8], b[8];
  asm volatile(
"ds_read_b64 %[a0], %[va] offset:0\n"
"ds_read_b64 %[a1], %[va] offset:8\n"
"ds_read_b64 %[a2], %[va] offset:16\n"
"ds_read_b64 %[a3], %[va] offset:24\n"
"ds_read_b64 %[a4], %[va] offset:32\n"
"ds_read_b64 %[a5], %[va] offset:40\n"
"ds_read_b64 %[a6], %[va] offset:48\n"
"ds_read_b64 %[a7], %[va] offset:56\n"
"ds_read_b64 %[b0], %[va] offset:64\n"
"ds_read_b64 %[b1], %[va] offset:72\n"
"ds_read_b64 %[b2], %[va] offset:80\n"
"ds_read_b64 %[b3], %[va] offset:88\n"
"ds_read_b64 %[b4], %[va] offset:96\n"
"ds_read_b64 %[b5], %[va] offset:104\n"
"ds_read_b64 %[b6], %[va] offset:112\n"
"ds_read_b64 %[b7], %[va] offset:120\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:128\n"
"ds_read_b64 %[a1], %[va] offset:136\n"
"ds_read_b64 %[a2], %[va] offset:144\n"
"ds_read_b64 %[a3], %[va] offset:152\n"
"ds_read_b64 %[a4], %[va] offset:160\n"
"ds_read_b64 %[a5], %[va] offset:168\n"
"ds_read_b64 %[a6], %[va] offset:176\n"
"ds_read_b64 %[a7], %[va] offset:184\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:192\n"
"ds_read_b64 %[b1], %[va] offset:200\n"
"ds_read_b64 %[b2], %[va] offset:208\n"
"ds_read_b64 %[b3], %[va] offset:216\n"
"ds_read_b64 %[b4], %[va] offset:224\n"
"ds_read_b64 %[b5], %[va] offset:232\n"
"ds_read_b64 %[b6], %[va] offset:240\n"
"ds_read_b64 %[b7], %[va] offset:248\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:256\n"
"ds_read_b64 %[a1], %[va] offset:264\n"
"ds_read_b64 %[a2], %[va] offset:272\n"
"ds_read_b64 %[a3], %[va] offset:280\n"
"ds_read_b64 %[a4], %[va] offset:288\n"
"ds_read_b64 %[a5], %[va] offset:296\n"
"ds_read_b64 %[a6], %[va] offset:304\n"
"ds_read_b64 %[a7], %[va] offset:312\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:320\n"
"ds_read_b64 %[b1], %[va] offset:328\n"
"ds_read_b64 %[b2], %[va] offset:336\n"
"ds_read_b64 %[b3], %[va] offset:344\n"
"ds_read_b64 %[b4], %[va] offset:352\n"
"ds_read_b64 %[b5], %[va] offset:360\n"
"ds_read_b64 %[b6], %[va] offset:368\n"
"ds_read_b64 %[b7], %[va] offset:376\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:384\n"
"ds_read_b64 %[a1], %[va] offset:392\n"
"ds_read_b64 %[a2], %[va] offset:400\n"
"ds_read_b64 %[a3], %[va] offset:408\n"
"ds_read_b64 %[a4], %[va] offset:416\n"
"ds_read_b64 %[a5], %[va] offset:424\n"
"ds_read_b64 %[a6], %[va] offset:432\n"
"ds_read_b64 %[a7], %[va] offset:440\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:448\n"
"ds_read_b64 %[b1], %[va] offset:456\n"
"ds_read_b64 %[b2], %[va] offset:464\n"
"ds_read_b64 %[b3], %[va] offset:472\n"
"ds_read_b64 %[b4], %[va] offset:480\n"
"ds_read_b64 %[b5], %[va] offset:488\n"
"ds_read_b64 %[b6], %[va] offset:496\n"
"ds_read_b64 %[b7], %[va] offset:504\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:512\n"
"ds_read_b64 %[a1], %[va] offset:520\n"
"ds_read_b64 %[a2], %[va] offset:528\n"
"ds_read_b64 %[a3], %[va] offset:536\n"
"ds_read_b64 %[a4], %[va] offset:544\n"
"ds_read_b64 %[a5], %[va] offset:552\n"
"ds_read_b64 %[a6], %[va] offset:560\n"
"ds_read_b64 %[a7], %[va] offset:568\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:576\n"
"ds_read_b64 %[b1], %[va] offset:584\n"
"ds_read_b64 %[b2], %[va] offset:592\n"
"ds_read_b64 %[b3], %[va] offset:600\n"
"ds_read_b64 %[b4], %[va] offset:608\n"
"ds_read_b64 %[b5], %[va] offset:616\n"
"ds_read_b64 %[b6], %[va] offset:624\n"
"ds_read_b64 %[b7], %[va] offset:632\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:640\n"
"ds_read_b64 %[a1], %[va] offset:648\n"
"ds_read_b64 %[a2], %[va] offset:656\n"
"ds_read_b64 %[a3], %[va] offset:664\n"
"ds_read_b64 %[a4], %[va] offset:672\n"
"ds_read_b64 %[a5], %[va] offset:680\n"
"ds_read_b64 %[a6], %[va] offset:688\n"
"ds_read_b64 %[a7], %[va] offset:696\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:704\n"
"ds_read_b64 %[b1], %[va] offset:712\n"
"ds_read_b64 %[b2], %[va] offset:720\n"
"ds_read_b64 %[b3], %[va] offset:728\n"
"ds_read_b64 %[b4], %[va] offset:736\n"
"ds_read_b64 %[b5], %[va] offset:744\n"
"ds_read_b64 %[b6], %[va] offset:752\n"
"ds_read_b64 %[b7], %[va] offset:760\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:768\n"
"ds_read_b64 %[a1], %[va] offset:776\n"
"ds_read_b64 %[a2], %[va] offset:784\n"
"ds_read_b64 %[a3], %[va] offset:792\n"
"ds_read_b64 %[a4], %[va] offset:800\n"
"ds_read_b64 %[a5], %[va] offset:808\n"
"ds_read_b64 %[a6], %[va] offset:816\n"
"ds_read_b64 %[a7], %[va] offset:824\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:832\n"
"ds_read_b64 %[b1], %[va] offset:840\n"
"ds_read_b64 %[b2], %[va] offset:848\n"
"ds_read_b64 %[b3], %[va] offset:856\n"
"ds_read_b64 %[b4], %[va] offset:864\n"
"ds_read_b64 %[b5], %[va] offset:872\n"
"ds_read_b64 %[b6], %[va] offset:880\n"
"ds_read_b64 %[b7], %[va] offset:888\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:896\n"
"ds_read_b64 %[a1], %[va] offset:904\n"
"ds_read_b64 %[a2], %[va] offset:912\n"
"ds_read_b64 %[a3], %[va] offset:920\n"
"ds_read_b64 %[a4], %[va] offset:928\n"
"ds_read_b64 %[a5], %[va] offset:936\n"
"ds_read_b64 %[a6], %[va] offset:944\n"
"ds_read_b64 %[a7], %[va] offset:952\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[b0], %[va] offset:960\n"
"ds_read_b64 %[b1], %[va] offset:968\n"
"ds_read_b64 %[b2], %[va] offset:976\n"
"ds_read_b64 %[b3], %[va] offset:984\n"
"ds_read_b64 %[b4], %[va] offset:992\n"
"ds_read_b64 %[b5], %[va] offset:1000\n"
"ds_read_b64 %[b6], %[va] offset:1008\n"
"ds_read_b64 %[b7], %[va] offset:1016\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 2f\n"
"v_add_f64 %[acc], %[acc], %[a0]\n"
"v_add_f64 %[acc], %[acc], %[a1]\n"
"v_add_f64 %[acc], %[acc], %[a2]\n"
"v_add_f64 %[acc], %[acc], %[a3]\n"
"v_add_f64 %[acc], %[acc], %[a4]\n"
"v_add_f64 %[acc], %[acc], %[a5]\n"
"v_add_f64 %[acc], %[acc], %[a6]\n"
"v_add_f64 %[acc], %[acc], %[a7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"ds_read_b64 %[a0], %[va] offset:1024\n"
"ds_read_b64 %[a1], %[va] offset:1032\n"
"ds_read_b64 %[a2], %[va] offset:1040\n"
"ds_read_b64 %[a3], %[va] offset:1048\n"
"ds_read_b64 %[a4], %[va] offset:1056\n"
"ds_read_b64 %[a5], %[va] offset:1064\n"
"ds_read_b64 %[a6], %[va] offset:1072\n"
"ds_read_b64 %[a7], %[va] offset:1080\n"
"s_waitcnt lgkmcnt(8)\n s_cmp_lt_i32 %[rem], 8\n s_cbranch_scc1 3f\n"
"v_add_f64 %[acc], %[acc], %[b0]\n"
"v_add_f64 %[acc], %[acc], %[b1]\n"
"v_add_f64 %[acc], %[acc], %[b2]\n"
"v_add_f64 %[acc], %[acc], %[b3]\n"
"v_add_f64 %[acc], %[acc], %[b4]\n"
"v_add_f64 %[acc], %[acc], %[b5]\n"
"v_add_f64 %[acc], %[acc], %[b6]\n"
"v_add_f64 %[acc], %[acc], %[b7]\n"
"s_sub_i32 %[rem], %[rem], 8\n"
"s_branch 9f\n"
"2:\n"
"s_cmp_lt_i32 %[rem], 1\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a0]\n"
"s_cmp_lt_i32 %[rem], 2\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a1]\n"
"s_cmp_lt_i32 %[rem], 3\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a2]\n"
"s_cmp_lt_i32 %[rem], 4\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a3]\n"
"s_cmp_lt_i32 %[rem], 5\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a4]\n"
"s_cmp_lt_i32 %[rem], 6\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a5]\n"
"s_cmp_lt_i32 %[rem], 7\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[a6]\n"
"s_branch 9f\n"
"3:\n"
"s_cmp_lt_i32 %[rem], 1\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b0]\n"
"s_cmp_lt_i32 %[rem], 2\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b1]\n"
"s_cmp_lt_i32 %[rem], 3\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b2]\n"
"s_cmp_lt_i32 %[rem], 4\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b3]\n"
"s_cmp_lt_i32 %[rem], 5\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b4]\n"
"s_cmp_lt_i32 %[rem], 6\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b5]\n"
"s_cmp_lt_i32 %[rem], 7\n s_cbranch_scc1 9f\n v_add_f64 %[acc], %[acc], %[b6]\n"
"9:\n s_waitcnt lgkmcnt(0)\n"
      : [acc] "+&v"(acc), [rem] "+&s"(rem), [a0] "=&v"(a[0]), [a1] "=&v"(a[1]), [a2] "=&v"(a[2]), [a3] "=&v"(a[3]), [a4] "=&v"(a[4]), [a5] "=&v"(a[5]), [a6] "=&v"(a[6]), [a7] "=&v"(a[7]), [b0] "=&v"(b[0]), [b1] "=&v"(b[1]), [b2] "=&v"(b[2]), [b3] "=&v"(b[3]), [b4] "=&v"(b[4]), [b5] "=&v"(b[5]), [b6] "=&v"(b[6]), [b7] "=&v"(b[7])
      : [va] "v"(va)
      : "scc", "memory");
  return acc;
}

// staged_sum with the loads 16 ahead: three register sets of 8 rotate
// (a wait covers only the batch it consumes); reads up to 24 past cnt
__device__ __forceinline__ double staged_sum3(double acc, const double *p, int cnt_) {
  const int cnt = __builtin_amdgcn_readfirstlane(cnt_);
  double a[8], b[8], c[8];
#pragma unroll
  for (int u = 0; u < 8; u++) {
    a[u] = p[u];
    b[u] = p[8 + u];
  }
  int q = 0;
  for (; q + 24 <= cnt; q += 24) {
#pragma unroll
    for (int u = 0; u < 8; u++) c[u] = p[q + 16 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = p[q + 24 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += b[u];
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = p[q + 32 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += c[u];
  }
  // tail: fewer than 24 left; a holds q..q+7, b holds q+8..q+15
#pragma unroll
  for (int u = 0; u < 8; u++)
    if (q + u < cnt) acc += a[u];
#pragma unroll
  for (int u = 0; u < 8; u++)
    if (q + 8 + u < cnt) acc += b[u];
  if (q + 16 < cnt) {
#pragma unroll
    for (int u = 0; u < 8; u++) c[u] = p[q + 16 + u];
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + 16 + u < cnt) acc += c[u];
  }
  return acc;
}

// ordered add-only chain acc + p[0] + ... + p[cnt-1] over LDS values, 8
// loaded ahead (reads up to 8 past cnt, not added)
__device__ __forceinline__ double staged_sum(double acc, const double *p, int cnt_) {
  const int cnt = __builtin_amdgcn_readfirstlane(cnt_);
  double a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; u++) a[u] = p[u];
  int q = 0;
  for (; q + 16 <= cnt; q += 16) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = p[q + 8 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = p[q + 16 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += b[u];
  }
  if (q + 8 <= cnt) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = p[q + 8 + u];
#pragma unroll
    for (int u = 0; u < 8; u++) acc += a[u];
    q += 8;
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + u < cnt) acc += b[u];
  } else {
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (q + u < cnt) acc += a[u];
  }
  return acc;
}

// rescale flags of the 8 addends e .. e+7 (e a multiple of 8)
__device__ __forceinline__ unsigned nrm2_bits(unsigned long long k0, unsigned long long k1, int e) {
  return (unsigned)(((e < 64) ? (k0 >> e) : (k1 >> (e - 64))) & 0xffULL);
}
// 8 steps of dnrm2's ssq recurrence: ssq += t (plain) or ssq = 1 + ssq t t
// (a new running maximum, rare: taken through scalar branches so the plain
// step stays one dependent add)
__device__ __forceinline__ double nrm2_batch(double ssq, const double (&t)[8], unsigned bits) {
  if (bits == 0u) {
#pragma unroll
    for (int u = 0; u < 8; u++) ssq += t[u];
  } else {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if ((bits >> u) & 1u) {
        __asm__ volatile("" ::: "memory");
        ssq = 1.0 + ssq * t[u] * t[u];
      } else {
        ssq += t[u];
      }
    }
  }
  return ssq;
}

// gslcblas dnrm2 of m <= 128 elements held in registers (element e = lane in
// x0, e = 64 + lane in x1; only e < m are read), by one wave; every lane
// returns the result.  Addends staged in sv (m rounded up to 8, zero-padded:
// +0.0 leaves ssq >= 1 unchanged).
__device__ double dnrm2_regs(double x0, double x1, int m, double *sv, bool tr, unsigned long long *tacc,
                             unsigned long long &tm) {
  const int lane = threadIdx.x & 63;
  const int m8 = (m + 7) & ~7;
  const int e0 = lane, e1 = lane + 64;
  const double a0 = e0 < m ? fabs(x0) : 0.0, a1 = e1 < m ? fabs(x1) : 0.0;
  double pm0, pm1;
  wave_prefix_max2_nonneg(a0, a1, pm0, pm1);
  const double c0 = readlane_d(pm0, 63);
  const double b0 = dpp_d<0x138, 0xf>(pm0);            // running max before e0 (lane 0: 0.0)
  const double b1 = fmax(dpp_d<0x138, 0xf>(pm1), c0);  // before e1
  const bool z0 = a0 != 0.0, z1 = a1 != 0.0;           // zero elements are skipped by dnrm2
  const bool n0 = z0 && b0 < a0, n1 = z1 && b1 < a1;   // a new running maximum
  // one division per element, operands selected (zeros: 0 / 1), no branches
  const double q0 = (z0 ? (n0 ? b0 : a0) : 0.0) / (z0 ? (n0 ? a0 : b0) : 1.0);
  const double q1 = (z1 ? (n1 ? b1 : a1) : 0.0) / (z1 ? (n1 ? a1 : b1) : 1.0);
  const unsigned long long k0 = __ballot(n0), k1 = __ballot(n1);
  sv[e0] = n0 ? q0 : q0 * q0;  // e >= m: q = 0 (sv holds 192 doubles)
  sv[e1] = n1 ? q1 : q1 * q1;
  const double carry = fmax(c0, readlane_d(pm1, 63));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (tr) {
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();
    tacc[0] += t_ - tm;
    tm = t_;
  }
  // the ssq recurrence in the reference's order: batches of 8 addends, the
  // next batch loaded while the current one is added (two register sets,
  // roles alternating: a wait covers only the batch it consumes)
  double ssq = 1.0;
  double a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; u++) a[u] = sv[u];
  for (int e = 0; e < m8; e += 16) {
#pragma unroll
    for (int u = 0; u < 8; u++) b[u] = sv[e + 8 + u];  // sv has 64 doubles of slack
    ssq = nrm2_batch(ssq, a, nrm2_bits(k0, k1, e));
    if (e + 8 >= m8) break;
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = sv[e + 16 + u];
    ssq = nrm2_batch(ssq, b, nrm2_bits(k0, k1, e + 8));
  }
  __builtin_amdgcn_wave_barrier();
  return (m == 1) ? fabs(x0) : carry * sqrt(ssq);
}

__global__ void __launch_bounds__(T2_TPB) k_tridiag_1wg2(int N, const double *__restrict__ C, double *gH,
                                                         double *tauOut, double *dOut, double *sdOut,
                                                         unsigned long long *trace) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x;
  const int lda = N + 1, VS = (int)t2_vec(N);
  double *M = smem;                       // strictly upper triangle, row r at r*lda
  double *dg = M + (size_t)N * lda + T2_VP;  // diagonal
  double *vbase = dg - T2_VP + VS;        // vA[2], tvA[2], xA[2]: absolute column index
  auto vA = [&](int p) { return vbase + (size_t)p * VS + T2_VP; };
  auto tvA = [&](int p) { return vbase + (size_t)(2 + p) * VS + T2_VP; };
  auto xA = [&](int p) { return vbase + (size_t)(4 + p) * VS + T2_VP; };
  double *xd = vbase + (size_t)6 * VS + T2_VP;  // descending chain + diagonal term, by j
  double *t2 = xd + VS;                          // ascending chain, by j
  double *sv = t2 + VS - T2_VP;                  // 192: dnrm2 addends, then the xv products
  double *scal = sv + 192;                       // 16 scalars
  const bool tr = trace && tid == 0;
  unsigned long long tacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, tm = tr ? __builtin_amdgcn_s_memtime() : 0;
#define T2_MARK(k)                                                \
  if (tr) {                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    tacc[k] += t_ - tm;                                           \
    tm = t_;                                                      \
  }
  for (size_t idx = tid; idx < t2_lds_doubles(N); idx += nt) smem[idx] = 0.0;
  __syncthreads();
  // symmetrise from the lower triangle (CMAES.cpp.base:908-913): upper
  // element (r, c > r) = C[c][r]; diagonal C[r][r]
  for (int idx = tid; idx < N * N; idx += nt) {
    const int r = idx / N, c = idx % N;
    if (c > r) M[(size_t)r * lda + c] = C[(size_t)c * N + r];
    else if (c == r) dg[r] = C[(size_t)r * N + r];
  }
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    const int n = N - i - 1, par = i & 1;
    double *va = vA(par), *tva = tvA(par), *xa = xA(par);
    // ---- A (wave 0): Householder vector of pivot row i; alpha = M[i][i+1],
    // dnrm2 over x_e = M[i][i+2+e], e < n-1
    if (wid == 0) {
      const double *prow = M + (size_t)i * lda;
      const int m = n - 1;
      const double alpha = prow[i + 1];
      const double x0 = prow[i + 2 + min(lane, m - 1)], x1 = prow[i + 2 + min(lane + 64, m - 1)];
      const double xnorm = dnrm2_regs(x0, x1, m, sv, tr, tacc + 8, tm);
      T2_MARK(6)
      double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
      int branch = 0;
      if (xnorm != 0) {
        beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fast(alpha, xnorm);
        const double sgap = alpha - beta;
        const bool big = fabs(sgap) > DMIN;
        tau_i = (beta - alpha) / beta;
        f1 = (big ? 1.0 : EPS) / sgap;  // independent of tau: both divisions in flight
        f2 = big ? 1.0 : 1.0 / EPS;
        branch = big ? 1 : 2;
      }
      const double v0out = branch ? beta : alpha;
      T2_MARK(7)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int e = lane + 64 * h;
        if (e < m) {
          double t = h ? x1 : x0;
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
        va[i + 1] = 1.0;
        tva[i + 1] = tau_i * 1.0;
        scal[0] = tau_i;
        tauOut[i] = tau_i;
        sdOut[i] = v0out;
      }
    }
    T2_MARK(0)
    __syncthreads();
    T2_MARK(1)
    const double tau_i = scal[0];
    if (tau_i == 0.0) continue;  // no update this step (uniform)
    // ---- E: dsymv chains, lockstep over columns; wave 0/1 descending for
    // rows j < 64 / j >= 64, wave 2/3 ascending (row r = i+1+j)
    if (wid < 4) {
      const int h = wid & 1, j = lane + 64 * h;
      const bool valid = j < n;
      const int r = valid ? i + 1 + j : N - 1;  // invalid lanes walk a zero row / discard
      if (wid < 2) {
        // c = N-1 down to r+1, then the diagonal term: T = n-1-jmin steps
        const double acc = lockstep_chain<-1>(tva + (N - 1), M + (size_t)r * lda + (N - 1), 1, max(0, n - 1 - 64 * h));
        if (valid) xd[j] = acc + tva[r] * dg[r];
      } else {
        // c = i+1 up to r-1: T = largest j of the wave
        const double acc =
            lockstep_chain<1>(va + (i + 1), M + (size_t)(i + 1) * lda + r, lda, 64 * h < n ? min(n, 64 * h + 64) - 1 : 0);
        if (valid) t2[j] = acc;
      }
    }
    T2_MARK(2)
    __syncthreads();
    T2_MARK(3)
    // ---- G, I, K (wave 0): x = xd + tau t2 and the xv products, the xv
    // chain, alpha = -(tau/2) xv, x += alpha v
    if (wid == 0) {
      double xr[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int j = lane + 64 * h;
        xr[h] = 0.0;
        if (j < n) {
          xr[h] = xd[j] + tau_i * t2[j];
          sv[j] = xr[h] * va[i + 1 + j];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const double alpha = -(tau_i / 2.0) * lds_chain_add(0.0, sv, n);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int j = lane + 64 * h;
        if (j < n) xa[i + 1 + j] = xr[h] + alpha * va[i + 1 + j];
      }
    }
    T2_MARK(4)
    __syncthreads();
    // ---- M: rank-2 update of the upper triangle and the diagonal; wave 0
    // updates the next pivot row (i+1) and goes straight on to its dnrm2
    const int r1 = i + 1;
    if (wid == 0) {
      const double nvr = -1.0 * va[r1], nxr = -1.0 * xa[r1];
      double *row = M + (size_t)r1 * lda;
      for (int c = r1 + 1 + lane; c < N; c += 64) row[c] += nvr * xa[c] + nxr * va[c];
      if (lane == 0) dg[r1] += nvr * xa[r1] + nxr * va[r1];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      // rows r = i+2+jr (jr < n-1) over waves 1..15; lane's columns c = r+1+lane, r+65+lane
      for (int jr = wid - 1; jr < n - 1; jr += 15) {
        const int r = r1 + 1 + jr;
        const double nvr = -1.0 * va[r], nxr = -1.0 * xa[r];
        double *row = M + (size_t)r * lda;
        for (int c = r + 1 + lane; c < N; c += 64) row[c] += nvr * xa[c] + nxr * va[c];
      }
      // diagonal entries of rows i+2.. (threads 64 .. 64+n-2)
      const int q = tid - 64;
      if (q < n - 1) {
        const int r = r1 + 1 + q;
        const double nvr = -1.0 * va[r], nxr = -1.0 * xa[r];
        dg[r] += nvr * xa[r] + nxr * va[r];
      }
    }
    T2_MARK(5)
  }
  __syncthreads();
#undef T2_MARK
  if (tr) {
    for (int k = 0; k < 6; k++) trace[8 + k] += tacc[k];
    trace[29] += tacc[6];
    trace[30] += tacc[7];
    trace[31] += tacc[8];
  }
  for (int r = tid; r < N; r += nt) {
    dOut[r] = dg[r];
    if (r == N - 2) sdOut[r] = M[(size_t)r * lda + r + 1];
  }
}

// Phase B for N > 128: the columns of Q are independent under
// householder_hm, so workgroups own UMW_COLS columns each (Q^T rows in LDS)
// and apply all reflectors without talking to each other; the next
// reflector row streams into a second LDS buffer while the current one is
// applied.
constexpr int UMW_COLS = 4;
constexpr int UMW_TPB = 256;
__host__ __device__ inline int umw_groups(int N) { return (N + UMW_COLS - 1) / UMW_COLS; }
size_t umw_lds_bytes(int N) { return (2 * (size_t)UMW_COLS * (N + 1) + 3 * (size_t)N + 16 + 32) * sizeof(double); }
// kAllH: every reflector row staged in LDS up front (packed: row i holds its
// N-i-1 entries), so no step waits on a global load; used while it fits
// (KORALI_AMD_UNPACK_ALLH=0 forces the streamed rows)
__host__ __device__ inline size_t umw_hoff(int N, int i) { return (size_t)i * (N - 1) - (size_t)i * (i - 1) / 2; }
__host__ __device__ inline size_t umw_hall_doubles(int N) { return N >= 3 ? umw_hoff(N, N - 2) : 0; }
bool umw_all_fits(int N) {
  if (const char *e = getenv("KORALI_AMD_UNPACK_ALLH"))
    if (!atoi(e)) return false;
  return N >= 3 && umw_lds_bytes(N) + umw_hall_doubles(N) * sizeof(double) <= 150 * 1024;
}

template <bool kAllH>
__global__ void __launch_bounds__(UMW_TPB) k_unpack_mw(int N, const double *__restrict__ gH,
                                                       const double *__restrict__ tau, double *gQt) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x;
  const int P = gridDim.x, g = blockIdx.x, lda = N + 1;
  double *Q = smem;                              // local k = column g + k P of Q
  double *hb = Q + (size_t)UMW_COLS * lda;       // 2 x N
  double *w = hb + 2 * (size_t)N;                // UMW_COLS
  double *ts = w + 16;                           // tau, N (kept off the per-step critical path)
  double *Pq = ts + N;                           // staged products col[r] h[r], UMW_COLS x lda
  for (int i = tid; i < N; i += nt) ts[i] = tau[i];
  for (int idx = tid; idx < UMW_COLS * lda; idx += nt) {
    const int k = idx / lda, r = idx % lda;
    Q[idx] = (r < N && r == g + k * P) ? 1.0 : 0.0;
  }
  constexpr int PF = 4;  // prefetch registers per thread (N <= 1024)
  double *Hs = Pq + (size_t)UMW_COLS * lda;
  if (kAllH) {
    // rows 0..N-3 over the (N-2) x N rectangle of gH, eight loads in flight per thread
    const int tot = (N - 2) * N;
    for (int q0 = tid; q0 < tot; q0 += nt * 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int q = q0 + u * nt, i = q / N, r = q - i * N;
        v[u] = (q < tot && r < N - i - 1) ? gH[q] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int q = q0 + u * nt, i = q / N, r = q - i * N;
        if (q < tot && r < N - i - 1) Hs[umw_hoff(N, i) + r] = v[u];
      }
    }
  } else if (N >= 3) {
    for (int r = tid; r < N - (N - 3) - 1; r += nt) hb[r] = gH[(size_t)(N - 3) * N + r];
  }
  __syncthreads();
  int buf = 0;
  for (int i = N - 3; i >= 0; i--) {
    const int n = N - i - 1;
    const double ti = ts[i];
    const double *h = kAllH ? Hs + umw_hoff(N, i) : hb + (size_t)buf * N;
    double pf[PF];
    if (!kAllH && i > 0) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        const int r = tid + u * nt;
        pf[u] = (r < n + 1) ? gH[(size_t)(i - 1) * N + r] : 0.0;
      }
    }
    if (ti != 0.0) {
      for (int k = 0; k < UMW_COLS; k++) {
        const int c = g + k * P;
        if (c <= i || c >= N) continue;  // uniform
        for (int r = 1 + tid; r < n; r += nt) Pq[(size_t)k * lda + r] = Q[(size_t)k * lda + i + 1 + r] * h[r];
      }
      __syncthreads();
      if (tid < UMW_COLS) {
        const int c = g + tid * P;
        if (c > i && c < N) w[tid] = staged_chain(Q[(size_t)tid * lda + i + 1], Pq + (size_t)tid * lda + 1, n - 1);
      }
      __syncthreads();
      for (int k = 0; k < UMW_COLS; k++) {
        const int c = g + k * P;
        if (c <= i || c >= N) continue;  // uniform
        double *col = Q + (size_t)k * lda + (i + 1);
        const double wj = w[k];
        for (int r = tid; r < n; r += nt) col[r] = (r == 0) ? col[0] - ti * wj : col[r] - ti * h[r] * wj;
      }
    }
    if (!kAllH && i > 0) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        const int r = tid + u * nt;
        if (r < n + 1) hb[(size_t)(buf ^ 1) * N + r] = pf[u];
      }
    }
    __syncthreads();
    buf ^= 1;
  }
  for (int idx = tid; idx < UMW_COLS * lda; idx += nt) {
    const int k = idx / lda, r = idx % lda, c = g + k * P;
    if (c < N) gQt[(size_t)c * lda + r] = Q[idx];
  }
}

// Phase B for N <= 128 with one WAVE per column of Q: the column lives in
// registers (lane l holds rows l and l + 64), every reflector row is staged
// in LDS once, and a step needs no workgroup barrier: the wave writes its
// products col[i+1+r] h[r] to its own LDS row, runs the ordered chain over
// them (kc_add, every lane the same wave-uniform sum) and updates its
// registers.  Same operations in the same order as k_unpack_mw (GSL
// householder_hm on the identity), so Q is bit-identical.  The chain is
// padded to whole groups of 16 with +0.0: the sum starts at a column entry,
// and every zero of Q here is +0.0 (identity entries; x - y of equal values
// rounds to +0.0), so acc + (+0.0) == acc.
constexpr int UWV_WAVES = 4, UWV_SV = 128 + 48;  // columns per workgroup; per-wave staging row
__host__ __device__ inline size_t uwv_lds_bytes(int N) {
  return (umw_hall_doubles(N) + (size_t)N + (size_t)UWV_WAVES * UWV_SV) * sizeof(double);
}
bool uwv_fits(int N) {
  if (const char *e = getenv("KORALI_AMD_UNPACK"))
    if (!strcmp(e, "mw")) return false;
  return N >= 3 && N <= 128 && uwv_lds_bytes(N) <= 150 * 1024;
}
__global__ void __launch_bounds__(64 * UWV_WAVES) k_unpack_wv(int N, const double *__restrict__ gH,
                                                             const double *__restrict__ tau, double *gQt) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, nt = blockDim.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = blockIdx.x * UWV_WAVES + wid;  // this wave's column
  double *Hs = smem;                              // reflector rows, packed (row i: N - i - 1 entries)
  double *ts = Hs + umw_hall_doubles(N);          // tau
  double *sv = ts + N + (size_t)wid * UWV_SV;     // this wave's products (index r, zero beyond)
  {
    const int tot = (N - 2) * N;
    for (int q0 = tid; q0 < tot; q0 += nt * 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int q = q0 + u * nt, i = q / N, r = q - i * N;
        v[u] = (q < tot && r < N - i - 1) ? gH[q] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int q = q0 + u * nt, i = q / N, r = q - i * N;
        if (q < tot && r < N - i - 1) Hs[umw_hoff(N, i) + r] = v[u];
      }
    }
    for (int i = tid; i < N; i += nt) ts[i] = tau[i];
    for (int q = lane; q < UWV_SV; q += 64) sv[q] = 0.0;
  }
  __syncthreads();
  if (c >= N) return;  // wave-uniform; no barrier follows
  // identity column c
  double q0 = (lane == c) ? 1.0 : 0.0, q1 = (lane + 64 == c) ? 1.0 : 0.0;
  for (int i = min(c - 1, N - 3); i >= 0; i--) {  // steps i < c touch column c
    const double ti = ts[i];
    if (ti == 0.0) continue;  // uniform
    const int n = N - i - 1;
    const double *h = Hs + umw_hoff(N, i);
    const int r0 = lane - i - 1, r1 = lane + 64 - i - 1;  // offsets of this lane's rows in the reflector
    const double h0 = (r0 >= 1 && r0 < n) ? h[r0] : 0.0, h1 = (r1 >= 1 && r1 < n) ? h[r1] : 0.0;
    if (r0 >= 1 && r0 < n) sv[r0] = q0 * h0;
    if (r1 >= 1 && r1 < n) sv[r1] = q1 * h1;
    // acc = Q[i+1][c] (wave-uniform), then the ordered sum over r = 1 .. n-1
    const int e = i + 1;
    const double qe = (e < 64) ? q0 : q1;
    const double acc = __longlong_as_double(
        ((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(qe) >> 32), e & 63) << 32) |
        (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(qe), e & 63));
    const unsigned pa = (unsigned)(size_t)(const __attribute__((address_space(3))) double *)(sv + 1);
    const double w = chains::kc_add(acc, pa, __builtin_amdgcn_readfirstlane((unsigned)(n - 1 + 15) >> 4));
    if (r0 == 0) q0 = q0 - ti * w;
    else if (r0 >= 1 && r0 < n) q0 = q0 - ti * h0 * w;
    if (r1 == 0) q1 = q1 - ti * w;
    else if (r1 >= 1 && r1 < n) q1 = q1 - ti * h1 * w;
  }
  const int lda = N + 1;
  if (lane < N) gQt[(size_t)c * lda + lane] = q0;
  if (lane + 64 <= N) gQt[(size_t)c * lda + lane + 64] = (lane + 64 < N) ? q1 : 0.0;
  if (lane == 0 && N < 64) gQt[(size_t)c * lda + N] = 0.0;
}

// ------------------------------------------------------------------------
// Phase C: the implicit-shift QR chase (eigen/symmv.c main loop + qrstep)
// on the tridiagonal d/sd.  It only produces the rotation sequence: per QR
// step a header (a, n) and n-1 Givens pairs (c, s); then the ABS_ASC
// selection sort gives eval (sorted) and the column permutation.
struct EigRec {
  int *hdr;     // 2 per step: a, n
  double *cs;   // 2 per rotation
  int *meta;    // [0] steps [1] rotations [2] overflow/error
  double *eval; // N sorted eigenvalues
  int *perm;    // N: sorted column i = unsorted column perm[i]
};

EigenSolver::Rec::operator EigRec() const { return EigRec{hdr, cs, meta, eval, perm}; }

// progress word of a streamed chase: seq (24 bits) | done (1) | QR steps (39)
__host__ __device__ inline unsigned long long chase_word(unsigned long long seq, int done, unsigned long long steps) {
  return ((seq & 0xffffffULL) << 40) | ((unsigned long long)(done ? 1 : 0) << 39) | steps;
}
__host__ __device__ inline void chase_publish(unsigned long long *prog, unsigned long long w) {
#if !defined(__HIP_DEVICE_COMPILE__)
  if (prog) {
    // host-coherent pinned memory may be write-combining on the CPU side:
    // sfence drains the step's headers / rotations before the progress word,
    // and the progress word itself right away
    __builtin_ia32_sfence();
    __atomic_store_n(prog, w, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
  }
#else
  (void)prog;
  (void)w;
#endif
}

__host__ __device__ inline int qr_chase(int N, double *d, double *sd, EigRec r, int maxRot, double *gc, double *gs,
                                        unsigned long long *prog = nullptr, unsigned long long seq = 0,
                                        int every = 1, bool fused = false) {
  chop_small(N, d, sd);
  int b = N - 1, steps = 0, rot = 0, err = 0;
  while (b > 0) {
    if (sd[b - 1] == 0.0 || sd[b - 1] != sd[b - 1]) {  // == 0 or NaN
      b--;
      continue;
    }
    int a = b - 1;
    while (a > 0) {
      if (sd[a - 1] == 0.0) break;
      a--;
    }
    const int nb = b - a + 1;
    if (rot + nb - 1 > maxRot) {
      err = 1;
      break;
    }
    if (fused) {
      qrstep_fused(nb, d + a, sd + a, r.cs + 2 * (size_t)rot);  // (rotations written in place, chop folded in)
    } else {
      qrstep(nb, d + a, sd + a, gc, gs);
      for (int k = 0; k + 1 < nb; k++) {
        r.cs[2 * (rot + k)] = gc[k];
        r.cs[2 * (rot + k) + 1] = gs[k];
      }
    }
    r.hdr[2 * steps] = a;
    r.hdr[2 * steps + 1] = nb;
    steps++;
    rot += nb - 1;
    if (steps % every == 0) chase_publish(prog, chase_word(seq, 0, (unsigned long long)steps));
    if (!fused) chop_small(nb, d + a, sd + a);
  }
  // gsl_eigen_symmv_sort(ABS_ASC): selection sort, strict < on |e|
  for (int i = 0; i < N; i++) {
    r.eval[i] = d[i];
    r.perm[i] = i;
  }
  for (int i = 0; i + 1 < N; i++) {
    int k = i;
    double ek = r.eval[i];
    for (int j = i + 1; j < N; j++)
      if (fabs(r.eval[j]) < fabs(ek)) {
        k = j;
        ek = r.eval[j];
      }
    if (k != i) {
      const double t = r.eval[i];
      r.eval[i] = r.eval[k];
      r.eval[k] = t;
      const int p = r.perm[i];
      r.perm[i] = r.perm[k];
      r.perm[k] = p;
    }
  }
  r.meta[0] = steps;
  r.meta[1] = rot;
  r.meta[2] = err;
  chase_publish(prog, chase_word(seq, 1, (unsigned long long)steps));
  return err;
}

// device variant of phase C: one lane (the chase is a strict dependency
// chain; see DESIGN.md for why the default runs it on the host core)
__global__ void __launch_bounds__(64) k_chase(int N, const double *__restrict__ dIn, const double *__restrict__ sdIn,
                                              EigRec r, int maxRot, double *work) {
  if (threadIdx.x != 0) return;
  double *d = work, *sd = work + N, *gc = work + 2 * N, *gs = work + 3 * N;
  for (int i = 0; i < N; i++) {
    d[i] = dIn[i];
    if (i + 1 < N) sd[i] = sdIn[i];
  }
  qr_chase(N, d, sd, r, maxRot, gc, gs);
}

// Phase C application + phase D write-back (CMAES::updateEigensystem).
// Row k of Q replays every Givens rotation in GSL's order:
//   (Q[k][a+i], Q[k][a+i+1]) <- (qi c - qj s, qi s + qj c)
// Rows are independent: workgroups own APPLY_ROWS rows each (their own
// LDS copy).  Along a row the rotations are a dependency chain, but QR step
// t+1 only needs the entries step t has finished: rotation i of step t+1
// touches columns a'+i, a'+i+1, final in step t after its rotation
// (a'-a)+i+1.  A team of APPLY_TEAM lanes per row therefore runs
// APPLY_TEAM consecutive steps at once in lockstep, lane s lagging lane s-1
// by 2 + (a_s - a_{s-1}) rotations -- for steps whose column range is
// nested in the previous one's (a_s >= a_{s-1}, a_s + nb_s <= a_{s-1} +
// nb_{s-1}); any other step starts a new group.  Every entry still sees the
// same operations in the same order, so the result is GSL's bit for bit.
// A team is one whole wave (64 steps in flight per row, one row per wave)
// by default; KORALI_AMD_APPLY_TEAM=16 selects the round-2 layout (16-lane
// teams, 4 rows per wave) for comparison.  Fewer, longer groups: a group of K
// nested steps costs about 2K + nb units, so 64-step groups need about half
// the units of 16-step ones at the CMA-ES shapes.
constexpr int APPLY_TPB = 256;
template <int TEAM> struct ApplyGeom {
  static constexpr int ROWS = APPLY_TPB / TEAM;
};
static int apply_team() {
  static const int t = (getenv("KORALI_AMD_APPLY_TEAM") && atoi(getenv("KORALI_AMD_APPLY_TEAM")) == 16) ? 16 : 64;
  return t;
}
static int apply_rows() { return APPLY_TPB / apply_team(); }
constexpr int APF = 4;  // apply: rotations prefetched ahead of the systolic replay

// x of lane l-1 within the team (16 lanes: row_shr:1 within each DPP row;
// 64 lanes: wave_shr:1); the team's lane 0 gets 0 and never uses it
template <int TEAM>
__device__ inline double dpp_shr1(double x) {
  constexpr int CTRL = TEAM == 64 ? 0x138 : 0x111;
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(v & 0xffffffffLL), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int APPLY_HCAP = 256;  // step headers per LDS chunk
constexpr int APPLY_MINSTEP = 16;  // streamed apply: smallest batch of new steps worth a chunk
// rotations per LDS chunk: up to 4096, what fits next to the rows (>= N - 1,
// one whole QR step, for every N the CMA-ES path accepts)
__host__ __device__ inline int apply_cap(int N, int rows) {
  const long long avail =
      160LL * 1024 - (long long)N * (rows + 1) * 8 - 8 * APPLY_HCAP - 16 - 8 * APPLY_TPB - 512;
  const long long c = avail / 16;
  return (int)(c > 4096 ? 4096 : c);
}
__host__ __device__ inline size_t apply_lds_bytes(int N, int rows) {
  return (size_t)N * (rows + 1) * sizeof(double) + 16 * (size_t)apply_cap(N, rows) + 8 * APPLY_HCAP + 16 +
         8 * APPLY_TPB;
}

// system-scope loads of host-coherent memory the host chase writes while
// the kernel runs (bypass every GPU cache: no stale line from an earlier
// generation can be read)
__device__ inline int ld_sys(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline double ld_sys(const double *p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((const unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
// agent-scope (sc1) loads / stores of the device staging copy (R1 hand-off)
__device__ inline int ld_agt(const int *p) {
  return __hip_atomic_load((const gu32i_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double ld_agt(const double *p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((const gu64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ inline void st_agt(int *p, int v) {
  __hip_atomic_store((gu32i_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agt(double *p, double v) {
  __hip_atomic_store((gu64_t *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// LDS fill from the device staging copy: eight agent-scope loads in flight
// per thread (each is an L2 round trip; one at a time they serialise)
template <typename T>
__device__ inline void fill_agt(T *dst, const T *src, int n, int tid) {
  for (int q = tid; q < n; q += APPLY_TPB * 8) {
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int qq = q + u * APPLY_TPB;
      v[u] = (qq < n) ? ld_agt(src + qq) : T(0);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int qq = q + u * APPLY_TPB;
      if (qq < n) dst[qq] = v[u];
    }
  }
}

// Streamed chase, fetcher workgroup: copies what the host chase publishes
// (host-coherent memory, read ONCE here) into the device staging buffers,
// then publishes a device progress word; the apply workgroups read only
// device memory.
__device__ void apply_fetcher(int N, EigRec hr, EigRec dr, unsigned long long *hprog, unsigned long long *dprog,
                              unsigned long long seq, unsigned int *errors, int *sh) {
  const int tid = threadIdx.x;
  int t0 = 0, ro0 = 0;
  for (;;) {
    if (tid == 0) {
      unsigned long long w = 0;
      int state = 0;
      for (unsigned spins = 0;; spins++) {
        w = __hip_atomic_load(hprog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((w >> 40) == (seq & 0xffffffULL) && (((w >> 39) & 1ULL) || (long long)(w & 0x7fffffffffULL) > t0)) {
          state = (int)((w >> 39) & 1ULL);
          break;
        }
        if (spins > KG_SPIN_LIMIT) {
          atomicOr(errors, KG_ERR_SYNC_TIMEOUT);
          state = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      sh[0] = (int)(w & 0x7fffffffffULL);
      sh[1] = state;
      sh[2] = 0;
    }
    __syncthreads();
    const int avail = sh[0], state = sh[1];
    if (state == 2) {
      // publish "done" with an error so the apply workgroups stop waiting
      if (tid == 0) {
        st_agt(dr.meta + 2, 1);
        __hip_atomic_store((gu64_t *)dprog, chase_word(seq, 1, (unsigned long long)t0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    // headers of the new steps and their rotation count; host reads are
    // PCIe round trips, so every thread keeps 16 of them in flight
    int rc = 0;
    for (int t = t0 + tid; t < avail; t += APPLY_TPB * 8) {
      int a[8], nb[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int tt = t + u * APPLY_TPB;
        a[u] = (tt < avail) ? ld_sys(hr.hdr + 2 * (size_t)tt) : 0;
        nb[u] = (tt < avail) ? ld_sys(hr.hdr + 2 * (size_t)tt + 1) : 1;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int tt = t + u * APPLY_TPB;
        if (tt < avail) {
          st_agt(dr.hdr + 2 * (size_t)tt, a[u]);
          st_agt(dr.hdr + 2 * (size_t)tt + 1, nb[u]);
          rc += nb[u] - 1;
        }
      }
    }
    atomicAdd(&sh[2], rc);
    __syncthreads();
    const int nrot = sh[2];
    {
      const double *src = hr.cs + 2 * (size_t)ro0;
      double *dst = dr.cs + 2 * (size_t)ro0;
      const int tot = 2 * nrot;
      for (int q = tid; q < tot; q += APPLY_TPB * 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int qq = q + u * APPLY_TPB;
          v[u] = (qq < tot) ? ld_sys(src + qq) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int qq = q + u * APPLY_TPB;
          if (qq < tot) st_agt(dst + qq, v[u]);
        }
      }
    }
    if (state == 1) {
      for (int i = tid; i < N; i += APPLY_TPB) {
        st_agt(dr.eval + i, ld_sys(hr.eval + i));
        st_agt(dr.perm + i, ld_sys(hr.perm + i));
      }
      if (tid < 3) st_agt(dr.meta + tid, ld_sys(hr.meta + tid));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains (R1)
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store((gu64_t *)dprog, chase_word(seq, state, (unsigned long long)avail), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    t0 = avail;
    ro0 += nrot;
    if (state == 1) return;
  }
}

// kStream: the Givens chase runs on the host WHILE this kernel applies its
// rotations: headers / rotations / eigenvalues are read from host-coherent
// memory, a chunk as soon as the chase has published it (progress word with
// a per-generation sequence number), so the apply trails the chase by about
// one chunk instead of starting after it.
template <bool kStream, int TEAM>
__global__ void __launch_bounds__(APPLY_TPB) k_apply(int N, const double *__restrict__ gQt, EigRec r,
                                                     double *__restrict__ B, double *__restrict__ D, double *minEig,
                                                     double *maxEig, double *eigenFailures, unsigned int *errors,
                                                     unsigned long long *trace, unsigned long long *prog,
                                                     unsigned long long seq, EigRec hr, unsigned long long *hprog) {
  unsigned long long ngroups = 0, nunits = 0, tstart = __builtin_amdgcn_s_memtime();
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lda = N + 1;
  constexpr int APPLY_ROWS = ApplyGeom<TEAM>::ROWS, APPLY_TEAM = TEAM;
  const int S = APPLY_ROWS + 1;                  // Lq[c * S + kl] = Q[k0 + kl][c]
  // kStream: workgroup 0 is the fetcher and row block rb = blockIdx - 1.  A
  // plain launch dispatches workgroups in order, so the fetcher every row
  // workgroup waits on is always already running: the grid needs no
  // co-residency, even when other processes share the device.
  const int rb = kStream ? (int)blockIdx.x - 1 : (int)blockIdx.x;
  const int k0 = rb * APPLY_ROWS;
  const int nrows = min(APPLY_ROWS, N - k0);
  double *Lq = smem;
  const int cap = apply_cap(N, APPLY_ROWS);
  double *csh = Lq + (size_t)N * S;              // cap (c, s) pairs
  int *hsh = (int *)(csh + 2 * (size_t)cap);      // APPLY_HCAP (a, nb)
  int *chunk = hsh + 2 * APPLY_HCAP;
  double *dummy = (double *)(chunk + 4) + threadIdx.x;  // stores of lanes with nothing to store
  if (kStream && blockIdx.x == 0) {  // the extra workgroup: fetcher
    apply_fetcher(N, hr, r, hprog, prog, seq, errors, chunk);
    return;
  }
  if (!kStream && r.meta[2]) {
    if (tid == 0 && rb == 0) atomicOr(errors, KG_ERR_EIGEN);
    return;
  }
  for (int idx = tid; idx < N * APPLY_ROWS; idx += APPLY_TPB) {
    const int c = idx / APPLY_ROWS, kl = idx % APPLY_ROWS;
    Lq[c * S + kl] = (kl < nrows) ? gQt[(size_t)c * lda + k0 + kl] : 0.0;
  }
  const int kl = tid / APPLY_TEAM, s = tid % APPLY_TEAM;
  const int lane = tid & 63;
  int t0 = 0, ro0 = 0;
  unsigned long long nchunks = 0, t_at_done = 0, tfirst = 0;
  __syncthreads();
  for (;;) {
    int avail;
    if (kStream) {
      if (tid == 0) {
        unsigned long long w = 0;
        int state = 0;
        for (unsigned spins = 0;; spins++) {
          w = __hip_atomic_load((gu64_t *)prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // proceed on a batch of >= APPLY_MINSTEP new steps (the systolic groups
          // need nested steps to fill a team) or when the chase is done
          if ((w >> 40) == (seq & 0xffffffULL) &&
              (((w >> 39) & 1ULL) || (long long)(w & 0x7fffffffffULL) >= t0 + APPLY_MINSTEP)) {
            state = (int)((w >> 39) & 1ULL);
            break;
          }
          if (spins > KG_SPIN_LIMIT) {
            atomicOr(errors, KG_ERR_SYNC_TIMEOUT);
            state = 2;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        chunk[2] = (int)(w & 0x7fffffffffULL);
        chunk[3] = state;
      }
      __syncthreads();
      avail = chunk[2];
      const int state = chunk[3];
      __syncthreads();
      if (state == 2) return;  // the host never published: give up (error raised)
      if (state == 1 && t_at_done == 0) t_at_done = (unsigned long long)t0 + 1;
      if (nchunks == 0) tfirst = __builtin_amdgcn_s_memtime() - tstart;
      nchunks++;
      if (avail <= t0) {
        if (state == 1) break;
        continue;
      }
    } else {
      avail = r.meta[0];
      if (t0 >= avail) break;
    }
    const int hn = min(APPLY_HCAP, avail - t0);
    if (kStream)
      fill_agt(hsh, r.hdr + 2 * (size_t)t0, 2 * hn, tid);
    else
      for (int idx = tid; idx < 2 * hn; idx += APPLY_TPB) hsh[idx] = r.hdr[2 * (size_t)t0 + idx];
    __syncthreads();
    if (tid < 64) {  // wave 0: the longest prefix of whole steps with <= cap rotations
      int base = 0, carry = 0, t1 = hn;
      for (; base < hn; base += 64) {
        const int t = base + lane;
        int v = (t < hn) ? hsh[2 * t + 1] - 1 : 0;
        for (int off = 1; off < 64; off <<= 1) {
          const int u = __shfl_up(v, off, 64);
          if (lane >= off) v += u;
        }
        const unsigned long long over = __ballot(t < hn && carry + v > cap);
        if (over) {
          t1 = base + __builtin_ctzll(over);
          carry += (t1 > base) ? __shfl(v, t1 - base - 1, 64) : 0;
          break;
        }
        carry += __shfl(v, 63, 64);
      }
      if (lane == 0) {
        chunk[0] = t1;
        chunk[1] = carry;
      }
    }
    __syncthreads();
    const int tn = chunk[0], nrot = chunk[1];
    if (kStream)
      fill_agt(csh, r.cs + 2 * (size_t)ro0, 2 * nrot, tid);
    else
      for (int idx = tid; idx < 2 * nrot; idx += APPLY_TPB) csh[idx] = r.cs[2 * (size_t)ro0 + idx];
    __syncthreads();
    double *col = Lq + kl;  // col[c * S] = Q[k0 + kl][c]
    int t = 0, ro = 0;
    while (t < tn) {
      // group of up to APPLY_TEAM nested steps (uniform across the workgroup)
      int my_a = 0, my_nb = 0, my_d = -1, my_ro = 0, T, K, ro_next;
      if constexpr (TEAM == 64) {
        // the whole wave is the team: lane s takes step t + s; the group ends
        // at the first step not nested in its predecessor.  Lags telescope,
        // d_s = 2 s + a_s - a_0, rotation offsets are a prefix sum of nb - 1.
        const int tt = t + s;
        const bool inr = tt < tn;
        const int a_s = inr ? hsh[2 * tt] : 0, nb_s = inr ? hsh[2 * tt + 1] : 1;
        const int a_p = __shfl_up(a_s, 1, 64), nb_p = __shfl_up(nb_s, 1, 64);
        const bool brk = s > 0 && (!inr || a_s < a_p || a_s + nb_s > a_p + nb_p);
        const unsigned long long bm = __ballot(brk);
        K = bm ? (int)__builtin_ctzll(bm) : 64;
        int inc = nb_s - 1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int u = __shfl_up(inc, off, 64);
          if (s >= off) inc += u;
        }
        const int a0 = __shfl(a_s, 0, 64);
        const bool mine = s < K;
        int tv = mine ? 2 * s + a_s - a0 + nb_s - 1 : 0;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) tv = max(tv, __shfl_xor(tv, off, 64));
        T = tv;
        if (mine) {
          my_a = a_s;
          my_nb = nb_s;
          my_d = 2 * s + a_s - a0;
          my_ro = ro + inc - (nb_s - 1);
        }
        ro_next = ro + __shfl(inc, K - 1, 64);
      } else {
        int pa = hsh[2 * t], pnb = hsh[2 * t + 1], pd = 0, pro = ro;
        T = pnb - 1;
        K = 1;
        if (s == 0) {
          my_a = pa;
          my_nb = pnb;
          my_d = 0;
          my_ro = pro;
        }
        while (K < APPLY_TEAM && t + K < tn) {
          const int a2 = hsh[2 * (t + K)], nb2 = hsh[2 * (t + K) + 1];
          if (a2 < pa || a2 + nb2 > pa + pnb) break;
          const int d2 = pd + 2 + (a2 - pa), ro2 = pro + pnb - 1;
          if (s == K) {
            my_a = a2;
            my_nb = nb2;
            my_d = d2;
            my_ro = ro2;
          }
          T = max(T, d2 + nb2 - 1);
          pa = a2;
          pnb = nb2;
          pd = d2;
          pro = ro2;
          K++;
        }
        ro_next = pro + pnb - 1;
      }
      // Systolic replay: lane s's qj at time tau is exactly the entry lane
      // s-1 finalised at tau-1 ("emit": its rotation output, or its carry
      // one unit after its last rotation), passed by a DPP row shift; lane 0
      // reads LDS (entries final since the previous group).  Every lane
      // also stores what it finalises, so LDS holds the group's result.
      const double *cs = csh + 2 * my_ro;
      const bool act = my_d >= 0 && kl < nrows;
      const int last = act ? my_nb - 1 : 0;  // i == last: emit the carry
      // branch-free body: every lane computes, selects keep the state, and
      // lanes with nothing to store write their own dummy slot.  The (c, s)
      // pair and the LDS entry of rotation i are loaded APF iterations ahead
      // into a register ring, so no iteration waits on an LDS round trip.
      auto clampi = [&](int i1) { return i1 < 0 ? 0 : (i1 > last - 1 ? (last > 0 ? last - 1 : 0) : i1); };
      double cR[APF], sR[APF], qR[APF];
#pragma unroll
      for (int p = 0; p < APF; p++) {
        const int icp = clampi(p - my_d);
        cR[p] = cs[2 * icp];
        sR[p] = cs[2 * icp + 1];
        qR[p] = col[(size_t)(my_a + icp + 1) * S];
      }
      double qi = col[(size_t)my_a * S], emit = 0.0;
      T += 1;  // the carry unit of the slowest lane
      // whole trips of APF units: a unit past T finds every lane past its
      // last rotation (no store, no state change), so no trip ends early and
      // the ring registers keep fixed roles (no copies, loads stay in flight)
      for (int tau0 = 0; tau0 < T; tau0 += APF) {
#pragma unroll
        for (int p = 0; p < APF; p++) {
          const int tau = tau0 + p;
          const double vin = dpp_shr1<TEAM>(emit);
          const int i = tau - my_d;
          const double c = cR[p], sn = sR[p], qjl = qR[p];
          const int icn = clampi(i + APF);
          cR[p] = cs[2 * icn];
          sR[p] = cs[2 * icn + 1];
          qR[p] = col[(size_t)(my_a + icn + 1) * S];
          qi = (s > 0 && i == -1) ? vin : qi;
          const double qj = (s == 0) ? qjl : vin;
          const double out = qi * c - qj * sn;
          const double qn = qi * sn + qj * c;
          const bool inrot = act && i >= 0 && i < last;
          const bool store = act && i >= 0 && i <= last;
          const double e = inrot ? out : qi;
          double *dst = store ? col + (size_t)(my_a + (store ? i : 0)) * S : dummy;
          *dst = e;
          emit = store ? e : emit;
          qi = inrot ? qn : qi;
        }
      }
      T -= 1;
      t += K;
      ro = ro_next;
      ngroups++;
      nunits += T;
    }
    __syncthreads();
    t0 += tn;
    ro0 += nrot;
  }
  if (trace && tid == 0 && rb == 0) {
    trace[4] += ngroups;
    trace[5] += nunits;
    trace[6] += t0;
    trace[7] += __builtin_amdgcn_s_memtime() - tstart;
    trace[26] += nchunks;
    trace[27] += t_at_done ? t_at_done - 1 : 0;  // steps applied before the chase finished
    trace[28] += tfirst;                          // ticks from kernel start to the first batch
  }
  if (kStream && ld_agt(r.meta + 2)) {  // the chase failed after streaming part of its steps
    if (tid == 0 && rb == 0) atomicOr(errors, KG_ERR_EIGEN);
    return;
  }
  // updateEigensystem: min/max eigenvalue; keep old B, D if min <= 0
  double *evs = csh;  // the rotation chunk is consumed: stage eval / perm in LDS
  int *pms = (int *)(csh + N);
  for (int i = tid; i < N; i += APPLY_TPB) {
    evs[i] = kStream ? ld_agt(r.eval + i) : r.eval[i];
    pms[i] = kStream ? ld_agt(r.perm + i) : r.perm[i];
  }
  __syncthreads();
  double mn = evs[0], mx = evs[0];
  for (int i = 1; i < N; i++) {
    mn = fmin(mn, evs[i]);
    mx = fmax(mx, evs[i]);
  }
  if (mn <= 0.0) {
    if (tid == 0 && rb == 0) *eigenFailures += 1.0;
    return;
  }
  for (int idx = tid; idx < nrows * N; idx += APPLY_TPB) {
    const int kk = idx / N, e = idx % N;
    B[(size_t)(k0 + kk) * N + e] = Lq[(size_t)pms[e] * S + kk];
  }
  if (rb == 0) {
    for (int i = tid; i < N; i += APPLY_TPB) D[i] = sqrt(evs[i]);
    if (tid == 0) {
      *minEig = mn;
      *maxEig = mx;
    }
  }
}

// diagonal covariance (CMAES::eigen diagonal branch): Q = I, eval = diag(C)
__global__ void __launch_bounds__(256) k_eigen_diag(int N, const double *__restrict__ C, double *B, double *D,
                                                    double *minEig, double *maxEig, double *eigenFailures) {
  __shared__ double mnmx[2];
  if (threadIdx.x == 0) {
    double mn = C[0], mx = C[0];
    for (int i = 1; i < N; i++) {
      const double v = C[(size_t)i * N + i];
      if (v < mn) mn = v;
      if (v > mx) mx = v;
    }
    mnmx[0] = mn;
    mnmx[1] = mx;
  }
  __syncthreads();
  if (mnmx[0] <= 0.0) {
    if (threadIdx.x == 0) *eigenFailures += 1.0;
    return;
  }
  for (int idx = threadIdx.x; idx < N * N; idx += blockDim.x) B[idx] = (idx / N == idx % N) ? 1.0 : 0.0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) D[i] = sqrt(C[(size_t)i * N + i]);
  if (threadIdx.x == 0) {
    *minEig = mnmx[0];
    *maxEig = mnmx[1];
  }
}

// The tridiagonal (d, sd) straight into host-coherent memory, then a
// sequence flag: the host chase starts as soon as it sees the flag (busy
// poll), with no DMA completion or event wake-up in between.
__global__ void __launch_bounds__(256) k_publish_dsd(int N, const double *__restrict__ dsd, double *hdsd,
                                                     unsigned long long *hflag, unsigned long long seq) {
  for (int i = threadIdx.x; i < 2 * N; i += blockDim.x)
    __hip_atomic_store((unsigned long long *)(hdsd + i), (unsigned long long)__double_as_longlong(dsd[i]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: the values before the flag
    __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// tri == 6: the covariance's lower triangle into host-coherent memory (rows
// of stride ldh, 16-byte stores of column pairs (c, c+1), c even, c <= r;
// one wave per row, rows dealt round-robin over the workgroups), then a
// sequence flag the host tridiagonalisation busy-polls.  Every thread fences
// its stores at system scope before its workgroup counts itself done; the
// last workgroup to finish (device-scope counter, reset by it for the next
// launch) publishes the flag.
constexpr int PUBC_WAVES = 4;
__global__ void __launch_bounds__(64 * PUBC_WAVES) k_publish_c(int N, const double *__restrict__ C, double *hC, int ldh,
                                                               unsigned long long *hflag, unsigned long long seq,
                                                               unsigned int *done) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = gridDim.x * PUBC_WAVES;
  for (int r = blockIdx.x * PUBC_WAVES + w; r < N; r += nw) {
    const double *src = C + (size_t)r * N;
    double *dst = hC + (size_t)r * ldh;
    for (int c = 2 * lane; c <= r; c += 128) {
      double2 v;
      v.x = src[c];
      v.y = (c + 1 < N) ? src[c + 1] : 0.0;
      *(double2 *)(dst + c) = v;
    }
  }
  __threadfence_system();  // this thread's stores before the count (system scope)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {  // every workgroup's stores are out
      __threadfence_system();
      *done = 0;
      __hip_atomic_store(hflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
inline int pubc_groups(int N) { return std::max(1, std::min(64, (N + PUBC_WAVES - 1) / PUBC_WAVES)); }

// tri == 6: waits for the host tridiagonalisation's flag, then copies the
// reflectors (row i: the N-1-i entries the unpack reads) and tau[0..N-2)
// from host-coherent memory into the device workspace (system-scope loads:
// no stale line of an earlier generation; 16 in flight per thread).
__global__ void __launch_bounds__(256) k_fetch_h(int N, const double *hH, double *gH, double *tau,
                                                 const unsigned long long *hflag, unsigned long long seq,
                                                 unsigned int *errors) {
  __shared__ int st;
  if (threadIdx.x == 0) {
    int ok = 1;
    for (unsigned spins = 0;; spins++) {
      if (__hip_atomic_load(hflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == seq) break;
      if (spins > KG_SPIN_LIMIT) {
        atomicOr(errors, KG_ERR_SYNC_TIMEOUT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    st = ok;
  }
  __syncthreads();
  if (!st) return;
  const int tot = (N - 2) * N;
  for (int q0 = threadIdx.x; q0 < tot; q0 += 256 * 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const int q = q0 + u * 256, i = q / N, r = q - i * N;
      v[u] = (q < tot && r < N - 1 - i) ? ld_sys(hH + q) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const int q = q0 + u * 256, i = q / N, r = q - i * N;
      if (q < tot && r < N - 1 - i) gH[q] = v[u];
    }
  }
  for (int i = threadIdx.x; i < N - 2; i += 256) tau[i] = ld_sys(hH + (size_t)N * N + i);
}

}  // namespace kg

#include "kg_tridiag.hip"

namespace kg {

// ------------------------------------------------------------------------
// Orchestration
size_t eig_mat_bytes(int N) { return (size_t)N * (N + 1) * sizeof(double); }
size_t tridiag_vec_bytes(int N) { return (size_t)(3 * N + 16 + (N > 64 ? N : 64) + 8) * sizeof(double); }
// one-workgroup phases (matrix in LDS) below N = 96; above, the multi-workgroup
// ones measured faster (C2, N = 128: 0.89 + 0.21 ms vs 0.95 + 0.38 ms)
bool eig_use_lds(int N) { return N < 96 && eig_mat_bytes(N) + tridiag_vec_bytes(N) + 256 <= 160 * 1024; }

int EigenSolver::init(int N_, bool hostChase_) {
  N = N_;
  hostChase = hostChase_;
  maxRot = 8 * N * N + 65536;  // GSL's implicit QR needs ~1.1 N^2 rotations
  const size_t mat = (size_t)N * (N + 1);
  KG_HIP(dev_alloc(&gA, mat * sizeof(double)));
  KG_HIP(dev_alloc(&gH, (size_t)N * N * sizeof(double)));
  KG_HIP(dev_alloc(&gQt, mat * sizeof(double)));
  KG_HIP(dev_alloc(&gWork, mat * sizeof(double)));
  KG_HIP(dev_alloc(&tau, (size_t)N * sizeof(double)));
  KG_HIP(dev_alloc(&dsd, 2 * (size_t)N * sizeof(double)));
  KG_HIP(dev_alloc(&chaseWork, 4 * (size_t)N * sizeof(double)));
  KG_HIP(dev_alloc(&dev.hdr, 2 * (size_t)(maxRot + N) * sizeof(int)));
  KG_HIP(dev_alloc(&dev.cs, 2 * (size_t)maxRot * sizeof(double)));
  KG_HIP(dev_alloc(&dev.meta, 4 * sizeof(int)));
  KG_HIP(dev_alloc(&dev.eval, (size_t)N * sizeof(double)));
  KG_HIP(dev_alloc(&dev.perm, (size_t)N * sizeof(int)));
  if (zero_fill(dev.meta, 4 * sizeof(int))) return 1;
  if (hostChase) {
    KG_HIP(host_alloc(&h_dsd, 2 * (size_t)N * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
    KG_HIP(hipHostGetDevicePointer((void **)&d_dsd_map, h_dsd, 0));
    // written by the host chase while k_apply<true> reads them: host-coherent, mapped
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    KG_HIP(host_alloc(&host.hdr, 2 * (size_t)(maxRot + N) * sizeof(int), fl));
    KG_HIP(host_alloc(&host.cs, 2 * (size_t)maxRot * sizeof(double), fl));
    KG_HIP(host_alloc(&host.meta, 4 * sizeof(int), fl));
    KG_HIP(host_alloc(&host.eval, (size_t)N * sizeof(double), fl));
    KG_HIP(host_alloc(&host.perm, (size_t)N * sizeof(int), fl));
    KG_HIP(host_alloc(&hprog, 4 * sizeof(unsigned long long), fl));
    hprog[0] = hprog[1] = hprog[2] = hprog[3] = 0;
    KG_HIP(hipHostGetDevicePointer((void **)&hmap.hdr, host.hdr, 0));
    KG_HIP(hipHostGetDevicePointer((void **)&hmap.cs, host.cs, 0));
    KG_HIP(hipHostGetDevicePointer((void **)&hmap.meta, host.meta, 0));
    KG_HIP(hipHostGetDevicePointer((void **)&hmap.eval, host.eval, 0));
    KG_HIP(hipHostGetDevicePointer((void **)&hmap.perm, host.perm, 0));
    KG_HIP(hipHostGetDevicePointer((void **)&dprog, hprog, 0));
    KG_HIP(dev_alloc(&dprogDev, 2 * sizeof(unsigned long long)));
    if (zero_fill(dprogDev, 2 * sizeof(unsigned long long))) return 1;
    KG_HIP(hipEventCreateWithFlags(&ev_dsd, hipEventDisableTiming));
    hgc.resize(N);
    hgs.resize(N);
  } else {
    KG_HIP(stream_acquire(&side));
    KG_HIP(hipEventCreateWithFlags(&ev_dsd, hipEventDisableTiming));
    KG_HIP(hipEventCreateWithFlags(&ev_chase, hipEventDisableTiming));
  }
  lds = eig_use_lds(N);
  if (const char *e = getenv("KORALI_AMD_EIGEN_MW_MIN"))  // multi-workgroup phases from this N up
    if (N >= atoi(e)) lds = false;
  // tridiagonalisation: one workgroup with the whole matrix in LDS while it
  // fits (no in-launch hand-offs), multi-workgroup above;
  // KORALI_AMD_TRIDIAG = lds | 1wg | mw forces one
  tri = sq_fits(N) ? 4 : (t2_fits(N) ? 3 : (t1_fits(N) ? 1 : (lds ? 0 : (mw2_fits(N) ? 5 : 2))));
  if (const char *e = getenv("KORALI_AMD_TRIDIAG")) {
    if (!strcmp(e, "sq") && sq_fits(N)) tri = 4;
    if (!strcmp(e, "mw2") && mw2_fits(N)) tri = 5;
    if (!strcmp(e, "lds") && eig_use_lds(N)) tri = 0;
    if (!strcmp(e, "1wg") && t1_fits(N)) tri = 1;
    if (!strcmp(e, "1wg2") && t2_fits(N)) tri = 3;
    if (!strcmp(e, "mw")) tri = 2;
  } else if (getenv("KORALI_AMD_EIGEN_MW_MIN") && !lds) {
    tri = mw2_fits(N) ? 5 : 2;
  }
  // the host core's tridiagonalisation (kg_host_tridiag.cpp) wherever the
  // chase runs there too, up to KORALI_AMD_HOST_TRIDIAG_MAX (default 512;
  // KORALI_AMD_TRIDIAG=host | a device kind forces one)
  {
    int hmax = 512;
    if (const char *e = getenv("KORALI_AMD_HOST_TRIDIAG_MAX")) hmax = atoi(e);
    const char *e = getenv("KORALI_AMD_TRIDIAG");
    if (hostChase && N >= 3 && ((e && !strcmp(e, "host")) || (!e && N <= hmax))) tri = 6;
  }
  if (tri == 6) {
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    ldc = (N + 1) & ~1;
    KG_HIP(host_alloc(&h_C, (size_t)N * ldc * sizeof(double), fl));
    KG_HIP(hipHostGetDevicePointer((void **)&d_C_map, h_C, 0));
    KG_HIP(host_alloc(&h_H, ((size_t)N * N + N) * sizeof(double), fl));
    KG_HIP(hipHostGetDevicePointer((void **)&d_H_map, h_H, 0));
    KG_CHECK(htri.init(N) == 0, "eigensolver: host tridiagonalisation workspace");
    KG_HIP(dev_alloc(&pubDone, 64));
    if (zero_fill(pubDone, 64)) return 1;
  }
  if (const char *e = getenv("KORALI_AMD_T1_FLAGS")) t1flags = atoi(e);
  sqDpp = true;  // measured round 4: 0.495 -> 0.450 ms per C2 tridiagonalisation (bench_sq0 / bench_sq1)
  if (const char *e = getenv("KORALI_AMD_SQ_DPP")) sqDpp = *e == '1';
  if (tri == 1)
    KG_HIP(allow_dynamic_lds((const void *)k_tridiag_1wg, (int)(t1_lds_doubles(N) * sizeof(double))));
  if (tri == 4)
    KG_HIP(allow_dynamic_lds((const void *)k_tridiag_sq<false>, (int)(sq_lds_doubles(N) * sizeof(double))));
  if (tri == 4)
    KG_HIP(allow_dynamic_lds((const void *)k_tridiag_sq<true>, (int)(sq_lds_doubles(N) * sizeof(double))));
  if (tri == 3)
    KG_HIP(allow_dynamic_lds((const void *)k_tridiag_1wg2, (int)(t2_lds_doubles(N) * sizeof(double))));
  if (tri == 5) {
    // the workgroups hand data to each other inside the launch: they must be
    // co-resident, which a cooperative launch guarantees (or refuses).  With
    // fewer co-resident slots than workgroups (fewer CUs visible, another
    // kernel's LDS), each workgroup takes more rows.
    int perCU = 0, dev = 0, cus = 0;
    KG_HIP(hipGetDevice(&dev));
    KG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (int rw = (N + 255) / 256; rw <= N; rw++) {
      g_mw2_rw[N] = rw;
      if (!mw2_fits(N) || mw2_rows(N) != rw) break;  // LDS exhausted (or rows forced by the environment)
      KG_HIP(allow_dynamic_lds((const void *)k_tridiag_mw2<false>, (int)mw2_lds_bytes(N)));
      KG_HIP(allow_dynamic_lds((const void *)k_tridiag_mw2<true>, (int)mw2_lds_bytes(N)));
      KG_HIP(resident_per_cu(sqDpp ? (const void *)k_tridiag_mw2<true> : (const void *)k_tridiag_mw2<false>, MW2_TPB,
                             mw2_lds_bytes(N), &perCU, nullptr));
      if (getenv("KORALI_AMD_DEBUG_OCC"))
        fprintf(stderr, "[korali_amd] mw2 N=%d rows=%d groups=%d lds=%zu perCU=%d cus=%d\n", N, rw, mw2_groups(N),
                mw2_lds_bytes(N), perCU, cus);
      if (perCU * cus >= mw2_groups(N)) break;
    }
    KG_CHECK(mw2_fits(N) && perCU * cus >= mw2_groups(N),
             "eigensolver: the multi-workgroup tridiagonalisation's " + std::to_string(mw2_groups(N)) +
                 " workgroups cannot be co-resident (" + std::to_string(cus) + " CUs x " + std::to_string(perCU) +
                 " per CU)");
  }
  if (!lds || tri == 2 || tri == 5) {
    KG_HIP(dev_alloc(&comm, tmw_comm_words(N) * sizeof(unsigned long long)));
    KG_HIP(allow_dynamic_lds((const void *)k_tridiag_mw, (int)tmw_lds_bytes(N)));
    if (uwv_fits(N))
      KG_HIP(allow_dynamic_lds((const void *)k_unpack_wv, (int)uwv_lds_bytes(N)));
    if (umw_all_fits(N))
      KG_HIP(allow_dynamic_lds((const void *)k_unpack_mw<true>, (int)(umw_lds_bytes(N) + umw_hall_doubles(N) * sizeof(double))));
    else
      KG_HIP(allow_dynamic_lds((const void *)k_unpack_mw<false>, (int)umw_lds_bytes(N)));
  }
  const int attr = 160 * 1024;
  KG_HIP(allow_dynamic_lds((const void *)k_tridiag<true>, attr));
  KG_HIP(allow_dynamic_lds((const void *)k_unpack<true>, attr));
  KG_HIP(allow_dynamic_lds((const void *)k_apply<false, 64>, (int)apply_lds_bytes(N, 4)));
  KG_HIP(allow_dynamic_lds((const void *)k_apply<true, 64>, (int)apply_lds_bytes(N, 4)));
  KG_HIP(allow_dynamic_lds((const void *)k_apply<false, 16>, (int)apply_lds_bytes(N, 16)));
  KG_HIP(allow_dynamic_lds((const void *)k_apply<true, 16>, (int)apply_lds_bytes(N, 16)));
  return 0;
}

void EigenSolver::drain() {
  if (side) (void)hipStreamSynchronize(side);
}

EigenSolver::~EigenSolver() {
  drain();
  for (void *p : {(void *)gA, (void *)gH, (void *)gQt, (void *)gWork, (void *)tau, (void *)dsd, (void *)chaseWork,
                  (void *)dev.hdr, (void *)dev.cs, (void *)dev.meta, (void *)dev.eval, (void *)dev.perm, (void *)comm,
                  (void *)dprogDev, (void *)pubDone})
    if (p) dev_release(p);
  for (void *p : {(void *)h_dsd, (void *)host.hdr, (void *)host.cs, (void *)host.meta, (void *)host.eval,
                  (void *)host.perm, (void *)hprog, (void *)h_C, (void *)h_H})
    if (p) host_release(p);
  if (side) stream_release(side);
  if (ev_dsd) (void)hipEventDestroy(ev_dsd);
  if (ev_chase) (void)hipEventDestroy(ev_chase);
}

// Phase A and B (+ the tridiagonal's hand-off to the chase): they touch only
// the solver's workspace, so a caller may enqueue them ahead of time (the
// next generation's, before its termination check) and complete the
// decomposition with run_finish.
int EigenSolver::run_begin(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
                           double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof, void *profCtx) {
  if (begun) return 0;  // (already issued for this C: kg_cmaes_update publishes it ahead of k_sigma)
  begun = true;
  if (diagonal) return 0;  // k_eigen_diag runs in run_finish
  if (tri == 6) {  // C to the host core; the rest waits for it in run_finish
    cSeq = ++pubSeq;  // (a new value per publication: a re-published C is never mistaken for the last one)
    if (prof) prof(profCtx, "eigen_publish_c", 0);
    hipLaunchKernelGGL(k_publish_c, dim3(pubc_groups(N)), dim3(64 * PUBC_WAVES), 0, s, N, C, d_C_map, ldc, dprog + 2,
                       cSeq, pubDone);
    KG_HIP(hipGetLastError());
    if (prof) prof(profCtx, "eigen_publish_c", 1);
    return 0;
  }
  const size_t matb = lds ? eig_mat_bytes(N) : 0;
  double *d = dsd, *sd = dsd + N;
  if (prof) prof(profCtx, "eigen_tridiag", 0);
  const bool fusedPublish = hostChase && tri == 4;  // the one-workgroup kernel publishes d | sd itself
  if (fusedPublish) dsdSeq = ++pubSeq;  // (unique per publication, as cSeq)
  if (tri == 4) {
    hipLaunchKernelGGL(sqDpp ? k_tridiag_sq<true> : k_tridiag_sq<false>, dim3(1), dim3(SQ_TPB),
                       sq_lds_doubles(N) * sizeof(double), s, N, C, gH, tau, d, sd, trace,
                       fusedPublish ? d_dsd_map : (double *)nullptr,
                       fusedPublish ? dprog + 1 : (unsigned long long *)nullptr, (unsigned long long)dsdSeq);
  }
  else if (tri == 3)
    hipLaunchKernelGGL(k_tridiag_1wg2, dim3(1), dim3(T2_TPB), t2_lds_doubles(N) * sizeof(double), s, N, C, gH, tau,
                       d, sd, trace);
  else if (tri == 1)
    hipLaunchKernelGGL(k_tridiag_1wg, dim3(1), dim3(T1_TPB), t1_lds_doubles(N) * sizeof(double), s, N, C, gH, tau, d,
                       sd, trace, t1flags);
  else if (tri == 0)
    hipLaunchKernelGGL(k_tridiag<true>, dim3(1), dim3(1024), eig_mat_bytes(N) + tridiag_vec_bytes(N), s, N, C, gA, gH,
                       tau, d, sd, trace);
  else if (tri == 5) {
    KG_HIP(hipMemsetAsync(comm, 0, tmw_comm_words(N) * sizeof(unsigned long long), s));
    int N_ = N;
    const double *C_ = C;
    double *gH_ = gH, *tau_ = tau, *d_ = d, *sd_ = sd;
    unsigned long long *comm_ = comm, *trace_ = trace;
    unsigned int *errors_ = errors;
    void *args[] = {&N_, &C_, &gH_, &tau_, &d_, &sd_, &comm_, &errors_, &trace_};
    KG_HIP(launch_resident(sqDpp ? (const void *)k_tridiag_mw2<true> : (const void *)k_tridiag_mw2<false>,
                           dim3(mw2_groups(N)), dim3(MW2_TPB), args, mw2_lds_bytes(N),
                           s));
  } else {
    KG_HIP(hipMemsetAsync(comm, 0, tmw_comm_words(N) * sizeof(unsigned long long), s));
    int N_ = N;
    const double *C_ = C;
    double *gH_ = gH, *tau_ = tau, *d_ = d, *sd_ = sd;
    unsigned long long *comm_ = comm, *trace_ = trace;
    unsigned int *errors_ = errors;
    void *args[] = {&N_, &C_, &gH_, &tau_, &d_, &sd_, &comm_, &errors_, &trace_};
    KG_HIP(launch_resident((const void *)k_tridiag_mw, dim3(tmw_groups(N)), dim3(TMW_TPB), args, tmw_lds_bytes(N), s));
  }
  KG_HIP(hipGetLastError());
  if (prof) prof(profCtx, "eigen_tridiag", 1);
  EigRec devRec = dev;
  if (hostChase) {
    if (!fusedPublish) {
      dsdSeq = ++pubSeq;
      hipLaunchKernelGGL(k_publish_dsd, dim3(1), dim3(256), 0, s, N, (const double *)dsd, d_dsd_map, dprog + 1,
                         dsdSeq);
      KG_HIP(hipGetLastError());
    }
  } else {
    KG_HIP(hipEventRecord(ev_dsd, s));
    KG_HIP(hipStreamWaitEvent(side, ev_dsd, 0));
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, side, N, d, sd, devRec, maxRot, chaseWork);
    KG_HIP(hipGetLastError());
    KG_HIP(hipEventRecord(ev_chase, side));
  }
  return launch_unpack(s, prof, profCtx);
}

// Phase B: Q from the reflectors in gH / tau (symmtd_unpack)
int EigenSolver::launch_unpack(hipStream_t s, ProfileFn prof, void *profCtx) {
  const size_t matb = lds ? eig_mat_bytes(N) : 0;
  if (prof) prof(profCtx, "eigen_unpack", 0);
  if (lds)
    hipLaunchKernelGGL(k_unpack<true>, dim3(1), dim3(1024), matb + 2 * N * sizeof(double), s, N, gH, tau, gQt);
  else if (uwv_fits(N))
    hipLaunchKernelGGL(k_unpack_wv, dim3((N + UWV_WAVES - 1) / UWV_WAVES), dim3(64 * UWV_WAVES), uwv_lds_bytes(N), s,
                       N, gH, tau, gQt);
  else if (umw_all_fits(N))
    hipLaunchKernelGGL(k_unpack_mw<true>, dim3(umw_groups(N)), dim3(UMW_TPB),
                       umw_lds_bytes(N) + umw_hall_doubles(N) * sizeof(double), s, N, gH, tau, gQt);
  else
    hipLaunchKernelGGL(k_unpack_mw<false>, dim3(umw_groups(N)), dim3(UMW_TPB), umw_lds_bytes(N), s, N, gH, tau,
                       gQt);
  KG_HIP(hipGetLastError());
  if (prof) prof(profCtx, "eigen_unpack", 1);
  return 0;
}

// Phases C and D: the Givens chase and the rotations' application (and the
// whole diagonal-covariance case)
int EigenSolver::run_finish(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
                            double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof,
                            void *profCtx) {
  begun = false;
  if (diagonal) {
    hipLaunchKernelGGL(k_eigen_diag, dim3(1), dim3(256), 0, s, N, C, B, D, minEig, maxEig, eigenFailures);
    KG_HIP(hipGetLastError());
    return 0;
  }
  EigRec devRec = dev;
  if (hostChase) {
    // the apply kernel is queued behind the unpack and consumes the Givens
    // rotations as this core's serial chase publishes them
    const unsigned long long seq = ++chaseSeq;
    if (tri == 6) {
      // the reflectors' copy and the unpack are queued now and start the
      // moment the host core publishes them
      if (prof) prof(profCtx, "eigen_fetch_h", 0);
      hipLaunchKernelGGL(k_fetch_h, dim3(1), dim3(256), 0, s, N, (const double *)d_H_map, gH, tau,
                         (const unsigned long long *)(dprog + 3), seq, errors);
      KG_HIP(hipGetLastError());
      if (prof) prof(profCtx, "eigen_fetch_h", 1);
      if (launch_unpack(s, prof, profCtx)) return 1;
    }
    if (prof) prof(profCtx, "eigen_apply", 0);
    EigRec mr = hmap;
    // the fetcher workgroup (0) + one workgroup per 4 rows (16 with 16-lane
    // teams); the row workgroups spin only on the fetcher's progress word,
    // and the fetcher is dispatched first, so a plain launch on this stream
    // is safe (launch_resident still checks the grid fits the device)
    {
      int N_ = N;
      const double *gQt_ = gQt;
      double *B_ = B, *D_ = D, *minEig_ = minEig, *maxEig_ = maxEig, *eigenFailures_ = eigenFailures;
      unsigned int *errors_ = errors;
      unsigned long long *trace_ = trace, *dprogDev_ = dprogDev, *dprog_ = dprog;
      unsigned long long seq_ = seq;
      void *args[] = {&N_, &gQt_, &devRec, &B_, &D_, &minEig_, &maxEig_, &eigenFailures_, &errors_, &trace_,
                      &dprogDev_, &seq_, &mr, &dprog_};
      const int rows = apply_rows();
      KG_HIP(launch_resident(rows == 4 ? (const void *)k_apply<true, 64> : (const void *)k_apply<true, 16>,
                             dim3((N + rows - 1) / rows + 1), dim3(APPLY_TPB), args, apply_lds_bytes(N, rows), s,
                             /*prefer_plain=*/true));
    }
    if (tri == 6) {
      if (prof) prof(profCtx, "eigen_c_wait", 2);
      htri.wake();  // (the helper threads of a multi-threaded pass spin from here on)
      const auto t0 = std::chrono::steady_clock::now();
      while (__atomic_load_n(hprog + 2, __ATOMIC_ACQUIRE) != cSeq) {  // busy-wait for C (µs)
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
          KG_HIP(hipStreamSynchronize(s));
          KG_CHECK(false, "eigensolver: the covariance never arrived on the host");
        }
      }
      if (prof) prof(profCtx, "eigen_c_wait", 3);
      if (prof) prof(profCtx, "eigen_tridiag_host", 2);
      const auto t1 = std::chrono::steady_clock::now();
      htri.run(h_C, ldc, h_H, h_H + (size_t)N * N, h_dsd, h_dsd + N);
      last_host_tridiag_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
      __builtin_ia32_sfence();
      __atomic_store_n(hprog + 3, seq, __ATOMIC_RELEASE);  // the device copies H / tau and unpacks
      __builtin_ia32_sfence();
      if (prof) prof(profCtx, "eigen_tridiag_host", 3);
    } else {
    if (prof) prof(profCtx, "eigen_dsd_wait", 2);
    {  // busy-wait for the tridiagonal (µs, not an interrupt wake-up)
      const auto t0 = std::chrono::steady_clock::now();
      while (__atomic_load_n(hprog + 1, __ATOMIC_ACQUIRE) != dsdSeq) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
          KG_HIP(hipStreamSynchronize(s));  // surfaces a device fault, if any
          KG_CHECK(false, "eigensolver: tridiagonal never arrived on the host");
        }
      }
    }
    if (prof) prof(profCtx, "eigen_dsd_wait", 3);
    }
    if (prof) prof(profCtx, "eigen_chase_host", 2);
    EigRec hr = host;
    chase_publish(hprog, chase_word(seq, 0, 0));
    // the progress word every `every` QR steps (KORALI_AMD_CHASE_PUBLISH_EVERY;
    // each write after a device poll of its line costs the core a miss)
    static const int every = [] {
      const char *e = getenv("KORALI_AMD_CHASE_PUBLISH_EVERY");
      const int v = e ? atoi(e) : 1;
      return v < 1 ? 1 : v;
    }();
    static const bool fused = [] {  // KORALI_AMD_CHASE_FUSED=0: the separate chop pass and rotation copy
      const char *e = getenv("KORALI_AMD_CHASE_FUSED");
      return !(e && *e == '0');
    }();
    qr_chase(N, h_dsd, h_dsd + N, hr, maxRot, hgc.data(), hgs.data(), hprog, seq, every, fused);
    if (prof) prof(profCtx, "eigen_chase_host", 3);
  } else {
    KG_HIP(hipStreamWaitEvent(s, ev_chase, 0));
    if (prof) prof(profCtx, "eigen_apply", 0);
    const int rows = apply_rows();
    if (rows == 4)
      hipLaunchKernelGGL((k_apply<false, 64>), dim3((N + rows - 1) / rows), dim3(APPLY_TPB), apply_lds_bytes(N, rows),
                         s, N, gQt, devRec, B, D, minEig, maxEig, eigenFailures, errors, trace,
                         (unsigned long long *)nullptr, 0ULL, devRec, (unsigned long long *)nullptr);
    else
      hipLaunchKernelGGL((k_apply<false, 16>), dim3((N + rows - 1) / rows), dim3(APPLY_TPB), apply_lds_bytes(N, rows),
                         s, N, gQt, devRec, B, D, minEig, maxEig, eigenFailures, errors, trace,
                         (unsigned long long *)nullptr, 0ULL, devRec, (unsigned long long *)nullptr);
    KG_HIP(hipGetLastError());
  }
  if (prof) prof(profCtx, "eigen_apply", 1);
  return 0;
}

int EigenSolver::run(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
                     double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof, void *profCtx) {
  if (!begun && run_begin(C, diagonal, B, D, minEig, maxEig, eigenFailures, errors, s, prof, profCtx)) return 1;
  return run_finish(C, diagonal, B, D, minEig, maxEig, eigenFailures, errors, s, prof, profCtx);
}

}  // namespace kg

extern "C" int kg_debug_host_tridiag(size_t N, const double *C, double *H, double *tau, double *d, double *sd) {
  if (!C || !H || !tau || !d || !sd || N == 0 || N > 65536) {
    kg::set_error("kg_debug_host_tridiag: null argument or bad order");
    return 1;
  }
  kg::HostTridiag t;
  if (t.init((int)N)) {
    kg::set_error("kg_debug_host_tridiag: out of memory");
    return 1;
  }
  t.run(C, (int)N, H, tau, d, sd);
  return 0;
}

// The host core's Givens chase (phase C, the product's qr_chase) on a given
// tridiagonal, `reps` times: the sorted eigenvalues and permutation, the
// QR-step and rotation counts, the first cs_cap rotation values and the mean
// wall time per chase.  fused: the sweep with the chop test and the rotation
// record folded in (qrstep_fused), else qrstep + copy + chop_small.  CPU only.
extern "C" int kg_debug_host_chase(size_t N, const double *d, const double *sd, int fused, size_t reps, double *eval,
                                   int *perm, double *cs, size_t cs_cap, int *counts, double *ns_per_chase) {
  if (!d || !sd || !eval || !perm || !counts || N < 1 || N > 65536 || reps < 1) {
    kg::set_error("kg_debug_host_chase: null argument or bad order");
    return 1;
  }
  const int n = (int)N, maxRot = 8 * n * n + 65536;
  std::vector<int> hdr(2 * (size_t)(maxRot + n)), meta(4);
  std::vector<double> csv(2 * (size_t)maxRot), wd(N), wsd(N), gc(N), gs(N);
  kg::EigRec r{hdr.data(), csv.data(), meta.data(), eval, perm};
  double tot = 0.0;
  for (size_t k = 0; k < reps; k++) {
    std::copy(d, d + N, wd.begin());
    std::copy(sd, sd + N - 1, wsd.begin());
    const auto t0 = std::chrono::steady_clock::now();
    kg::qr_chase(n, wd.data(), wsd.data(), r, maxRot, gc.data(), gs.data(), nullptr, 0, 1, fused != 0);
    tot += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
  }
  counts[0] = meta[0], counts[1] = meta[1], counts[2] = meta[2];
  if (cs) std::copy(csv.begin(), csv.begin() + std::min<size_t>(cs_cap, 2 * (size_t)meta[1]), cs);
  if (ns_per_chase) *ns_per_chase = tot / (double)reps;
  return 0;
}
