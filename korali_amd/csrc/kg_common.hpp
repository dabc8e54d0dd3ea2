// kg_common.hpp — shared device/host helpers for the korali_amd HIP path.
//
// * HIP error plumbing into the C-ABI's (int status, kg_last_error()) model.
// * Correctly-rounded double-precision log / exp on the device, evaluated in
//   double-double (~2^-100 relative) and rounded once.  The reference's
//   committed generation files were produced with a correctly-rounded libm
//   log (see oracle/refcpu.c): CR transcendentals are what make the device
//   polar normals equal the reference's bit for bit.
// * GSL mt19937 recurrence / tempering helpers.
//
// Everything here is compiled with -ffp-contract=off: the only fused
// multiply-adds are the explicit fma() calls of the exact two-product.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace kg {

// ------------------------------------------------------------------ errors
void set_error(const std::string &msg);
const char *last_error();

#define KG_HIP(call)                                                                      \
  do {                                                                                    \
    hipError_t _e = (call);                                                               \
    if (_e != hipSuccess) {                                                               \
      ::kg::set_error(std::string(#call) + ": " + hipGetErrorString(_e) + " (" __FILE__ ":" + \
                      std::to_string(__LINE__) + ")");                                    \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

#define KG_CHECK(cond, msg)       \
  do {                            \
    if (!(cond)) {                \
      ::kg::set_error(msg);       \
      return 1;                   \
    }                             \
  } while (0)

// Device-side error flags (bitmask in the scalar block; read back at sync
// points and turned into KORALI_LOG_ERROR-style messages by the host).
enum : uint32_t {
  KG_ERR_NONFINITE_F = 1u << 0,     // optimization.cpp.base:32-33
  KG_ERR_RNG_UNDERRUN = 1u << 1,    // producer did not generate enough words
  KG_ERR_RESAMPLE_RESERVE = 1u << 2,// more infeasible draws than the reserve
  KG_ERR_ZERO_LIST = 1u << 3,       // > KG_MAX_ZERO_WORDS zero MT words pending
  KG_ERR_EIGEN = 1u << 4,           // QR iteration did not converge
  KG_ERR_CHOLESKY = 1u << 5,        // covariance not positive definite
};

// ------------------------------------------------------- double-double math
struct dd {
  double hi, lo;
};

__host__ __device__ inline dd dd_qts(double a, double b) {  // |a| >= |b|
  double s = a + b;
  return {s, b - (s - a)};
}
__host__ __device__ inline dd dd_ts(double a, double b) {
  double s = a + b;
  double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd dd_tp(double a, double b) {  // exact product via fma
  double p = a * b;
  return {p, fma(a, b, -p)};
}
__host__ __device__ inline dd dd_add(dd a, dd b) {
  dd s = dd_ts(a.hi, b.hi), t = dd_ts(a.lo, b.lo);
  s.lo += t.hi;
  s = dd_qts(s.hi, s.lo);
  s.lo += t.lo;
  return dd_qts(s.hi, s.lo);
}
__host__ __device__ inline dd dd_mul(dd a, dd b) {
  dd p = dd_tp(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return dd_qts(p.hi, p.lo);
}
__host__ __device__ inline dd dd_mul_d(dd a, double b) {
  dd p = dd_tp(a.hi, b);
  p.lo += a.lo * b;
  return dd_qts(p.hi, p.lo);
}
__host__ __device__ inline dd dd_div(dd a, dd b) {
  double q1 = a.hi / b.hi;
  dd r = dd_add(a, dd_mul_d(b, -q1));
  double q2 = r.hi / b.hi;
  r = dd_add(r, dd_mul_d(b, -q2));
  double q3 = r.hi / b.hi;
  return dd_add(dd_qts(q1, q2), dd{q3, 0.0});
}

// 1/(2j+1) as double-doubles, j = 0..21 (atanh series), and 1/j, j=0..14
// (exp Taylor).  Exact to ~2^-106; filled by the host at library load.
struct dd_tables {
  double inv_odd_hi[22], inv_odd_lo[22];
  double inv_int_hi[15], inv_int_lo[15];
};
extern __constant__ dd_tables c_dd_tab;
void upload_dd_tables();  // host

constexpr double LN2_HI = 6.93147180559945286227e-01;
constexpr double LN2_LO = 2.31904681384629955842e-17;

// log(x), x finite > 0 normal, as a double-double.  The table is passed in
// so that the host (BTPE, log-evidence) evaluates the very same function.
template <class Tab>
__host__ __device__ inline dd dd_log_tab(double x, const Tab &t) {
  int k;
  double m = frexp(x, &k);  // x = m 2^k, m in [0.5, 1)
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    k -= 1;
  }
  // s = (m-1)/(m+1); m-1 exact (Sterbenz)
  dd s = dd_div(dd{m - 1.0, 0.0}, dd_ts(m, 1.0));
  dd z = dd_mul(s, s);
  dd p{t.inv_odd_hi[21], t.inv_odd_lo[21]};
#pragma unroll
  for (int j = 20; j >= 0; j--) p = dd_add(dd_mul(p, z), dd{t.inv_odd_hi[j], t.inv_odd_lo[j]});
  p = dd_mul(dd_mul_d(s, 2.0), p);
  return dd_add(dd_mul_d(dd{LN2_HI, LN2_LO}, (double)k), p);
}

__device__ inline dd dd_log(double x) { return dd_log_tab(x, c_dd_tab); }

// host twin of log_cr (same double-double evaluation, host copy of the table)
double host_log_cr(double x);

// correctly rounded log for the inputs the solvers produce (finite, > 0)
__device__ inline double log_cr(double x) {
  if (!(x > 0.0) || isinf(x)) return log(x);
  if (x == 1.0) return 0.0;
  if (x < 2.2250738585072014e-308) return log(x);  // subnormal: never produced here
  dd r = dd_log(x);
  return r.hi + r.lo;
}

__device__ inline dd dd_exp(dd a) {
  const double kd = floor(a.hi / LN2_HI + 0.5);
  dd r = dd_add(a, dd_mul_d(dd{LN2_HI, LN2_LO}, -kd));
  r = dd_mul_d(r, 1.0 / 256.0);
  dd p{1.0, 0.0};
#pragma unroll
  for (int j = 14; j >= 1; j--)
    p = dd_add(dd{1.0, 0.0}, dd_mul(dd_mul(p, r), dd{c_dd_tab.inv_int_hi[j], c_dd_tab.inv_int_lo[j]}));
#pragma unroll
  for (int j = 0; j < 8; j++) p = dd_mul(p, p);
  p.hi = ldexp(p.hi, (int)kd);
  p.lo = ldexp(p.lo, (int)kd);
  return p;
}

__device__ inline double exp_cr(double x) {
  if (isnan(x)) return x;
  if (x > 709.0 || x < -708.0) return exp(x);
  if (x == 0.0) return 1.0;
  dd r = dd_exp(dd{x, 0.0});
  return r.hi + r.lo;
}

__device__ inline double pow_cr(double x, double y) {
  if (y == 2.0) return x * x;
  if (!(x > 0.0) || isinf(x) || isinf(y) || isnan(y)) return pow(x, y);
  dd l = dd_mul_d(dd_log(x), y);
  if (l.hi > 709.0 || l.hi < -708.0) return pow(x, y);
  l = dd_exp(l);
  return l.hi + l.lo;
}

// ---------------------------------------------------------------- mt19937
constexpr int MT_N = 624;
constexpr int MT_M = 397;
__host__ __device__ inline uint32_t mt_temper(uint32_t k) {
  k ^= (k >> 11);
  k ^= (k << 7) & 0x9d2c5680u;
  k ^= (k << 15) & 0xefc60000u;
  k ^= (k >> 18);
  return k;
}
// s_j from s_{j-624}, s_{j-623}, s_{j-227}
__host__ __device__ inline uint32_t mt_next(uint32_t a624, uint32_t a623, uint32_t a227) {
  uint32_t y = (a624 & 0x80000000u) | (a623 & 0x7fffffffu);
  return a227 ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// block-id remap so that consecutive tiles land on one XCD (speed only)
__device__ inline int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

}  // namespace kg
