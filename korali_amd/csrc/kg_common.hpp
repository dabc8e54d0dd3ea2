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

#include <map>
#include <mutex>

#include <algorithm>
#include <cstdlib>

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <tuple>

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

// Device blocks and streams of the solver handles come from a process-wide
// cache: an engine run creates a handle (tens of buffers, two streams) and
// releases it at the end, and hipMalloc / hipFree / hipStreamCreate cost a few
// milliseconds per handle -- the fixed cost of a run, against ~1 ms
// generations (engine fixed cost).
//   dev_alloc    a block of >= bytes on the current device (cached blocks of
//                the same rounded size first; on out-of-memory the cache is
//                emptied and the allocation retried);
//   dev_release  back to the cache.  The caller has drained every stream
//                that used the block (the handles' destroy synchronises its
//                streams first); a mid-life reallocation passes its stream.
//   stream_acquire / stream_release  non-blocking streams, pooled per device.
// KORALI_AMD_DEVICE_CACHE_MB bounds the idle bytes kept (default 8192; 0
// turns the cache off: every release is a hipFree).
//   host_alloc / host_release  the same for pinned host blocks (hipHostMalloc
//                flags are part of the key); a reused block is zeroed, as a
//                fresh one is.
hipError_t dev_alloc(void **p, size_t bytes);
template <class T>
inline hipError_t dev_alloc(T **p, size_t bytes) {
  return dev_alloc((void **)p, bytes);
}
void dev_release(void *p, hipStream_t drain = nullptr);
hipError_t host_alloc(void **p, size_t bytes, unsigned flags);
template <class T>
inline hipError_t host_alloc(T **p, size_t bytes, unsigned flags) {
  return host_alloc((void **)p, bytes, flags);
}
void host_release(void *p);
hipError_t stream_acquire(hipStream_t *s);
void stream_release(hipStream_t s);

// Zero-fill device memory and wait for it.  hipMemset runs on the null
// stream, which does not order against the non-blocking streams the handles
// launch on: a fill still queued could land after (and clobber) the first
// stream-ordered writes, so every fill completes before it returns.
inline int zero_fill(void *p, size_t bytes) {
  KG_HIP(hipMemsetAsync(p, 0, bytes, nullptr));
  KG_HIP(hipStreamSynchronize(nullptr));
  return 0;
}
// the same fill, not waited for: a handle's create issues all its fills and
// then waits once on the null stream before any stream-ordered work
inline int zero_fill_async(void *p, size_t bytes) {
  KG_HIP(hipMemsetAsync(p, 0, bytes, nullptr));
  return 0;
}

// hipFuncAttributeMaxDynamicSharedMemorySize is per kernel and process-wide,
// while handles of different sizes need different amounts: the attribute only
// ever grows here (the largest request any handle made).  Round 3 set it per
// handle, so a smaller handle created after a larger one lowered it below the
// larger one's launches, and the runtime's occupancy query then answered 0
// blocks per CU for them (the "occupancy anomaly" of the full pytest process).
inline hipError_t allow_dynamic_lds(const void *f, size_t bytes) {
  static std::mutex mtx;
  static std::map<const void *, size_t> cur;
  std::lock_guard<std::mutex> lock(mtx);
  size_t &c = cur[f];
  if (bytes <= c) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) c = bytes;
  return e;
}

// Grids whose workgroups wait on one another inside the launch (spin
// hand-offs) go through launch_resident: a cooperative launch, so HIP
// guarantees co-residency or fails the launch.  KORALI_AMD_PLAIN_LAUNCH=1
// launches them with hipLaunchKernel after the same occupancy check instead
// (A/B).  Under rocprofv3 (ROCm 7.2) a process that made a cooperative launch
// dies with SIGSEGV in its exit handlers after the tool wrote its output and
// finalized: libamdhip64's exit-time teardown calls into libhsa-runtime64
// through the profiler's already finalized interception (stack in
// profiles/r5/c4_teardown_segv.txt, KORALI_AMD_SEGV_MAPS=1); the profile
// files are complete, and plain-launch processes never reach that path.
//
// prefer_plain: a grid whose waiting workgroups depend only on a workgroup
// dispatched before them (the streamed Givens apply: every row workgroup
// waits on the fetcher, workgroup 0), launched every generation on the
// handle's stream.  ROCm runs cooperative launches on a queue of their own,
// and the hand-over to and from it cost 12-15 us on each side of the launch
// (kernel trace, round 3); a plain launch stays on the stream's queue.
//
// The capacity is the runtime's occupancy answer; the kernel's own VGPR / LDS
// arithmetic (own_blocks_per_cu) can only lower it (it ignores AGPR / SGPR
// limits, so it never allows a launch the runtime would not).
inline int own_blocks_per_cu(const void *f, int threads, size_t lds) {
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, f) != hipSuccess) return 0;
  const int wavesPerWg = (threads + 63) / 64;
  int vgpr = a.numRegs > 0 ? a.numRegs : 1;
  vgpr = (vgpr + 7) & ~7;
  const int wavesPerSimd = std::min(8, 512 / vgpr);
  const int byWaves = (4 * wavesPerSimd) / wavesPerWg;
  const size_t ldsTot = a.sharedSizeBytes + lds;
  const int byLds = ldsTot ? (int)((160 * 1024) / ldsTot) : 32;
  return std::max(0, std::min(byWaves, byLds));
}
inline hipError_t resident_per_cu(const void *f, int threads, size_t lds, int *per, int *runtimePer) {
  int rt = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&rt, f, threads, lds);
  if (e != hipSuccess) return e;
  const int own = own_blocks_per_cu(f, threads, lds);
  if (getenv("KORALI_AMD_DEBUG_OCC")) {
    hipFuncAttributes a{};
    (void)hipFuncGetAttributes(&a, f);
    fprintf(stderr, "[korali_amd occ] f=%p threads=%d dyn_lds=%zu static_lds=%zu max_dyn=%d vgpr=%d runtime=%d own=%d\n",
            f, threads, lds, (size_t)a.sharedSizeBytes, a.maxDynamicSharedSizeBytes, a.numRegs, rt, own);
  }
  *per = std::min(rt, own);
  if (runtimePer) *runtimePer = rt;
  return hipSuccess;
}

inline hipError_t launch_resident(const void *f, dim3 grid, dim3 block, void **args, size_t lds, hipStream_t s,
                                  bool prefer_plain = false) {
  static const bool plain_env = [] {
    const char *e = getenv("KORALI_AMD_PLAIN_LAUNCH");
    return e && *e && *e != '0';
  }();
  static const bool coop_env = [] {
    const char *e = getenv("KORALI_AMD_COOP_LAUNCH");  // every resident grid cooperative (A/B)
    return e && *e && *e != '0';
  }();
  const bool plain = plain_env || (prefer_plain && !coop_env);
  if (!plain) return hipLaunchCooperativeKernel(f, grid, block, args, (unsigned int)lds, s);
  // the capacity of (device, kernel, block, LDS), queried once per process:
  // these grids launch every generation, and the occupancy query costs
  // tens of microseconds
  struct Key {
    int dev;
    const void *f;
    unsigned threads;
    size_t lds;
    bool operator<(const Key &o) const {
      return std::tie(dev, f, threads, lds) < std::tie(o.dev, o.f, o.threads, o.lds);
    }
  };
  static std::mutex mu;
  static std::map<Key, long long> capacity;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const Key k{dev, f, block.x * block.y * block.z, lds};
  long long cap = -1;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = capacity.find(k);
    if (it != capacity.end()) cap = it->second;
  }
  if (cap < 0) {
    int cus = 0, per = 0;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = resident_per_cu(f, (int)k.threads, lds, &per, nullptr);
    if (e != hipSuccess) return e;
    cap = (long long)per * cus;
    std::lock_guard<std::mutex> lk(mu);
    capacity[k] = cap;
  }
  if (cap < (long long)grid.x * grid.y * grid.z) return hipErrorCooperativeLaunchTooLarge;
  return hipLaunchKernel(f, grid, block, args, lds, s);
}

// Device-side error flags (bitmask in the scalar block; read back at sync
// points and turned into KORALI_LOG_ERROR-style messages by the host).
enum : uint32_t {
  KG_ERR_NONFINITE_F = 1u << 0,     // optimization.cpp.base:32-33
  KG_ERR_RNG_UNDERRUN = 1u << 1,    // producer did not generate enough words
  KG_ERR_DRAW_GUARD = 1u << 2,      // a draw the overflow guard proved finite was not (internal)
  KG_ERR_CONSTRAINT = 1u << 7,      // CCMA-ES: no sample without constraint violations
  KG_ERR_ZERO_LIST = 1u << 3,       // > KG_MAX_ZERO_WORDS zero MT words pending
  KG_ERR_EIGEN = 1u << 4,           // QR iteration did not converge
  KG_ERR_CHOLESKY = 1u << 5,        // covariance not positive definite
  KG_ERR_SYNC_TIMEOUT = 1u << 6,    // an in-launch workgroup hand-off timed out
};

// In-launch workgroup hand-off (MI355X_MICROARCH.md, inter-workgroup
// visibility, R2 granules): a double travels as two 8-byte {tag, half}
// granules stored write-through (agent-scope relaxed atomics: sc1) and read
// back with sc1 loads until both tags match; the data is its own flag, so no
// fence is involved.  Buffers are zeroed before every launch, tags are
// phase + 1.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gu32i_t;
constexpr unsigned KG_SPIN_LIMIT = 1u << 21;  // ~seconds: a hang becomes an error

__device__ inline void put_granule_dbl(unsigned long long *p, unsigned tag, double x) {
  gu64_t *g = (gu64_t *)p;
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const unsigned long long t = (unsigned long long)tag << 32;
  __hip_atomic_store(g, t | (b & 0xffffffffULL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, t | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// All threads of the workgroup gather two granule segments in one polling
// sweep: element e < countA from baseA[2e] into dstA[e], then countB
// elements from baseB into dstB.  Returns false when the spin limit or
// another workgroup's abort ended the wait.
__device__ inline bool poll_granule_dbls(unsigned long long *baseA, int countA, double *dstA,
                                         unsigned long long *baseB, int countB, double *dstB, unsigned tag,
                                         unsigned long long *abortw, unsigned *errors) {
  const int t = threadIdx.x, nt = blockDim.x, count = countA + countB;
  for (int e0 = 0; e0 < count; e0 += nt) {
    const int e = e0 + t;
    bool done = e >= count;
    const bool inA = e < countA;
    gu64_t *g = (gu64_t *)(inA ? baseA + 2 * (size_t)e : baseB + 2 * (size_t)(e - countA));
    double *dst = inA ? dstA + e : dstB + (e - countA);
    unsigned spins = 0;
    for (;;) {
      if (!done) {
        const unsigned long long lo = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long hi = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(lo >> 32) == tag && (unsigned)(hi >> 32) == tag) {
          *dst = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffULL)));
          done = true;
        }
      }
      if (__all(done)) break;
      ++spins;
      if ((spins & 255u) == 0) {
        if (__hip_atomic_load((gu64_t *)abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
        if (spins > KG_SPIN_LIMIT) {
          __hip_atomic_store((gu64_t *)abortw, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          atomicOr(errors, KG_ERR_SYNC_TIMEOUT);
          return false;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return true;
}

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

// cos(x) correctly rounded (for |x| < 2^30): Cody-Waite reduction by a
// triple-double pi/2 with exact products, then the Taylor series of cos or
// sin of the reduced argument in double-double (15 terms, |r| <= pi/4,
// ~2^-104 relative) and one final rounding.  Branch-free in the quadrant
// so a wavefront runs one instruction stream.  The oracle evaluates the
// same sequence (oracle/refcpu.c kr_cos_cr), so Ackley objectives agree bit
// for bit.
__host__ __device__ inline double cos_cr(double x) {
  if (!(fabs(x) < 1073741824.0)) return cos(x);  // NaN / inf / huge: never produced by the objectives
  constexpr double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
  constexpr double INV_PIO2 = 0x1.45f306dc9c883p-1;
  constexpr double CH[15] = {0x1p+0, -0x1p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
                             -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37,
                             0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62,
                             -0x1.0ce396db7f853p-70, 0x1.f2cf01972f578p-80, -0x1.88e85fc6a4e5ap-89,
                             0x1.0a18a2635085dp-98};
  constexpr double CL[15] = {0.0, 0.0, 0x1.5555555555555p-59, 0x1.f49f49f49f49fp-65, 0x1.a01a01a01a01ap-76,
                             -0x1.cbbc05b4fa99ap-76, -0x1.2aec959e14c06p-83, -0x1.05d6f8a2efd1fp-92,
                             0x1.1d8656b0ee8cbp-101, -0x1.eec01221a8b0bp-107, 0x1.ea72b4afe3c2fp-120,
                             0x1.aebcdbd20331cp-124, -0x1.9ada5fcc1ab14p-135, 0x1.71c37ebd16540p-143,
                             0x1.b9e2e28e1aa54p-153};
  constexpr double SH[15] = {0x1p+0, -0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
                             0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33,
                             -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57,
                             0x1.71b8ef6dcf572p-66, -0x1.761b41316381ap-75, 0x1.3f3ccdd165fa9p-84,
                             -0x1.d1ab1c2dccea3p-94, 0x1.259f98b4358adp-103};
  constexpr double SL[15] = {0.0, -0x1.5555555555555p-57, 0x1.1111111111111p-63, -0x1.a01a01a01a01ap-73,
                             -0x1.c154f8ddc6c00p-73, 0x1.c062e06d1f209p-80, 0x1.f28e0cc748ebep-87,
                             -0x1.1d8656b0ee8cbp-97, 0x1.ac981465ddc6cp-103, -0x1.2650f61dbdcb4p-112,
                             -0x1.d043ae40c4647p-120, 0x1.3423c7d91404fp-130, -0x1.58ddadf344487p-139,
                             -0x1.054d0c78aea14p-149, 0x1.eaf8c39dd9bc5p-157};
  const double kd = floor(x * INV_PIO2 + 0.5);
  const dd t1 = dd_tp(kd, P1), t2 = dd_tp(kd, P2);
  dd r = dd_add(dd{x, 0.0}, dd{-t1.hi, -t1.lo});
  r = dd_add(r, dd{-t2.hi, -t2.lo});
  r = dd_add(r, dd{-(kd * P3), 0.0});
  const int q = (int)((long long)kd & 3);
  const bool odd = (q & 1) != 0;
  const dd z = dd_mul(r, r);
  dd p{odd ? SH[14] : CH[14], odd ? SL[14] : CL[14]};
#pragma unroll
  for (int j = 13; j >= 0; j--) p = dd_add(dd_mul(p, z), dd{odd ? SH[j] : CH[j], odd ? SL[j] : CL[j]});
  p = dd_mul(p, odd ? r : dd{1.0, 0.0});
  const double v = p.hi + p.lo;
  return (q == 1 || q == 2) ? -v : v;
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

// acc + t(0) + t(1) + ... + t(cnt-1), added strictly left to right (the
// reference's sequential order), with the next 8 terms evaluated while the
// current 8 are added: the LDS loads behind t() overlap the dependent
// 14-cycle FP64 add chain instead of preceding every group of 8.
template <class T>
__device__ __forceinline__ double ordered_sum(double acc, int cnt, T t) {
  int q = 0;
  if (cnt >= 8) {
    double cur[8];
#pragma unroll
    for (int u = 0; u < 8; u++) cur[u] = t(u);
    for (q = 8; q + 8 <= cnt; q += 8) {
      double nx[8];
#pragma unroll
      for (int u = 0; u < 8; u++) nx[u] = t(q + u);
#pragma unroll
      for (int u = 0; u < 8; u++) acc += cur[u];
#pragma unroll
      for (int u = 0; u < 8; u++) cur[u] = nx[u];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc += cur[u];
  }
  for (; q < cnt; q++) acc += t(q);
  return acc;
}

// block-id remap so that consecutive tiles land on one XCD (speed only)
__device__ inline int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

}  // namespace kg
