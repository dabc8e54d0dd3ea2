// ubench_nrm2.hip — cost of dnrm2_wave (kg_eigen.hip) pieces in isolation
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__device__ __attribute__((unused)) inline double readlane_d(double x, int l) {
  const long long v = __double_as_longlong(x);
  int lo = (int)(v & 0xffffffffLL), hi = (int)(v >> 32);
  lo = __builtin_amdgcn_readlane(lo, l);
  hi = __builtin_amdgcn_readlane(hi, l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
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
template <int MODE> __device__ double dnrm2_wave_t(const double *x, int stride, int m, double *sv, unsigned long long *msk) {
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
  if (MODE == 1) return carry;
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

template <int MODE>
__global__ void __launch_bounds__(64) k(const double *in, double *out, unsigned long long *ticks, int m, int reps) {
  extern __shared__ double sm[];
  double *x = sm, *sv = sm + 1024;
  unsigned long long *msk = (unsigned long long *)(sm + 2048 + 64);
  for (int i = threadIdx.x; i < 1024; i += 64) x[i] = in[i];
  __syncthreads();
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) acc += dnrm2_wave_t<MODE>(x + (r & 1), 1, m, sv, msk);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) ticks[MODE] = t1 - t0;
}
int main() {
  double *in, *out; unsigned long long *t, h[4];
  hipMalloc(&in, 1024 * 8); hipMalloc(&out, 64 * 8); hipMalloc(&t, 32);
  double hin[1024];
  for (int i = 0; i < 1024; i++) hin[i] = std::sin(i * 12.9898) * 43758.5453 - std::floor(std::sin(i * 12.9898) * 43758.5453) - 0.5;
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  const int m = 254, reps = 50;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 3000 * 8, 0, in, out, t, m, reps);
    hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 3000 * 8, 0, in, out, t, m, reps);
    hipDeviceSynchronize();
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    if (rep) printf("dnrm2 m=%d: full %.0f ticks, staging only %.0f ticks, serial %.1f ticks/elem\n", m,
                    (double)h[0] / reps, (double)h[1] / reps, (double)(h[0] - h[1]) / reps / m);
  }
  return 0;
}
