// ubench_dsymv.hip — cost per element of the one-workgroup tridiagonalisation's
// dsymv chains (kg_eigen.hip inline_chain) in isolation: 1024-thread block,
// matrix rows in LDS with lda = N+1, W waves running one chain per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

__device__ __forceinline__ double keep_if(double x, bool keep) {
  return __longlong_as_double(__double_as_longlong(x) & -(long long)keep);
}
// MODE 0: products a[-k]*b[-k] from LDS (a uniform, b per lane)
// MODE 1: a from a register constant (no second LDS read)
// MODE 2: staged: b only (products precomputed)
template <int MODE>
__device__ __forceinline__ double chain(const double *a, const double *b, int cnt) {
  double acc = 0.0, p[8], q[8];
  const double ca = 1.0000001;
#pragma unroll
  for (int u = 0; u < 8; u++) p[u] = MODE == 0 ? a[-u] * b[-u] : MODE == 1 ? ca * b[-u] : b[-u];
  for (int k0 = 8; k0 + 16 <= cnt; k0 += 16) {
    const double *ak = a - k0, *bk = b - k0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      q[u] = MODE == 0 ? ak[-u] * bk[-u] : MODE == 1 ? ca * bk[-u] : bk[-u];
      acc += p[u];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      p[u] = MODE == 0 ? ak[-(8 + u)] * bk[-(8 + u)] : MODE == 1 ? ca * bk[-(8 + u)] : bk[-(8 + u)];
      acc += q[u];
    }
  }
#pragma unroll
  for (int u = 0; u < 8; u++) acc += p[u];
  return acc;
}

template <int MODE>
__global__ void __launch_bounds__(1024) k(const double *in, double *out, unsigned long long *ticks, int N, int W,
                                          int reps) {
  extern __shared__ double M[];
  const int lda = N + 1, tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  for (int i = tid; i < N * lda + 2 * N; i += blockDim.x) M[i] = in[i % 4096];
  __syncthreads();
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    if (wid < W) {
      const int row = (lane + 64 * wid) % N;
      acc += chain<MODE>(M + N * lda + N - 1, M + (size_t)row * lda + N - 1, N - 1);
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[tid] = acc;
  if (tid == 0) ticks[0] = t1 - t0;
}

int main() {
  double *in, *out;
  unsigned long long *t, h;
  hipMalloc(&in, 4096 * 8);
  hipMalloc(&out, 1024 * 8);
  hipMalloc(&t, 8);
  double hin[4096];
  for (int i = 0; i < 4096; i++) hin[i] = 1e-3 * ((i * 37) % 101 - 50);
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  const int N = 128, reps = 50;
  const size_t lds = (size_t)(N * (N + 1) + 2 * N) * 8;
  hipFuncSetAttribute((const void *)k<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipFuncSetAttribute((const void *)k<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipFuncSetAttribute((const void *)k<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int W : {1, 2, 4}) {
    for (int mode = 0; mode < 3; mode++) {
      for (int rep = 0; rep < 2; rep++) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(1024), lds, 0, in, out, t, N, W, reps);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(1024), lds, 0, in, out, t, N, W, reps);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(1024), lds, 0, in, out, t, N, W, reps);
        hipDeviceSynchronize();
      }
      hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      printf("waves %d mode %d (%s): %.1f ticks per element\n", W, mode,
             mode == 0 ? "two LDS operands" : mode == 1 ? "one LDS operand x const" : "staged",
             (double)h / reps / (N - 1));
    }
  }
  return 0;
}
