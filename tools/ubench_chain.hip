// ubench_chain.hip — wall-clock cost of a dependent FP64 add chain on one
// lane vs one wave vs many waves, and the s_memtime tick rate (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_chain(double *out, const double *in, int n, unsigned long long *ticks) {
  double acc = 0.0;
  const double *p = in + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 8) {
    double t[8];
#pragma unroll
    for (int q = 0; q < 8; q++) t[q] = p[((i + q) & 1023) * 64];
#pragma unroll
    for (int q = 0; q < 8; q++) acc += t[q];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) ticks[0] = t1 - t0;
}
__global__ void k_regchain(double *out, double seed, int n, unsigned long long *ticks) {
  double acc = seed, a = seed * 1e-3, b = seed * 2e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) { acc += a; acc += b; acc += a; acc += b; }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) ticks[0] = t1 - t0;
}
int main() {
  double *o, *in; unsigned long long *t, h;
  hipMalloc(&o, 1 << 20); hipMalloc(&in, 64 * 1024 * 8); hipMalloc(&t, 8);
  hipMemset(in, 0, 64 * 1024 * 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 3; rep++) {
    const int n = 1 << 20;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_regchain, dim3(1), dim3(64), 0, 0, o, 1.5, n / 4, t);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("register add chain: %.3f ns/add, %.2f ticks/add, tick rate %.1f MHz\n", ms * 1e6 / n, (double)h / n,
           (double)h / (ms * 1e-3) / 1e6);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, o, in, 8192, t);
    hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("L2-resident load+add chain (1 wave, 8192): %.1f us kernel, %.3f ns/add\n", ms * 1e3, ms * 1e6 / 8192);
  }
  return 0;
}
