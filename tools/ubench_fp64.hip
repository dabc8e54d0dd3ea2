// ubench_fp64.hip — latency of dependent FP64 operations on one lane (gfx950).
// Used to size the serial QR chase of the eigensolver.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double *out, unsigned long long *cyc, double seed, int n) {
  if (threadIdx.x != 0) return;
  double x = seed, y = seed * 0.5 + 1.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = fma(x, 0.999999, 1e-9);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = y / x + 0.5;
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = sqrt(x) + 1.0;
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = x * 1.0000001 + 1e-12;
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  double c = 0.6, s = 0.8, bk = x;
  for (int i = 0; i < n; i++) {  // givens + rotation chain like qrstep
    double t = -bk / (s + 2.0);
    double s1 = 1.0 / sqrt(1 + t * t);
    c = s1 * t; s = s1;
    bk = c * (s * 1.5 + c * bk) - s * (s * bk + c * 0.7);
  }
  unsigned long long t5 = __builtin_amdgcn_s_memtime();
  out[0] = x + bk;
  cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4;
}
int main() {
  double *o; unsigned long long *c, h[5];
  hipMalloc(&o, 8); hipMalloc(&c, 40);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, 1.5, 1000);
    hipMemcpy(h, c, 40, hipMemcpyDeviceToHost);
  }
  printf("per-op cycles: fma %.1f  div+add %.1f  sqrt+add %.1f  mul+add %.1f  givens-step %.1f\n",
         h[0] / 1000.0, h[1] / 1000.0, h[2] / 1000.0, h[3] / 1000.0, h[4] / 1000.0);
  return 0;
}
