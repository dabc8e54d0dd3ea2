#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(512) k(unsigned *ids, unsigned long long *ticks) {
  unsigned hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if ((threadIdx.x & 63) == 0) ids[threadIdx.x >> 6] = hw;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1000; i++) __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) ticks[0] = t1 - t0;
  // one ds_write then ds_read by the same wave, round trip
  __shared__ double s[64];
  double v = threadIdx.x;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1000; i++) {
    s[threadIdx.x & 63] = v;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    v = s[(threadIdx.x + 1) & 63] + 1.0;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) ticks[1] = t1 - t0;
  if (v == -1.0) ids[0] = 0;
}
int main() {
  unsigned *ids; unsigned long long *t;
  hipMalloc(&ids, 64); hipMalloc(&t, 64);
  hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, ids, t);
  hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, ids, t);
  unsigned h[8]; unsigned long long tt[2];
  hipMemcpy(h, ids, 32, hipMemcpyDeviceToHost); hipMemcpy(tt, t, 16, hipMemcpyDeviceToHost);
  for (int w = 0; w < 8; w++) printf("wave %d: hw_id 0x%08x wave_slot %u simd %u cu %u\n", w, h[w], h[w] & 15, (h[w] >> 4) & 3, (h[w] >> 8) & 15);
  printf("barrier (8 waves) %.1f ticks, LDS write->read round trip %.1f ticks\n", tt[0] / 1000.0, tt[1] / 1000.0);
}
