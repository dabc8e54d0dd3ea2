// ubench_issue.hip — per-instruction cycle costs on gfx950 that shape the
// eigensolver's latency chains: dependent / independent FP64 add, mul, fma,
// an LDS read feeding an add, and the cost of a single wave vs 4 waves per
// SIMD.  s_memtime ticks (shader clock) around a fixed instruction stream.
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int KIND>
__global__ void k_probe(double *out, unsigned long long *ticks, double seed) {
  __shared__ double lds[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = seed * i;
  __syncthreads();
  double a = seed, b = seed * 0.5, c = seed * 0.25, d = seed * 0.125, e = seed * 0.75, f = seed, g = seed, h = seed;
  const double m = 1.0000001;
  unsigned addr = (unsigned)(size_t)((__attribute__((address_space(3))) double *)lds + (threadIdx.x & 63));
  unsigned addrb = (unsigned)(size_t)((__attribute__((address_space(3))) double *)lds);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 16; it++) {
    if (KIND == 0) {  // dependent add chain
      REP64(asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if (KIND == 1) {  // 4 independent add chains (issue rate)
      REP8(REP8(asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4"
                             : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(b));))
    } else if (KIND == 2) {  // dependent mul chain
      REP64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(m));)
    } else if (KIND == 3) {  // 4 independent fma chains
      REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4"
                             : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(m));))
    } else if (KIND == 4) {  // 8 independent adds (issue rate, more ILP)
      REP8(asm volatile(
               "v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n"
               "v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8"
               : "+v"(a), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+v"(b) : "v"(m));)
    } else if (KIND == 5) {  // add chain + an independent mul per add (inline product)
      REP64(asm volatile("v_mul_f64 %1, %2, %3\n v_add_f64 %0, %0, %1" : "+v"(a), "=&v"(c) : "v"(b), "v"(m));)
    } else if (KIND == 6) {  // add chain + one ds_read_b64 per add (loaded 8 ahead, counted waits)
      double r0, r1, r2, r3, r4, r5, r6, r7;
      REP8(asm volatile(
               "ds_read_b64 %1, %9\n ds_read_b64 %2, %9 offset:512\n ds_read_b64 %3, %9 offset:1024\n"
               "ds_read_b64 %4, %9 offset:1536\n ds_read_b64 %5, %9 offset:2048\n ds_read_b64 %6, %9 offset:2560\n"
               "ds_read_b64 %7, %9 offset:3072\n ds_read_b64 %8, %9 offset:3584\n"
               "s_waitcnt lgkmcnt(7)\n v_add_f64 %0, %0, %1\n s_waitcnt lgkmcnt(6)\n v_add_f64 %0, %0, %2\n"
               "s_waitcnt lgkmcnt(5)\n v_add_f64 %0, %0, %3\n s_waitcnt lgkmcnt(4)\n v_add_f64 %0, %0, %4\n"
               "s_waitcnt lgkmcnt(3)\n v_add_f64 %0, %0, %5\n s_waitcnt lgkmcnt(2)\n v_add_f64 %0, %0, %6\n"
               "s_waitcnt lgkmcnt(1)\n v_add_f64 %0, %0, %7\n s_waitcnt lgkmcnt(0)\n v_add_f64 %0, %0, %8"
               : "+v"(a), "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
               : "v"(addr));)
    } else if (KIND == 10) {  // add chain over LDS values, 8 loads ahead, one wait per 8 adds
      double r0, r1, r2, r3, r4, r5, r6, r7, q0, q1, q2, q3, q4, q5, q6, q7;
      asm volatile(
          "ds_read_b64 %0, %8\n ds_read_b64 %1, %8 offset:512\n ds_read_b64 %2, %8 offset:1024\n"
          "ds_read_b64 %3, %8 offset:1536\n ds_read_b64 %4, %8 offset:2048\n ds_read_b64 %5, %8 offset:2560\n"
          "ds_read_b64 %6, %8 offset:3072\n ds_read_b64 %7, %8 offset:3584\n"
          : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7) : "v"(addr));
      REP8(asm volatile(
               "ds_read_b64 %9, %17\n ds_read_b64 %10, %17 offset:512\n ds_read_b64 %11, %17 offset:1024\n"
               "ds_read_b64 %12, %17 offset:1536\n ds_read_b64 %13, %17 offset:2048\n ds_read_b64 %14, %17 offset:2560\n"
               "ds_read_b64 %15, %17 offset:3072\n ds_read_b64 %16, %17 offset:3584\n"
               "s_waitcnt lgkmcnt(8)\n"
               "v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %3\n v_add_f64 %0, %0, %4\n"
               "v_add_f64 %0, %0, %5\n v_add_f64 %0, %0, %6\n v_add_f64 %0, %0, %7\n v_add_f64 %0, %0, %8\n"
               "ds_read_b64 %1, %17\n ds_read_b64 %2, %17 offset:512\n ds_read_b64 %3, %17 offset:1024\n"
               "ds_read_b64 %4, %17 offset:1536\n ds_read_b64 %5, %17 offset:2048\n ds_read_b64 %6, %17 offset:2560\n"
               "ds_read_b64 %7, %17 offset:3072\n ds_read_b64 %8, %17 offset:3584\n"
               "s_waitcnt lgkmcnt(8)\n"
               "v_add_f64 %0, %0, %9\n v_add_f64 %0, %0, %10\n v_add_f64 %0, %0, %11\n v_add_f64 %0, %0, %12\n"
               "v_add_f64 %0, %0, %13\n v_add_f64 %0, %0, %14\n v_add_f64 %0, %0, %15\n v_add_f64 %0, %0, %16\n"
               : "+v"(a), "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7),
                 "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(q4), "=&v"(q5), "=&v"(q6), "=&v"(q7)
               : "v"(addr));)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      a += r0 + r7;
    } else if (KIND == 12) {  // add chain over LDS values, 8 loads ahead, one wait per 8 adds
      double r0, r1, r2, r3, r4, r5, r6, r7, q0, q1, q2, q3, q4, q5, q6, q7;
      asm volatile(
          "ds_read_b64 %0, %8\n ds_read_b64 %1, %8 offset:8\n ds_read_b64 %2, %8 offset:16\n"
          "ds_read_b64 %3, %8 offset:24\n ds_read_b64 %4, %8 offset:32\n ds_read_b64 %5, %8 offset:40\n"
          "ds_read_b64 %6, %8 offset:48\n ds_read_b64 %7, %8 offset:56\n"
          : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7) : "v"(addrb));
      REP8(asm volatile(
               "ds_read_b64 %9, %17\n ds_read_b64 %10, %17 offset:8\n ds_read_b64 %11, %17 offset:16\n"
               "ds_read_b64 %12, %17 offset:24\n ds_read_b64 %13, %17 offset:32\n ds_read_b64 %14, %17 offset:40\n"
               "ds_read_b64 %15, %17 offset:48\n ds_read_b64 %16, %17 offset:56\n"
               "s_waitcnt lgkmcnt(8)\n"
               "v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %3\n v_add_f64 %0, %0, %4\n"
               "v_add_f64 %0, %0, %5\n v_add_f64 %0, %0, %6\n v_add_f64 %0, %0, %7\n v_add_f64 %0, %0, %8\n"
               "ds_read_b64 %1, %17\n ds_read_b64 %2, %17 offset:8\n ds_read_b64 %3, %17 offset:16\n"
               "ds_read_b64 %4, %17 offset:24\n ds_read_b64 %5, %17 offset:32\n ds_read_b64 %6, %17 offset:40\n"
               "ds_read_b64 %7, %17 offset:48\n ds_read_b64 %8, %17 offset:56\n"
               "s_waitcnt lgkmcnt(8)\n"
               "v_add_f64 %0, %0, %9\n v_add_f64 %0, %0, %10\n v_add_f64 %0, %0, %11\n v_add_f64 %0, %0, %12\n"
               "v_add_f64 %0, %0, %13\n v_add_f64 %0, %0, %14\n v_add_f64 %0, %0, %15\n v_add_f64 %0, %0, %16\n"
               : "+v"(a), "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7),
                 "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(q4), "=&v"(q5), "=&v"(q6), "=&v"(q7)
               : "v"(addrb));)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      a += r0 + r7;
    } else if (KIND == 11) {  // add chain with one s_waitcnt lgkmcnt(0) (no LDS op outstanding) per add
      REP64(asm volatile("s_waitcnt lgkmcnt(0)\n v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if (KIND == 7) {  // dependent v_max_f64 (prefix-max step cost without the DPP)
      REP64(asm volatile("v_max_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
    } else if (KIND == 8) {  // dependent 32-bit DPP row_shr mov chain
      int x = threadIdx.x;
      REP64(asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x));)
      a += x;
    } else if (KIND == 9) {  // 4 independent muls
      REP8(REP8(asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4"
                             : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(m));))
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + c + d + e + f + g + h;
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int K>
void run(const char *name, int ops_per_it, int threads, double *o, unsigned long long *t) {
  unsigned long long h[16];
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_probe<K>, dim3(1), dim3(threads), 0, 0, o, t, 1.0);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int w = 0; w < threads / 64; w++) mx = h[w] > mx ? h[w] : mx;
  printf("%-44s waves %2d: %6.2f cycles/op (per wave)\n", name, threads / 64, (double)mx / (16.0 * ops_per_it));
}

int main() {
  double *o;
  unsigned long long *t;
  hipMalloc(&o, 1 << 20);
  hipMalloc(&t, 4096);
  for (int th : {64, 1024}) {
    run<0>("dependent v_add_f64", 64, th, o, t);
    run<1>("4 independent v_add_f64", 256, th, o, t);
    run<4>("8 independent v_add_f64", 64, th, o, t);
    run<9>("4 independent v_mul_f64", 256, th, o, t);
    run<2>("dependent v_mul_f64", 64, th, o, t);
    run<3>("4 independent v_fma_f64", 256, th, o, t);
    run<5>("add chain + inline mul (per element)", 64, th, o, t);
    run<6>("add chain + ds_read_b64 (per element)", 64, th, o, t);
    run<10>("add chain, LDS 8 ahead, 1 wait per 8", 128, th, o, t);
    run<11>("add chain + s_waitcnt per add", 64, th, o, t);
    run<12>("add chain, broadcast LDS 8 ahead, 1 wait", 128, th, o, t);
    run<7>("dependent v_max_f64", 64, th, o, t);
    run<8>("dependent v_mov_b32_dpp", 64, th, o, t);
  }
  return 0;
}
