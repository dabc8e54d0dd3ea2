// ubench_chain2.hip — cycles per element of an ordered FP64 dot-product
// chain over LDS (the shape of the eigensolver's gslcblas chains): 8 lanes
// of one wave each run their own chain of length n (strided rows, like the
// dsymv row chains), variants of load scheduling.  Reports s_memtime ticks
// (shader clock) per element.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NN = 512, LDA = NN + 1, ROWS = 8;

template <int V>
__global__ void __launch_bounds__(64) k_chain(const double *in, double *out, unsigned long long *ticks, int n) {
  extern __shared__ double sm[];
  double *M = sm;                 // ROWS x LDA
  double *tv = sm + ROWS * LDA;   // NN
  double *P = tv + NN;            // ROWS x LDA staged products
  const int lane = threadIdx.x;
  for (int i = lane; i < ROWS * LDA; i += 64) M[i] = in[i % 4096] + 1e-3 * i;
  for (int i = lane; i < NN; i += 64) tv[i] = in[(i * 7) % 4096];
  for (int i = lane; i < ROWS * LDA; i += 64) P[i] = M[i] * tv[i % LDA < NN ? i % LDA : 0];
  __syncthreads();
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (lane < ROWS) {
    const double *row = M + lane * LDA;
    if (V == 0) {  // original: 8 loads, 8 muls, 8 adds per batch
      int q = 0;
      for (; q + 8 <= n; q += 8) {
        double p[8];
#pragma unroll
        for (int u = 0; u < 8; u++) p[u] = tv[q + u] * row[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += p[u];
      }
    } else if (V == 1) {  // next batch loaded while the current is added (copies)
      double cur[8];
#pragma unroll
      for (int u = 0; u < 8; u++) cur[u] = tv[u] * row[u];
      int q = 8;
      for (; q + 8 <= n; q += 8) {
        double nx[8];
#pragma unroll
        for (int u = 0; u < 8; u++) nx[u] = tv[q + u] * row[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += cur[u];
#pragma unroll
        for (int u = 0; u < 8; u++) cur[u] = nx[u];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) acc += cur[u];
    } else if (V == 2) {  // ping-pong, no copies
      double a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; u++) a[u] = tv[u] * row[u];
      int q = 8;
      for (; q + 16 <= n; q += 16) {
#pragma unroll
        for (int u = 0; u < 8; u++) b[u] = tv[q + u] * row[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += a[u];
#pragma unroll
        for (int u = 0; u < 8; u++) a[u] = tv[q + 8 + u] * row[q + 8 + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += b[u];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) acc += a[u];
    } else if (V == 3) {  // products staged: add-only chain, 16 loads ahead
      const double *pr = P + lane * LDA;
      double a[16];
#pragma unroll
      for (int u = 0; u < 16; u++) a[u] = pr[u];
      int q = 16;
      for (; q + 16 <= n; q += 16) {
        double b[16];
#pragma unroll
        for (int u = 0; u < 16; u++) b[u] = pr[q + u];
#pragma unroll
        for (int u = 0; u < 16; u++) acc += a[u];
#pragma unroll
        for (int u = 0; u < 16; u++) a[u] = b[u];
      }
#pragma unroll
      for (int u = 0; u < 16; u++) acc += a[u];
    } else if (V == 4) {  // staged products, plain 8-batch
      const double *pr = P + lane * LDA;
      for (int q = 0; q + 8 <= n; q += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) t[u] = pr[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += t[u];
      }
    } else if (V == 5) {  // uniform chain (every lane the same addresses)
      for (int q = 0; q + 8 <= n; q += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) t[u] = tv[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += t[u];
      }
    } else if (V == 6) {  // register-only chain (latency floor)
      double x = tv[lane], y = tv[lane + 1];
      for (int q = 0; q < n; q += 2) {
        acc += x;
        acc += y;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) ticks[V] = t1 - t0;
}

int main() {
  double *in, *out;
  unsigned long long *t, h[8];
  hipMalloc(&in, 4096 * 8);
  hipMalloc(&out, 64 * 8);
  hipMalloc(&t, 8 * 8);
  double hin[4096];
  for (int i = 0; i < 4096; i++) hin[i] = 1.0 / (i + 1);
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  const size_t lds = (2 * ROWS * LDA + NN) * sizeof(double);
  hipFuncSetAttribute((const void *)k_chain<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const char *names[] = {"orig 8-batch mul+add", "pipelined copies", "ping-pong", "staged 16-ahead",
                         "staged 8-batch", "uniform 8-batch", "register floor"};
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipLaunchKernelGGL(k_chain<5>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipLaunchKernelGGL(k_chain<6>, dim3(1), dim3(64), lds, 0, in, out, t, NN);
    hipDeviceSynchronize();
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    if (rep)
      for (int v = 0; v < 7; v++) printf("%-24s %6.2f ticks/element\n", names[v], (double)h[v] / NN);
  }
  return 0;
}
