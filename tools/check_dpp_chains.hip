// check_dpp_chains.hip — bit-exactness of the register/DPP chain primitives
// (kc_add_dpp, kc_nrm2_dpp, kc_row16) against the LDS-streamed ones (kc_add,
// kc_nrm2) and a host restatement, on random inputs, every group count
// 1..8 and random rescale masks.  One wave per trial, as in k_tridiag_sq's
// wave 0.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//     -I korali_amd/csrc -o tools/check_dpp_chains tools/check_dpp_chains.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "kg_chains.hpp"
#include "kg_chains_experimental.hpp"

using namespace kg::chains;

__device__ __forceinline__ unsigned la(const double *p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) double *)p;
}

// trial t: v[t][0..127], g[t], mask[t][0..1]; out[t][0..3] = add (stream),
// add (dpp), nrm2 (stream), nrm2 (dpp)
__global__ void __launch_bounds__(64) k_check(const double *v, const unsigned *g, const unsigned long long *mask,
                                              double *out) {
  __shared__ double sv[160];
  const int t = blockIdx.x, lane = threadIdx.x;
  sv[lane] = v[(size_t)t * 128 + lane];
  sv[64 + lane] = v[(size_t)t * 128 + 64 + lane];
  if (lane < 32) sv[128 + lane] = 0.0;
  __syncthreads();
  const unsigned G = __builtin_amdgcn_readfirstlane(g[t]);
  const unsigned long long k0 = mask[2 * t], k1 = mask[2 * t + 1];
  double q[8];
#pragma unroll
  for (int k = 0; k < 8; k++) q[k] = sv[16 * k + (lane & 15)];
  const double a0 = kc_add(0.0, la(sv), G);
  const double a1 = kc_add_dpp(0.0, q, G);
  const double n0 = kc_nrm2(1.0, la(sv), G, k0, k1);
  const double n1 = kc_nrm2_dpp(1.0, q, G, k0, k1);
  if (lane == 0) {
    out[4 * t + 0] = a0;
    out[4 * t + 1] = a1;
    out[4 * t + 2] = n0;
    out[4 * t + 3] = n1;
  }
}

int main(int argc, char **argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 4096;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<double> v((size_t)T * 128), out((size_t)T * 4);
  std::vector<unsigned> g(T);
  std::vector<unsigned long long> mask(2 * (size_t)T);
  for (int t = 0; t < T; t++) {
    g[t] = 1 + t % 8;
    const int m = 16 * (int)g[t] - (int)(rng() % 16);  // ragged: trailing zeros as the kernels stage them
    const int mode = t % 3;                            // 0: no rescales, 1: sparse, 2: dense rescales
    unsigned long long k[2] = {0, 0};
    for (int e = 0; e < 128; e++) {
      double x = 0.0;
      if (e < m) {
        x = U(rng);
        const bool r = mode == 1 ? (rng() % 29 == 0) : (mode == 2 ? (rng() % 3 == 0) : false);
        if (r) k[e >> 6] |= 1ull << (e & 63);
      }
      v[(size_t)t * 128 + e] = x;
    }
    mask[2 * t] = k[0];
    mask[2 * t + 1] = k[1];
  }
  double *dv, *dout;
  unsigned *dg;
  unsigned long long *dm;
  hipMalloc(&dv, v.size() * sizeof(double));
  hipMalloc(&dout, out.size() * sizeof(double));
  hipMalloc(&dg, g.size() * sizeof(unsigned));
  hipMalloc(&dm, mask.size() * sizeof(unsigned long long));
  hipMemcpy(dv, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice);
  hipMemcpy(dg, g.data(), g.size() * sizeof(unsigned), hipMemcpyHostToDevice);
  hipMemcpy(dm, mask.data(), mask.size() * sizeof(unsigned long long), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_check, dim3(T), dim3(64), 0, 0, dv, dg, dm, dout);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 2;
  }
  hipMemcpy(out.data(), dout, out.size() * sizeof(double), hipMemcpyDeviceToHost);
  int bad[4] = {0, 0, 0, 0};
  for (int t = 0; t < T; t++) {
    double a = 0.0, n = 1.0;
    for (int e = 0; e < 16 * (int)g[t]; e++) {
      const double x = v[(size_t)t * 128 + e];
      a = a + x;
      if ((mask[2 * t + (e >> 6)] >> (e & 63)) & 1) {
        const double tmp = n * x;
        n = 1.0 + tmp * x;
      } else {
        n = n + x;
      }
    }
    const double ref[4] = {a, a, n, n};
    for (int c = 0; c < 4; c++)
      if (memcmp(&ref[c], &out[4 * t + c], sizeof(double))) {
        if (bad[c] < 4)
          printf("mismatch trial %d (G=%u, mode %d) col %d: host %.17g device %.17g\n", t, g[t], t % 3, c, ref[c],
                 out[4 * t + c]);
        bad[c]++;
      }
  }
  printf("trials %d: kc_add %d bad, kc_add_dpp %d bad, kc_nrm2 %d bad, kc_nrm2_dpp %d bad\n", T, bad[0], bad[1],
         bad[2], bad[3]);
  return (bad[0] || bad[1] || bad[2] || bad[3]) ? 1 : 0;
}
