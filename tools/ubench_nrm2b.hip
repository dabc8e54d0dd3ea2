// ubench_nrm2b.hip — cycles of the one-workgroup tridiagonalisation's
// dnrm2 (kg::dnrm2_regs) and of a bare staged add chain, one wave alone,
// m = 63 / 127 elements of random data.
#include <cstring>
#include "../korali_amd/csrc/kg_eigen.hip"

#include <cstdio>
#include <string>
#include <vector>

namespace kg {
void set_error(const std::string &) {}  // the library's error sink (not linked here)
}  // namespace kg

__global__ void k_nrm2(const double *x, int m, double *out, unsigned long long *ticks, int reps) {
  __shared__ __attribute__((aligned(16))) double sv[256];
  const int lane = threadIdx.x;
  double x0 = x[min(lane, m - 1)], x1 = x[min(lane + 64, m - 1)];
  double acc = 0.0;
  unsigned long long tacc[2] = {0, 0}, tm = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; r++) {
    acc += kg::dnrm2_regs(x0, x1, m, sv, false, tacc, tm);
    x0 += 1e-300;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  // bare chain: m staged adds
  for (int e = lane; e < 256; e += 64) sv[e] = x[e & 127];
  __syncthreads();
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  double s2 = 0.0;
  for (int r = 0; r < reps; r++) s2 = kg::staged_sum(s2, sv, m);
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  // chain over values held one per lane, read with v_readlane (SGPR operand)
  const double vr0 = x[lane], vr1 = x[lane + 64];
  double s3 = 0.0;
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  if (lane == 0)
    for (int r = 0; r < reps; r++) s3 = kg::lds_chain_add(s3, sv, m);
  s3 = __shfl(s3, 0);
  unsigned long long t5 = __builtin_amdgcn_s_memtime();
  out[lane] = acc + s2 + s3;
  if (lane == 0) ticks[3] = (s2 == s3) ? 1 : 0;
  if (lane == 0) ticks[2] = (t5 - t4) / reps;
  if (lane == 0) {
    ticks[0] = (t1 - t0) / reps;
    ticks[1] = (t3 - t2) / reps;
  }
}

int main() {
  std::vector<double> h(256);
  unsigned long long s = 12345;
  for (auto &v : h) {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    v = ((s >> 11) * (1.0 / 9007199254740992.0)) - 0.5;
  }
  double *x, *o;
  unsigned long long *t, ht[4];
  (void)hipMalloc(&x, 256 * 8);
  (void)hipMalloc(&o, 64 * 8);
  (void)hipMalloc(&t, 32);
  (void)hipMemcpy(x, h.data(), 256 * 8, hipMemcpyHostToDevice);
  for (int m : {15, 63, 127}) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(k_nrm2, dim3(1), dim3(64), 0, 0, x, m, o, t, 64);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(ht, t, 32, hipMemcpyDeviceToHost);
    printf("m=%3d  dnrm2_regs %6llu cycles (%.1f/elem)   staged_sum %6llu (%.1f/elem)   lds_chain_add %6llu (%.1f/elem) same=%llu\n",
           m, ht[0], (double)ht[0] / m, ht[1], (double)ht[1] / m, ht[2], (double)ht[2] / m, ht[3]);
  }
  return 0;
}
