// ubench_chains.hip — cycles per element of the kg_chains.hpp primitives on
// gfx950, alone and beside other waves' LDS traffic (s_memtime ticks of
// wave 0, 512-thread workgroup as in k_tridiag_sq).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//     -I korali_amd/csrc -o tools/ubench_chains tools/ubench_chains.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "kg_chains.hpp"
#include "kg_chains_experimental.hpp"

using namespace kg::chains;

__device__ __forceinline__ unsigned la(const double *p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) double *)p;
}

constexpr int LD = 130;  // (even: 16-byte aligned row pairs for the ds_read_b128 chains)

// mode: 0 kc_add alone, 1 kc_add + 7 waves of LDS read/modify/write traffic,
// 2 kc_nrm2 alone (no rescale), 3 kc_lock_desc on wave 0 alone,
// 4 kc_lock_asc on wave 0 alone, 5 four lockstep waves (2 desc + 2 asc),
// 6 dependent v_add_f64 chain in registers (reference), 7 kc_add_desc alone
__global__ void __launch_bounds__(512) k_bench(int mode, int reps, double *out, unsigned long long *ticks) {
  extern __shared__ __attribute__((aligned(16))) double s[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double *M = s;                     // 144 x 129
  double *w = M + 144 * LD + 32;     // vector (padded)
  double *stage = w + 256;           // 256
  double *stage2 = M;                // mode 20: 512 values (rows of M, before any mode writes them)
  for (int i = tid; i < 144 * LD + 32 + 256 + 256 + 64; i += 512) s[i] = 1.0 / (1 + (i % 97));
  __syncthreads();
  double acc = 0.0;
  unsigned long long t0 = 0, t1 = 0;
  const int cnt = 128;
  if (mode == 0 || mode == 1 || mode == 2 || mode == 7) {
    if (wid == 0) {
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; r++) {
        if (mode == 2) acc = kc_nrm2(acc + 1.0, la(stage), __builtin_amdgcn_readfirstlane(cnt / 16), 0ull, 0ull);
        else if (mode == 7) acc = kc_add_desc(acc, la(stage + cnt - 16), __builtin_amdgcn_readfirstlane(cnt / 16));
        else acc = kc_add(acc, la(stage), __builtin_amdgcn_readfirstlane(cnt / 16));
      }
      t1 = __builtin_amdgcn_s_memtime();
    } else if (mode == 1) {
      for (int r = 0; r < reps * 4; r++)
        for (int c = lane; c < 128; c += 64) {
          double *row = M + (size_t)(wid * 16 + (r & 15)) * LD;
          row[c] += w[c] * w[c + 1] + row[c + 1];
        }
    }
  } else if (mode == 3 || mode == 4 || mode == 5) {
    const bool active = (mode == 5) ? wid < 4 : wid == 0;
    if (active) {
      const bool desc = (mode == 3) || (mode == 5 && wid < 2);
      const int r = lane + 64 * (wid & 1);
      t0 = __builtin_amdgcn_s_memtime();
      for (int k = 0; k < reps; k++) {
        if (desc) acc += kc_lock_desc(0.0, la(w + 120), la(M + (size_t)r * LD + 120), __builtin_amdgcn_readfirstlane(cnt / 8));
        else acc += kc_lock_asc<LD * 8>(0.0, la(w), la(M + r), __builtin_amdgcn_readfirstlane(cnt / 8));
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode == 8 || mode == 9) {
    if (wid == 0) {
      double b = stage[lane], c = b * 0.5, d = b * 0.25, e = b * 0.125, m_ = 1.0000001, tmp;
      t0 = __builtin_amdgcn_s_memtime();
      for (int k = 0; k < reps * cnt / 16; k++) {
        if (mode == 8) {  // 4 independent add chains: issue rate of v_add_f64 (16 adds = 4 elements of each)
#pragma unroll
          for (int u = 0; u < 4; u++)
            asm volatile("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4"
                         : "+v"(acc), "+v"(c), "+v"(d), "+v"(e) : "v"(b));
        } else {  // product formed inline: v_mul_f64 + dependent v_add_f64 per element
#pragma unroll
          for (int u = 0; u < 16; u++) asm volatile("v_mul_f64 %1, %2, %3\n v_add_f64 %0, %0, %1" : "+v"(acc), "=&v"(tmp) : "v"(b), "v"(m_));
        }
      }
      t1 = __builtin_amdgcn_s_memtime();
      acc += c + d + e;
    }
  } else if (mode == 10 || mode == 11) {  // kc_add on waves 0-3 (10) or on waves 0 and 4 (11) at once
    const bool active = mode == 10 ? wid < 4 : (wid == 0 || wid == 4);
    if (active) {
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; r++) acc = kc_add(acc, la(stage), __builtin_amdgcn_readfirstlane(cnt / 16));
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode == 12 || mode == 13 || mode == 14 || mode == 15) {
    // single-lane forms: EXEC = lane 0 only (12 register chain, 13 kc_add),
    // 14 register chain with a scalar (SGPR pair) operand, full EXEC;
    // 15 the SGPR-operand chain with EXEC = lane 0
    if (wid == 0) {
      const double b = stage[lane];
      const unsigned long long bb = (unsigned long long)__double_as_longlong(stage[3]);
      const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)bb), hi = __builtin_amdgcn_readfirstlane((unsigned)(bb >> 32));
      const double bs = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
      t0 = __builtin_amdgcn_s_memtime();
      if (mode == 14) {
        for (int k = 0; k < reps * cnt / 16; k++) {
#pragma unroll
          for (int u = 0; u < 16; u++) asm volatile("v_add_f64 %0, %0, %1" : "+v"(acc) : "s"(bs));
        }
      } else if (lane == 0) {
        if (mode == 12) {
          for (int k = 0; k < reps * cnt / 16; k++) {
#pragma unroll
            for (int u = 0; u < 16; u++) asm volatile("v_add_f64 %0, %0, %1" : "+v"(acc) : "v"(b));
          }
        } else if (mode == 15) {
          for (int k = 0; k < reps * cnt / 16; k++) {
#pragma unroll
            for (int u = 0; u < 16; u++) asm volatile("v_add_f64 %0, %0, %1" : "+v"(acc) : "s"(bs));
          }
        } else {
          for (int r = 0; r < reps; r++) acc = kc_add(acc, la(stage), __builtin_amdgcn_readfirstlane(cnt / 16));
        }
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode == 16 || mode == 17) {
    // 128-element chain over DPP row_newbcast broadcasts: the staged values
    // sit in 8 VGPR pairs (lane j of each row: element 16 k + j) and the chain
    // is v_fmac_f64 acc, q_k[j], 1.0 (= acc + q exactly) with no memory ops;
    // 17: seven other waves doing LDS read/modify/write traffic meanwhile
    if (wid == 0) {
      double q[8];
#pragma unroll
      for (int k = 0; k < 8; k++) q[k] = stage[16 * k + (lane & 15)];
      const double one = 1.0;
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; r++) {
#define DPPSTEP(K, J) asm volatile("v_fmac_f64 %0, %1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(q[K]), "v"(one));
#define DPPROW(K) DPPSTEP(K,0) DPPSTEP(K,1) DPPSTEP(K,2) DPPSTEP(K,3) DPPSTEP(K,4) DPPSTEP(K,5) DPPSTEP(K,6) DPPSTEP(K,7) \
                  DPPSTEP(K,8) DPPSTEP(K,9) DPPSTEP(K,10) DPPSTEP(K,11) DPPSTEP(K,12) DPPSTEP(K,13) DPPSTEP(K,14) DPPSTEP(K,15)
        DPPROW(0) DPPROW(1) DPPROW(2) DPPROW(3) DPPROW(4) DPPROW(5) DPPROW(6) DPPROW(7)
#undef DPPROW
#undef DPPSTEP
      }
      t1 = __builtin_amdgcn_s_memtime();
    } else if (mode == 17) {
      for (int r = 0; r < reps * 4; r++)
        for (int c = lane; c < 128; c += 64) {
          double *row = M + (size_t)(wid * 16 + (r & 15)) * LD;
          row[c] += w[c] * w[c + 1] + row[c + 1];
        }
    }
  } else if (mode == 20) {
    // four independent chains per wave, one per 16-lane row: row r sums
    // stage[128 r .. 128 r + 127] in order (per-row row_newbcast semantics;
    // checked against the host's sequential sums below)
    if (wid == 0) {
      double q[8];
      const int r = lane >> 4;
#pragma unroll
      for (int k = 0; k < 8; k++) q[k] = stage2[128 * r + 16 * k + (lane & 15)];
      const double one = 1.0;
      t0 = __builtin_amdgcn_s_memtime();
#define DPPSTEP(K, J) asm volatile("v_fmac_f64 %0, %1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(q[K]), "v"(one));
#define DPPROW(K) DPPSTEP(K,0) DPPSTEP(K,1) DPPSTEP(K,2) DPPSTEP(K,3) DPPSTEP(K,4) DPPSTEP(K,5) DPPSTEP(K,6) DPPSTEP(K,7) \
                  DPPSTEP(K,8) DPPSTEP(K,9) DPPSTEP(K,10) DPPSTEP(K,11) DPPSTEP(K,12) DPPSTEP(K,13) DPPSTEP(K,14) DPPSTEP(K,15)
      DPPROW(0) DPPROW(1) DPPROW(2) DPPROW(3) DPPROW(4) DPPROW(5) DPPROW(6) DPPROW(7)
#undef DPPROW
#undef DPPSTEP
      t1 = __builtin_amdgcn_s_memtime();
      t1 = t0 + (t1 - t0) * reps;  // (one pass; scaled to the common per-element report)
    }
  } else if (mode == 18 || mode == 19) {
    // dsymv-like per-lane chain: acc_lane += w_t * m_t with w wave-uniform in
    // SGPRs (18) or broadcast from LDS (19, kc_lock_desc-like), m per lane
    // from LDS (ds_read2 per two elements)
    if (wid == 0) {
      const double *mr = M + (size_t)lane * LD;
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; r++) {
        for (int c0 = 0; c0 < 128; c0 += 16) {
          double mv[16], wv[16];
#pragma unroll
          for (int u = 0; u < 16; u++) mv[u] = mr[c0 + u];
          if (mode == 18) {
#pragma unroll
            for (int u = 0; u < 16; u++) {
              const unsigned long long bb = (unsigned long long)__double_as_longlong(w[c0 + u]);
              const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)bb), hi = __builtin_amdgcn_readfirstlane((unsigned)(bb >> 32));
              wv[u] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
            }
          } else {
#pragma unroll
            for (int u = 0; u < 16; u++) wv[u] = w[c0 + u];
          }
#pragma unroll
          for (int u = 0; u < 16; u++) {
            double p;
            if (mode == 18) asm volatile("v_mul_f64 %0, %1, %2" : "=&v"(p) : "s"(wv[u]), "v"(mv[u]));
            else asm volatile("v_mul_f64 %0, %1, %2" : "=&v"(p) : "v"(wv[u]), "v"(mv[u]));
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(acc) : "v"(p));
          }
        }
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode == 26 || mode == 27) {
    // the dsymv lockstep chains with w broadcast from registers (DPP):
    // 26 kc_lock_desc_dpp on wave 0 alone, 27 four lockstep waves (2 desc + 2 asc)
    const bool active = (mode == 27) ? wid < 4 : wid == 0;
    if (active) {
      const bool desc = (mode == 26) || (mode == 27 && wid < 2);
      const int r = lane + 64 * (wid & 1);
      t0 = __builtin_amdgcn_s_memtime();
      for (int k = 0; k < reps; k++) {
        if (desc)
          acc += kc_lock_desc_dpp(0.0, la(w + 120) + ((lane & 7) << 3), la(M + (size_t)r * LD + 120),
                                  __builtin_amdgcn_readfirstlane(cnt / 8));
        else
          acc += kc_lock_asc_dpp<LD * 8>(0.0, la(w) + ((lane & 7) << 3), la(M + r), __builtin_amdgcn_readfirstlane(cnt / 8));
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode >= 28 && mode <= 31) {
    // kc_nrm2_dpp8 / kc_nrm2_dpp4 (three-operation spans) without / with the
    // three rescales of modes 21-25
    if (wid == 0) {
      double q[8], a[8];
#pragma unroll
      for (int k = 0; k < 8; k++) q[k] = stage[16 * k + (lane & 15)], a[k] = 1.0;
      const bool ev = mode == 29 || mode == 31;
      const unsigned long long k0 = ev ? ((1ull << 5) | (1ull << 40)) : 0ull, k1 = ev ? (1ull << 26) : 0ull;
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; r++) {
        if (mode <= 29) acc = kc_nrm2_dpp8(acc + 1.0, a, q, 8u, k0, k1);
        else acc = kc_nrm2_dpp4(acc + 1.0, a, q, 8u, k0, k1);
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode >= 21 && mode <= 25) {
    // the ssq recurrence on register-held elements: kc_nrm2_dpp without /
    // with three rescale events (elements 5, 40, 90: three different
    // halves), the per-element-check form without / with them, and the
    // branch-free three-operation form
    if (wid == 0) {
      double q[8], a[8];
#pragma unroll
      for (int k = 0; k < 8; k++) q[k] = stage[16 * k + (lane & 15)], a[k] = 1.0;
      const bool ev = mode == 22 || mode == 25;
      const unsigned long long k0 = ev ? ((1ull << 5) | (1ull << 40)) : 0ull, k1 = ev ? (1ull << 26) : 0ull;
      t0 = __builtin_amdgcn_s_memtime();
      for (int r = 0; r < reps; r++) {
        if (mode == 21 || mode == 22) acc = kc_nrm2_dpp(acc + 1.0, q, 8u, k0, k1);
        else if (mode == 23) acc = kc_nrm2_dpp3(acc + 1.0, a, q, 8u);
        else acc = kc_nrm2_dppc(acc + 1.0, q, 8u, k0, k1);
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  } else if (mode == 6) {
    if (wid == 0) {
      double b = stage[lane];
      t0 = __builtin_amdgcn_s_memtime();
      for (int k = 0; k < reps * cnt / 16; k++) {
#pragma unroll
        for (int u = 0; u < 16; u++) asm volatile("v_add_f64 %0, %0, %1" : "+v"(acc) : "v"(b));
      }
      t1 = __builtin_amdgcn_s_memtime();
    }
  }
  out[tid] = acc;
  if (tid == 0) ticks[mode] = t1 - t0;
}

int main() {
  double *out;
  unsigned long long *ticks;
  hipMalloc(&out, 512 * sizeof(double));
  hipMalloc(&ticks, 32 * sizeof(unsigned long long));
  const size_t lds = (144 * LD + 32 + 256 + 256 + 64) * sizeof(double);
  hipFuncSetAttribute((const void *)k_bench, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int reps = 200;
  const char *names[] = {"kc_add alone", "kc_add + 7 LDS waves", "kc_nrm2 alone", "kc_lock_desc alone",
                         "kc_lock_asc alone", "4 lockstep waves", "register add chain", "kc_add_desc alone",
                         "4 indep. add chains (per add)", "inline mul+add chain", "kc_add on waves 0-3",
                         "kc_add on waves 0 and 4", "reg chain, exec=lane0", "kc_add, exec=lane0",
                         "reg chain, sgpr operand", "sgpr chain, exec=lane0", "dpp-bcast fmac chain",
                         "dpp-bcast chain + 7 LDS waves", "dsymv lane chain, sgpr w", "dsymv lane chain, lds w",
                         "4 row chains / wave (dpp)", "nrm2_dpp, no rescale", "nrm2_dpp, 3 rescales",
                         "nrm2 branch-free 3-op", "nrm2 per-elt check, none", "nrm2 per-elt check, 3",
                         "kc_lock_desc_dpp alone", "4 lockstep waves (dpp w)", "nrm2 8-spans, none",
                         "nrm2 8-spans, 3", "nrm2 4-spans, none", "nrm2 4-spans, 3"};
  for (int mode = 0; mode < 32; mode++) {
    for (int warm = 0; warm < 2; warm++) hipLaunchKernelGGL(k_bench, dim3(1), dim3(512), lds, 0, mode, reps, out, ticks);
    hipDeviceSynchronize();
    unsigned long long t[32];
    hipMemcpy(t, ticks, sizeof(t), hipMemcpyDeviceToHost);
    printf("%-24s %8.2f ticks/element\n", names[mode], (double)t[mode] / (reps * 128.0));
    if (mode == 20) {  // per-row sums vs the host's sequential sums of the same inputs
      double o[512];
      hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
      int ok = 1;
      for (int r = 0; r < 4; r++) {
        double a = 0.0;
        for (int e = 0; e < 128; e++) a += 1.0 / (1 + ((128 * r + e) % 97));
        for (int l = 16 * r; l < 16 * r + 16; l++) ok &= (o[l] == a);
      }
      printf("  per-row chains bit-exact vs host: %s\n", ok ? "yes" : "NO");
    }
  }
  return 0;
}
