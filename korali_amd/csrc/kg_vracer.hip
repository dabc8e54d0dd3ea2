// kg_vracer.hip — VRACER on MI355X.
//
// The agent's whole training loop runs on the device: E concurrent CartPole
// environments step together (one thread per environment, the episode kept
// in HBM until it ends), finished episodes are appended to a device-resident
// replay memory (SoA ring in HBM, the reference's cBuffer view: logical 0 =
// oldest), and every policy update — mini-batch draw + sort, the critic/policy
// network forward on 2B rows (mini-batch states + their truncated states),
// REF-ER metadata, retrace chains, the VRACER loss gradient, the backward pass
// and fAdam — is a short chain of kernels with no host round trip.  Dense
// layers run on the FP32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32
// products, f32 accumulation) from LDS-staged 64x64 tiles; the layers whose
// other dimension is the state / action size run on the VALU.
//
// Reference (paths relative to the korali root):
//   Agent::trainingGeneration / processEpisode / generateMiniBatch /
//   updateExperienceMetadata        solver/agent/agent.cpp.base:162-735
//   VRACER::trainPolicy / calculatePolicyGradients / runPolicy
//                                   solver/agent/continuous/VRACER/VRACER.cpp.base:65-205
//   Continuous (Normal policy)      solver/agent/continuous/continuous.cpp.base:34-61,
//                                   :137-150, :278-440, :697-732
//   DeepSupervisor::runGeneration   solver/learner/deepSupervisor/deepSupervisor.cpp.base:97-161
//   Linear / Output layers          neuralNetwork/layer/{linear,output}/*.cpp.base
//   fAdam::processResult            solver/learner/deepSupervisor/optimizers/fAdam.cpp:64-91
//   CartPole environment            examples/learning/reinforcement/cartpole/_model
// The CPU restatement is oracle/vracer_ref.py (test infrastructure only).
#include "kg_common.hpp"
#include "../../include/korali_amd.h"

#include <unistd.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace kg {
namespace vr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int MAXA = 4;  // action dimensions supported by the device kernels
constexpr int MAXO = 1 + 2 * MAXA;
constexpr int MAXB = 2048;  // mini-batch size limit (one-workgroup sort / metadata)
constexpr int MAXENV = 64;  // reward rescaling: up to this many environment ids are staged in LDS (any count runs)
constexpr int MAXS = 8;     // state dimensions with state rescaling
enum : int { NON_TERMINAL = 0, TERMINAL = 1, TRUNCATED = 2 };
enum : unsigned {
  ERR_NONFINITE_GRADIENT = 1u,
  ERR_NONFINITE_VALUE = 2u,
  ERR_NONFINITE_IW = 4u,
  ERR_ENV_ODE = 8u,
  ERR_EPISODE_LONG = 16u  // a host environment's episode outgrew max_episode_steps
};

// Device-resident agent scalars (float where the reference keeps float).
struct State {
  float lr, beta, cutoff, off_ratio, eta, b1p, b2p, pad0;
  long long off_count, update_count;
  unsigned long long total;       // experiences ever appended (ring position)
  unsigned long long size;        // replay memory size
  unsigned long long episode;     // _currentEpisode
  unsigned long long sample_id;   // _currentSampleID (next environment launch)
  unsigned long long mb_counter;  // philox counter of the mini-batch uniforms
  unsigned long long env_step;    // philox counter of the action noise
  unsigned long long step_new, step_base, step_episodes, step_episode_base, step_sample_base;
  unsigned long long experience_count;
  unsigned errors;
  unsigned rr_all;                // reward rescaling: every id's sigma recomputed once (the first episode's update)
  double step_reward_sum;         // cumulative rewards of the episodes finished by the last step
  // state rescaling (agent.cpp.base:92-94, :291-322): the moments episodes
  // launched from now on scale their states with (identity until set)
  float smean[MAXS], ssdev[MAXS];
  // k_vr_meta's phases (s_memrealtime, 100 MHz ticks, summed over updates):
  // setup + importance weights, retrace chains, loss gradient + metadata
  unsigned long long mtr[9];  // k_vr_meta: phase ticks x3; sums of the longest walk, walked entries, walks; walk sub-phase ticks x3
};

struct Params {  // launch-constant configuration
  int S, A, H, L, O, E, B, T;     // T = max episode steps
  long long R;                    // replay memory capacity
  int env_count, l2;
  float gamma, lr0, iw_trunc, cutoff_scale, off_target, anneal, l2imp;
  float scale[MAXO], shift[MAXO];
  int soft[MAXO];
  unsigned long long seed;
  int clipped;                    // Policy Distribution: 0 Normal, 1 Clipped Normal
  float lb[MAXA], ub[MAXA];       // action bounds (Variables' Lower / Upper Bound)
  int rr;                         // Reward / Rescaling / Enabled
  int srs;                        // State Rescaling / Enabled
  int host;                       // a host 'Environment Function' feeds the environment steps
};

// ---------------------------------------------------------------- philox
struct u4 {
  unsigned x, y, z, w;
};
__host__ __device__ inline u4 philox4x32(u4 c, unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x, p1 = (unsigned long long)0xCD9E8D57u * c.z;
    c = u4{(unsigned)(p1 >> 32) ^ c.y ^ k0, (unsigned)p1, (unsigned)(p0 >> 32) ^ c.w ^ k1, (unsigned)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// Two standard normals (Box-Muller in double) from one philox block; the
// stream is keyed by (seed, purpose) and counted by (a, b).
__device__ inline void philox_normals(unsigned long long seed, unsigned purpose, unsigned long long a, unsigned b,
                                      float &n0, float &n1) {
  const u4 r = philox4x32(u4{(unsigned)a, (unsigned)(a >> 32), b, purpose}, (unsigned)seed, (unsigned)(seed >> 32));
  const double u1 = ((double)r.x + 1.0) * 2.3283064365386963e-10;  // (0, 1]
  const double u2 = (double)r.y * 2.3283064365386963e-10;          // [0, 1)
  const double rad = sqrt(-2.0 * log(u1));
  n0 = (float)(rad * cos(6.283185307179586 * u2));
  n1 = (float)(rad * sin(6.283185307179586 * u2));
}
__device__ inline float philox_uniform24(unsigned long long seed, unsigned long long ctr) {
  const u4 r = philox4x32(u4{(unsigned)ctr, (unsigned)(ctr >> 32), 0u, 0x4D42u}, (unsigned)seed, (unsigned)(seed >> 32));
  return (float)(r.x >> 8) * 5.9604644775390625e-08f;  // [0, 1)
}

// ------------------------------------------------------- Normal policy math
// auxiliar/math.hpp:269-274 with T = float: 2*M_PI and KORALI_EPSILON
// promote the expressions to double; norm and d are stored as float.
__device__ __noinline__ float normal_logp(float x, float mean, float sigma) {
  const float norm = (float)(-0.5 * log(2.0 * M_PI * (double)sigma * (double)sigma));
  const float d = (float)((double)(x - mean) / ((double)sigma + 0.00000000001));
  return (float)((double)norm - 0.5 * (double)d * (double)d);
}

// Clipped Normal pieces (auxiliar/math.hpp:297-328, T = float): z is rounded
// to float, log(0.5) + log erfc in double.  GSL's gsl_sf_log_erfc is
// restated as log(erfc(x)) with the asymptotic series where erfc underflows.
__device__ __noinline__ double log_erfc_d(double x) {
  if (x < 26.0) return log(erfc(x));
  const double x2 = x * x, h = 1.0 / (2.0 * x2);
  return -x2 - log(x) - 0.57236494292470008707 + log(1.0 - h + 3.0 * h * h - 15.0 * h * h * h);
}
__device__ __noinline__ float normal_logcdf(float x, float mean, float sigma) {
  const float z = (float)((double)(x - mean) / ((double)sigma * M_SQRT2));
  return (float)(log(0.5) + log_erfc_d(-(double)z));
}
__device__ __noinline__ float normal_logccdf(float x, float mean, float sigma) {
  const float z = (float)((double)(x - mean) / ((double)sigma * M_SQRT2));
  return (float)(log(0.5) + log_erfc_d((double)z));
}
// log-density of one action component (continuous.cpp.base:283-340)
__device__ inline float policy_logp(const Params &P, int i, float a, float m, float s) {
  if (P.clipped) {
    if (a <= P.lb[i]) return normal_logcdf(P.lb[i], m, s);
    if (P.ub[i] <= a) return normal_logccdf(P.ub[i], m, s);
  }
  return normal_logp(a, m, s);
}

// ------------------------------------------------------------ layer kernels
// Input layer (K = state size): H = tanh(X W1^T + b1), one thread per output.
__global__ void k_vr_fwd_in(int M, int S, int H, const float *__restrict__ X, const float *__restrict__ W,
                            const float *__restrict__ b, float *__restrict__ Y) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)M * H) return;
  const int m = (int)(t / H), o = (int)(t % H);
  float acc = 0.f;
  for (int i = 0; i < S; i++) acc += W[o * S + i] * X[(long long)m * S + i];
  Y[t] = tanhf(acc + b[o]);
}

// Output layer (N = 1 + 2A): Linear + Output-layer transformation
// (output.cpp.base:140-160: Softplus 0.5 (x + sqrt(1 + x^2)) in double, then
// Scale and Shift in float).  One wave per row: each lane takes H/64
// consecutive columns, the O partial sums are reduced across the wave.
__global__ __launch_bounds__(256) void k_vr_fwd_out(int M, int H, int O, const float *__restrict__ Hs,
                                                    const float *__restrict__ W, const float *__restrict__ b,
                                                    float *__restrict__ out, Params P) {
  const int lane = threadIdx.x & 63, m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float acc[MAXO];  // (static indices only: loops unrolled to MAXO, o < O guarded)
#pragma unroll
  for (int o = 0; o < MAXO; o++) acc[o] = 0.f;
  const float *h = Hs + (long long)m * H;
  // four columns' loads in flight per lane before their products (each
  // lane's sums still run over its columns in ascending order)
  constexpr int U = 4;
  for (int i0 = lane; i0 < H; i0 += 64 * U) {
    float xs[U], ws[U][MAXO];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int i = i0 + 64 * u;
      xs[u] = i < H ? h[i] : 0.f;
#pragma unroll
      for (int o = 0; o < MAXO; o++) ws[u][o] = (o < O && i < H) ? W[o * H + i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (i0 + 64 * u < H) {
#pragma unroll
        for (int o = 0; o < MAXO; o++)
          if (o < O) acc[o] += ws[u][o] * xs[u];
      }
  }
#pragma unroll
  for (int o = 0; o < MAXO; o++)
    if (o < O)
      for (int d = 32; d > 0; d >>= 1) acc[o] += __shfl_xor(acc[o], d, 64);
  if (lane < O) {
    float x = 0.f;
#pragma unroll
    for (int o = 0; o < MAXO; o++)
      if (o == lane) x = acc[o];
    x = x + b[lane];
    if (P.soft[lane]) x = (float)(0.5 * ((double)x + sqrt(1.0 + (double)x * (double)x)));
    out[(long long)m * O + lane] = x * P.scale[lane] + P.shift[lane];
  }
}

// C[m][n] = sum_k A(m,k) B(n,k) on v_mfma_f32_16x16x4_f32.  These products
// are small (M, N <= 4096 x 256, K <= 512) and sit on the per-update latency
// chain, so a workgroup owns a 32x32 tile and stages its whole A and B panels
// (up to 256 k-columns at a time) in LDS with every load in flight at once;
// each wave then computes one 16x16 block over the panel with two
// interleaved accumulators (the 40-cycle dependent MFMA latency hidden behind
// the 32-cycle issue).  Any element strides (X W^T, W^T-side and
// batch-reduction products share the kernel).  Epilogues: bias + tanh
// (forward), times (1 - T^2) (tanh backward), plain.
enum : int { EP_STORE = 0, EP_BIAS_TANH = 1, EP_DTANH = 2 };
constexpr int GT = 32, GK = 256, GP = GT + 1;
template <int EP>
__device__ __forceinline__ void vr_gemm_tile(int M, int N, int K, const float *__restrict__ A, long long sam,
                                             long long sak, const float *__restrict__ B, long long sbn, long long sbk,
                                             float *__restrict__ C, long long ldc, const float *__restrict__ bias,
                                             const float *__restrict__ T, long long ldt, int vec, int bx, int by,
                                             float (&As)[GK][GP], float (&Bs)[GK][GP]) {
  const int m0 = by * GT, n0 = bx * GT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, br = wave >> 1, bc = wave & 1, li = lane & 15,
            lk = lane >> 4;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  for (int k0 = 0; k0 < K; k0 += GK) {
    const int kc = min(GK, K - k0);
    if (vec && m0 + GT <= M && n0 + GT <= N) {
      // full tile, 16-byte aligned strides: every thread issues all its float4
      // loads (8 per panel at kc = 256) before the first LDS store
      float4 ra[8], rb[8];
      const int nv = GT * kc / 4;  // float4s per panel (kc % 4 == 0)
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int e = t + 256 * q;
        if (e < nv) {
          if (sak == 1) ra[q] = *reinterpret_cast<const float4 *>(A + (m0 + e / (kc / 4)) * sam + k0 + 4 * (e % (kc / 4)));
          else ra[q] = *reinterpret_cast<const float4 *>(A + (long long)(k0 + e / 8) * sak + m0 + 4 * (e % 8));
          if (sbk == 1) rb[q] = *reinterpret_cast<const float4 *>(B + (n0 + e / (kc / 4)) * sbn + k0 + 4 * (e % (kc / 4)));
          else rb[q] = *reinterpret_cast<const float4 *>(B + (long long)(k0 + e / 8) * sbk + n0 + 4 * (e % 8));
        }
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const int e = t + 256 * q;
        if (e < nv) {
          if (sak == 1) {
            const int r = e / (kc / 4), k = 4 * (e % (kc / 4));
            As[k][r] = ra[q].x, As[k + 1][r] = ra[q].y, As[k + 2][r] = ra[q].z, As[k + 3][r] = ra[q].w;
          } else {
            const int k = e / 8, r = 4 * (e % 8);
            As[k][r] = ra[q].x, As[k][r + 1] = ra[q].y, As[k][r + 2] = ra[q].z, As[k][r + 3] = ra[q].w;
          }
          if (sbk == 1) {
            const int r = e / (kc / 4), k = 4 * (e % (kc / 4));
            Bs[k][r] = rb[q].x, Bs[k + 1][r] = rb[q].y, Bs[k + 2][r] = rb[q].z, Bs[k + 3][r] = rb[q].w;
          } else {
            const int k = e / 8, r = 4 * (e % 8);
            Bs[k][r] = rb[q].x, Bs[k][r + 1] = rb[q].y, Bs[k][r + 2] = rb[q].z, Bs[k][r + 3] = rb[q].w;
          }
        }
      }
      for (int e = t; e < GT * (GK - kc); e += 256) {  // zero rows past kc (MFMA reads up to kc rounded to 8)
        const int k = kc + e / GT, r = e % GT;
        As[k][r] = 0.f, Bs[k][r] = 0.f;
      }
    } else
    // stage: element (r, k) of the 32-row panel; k fastest when k is the contiguous stride
    for (int e = t; e < GT * GK; e += 256) {
      int r, k;
      if (sak == 1) k = e % GK, r = e / GK;
      else r = e % GT, k = e / GT;
      const int gm = m0 + r;
      As[k][r] = (k < kc && gm < M) ? A[gm * sam + (long long)(k0 + k) * sak] : 0.f;
      if (sbk == 1) k = e % GK, r = e / GK;
      else r = e % GT, k = e / GT;
      const int gn = n0 + r;
      Bs[k][r] = (k < kc && gn < N) ? B[gn * sbn + (long long)(k0 + k) * sbk] : 0.f;
    }
    __syncthreads();
    const int kr = (kc + 7) & ~7;
    for (int kk = 0; kk < kr; kk += 8) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(As[kk + lk][br * 16 + li], Bs[kk + lk][bc * 16 + li], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(As[kk + 4 + lk][br * 16 + li], Bs[kk + 4 + lk][bc * 16 + li], acc1,
                                                  0, 0, 0);
    }
    __syncthreads();
  }
  // C/D layout of the f32 16x16x4 form: col = lane & 15, row = 4 (lane >> 4) + reg
  const int col = n0 + bc * 16 + li;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = m0 + br * 16 + lk * 4 + r;
    if (row >= M || col >= N) continue;
    float v = acc0[r] + acc1[r];
    if (EP == EP_BIAS_TANH) v = tanhf(v + bias[col]);
    if (EP == EP_DTANH) {
      const float y = T[row * ldt + col];
      v = v * (1.0f - y * y);
    }
    C[row * ldc + col] = v;
  }
}
template <int EP>
__global__ __launch_bounds__(256) void k_vr_gemm(int M, int N, int K, const float *__restrict__ A, long long sam,
                                                 long long sak, const float *__restrict__ B, long long sbn,
                                                 long long sbk, float *__restrict__ C, long long ldc,
                                                 const float *__restrict__ bias, const float *__restrict__ T,
                                                 long long ldt, int vec) {
  __shared__ float As[GK][GP];
  __shared__ float Bs[GK][GP];
  vr_gemm_tile<EP>(M, N, K, A, sam, sak, B, sbn, sbk, C, ldc, bias, T, ldt, vec, blockIdx.x, blockIdx.y, As, Bs);
}

// Output-layer backward (output.cpp.base:170-210) and the last Linear's data
// gradient: dZ = transformed G; dH[b][i] = (sum_o dZ[b][o] W[o][i]) (1 - h^2).
__global__ void k_vr_bwd_out(int Bn, int H, int O, const float *__restrict__ G, const float *__restrict__ out,
                             const float *__restrict__ W, const float *__restrict__ Hs, float *__restrict__ dZ,
                             float *__restrict__ dH, Params P) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)Bn * H) return;
  const int b = (int)(t / H), i = (int)(t % H);
  float dz[MAXO];  // (static indices only: loops unrolled to MAXO, o < O guarded)
  float xo[MAXO], go[MAXO], wo[MAXO];
  // every operand's load in flight first (the arithmetic below is unchanged)
#pragma unroll
  for (int o = 0; o < MAXO; o++) {
    xo[o] = o < O ? out[b * O + o] : 0.f;
    go[o] = o < O ? G[b * O + o] : 0.f;
    wo[o] = o < O ? W[o * H + i] : 0.f;
  }
  const float y = Hs[(long long)b * H + i];
  float acc = 0.f;
#pragma unroll
  for (int o = 0; o < MAXO; o++) {
    dz[o] = 0.f;
    if (o < O) {
      float x = xo[o], g = go[o];
      x = x - P.shift[o];
      x = x / P.scale[o];
      g = g * P.scale[o];
      if (P.soft[o]) {
        const float nnx = x - 0.25f / x;
        g = (float)((double)g * 0.5 * (1.0 + (double)nnx / sqrt((double)nnx * (double)nnx + 1.0)));
      }
      dz[o] = g;
      acc += dz[o] * wo[o];
    }
  }
  if (i == 0)
#pragma unroll
    for (int o = 0; o < MAXO; o++)
      if (o < O) dZ[b * O + o] = dz[o];
  dH[t] = acc * (1.0f - y * y);
}

// Weight gradients of a layer with a small dimension, and bias gradients:
// dW[o][i] = sum_b G[b][o] Act[b][i] for i < Ni, db[o] = sum_b G[b][o]
// (linear.cpp.base:337-350: summed over the batch).  One workgroup per
// (o, column chunk): CW columns x (256 / CW) batch lanes, partial sums
// reduced through LDS in a fixed order (deterministic).
__device__ __forceinline__ void vr_adam_elem(long long j, float g, float *__restrict__ theta, float *__restrict__ m1,
                                             float *__restrict__ m2, const State *__restrict__ st, int l2,
                                             float l2imp) {
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-08f;
  const float f1 = 1.0f / (1.0f - st->b1p), f2 = 1.0f / (1.0f - st->b2p);
  if (l2) g -= l2imp * theta[j];
  const float m = b1 * m1[j] - (1.0f - b1) * g;
  const float v = b2 * m2[j] + (1.0f - b2) * g * g;
  m1[j] = m;
  m2[j] = v;
  theta[j] -= st->eta / (sqrtf(v * f2) + eps) * m * f1;
}
struct VrAdamJob {
  float *theta, *m1, *m2;
  const float *grad;
  const State *st;
  long long lo, hi;  // the parameters the adam blocks update (the wgrad blocks update their own)
  int l2;
  float l2imp;
};
__device__ __forceinline__ void vr_wgrad_block(int No, int Ni, int Bn, const float *__restrict__ G, int ldg,
                                               const float *__restrict__ Act, int lda, float *__restrict__ dW,
                                               float *__restrict__ db, int CW, int bx, int by, float *part,
                                               const VrAdamJob *adam = nullptr) {
  const int o = bx, t = threadIdx.x, lanes = 256 / CW, c = t % CW, l = t / CW;
  const int i = by * CW + c;
  float acc = 0.f;
  if (i <= Ni)
#pragma unroll 4
    for (int b = l; b < Bn; b += lanes) {
      const float g = G[b * ldg + o];
      acc += i < Ni ? g * Act[(long long)b * lda + i] : g;
    }
  part[t] = acc;
  __syncthreads();
  for (int w = lanes >> 1; w > 0; w >>= 1) {
    if (l < w) part[t] += part[t + w * CW];
    __syncthreads();
  }
  if (l == 0 && i <= Ni) {
    float *gp = i < Ni ? dW + o * Ni + i : db + o;
    *gp = part[c];
    if (adam) vr_adam_elem(gp - adam->grad, part[c], adam->theta, adam->m1, adam->m2, adam->st, adam->l2, adam->l2imp);
  }
}
__global__ __launch_bounds__(256) void k_vr_wgrad_small(int No, int Ni, int Bn, const float *__restrict__ G, int ldg,
                                                        const float *__restrict__ Act, int lda,
                                                        float *__restrict__ dW, float *__restrict__ db, int CW) {
  __shared__ float part[256];
  vr_wgrad_block(No, Ni, Bn, G, ldg, Act, lda, dW, db, CW, blockIdx.x, blockIdx.y, part);
}

// Independent weight-gradient products of one backward step in ONE launch
// (round 4): the output layer's wgrad, dW_l, db_l and dH_(l-1) only read
// dZ / dH_l and the activations, so their blocks run side by side instead
// of as four dependent launches.  Each job's blocks run the same bodies as
// the separate kernels (identical results); blockIdx selects the job.
struct VrGemmJob {
  const float *A, *B, *bias, *T;
  float *C;
  long long sam, sak, sbn, sbk, ldc, ldt;
  int M, N, K, vec, ep, gx, n;
};
struct VrWgradJob {
  const float *G, *Act;
  float *dW, *db;
  int No, Ni, Bn, ldg, lda, cw, n;
};
struct VrMulti {
  VrWgradJob w[2];
  VrGemmJob g[2];
  int nw, ng;
};
// The input layer's weight gradients and the whole Adam step in one launch:
// the wgrad blocks apply Adam to the parameters they just reduced (W_0, b_0),
// the others to every parameter the previous launches' gradients finished
__global__ __launch_bounds__(256) void k_vr_wgrad_adam(VrWgradJob w, VrAdamJob a) {
  __shared__ float part[256];
  const int b = blockIdx.x;
  if (b < w.n) {
    vr_wgrad_block(w.No, w.Ni, w.Bn, w.G, w.ldg, w.Act, w.lda, w.dW, w.db, w.cw, b % w.No, b / w.No, part, &a);
    return;
  }
  const long long j = a.lo + (long long)(b - w.n) * 256 + threadIdx.x;
  if (j < a.hi) vr_adam_elem(j, a.grad[j], a.theta, a.m1, a.m2, a.st, a.l2, a.l2imp);
}
__global__ __launch_bounds__(256) void k_vr_multi(VrMulti J) {
  __shared__ float As[GK][GP];
  __shared__ float Bs[GK][GP];
  int b = blockIdx.x;
  for (int q = 0; q < J.nw; q++) {
    const VrWgradJob &w = J.w[q];
    if (b < w.n) {
      vr_wgrad_block(w.No, w.Ni, w.Bn, w.G, w.ldg, w.Act, w.lda, w.dW, w.db, w.cw, b % w.No, b / w.No, &As[0][0]);
      return;
    }
    b -= w.n;
  }
  for (int q = 0; q < J.ng; q++) {
    const VrGemmJob &g = J.g[q];
    if (b < g.n) {
      const int bx = b % g.gx, by = b / g.gx;
      if (g.ep == EP_STORE)
        vr_gemm_tile<EP_STORE>(g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbn, g.sbk, g.C, g.ldc, g.bias, g.T, g.ldt,
                               g.vec, bx, by, As, Bs);
      else if (g.ep == EP_DTANH)
        vr_gemm_tile<EP_DTANH>(g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbn, g.sbk, g.C, g.ldc, g.bias, g.T, g.ldt,
                               g.vec, bx, by, As, Bs);
      else
        vr_gemm_tile<EP_BIAS_TANH>(g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbn, g.sbk, g.C, g.ldc, g.bias, g.T,
                                   g.ldt, g.vec, bx, by, As, Bs);
      return;
    }
    b -= g.n;
  }
}

// fAdam::processResult (fAdam.cpp:64-91), optional L2 term
// (deepSupervisor.cpp.base:147-153); eta and the beta powers were advanced
// by the metadata kernel of the same update.
__global__ void k_vr_adam(long long n, float *__restrict__ theta, const float *__restrict__ grad,
                          float *__restrict__ m1, float *__restrict__ m2, const State *__restrict__ st, int l2,
                          float l2imp) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  vr_adam_elem(j, grad[j], theta, m1, m2, st, l2, l2imp);
}

// ------------------------------------------------------------ replay memory
struct Replay {
  float *st, *act, *rew, *tst, *exp_pol, *cur_pol, *exp_v, *v, *ret, *iw, *tiw, *tv;
  int *env, *term, *onp, *ep_pos;
  long long *ep_id;
  // reward rescaling (agent.cpp.base:96-98, :423-437, :557-563), one entry
  // per environment id (Problem / Environment Count)
  float *rsig;      // getScaledReward's sigma (1.0 until the first update)
  float *rsum;      // sum of squared rewards in the replay memory
  long long *rcnt;  // experiences in the replay memory
};
__device__ inline long long phys(const State *s, long long R, long long i) {
  return (long long)((s->total - s->size + (unsigned long long)i) % (unsigned long long)R);
}

// generateMiniBatch (agent.cpp.base:574-597): B uniforms -> floor(x (size-1)),
// sorted (bitonic in LDS); gathers the mini-batch states into rows [0, B) and
// their truncated states into rows [B, 2B) of X.
// the mini-batch's sorted replay ids into key[0, B) (every thread of the
// workgroup; the draw counter is advanced by the caller's last kernel)
__device__ __forceinline__ void vr_minibatch_keys(const Params &P, const State *st, const unsigned *forced,
                                                  unsigned *key, unsigned long long ctr_ahead = 0) {
  const int t = threadIdx.x, nt = blockDim.x, B = P.B;
  int n2 = 1;
  while (n2 < B) n2 <<= 1;
  const unsigned long long ctr = st->mb_counter + ctr_ahead;
  const float sz1 = (float)(st->size - 1);
  for (int i = t; i < n2; i += nt) {
    unsigned id = 0xffffffffu;
    if (i < B) {
      id = forced ? forced[i] : (unsigned)floorf(philox_uniform24(P.seed, ctr + i) * sz1);
      if (id >= st->size) id = (unsigned)(st->size - 1);  // never reached for ids the host checked
    }
    key[i] = id;
  }
  __syncthreads();
  if (n2 <= nt) {
    // one key per thread: the same compare-exchange network, the stages
    // with partners inside the wave (j < 64) through lane shuffles, the
    // others through LDS (3 barrier pairs at B = 256 instead of 36 barriers)
    unsigned x = t < n2 ? key[t] : 0xffffffffu;
    for (int k = 2; k <= n2; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        unsigned y;
        if (j >= 64) {
          if (t < n2) key[t] = x;
          __syncthreads();
          y = t < n2 ? key[t ^ j] : 0xffffffffu;
          __syncthreads();
        } else {
          y = (unsigned)__shfl_xor((int)x, j, 64);
        }
        // the pair's lower element keeps the minimum in an ascending block
        x = (((t & j) == 0) == ((t & k) == 0)) ? min(x, y) : max(x, y);
      }
    if (t < n2) key[t] = x;
    __syncthreads();
  } else {
    for (int k = 2; k <= n2; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = t; i < n2; i += nt) {
          const int l = i ^ j;
          if (l > i) {
            const unsigned a = key[i], c = key[l];
            if ((a > c) == ((i & k) == 0)) key[i] = c, key[l] = a;
          }
        }
        __syncthreads();
      }
  }
}

__global__ __launch_bounds__(1024) void k_vr_minibatch(Params P, State *st, Replay er, unsigned *mb,
                                                       const unsigned *forced, float *X) {
  __shared__ unsigned key[MAXB];
  const int t = threadIdx.x, nt = blockDim.x, B = P.B;
  const unsigned long long ctr = st->mb_counter;
  vr_minibatch_keys(P, st, forced, key);
  const unsigned long long R = (unsigned long long)P.R, base = (st->total - st->size) % R;
  for (int i = t; i < B * P.S; i += nt) {
    const int b = i / P.S, k = i % P.S;
    unsigned long long q = base + key[b];
    if (q >= R) q -= R;
    const long long p = (long long)q;
    X[(long long)b * P.S + k] = er.st[p * P.S + k];
    X[(long long)(B + b) * P.S + k] = er.tst[p * P.S + k];
  }
  for (int i = t; i < B; i += nt) mb[i] = key[i];
  __syncthreads();
  if (t == 0) st->mb_counter = ctr + (forced ? 0 : (unsigned long long)B);
}

// A graph of policy updates (kg_vracer_train_policy) draws its mini-batches
// up front: workgroup u draws and sorts update u's ids from the draw counter
// + u B (the replay memory's size does not change between the environment
// steps, and each update's k_vr_meta advances the counter by B), so the ids
// are those the updates would draw one by one.
__global__ __launch_bounds__(256) void k_vr_draw_ahead(Params P, const State *st, unsigned *keys) {
  __shared__ unsigned key[MAXB];
  vr_minibatch_keys(P, st, (const unsigned *)nullptr, key, (unsigned long long)blockIdx.x * P.B);
  for (int i = threadIdx.x; i < P.B; i += blockDim.x) keys[(size_t)blockIdx.x * P.B + i] = key[i];
}

// ... and each update then gathers its rows while forming the input layer
// (k_vr_minibatch's gather + k_vr_fwd_in's products, same order, one launch):
// thread (m, o) loads row m's state (row b < B: entry b's state, row B + b
// its truncated state), writes it to Xmb (o = 0) and forms tanh(W x + b)[o].
__global__ void k_vr_gather_in(Params P, const State *st, Replay er, const unsigned *__restrict__ keys,
                               unsigned *mb, float *Xmb, const float *__restrict__ W, const float *__restrict__ bias,
                               float *__restrict__ Y) {
  const int B = P.B, S = P.S, H = P.H;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 2LL * B * H) return;
  const int m = (int)(e / H), o = (int)(e % H), b = m < B ? m : m - B;
  const unsigned long long R = (unsigned long long)P.R, base = (st->total - st->size) % R;
  unsigned long long q = base + keys[b];
  if (q >= R) q -= R;
  const float *src = (m < B ? er.st : er.tst) + (long long)q * S;
  float x[MAXS], w[MAXS];  // (unrolled with guards: registers, every load in flight)
#pragma unroll
  for (int i = 0; i < MAXS; i++) {
    x[i] = i < S ? src[i] : 0.f;
    w[i] = i < S ? W[o * S + i] : 0.f;
  }
  if (o == 0) {
#pragma unroll
    for (int i = 0; i < MAXS; i++)
      if (i < S) Xmb[(long long)m * S + i] = x[i];
  }
  if (e < B) mb[e] = keys[e];
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < MAXS; i++)
    if (i < S) acc += w[i] * x[i];
  Y[e] = tanhf(acc + bias[o]);
}

// The mini-batch draw fused with the input layer (round 5): every workgroup
// draws and sorts the B ids (vr_minibatch_keys: the same ids everywhere),
// gathers its MI rows -- row b < B the state of mini-batch entry b, row B + b
// its truncated state -- into Xmb and forms their input-layer activations
// exactly as k_vr_fwd_in does (same products, same order, tanhf(acc + b)).
// Workgroup 0 stores the ids; the draw counter advances in k_vr_meta.  Saves
// k_vr_fwd_in's launch and its dependency on a one-workgroup draw.
constexpr int MI = 8;
__global__ __launch_bounds__(256) void k_vr_minibatch_in(Params P, const State *st, Replay er, unsigned *mb,
                                                        const unsigned *forced, float *Xmb, const float *__restrict__ W,
                                                        const float *__restrict__ bias, float *__restrict__ Y) {
  __shared__ unsigned key[MAXB];
  __shared__ float xs[MI * 16];
  const int t = threadIdx.x, B = P.B, S = P.S, H = P.H, M = 2 * B;
  vr_minibatch_keys(P, st, forced, key);
  const int m0 = blockIdx.x * MI;
  const unsigned long long R = (unsigned long long)P.R, base = (st->total - st->size) % R;
  for (int e = t; e < MI * S; e += 256) {
    const int r = e / S, i = e % S, m = m0 + r;
    if (m < M) {
      const int b = m < B ? m : m - B;
      unsigned long long q = base + key[b];
      if (q >= R) q -= R;
      const float x = (m < B ? er.st : er.tst)[(long long)q * S + i];
      xs[e] = x;
      Xmb[(long long)m * S + i] = x;
    }
  }
  if (blockIdx.x == 0)
    for (int i = t; i < B; i += 256) mb[i] = key[i];
  __syncthreads();
  for (int e = t; e < MI * H; e += 256) {
    const int r = e / H, o = e % H, m = m0 + r;
    if (m >= M) break;
    float acc = 0.f;
    for (int i = 0; i < S; i++) acc += W[o * S + i] * xs[r * S + i];
    Y[(long long)m * H + o] = tanhf(acc + bias[o]);
  }
}

// The whole forward pass (input layer, the L-1 hidden H x H layers, the
// output layer) in ONE launch (round 5): a workgroup owns 16 rows and keeps
// their activations in LDS between layers, the hidden layers on
// v_mfma_f32_16x16x4_f32 with the weights streamed through LDS in 64-k
// chunks.  Every value is formed by the same operations in the same order as
// k_vr_fwd_in / k_vr_gemm<EP_BIAS_TANH> / k_vr_fwd_out (the same k order and
// the two interleaved accumulators per 16x16 block, the same lane partial
// sums and shuffle tree of the output layer): the results are those of the
// three-kernel form bit for bit, with one launch instead of L + 1 and no
// activation round trips through HBM between layers (the layers' outputs are
// still stored for the backward pass).  H <= 256.  MB (a policy update's
// forward): every workgroup also draws and sorts the mini-batch ids
// (k_vr_minibatch's vr_minibatch_keys, the same ids everywhere) and gathers
// its rows -- row b < B the state of mini-batch entry b, row B + b its
// truncated state -- into LDS and Xmb; workgroup 0 stores the ids.  The draw
// counter then advances in k_vr_meta (no workgroup may see it move).
constexpr int FR = 16, FK = 64, FHP = FR + 1, FNP = 256 + 1;
template <bool MB>
__global__ __launch_bounds__(256) void k_vr_fwd_fused(Params P, int M, const float *__restrict__ X,
                                                      const float *__restrict__ theta, const long long *offs,
                                                      float *__restrict__ acts, long long rowsMax,
                                                      float *__restrict__ out, const State *st, Replay er,
                                                      unsigned *mb, const unsigned *forced, float *Xmb) {
  __shared__ float Aa[256][FHP], Ab[256][FHP];  // activations [k][row] (the MFMA A operand's layout)
  __shared__ float Ws[FK][FNP];                 // a 64-k chunk of a layer's weights [k][out column]
  __shared__ unsigned key[MB ? MAXB : 1];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, li = lane & 15, lk = lane >> 4;
  const int H = P.H, S = P.S, O = P.O, L = P.L;
  const int m0 = blockIdx.x * FR;
  const float *xr = X;  // the input rows (MB: staged in Ws, row stride S)
  long long xs = (long long)m0 * S;
  if (MB) {
    vr_minibatch_keys(P, st, forced, key);
    const int B = P.B;
    const unsigned long long R = (unsigned long long)P.R, base = (st->total - st->size) % R;
    float *stg = &Ws[0][0];
    for (int e = t; e < FR * S; e += 256) {
      const int r = e / S, i = e % S, m = m0 + r;
      if (m < M) {
        const int b = m < B ? m : m - B;
        unsigned long long q = base + key[b];
        if (q >= R) q -= R;
        const float x = (m < B ? er.st : er.tst)[(long long)q * S + i];
        stg[e] = x;
        Xmb[(long long)m * S + i] = x;
      }
    }
    if (blockIdx.x == 0)
      for (int i = t; i < B; i += 256) mb[i] = key[i];
    __syncthreads();
    xr = stg, xs = 0;
  }
  const int Hp = (H + 15) & ~15;  // columns in whole 16-wide blocks
  const int Kr = (H + 7) & ~7;    // MFMA k extent (zero rows past H)
  // ---- input layer (k_vr_fwd_in's per-element loop), its operands staged in
  // LDS first (the rows, W_0 and b_0: every load in flight at once)
  {
    const float *W = theta + offs[0], *b = theta + offs[L + 1];
    float *stg = &Ws[0][0];
    const bool staged = FR * S + H * S + H <= FK * FNP;
    auto copy = [&](float *dst, const float *src, int n) __attribute__((always_inline)) {
      for (int i0 = t; i0 < n; i0 += 8 * 256) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = i0 + 256 * u < n ? src[i0 + 256 * u] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (i0 + 256 * u < n) dst[i0 + 256 * u] = v[u];
      }
    };
    if (staged) {
      if (!MB) copy(stg, X + (long long)m0 * S, min(FR, M - m0) * S);  // (MB: gathered above)
      copy(stg + FR * S, W, H * S);
      copy(stg + FR * S + H * S, b, H);
      __syncthreads();
      xr = stg, xs = 0, W = stg + FR * S, b = stg + FR * S + H * S;
    }
    for (int e = t; e < FR * Hp; e += 256) {
      const int r = e / Hp, o = e % Hp, m = m0 + r;
      float y = 0.f;
      if (o < H && m < M) {
        float acc = 0.f;
        for (int i = 0; i < S; i++) acc += W[o * S + i] * xr[xs + (long long)r * S + i];
        y = tanhf(acc + b[o]);
        acts[(long long)m * H + o] = y;
      }
      Aa[o][r] = y;
    }
    for (int e = t; e < FR * (256 - Hp); e += 256) Aa[Hp + e / FR][e % FR] = 0.f;
  }
  __syncthreads();  // (MB: the staged rows are read before Ws takes weights)
  float(*cur)[FHP] = Aa;
  float(*nxt)[FHP] = Ab;
  // ---- hidden layers l = 1 .. L-1 (k_vr_gemm<EP_BIAS_TANH>: C = tanh(A W^T + b))
  for (int l = 1; l < L; l++) {
    const float *W = theta + offs[l], *b = theta + offs[L + 1 + l];
    const bool vec4 = H % 64 == 0 && ((uintptr_t)W & 15) == 0;
    f32x4 acc0[4], acc1[4];  // column blocks wave, wave + 4, wave + 8, wave + 12
#pragma unroll
    for (int q = 0; q < 4; q++) acc0[q] = f32x4{0.f, 0.f, 0.f, 0.f}, acc1[q] = acc0[q];
    for (int k0 = 0; k0 < Kr; k0 += FK) {
      const int kc = min(FK, Kr - k0);
      __syncthreads();  // the previous chunk's reads (and the layer's activations) are complete
      // W[n][k0 .. k0+kc) for every column n < Hp (zeros past H): all of a
      // thread's loads in flight before its first LDS store
      if (vec4 && kc == FK) {
        float4 rw[16];  // Hp * FK / 4 / 256 <= 16 float4 per thread
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int e = t + 256 * u, n = e >> 4, k = 4 * (e & 15);
          if (n < Hp) rw[u] = *reinterpret_cast<const float4 *>(W + (long long)n * H + k0 + k);
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int e = t + 256 * u, n = e >> 4, k = 4 * (e & 15);
          if (n < Hp) Ws[k][n] = rw[u].x, Ws[k + 1][n] = rw[u].y, Ws[k + 2][n] = rw[u].z, Ws[k + 3][n] = rw[u].w;
        }
      } else {
        for (int e0 = t; e0 < Hp * FK; e0 += 8 * 256) {
          float rv[8];
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int e = e0 + 256 * u, n = e / FK, k = e % FK;
            rv[u] = (e < Hp * FK && n < H && k < kc && k0 + k < H) ? W[(long long)n * H + k0 + k] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int e = e0 + 256 * u;
            if (e < Hp * FK) Ws[e % FK][e / FK] = rv[u];
          }
        }
      }
      __syncthreads();
      for (int kk = 0; kk < kc; kk += 8) {
        const float a0 = cur[k0 + kk + lk][li], a1 = cur[k0 + kk + 4 + lk][li];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int nb = (wave + 4 * q) * 16;
          if (nb < Hp) {
            acc0[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, Ws[kk + lk][nb + li], acc0[q], 0, 0, 0);
            acc1[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, Ws[kk + 4 + lk][nb + li], acc1[q], 0, 0, 0);
          }
        }
      }
    }
    // epilogue: C/D layout col = lane & 15, row = 4 (lane >> 4) + reg
    float *Y = acts + (size_t)l * rowsMax * H;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int nb = (wave + 4 * q) * 16, col = nb + li;
      if (nb >= Hp) continue;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = lk * 4 + r, m = m0 + row;
        float v = 0.f;
        if (col < H) {
          v = tanhf(acc0[q][r] + acc1[q][r] + b[col]);
          if (m < M) Y[(long long)m * H + col] = v;
        }
        nxt[col][row] = v;
      }
    }
    for (int e = t; e < FR * (256 - Hp); e += 256) nxt[Hp + e / FR][e % FR] = 0.f;
    float(*tmp)[FHP] = cur;
    cur = nxt;
    nxt = tmp;
  }
  // ---- output layer (k_vr_fwd_out: one wave per row, lane partial sums over
  // columns lane, lane + 64, ..., the xor-shuffle tree, then the transform);
  // W_L and b_L staged in LDS (Ws is free once the last layer's products are done)
  const float *W = theta + offs[L], *bo = theta + offs[2 * L + 1];
  __syncthreads();
  if (O * H + O <= FK * FNP) {
    float *stg = &Ws[0][0];
    const int n = O * H + O;
    for (int i0 = t; i0 < n; i0 += 8 * 256) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + 256 * u;
        v[u] = i < O * H ? W[i] : (i < n ? bo[i - O * H] : 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (i0 + 256 * u < n) stg[i0 + 256 * u] = v[u];
    }
    W = stg, bo = stg + O * H;
  }
  __syncthreads();
  for (int r = wave; r < FR; r += 4) {
    const int m = m0 + r;
    if (m >= M) break;
    float acc[MAXO];
#pragma unroll
    for (int o = 0; o < MAXO; o++) acc[o] = 0.f;
    for (int i = lane; i < H; i += 64) {
      const float x = cur[i][r];
#pragma unroll
      for (int o = 0; o < MAXO; o++)
        if (o < O) acc[o] += W[o * H + i] * x;
    }
#pragma unroll
    for (int o = 0; o < MAXO; o++)
      if (o < O)
        for (int d = 32; d > 0; d >>= 1) acc[o] += __shfl_xor(acc[o], d, 64);
    if (lane < O) {
      float x = 0.f;
#pragma unroll
      for (int o = 0; o < MAXO; o++)
        if (o == lane) x = acc[o];
      x = x + bo[lane];
      if (P.soft[lane]) x = (float)(0.5 * ((double)x + sqrt(1.0 + (double)x * (double)x)));
      out[(long long)m * O + lane] = x * P.scale[lane] + P.shift[lane];
    }
  }
}

// One action component's importance-weight gradient factors, before the
// weight's scaling, and its log-densities under the current and the
// experience's policy (continuous.cpp.base:404-440 Normal, :482-560 Clipped
// Normal; component i's bounds)
__device__ inline void iw_grad_terms(const Params &P, int i, float a, float cm, float cs, float om, float osd,
                                     float &pg0, float &pg1, float &lc, float &lo) {
  const float dif = a - cm;
  if (!P.clipped) {
    const float inv_var = 1.f / (cs * cs);
    pg0 = dif * inv_var;
    pg1 = (dif * dif) * (inv_var / cs) - 1.f / cs;
    lc = normal_logp(a, cm, cs);
    lo = normal_logp(a, om, osd);
    return;
  }
  const float inv_sig = 1.f / cs, lb = P.lb[i], ub = P.ub[i];
  if (a <= lb) {
    const float lcdf = normal_logcdf(lb, cm, cs);
    const float r = expf(normal_logp(lb, cm, cs) - lcdf);
    pg0 = -r;
    pg1 = -dif * inv_sig * r;
    lc = lcdf;
    lo = normal_logcdf(lb, om, osd);
  } else if (ub <= a) {
    const float lccdf = normal_logccdf(ub, cm, cs);
    const float r = expf(normal_logp(ub, cm, cs) - lccdf);
    pg0 = r;
    pg1 = dif * inv_sig * r;
    lc = lccdf;
    lo = normal_logccdf(ub, om, osd);
  } else {
    const float inv_sig3 = inv_sig * inv_sig * inv_sig;
    pg0 = dif * inv_sig * inv_sig;
    pg1 = dif * dif * inv_sig3 - inv_sig;
    lc = normal_logp(a, cm, cs);
    lo = normal_logp(a, om, osd);
  }
}

// One action component's KL-divergence gradient with respect to the current
// mean and sigma (continuous.cpp.base:697-732 Normal, :734-777 Clipped Normal)
__device__ inline void kl_grad_terms(const Params &P, int i, float cm, float cs, float om, float osd, float &km,
                                     float &ks) {
  const float inv_sig = (float)(1. / (double)cs);
  const float inv_var = (float)(1. / (double)(cs * cs));
  const float inv_sig3 = (float)(1. / (double)(cs * cs * cs));
  const float d = cm - om;
  km = d * inv_var;
  ks = -inv_sig3 * osd * osd + -(d * d) * inv_sig3 + inv_sig;
  if (!P.clipped) return;
  const float lb = P.lb[i], ub = P.ub[i];
  const float oldVar = osd * osd, oldInvSig = 1.f / osd, curInvSig = 1.f / cs;
  const float curInvVar = 1.f / (cs * cs), curInvSig3 = 1.f / (cs * cs * cs), muDif = om - cm;
  const float invSqrt2Pi = (float)(M_SQRT1_2 * sqrt(M_1_PI));
  const float oldAdjLb = (lb - om) * oldInvSig, oldAdjUb = (ub - om) * oldInvSig;
  const float curAdjLb = (lb - cm) * curInvSig, curAdjUb = (ub - cm) * curInvSig;
  const float erfLb = (float)erf(M_SQRT1_2 * (double)oldAdjLb), erfUb = (float)erf(M_SQRT1_2 * (double)oldAdjUb);
  const float expLb = expf(-0.5f * oldAdjLb * oldAdjLb), expUb = expf(-0.5f * oldAdjUb * oldAdjUb);
  const float cdfA = expf(normal_logcdf(lb, om, osd) + normal_logp(lb, cm, cs) - normal_logcdf(lb, cm, cs));
  const float ccdfB = expf(normal_logccdf(ub, om, osd) + normal_logp(ub, cm, cs) - normal_logccdf(ub, cm, cs));
  km = cdfA;
  km -= 0.5f * muDif * curInvVar * (erfUb - erfLb);
  km += invSqrt2Pi * osd * curInvVar * (expUb - expLb);
  km -= ccdfB;
  ks = curAdjLb * cdfA;
  ks += 0.5f * (curInvSig - muDif * muDif * curInvSig3 - oldVar * curInvSig3) * (erfUb - erfLb);
  ks += invSqrt2Pi * curInvSig3 * (oldVar * oldAdjUb + 2.f * osd * muDif) * expUb;
  ks -= invSqrt2Pi * curInvSig3 * (oldVar * oldAdjLb + 2.f * osd * muDif) * expLb;
  ks -= curAdjUb * ccdfB;
}

// updateExperienceMetadata (agent.cpp.base:599-735) + the VRACER loss
// gradient (VRACER.cpp.base:89-181) + the REF-ER schedule (agent.cpp.base:
// 221-231), one workgroup.  Every mini-batch row's metadata lives in LDS
// between the phases: the retrace chains take the updated state values and
// truncated weights of mini-batch entries from LDS and leave each row's
// retrace value (and its successor's) there, so the gradient phase reads no
// global memory, and the replay-memory metadata is written once at the end
// (no global store is waited for at the first barrier).  One action
// component's operands live in LDS; with more, the gradient phase reads them
// from the replay memory and the forward's output.
constexpr int MB_META = 1024;
#ifndef VR_RC
#define VR_RC 16  // retrace chunk: entries per load round trip of a walk
#endif
// a byte flag from LDS as a full 32-bit value (keeps compares on it out of SDWA byte-select forms)
__device__ __forceinline__ int u8v(unsigned char b) {
  int v = b;
  asm volatile("" : "+v"(v));
  return v;
}
// a 16-bit LDS value as a full 32-bit one (no SDWA word selects on it)
__device__ __forceinline__ int u16v(unsigned short h) {
  int v = h;
  asm volatile("" : "+v"(v));
  return v;
}
// RR: reward rescaling enabled (every reward through getScaledReward: the
// divisions are exact no-ops at sigma 1.0, but the retrace walk then also
// loads each entry's environment id, so the plain form does without)
template <bool RR>
__global__ __launch_bounds__(512) void k_vr_meta(Params P, State *st, Replay er, const unsigned *mb,
                                                 const float *__restrict__ out, float *__restrict__ G,
                                                 unsigned long long advance, int staged) {
  __shared__ unsigned s_mb[MB_META];
  __shared__ float s_V[MB_META], s_tiw[MB_META], s_iw[MB_META], s_ret[MB_META], s_retn[MB_META], s_rew[MB_META],
      s_tv[MB_META], s_act[MB_META], s_cur[2 * MB_META], s_old[2 * MB_META];
  __shared__ unsigned char s_term[MB_META], s_onp[MB_META], s_uniq[MB_META];
  __shared__ int s_delta, s_wmax, s_wtot, s_wcnt;
  __shared__ float s_rsig[MAXENV];
  const int t = threadIdx.x, nt = blockDim.x, B = P.B, O = P.O;
  // every scalar read once into registers
  const float cutoff = st->cutoff, beta = st->beta, lr = st->lr, b1p = st->b1p, b2p = st->b2p;
  const long long off0 = st->off_count, upd0 = st->update_count;
  const unsigned long long size0 = st->size;
  const unsigned long long R = (unsigned long long)P.R, base = (st->total - st->size) % R;
  auto ph = [&](long long i) -> long long {
    unsigned long long q = base + (unsigned long long)i;
    if (q >= R) q -= R;
    return (long long)q;
  };
  const unsigned long long tm0 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) s_delta = 0, s_wmax = 0, s_wtot = 0, s_wcnt = 0;
  const bool rsl = P.env_count <= MAXENV;  // the sigmas staged in LDS (else read from the replay memory's table)
  if (RR && rsl && t < P.env_count) s_rsig[t] = er.rsig[t];
  __syncthreads();
  // ---- importance weights and on-policy flags (agent.cpp.base:613-657);
  // duplicates compute the same values, only the first occurrence counts
  int delta = 0;
  for (int b = t; b < B; b += nt) {
    const unsigned id = mb[b];
    const bool uniq = b == 0 || id != mb[b - 1];
    const long long p = ph(id);
    const float a = er.act[p * P.A], om = er.exp_pol[2 * P.A * p], osd = er.exp_pol[2 * P.A * p + P.A],
                rew = RR ? er.rew[p] / er.rsig[er.env[p]] : er.rew[p];
    const int was = er.onp[p], term = er.term[p];
    const float V = out[(long long)b * O], cm = out[(long long)b * O + 1], cs = out[(long long)b * O + 1 + P.A];
    const float tvv = term == TRUNCATED ? out[(long long)(B + b) * O] : 0.0f;
    float liw;
    if (P.A == 1) {
      liw = policy_logp(P, 0, a, cm, cs) - policy_logp(P, 0, a, om, osd);
    } else {  // calculateImportanceWeight's sums over the action components, in order
      const int A = P.A;
      float lc = 0.0f, lo = 0.0f;
      for (int i = 0; i < A; i++) {
        const float ai = er.act[p * A + i];
        lc += policy_logp(P, i, ai, out[(long long)b * O + 1 + i], out[(long long)b * O + 1 + A + i]);
        lo += policy_logp(P, i, ai, er.exp_pol[p * 2 * A + i], er.exp_pol[p * 2 * A + A + i]);
      }
      liw = lc - lo;
    }
    if (liw > 7.f) liw = 7.f;
    if (liw < -7.f) liw = -7.f;
    if (!isfinite(liw)) atomicOr(&st->errors, (unsigned)ERR_NONFINITE_IW);
    if (!isfinite(V)) atomicOr(&st->errors, (unsigned)ERR_NONFINITE_VALUE);
    const float iw = expf(liw);
    const float tiw = iw < P.iw_trunc ? iw : P.iw_trunc;  // std::min(level, iw)
    const int onp = (iw > 1.0f / cutoff) && (iw < cutoff);
    if (uniq) {
      if (was && !onp) delta++;
      if (!was && onp) delta--;
    }
    s_mb[b] = id, s_uniq[b] = uniq;
    s_V[b] = V, s_tiw[b] = tiw, s_iw[b] = iw, s_rew[b] = rew, s_tv[b] = tvv, s_act[b] = a;
    s_cur[2 * b] = cm, s_cur[2 * b + 1] = cs, s_old[2 * b] = om, s_old[2 * b + 1] = osd;
    s_term[b] = (unsigned char)term, s_onp[b] = (unsigned char)onp;
  }
  if (delta) atomicAdd(&s_delta, delta);
  __syncthreads();
  const unsigned long long tm1 = __builtin_amdgcn_s_memrealtime();
  const long long off1 = off0 + s_delta;
  const float off_ratio = (float)off1 / (float)size0;
  // ---- retrace chains of the oldest mini-batch entries of each episode
  // (agent.cpp.base:679-733, same operation order): a walk runs from the
  // episode's last mini-batch entry down to the episode's start, retV = v +
  // tiw (r + g retV - v) per entry.  One thread walking its episode through
  // the replay memory pays one load round trip per 16 entries (19 us of the
  // kernel's 22 at C5, longest walk ~84 entries).  Staged form: the whole
  // workgroup first loads every walk's entries into LDS in one strided,
  // coalesced pass (entry f of the concatenated walks on lane f mod 256),
  // then each walk runs from LDS, then the retrace values go back in a second
  // coalesced pass.  The same operations in the same order per walk; walks
  // whose entries exceed the staging space take the one-thread form below.
  constexpr int WCAP = 6144;
  __shared__ float w_v[WCAP], w_t[WCAP], w_r[WCAP];
  __shared__ unsigned short w_row[WCAP];
  __shared__ int s_woff[MB_META + 1], s_fk[MB_META], s_wsum[16];  // (one per wave, up to 1024 threads)
  __shared__ float s_wretn[MB_META];
  {
    // walking rows (the last mini-batch row of each episode): length, initial
    // value (into s_ret, read by the walk before the rows' values replace it)
    // and the old value of the entry after the walk's first (s_wretn); rows
    // [t per, (t + 1) per) on thread t
    const int per = (B + nt - 1) / nt;
    int cnt = 0, lmax = 0, lcnt = 0;
    for (int b = t * per; b < B && b < (t + 1) * per; b++) {
      const long long end = s_mb[b];
      const long long pe = ph(end), pn = ph(b < B - 1 ? (long long)s_mb[b + 1] : end), pnext = ph(end + 1);
      const long long epe = er.ep_id[pe], epn = er.ep_id[pn];
      const int pos = er.ep_pos[pe], term = u8v(s_term[b]);
      const float retn = er.ret[pnext];
      int L = 0;
      if (!(b < B - 1 && epe == epn)) {
        long long start = end - pos;
        if (start < 0) start = 0;
        float retV = 0.0f;
        if (term == TRUNCATED) retV = s_tv[b];
        if (term == NON_TERMINAL) retV = retn;
        s_ret[b] = retV, s_wretn[b] = retn;
        L = (int)(end - start + 1);
        lmax = max(lmax, L), lcnt++;
      }
      s_woff[b] = L;  // (lengths; offsets after the scan)
      cnt += L;
    }
    int inc = cnt;  // exclusive scan of the per-thread entry counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if ((t & 63) >= o) inc += y;
      lmax = max(lmax, __shfl_xor(lmax, o, 64));
      lcnt += __shfl_xor(lcnt, o, 64);
    }
    if ((t & 63) == 63) {
      s_wsum[t >> 6] = inc;
      atomicMax(&s_wmax, lmax);  // (walk statistics: one atomic per wave)
      atomicAdd(&s_wtot, inc);
      atomicAdd(&s_wcnt, lcnt);
    }
    __syncthreads();
    int ex = inc - cnt;
    for (int w = 0; w < (t >> 6); w++) ex += s_wsum[w];
    for (int b = t * per; b < B && b < (t + 1) * per; b++) {
      const int L = s_woff[b];
      s_woff[b] = ex;
      if (ex + L <= WCAP)
        for (int f = ex; f < ex + L; f++) w_row[f] = (unsigned short)b;
      ex += L;
    }
    if (t == nt - 1) s_woff[B] = ex;
    __syncthreads();
  }
  const int wtot = s_woff[B];
  const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long tw1 = tw0, tw2 = tw0;
  if (staged && wtot <= WCAP) {
    // entry f of walk b = w_row[f] is replay entry c = mb[b] - (f - off[b])
    // (sixteen entries' loads in flight per thread before its LDS stores)
    for (int f0 = t; f0 < wtot; f0 += 16 * nt) {
      float lv[16], lt[16], lr[16];
      int le[16];
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int f = f0 + u * nt;
        if (f < wtot) {
          const int b = u16v(w_row[f]);
          const long long q = ph((long long)s_mb[b] - (f - s_woff[b]));
          lv[u] = er.v[q], lt[u] = er.tiw[q], lr[u] = er.rew[q];
          if (RR) le[u] = er.env[q];
        }
      }
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int f = f0 + u * nt;
        if (f < wtot) {
          w_v[f] = lv[u], w_t[f] = lt[u];
          w_r[f] = RR ? lr[u] / (rsl ? s_rsig[le[u]] : er.rsig[le[u]]) : lr[u];  // getScaledReward (agent.cpp.base:720)
        }
      }
    }
    __syncthreads();
    // every mini-batch row's entry takes the values this kernel updated (the
    // walk then needs no per-entry check); s_fk: the entry, or -(walk + 1)
    // when it is the walk's first (its successor's value is the old one)
    for (int k = t; k < B; k += nt) {
      int wb = k;
      while (wb < B - 1 && s_woff[wb + 1] == s_woff[wb]) wb++;  // the walking row of k's episode
      const int f = s_woff[wb] + (int)((long long)s_mb[wb] - (long long)s_mb[k]);
      w_v[f] = s_V[k], w_t[f] = s_tiw[k];  // (duplicate rows store the same values)
      s_fk[k] = f == s_woff[wb] ? -(wb + 1) : f;
    }
    __syncthreads();
    tw1 = __builtin_amdgcn_s_memrealtime();
    const float g = P.gamma;
    for (int b = t; b < B; b += nt) {
      const int f0 = s_woff[b], f1 = s_woff[b + 1];
      float x = s_ret[b];
      int f = f0;
      for (; f + 4 <= f1; f += 4) {  // four entries' operands read ahead of the recurrence
        float vv[4], tw[4], rw[4];
#pragma unroll
        for (int j = 0; j < 4; j++) vv[j] = w_v[f + j], tw[j] = w_t[f + j], rw[j] = w_r[f + j];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          x = vv[j] + tw[j] * (rw[j] + g * x - vv[j]);
          w_v[f + j] = x;
        }
      }
      for (; f < f1; f++) {
        x = w_v[f] + w_t[f] * (w_r[f] + g * x - w_v[f]);
        w_v[f] = x;
      }
    }
    __syncthreads();
    tw2 = __builtin_amdgcn_s_memrealtime();
    for (int k = t; k < B; k += nt) {
      const int e = s_fk[k];
      if (e < 0) {
        const int wb = -e - 1;
        s_ret[k] = w_v[s_woff[wb]], s_retn[k] = s_wretn[wb];
      } else {
        s_ret[k] = w_v[e], s_retn[k] = w_v[e - 1];
      }
    }
    for (int f = t; f < wtot; f += nt) {
      const int b = u16v(w_row[f]);
      er.ret[ph((long long)s_mb[b] - (f - s_woff[b]))] = w_v[f];
    }
  } else {
    // the one-thread walks through the replay memory
    for (int b = t; b < B; b += nt) {
      const long long end = s_mb[b];
      const long long pe = ph(end), pn = ph(b < B - 1 ? (long long)s_mb[b + 1] : end), pnext = ph(end + 1);
      const long long epe = er.ep_id[pe], epn = er.ep_id[pn];
      const int pos = er.ep_pos[pe], term = u8v(s_term[b]);
      const float retn = er.ret[pnext];
      if (b < B - 1 && epe == epn) continue;
      long long start = end - pos;
      if (start < 0) start = 0;
      float retV = 0.0f;
      if (term == TRUNCATED) retV = s_tv[b];
      if (term == NON_TERMINAL) retV = retn;
      float prev = retn;  // retrace value of the entry after the current one
      int k = b;          // mini-batch rows of this episode, walked downwards
      // per chunk: inputs loaded and mini-batch overrides applied first (no
      // dependence on the recurrence), then the recurrence alone (4 dependent
      // float operations per entry), then the mini-batch rows' values to LDS.
      // The next chunk's loads are issued before the current chunk's
      // recurrence (two register sets: 48 loads in flight behind the awaited
      // ones, inside the 63 of vmcnt), so the latency of the replay memory's
      // loads overlaps the previous chunk's recurrence (without the prefetch:
      // 27 us per update at C5)
      constexpr int RC = VR_RC;
      // (unconditional: entries past the chunk or the episode are valid slots
      // of the ring whose values go unused; no branch splits the loads from
      // the waits, so those stay counted)
      int ea[RC], eb[RC];  // (RR: the entries' environment ids)
      // (a chunk that does not wrap around the ring, the common case, is
      // addressed from one base with constant offsets: no per-entry 64-bit
      // wrap arithmetic in this single-wave, instruction-bound walk)
      auto load = [&](long long p0, float (&vv)[RC], float (&tw)[RC], float (&rw)[RC], int (&en)[RC])
                      __attribute__((always_inline)) {
        if (p0 >= RC - 1) {
          const float *v = er.v + p0, *w = er.tiw + p0, *r = er.rew + p0;
          const int *ev = er.env + p0;
  #pragma unroll
          for (int j = 0; j < RC; j++) {
            vv[j] = v[-j], tw[j] = w[-j], rw[j] = r[-j];
            if (RR) en[j] = ev[-j];
          }
        } else {
          long long q = p0;
  #pragma unroll
          for (int j = 0; j < RC; j++) {
            vv[j] = er.v[q], tw[j] = er.tiw[q], rw[j] = er.rew[q];
            if (RR) en[j] = er.env[q];
            q = q == 0 ? (long long)R - 1 : q - 1;
          }
        }
      };
      auto process = [&](long long c, long long p0, float (&vv)[RC], float (&tw)[RC], float (&rw)[RC],
                         const int (&en)[RC]) __attribute__((always_inline)) {
        if (RR)
  #pragma unroll
          for (int j = 0; j < RC; j++) rw[j] = rw[j] / (rsl ? s_rsig[en[j]] : er.rsig[en[j]]);  // getScaledReward (agent.cpp.base:720)
        const int n = (int)min((long long)RC, c - start + 1);
        int kk = k;
        unsigned long long inmb = 0;
        // the highest mini-batch row not yet passed is <= c: only when it lies
        // in this chunk (rare: B rows over the whole memory) are the entries
        // checked one by one (each check a dependent LDS read)
        if (kk >= 0 && (long long)s_mb[kk] > c - n)
  #pragma unroll
          for (int j = 0; j < RC; j++)
            if (j < n && kk >= 0 && (long long)s_mb[kk] == c - j) {
              vv[j] = s_V[kk], tw[j] = s_tiw[kk];  // updated by this kernel
              inmb |= 1ull << j;
              while (kk >= 0 && (long long)s_mb[kk] == c - j) kk--;
            }
        float rr[RC];
        const float g = P.gamma;
        if (n == RC) {  // a full chunk: no per-entry predicate
  #pragma unroll
          for (int j = 0; j < RC; j++) rr[j] = retV = vv[j] + tw[j] * (rw[j] + g * retV - vv[j]);
        } else {
  #pragma unroll
          for (int j = 0; j < RC; j++)
            if (j < n) rr[j] = retV = vv[j] + tw[j] * (rw[j] + g * retV - vv[j]);
        }
        if (n == RC && p0 >= RC - 1) {
          float *rp = er.ret + p0;
  #pragma unroll
          for (int j = 0; j < RC; j++) rp[-j] = rr[j];
        } else {
          long long q = p0;
  #pragma unroll
          for (int j = 0; j < RC; j++) {
            if (j < n) er.ret[q] = rr[j];
            q = q == 0 ? (long long)R - 1 : q - 1;
          }
        }
        if (inmb)
  #pragma unroll
          for (int j = 0; j < RC; j++)
            if (inmb >> j & 1ull) {
              const float before = j == 0 ? prev : rr[j - 1];
              while (k >= 0 && (long long)s_mb[k] == c - j) s_ret[k] = rr[j], s_retn[k] = before, k--;
            }
        prev = retV;  // the chunk's last entry
      };
      // the chunk after the one at (c, pc): its first entry and physical slot
      auto next = [&](long long c, long long pc, long long &c1, long long &pc1) __attribute__((always_inline)) {
        const long long n = min((long long)RC, c - start + 1);
        c1 = c - n;
        pc1 = pc >= n ? pc - n : pc - n + (long long)R;
      };
      float av[RC], at[RC], ar[RC], bv[RC], bt[RC], br[RC];
      long long c = end, pc = ph(end);
      load(pc, av, at, ar, ea);
      while (c >= start) {
        long long c1, pc1;
        next(c, pc, c1, pc1);
        load(pc1, bv, bt, br, eb);
        process(c, pc, av, at, ar, ea);
        c = c1, pc = pc1;
        if (c < start) break;
        next(c, pc, c1, pc1);
        load(pc1, av, at, ar, ea);
        process(c, pc, bv, bt, br, eb);
        c = c1, pc = pc1;
      }
    }
  }
  __syncthreads();
  const unsigned long long tm2 = __builtin_amdgcn_s_memrealtime();
  // ---- the VRACER loss gradient (VRACER.cpp.base:104-177), all from LDS;
  // then the replay memory's metadata (first occurrences)
  const float klm = -(1.0f - beta);
  const int A = P.A;
  for (int b = t; b < B; b += nt) {
    const long long p = ph(s_mb[b]);
    // action component i of row b: the stored action, the current policy (the
    // forward's output) and the experience's policy; one component from LDS
    auto comp = [&](int i, float &a, float &cm, float &cs, float &om, float &osd) __attribute__((always_inline)) {
      if (A == 1) {
        a = s_act[b], cm = s_cur[2 * b], cs = s_cur[2 * b + 1], om = s_old[2 * b], osd = s_old[2 * b + 1];
      } else {
        a = er.act[p * A + i], cm = out[(long long)b * O + 1 + i], cs = out[(long long)b * O + 1 + A + i];
        om = er.exp_pol[p * 2 * A + i], osd = er.exp_pol[p * 2 * A + A + i];
      }
    };
    const float V = s_V[b];
    const int term = u8v(s_term[b]);
    // (means and sigmas in separate register arrays: every index a
    // compile-time constant, no indexed register access)
    float gm[MAXA], gs[MAXA];
#pragma unroll
    for (int i = 0; i < MAXA; i++) gm[i] = gs[i] = 0.f;
    const float g0 = s_ret[b] - V;
    if (u8v(s_onp[b])) {
      float q = s_rew[b];
      if (term == NON_TERMINAL) q += P.gamma * s_retn[b];
      if (term == TRUNCATED) q += P.gamma * s_tv[b];
      const float loss = q - V;
      // calculateImportanceWeightGradient: per component the factors, the
      // log-densities summed in component order, then the weight
      float pm[MAXA], ps[MAXA], lcs = 0.0f, los = 0.0f;
#pragma unroll
      for (int i = 0; i < MAXA; i++)
        if (i < A) {
          float a, cm, cs, om, osd, lc, lo;
          comp(i, a, cm, cs, om, osd);
          iw_grad_terms(P, i, a, cm, cs, om, osd, pm[i], ps[i], lc, lo);
          lcs += lc;
          los += lo;
        }
      const float iwg = expf(lcs - los);
#pragma unroll
      for (int i = 0; i < MAXA; i++)
        if (i < A) {
          gm[i] = beta * loss * (pm[i] * iwg);
          gs[i] = beta * loss * (ps[i] * iwg);
        }
    }
#pragma unroll
    for (int i = 0; i < MAXA; i++)
      if (i < A) {
        float a, cm, cs, om, osd, km, ks;
        comp(i, a, cm, cs, om, osd);
        kl_grad_terms(P, i, cm, cs, om, osd, km, ks);
        gm[i] += klm * km;
        gs[i] += klm * ks;
      }
    unsigned bad = !isfinite(g0);
    G[(long long)b * O] = g0;
#pragma unroll
    for (int i = 0; i < MAXA; i++)
      if (i < A) {
        bad |= !isfinite(gm[i]) | !isfinite(gs[i]);
        G[(long long)b * O + 1 + i] = gm[i];
        G[(long long)b * O + 1 + A + i] = gs[i];
      }
    if (bad) atomicOr(&st->errors, (unsigned)ERR_NONFINITE_GRADIENT);
    if (u8v(s_uniq[b])) {
#pragma unroll
      for (int i = 0; i < MAXA; i++)
        if (i < A) {
          float a, cm, cs, om, osd;
          comp(i, a, cm, cs, om, osd);
          er.cur_pol[p * 2 * A + i] = cm, er.cur_pol[p * 2 * A + A + i] = cs;
        }
      er.v[p] = V;
      er.tv[p] = s_tv[b];
      er.iw[p] = s_iw[b];
      er.onp[p] = s_onp[b];
      er.tiw[p] = s_tiw[b];
    }
  }
  __syncthreads();
  if (t == 0) {
    const unsigned long long tm3 = __builtin_amdgcn_s_memrealtime();
    st->mtr[0] += tm1 - tm0, st->mtr[1] += tm2 - tm1, st->mtr[2] += tm3 - tm2;
    st->mtr[3] += (unsigned long long)s_wmax, st->mtr[4] += (unsigned long long)s_wtot, st->mtr[5] += (unsigned long long)s_wcnt;
    st->mtr[6] += tw0 - tm1, st->mtr[7] += tw1 - tw0, st->mtr[8] += tw2 - tw1;
    st->off_count = off1;
    st->off_ratio = off_ratio;
    st->mb_counter += advance;  // (the draws of a fused forward's mini-batch)
    st->cutoff = P.cutoff_scale / (1.0f + P.anneal * (float)upd0);
    // the learner's eta for this update, then agent.cpp.base:221-231
    st->eta = lr;
    st->b1p = b1p * 0.9f;
    st->b2p = b2p * 0.999f;
    st->update_count = upd0 + 1;
    const float lr1 = P.lr0 / (1.0f + P.anneal * (float)(upd0 + 1));
    st->lr = lr1;
    if (off_ratio > P.off_target) st->beta = (1.0f - lr1) * beta;
    else st->beta = (1.0f - lr1) * beta + lr1;
  }
}

// ---------------------------------------------------------------- CartPole
// examples/learning/reinforcement/cartpole/_model/cartpole.py (advance: scipy
// ode 'dopri5' from t to t + 0.02, restated below) and env.py (3 reward
// variants, reset seeded with numpy's legacy mt19937 by sampleId*1024 + launchId).
// cartpole.py:37-46 in its operation order (w**2 and costh**2 squared first)
__device__ inline void cp_system(const double *y, double act, double *d) {
  const double mp = 0.1, mc = 1.0, l = 0.5, g = 9.81;
  const double th = y[2], w = y[3];
  const double c = cos(th), s = sin(th);
  const double tot = mp + mc;
  const double tmp = (act + l * (w * w) * s) / tot;
  const double wdot = (g * s - c * tmp) / (l * (4.0 / 3.0 - mp * (c * c) / tot));
  const double vdot = tmp - l * wdot * c / tot;
  d[0] = y[1], d[1] = vdot, d[2] = w, d[3] = wdot;
}

// scipy.integrate.ode 'dopri5' = Hairer & Wanner's DOPRI5 (Dormand-Prince
// 5(4)) as scipy calls it for one integrate(): rtol 1e-6, atol 1e-12 (ITOL 0),
// UROUND 2.3e-16, SAFE 0.9, FAC1 0.2, FAC2 10, BETA 0.04 (scipy's beta 0 ->
// the code's default), HMAX = XEND - X, first step from HINIT, at most 500
// steps, no dense output; stiffness detection only prints and is left out.
// Fortran's left-to-right order term by term (oracle/vracer_ref.py
// dopri5_advance, bit-exact against the reference's own trajectories in
// tests/golden/cartpole_dopri5.json).  Returns false past NMAX or a vanishing
// step (scipy reports those as failures).
namespace dp {
constexpr double C2 = 0.2, C3 = 0.3, C4 = 0.8, C5 = 8.0 / 9.0, A21 = 0.2;
constexpr double A31 = 3.0 / 40.0, A32 = 9.0 / 40.0;
constexpr double A41 = 44.0 / 45.0, A42 = -56.0 / 15.0, A43 = 32.0 / 9.0;
constexpr double A51 = 19372.0 / 6561.0, A52 = -25360.0 / 2187.0, A53 = 64448.0 / 6561.0, A54 = -212.0 / 729.0;
constexpr double A61 = 9017.0 / 3168.0, A62 = -355.0 / 33.0, A63 = 46732.0 / 5247.0, A64 = 49.0 / 176.0,
                 A65 = -5103.0 / 18656.0;
constexpr double A71 = 35.0 / 384.0, A73 = 500.0 / 1113.0, A74 = 125.0 / 192.0, A75 = -2187.0 / 6784.0,
                 A76 = 11.0 / 84.0;
constexpr double E1 = 71.0 / 57600.0, E3 = -71.0 / 16695.0, E4 = 71.0 / 1920.0, E5 = -17253.0 / 339200.0,
                 E6 = 22.0 / 525.0, E7 = -1.0 / 40.0;
constexpr double RTOL = 1e-6, ATOL = 1e-12, UROUND = 2.3e-16, SAFE = 0.9, FAC1 = 0.2, FAC2 = 10.0, BETA = 0.04;
constexpr int NMAX = 500;
}  // namespace dp

__device__ inline bool cp_dopri5(double *y, double x, double xend, double F) {
  using namespace dp;
  double k1[4], k2[4], k3[4], k4[4], k5[4], k6[4], y1[4], ys[4];
  const double expo1 = 0.2 - BETA * 0.75, facc1 = 1.0 / FAC1, facc2 = 1.0 / FAC2;
  double facold = 1.0e-4;
  const double hmax = fabs(xend - x);
  cp_system(y, F, k1);
  double h;
  {  // HINIT
    double dnf = 0.0, dny = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const double sk = ATOL + RTOL * fabs(y[i]);
      const double a = k1[i] / sk, b = y[i] / sk;
      dnf = dnf + a * a;
      dny = dny + b * b;
    }
    h = (dnf <= 1.0e-10 || dny <= 1.0e-10) ? 1.0e-6 : sqrt(dny / dnf) * 0.01;
    h = fmin(h, hmax);
#pragma unroll
    for (int i = 0; i < 4; i++) y1[i] = y[i] + h * k1[i];
    cp_system(y1, F, k2);
    double der2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const double sk = ATOL + RTOL * fabs(y[i]);
      const double a = (k2[i] - k1[i]) / sk;
      der2 = der2 + a * a;
    }
    der2 = sqrt(der2) / h;
    const double der12 = fmax(fabs(der2), sqrt(dnf));
    const double h1 = der12 <= 1.0e-15 ? fmax(1.0e-6, fabs(h) * 1.0e-3) : pow(0.01 / der12, 1.0 / 5);
    h = fmin(fmin(100 * fabs(h), h1), hmax);
  }
  bool last = false, reject = false;
  for (int nstep = 0;; nstep++) {
    if (nstep > NMAX || 0.1 * fabs(h) <= fabs(x) * UROUND) return false;
    if ((x + 1.01 * h - xend) > 0.0) {
      h = xend - x;
      last = true;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) y1[i] = y[i] + h * A21 * k1[i];
    cp_system(y1, F, k2);
#pragma unroll
    for (int i = 0; i < 4; i++) y1[i] = y[i] + h * (A31 * k1[i] + A32 * k2[i]);
    cp_system(y1, F, k3);
#pragma unroll
    for (int i = 0; i < 4; i++) y1[i] = y[i] + h * (A41 * k1[i] + A42 * k2[i] + A43 * k3[i]);
    cp_system(y1, F, k4);
#pragma unroll
    for (int i = 0; i < 4; i++) y1[i] = y[i] + h * (A51 * k1[i] + A52 * k2[i] + A53 * k3[i] + A54 * k4[i]);
    cp_system(y1, F, k5);
#pragma unroll
    for (int i = 0; i < 4; i++) ys[i] = y[i] + h * (A61 * k1[i] + A62 * k2[i] + A63 * k3[i] + A64 * k4[i] + A65 * k5[i]);
    const double xph = x + h;
    cp_system(ys, F, k6);
#pragma unroll
    for (int i = 0; i < 4; i++) y1[i] = y[i] + h * (A71 * k1[i] + A73 * k3[i] + A74 * k4[i] + A75 * k5[i] + A76 * k6[i]);
    cp_system(y1, F, k2);
    double err = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const double e = (E1 * k1[i] + E3 * k3[i] + E4 * k4[i] + E5 * k5[i] + E6 * k6[i] + E7 * k2[i]) * h;
      const double sk = ATOL + RTOL * fmax(fabs(y[i]), fabs(y1[i]));
      const double q = e / sk;
      err = err + q * q;
    }
    err = sqrt(err / 4);
    const double fac11 = pow(err, expo1);
    const double fac = fmax(facc2, fmin(facc1, (fac11 / pow(facold, BETA)) / SAFE));
    double hnew = h / fac;
    if (err <= 1.0) {
      facold = fmax(err, 1.0e-4);
#pragma unroll
      for (int i = 0; i < 4; i++) k1[i] = k2[i], y[i] = y1[i];
      x = xph;
      if (last) return true;
      if (fabs(hnew) > hmax) hnew = hmax;
      if (reject) hnew = fmin(fabs(hnew), fabs(h));
      reject = false;
    } else {
      hnew = h / fmin(facc1, fac11 / SAFE);
      reject = true;
      last = false;
    }
    h = hnew;
  }
}

// CartPole::advance (cartpole.py:48-62): F clipped to [-10, 10], the ODE
// from the environment's time t to t + dt, then t += dt
__device__ inline bool cp_advance(double *u, double &t, double action) {
  double F = action;
  if (F > 10.0) F = 10.0;
  else if (F < -10.0) F = -10.0;
  const bool ok = cp_dopri5(u, t, t + 0.02, F);
  t = t + 0.02;
  return ok;
}
__device__ inline bool cp_failed(const double *u) {
  return fabs(u[0]) > 2.4 || fabs(u[2]) > M_PI / 15;
}
// numpy RandomState(seed).uniform(-0.05, 0.05, 4): init_genrand, one twist of
// the first 8 words, tempering, random_double = (a>>5, b>>6) / 2^53.
//
// Every private-array index here is a compile-time constant (unrolled
// loops): a runtime-indexed write inside the 405-step recurrence (the
// round-2 form, `if (i <= 8) lo[i] = x`) was if-converted by the compiler
// into an unconditional VGPR-indexed write v[base + i] with i up to 404 —
// far past the array — which corrupted other registers and memory-faulted
// on MI355X.
__device__ inline void cp_reset(unsigned seed, double *u) {
  unsigned lo[9], hi[8];
  unsigned x = seed;
  lo[0] = x;
#pragma unroll
  for (int i = 1; i <= 8; i++) {
    x = 1812433253u * (x ^ (x >> 30)) + (unsigned)i;
    lo[i] = x;
  }
  for (int i = 9; i < 397; i++) x = 1812433253u * (x ^ (x >> 30)) + (unsigned)i;
#pragma unroll
  for (int i = 397; i <= 404; i++) {
    x = 1812433253u * (x ^ (x >> 30)) + (unsigned)i;
    hi[i - 397] = x;
  }
  unsigned out[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const unsigned y = (lo[i] & 0x80000000u) | (lo[i + 1] & 0x7fffffffu);
    unsigned z = hi[i] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    z ^= z >> 11;
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= z >> 18;
    // opaque to the optimiser: the later >> 5 / >> 6 stay plain shifts (the
    // SDWA peephole otherwise folds (z >> 24) into a byte-select v_xor_b32_sdwa;
    // such a build of this kernel memory-faulted on MI355X in round 2, see
    // DESIGN.md section 9)
    asm volatile("" : "+v"(z));
    out[i] = z;
  }
  const double low = -0.05, range = 0.05 - -0.05;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const double d = ((double)(out[2 * k] >> 5) * 67108864.0 + (double)(out[2 * k + 1] >> 6)) / 9007199254740992.0;
    u[k] = low + range * d;
  }
}

struct Envs {
  double *u;          // E x 4 CartPole state
  double *time;       // E: the CartPole's ODE time t (cartpole.py: reset to 0, += dt per advance)
  int *t, *env_id;    // steps taken in the episode, environment id
  unsigned long long *sample;
  float *cum;         // cumulative training reward of the running episode
  int *fin, *len;     // finished flag (termination) and episode length after the step
  long long *off;     // exclusive prefix of finished lengths
  int *rank;          // rank of the finished episode in environment order
  int *fin_env;       // environment of the finished episode of each rank
  float *eb_st, *eb_act, *eb_pol, *eb_v, *eb_rew;  // E x T episode buffers
  float *rewards;     // cumulative rewards of the episodes finished by the last step (by rank)
  float *sig2;        // rank x 2: the rescaling sigmas of the episode's id and of the entry before it, before its update
  int *fin_id;        // environment id of the finished episode of each rank
  float *pm, *ps;     // E x S: the state-rescaling moments the running episode was launched with
  float *hraw;        // E x S: a host environment's raw launch state (State Rescaling re-scales it)
};
// requestNewPolicy's normalisation (reinforcementLearning.cpp.base:361-370)
// of environment e's state component k
__device__ __forceinline__ float vr_scale_state(const Params &P, const Envs &ev, int e, int k, double y) {
  const float x = (float)y;
  return P.srs ? (x - ev.pm[e * P.S + k]) / ev.ps[e * P.S + k] : x;
}

__global__ void k_vr_env_reset(Params P, const State *st, Envs ev, float *X, unsigned long long sample0,
                               const int *only_fin) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.E) return;
  const unsigned long long sid = sample0 + e;
  double u[4];
  cp_reset((unsigned)(sid * 1024ull + sid), u);
  if (P.srs)
    for (int k = 0; k < P.S; k++) ev.pm[e * P.S + k] = st->smean[k], ev.ps[e * P.S + k] = st->ssdev[k];
  for (int k = 0; k < 4; k++) ev.u[e * 4 + k] = u[k], X[e * 4 + k] = vr_scale_state(P, ev, e, k, u[k]);
  ev.time[e] = 0.0;
  ev.t[e] = 0;
  ev.sample[e] = sid;
  ev.env_id[e] = (int)(sid % (unsigned long long)P.env_count);
  ev.cum[e] = 0.f;
  (void)only_fin;
}

// Testing episodes (Agent::testingGeneration, agent.cpp.base:267-289;
// ReinforcementLearning::runTestingEpisode, reinforcementLearning.cpp.base:
// 207-255): episode j resets CartPole with seed sample_id * 1024 + launch_id
// (env.py), takes the policy's mode as the action (generateTestingAction,
// continuous.cpp.base:219-260: the Normal mean; Clipped Normal: the mean
// clipped to the bounds), and adds the reward of environment 0 (env.py:
// testing runs environment 0) until the pole falls or max_episode_steps.
// (testing agents take the agent's State Rescaling moments, agent.cpp.base:279-280,
// and always rescale, reinforcementLearning.cpp.base:361-370: with the
// defaults 0 / 1 that is the identity)
__device__ __forceinline__ float vr_test_state(const Params &P, const State *st, int k, double y) {
  const float x = (float)y;
  (void)P;
  return (x - st->smean[k]) / st->ssdev[k];
}
__global__ void k_vr_test_reset(Params P, const State *st, int n, int S, const unsigned long long *__restrict__ sid,
                                const unsigned long long *__restrict__ lid, double *u, double *tm, int *steps,
                                int *done, float *cum, float *X) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  double y[4];
  cp_reset((unsigned)(sid[e] * 1024ull + lid[e]), y);
  for (int k = 0; k < 4; k++) u[e * 4 + k] = y[k], X[e * S + k] = vr_test_state(P, st, k, y[k]);
  tm[e] = 0.0;
  steps[e] = 0;
  done[e] = 0;
  cum[e] = 0.f;
}
__global__ void k_vr_test_act(Params P, const State *st, int n, const float *__restrict__ out, double *u, double *tm,
                              int *steps, int *done, float *cum, float *X, unsigned *errors, int *running) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n || done[e]) return;
  float act = out[(long long)e * P.O + 1];  // the mode (A = 1: the CartPole kernel)
  if (P.clipped) {
    if (act >= P.ub[0]) act = P.ub[0];
    if (act <= P.lb[0]) act = P.lb[0];
  }
  double y[4];
#pragma unroll
  for (int k = 0; k < 4; k++) y[k] = u[e * 4 + k];
  double t = tm[e];
  if (!cp_advance(y, t, (double)act)) atomicOr(errors, (unsigned)ERR_ENV_ODE);
  tm[e] = t;
#pragma unroll
  for (int k = 0; k < 4; k++) u[e * 4 + k] = y[k], X[e * P.S + k] = vr_test_state(P, st, k, y[k]);
  const bool failed = cp_failed(y);
  cum[e] += (float)(1.0 - 1.0 * (failed ? 1.0 : 0.0));
  const int ns = steps[e] + 1;
  steps[e] = ns;
  if (failed || ns >= P.T) done[e] = 1;
  else atomicAdd(running, 1);
}

// One action of every environment (continuous.cpp.base:95-150 Normal policy:
// action = mean + sigma N(0,1)); the experience is kept in the episode buffer.
__global__ void k_vr_env_act(Params P, State *st, Envs ev, const float *__restrict__ out, float *X,
                             const float *__restrict__ forced_noise) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.E) return;
  const int A = P.A, S = P.S, O = P.O;
  const int t = ev.t[e];
  const long long slot = (long long)e * P.T + t;
  const float V = out[(long long)e * O];
  float act[MAXA];
  for (int i = 0; i < A; i += 2) {
    float n0, n1;
    if (forced_noise) {
      n0 = forced_noise[e * A + i];
      n1 = i + 1 < A ? forced_noise[e * A + i + 1] : 0.f;
    } else {
      philox_normals(P.seed, 0x4E4Fu, st->env_step, (unsigned)(e * MAXA + i), n0, n1);
    }
    act[i] = out[(long long)e * O + 1 + i] + out[(long long)e * O + 1 + A + i] * n0;
    if (i + 1 < A) act[i + 1] = out[(long long)e * O + 2 + i] + out[(long long)e * O + 2 + A + i] * n1;
  }
  if (P.clipped)  // continuous.cpp.base:172-183
    for (int i = 0; i < A; i++) {
      if (act[i] >= P.ub[i]) act[i] = P.ub[i];
      if (act[i] <= P.lb[i]) act[i] = P.lb[i];
    }
  for (int k = 0; k < S; k++) ev.eb_st[slot * S + k] = X[(long long)e * S + k];
  for (int i = 0; i < A; i++) ev.eb_act[slot * A + i] = act[i];
  for (int i = 0; i < 2 * A; i++) ev.eb_pol[slot * 2 * A + i] = out[(long long)e * O + 1 + i];
  ev.eb_v[slot] = V;
  double y[4];
#pragma unroll
  for (int k = 0; k < 4; k++) y[k] = ev.u[e * 4 + k];
  double tm = ev.time[e];
  if (!cp_advance(y, tm, (double)act[0])) atomicOr(&st->errors, (unsigned)ERR_ENV_ODE);
  ev.time[e] = tm;
#pragma unroll
  for (int k = 0; k < 4; k++) ev.u[e * 4 + k] = y[k], X[e * 4 + k] = vr_scale_state(P, ev, e, k, y[k]);
  const bool failed = cp_failed(y);
  const double r = 1.0 - 1.0 * (failed ? 1.0 : 0.0);
  const int vid = ev.env_id[e] % 3;
  const float rew = (float)(vid == 0 ? r : vid == 1 ? r - 1.0 : r * 0.1);
  ev.eb_rew[slot] = rew;
  ev.cum[e] += rew;
  const int steps = t + 1;
  ev.t[e] = steps;
  ev.len[e] = steps;
  ev.fin[e] = failed ? TERMINAL : (steps >= P.T ? TRUNCATED : NON_TERMINAL);
}

// ---- host-fed environments (a user 'Environment Function',
// reinforcementLearning.cpp.base:58-83, :276-340).  The engine runs each
// environment's function as a coroutine (a thread handing control back and
// forth at Sample::update); the device keeps the policy, the episode buffers
// and the replay memory exactly as for the CartPole kernel, only the state
// transitions come from the host.
//
// the first launch of every environment: its initial state (raw, rescaled
// here with the moments it is launched with) and its Environment Id
__global__ void k_vr_host_launch(Params P, const State *st, Envs ev, float *X, const float *__restrict__ states,
                                 const int *__restrict__ env_ids) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.E) return;
  if (P.srs)
    for (int k = 0; k < P.S; k++) ev.pm[e * P.S + k] = st->smean[k], ev.ps[e * P.S + k] = st->ssdev[k];
  for (int k = 0; k < P.S; k++) {
    const float x = states[(long long)e * P.S + k];
    ev.hraw[(long long)e * P.S + k] = x;
    X[(long long)e * P.S + k] = vr_scale_state(P, ev, e, k, x);
  }
  ev.t[e] = 0;
  ev.sample[e] = (unsigned long long)e;
  ev.env_id[e] = env_ids[e];
  ev.cum[e] = 0.f;
}

// the policy's action for every environment's current state (as the first
// half of k_vr_env_act: continuous.cpp.base:95-150), the experience kept in
// the episode buffer and the action handed to the host
__global__ void k_vr_host_act(Params P, State *st, Envs ev, const float *__restrict__ out, const float *__restrict__ X,
                              const float *__restrict__ forced_noise, float *__restrict__ actions) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.E) return;
  const int A = P.A, S = P.S, O = P.O;
  const int t = ev.t[e];
  if (t >= P.T) {  // (k_vr_host_feed flags it; nothing is stored past the buffer)
    for (int i = 0; i < A; i++) actions[e * A + i] = 0.f;
    return;
  }
  const long long slot = (long long)e * P.T + t;
  float act[MAXA];
  for (int i = 0; i < A; i += 2) {
    float n0, n1;
    if (forced_noise) {
      n0 = forced_noise[e * A + i];
      n1 = i + 1 < A ? forced_noise[e * A + i + 1] : 0.f;
    } else {
      philox_normals(P.seed, 0x4E4Fu, st->env_step, (unsigned)(e * MAXA + i), n0, n1);
    }
    act[i] = out[(long long)e * O + 1 + i] + out[(long long)e * O + 1 + A + i] * n0;
    if (i + 1 < A) act[i + 1] = out[(long long)e * O + 2 + i] + out[(long long)e * O + 2 + A + i] * n1;
  }
  if (P.clipped)  // continuous.cpp.base:172-183
    for (int i = 0; i < A; i++) {
      if (act[i] >= P.ub[i]) act[i] = P.ub[i];
      if (act[i] <= P.lb[i]) act[i] = P.lb[i];
    }
  for (int k = 0; k < S; k++) ev.eb_st[slot * S + k] = X[(long long)e * S + k];
  for (int i = 0; i < A; i++) ev.eb_act[slot * A + i] = act[i], actions[e * A + i] = act[i];
  for (int i = 0; i < 2 * A; i++) ev.eb_pol[slot * 2 * A + i] = out[(long long)e * O + 1 + i];
  ev.eb_v[slot] = out[(long long)e * O];
}

// what each environment returned for its action: reward, state after it
// (raw; for an episode that ended, its last state: the truncated state),
// termination (0 non terminal, 1 terminal, 2 truncated) -- the second half
// of k_vr_env_act
__global__ void k_vr_host_feed(Params P, State *st, Envs ev, float *X, const float *__restrict__ rewards,
                               const float *__restrict__ states, const int *__restrict__ terms) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.E) return;
  const int t = ev.t[e];
  if (t >= P.T) {
    atomicOr(&st->errors, (unsigned)ERR_EPISODE_LONG);
    ev.fin[e] = NON_TERMINAL;
    return;
  }
  const long long slot = (long long)e * P.T + t;
  const float rew = rewards[e];
  ev.eb_rew[slot] = rew;
  ev.cum[e] += rew;
  for (int k = 0; k < P.S; k++) X[(long long)e * P.S + k] = vr_scale_state(P, ev, e, k, states[(long long)e * P.S + k]);
  const int steps = t + 1;
  ev.t[e] = steps;
  ev.len[e] = steps;
  const int term = terms[e];
  ev.fin[e] = term == 1 ? TERMINAL : (term == 2 ? TRUNCATED : NON_TERMINAL);
}

// Finished episodes in environment order (the order attendAgent visits them):
// exclusive prefix of their lengths, ranks, and the scalar bookkeeping.
__global__ __launch_bounds__(1024) void k_vr_scan(Params P, State *st, Envs ev) {
  __shared__ long long s_len[1024];
  __shared__ int s_cnt[1024];
  const int t = threadIdx.x, nt = blockDim.x, E = P.E;
  const int per = (E + nt - 1) / nt, e0 = t * per, e1 = min(E, e0 + per);
  long long L = 0;
  int c = 0;
  for (int e = e0; e < e1; e++)
    if (ev.fin[e]) L += ev.len[e], c++;
  s_len[t] = L, s_cnt[t] = c;
  __syncthreads();
  for (int d = 1; d < nt; d <<= 1) {  // inclusive Hillis-Steele scan
    long long lv = t >= d ? s_len[t - d] : 0;
    int cv = t >= d ? s_cnt[t - d] : 0;
    __syncthreads();
    s_len[t] += lv, s_cnt[t] += cv;
    __syncthreads();
  }
  L = s_len[t] - L, c = s_cnt[t] - c;
  for (int e = e0; e < e1; e++) {
    ev.off[e] = L;
    ev.rank[e] = c;
    if (ev.fin[e]) ev.fin_env[c] = e, L += ev.len[e], c++;
  }
  if (t == nt - 1) {
    const unsigned long long add = (unsigned long long)s_len[nt - 1], neps = (unsigned long long)s_cnt[nt - 1];
    st->step_base = st->total;
    st->step_new = add;
    st->step_episodes = neps;
    st->step_episode_base = st->episode;
    st->step_sample_base = st->sample_id;
    st->total += add;
    st->size = st->size + add < (unsigned long long)P.R ? st->size + add : (unsigned long long)P.R;
    st->episode += neps;
    st->sample_id += neps;
    st->experience_count += add;
    st->env_step += 1;
    st->step_reward_sum = 0.0;
  }
}

// Eviction accounting of this step's appends (agent.cpp.base:504-506: an
// evicted off-policy experience decrements the off-policy count), before any
// new entry is written: the new offsets j < min(new, R) overwrite the slots
// of the old occupants base + j - R (those >= 0); offsets j >= R overwrite
// entries of this same batch, which are on-policy.  One workgroup, one
// atomic per thread.
__global__ __launch_bounds__(256) void k_vr_evict(Params P, State *st, Replay er) {
  const unsigned long long base = st->step_base, nnew = st->step_new;
  const long long R = P.R, cnt = (long long)(nnew < (unsigned long long)R ? nnew : (unsigned long long)R);
  unsigned long long evicted = 0;
  for (long long j = threadIdx.x; j < cnt; j += blockDim.x) {
    const long long prev = (long long)base + j - R;
    if (prev >= 0 && er.onp[((long long)base + j) % R] == 0) evicted++;
  }
  if (evicted) atomicAdd((unsigned long long *)&st->off_count, (unsigned long long)(-(long long)evicted));
}

// Reward rescaling's bookkeeping (agent.cpp.base:423-437, :557-563) for this
// step's finished episodes in processEpisode order, one thread (the sums
// are sequential float sums, as the reference's): per experience the new
// reward's square in and, with the memory full, the evicted one's out; per
// episode the sigmas before it (its initial retrace values use them) and
// after it.  Runs before k_vr_append overwrites the evicted slots; only
// when rescaling is enabled (the sums only feed the sigmas).
__device__ inline float rr_sigma(float sum, long long cnt) {
  return (float)(sqrt((double)sum / ((double)(float)cnt + 1e-9)) + 1e-9);
}
__global__ void k_vr_reward_sums(Params P, State *st, Replay er, Envs ev) {
  if (threadIdx.x || blockIdx.x) return;
  const unsigned long long base = st->step_base, neps = st->step_episodes;
  const long long R = P.R;
  const int EC = P.env_count;
  // (LDS, not registers: the environment id indexes them; more ids than
  // MAXENV work on the replay memory's tables in place)
  __shared__ float ssum[MAXENV], ssig[MAXENV];
  __shared__ long long scnt[MAXENV];
  const bool lds = EC <= MAXENV;
  float *sum = lds ? ssum : er.rsum, *sig = lds ? ssig : er.rsig;
  long long *cnt = lds ? scnt : er.rcnt;
  if (lds)
    for (int i = 0; i < EC; i++) sum[i] = er.rsum[i], cnt[i] = er.rcnt[i], sig[i] = er.rsig[i];
  // the batch entry at offset j (episodes in rank order): a forward cursor
  int cr = 0;
  long long cend = neps ? ev.len[ev.fin_env[0]] : 0, cbeg = 0;
  // the id of the new entry's evicted predecessor (memory full), or -1
  auto evicted = [&](long long a, float &ro) -> int {
    if (a < R) return -1;
    const long long old = a - R;
    if (old >= (long long)base) {  // an entry of this same batch
      const long long j = old - (long long)base;
      while (j >= cend) {
        cr++;
        cbeg = cend;
        cend += ev.len[ev.fin_env[cr]];
      }
      const int eo = ev.fin_env[cr];
      ro = ev.eb_rew[(long long)eo * P.T + (j - cbeg)];
      return ev.env_id[eo];
    }
    ro = er.rew[old % R];
    return er.env[old % R];
  };
  for (unsigned long long r = 0; r < neps; r++) {
    const int e = ev.fin_env[r], id = ev.env_id[e], len = ev.len[e];
    const long long off = ev.off[e];
    ev.fin_id[r] = id;
    // the sigmas before this episode's update that its initial retrace values
    // read (k_vr_append): its own id's and the previous entry's
    int pid = id;
    if (len < 2) pid = r > 0 ? ev.fin_id[r - 1] : (base >= 1 ? er.env[((long long)base - 1) % R] : id);
    ev.sig2[2 * r] = sig[id];
    ev.sig2[2 * r + 1] = sig[pid];
    const int cr0 = cr;
    const long long cb0 = cbeg, ce0 = cend;
    for (int k = 0; k < len; k++) {
      const float rw = ev.eb_rew[(long long)e * P.T + k];
      sum[id] += rw * rw;
      cnt[id]++;
      float ro;
      const int io = evicted((long long)base + off + k, ro);  // full: the oldest entry a - R leaves
      if (io >= 0) {
        sum[io] -= ro * ro;
        cnt[io]--;
      }
    }
    // every id's sigma after the episode (agent.cpp.base:557-563); an id whose
    // sums did not change keeps the value it has, so after the first
    // episode's full pass only this episode's id and the evicted entries' ids
    // are recomputed
    if (!st->rr_all) {
      for (int i = 0; i < EC; i++) sig[i] = rr_sigma(sum[i], cnt[i]);
      st->rr_all = 1;
    } else {
      sig[id] = rr_sigma(sum[id], cnt[id]);
      const int cr1 = cr;
      const long long cb1 = cbeg, ce1 = cend;
      cr = cr0, cbeg = cb0, cend = ce0;
      for (int k = 0; k < len; k++) {
        float ro;
        const int io = evicted((long long)base + off + k, ro);
        if (io >= 0) sig[io] = rr_sigma(sum[io], cnt[io]);
      }
      cr = cr1, cbeg = cb1, cend = ce1;
    }
  }
  if (lds)
    for (int i = 0; i < EC; i++) er.rsum[i] = sum[i], er.rcnt[i] = cnt[i], er.rsig[i] = sig[i];
}

// processEpisode (agent.cpp.base:376-572) for every finished episode at once:
// one workgroup per environment copies its episode into the replay memory,
// counts evicted off-policy entries, sets the initial retrace values (the
// reference's last-two-entries window, see oracle/vracer_ref.py) and resets
// the environment for its next launch.
__global__ __launch_bounds__(256) void k_vr_append(Params P, State *st, Replay er, Envs ev,
                                                   const float *__restrict__ outF, float *X,
                                                   const float *__restrict__ hnext, const int *__restrict__ hnext_id) {
  const int e = blockIdx.x;
  const int term = ev.fin[e];
  if (!term) return;
  const int t = threadIdx.x, nt = blockDim.x, S = P.S, A = P.A;
  const int len = ev.len[e], rank = ev.rank[e];
  const long long off = ev.off[e];
  const unsigned long long base = st->step_base, nnew = st->step_new, ep0 = st->step_episode_base,
                           neps = st->step_episodes, sid0 = st->step_sample_base;
  const long long R = P.R;
  // the next finished episode (rank + 1) sets our last entry's initial
  // retrace value when it has one experience: then no placeholder is written
  // for it here (the two workgroups are not ordered)
  const bool own_end = !((unsigned long long)(rank + 1) < neps && ev.len[ev.fin_env[rank + 1]] == 1);
  for (int k = t; k < len; k += nt) {
    const long long j = off + k;
    if ((long long)nnew - j > R) continue;  // overwritten within this batch (evictions: k_vr_evict)
    const long long abs_i = (long long)base + j, p = abs_i % R;
    const long long slot = (long long)e * P.T + k;
    const int tk = k == len - 1 ? term : NON_TERMINAL;
    for (int q = 0; q < S; q++) {
      er.st[p * S + q] = ev.eb_st[slot * S + q];
      er.tst[p * S + q] = tk == TRUNCATED ? X[(long long)e * S + q] : 0.f;
    }
    for (int i = 0; i < A; i++) er.act[p * A + i] = ev.eb_act[slot * A + i];
    for (int i = 0; i < 2 * A; i++) er.exp_pol[p * 2 * A + i] = er.cur_pol[p * 2 * A + i] = ev.eb_pol[slot * 2 * A + i];
    er.rew[p] = ev.eb_rew[slot];
    er.env[p] = ev.env_id[e];
    er.term[p] = tk;
    er.exp_v[p] = er.v[p] = ev.eb_v[slot];
    if (k != len - 1 || own_end) er.ret[p] = 0.f;
    er.iw[p] = 1.f;
    er.tiw[p] = 1.f;
    er.tv[p] = 0.f;
    er.onp[p] = 1;
    er.ep_id[p] = (long long)(ep0 + rank);
    er.ep_pos[p] = k;
  }
  __syncthreads();
  if (t == 0) {
    // initial retrace values (agent.cpp.base:520-555), rewards through
    // getScaledReward with the sigmas before this episode's update
    // (the sigmas before this episode's update: of its own id, and of the
    // entry before its first when it has one experience; k_vr_reward_sums)
    const float sgs = P.rr ? ev.sig2[2 * (long long)rank] : 1.0f, sgp = P.rr ? ev.sig2[2 * (long long)rank + 1] : 1.0f;
    const bool sg = P.rr != 0;
    auto scaled = [&](float r, bool own) { return sg ? r / (own ? sgs : sgp) : r; };
    float retV = 0.0f;
    if (term == TRUNCATED) retV += P.gamma * outF[(long long)e * P.O];
    const long long endj = off + len - 1;
    retV = P.gamma * retV + scaled(ev.eb_rew[(long long)e * P.T + len - 1], true);
    // an entry overwritten later in this same batch (more new experiences
    // than the capacity) keeps the later entry's values, as the reference's
    // sequential processEpisode calls leave it
    const long long survive = (long long)nnew - R;  // new-entry offsets below this were overwritten
    if (own_end && endj >= survive) er.ret[((long long)base + endj) % R] = retV;
    const long long prevj = endj - 1;
    if ((long long)base + prevj >= 0 && prevj >= survive) {
      float r;
      if (len >= 2) r = scaled(ev.eb_rew[(long long)e * P.T + len - 2], true);
      else if (rank > 0) {
        const int pe = ev.fin_env[rank - 1];
        r = scaled(ev.eb_rew[(long long)pe * P.T + ev.len[pe] - 1], false);
      } else {
        const long long q = ((long long)base + prevj) % R;
        r = scaled(er.rew[q], false);
      }
      retV = P.gamma * retV + r;
      er.ret[((long long)base + prevj) % R] = retV;
    }
    ev.rewards[rank] = ev.cum[e];
    atomicAdd(&st->step_reward_sum, (double)ev.cum[e]);
    // the next launch: sample id sid0 + rank + E (launch id = sample id)
    const unsigned long long sid = sid0 + (unsigned long long)rank + (unsigned long long)P.E;
    if (P.srs)  // the relaunched episode runs with the current moments (agent.cpp.base:186-187)
      for (int q = 0; q < S; q++) ev.pm[e * S + q] = st->smean[q], ev.ps[e * S + q] = st->ssdev[q];
    if (hnext) {  // a host environment: the initial state its function returned at its first update
      for (int q = 0; q < S; q++) {
        const float x = hnext[(long long)e * S + q];
        ev.hraw[(long long)e * S + q] = x;
        X[(long long)e * S + q] = vr_scale_state(P, ev, e, q, x);
      }
      ev.env_id[e] = hnext_id[e];
    } else {  // CartPole (env.py: cart.reset(sampleId * 1024 + launchId))
      double u[4];
      cp_reset((unsigned)(sid * 1024ull + sid), u);
      for (int q = 0; q < 4; q++) ev.u[e * 4 + q] = u[q], X[(long long)e * S + q] = vr_scale_state(P, ev, e, q, u[q]);
      ev.env_id[e] = (int)(sid % (unsigned long long)P.env_count);
    }
    ev.time[e] = 0.0;
    ev.t[e] = 0;
    ev.sample[e] = sid;
    ev.cum[e] = 0.f;
  }
}

// rescaleStates (agent.cpp.base:291-322): one lane per state dimension adds
// the replay memory's states in order (float, the reference's sums), the
// moments go to the agent state; then every stored state is rescaled (the
// truncated states are not, as in the reference) and the environments
// relaunched by the last step, which have not acted yet, take the new
// moments (the reference relaunches them at the top of the next loop
// iteration, after this rescaling)
__global__ void k_vr_srs_moments(Params P, State *st, Replay er) {
  const int d = threadIdx.x;
  if (blockIdx.x || d >= P.S) return;
  const unsigned long long n = st->size, R = (unsigned long long)P.R, base = (st->total - st->size) % R;
  float sum = 0.0f, sq = 0.0f;
  for (unsigned long long i = 0; i < n; i++) {
    unsigned long long q = base + i;
    if (q >= R) q -= R;
    const float x = er.st[q * P.S + d];
    sum += x;
    sq += x * x;
  }
  float m = sum / (float)n;
  if (!isfinite(m)) m = 0.0f;
  float sg = sqrtf(sq / (float)n - m * m);
  if (!isfinite(sg)) sg = 1.0f;
  if (sg <= 1e-9) sg = 1.0f;
  st->smean[d] = m;
  st->ssdev[d] = sg;
}
__global__ void k_vr_srs_apply(Params P, const State *st, Replay er, Envs ev, float *X) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)st->size * P.S;
  if (i < n) {
    const unsigned long long R = (unsigned long long)P.R, base = (st->total - st->size) % R;
    unsigned long long q = base + (unsigned long long)(i / P.S);
    if (q >= R) q -= R;
    const int d = (int)(i % P.S);
    float *x = er.st + q * P.S + d;
    *x = (*x - st->smean[d]) / st->ssdev[d];
  }
  if (i < (long long)P.E && ev.t[i] == 0) {
    const int e = (int)i;
    for (int k = 0; k < P.S; k++) ev.pm[e * P.S + k] = st->smean[k], ev.ps[e * P.S + k] = st->ssdev[k];
    if (P.host)
      for (int k = 0; k < P.S; k++) X[(long long)e * P.S + k] = vr_scale_state(P, ev, e, k, ev.hraw[(long long)e * P.S + k]);
    else
      for (int k = 0; k < 4; k++) X[(long long)e * P.S + k] = vr_scale_state(P, ev, e, k, ev.u[e * 4 + k]);
  }
}

__global__ void k_vr_init_state(State *st, float lr, float beta, float cutoff) {
  if (threadIdx.x || blockIdx.x) return;
  State s = {};
  s.lr = lr, s.beta = beta, s.cutoff = cutoff, s.eta = lr, s.b1p = 1.0f, s.b2p = 1.0f;
  for (int i = 0; i < MAXS; i++) s.smean[i] = 0.0f, s.ssdev[i] = 1.0f;
  *st = s;
}

}  // namespace vr
}  // namespace kg

// ======================================================================= host
using namespace kg::vr;

struct kg_vracer_s {
  Params P;
  int device;
  hipStream_t stream;
  size_t nparam;                   // device hyperparameters (hidden width padded to P.H)
  std::vector<size_t> offW, offb;  // per layer, device layout
  // Hidden widths that are not multiples of 64 run padded to P.H = the next
  // multiple: the padded units have zero weights in and out and a zero bias,
  // so their activations tanh(0) = 0 contribute nothing and their gradients,
  // Adam moments and L2 terms stay exactly 0.  The user-facing layout (the
  // reference's hyperparameter vector, nuser values) maps to the device one
  // through umap (empty when nothing is padded).
  size_t nuser;
  std::vector<size_t> umap;
  float *theta, *grad, *m1, *m2;
  float *X;          // E x S current environment states
  float *Xmb;        // 2B x S mini-batch (+ truncated) states
  float *Xs;         // rowsMax x S run_policy staging
  float *acts;       // L x rowsMax x H activations
  long long *offs = nullptr;  // offW[0..L], offb[0..L] on the device (k_vr_fwd_fused)
  float *out, *outF; // rowsMax x O
  float *G, *dZ, *dHa, *dHb;
  unsigned *mb, *forced_mb;
  float *forced_noise;
  int use_forced_noise;
  // host environments: states / next launches' states (E x S), rewards,
  // actions (E x A), terminations and environment ids (E) staged on the device
  float *h_states = nullptr, *h_next = nullptr, *h_rew = nullptr, *h_act = nullptr;
  int *h_term = nullptr, *h_ids = nullptr;
  State *st, *st_host;
  Replay er;
  Envs ev;
  size_t rowsMax;
  // stage timers (kg_vracer_profile): HIP events on the handle's stream
  int prof = 0;
  struct Ev {
    std::string stage;
    hipEvent_t a, b;
    size_t weight;  // stage instances the interval covers (a graph of updates: its length)
  };
  std::vector<Ev> events;
  std::vector<hipEvent_t> pool;
  std::map<std::string, std::pair<double, size_t>> totals;
  // session counters of Agent::trainingGeneration (agent.cpp.base:176-235)
  unsigned long long session_experiences, session_updates, until_start, start_size;
  double ebpu;
  // trainPolicy's updates replayed from one captured graph of upd_graph_n
  // back-to-back updates (their kernels read all varying state from device
  // memory, so one capture serves every later update)
  hipGraphExec_t upd_graph = nullptr;
  int upd_graph_n = 0;
  unsigned *drawKeys = nullptr;  // the graph's mini-batch ids, drawn up front (upd_graph_n x B)
  size_t drawCap = 0;
  // every device buffer in allocation order (kg_vracer_save_state / _load_state)
  std::vector<std::pair<void **, size_t>> bufs;
};

namespace {

int vr_alloc(void **p, size_t bytes) {
  KG_HIP(dev_alloc(p, bytes ? bytes : 16));
  return kg::zero_fill(*p, bytes ? bytes : 16);
}
#define VR_ALLOC(ptr, bytes)                                   \
  do {                                                         \
    if (vr_alloc((void **)&(ptr), (bytes))) return 1;          \
  } while (0)

unsigned vr_blocks(long long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// Scoped stage timer: events recorded on the handle's stream around a stage.
struct VrStage {
  kg_vracer_t h;
  size_t idx = (size_t)-1;
  VrStage(kg_vracer_t h_, const char *name, size_t weight = 1) : h(h_) {
    if (!h->prof) return;
    auto take = [&]() {
      hipEvent_t e = nullptr;
      if (!h->pool.empty()) {
        e = h->pool.back();
        h->pool.pop_back();
      } else if (hipEventCreate(&e) != hipSuccess) {
        e = nullptr;
      }
      return e;
    };
    hipEvent_t a = take(), b = take();
    if (!a || !b) return;
    if (hipEventRecord(a, h->stream) != hipSuccess) return;
    h->events.push_back({name, a, b, weight});
    idx = h->events.size() - 1;
  }
  ~VrStage() {
    if (idx != (size_t)-1) (void)hipEventRecord(h->events[idx].b, h->stream);
  }
};

int vr_collect(kg_vracer_t h) {
  for (auto &e : h->events) {
    KG_HIP(hipEventSynchronize(e.b));
    float ms = 0.f;
    KG_HIP(hipEventElapsedTime(&ms, e.a, e.b));
    auto &t = h->totals[e.stage];
    t.first += ms;
    t.second += e.weight;
    h->pool.push_back(e.a);
    h->pool.push_back(e.b);
  }
  h->events.clear();
  return 0;
}

bool vr_gemm_vec(int K, const float *A, long long sam, long long sak, const float *Bm, long long sbn, long long sbk) {
  auto al = [](const void *p) { return ((uintptr_t)p & 15) == 0; };
  return al(A) && al(Bm) && K % 4 == 0 && (sak == 1 ? sam % 4 == 0 : (sam == 1 && sak % 4 == 0)) &&
         (sbk == 1 ? sbn % 4 == 0 : (sbn == 1 && sbk % 4 == 0));
}
template <int EP>
void vr_gemm(kg_vracer_t h, int M, int N, int K, const float *A, long long sam, long long sak, const float *Bm,
             long long sbn, long long sbk, float *C, long long ldc, const float *bias, const float *T, long long ldt) {
  const bool vec = vr_gemm_vec(K, A, sam, sak, Bm, sbn, sbk);
  hipLaunchKernelGGL(k_vr_gemm<EP>, dim3(vr_blocks(N, GT), vr_blocks(M, GT)), dim3(256), 0, h->stream, M, N, K, A, sam,
                     sak, Bm, sbn, sbk, C, ldc, bias, T, ldt, vec ? 1 : 0);
}
VrGemmJob vr_gemm_job(int ep, int M, int N, int K, const float *A, long long sam, long long sak, const float *Bm,
                      long long sbn, long long sbk, float *C, long long ldc, const float *bias, const float *T,
                      long long ldt) {
  VrGemmJob g{};
  g.A = A, g.B = Bm, g.bias = bias, g.T = T, g.C = C;
  g.sam = sam, g.sak = sak, g.sbn = sbn, g.sbk = sbk, g.ldc = ldc, g.ldt = ldt;
  g.M = M, g.N = N, g.K = K, g.vec = vr_gemm_vec(K, A, sam, sak, Bm, sbn, sbk) ? 1 : 0, g.ep = ep;
  g.gx = vr_blocks(N, GT);
  g.n = g.gx * vr_blocks(M, GT);
  return g;
}

int vr_forward(kg_vracer_t h, const float *X, int M, float *out, bool input_done = false) {
  const Params &P = h->P;
  KG_CHECK((size_t)M <= h->rowsMax, "vracer: forward batch exceeds the allocated rows");
  // KORALI_AMD_VR_FUSED=1: one launch for the whole forward pass (bit-identical
  // results; measured slower than the per-layer kernels at C5, round 5: kept
  // for A/B and the equality test)
  const char *fe = getenv("KORALI_AMD_VR_FUSED");
  if (P.H <= 256 && fe && *fe == '1') {
    VrStage tg(h, M == P.E ? "gemm_rollout" : (M == 2 * P.B ? "gemm_update" : "gemm_other"));
    hipLaunchKernelGGL(k_vr_fwd_fused<false>, dim3(vr_blocks(M, FR)), dim3(256), 0, h->stream, P, M, X,
                       (const float *)h->theta, (const long long *)h->offs, h->acts, (long long)h->rowsMax, out,
                       (const State *)nullptr, Replay{}, (unsigned *)nullptr, (const unsigned *)nullptr,
                       (float *)nullptr);
    KG_HIP(hipGetLastError());
    return 0;
  }
  float *a1 = h->acts;
  if (!input_done)
    hipLaunchKernelGGL(k_vr_fwd_in, dim3(vr_blocks((long long)M * P.H, 256)), dim3(256), 0, h->stream, M, P.S, P.H, X,
                       h->theta + h->offW[0], h->theta + h->offb[0], a1);
  VrStage tg(h, M == P.E ? "gemm_rollout" : (M == 2 * P.B ? "gemm_update" : "gemm_other"));
  for (int l = 1; l < P.L; l++) {
    float *prev = h->acts + (size_t)(l - 1) * h->rowsMax * P.H, *cur = h->acts + (size_t)l * h->rowsMax * P.H;
    vr_gemm<EP_BIAS_TANH>(h, M, P.H, P.H, prev, P.H, 1, h->theta + h->offW[l], P.H, 1, cur, P.H,
                          h->theta + h->offb[l], nullptr, 0);
  }
  const float *last = h->acts + (size_t)(P.L - 1) * h->rowsMax * P.H;
  hipLaunchKernelGGL(k_vr_fwd_out, dim3(vr_blocks(M, 4)), dim3(256), 0, h->stream, M, P.H, P.O, last,
                     h->theta + h->offW[P.L], h->theta + h->offb[P.L], out, P);
  KG_HIP(hipGetLastError());
  return 0;
}

int vr_wgrad_cw(int Ni) {
  int cw = 1;
  while (cw < Ni + 1 && cw < 16) cw <<= 1;  // >= 16 batch lanes: <= B/16 loads per thread
  return cw;
}
void vr_wgrad(kg_vracer_t h, int No, int Ni, int Bn, const float *G, int ldg, const float *Act, int lda, float *dW,
              float *db) {
  const int cw = vr_wgrad_cw(Ni);
  hipLaunchKernelGGL(k_vr_wgrad_small, dim3(No, vr_blocks(Ni + 1, cw)), dim3(256), 0, h->stream, No, Ni, Bn, G, ldg, Act,
                     lda, dW, db, cw);
}
VrWgradJob vr_wgrad_job(int No, int Ni, int Bn, const float *G, int ldg, const float *Act, int lda, float *dW,
                        float *db) {
  VrWgradJob w{};
  w.G = G, w.Act = Act, w.dW = dW, w.db = db;
  w.No = No, w.Ni = Ni, w.Bn = Bn, w.ldg = ldg, w.lda = lda, w.cw = vr_wgrad_cw(Ni);
  w.n = No * vr_blocks(Ni + 1, w.cw);
  return w;
}
void vr_multi(kg_vracer_t h, const VrMulti &J) {
  int n = 0;
  for (int q = 0; q < J.nw; q++) n += J.w[q].n;
  for (int q = 0; q < J.ng; q++) n += J.g[q].n;
  hipLaunchKernelGGL(k_vr_multi, dim3(n), dim3(256), 0, h->stream, J);
}

// the metadata kernel's retrace walks staged through LDS (C5, round 5: the
// walk phase 14.2 against 21.0 us for the one-thread walks through the replay
// memory; KORALI_AMD_VR_STAGED=0 selects those, A/B and the equality test)
// the mini-batch draw fused with the input layer (k_vr_minibatch_in,
// KORALI_AMD_VR_DRAW_IN=1; bit-identical, measured slower at C5, round 5:
// 10.6 us against 7.1 + 5.0 for the two kernels it replaces, but 65.2 against
// 64.3 us per graph-replayed update -- every workgroup repeats the draw and
// sort, ~5 us of latency; kept for A/B and the equality test)
static bool vr_draw_in() {
  const char *e = getenv("KORALI_AMD_VR_DRAW_IN");
  return e && *e == '1';
}

static bool vr_staged_walks() {
  const char *e = getenv("KORALI_AMD_VR_STAGED");
  return !(e && *e == '0');
}

int vr_update(kg_vracer_t h, const unsigned *forced, const unsigned *drawn = nullptr) {
  const Params &P = h->P;
  const int B = P.B;
  KG_CHECK(h->st_host->size >= 2, "vracer: policy updates need at least two experiences in the replay memory");
  VrStage tu(h, "update");
  const char *fe = getenv("KORALI_AMD_VR_FUSED");
  const bool fused = P.H <= 256 && fe && *fe == '1';
  if (fused) {
    // the mini-batch draw, its gather and the whole forward pass: one launch
    VrStage tg(h, "gemm_update");
    hipLaunchKernelGGL(k_vr_fwd_fused<true>, dim3(vr_blocks(2 * B, FR)), dim3(256), 0, h->stream, P, 2 * B,
                       (const float *)nullptr, (const float *)h->theta, (const long long *)h->offs, h->acts,
                       (long long)h->rowsMax, h->out, (const State *)h->st, h->er, h->mb, forced, h->Xmb);
  } else if (drawn) {  // ids drawn ahead by the graph's k_vr_draw_ahead
    hipLaunchKernelGGL(k_vr_gather_in, dim3(vr_blocks(2LL * B * P.H, 256)), dim3(256), 0, h->stream, P,
                       (const State *)h->st, h->er, drawn, h->mb, h->Xmb, (const float *)(h->theta + h->offW[0]),
                       (const float *)(h->theta + h->offb[0]), h->acts);
    if (vr_forward(h, h->Xmb, 2 * B, h->out, true)) return 1;
  } else if (vr_draw_in() && P.S <= 16) {
    hipLaunchKernelGGL(k_vr_minibatch_in, dim3(vr_blocks(2 * B, MI)), dim3(256), 0, h->stream, P, (const State *)h->st,
                       h->er, h->mb, forced, h->Xmb, (const float *)(h->theta + h->offW[0]),
                       (const float *)(h->theta + h->offb[0]), h->acts);
    if (vr_forward(h, h->Xmb, 2 * B, h->out, true)) return 1;
  } else {
    hipLaunchKernelGGL(k_vr_minibatch, dim3(1), dim3(1024), 0, h->stream, P, h->st, h->er, h->mb, forced, h->Xmb);
    if (vr_forward(h, h->Xmb, 2 * B, h->out)) return 1;
  }
  const bool drawIn = !fused && !drawn && vr_draw_in() && P.S <= 16;
  const unsigned long long advance = ((fused || drawIn || drawn) && !forced) ? (unsigned long long)B : 0ULL;
  // threads of the one-workgroup metadata kernel: 512 stage every walk entry
  // of a C5 update (~5 500) in one pass of 16 loads in flight per thread
  // (staging 4.7 -> 2.9 us, update 64.1 -> 60.8 us, round 5; 1024 would cap
  // the kernel at 128 VGPRs and spill; KORALI_AMD_VR_META_TPB=256 for A/B)
  static const int metaTpb = [] {
    const char *e = getenv("KORALI_AMD_VR_META_TPB");
    const int v = e ? atoi(e) : 512;
    return (v == 256 || v == 512) ? v : 512;
  }();
  hipLaunchKernelGGL(P.rr ? k_vr_meta<true> : k_vr_meta<false>, dim3(1), dim3(metaTpb), 0, h->stream, P, h->st, h->er,
                     (const unsigned *)h->mb, (const float *)h->out, h->G, advance, vr_staged_walks() ? 1 : 0);
  // backward (DeepSupervisor, Direct Gradient) on the B mini-batch rows
  const size_t rs = h->rowsMax * P.H;
  const float *lastA = h->acts + (size_t)(P.L - 1) * rs;
  hipLaunchKernelGGL(k_vr_bwd_out, dim3(vr_blocks((long long)B * P.H, 256)), dim3(256), 0, h->stream, B, P.H, P.O,
                     (const float *)h->G, (const float *)h->out, (const float *)(h->theta + h->offW[P.L]), lastA, h->dZ,
                     h->dHa, P);
  const VrWgradJob outJob =
      vr_wgrad_job(P.O, P.H, B, h->dZ, P.O, lastA, P.H, h->grad + h->offW[P.L], h->grad + h->offb[P.L]);
  if (P.L == 1) {
    VrMulti J{};
    J.w[J.nw++] = outJob;
    vr_multi(h, J);
  }
  float *dcur = h->dHa, *dnext = h->dHb;
  for (int l = P.L - 1; l >= 1; l--) {
    const float *ain = h->acts + (size_t)(l - 1) * rs;
    VrMulti J{};
    if (l == P.L - 1) J.w[J.nw++] = outJob;
    // db_l[o] = sum_b dH[b][o]
    J.w[J.nw++] = vr_wgrad_job(P.H, 0, B, dcur, P.H, ain, P.H, nullptr, h->grad + h->offb[l]);
    // dW_l[o][i] = sum_b dH[b][o] a_{l-1}[b][i]
    J.g[J.ng++] = vr_gemm_job(EP_STORE, P.H, P.H, B, dcur, 1, P.H, ain, 1, P.H, h->grad + h->offW[l], P.H, nullptr,
                              nullptr, 0);
    // dH_{l-1} = (dH W_l) * (1 - a_{l-1}^2)
    J.g[J.ng++] = vr_gemm_job(EP_DTANH, B, P.H, P.H, dcur, P.H, 1, h->theta + h->offW[l], 1, P.H, dnext, P.H, nullptr,
                              ain, P.H);
    vr_multi(h, J);
    float *tmp = dcur;
    dcur = dnext, dnext = tmp;
  }
  {
    // the input layer's gradients (W_0, b_0: the first S H + H parameters),
    // with Adam on every parameter in the same launch
    const VrWgradJob w0 = vr_wgrad_job(P.H, P.S, B, dcur, P.H, h->Xmb, P.S, h->grad + h->offW[0], h->grad + h->offb[0]);
    VrAdamJob a{};
    a.theta = h->theta, a.m1 = h->m1, a.m2 = h->m2, a.grad = h->grad, a.st = (const State *)h->st;
    a.lo = (long long)h->offb[0] + P.H, a.hi = (long long)h->nparam, a.l2 = P.l2, a.l2imp = P.l2imp;
    const int na = (int)vr_blocks(a.hi - a.lo, 256);
    hipLaunchKernelGGL(k_vr_wgrad_adam, dim3(w0.n + na), dim3(256), 0, h->stream, w0, a);
  }
  KG_HIP(hipGetLastError());
  return 0;
}

int vr_read_state(kg_vracer_t h) {
  KG_HIP(hipMemcpyAsync(h->st_host, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  if (h->st_host->errors) {
    const unsigned e = h->st_host->errors;
    if (e & ERR_NONFINITE_GRADIENT) kg::set_error("Gradient loss returned an invalid value (VRACER.cpp.base:173-175)");
    else if (e & ERR_NONFINITE_VALUE) kg::set_error("Calculated state value returned an invalid value (agent.cpp.base:629-630)");
    else if (e & ERR_ENV_ODE) kg::set_error("CartPole: the dopri5 integration failed (more than 500 steps or a vanishing step)");
    else if (e & ERR_EPISODE_LONG)
      kg::set_error("An environment's episode exceeded 'Max Episode Steps' (the device's episode buffer); raise it");
    else kg::set_error("NaN detected in the calculation of importance weight (continuous.cpp.base:391)");
    return 1;
  }
  return 0;
}

struct VrField {
  void *ptr;
  size_t elem, count;
  bool param;  // a hyperparameter-shaped array (user layout <-> device layout)
};
bool vr_field(kg_vracer_t h, const char *name, VrField &f) {
  const Params &P = h->P;
  const size_t R = (size_t)P.R, E = (size_t)P.E;
  struct {
    const char *n;
    void *p;
    size_t elem, count;
  } tab[] = {
      {"state", h->er.st, 4, R * P.S},         {"action", h->er.act, 4, R * P.A},
      {"reward", h->er.rew, 4, R},             {"environment_id", h->er.env, 4, R},
      {"termination", h->er.term, 4, R},       {"truncated_state", h->er.tst, 4, R * P.S},
      {"exp_policy", h->er.exp_pol, 4, R * 2 * P.A}, {"cur_policy", h->er.cur_pol, 4, R * 2 * P.A},
      {"exp_state_value", h->er.exp_v, 4, R},  {"state_value", h->er.v, 4, R},
      {"retrace", h->er.ret, 4, R},            {"importance_weight", h->er.iw, 4, R},
      {"truncated_importance_weight", h->er.tiw, 4, R}, {"truncated_state_value", h->er.tv, 4, R},
      {"on_policy", h->er.onp, 4, R},          {"episode_id", h->er.ep_id, 8, R},
      {"episode_pos", h->er.ep_pos, 4, R},     {"hyperparameters", h->theta, 4, h->nuser},
      {"adam_first_moment", h->m1, 4, h->nuser}, {"adam_second_moment", h->m2, 4, h->nuser},
      {"gradient", h->grad, 4, h->nuser},      {"env_states", h->X, 4, E * P.S},
      {"env_u", h->ev.u, 8, E * 4},            {"env_time", h->ev.time, 8, E},
      {"env_steps", h->ev.t, 4, E},
      {"env_ids", h->ev.env_id, 4, E},         {"env_sample_ids", h->ev.sample, 8, E},
      {"finished_rewards", h->ev.rewards, 4, E}, {"finished_env", h->ev.fin_env, 4, E},
      {"mini_batch", h->mb, 4, (size_t)P.B},   {"loss_gradient", h->G, 4, (size_t)P.B * P.O},
      {"policy_output", h->out, 4, h->rowsMax * P.O},
      {"reward_rescaling_sigma", h->er.rsig, 4, (size_t)P.env_count},
      {"reward_rescaling_sum", h->er.rsum, 4, (size_t)P.env_count},
      {"reward_rescaling_count", h->er.rcnt, 8, (size_t)P.env_count},
      {"state_rescaling_means", &h->st->smean[0], 4, (size_t)std::min(P.S, MAXS)},
      {"state_rescaling_sigmas", &h->st->ssdev[0], 4, (size_t)std::min(P.S, MAXS)},
      {"meta_phase_ticks", &h->st->mtr[0], 8, (size_t)9},
  };
  for (auto &x : tab)
    if (!strcmp(x.n, name)) {
      f = VrField{x.p, x.elem, x.count,
                  x.p == h->theta || x.p == h->grad || x.p == h->m1 || x.p == h->m2};
      return true;
    }
  return false;
}

}  // namespace

extern "C" {

int kg_vracer_create(const kg_vracer_config *c, kg_vracer_t *out) {
  KG_CHECK(c && out, "vracer: null argument");
  KG_CHECK(c->state_size >= 1 && c->action_size >= 1 && c->action_size <= (size_t)MAXA,
           "vracer: action size must be 1..4 and state size >= 1");
  KG_CHECK(c->host_environment || (c->state_size == 4 && c->action_size == 1),
           "vracer: the device environment is the CartPole of examples/learning/reinforcement/cartpole (4 states, 1 action)");
  KG_CHECK(c->hidden_size >= 1 && c->hidden_size <= 4096, "vracer: hidden layer width must be 1..4096");
  KG_CHECK(c->hidden_layers >= 1, "vracer: at least one hidden layer");
  KG_CHECK(c->mini_batch_size >= 2 && c->mini_batch_size <= (size_t)MB_META, "vracer: Mini Batch Size must be 2..1024");
  KG_CHECK(c->environments >= 1 && c->environments <= (1u << 20), "vracer: Concurrent Environments out of range");
  KG_CHECK(c->environment_count >= 1, "vracer: Environment Count must be >= 1");
  KG_CHECK(c->replay_maximum_size >= 2 && c->replay_start_size <= c->replay_maximum_size,
           "vracer: Experience Replay Start Size must not exceed Maximum Size");
  KG_CHECK(c->max_episode_steps >= 1, "vracer: episodes need at least one step");
  KG_CHECK(c->off_policy_cutoff_scale >= 0.0, "Experience Replay Cutoff Scale must be larger 0.0");
  for (size_t i = 0; i < c->action_size; i++)
    KG_CHECK(c->initial_exploration_noise && c->initial_exploration_noise[i] > 0.0,
             "Provided initial noise for an action variable is not defined or negative.");
  KG_CHECK(c->policy_distribution == 0 || c->policy_distribution == 1,
           "vracer: policy distribution must be 0 (Normal) or 1 (Clipped Normal)");
  if (c->policy_distribution == 1)
    for (size_t i = 0; i < c->action_size; i++)
      KG_CHECK(c->action_lower_bounds && c->action_upper_bounds && std::isfinite(c->action_lower_bounds[i]) &&
                   std::isfinite(c->action_upper_bounds[i]),
               "Provided bound for an action variable is non-finite, but the distribution (Clipped Normal) is bounded.");
  KG_HIP(hipSetDevice(c->device));
  auto *h = new kg_vracer_s();
  Params &P = h->P;
  P.S = (int)c->state_size, P.A = (int)c->action_size, P.H = (int)((c->hidden_size + 63) / 64 * 64), P.L = (int)c->hidden_layers;
  P.O = 1 + 2 * P.A, P.E = (int)c->environments, P.B = (int)c->mini_batch_size, P.T = (int)c->max_episode_steps;
  P.R = (long long)c->replay_maximum_size;
  P.env_count = (int)c->environment_count;
  P.rr = c->reward_rescaling ? 1 : 0;
  P.srs = c->state_rescaling ? 1 : 0;
  P.host = c->host_environment ? 1 : 0;
  KG_CHECK(!P.srs || c->state_size <= (size_t)MAXS, "vracer: State Rescaling on the device supports up to 8 state variables");
  KG_CHECK(c->environment_count >= 1, "vracer: Environment Count must be at least 1");
  P.l2 = c->l2_regularization_enabled ? 1 : 0;
  P.gamma = (float)c->discount_factor, P.lr0 = (float)c->learning_rate, P.iw_trunc = (float)c->importance_weight_truncation_level;
  P.cutoff_scale = (float)c->off_policy_cutoff_scale, P.off_target = (float)c->off_policy_target;
  P.anneal = (float)c->off_policy_annealing_rate, P.l2imp = (float)c->l2_regularization_importance;
  P.seed = c->seed;
  for (int o = 0; o < MAXO; o++) P.scale[o] = 1.f, P.shift[o] = 0.f, P.soft[o] = 0;
  P.clipped = c->policy_distribution == 1 ? 1 : 0;
  for (int i = 0; i < P.A; i++) {
    P.scale[1 + P.A + i] = 2.0f * (float)c->initial_exploration_noise[i];
    P.soft[1 + P.A + i] = 1;
    P.lb[i] = c->action_lower_bounds ? (float)c->action_lower_bounds[i] : -INFINITY;
    P.ub[i] = c->action_upper_bounds ? (float)c->action_upper_bounds[i] : INFINITY;
    // bounded distributions shift the means by the action shift (continuous.cpp.base:20-30, :53-54)
    if (P.clipped) P.shift[1 + i] = (P.ub[i] + P.lb[i]) * 0.5f;
  }
  h->device = c->device;
  h->ebpu = c->experiences_between_policy_updates;
  h->start_size = c->replay_start_size;
  h->until_start = c->replay_start_size;
  // hyperparameter layout: [W (out x in), b] per layer (linear.cpp.base:28-49)
  std::vector<int> sz{P.S};
  for (int l = 0; l < P.L; l++) sz.push_back(P.H);
  sz.push_back(P.O);
  size_t k = 0;
  for (size_t l = 0; l + 1 < sz.size(); l++) {
    h->offW.push_back(k);
    k += (size_t)sz[l] * sz[l + 1];
    h->offb.push_back(k);
    k += (size_t)sz[l + 1];
  }
  h->nparam = k;
  // the user layout (hidden width c->hidden_size) and its device positions
  {
    const size_t Hu = c->hidden_size;
    std::vector<size_t> su{(size_t)P.S};
    for (int l = 0; l < P.L; l++) su.push_back(Hu);
    su.push_back((size_t)P.O);
    size_t ku = 0;
    for (size_t l = 0; l + 1 < su.size(); l++) ku += su[l] * su[l + 1] + su[l + 1];
    h->nuser = ku;
    if (Hu != (size_t)P.H) {
      h->umap.reserve(ku);
      for (size_t l = 0; l + 1 < su.size(); l++) {
        const size_t in_d = (size_t)sz[l];  // device row length of this layer's W
        for (size_t o = 0; o < su[l + 1]; o++)
          for (size_t i = 0; i < su[l]; i++) h->umap.push_back(h->offW[l] + o * in_d + i);
        for (size_t o = 0; o < su[l + 1]; o++) h->umap.push_back(h->offb[l] + o);
      }
    }
  }
  h->rowsMax = std::max((size_t)P.E, (size_t)2 * P.B);
  const size_t R = (size_t)P.R, E = (size_t)P.E, ET = E * (size_t)P.T;
  int rc = 0;
  auto alloc = [&](auto *&p, size_t bytes) {
    if (!rc && vr_alloc((void **)&p, bytes)) rc = 1;
    if (!rc) h->bufs.push_back({(void **)&p, bytes ? bytes : 16});
  };
  hipError_t se = kg::stream_acquire(&h->stream);
  if (se != hipSuccess) {
    delete h;
    kg::set_error(std::string("hipStreamCreate: ") + hipGetErrorString(se));
    return 1;
  }
  alloc(h->theta, k * 4), alloc(h->grad, k * 4), alloc(h->m1, k * 4), alloc(h->m2, k * 4);
  alloc(h->X, E * P.S * 4), alloc(h->Xmb, 2 * (size_t)P.B * P.S * 4), alloc(h->Xs, h->rowsMax * P.S * 4);
  alloc(h->acts, (size_t)P.L * h->rowsMax * P.H * 4);
  alloc(h->offs, 2 * ((size_t)P.L + 1) * sizeof(long long));
  if (!rc) {
    std::vector<long long> o;
    for (auto v : h->offW) o.push_back((long long)v);
    for (auto v : h->offb) o.push_back((long long)v);
    if (hipMemcpy(h->offs, o.data(), o.size() * sizeof(long long), hipMemcpyHostToDevice) != hipSuccess) rc = 1;
  }
  alloc(h->out, h->rowsMax * P.O * 4), alloc(h->outF, h->rowsMax * P.O * 4);
  alloc(h->G, (size_t)P.B * P.O * 4), alloc(h->dZ, (size_t)P.B * P.O * 4);
  alloc(h->dHa, (size_t)P.B * P.H * 4), alloc(h->dHb, (size_t)P.B * P.H * 4);
  alloc(h->mb, (size_t)P.B * 4), alloc(h->forced_mb, (size_t)P.B * 4), alloc(h->forced_noise, E * P.A * 4);
  if (c->host_environment) {
    alloc(h->h_states, E * P.S * 4), alloc(h->h_next, E * P.S * 4), alloc(h->h_rew, E * 4), alloc(h->h_act, E * P.A * 4);
    alloc(h->h_term, E * 4), alloc(h->h_ids, E * 4);
  }
  alloc(h->st, sizeof(State));
  Replay &er = h->er;
  alloc(er.st, R * P.S * 4), alloc(er.act, R * P.A * 4), alloc(er.rew, R * 4), alloc(er.tst, R * P.S * 4);
  alloc(er.exp_pol, R * 2 * P.A * 4), alloc(er.cur_pol, R * 2 * P.A * 4), alloc(er.exp_v, R * 4), alloc(er.v, R * 4);
  alloc(er.ret, R * 4), alloc(er.iw, R * 4), alloc(er.tiw, R * 4), alloc(er.tv, R * 4);
  alloc(er.env, R * 4), alloc(er.term, R * 4), alloc(er.onp, R * 4), alloc(er.ep_pos, R * 4), alloc(er.ep_id, R * 8);
  const size_t EC = (size_t)P.env_count;
  alloc(er.rsig, EC * 4), alloc(er.rsum, EC * 4), alloc(er.rcnt, EC * 8);
  if (!rc) {  // getScaledReward's sigma starts at 1.0 for every id (agent.cpp.base:96-98)
    const std::vector<float> ones(EC, 1.0f);
    if (hipMemcpy(er.rsig, ones.data(), EC * 4, hipMemcpyHostToDevice) != hipSuccess) rc = 1;
  }
  Envs &ev = h->ev;
  alloc(ev.u, E * 4 * 8), alloc(ev.time, E * 8), alloc(ev.t, E * 4), alloc(ev.env_id, E * 4), alloc(ev.sample, E * 8), alloc(ev.cum, E * 4);
  alloc(ev.fin, E * 4), alloc(ev.len, E * 4), alloc(ev.off, E * 8), alloc(ev.rank, E * 4), alloc(ev.fin_env, E * 4);
  alloc(ev.eb_st, ET * P.S * 4), alloc(ev.eb_act, ET * P.A * 4), alloc(ev.eb_pol, ET * 2 * P.A * 4);
  alloc(ev.eb_v, ET * 4), alloc(ev.eb_rew, ET * 4), alloc(ev.rewards, E * 4);
  alloc(ev.sig2, E * 2 * 4), alloc(ev.fin_id, E * 4);
  alloc(ev.pm, (size_t)E * P.S * 4), alloc(ev.ps, (size_t)E * P.S * 4);
  if (P.host) alloc(ev.hraw, (size_t)E * P.S * 4);
  if (!rc && host_alloc((void **)&h->st_host, sizeof(State), hipHostMallocDefault) != hipSuccess) {
    kg::set_error("vracer: hipHostMalloc failed");
    rc = 1;
  }
  if (!rc) memset(h->st_host, 0, sizeof(State));
  if (rc) {
    kg_vracer_destroy(h);
    return 1;
  }
  hipLaunchKernelGGL(k_vr_init_state, dim3(1), dim3(1), 0, h->stream, h->st, P.lr0, (float)c->off_policy_refer_beta,
                     P.cutoff_scale);
  // the first launch of every environment: sample ids 0 .. E-1 (a host
  // environment's come with kg_vracer_host_launch)
  if (!P.host)
    hipLaunchKernelGGL(k_vr_env_reset, dim3(vr_blocks(P.E, 256)), dim3(256), 0, h->stream, P, (const State *)h->st,
                       h->ev, h->X, 0ull, (const int *)nullptr);
  if (hipGetLastError() != hipSuccess || vr_read_state(h)) {
    if (!*kg::last_error()) kg::set_error("vracer: initial launches failed");
    kg_vracer_destroy(h);
    return 1;
  }
  *out = h;
  return 0;
}

// kg_debug_cartpole_at: trajectory j advances `steps` times with
// force[j][k] from u0[j] at time t0[j] (0 without t0); the time after the
// last advance in t_out[j] (the device CartPole of k_vr_env_act)
__global__ void k_vr_cartpole_debug(size_t n, size_t steps, const double *u0, const double *t0, const double *force,
                                    double *u_out, double *t_out, int *over) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double y[4], t = t0 ? t0[j] : 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) y[k] = u0[j * 4 + k];
  for (size_t s = 0; s < steps; s++) {
    const bool ok = cp_advance(y, t, force[j * steps + s]);
#pragma unroll
    for (int k = 0; k < 4; k++) u_out[(j * steps + s) * 4 + k] = y[k];
    over[j * steps + s] = ok ? (cp_failed(y) ? 1 : 0) : -1;
  }
  if (t_out) t_out[j] = t;
}

extern "C" int kg_debug_cartpole_at(int device, const double *u0, const double *t0, const double *force, size_t n,
                                    size_t steps, double *u_out, double *t_out, int *over) {
  KG_CHECK(u0 && force && u_out && over, "kg_debug_cartpole: null argument");
  KG_CHECK(n >= 1 && steps >= 1 && n * steps <= (1u << 24), "kg_debug_cartpole: 1 <= n * steps <= 2^24");
  KG_HIP(hipSetDevice(device));
  double *d = nullptr;
  const size_t nb = (n * 4 + 2 * n + n * steps + n * steps * 4 + n * steps) * sizeof(double);
  KG_HIP(dev_alloc(&d, nb));
  double *du0 = d, *dt0 = du0 + n * 4, *dt1 = dt0 + n, *dforce = dt1 + n, *dout = dforce + n * steps;
  int *o = (int *)(dout + n * steps * 4);
  int rc = 0;
  if (hipMemcpy(du0, u0, n * 4 * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      (t0 && hipMemcpy(dt0, t0, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(dforce, force, n * steps * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    rc = 1;
  if (!rc) {
    hipLaunchKernelGGL(k_vr_cartpole_debug, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, 0, n, steps, du0,
                       t0 ? (const double *)dt0 : nullptr, dforce, dout, dt1, o);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(u_out, dout, n * steps * 4 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(over, o, n * steps * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess ||
        (t_out && hipMemcpy(t_out, dt1, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
      rc = 1;
  }
  dev_release(d);
  if (rc) kg::set_error("kg_debug_cartpole: device call failed");
  return rc;
}

extern "C" int kg_debug_cartpole(int device, const double *u0, const double *force, size_t n, size_t steps,
                                 double *u_out, int *over) {
  return kg_debug_cartpole_at(device, u0, nullptr, force, n, steps, u_out, nullptr, over);
}

int kg_vracer_destroy(kg_vracer_t h) {
  if (!h) return 0;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->upd_graph) (void)hipGraphExecDestroy(h->upd_graph);
  if (h->drawKeys) kg::dev_release(h->drawKeys);
  void *ptrs[] = {h->offs, h->theta, h->grad, h->m1, h->m2, h->X, h->Xmb, h->Xs, h->acts, h->out, h->outF, h->G, h->dZ, h->dHa,
                  h->dHb, h->mb, h->forced_mb, h->forced_noise, h->st, h->er.st, h->er.act, h->er.rew, h->er.tst,
                  h->er.exp_pol, h->er.cur_pol, h->er.exp_v, h->er.v, h->er.ret, h->er.iw, h->er.tiw, h->er.tv,
                  h->er.env, h->er.term, h->er.onp, h->er.ep_pos, h->er.ep_id, h->ev.u, h->ev.time, h->ev.t, h->ev.env_id,
                  h->ev.sample, h->ev.cum, h->ev.fin, h->ev.len, h->ev.off, h->ev.rank, h->ev.fin_env, h->ev.eb_st,
                  h->ev.eb_act, h->ev.eb_pol, h->ev.eb_v, h->ev.eb_rew, h->ev.rewards, h->ev.sig2, h->ev.fin_id,
                  h->ev.pm, h->ev.ps, h->ev.hraw, h->er.rsig, h->er.rsum, h->er.rcnt};
  for (void *p : ptrs)
    if (p) dev_release(p);
  if (h->st_host) host_release(h->st_host);
  for (auto &e : h->events) (void)hipEventDestroy(e.a), (void)hipEventDestroy(e.b);
  for (auto e : h->pool) (void)hipEventDestroy(e);
  if (h->stream) stream_release(h->stream);
  delete h;
  return 0;
}

int kg_vracer_hyperparameter_count(kg_vracer_t h, size_t *n) {
  KG_CHECK(h && n, "vracer: null argument");
  *n = h->nuser;
  return 0;
}

int kg_vracer_field_size(kg_vracer_t h, const char *name, size_t *elem_bytes, size_t *count) {
  KG_CHECK(h && name, "vracer: null argument");
  VrField f;
  KG_CHECK(vr_field(h, name, f), std::string("vracer: unknown field '") + name + "'");
  if (elem_bytes) *elem_bytes = f.elem;
  if (count) *count = f.count;
  return 0;
}

int kg_vracer_get_field(kg_vracer_t h, const char *name, void *dst, size_t bytes) {
  KG_CHECK(h && name && dst, "vracer: null argument");
  VrField f;
  KG_CHECK(vr_field(h, name, f), std::string("vracer: unknown field '") + name + "'");
  KG_CHECK(bytes <= f.elem * f.count, "vracer: field read exceeds its size");
  if (f.param && !h->umap.empty()) {  // padded hidden width: gather the user layout
    std::vector<float> dev(h->nparam);
    KG_HIP(hipMemcpyAsync(dev.data(), f.ptr, h->nparam * 4, hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    float *o = (float *)dst;
    for (size_t i = 0; i < bytes / 4; i++) o[i] = dev[h->umap[i]];
    return 0;
  }
  KG_HIP(hipMemcpyAsync(dst, f.ptr, bytes, hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_vracer_set_field(kg_vracer_t h, const char *name, const void *src, size_t bytes) {
  KG_CHECK(h && name && src, "vracer: null argument");
  VrField f;
  KG_CHECK(vr_field(h, name, f), std::string("vracer: unknown field '") + name + "'");
  KG_CHECK(bytes <= f.elem * f.count, "vracer: field write exceeds its size");
  if (f.param && !h->umap.empty()) {  // padded hidden width: scatter, padding stays 0
    std::vector<float> dev(h->nparam);
    KG_HIP(hipMemcpyAsync(dev.data(), f.ptr, h->nparam * 4, hipMemcpyDeviceToHost, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    const float *in = (const float *)src;
    for (size_t i = 0; i < bytes / 4; i++) dev[h->umap[i]] = in[i];
    KG_HIP(hipMemcpyAsync(f.ptr, dev.data(), h->nparam * 4, hipMemcpyHostToDevice, h->stream));
    KG_HIP(hipStreamSynchronize(h->stream));
    return 0;
  }
  KG_HIP(hipMemcpyAsync(f.ptr, src, bytes, hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

static const char *const kScalarNames[] = {"learning_rate", "refer_beta", "off_policy_cutoff", "off_policy_ratio",
                                           "adam_eta", "adam_beta1_pow", "adam_beta2_pow", "off_policy_count",
                                           "policy_update_count", "total", "size", "current_episode",
                                           "current_sample_id", "mini_batch_counter", "environment_step",
                                           "step_new_experiences", "step_episodes", "experience_count",
                                           "step_reward_sum"};

int kg_vracer_get_scalar(kg_vracer_t h, const char *name, double *v) {
  KG_CHECK(h && name && v, "vracer: null argument");
  KG_HIP(hipMemcpyAsync(h->st_host, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  const State &s = *h->st_host;
  const double vals[] = {s.lr, s.beta, s.cutoff, s.off_ratio, s.eta, s.b1p, s.b2p, (double)s.off_count,
                         (double)s.update_count, (double)s.total, (double)s.size, (double)s.episode,
                         (double)s.sample_id, (double)s.mb_counter, (double)s.env_step, (double)s.step_new,
                         (double)s.step_episodes, (double)s.experience_count, s.step_reward_sum};
  for (size_t i = 0; i < sizeof(vals) / sizeof(vals[0]); i++)
    if (!strcmp(kScalarNames[i], name)) {
      *v = vals[i];
      return 0;
    }
  kg::set_error(std::string("vracer: unknown scalar '") + name + "'");
  return 1;
}

int kg_vracer_set_scalar(kg_vracer_t h, const char *name, double v) {
  KG_CHECK(h && name, "vracer: null argument");
  KG_HIP(hipMemcpyAsync(h->st_host, h->st, sizeof(State), hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  State &s = *h->st_host;
  const std::string n(name);
  if (n == "learning_rate") s.lr = (float)v;
  else if (n == "refer_beta") s.beta = (float)v;
  else if (n == "off_policy_cutoff") s.cutoff = (float)v;
  else if (n == "off_policy_ratio") s.off_ratio = (float)v;
  else if (n == "off_policy_count") s.off_count = (long long)v;
  else if (n == "policy_update_count") s.update_count = (long long)v;
  else if (n == "total") s.total = (unsigned long long)v;
  else if (n == "size") s.size = (unsigned long long)v;
  else if (n == "current_episode") s.episode = (unsigned long long)v;
  else if (n == "mini_batch_counter") s.mb_counter = (unsigned long long)v;
  else if (n == "experience_count") s.experience_count = (unsigned long long)v;
  else {
    kg::set_error("vracer: scalar '" + n + "' is not settable");
    return 1;
  }
  KG_HIP(hipMemcpyAsync(h->st, h->st_host, sizeof(State), hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_vracer_run_policy(kg_vracer_t h, const float *states, size_t n, float *out) {
  KG_CHECK(h && states && out, "vracer: null argument");
  KG_CHECK(n <= h->rowsMax, "vracer: run_policy batch exceeds max(Concurrent Environments, 2 x Mini Batch Size)");
  KG_HIP(hipMemcpyAsync(h->Xs, states, n * h->P.S * 4, hipMemcpyHostToDevice, h->stream));
  if (vr_forward(h, h->Xs, (int)n, h->out)) return 1;
  KG_HIP(hipMemcpyAsync(out, h->out, n * h->P.O * 4, hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_vracer_test_episodes(kg_vracer_t h, const uint64_t *sample_ids, const uint64_t *launch_ids, size_t n,
                            float *rewards) {
  KG_CHECK(h && sample_ids && launch_ids && rewards, "vracer: null argument");
  KG_CHECK(h->P.A == 1 && h->P.S == 4, "vracer: testing episodes run the CartPole kernel (4 states, 1 action)");
  const size_t chunk = h->rowsMax;  // episodes per batch (the forward's rows)
  unsigned long long *dsid = nullptr, *dlid = nullptr;
  double *u = nullptr, *tm = nullptr;
  int *steps = nullptr, *done = nullptr, *running = nullptr;
  float *cum = nullptr;
  unsigned *errs = nullptr;
  int rc = 0;
  bool named = false;  // an error message was set
  auto fail = [&](hipError_t e) {
    if (e != hipSuccess) rc = 1;
    return e != hipSuccess;
  };
  if (fail(dev_alloc(&dsid, chunk * 8)) || fail(dev_alloc(&dlid, chunk * 8)) || fail(dev_alloc(&u, chunk * 32)) ||
      fail(dev_alloc(&tm, chunk * 8)) || fail(dev_alloc(&steps, chunk * 4)) || fail(dev_alloc(&done, chunk * 4)) ||
      fail(dev_alloc(&cum, chunk * 4)) || fail(dev_alloc(&running, 4)) || fail(dev_alloc(&errs, 4)))
    kg::set_error("vracer: testing buffers could not be allocated"), named = true;
  for (size_t b0 = 0; rc == 0 && b0 < n; b0 += chunk) {
    const int m = (int)std::min(chunk, n - b0);
    const dim3 grid((m + 255) / 256);
    if (fail(hipMemcpyAsync(dsid, sample_ids + b0, m * 8, hipMemcpyHostToDevice, h->stream)) ||
        fail(hipMemcpyAsync(dlid, launch_ids + b0, m * 8, hipMemcpyHostToDevice, h->stream)) ||
        fail(hipMemsetAsync(errs, 0, 4, h->stream)))
      break;
    hipLaunchKernelGGL(k_vr_test_reset, grid, dim3(256), 0, h->stream, h->P, (const State *)h->st, m, h->P.S, dsid,
                       dlid, u, tm, steps, done, cum, h->Xs);
    for (int t = 0; t < h->P.T; t++) {
      if (vr_forward(h, h->Xs, m, h->out)) {
        rc = 1, named = true;
        break;
      }
      if (t % 16 == 0 && fail(hipMemsetAsync(running, 0, 4, h->stream))) break;
      hipLaunchKernelGGL(k_vr_test_act, grid, dim3(256), 0, h->stream, h->P, (const State *)h->st, m,
                         (const float *)h->out, u, tm, steps, done, cum, h->Xs, errs, running);
      if (t % 16 == 15) {  // every 16 steps: stop once every episode has ended
        int r = 0;
        if (fail(hipMemcpyAsync(&r, running, 4, hipMemcpyDeviceToHost, h->stream)) ||
            fail(hipStreamSynchronize(h->stream)))
          break;
        if (r == 0) break;
      }
    }
    unsigned e = 0;
    if (rc == 0 && (fail(hipMemcpyAsync(rewards + b0, cum, m * 4, hipMemcpyDeviceToHost, h->stream)) ||
                    fail(hipMemcpyAsync(&e, errs, 4, hipMemcpyDeviceToHost, h->stream)) ||
                    fail(hipStreamSynchronize(h->stream))))
      break;
    if (e) {
      kg::set_error("CartPole: the dopri5 integration failed (more than 500 steps or a vanishing step)");
      rc = 1, named = true;
    }
  }
  for (void *p : {(void *)dsid, (void *)dlid, (void *)u, (void *)tm, (void *)steps, (void *)done, (void *)cum,
                  (void *)running, (void *)errs})
    if (p) dev_release(p, h->stream);
  if (rc && !named) kg::set_error("vracer: testing episodes failed (HIP error)");
  return rc;
}

int kg_vracer_set_action_noise(kg_vracer_t h, const float *noise, size_t n) {
  KG_CHECK(h, "vracer: null argument");
  if (!noise) {
    h->use_forced_noise = 0;
    return 0;
  }
  KG_CHECK(n == (size_t)h->P.E * h->P.A, "vracer: action noise must hold Concurrent Environments x action size values");
  KG_HIP(hipMemcpyAsync(h->forced_noise, noise, n * 4, hipMemcpyHostToDevice, h->stream));
  h->use_forced_noise = 1;
  return 0;
}

int kg_vracer_environment_step(kg_vracer_t h, size_t *new_experiences) {
  KG_CHECK(h, "vracer: null argument");
  KG_CHECK(!h->P.host, "vracer: a host environment steps through kg_vracer_host_act / kg_vracer_host_feed");
  const Params &P = h->P;
  {
  VrStage te(h, "environment_step");
  if (vr_forward(h, h->X, P.E, h->out)) return 1;
  hipLaunchKernelGGL(k_vr_env_act, dim3(vr_blocks(P.E, 256)), dim3(256), 0, h->stream, P, h->st, h->ev,
                     (const float *)h->out, h->X, h->use_forced_noise ? (const float *)h->forced_noise : nullptr);
  h->use_forced_noise = 0;
  if (vr_forward(h, h->X, P.E, h->outF)) return 1;  // V of truncated states (agent.cpp.base:530-545)
  hipLaunchKernelGGL(k_vr_scan, dim3(1), dim3(1024), 0, h->stream, P, h->st, h->ev);
  hipLaunchKernelGGL(k_vr_evict, dim3(1), dim3(256), 0, h->stream, P, h->st, h->er);
  if (P.rr) hipLaunchKernelGGL(k_vr_reward_sums, dim3(1), dim3(64), 0, h->stream, P, h->st, h->er, h->ev);
  hipLaunchKernelGGL(k_vr_append, dim3(P.E), dim3(256), 0, h->stream, P, h->st, h->er, h->ev, (const float *)h->outF,
                     h->X, (const float *)nullptr, (const int *)nullptr);
  KG_HIP(hipGetLastError());
  }
  if (vr_read_state(h)) return 1;
  h->session_experiences += h->st_host->step_new;
  if (new_experiences) *new_experiences = (size_t)h->st_host->step_new;
  return 0;
}

int kg_vracer_host_launch(kg_vracer_t h, const float *states, const int *env_ids) {
  KG_CHECK(h && states && env_ids, "vracer: null argument");
  const Params &P = h->P;
  KG_CHECK(P.host, "vracer: the agent was created for the CartPole kernel, not a host environment");
  for (int e = 0; e < P.E; e++)
    KG_CHECK(env_ids[e] >= 0 && env_ids[e] < P.env_count, "Environment Id provided (" + std::to_string(env_ids[e]) +
                                                              ") exceeds the maximum environment count defined (>= " +
                                                              std::to_string(P.env_count) + ").");
  KG_HIP(hipMemcpyAsync(h->h_states, states, (size_t)P.E * P.S * 4, hipMemcpyHostToDevice, h->stream));
  KG_HIP(hipMemcpyAsync(h->h_ids, env_ids, (size_t)P.E * 4, hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(k_vr_host_launch, dim3(vr_blocks(P.E, 256)), dim3(256), 0, h->stream, P, (const State *)h->st,
                     h->ev, h->X, (const float *)h->h_states, (const int *)h->h_ids);
  KG_HIP(hipGetLastError());
  return vr_read_state(h);
}

int kg_vracer_host_act(kg_vracer_t h, float *actions) {
  KG_CHECK(h && actions, "vracer: null argument");
  const Params &P = h->P;
  KG_CHECK(P.host, "vracer: the agent was created for the CartPole kernel, not a host environment");
  {
    VrStage te(h, "environment_step");
    if (vr_forward(h, h->X, P.E, h->out)) return 1;
    hipLaunchKernelGGL(k_vr_host_act, dim3(vr_blocks(P.E, 256)), dim3(256), 0, h->stream, P, h->st, h->ev,
                       (const float *)h->out, (const float *)h->X,
                       h->use_forced_noise ? (const float *)h->forced_noise : nullptr, h->h_act);
    KG_HIP(hipGetLastError());
  }
  h->use_forced_noise = 0;
  KG_HIP(hipMemcpyAsync(actions, h->h_act, (size_t)P.E * P.A * 4, hipMemcpyDeviceToHost, h->stream));
  KG_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int kg_vracer_host_feed(kg_vracer_t h, const float *rewards, const float *states, const int *terminations,
                        const float *next_states, const int *next_env_ids, size_t *new_experiences) {
  KG_CHECK(h && rewards && states && terminations && next_states && next_env_ids, "vracer: null argument");
  const Params &P = h->P;
  KG_CHECK(P.host, "vracer: the agent was created for the CartPole kernel, not a host environment");
  for (int e = 0; e < P.E; e++) {
    KG_CHECK(terminations[e] >= 0 && terminations[e] <= 2, "vracer: terminations must be 0, 1 (Terminal) or 2 (Truncated)");
    KG_CHECK(terminations[e] == 0 || (next_env_ids[e] >= 0 && next_env_ids[e] < P.env_count),
             "Environment Id provided (" + std::to_string(next_env_ids[e]) +
                 ") exceeds the maximum environment count defined (>= " + std::to_string(P.env_count) + ").");
  }
  {
    VrStage te(h, "environment_step");
    KG_HIP(hipMemcpyAsync(h->h_rew, rewards, (size_t)P.E * 4, hipMemcpyHostToDevice, h->stream));
    KG_HIP(hipMemcpyAsync(h->h_states, states, (size_t)P.E * P.S * 4, hipMemcpyHostToDevice, h->stream));
    KG_HIP(hipMemcpyAsync(h->h_term, terminations, (size_t)P.E * 4, hipMemcpyHostToDevice, h->stream));
    KG_HIP(hipMemcpyAsync(h->h_next, next_states, (size_t)P.E * P.S * 4, hipMemcpyHostToDevice, h->stream));
    KG_HIP(hipMemcpyAsync(h->h_ids, next_env_ids, (size_t)P.E * 4, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(k_vr_host_feed, dim3(vr_blocks(P.E, 256)), dim3(256), 0, h->stream, P, h->st, h->ev, h->X,
                       (const float *)h->h_rew, (const float *)h->h_states, (const int *)h->h_term);
    if (vr_forward(h, h->X, P.E, h->outF)) return 1;  // V of truncated states (agent.cpp.base:530-545)
    hipLaunchKernelGGL(k_vr_scan, dim3(1), dim3(1024), 0, h->stream, P, h->st, h->ev);
    hipLaunchKernelGGL(k_vr_evict, dim3(1), dim3(256), 0, h->stream, P, h->st, h->er);
    if (P.rr) hipLaunchKernelGGL(k_vr_reward_sums, dim3(1), dim3(64), 0, h->stream, P, h->st, h->er, h->ev);
    hipLaunchKernelGGL(k_vr_append, dim3(P.E), dim3(256), 0, h->stream, P, h->st, h->er, h->ev,
                       (const float *)h->outF, h->X, (const float *)h->h_next, (const int *)h->h_ids);
    KG_HIP(hipGetLastError());
  }
  if (vr_read_state(h)) return 1;
  h->session_experiences += h->st_host->step_new;
  if (new_experiences) *new_experiences = (size_t)h->st_host->step_new;
  return 0;
}

int kg_vracer_rescale_states(kg_vracer_t h) {
  KG_CHECK(h, "vracer: null argument");
  const Params &P = h->P;
  KG_CHECK(P.srs, "vracer: State Rescaling is not enabled for this agent");
  KG_CHECK(h->st_host->size > 0, "vracer: State Rescaling needs experiences in the replay memory");
  hipLaunchKernelGGL(k_vr_srs_moments, dim3(1), dim3(64), 0, h->stream, P, h->st, h->er);
  const long long n = std::max<long long>((long long)h->st_host->size * P.S, P.E);
  hipLaunchKernelGGL(k_vr_srs_apply, dim3(vr_blocks(n, 256)), dim3(256), 0, h->stream, P, (const State *)h->st, h->er,
                     h->ev, h->X);
  KG_HIP(hipGetLastError());
  return vr_read_state(h);
}

// a graph's mini-batches drawn up front (k_vr_draw_ahead + k_vr_gather_in:
// update 60.9 -> 55.1 us, C5 16.6 k -> 18.4 k experiences/s, round 5;
// KORALI_AMD_VR_DRAW_AHEAD=0: k_vr_minibatch + k_vr_fwd_in per update)
static bool vr_draw_ahead() {
  const char *e = getenv("KORALI_AMD_VR_DRAW_AHEAD");
  return !(e && *e == '0');
}

// updates per captured graph (KORALI_AMD_VR_GRAPH; 0: every update launched
// kernel by kernel).  The fused forward pass advances a host-chosen cursor,
// so it is never captured.
static int vr_graph_len(const Params &P) {
  const char *e = getenv("KORALI_AMD_VR_GRAPH");
  const int n = e ? atoi(e) : 64;
  const char *fe = getenv("KORALI_AMD_VR_FUSED");
  if (P.H <= 256 && fe && *fe == '1') return 0;
  return n < 0 ? 0 : n > 256 ? 256 : n;
}

static int vr_capture_updates(kg_vracer_t h, int n) {
  const int prof = h->prof;
  h->prof = 0;  // no stage events inside the graph
  const size_t nk = (size_t)n * h->P.B;
  if (h->drawCap < nk) {  // (before the capture: no allocation inside it)
    if (h->drawKeys) kg::dev_release(h->drawKeys);
    h->drawKeys = nullptr;
    h->drawCap = 0;
    KG_HIP(kg::dev_alloc((void **)&h->drawKeys, nk * sizeof(unsigned)));
    h->drawCap = nk;
  }
  hipGraph_t g = nullptr;
  KG_HIP(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  int rc = 0;
  if (vr_draw_ahead()) {
    hipLaunchKernelGGL(k_vr_draw_ahead, dim3(n), dim3(256), 0, h->stream, h->P, (const State *)h->st, h->drawKeys);
    for (int i = 0; i < n && !rc; i++) rc = vr_update(h, nullptr, h->drawKeys + (size_t)i * h->P.B);
  } else {
    for (int i = 0; i < n && !rc; i++) rc = vr_update(h, nullptr);
  }
  const hipError_t e = hipStreamEndCapture(h->stream, &g);
  h->prof = prof;
  if (rc || e != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    KG_CHECK(rc == 0 && e == hipSuccess, "vracer: capturing the policy updates failed");
    return 1;
  }
  const hipError_t ie = hipGraphInstantiate(&h->upd_graph, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  KG_HIP(ie);
  h->upd_graph_n = n;
  return 0;
}

int kg_vracer_train_policy(kg_vracer_t h, size_t updates) {
  KG_CHECK(h, "vracer: null argument");
  size_t u = 0;
  const int G = vr_graph_len(h->P);
  if (G > 0 && updates >= (size_t)G) {
    KG_CHECK(h->st_host->size >= 2, "vracer: policy updates need at least two experiences in the replay memory");
    if (h->upd_graph && h->upd_graph_n != G) {
      KG_HIP(hipStreamSynchronize(h->stream));
      KG_HIP(hipGraphExecDestroy(h->upd_graph));
      h->upd_graph = nullptr;
    }
    if (!h->upd_graph && vr_capture_updates(h, G)) return 1;
    for (; u + G <= updates; u += G) {
      VrStage tu(h, "update", (size_t)G);
      KG_HIP(hipGraphLaunch(h->upd_graph, h->stream));
    }
  }
  for (; u < updates; u++)
    if (vr_update(h, nullptr)) return 1;
  h->session_updates += updates;
  return 0;
}

int kg_vracer_train_policy_minibatch(kg_vracer_t h, const uint32_t *ids, size_t count) {
  KG_CHECK(h && ids, "vracer: null argument");
  KG_CHECK(count == (size_t)h->P.B, "vracer: the mini-batch must hold Mini Batch Size ids");
  for (size_t i = 1; i < count; i++) KG_CHECK(ids[i - 1] <= ids[i], "vracer: mini-batch ids must be sorted");
  KG_CHECK(ids[count - 1] < h->st_host->size, "vracer: mini-batch id beyond the replay memory size");
  KG_HIP(hipMemcpyAsync(h->forced_mb, ids, count * 4, hipMemcpyHostToDevice, h->stream));
  if (vr_update(h, h->forced_mb)) return 1;
  h->session_updates += 1;
  return 0;
}

int kg_vracer_train_pending(kg_vracer_t h, size_t *updates) {
  KG_CHECK(h, "vracer: null argument");
  size_t n = 0;
  // Agent::trainingGeneration (agent.cpp.base:201-231)
  if (h->st_host->experience_count >= h->start_size) {
    if (h->P.srs && h->st_host->update_count == 0 && kg_vracer_rescale_states(h)) return 1;
    while ((double)h->session_experiences > h->ebpu * (double)(h->session_updates + n) + (double)h->until_start) n++;
  }
  if (n && kg_vracer_train_policy(h, n)) return 1;
  if (updates) *updates = n;
  return 0;
}

int kg_vracer_training_step(kg_vracer_t h, size_t *new_experiences, size_t *updates) {
  KG_CHECK(h, "vracer: null argument");
  KG_CHECK(!h->P.host, "vracer: a host environment steps through kg_vracer_host_act / kg_vracer_host_feed");
  size_t added = 0;
  if (kg_vracer_environment_step(h, &added)) return 1;
  if (kg_vracer_train_pending(h, updates)) return 1;
  if (new_experiences) *new_experiences = added;
  return 0;
}

// The agent's whole training state (Agent::serializeExperienceReplay /
// deserializeExperienceReplay, agent.cpp.base:849-976, which write the replay
// memory to <result path>/state.json): here every device buffer — the replay
// memory, the concurrent environments' episodes in flight, the policy and its
// Adam moments, the agent scalars and counters — and the host session
// counters, in one binary file, so that a resumed run continues bit for bit.
namespace {
constexpr char VR_STATE_MAGIC[8] = {'K', 'G', 'V', 'R', 'S', 'T', '0', '1'};
struct VrHostState {
  unsigned long long session_experiences, session_updates, until_start, start_size;
  double ebpu;
  int use_forced_noise;
};
}  // namespace

int kg_vracer_save_state(kg_vracer_t h, const char *path, const void *user, size_t user_bytes) {
  KG_CHECK(h && path && (user || !user_bytes), "vracer: null argument");
  KG_HIP(hipStreamSynchronize(h->stream));
  // written to <path>.tmp, flushed and synced, then renamed over <path>: a
  // crash during a save leaves the previous checkpoint intact
  const std::string tmpPath = std::string(path) + ".tmp";
  FILE *f = fopen(tmpPath.c_str(), "wb");
  KG_CHECK(f, std::string("vracer: cannot write the training state file ") + tmpPath);
  bool ok = fwrite(VR_STATE_MAGIC, 1, 8, f) == 8;
  const unsigned long long psz = sizeof(Params), nb = h->bufs.size(), ub = user_bytes;
  ok = ok && fwrite(&psz, 8, 1, f) == 1 && fwrite(&h->P, sizeof(Params), 1, f) == 1 && fwrite(&nb, 8, 1, f) == 1;
  for (auto &b : h->bufs) {
    const unsigned long long n = b.second;
    ok = ok && fwrite(&n, 8, 1, f) == 1;
  }
  const VrHostState hs{h->session_experiences, h->session_updates, h->until_start, h->start_size, h->ebpu,
                       h->use_forced_noise};
  ok = ok && fwrite(&hs, sizeof hs, 1, f) == 1 && fwrite(&ub, 8, 1, f) == 1;
  if (ub) ok = ok && fwrite(user, 1, ub, f) == ub;
  std::vector<unsigned char> tmp;
  for (auto &b : h->bufs) {
    if (!ok) break;
    tmp.resize(b.second);
    if (hipMemcpy(tmp.data(), *b.first, b.second, hipMemcpyDeviceToHost) != hipSuccess) {
      fclose(f);
      remove(tmpPath.c_str());
      KG_CHECK(false, "vracer: reading a device buffer for the training state failed");
    }
    ok = fwrite(tmp.data(), 1, b.second, f) == b.second;
  }
  ok = ok && fflush(f) == 0 && fsync(fileno(f)) == 0;
  ok = (fclose(f) == 0) && ok;
  if (!ok) remove(tmpPath.c_str());
  KG_CHECK(ok, std::string("vracer: writing the training state file failed: ") + tmpPath);
  KG_CHECK(rename(tmpPath.c_str(), path) == 0, std::string("vracer: cannot move the training state into ") + path);
  return 0;
}

int kg_vracer_load_state(kg_vracer_t h, const char *path, void *user, size_t user_capacity, size_t *user_bytes) {
  KG_CHECK(h && path, "vracer: null argument");
  FILE *f = fopen(path, "rb");
  KG_CHECK(f, std::string("Trying to resume training or test policy but could not find or deserialize agent's state "
                          "from file ") + path);
  auto bad = [&](const char *why) {
    fclose(f);
    kg::set_error(std::string("vracer: training state file ") + path + ": " + why);
    return 1;
  };
  char magic[8];
  unsigned long long psz = 0, nb = 0, ub = 0;
  Params Pf;
  if (fread(magic, 1, 8, f) != 8 || memcmp(magic, VR_STATE_MAGIC, 8) != 0) return bad("not a VRACER state file");
  if (fread(&psz, 8, 1, f) != 1 || psz != sizeof(Params) || fread(&Pf, sizeof(Params), 1, f) != 1)
    return bad("agent layout mismatch");
  {  // the same agent apart from the seed (a resumed experiment's seed counter moved on)
    Params a = h->P, b = Pf;
    a.seed = b.seed = 0;
    if (memcmp(&a, &b, sizeof(Params)) != 0) return bad("saved by an agent of another configuration");
  }
  if (fread(&nb, 8, 1, f) != 1 || nb != h->bufs.size()) return bad("buffer count mismatch");
  for (auto &b : h->bufs) {
    unsigned long long n = 0;
    if (fread(&n, 8, 1, f) != 1 || n != b.second) return bad("buffer size mismatch");
  }
  VrHostState hs;
  if (fread(&hs, sizeof hs, 1, f) != 1 || fread(&ub, 8, 1, f) != 1) return bad("truncated");
  std::vector<unsigned char> u(ub);
  if (ub && fread(u.data(), 1, ub, f) != ub) return bad("truncated");
  if (ub > user_capacity) return bad("user block larger than the caller's buffer");
  // every buffer is read into host memory before the first upload: a short
  // or truncated file leaves the handle untouched
  std::vector<std::vector<unsigned char>> all(h->bufs.size());
  for (size_t i = 0; i < h->bufs.size(); i++) {
    all[i].resize(h->bufs[i].second);
    if (fread(all[i].data(), 1, all[i].size(), f) != all[i].size()) return bad("truncated");
  }
  fclose(f);
  KG_HIP(hipStreamSynchronize(h->stream));
  for (size_t i = 0; i < h->bufs.size(); i++)
    KG_CHECK(hipMemcpy(*h->bufs[i].first, all[i].data(), all[i].size(), hipMemcpyHostToDevice) == hipSuccess,
             std::string("vracer: training state file ") + path + ": upload failed");
  h->P.seed = Pf.seed;
  if (h->upd_graph) {  // (captured with the old parameters)
    KG_HIP(hipGraphExecDestroy(h->upd_graph));
    h->upd_graph = nullptr;
  }
  h->session_experiences = hs.session_experiences, h->session_updates = hs.session_updates;
  h->until_start = hs.until_start, h->start_size = hs.start_size, h->ebpu = hs.ebpu;
  h->use_forced_noise = hs.use_forced_noise;
  if (ub) memcpy(user, u.data(), ub);
  if (user_bytes) *user_bytes = ub;
  return vr_read_state(h);
}

int kg_vracer_synchronize(kg_vracer_t h) {
  KG_CHECK(h, "vracer: null argument");
  return vr_read_state(h);
}

int kg_vracer_profile(kg_vracer_t h, int enable) {
  KG_CHECK(h, "vracer: null argument");
  if (vr_collect(h)) return 1;
  h->prof = enable ? 1 : 0;
  h->totals.clear();
  return 0;
}

int kg_vracer_profile_read(kg_vracer_t h, const char *stage, double *ms_total, size_t *count) {
  KG_CHECK(h && stage && ms_total && count, "vracer: null argument");
  if (vr_collect(h)) return 1;
  auto it = h->totals.find(stage);
  *ms_total = it == h->totals.end() ? 0.0 : it->second.first;
  *count = it == h->totals.end() ? 0 : it->second.second;
  if (it != h->totals.end()) h->totals.erase(it);
  return 0;
}

int kg_vracer_stream(kg_vracer_t h, void **stream) {
  KG_CHECK(h && stream, "vracer: null argument");
  *stream = (void *)h->stream;
  return 0;
}

}  // extern "C"
