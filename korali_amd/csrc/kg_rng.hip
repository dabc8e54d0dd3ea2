// kg_rng.hip — device GSL mt19937 stream: producer, polar normals, uniforms.
// Semantics: GSL 2.6 rng/mt.c + randist/gauss.c (polar), as called by
// Korali's Normal/Uniform distributions (univariate/normal/normal.cpp.base:
// 32-35, univariate/uniform/uniform.cpp.base:30-36).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kg_rng.hpp"

namespace kg {

namespace {

constexpr int POLAR_TPB = 256;     // threads per block
constexpr int POLAR_APT = 8;       // attempts per thread
constexpr int POLAR_APB = POLAR_TPB * POLAR_APT;

// the stream position and zero-word list, read once per thread (the zero
// list itself stays in global memory: it is empty except once per ~4e9 words)
struct PosView {
  unsigned long long pos;
  unsigned int nzero;
  const unsigned long long *zeros;
};

__device__ inline PosView pos_view(const StreamState *st) {
  return {st->pos, st->nzero < KG_MAX_ZERO_WORDS ? st->nzero : KG_MAX_ZERO_WORDS, st->zeros};
}

__device__ inline unsigned long long compact_to_abs(const PosView &st, unsigned long long c) {
  // absolute index of the c-th non-zero word at/after pos
  unsigned long long j = st.pos + c;
  if (st.nzero == 0) return j;
  for (;;) {
    unsigned int k = 0;
    for (unsigned int i = 0; i < st.nzero; i++)
      if (st.zeros[i] >= st.pos && st.zeros[i] <= j) k++;
    const unsigned long long jn = st.pos + c + k;
    if (jn == j) return j;
    j = jn;
  }
}

// One workgroup, 4 waves: every step produces the next 227 words (the
// recurrence's lag: s_j needs s_{j-624}, s_{j-623}, s_{j-227}), one word per
// thread, from a 1024-word LDS window; one barrier per step.
constexpr int MT_TPB = 256;
__global__ void __launch_bounds__(MT_TPB) k_mt_produce(uint32_t *__restrict__ ring, unsigned long long R,
                                                       StreamState *st, unsigned long long ahead) {
  __shared__ uint32_t L[1024];
  const int t = threadIdx.x;
  const unsigned long long hi0 = st->hi;
  unsigned long long target = st->pos + ahead;
  const unsigned long long cap = st->lo + R;
  if (target > cap) {
    if (t == 0) atomicOr(&st->errors, KG_ERR_RNG_UNDERRUN);
    target = cap;
  }
  if (hi0 >= target) return;
  for (int i = t; i < MT_N; i += MT_TPB) {
    const unsigned long long j = hi0 - MT_N + i;
    L[j & 1023] = ring[j & (R - 1)];
  }
  __syncthreads();
  for (unsigned long long c = hi0; c < target; c += 227) {
    const int cnt = (int)((target - c) < 227 ? (target - c) : 227);
    if (t < cnt) {
      const unsigned long long j = c + t;
      const uint32_t s = mt_next(L[(j - 624) & 1023], L[(j - 623) & 1023], L[(j - 227) & 1023]);
      L[j & 1023] = s;
      ring[j & (R - 1)] = s;
      if (s == 0u) {  // tempered word is zero iff untempered is (bijection)
        const unsigned int z = atomicAdd(&st->nzero, 1u);
        if (z < KG_MAX_ZERO_WORDS)
          st->zeros[z] = j;
        else
          atomicOr(&st->errors, KG_ERR_ZERO_LIST);
      }
    }
    __syncthreads();
  }
  if (t == 0) st->hi = target;
}

// ---- chunked production (see kg_rng.hpp ChunkPlan, kg_mtjump.hip) ----
// out[m] = XOR_{i: bit i of poly} seq[m + i], m < 624 (256 threads, three
// outputs each; the bit loop is uniform, the reads consecutive across lanes)
// the partial combination over the polynomial's words [w0, w1).  The set
// bits' indices are found on the scalar unit (the polynomial is uniform),
// eight at a time, so a batch is eight address adds, 24 LDS reads in flight
// and 24 XORs per wave; a batch's unused slots read the zero pad at
// MT_ZPAD (XOR with 0).  (One set bit at a time with its three reads waited
// for, or with per-lane bit arithmetic, made the combine the producer's
// dominant cost: ~300 us per chunk workgroup at C2, round 5.)
constexpr int MT_ZPAD = ((MT_SEQ + 3) & ~3) + 1024;  // 768 zero words after the rolling window
__device__ __forceinline__ void mt_zero_pad(uint32_t *lds) {
  for (int i = threadIdx.x; i < 768; i += blockDim.x) lds[MT_ZPAD + i] = 0u;
}
__device__ __forceinline__ void mt_combine_words(const uint32_t *seq, const uint64_t *__restrict__ poly, int w0,
                                                 int w1, uint32_t &a0, uint32_t &a1, uint32_t &a2) {
  const int t = threadIdx.x;
  for (int w = w0; w < w1; w++) {
    const uint64_t pw = poly[w];
    unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)pw), hi = __builtin_amdgcn_readfirstlane((unsigned)(pw >> 32));
    uint64_t bits = ((uint64_t)hi << 32) | lo;
    while (bits) {
      int idx[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        idx[u] = bits ? w * 64 + __builtin_ctzll(bits) : MT_ZPAD;
        bits &= bits - 1;  // (0 stays 0)
      }
      uint32_t r0[8], r1[8], r2[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t *p = seq + t + idx[u];
        r0[u] = p[0], r1[u] = p[256], r2[u] = p[512];  // (lanes t >= 112: p[512] unused)
      }
#pragma unroll
      for (int u = 0; u < 8; u++) a0 ^= r0[u], a1 ^= r1[u], a2 ^= r2[u];
    }
  }
}

// seq[624 .. lim) from the window seq[0..624); optionally also stored to
// the ring at absolute positions base + k - 624 (zero words recorded)
__device__ inline void mt_fill_seq(uint32_t *seq, uint32_t *ring, unsigned long long R, StreamState *st,
                                   unsigned long long base, int lim = MT_SEQ) {
  const int t = threadIdx.x;
  for (int k0 = MT_N; k0 < lim; k0 += 227) {
    const int k = k0 + t;
    if (t < 227 && k < lim) {
      const uint32_t v = mt_next(seq[k - 624], seq[k - 623], seq[k - 227]);
      seq[k] = v;
      if (ring) {
        const unsigned long long j = base + (unsigned long long)(k - MT_N);
        ring[j & (R - 1)] = v;
        if (v == 0u) {
          const unsigned int z = atomicAdd(&st->nzero, 1u);
          if (z < KG_MAX_ZERO_WORDS)
            st->zeros[z] = j;
          else
            atomicOr(&st->errors, KG_ERR_ZERO_LIST);
        }
      }
    }
    __syncthreads();
  }
}

__global__ void k_mt_plan(StreamState *st, ChunkPlan *plan, unsigned long long ahead, unsigned long long R,
                          unsigned long long W, unsigned long long K) {
  if (threadIdx.x != 0) return;
  unsigned long long target = st->pos + ahead;
  const unsigned long long cap = st->lo + R, hi = st->hi;
  if (target > cap) {
    st->errors |= KG_ERR_RNG_UNDERRUN;
    target = cap;
  }
  unsigned long long n = 0;
  if (hi < target) {
    n = (target - hi + W - 1) / W;
    if (n > K) n = K;
    while (n > 0 && hi + n * W > cap) n--;
  }
  plan->c_first = hi / W;
  plan->n = n;
  st->hi = hi + n * W;
}

// Seed windows live in 3K slots (chunk c's in slot c mod 3K).  Workgroups
// [0, K) produce chunks; workgroups K + q parts + r jump chunk q's start
// window K W words ahead, part r of the polynomial's words each, XOR-ing
// into slot (c + K) mod 3K, which the producer of chunk c - K zeroed in an
// earlier launch (a launch holds at most K consecutive chunks, so the slots
// read (c), written (c + K) and zeroed (c + 2K) by one launch are disjoint).
// (One workgroup producing AND jumping made the ~10^4-term combine the
// chunk's critical path: 214 us per C2 launch, round 5.)
__global__ void __launch_bounds__(MT_TPB) k_mt_chunks(uint32_t *__restrict__ ring, unsigned long long R,
                                                     StreamState *st, const ChunkPlan *__restrict__ plan,
                                                     uint32_t *__restrict__ seeds, unsigned long long K,
                                                     unsigned long long W, const uint64_t *__restrict__ jumpPoly,
                                                     int parts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t msm[];
  uint32_t *seq = msm, *roll = msm + ((MT_SEQ + 3) & ~3);
  const ChunkPlan pl = *plan;
  const int t = threadIdx.x;
  if (blockIdx.x >= K) {
    const unsigned long long q = (blockIdx.x - K) / parts;
    const int part = (int)((blockIdx.x - K) % parts);
    if (q >= pl.n) return;
    const unsigned long long c = pl.c_first + q;
    const int w0 = part * MT_POLY_WORDS / parts, w1 = (part + 1) * MT_POLY_WORDS / parts;
    const uint32_t *src = seeds + (size_t)(c % (3 * K)) * MT_N;
    mt_zero_pad(msm);
    for (int i = t; i < MT_N; i += MT_TPB) seq[i] = src[i];
    __syncthreads();
    mt_fill_seq(seq, nullptr, 0, nullptr, 0, min(MT_SEQ, MT_N - 1 + 64 * w1));  // terms i < 64 w1
    uint32_t a0 = 0, a1 = 0, a2 = 0;
    mt_combine_words(seq, jumpPoly, w0, w1, a0, a1, a2);
    uint32_t *out = seeds + (size_t)((c + K) % (3 * K)) * MT_N;
    atomicXor(out + t, a0);
    atomicXor(out + t + 256, a1);
    if (t + 512 < MT_N) atomicXor(out + t + 512, a2);
    return;
  }
  if (blockIdx.x >= pl.n) return;
  const unsigned long long c = pl.c_first + blockIdx.x;
  const uint32_t *src = seeds + (size_t)(c % (3 * K)) * MT_N;
  for (int i = t; i < MT_N; i += MT_TPB) seq[i] = src[i];
  {  // chunk c - K's window: read in an earlier launch; chunk c + K's jump fills it
    uint32_t *old = seeds + (size_t)((c + 2 * K) % (3 * K)) * MT_N;
    for (int i = t; i < MT_N; i += MT_TPB) old[i] = 0u;
  }
  __syncthreads();
  const unsigned long long base = c * W;
  mt_fill_seq(seq, ring, R, st, base);  // words base .. base + MT_SEQ - 625
  // rest of the chunk from a rolling 1024-word window
  const unsigned long long j0 = base + (MT_SEQ - MT_N);
  for (int i = t; i < MT_N; i += MT_TPB) roll[(j0 - MT_N + i) & 1023] = seq[MT_SEQ - MT_N + i];
  __syncthreads();
  for (unsigned long long c0 = j0; c0 < base + W; c0 += 227) {
    const unsigned long long j = c0 + t;
    if (t < 227 && j < base + W) {
      const uint32_t v = mt_next(roll[(j - 624) & 1023], roll[(j - 623) & 1023], roll[(j - 227) & 1023]);
      roll[j & 1023] = v;
      ring[j & (R - 1)] = v;
      if (v == 0u) {
        const unsigned int z = atomicAdd(&st->nzero, 1u);
        if (z < KG_MAX_ZERO_WORDS)
          st->zeros[z] = j;
        else
          atomicOr(&st->errors, KG_ERR_ZERO_LIST);
      }
    }
    __syncthreads();
  }
}

// initial seeds: chunk c0 + k (2^l <= k < 2^(l+1)) from chunk c0 + k - 2^l.
// A jump is a XOR over the ~10^4 set bits of its polynomial; the words of
// the polynomial are split over MT_JUMP_PARTS workgroups per window, each
// extending the sequence only as far as its terms read and XOR-ing its
// partial sums into the (zeroed) output window.  Eight levels seed 256
// chunks once per handle: one workgroup per window made that ~3.2 ms of
// the handle's creation (C2, KORALI_AMD_RUN_PHASES).
constexpr int MT_JUMP_PARTS = 16;
__global__ void __launch_bounds__(MT_TPB) k_mt_jump_level(uint32_t *__restrict__ seeds, unsigned long long K,
                                                         unsigned long long c0, int l,
                                                         const uint64_t *__restrict__ poly) {
  extern __shared__ __attribute__((aligned(16))) uint32_t msm[];
  const unsigned long long k = (1ULL << l) + blockIdx.x / MT_JUMP_PARTS;
  const int part = (int)(blockIdx.x % MT_JUMP_PARTS);
  if (k >= K) return;
  const int w0 = part * MT_POLY_WORDS / MT_JUMP_PARTS, w1 = (part + 1) * MT_POLY_WORDS / MT_JUMP_PARTS;
  const uint32_t *src = seeds + (size_t)((c0 + k - (1ULL << l)) % (3 * K)) * MT_N;
  mt_zero_pad(msm);
  for (int i = threadIdx.x; i < MT_N; i += MT_TPB) msm[i] = src[i];
  __syncthreads();
  // terms i < 64 w1 read seq[m + i], m < 624
  mt_fill_seq(msm, nullptr, 0, nullptr, 0, min(MT_SEQ, MT_N - 1 + 64 * w1));
  const int t = threadIdx.x;
  uint32_t a0 = 0, a1 = 0, a2 = 0;
  mt_combine_words(msm, poly, w0, w1, a0, a1, a2);
  uint32_t *out = seeds + (size_t)((c0 + k) % (3 * K)) * MT_N;
  atomicXor(out + t, a0);
  atomicXor(out + t + 256, a1);
  if (t + 512 < MT_N) atomicXor(out + t + 512, a2);
}

size_t mt_chunk_lds_bytes() { return (size_t)(MT_ZPAD + 768) * sizeof(uint32_t); }

__device__ inline bool polar_pair(const uint32_t *__restrict__ ring, unsigned long long R, const PosView &st,
                                  unsigned long long a, double &y, double &r2) {
  const unsigned long long j0 = compact_to_abs(st, 2 * a), j1 = compact_to_abs(st, 2 * a + 1);
  const uint32_t w0 = mt_temper(ring[j0 & (R - 1)]), w1 = mt_temper(ring[j1 & (R - 1)]);
  const double u0 = w0 / 4294967296.0, u1 = w1 / 4294967296.0;
  const double x = -1 + 2 * u0;
  y = -1 + 2 * u1;
  r2 = x * x + y * y;
  return !(r2 > 1.0 || r2 == 0);
}

__global__ void __launch_bounds__(POLAR_TPB) k_polar_count(const uint32_t *__restrict__ ring, unsigned long long R,
                                                          const StreamState *__restrict__ stp, unsigned long long A,
                                                          unsigned int *__restrict__ counts) {
  __shared__ unsigned int wsum[POLAR_TPB / 64];
  const PosView st = pos_view(stp);
  const unsigned long long base = (unsigned long long)blockIdx.x * POLAR_APB + threadIdx.x * POLAR_APT;
  unsigned int c = 0;
#pragma unroll
  for (int q = 0; q < POLAR_APT; q++) {
    const unsigned long long a = base + q;
    double y, r2;
    if (a < A && polar_pair(ring, R, st, a, y, r2)) c++;
  }
  // block reduction
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int t = 0;
    for (int w = 0; w < POLAR_TPB / 64; w++) t += wsum[w];
    counts[blockIdx.x] = t;
  }
}

// exclusive scan of nb block counts (single block); offsets[nb] = total
__global__ void __launch_bounds__(1024) k_scan_counts(const unsigned int *__restrict__ counts, unsigned long long *__restrict__ offsets,
                                                      int nb, StreamState *st) {
  __shared__ unsigned long long wtot[16];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    unsigned long long v = (i < nb) ? counts[i] : 0;
    // inclusive wave scan
    unsigned long long x = v;
    for (int off = 1; off < 64; off <<= 1) {
      unsigned long long t = __shfl_up(x, off, 64);
      if (lane >= off) x += t;
    }
    if (lane == 63) wtot[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long acc = 0;
      for (int w = 0; w < 16; w++) {
        unsigned long long t = wtot[w];
        wtot[w] = acc;
        acc += t;
      }
    }
    __syncthreads();
    const unsigned long long excl = carry + wtot[wid] + x - v;
    if (i < nb) offsets[i] = excl;
    __syncthreads();
    if (threadIdx.x == 1023) carry = excl + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    offsets[nb] = carry;
    st->total_normals = carry;
  }
}

__global__ void __launch_bounds__(POLAR_TPB) k_polar_scatter(const uint32_t *__restrict__ ring, unsigned long long R,
                                                            StreamState *__restrict__ stp, unsigned long long A,
                                                            const unsigned long long *__restrict__ offsets,
                                                            double *__restrict__ z, unsigned long long M,
                                                            unsigned long long block_len,
                                                            unsigned long long *__restrict__ block_end,
                                                            unsigned long long k_lo, unsigned long long k_hi) {
  __shared__ unsigned int woff[POLAR_TPB / 64];
  // the wave's normals in order: a wave's lanes hold consecutive ranges of
  // normal indices, so each wave stages its normals here and stores them
  // contiguously (a lane storing its own few 8-byte normals wrote 2.08x the
  // normals' bytes to HBM at C4, round-4 PMC)
  __shared__ double zbuf[POLAR_TPB / 64][64 * POLAR_APT];
  const PosView st = pos_view(stp);
  const unsigned long long base = (unsigned long long)blockIdx.x * POLAR_APB + threadIdx.x * POLAR_APT;
  double yv[POLAR_APT], rv[POLAR_APT];
  unsigned int acc = 0, mask = 0;
#pragma unroll
  for (int q = 0; q < POLAR_APT; q++) {
    const unsigned long long a = base + q;
    if (a < A && polar_pair(ring, R, st, a, yv[q], rv[q])) {
      mask |= 1u << q;
      acc++;
    }
  }
  // exclusive scan of per-thread counts across the block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned int x = acc;
  for (int off = 1; off < 64; off <<= 1) {
    unsigned int t = __shfl_up(x, off, 64);
    if (lane >= off) x += t;
  }
  if (lane == 63) woff[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int s = 0;
    for (int w = 0; w < POLAR_TPB / 64; w++) {
      unsigned int t = woff[w];
      woff[w] = s;
      s += t;
    }
  }
  __syncthreads();
  const unsigned long long kw = offsets[blockIdx.x] + woff[wid];  // the wave's first normal
  const unsigned int wt = (unsigned int)__shfl(x, 63, 64);          // the wave's normals
  unsigned long long k = kw + (x - acc);
#pragma unroll
  for (int q = 0; q < POLAR_APT; q++) {
    if (mask & (1u << q)) {
      if (k < M) {
        // gsl_ran_gaussian: sigma * y * sqrt(-2 log(r2) / r2); Normal adds mean 0
        // (only normals k in [k_lo, k_hi) are materialised: a population shard)
        if (k >= k_lo && k < k_hi) {
          const double r2 = rv[q];
          const double g = 1.0 * yv[q] * sqrt(-2.0 * log_cr(r2) / r2);
          zbuf[wid][k - kw] = 0.0 + g;
        }
        if (block_end && ((k + 1) % block_len) == 0) block_end[(k + 1) / block_len - 1] = base + q;
        if (k == M - 1) stp->last_attempt = base + q;
      }
      k++;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (unsigned int i = lane; i < wt; i += 64) {
    const unsigned long long kk = kw + i;
    if (kk < M && kk >= k_lo && kk < k_hi) z[kk - k_lo] = zbuf[wid][i];
  }
}

// advance the stream by the words behind `attempts` polar attempts
__global__ void k_consume(StreamState *st, unsigned long long normals_used, unsigned long long block_len,
                          const unsigned long long *block_end, int use_block_end,
                          const unsigned long long *used_blocks_dev) {
  if (threadIdx.x != 0) return;
  if (used_blocks_dev) normals_used = (*used_blocks_dev) * block_len;
  if (normals_used == 0) return;
  if (st->total_normals < normals_used) {
    st->errors |= KG_ERR_RNG_UNDERRUN;
    return;
  }
  const unsigned long long last = use_block_end ? block_end[normals_used / block_len - 1] : st->last_attempt;
  const unsigned long long words = 2 * (last + 1);
  const unsigned long long p = compact_to_abs(pos_view(st), words - 1) + 1;
  if (p > st->hi) st->errors |= KG_ERR_RNG_UNDERRUN;
  st->pos = p;
  st->lo = 624ULL * ((p - 1) / 624ULL);
  // drop zero records that are behind the new position
  unsigned int w = 0;
  for (unsigned int i = 0; i < st->nzero && i < KG_MAX_ZERO_WORDS; i++)
    if (st->zeros[i] >= p) st->zeros[w++] = st->zeros[i];
  st->nzero = w;
}

__global__ void k_uniforms(const uint32_t *__restrict__ ring, unsigned long long R, const StreamState *__restrict__ stp,
                           double *__restrict__ u, unsigned long long M) {
  const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const unsigned long long j = stp->pos + i;
  u[i] = mt_temper(ring[j & (R - 1)]) / 4294967296.0;
}

__global__ void k_consume_words(StreamState *st, unsigned long long words, const unsigned long long *wordsDev) {
  if (wordsDev) words = *wordsDev;
  if (threadIdx.x != 0 || words == 0) return;
  const unsigned long long p = st->pos + words;
  if (p > st->hi) st->errors |= KG_ERR_RNG_UNDERRUN;
  st->pos = p;
  st->lo = 624ULL * ((p - 1) / 624ULL);
  unsigned int w = 0;
  for (unsigned int i = 0; i < st->nzero && i < KG_MAX_ZERO_WORDS; i++)
    if (st->zeros[i] >= p) st->zeros[w++] = st->zeros[i];
  st->nzero = w;
}

unsigned long long next_pow2(unsigned long long x) {
  unsigned long long r = 1;
  while (r < x) r <<= 1;
  return r;
}

}  // namespace

void MtStream::drain() {
  if (side_) (void)hipStreamSynchronize(side_);
}

MtStream::~MtStream() {
  drain();
  if (seeds_) dev_release(seeds_);
  if (polys_) dev_release(polys_);
  if (plan_) dev_release(plan_);
  if (side_) {
    (void)hipStreamSynchronize(side_);
    stream_release(side_);
  }
  if (ev_main_) (void)hipEventDestroy(ev_main_);
  if (ev_side_) (void)hipEventDestroy(ev_side_);
  if (ring_) dev_release(ring_);
  if (st_) dev_release(st_);
  if (counts_) dev_release(counts_);
  if (offsets_) dev_release(offsets_);
}

int MtStream::init(size_t capacity_words, size_t parallel_min) {
  if (const char *e = getenv("KORALI_AMD_MT_PARALLEL_MIN")) parallel_min = (size_t)strtoull(e, nullptr, 10);
  par_ = capacity_words >= parallel_min;
  if (par_) {
    // chunk size: 2^15 words for per-generation streams of a few million
    // words (C2: 1.3 M; 128 chunks in flight beat one producer workgroup by
    // 12% of the generation, measured), 2^19 for the very long ones (C4: 85 M)
    int lw = capacity_words < (16u << 20) ? 15 : 19;
    if (const char *e = getenv("KORALI_AMD_MT_CHUNK_LOG2")) lw = atoi(e);
    KG_CHECK(lw >= 15 && lw <= 26, "KORALI_AMD_MT_CHUNK_LOG2 must be in [15, 26]");
    W_ = 1ULL << lw;
    K_ = 256;
    if (const char *e = getenv("KORALI_AMD_MT_CHUNK_PARTS")) parts_ = std::min(64, std::max(1, atoi(e)));  // (A/B)
    int lk = 0;
    while ((1 << lk) < K_) lk++;
    KG_HIP(dev_alloc(&seeds_, 3 * (size_t)K_ * MT_N * sizeof(uint32_t)));
    KG_HIP(dev_alloc(&plan_, sizeof(ChunkPlan)));
    KG_HIP(dev_alloc(&polys_, (size_t)(lk + 1) * MT_POLY_WORDS * sizeof(uint64_t)));
    std::vector<uint64_t> hp((size_t)(lk + 1) * MT_POLY_WORDS);
    for (int l = 0; l <= lk; l++)
      if (mt_jump_poly_pow2(lw + l, hp.data() + (size_t)l * MT_POLY_WORDS)) return 1;
    KG_HIP(hipMemcpy(polys_, hp.data(), hp.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    const int lds = (int)mt_chunk_lds_bytes();
    KG_HIP(allow_dynamic_lds((const void *)k_mt_chunks, lds));
    KG_HIP(allow_dynamic_lds((const void *)k_mt_jump_level, lds));
    capacity_words += W_;  // production rounds up to whole chunks
  }
  R_ = next_pow2(capacity_words + 2 * MT_N + 4096);
  KG_HIP(dev_alloc(&ring_, R_ * sizeof(uint32_t)));
  KG_HIP(dev_alloc(&st_, sizeof(StreamState)));
  if (zero_fill(st_, sizeof(StreamState))) return 1;
  return 0;
}

int MtStream::ensure_scratch(size_t nb) {
  if (nb <= scratch_blocks_) return 0;
  if (counts_ || offsets_) KG_HIP(hipDeviceSynchronize());  // (cached blocks are reused at once)
  if (counts_) dev_release(counts_);
  if (offsets_) dev_release(offsets_);
  KG_HIP(dev_alloc(&counts_, nb * sizeof(unsigned int)));
  KG_HIP(dev_alloc(&offsets_, (nb + 1) * sizeof(unsigned long long)));
  scratch_blocks_ = nb;
  return 0;
}

int MtStream::import_gsl(const void *state5000, hipStream_t s) {
  const unsigned char *b = (const unsigned char *)state5000;
  std::vector<uint32_t> w(MT_N);
  for (int i = 0; i < MT_N; i++) {
    uint64_t v;
    memcpy(&v, b + 8 * i, 8);
    w[i] = (uint32_t)(v & 0xffffffffULL);
  }
  int32_t mti;
  memcpy(&mti, b + 8 * MT_N, 4);
  KG_CHECK(mti >= 0 && mti <= MT_N, "invalid mt19937 state (mti out of range)");
  StreamState h;
  memset(&h, 0, sizeof(h));
  h.lo = 0;
  h.pos = (unsigned long long)mti;
  h.hi = MT_N;
  for (int i = mti; i < MT_N; i++)
    if (w[i] == 0 && h.nzero < KG_MAX_ZERO_WORDS) h.zeros[h.nzero++] = (unsigned long long)i;
  KG_HIP(hipMemcpyAsync(ring_, w.data(), MT_N * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  KG_HIP(hipMemcpyAsync(st_, &h, sizeof(h), hipMemcpyHostToDevice, s));
  if (par_ && seed_chunks(h.pos, s)) return 1;
  KG_HIP(hipStreamSynchronize(s));
  return 0;
}

int MtStream::seed_chunks(unsigned long long pos, hipStream_t s) {
  // serial up to the first chunk boundary W exactly (pos + ahead = W), whose
  // start window seeds chunk 1; chunks 2..K by log-depth jumps (level l
  // jumps 2^l W words)
  hipLaunchKernelGGL(k_mt_produce, dim3(1), dim3(MT_TPB), 0, s, ring_, R_, st_, W_ - pos);
  KG_HIP(hipGetLastError());
  const int K = K_;
  // the levels XOR their partial jumps into zeroed windows
  KG_HIP(hipMemsetAsync(seeds_, 0, 3 * (size_t)K * MT_N * sizeof(uint32_t), s));
  KG_HIP(hipMemcpyAsync(seeds_ + (size_t)(1 % (3 * K)) * MT_N, ring_ + ((W_ - MT_N) & (R_ - 1)),
                        MT_N * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  for (int l = 0; (1 << l) < K; l++) {
    const int cnt = std::min(1 << l, K - (1 << l));
    hipLaunchKernelGGL(k_mt_jump_level, dim3(cnt * MT_JUMP_PARTS), dim3(MT_TPB), mt_chunk_lds_bytes(), s, seeds_,
                       (unsigned long long)K, 1ULL, l, (const uint64_t *)(polys_ + (size_t)l * MT_POLY_WORDS));
    KG_HIP(hipGetLastError());
  }
  return 0;
}

int MtStream::produce_chunks(unsigned long long ahead, hipStream_t s) {
  int lk = 0;
  while ((1 << lk) < K_) lk++;
  const unsigned long long per = (unsigned long long)K_ * W_;
  const unsigned long long launches = (ahead + W_) / per + 1;
  for (unsigned long long q = 0; q < launches; q++) {
    hipLaunchKernelGGL(k_mt_plan, dim3(1), dim3(1), 0, s, st_, plan_, ahead, R_, W_, (unsigned long long)K_);
    KG_HIP(hipGetLastError());
    const int parts = parts_;
    hipLaunchKernelGGL(k_mt_chunks, dim3(K_ * (1 + parts)), dim3(MT_TPB), mt_chunk_lds_bytes(), s, ring_, R_, st_,
                       (const ChunkPlan *)plan_, seeds_, (unsigned long long)K_, W_,
                       (const uint64_t *)(polys_ + (size_t)lk * MT_POLY_WORDS), parts);
    KG_HIP(hipGetLastError());
  }
  return 0;
}

int MtStream::produce(unsigned long long ahead, hipStream_t s) {
  if (par_) return produce_chunks(ahead, s);
  hipLaunchKernelGGL(k_mt_produce, dim3(1), dim3(MT_TPB), 0, s, ring_, R_, st_, ahead);
  KG_HIP(hipGetLastError());
  return 0;
}

int MtStream::export_gsl(void *state5000, hipStream_t s) {
  // the whole current block must exist
  StreamState h;
  KG_HIP(hipMemcpyAsync(&h, st_, sizeof(h), hipMemcpyDeviceToHost, s));
  KG_HIP(hipStreamSynchronize(s));
  if (h.hi < h.lo + MT_N) {
    if (produce(h.lo + MT_N - h.pos, s)) return 1;
    KG_HIP(hipMemcpyAsync(&h, st_, sizeof(h), hipMemcpyDeviceToHost, s));
    KG_HIP(hipStreamSynchronize(s));
  }
  std::vector<uint32_t> w(MT_N);
  const unsigned long long off = h.lo & (R_ - 1);
  if (off + MT_N <= R_) {
    KG_HIP(hipMemcpyAsync(w.data(), ring_ + off, MT_N * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  } else {
    const size_t first = R_ - off;
    KG_HIP(hipMemcpyAsync(w.data(), ring_ + off, first * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    KG_HIP(hipMemcpyAsync(w.data() + first, ring_, (MT_N - first) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  KG_HIP(hipStreamSynchronize(s));
  unsigned char *b = (unsigned char *)state5000;
  memset(b, 0, 5000);
  for (int i = 0; i < MT_N; i++) {
    uint64_t v = w[i];
    memcpy(b + 8 * i, &v, 8);
  }
  int32_t mti = (int32_t)(h.pos - h.lo);
  memcpy(b + 8 * MT_N, &mti, 4);
  return 0;
}

size_t MtStream::words_for_normals(size_t M) const {
  // attempts ~ M / (pi/4); 12 sigma margin of the geometric sum
  const double A = (double)M * 1.2732395447351628 + 12.0 * std::sqrt((double)M * 0.3484) + 64.0;
  return (size_t)(2.0 * A) + 64;
}

int MtStream::prefetch(size_t M, hipStream_t main) {
  if (!side_) {
    KG_HIP(stream_acquire(&side_));
    KG_HIP(hipEventCreateWithFlags(&ev_main_, hipEventDisableTiming));
    KG_HIP(hipEventCreateWithFlags(&ev_side_, hipEventDisableTiming));
  }
  const unsigned long long words = words_for_normals(M);
  KG_HIP(hipEventRecord(ev_main_, main));
  KG_HIP(hipStreamWaitEvent(side_, ev_main_, 0));
  if (produce(2 * (words + 2 * KG_MAX_ZERO_WORDS), side_)) return 1;
  KG_HIP(hipEventRecord(ev_side_, side_));
  prefetch_pending_ = true;
  return 0;
}

int MtStream::polar_normals_ahead(double *z, size_t M, size_t block_len, hipStream_t main) {
  if (!side_) return 1;
  KG_HIP(hipEventRecord(ev_main_, main));
  KG_HIP(hipStreamWaitEvent(side_, ev_main_, 0));
  if (polar_normals(z, M, block_len, nullptr, side_)) return 1;
  KG_HIP(hipEventRecord(ev_side_, side_));
  prefetch_pending_ = true;
  return 0;
}

int MtStream::join(hipStream_t main) {
  if (!side_) return 0;
  KG_HIP(hipEventRecord(ev_side_, side_));
  KG_HIP(hipStreamWaitEvent(main, ev_side_, 0));
  prefetch_pending_ = false;
  return 0;
}

int MtStream::polar_normals(double *z, size_t M, size_t block_len, unsigned long long *block_end, hipStream_t s,
                            size_t k_lo, size_t k_hi) {
  const unsigned long long words = words_for_normals(M);
  const unsigned long long A = words / 2;
  const size_t nb = (size_t)((A + POLAR_APB - 1) / POLAR_APB);
  if (ensure_scratch(nb)) return 1;
  if (prefetch_pending_) {
    KG_HIP(hipStreamWaitEvent(s, ev_side_, 0));
    prefetch_pending_ = false;
  }
  if (produce(words + 2 * KG_MAX_ZERO_WORDS, s)) return 1;
  hipLaunchKernelGGL(k_polar_count, dim3(nb), dim3(POLAR_TPB), 0, s, ring_, R_, st_, A, counts_);
  KG_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, counts_, offsets_, (int)nb, st_);
  KG_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_polar_scatter, dim3(nb), dim3(POLAR_TPB), 0, s, ring_, R_, st_, A, offsets_, z,
                     (unsigned long long)M, (unsigned long long)(block_len ? block_len : 1), block_end,
                     (unsigned long long)k_lo, (unsigned long long)(k_hi < M ? k_hi : M));
  KG_HIP(hipGetLastError());
  return 0;
}

int MtStream::consume_normals(size_t used, size_t block_len, const unsigned long long *block_end, hipStream_t s) {
  hipLaunchKernelGGL(k_consume, dim3(1), dim3(1), 0, s, st_, (unsigned long long)used,
                     (unsigned long long)(block_len ? block_len : 1), block_end, block_end ? 1 : 0,
                     (const unsigned long long *)nullptr);
  KG_HIP(hipGetLastError());
  return 0;
}

int MtStream::consume_normals_dev(const unsigned long long *used_blocks, size_t block_len,
                                  const unsigned long long *block_end, hipStream_t s) {
  hipLaunchKernelGGL(k_consume, dim3(1), dim3(1), 0, s, st_, 0ULL, (unsigned long long)block_len, block_end, 1,
                     used_blocks);
  KG_HIP(hipGetLastError());
  return 0;
}

int MtStream::uniforms(double *u, size_t M, hipStream_t s) {
  if (M == 0) return 0;
  if (produce(M + 2, s)) return 1;
  hipLaunchKernelGGL(k_uniforms, dim3((M + 255) / 256), dim3(256), 0, s, ring_, R_, st_, u, (unsigned long long)M);
  KG_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_consume_words, dim3(1), dim3(1), 0, s, st_, (unsigned long long)M,
                     (const unsigned long long *)nullptr);
  KG_HIP(hipGetLastError());
  return 0;
}

int MtStream::peek_uniforms(double *u, size_t M, hipStream_t s) {
  if (M == 0) return 0;
  if (produce(M + 2, s)) return 1;
  hipLaunchKernelGGL(k_uniforms, dim3((M + 255) / 256), dim3(256), 0, s, ring_, R_, st_, u, (unsigned long long)M);
  KG_HIP(hipGetLastError());
  return 0;
}

int MtStream::consume_words_dev(const unsigned long long *words, hipStream_t s) {
  hipLaunchKernelGGL(k_consume_words, dim3(1), dim3(1), 0, s, st_, 0ULL, words);
  KG_HIP(hipGetLastError());
  return 0;
}

}  // namespace kg
