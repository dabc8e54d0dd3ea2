// kg_rng.hpp — a GSL mt19937 stream resident in HBM.
//
// The reference draws every normal of a generation from ONE sequential GSL
// mt19937 stream (Normal::getRandomNumber → gsl_ran_gaussian, Marsaglia
// polar on gsl_rng_uniform_pos; univariate/normal/normal.cpp.base:32-35).
// The stream is a fixed sequence independent of the solver state, so the
// device keeps its untempered words s_j (absolute index j) in a ring buffer:
//
//   s_j = s_{j-227} ^ twist(s_{j-624}, s_{j-623})      (GSL rng/mt.c)
//
// * k_mt_produce extends the generated frontier with one wavefront: 227
//   independent words per step (the recurrence's minimum lag), LDS ring of
//   the last 1024 words, coalesced stores to HBM.
// * polar normals are then data-parallel: attempt a uses compacted words
//   (2a, 2a+1) (zero words skipped, as uniform_pos does), an accept-count
//   pass + block scan + scatter pass places normal k exactly where the
//   sequential reference would, and the consumed-word count re-derives the
//   exact GSL state (mt[624], mti) for export.
#pragma once

#include "kg_common.hpp"

namespace kg {

constexpr int KG_MAX_ZERO_WORDS = 64;

// jump-ahead (kg_mtjump.hip): characteristic polynomial degree and the
// 64-bit words of a polynomial of degree < MT_L
constexpr int MT_L = 19937;
constexpr int MT_POLY_WORDS = (MT_L + 64) / 64;  // 312
constexpr int MT_SEQ = MT_N + MT_L - 1;          // words a jump reads (20560)
int mt_poly_degree();
int mt_jump_poly_pow2(int e, uint64_t *out);     // x^(2^e) mod P
int mt_jump_host(const uint32_t *window, unsigned long long J, uint32_t *out);

// chunked parallel production: chunk c = words [cW, (c+1)W) of the stream
// (positions relative to the import point), made by its own workgroup from
// a start window seeds[c mod 2K]; producing chunk c also jumps its window
// K*W words ahead to seed chunk c+K.
struct ChunkPlan {
  unsigned long long c_first, n;
};

struct StreamState {
  unsigned long long lo;   // absolute index of the current GSL block start (624*b)
  unsigned long long pos;  // next unconsumed absolute index
  unsigned long long hi;   // generated frontier (exclusive)
  unsigned int nzero;      // recorded zero words (absolute positions >= lo)
  unsigned int errors;
  unsigned long long zeros[KG_MAX_ZERO_WORDS];
  unsigned long long last_attempt;  // polar: attempt index of the last consumed normal
  unsigned long long total_normals; // polar: accepted normals available in the window
};

class MtStream {
 public:
  MtStream() = default;
  ~MtStream();
  void drain();  // waits for the side stream's pending production
  // capacity: words the ring must hold beyond the current block.  Streams
  // whose demand reaches `parallel_min` words (1 M: C2 and up) use the
  // chunked multi-workgroup producer (env KORALI_AMD_MT_PARALLEL_MIN / KORALI_AMD_MT_CHUNK_LOG2
  // override the threshold and chunk size for tests).
  int init(size_t capacity_words, size_t parallel_min = 1u << 20);
  bool parallel() const { return par_; }
  int import_gsl(const void *state5000, hipStream_t s);
  int export_gsl(void *state5000, hipStream_t s);
  // make sure words [pos, pos + ahead) exist (device-side target)
  int produce(unsigned long long ahead, hipStream_t s);

  // Polar normals (gsl_ran_gaussian, sigma = 1, mean 0 added): M normals into
  // z (device, sample-major).  If block_len > 0, block_end[b] receives the
  // attempt index of normal (b+1)*block_len-1 (resampling support).  The
  // stream is NOT advanced; call consume_normals() with the number of
  // normals actually used.
  // Normals k outside [k_lo, k_hi) are counted (stream positions stay exact)
  // but not written; z receives normal k at z[k - k_lo].
  int polar_normals(double *z, size_t M, size_t block_len, unsigned long long *block_end, hipStream_t s,
                    size_t k_lo = 0, size_t k_hi = (size_t)-1);
  // advance past `normals_used` normals (device-side: uses last attempt of
  // normal normals_used-1 found in block_end[(normals_used/block_len)-1] or
  // the polar pass's own record when block_end == nullptr)
  int consume_normals(size_t normals_used, size_t block_len, const unsigned long long *block_end, hipStream_t s);
  // same, with the number of consumed blocks of block_len normals read from
  // device memory (decided on the device by the resampling pass)
  int consume_normals_dev(const unsigned long long *used_blocks, size_t block_len,
                          const unsigned long long *block_end, hipStream_t s);

  // GSL gsl_rng_uniform draws: M uniforms (no zero skip) consumed at once
  int uniforms(double *u, size_t M, hipStream_t s);
  // the next M uniforms without consuming them, then consume a count the
  // device decided (variable consumption: CMA-ES discrete mutations)
  int peek_uniforms(double *u, size_t M, hipStream_t s);
  int consume_words_dev(const unsigned long long *words, hipStream_t s);

  // Launch the producer for this and the next draw on a side stream so it
  // runs concurrently with whatever the main stream does next (the
  // eigendecomposition); polar_normals() then waits for it.
  int prefetch(size_t M_normals, hipStream_t main);
  // polar_normals() on the side stream, after everything queued on `main`
  // so far (the stream is not advanced: a later consume_normals() on `main`,
  // after join(main), takes them).  Returns 1 when no side stream exists yet
  // (nothing launched, nothing else to do).
  int polar_normals_ahead(double *z, size_t M, size_t block_len, hipStream_t main);

  // the producer's side stream (created by the first prefetch), and a join
  // that makes `main` wait for everything queued on it so far
  hipStream_t side_stream() const { return side_; }
  int join(hipStream_t main);

  StreamState *state() { return st_; }
  unsigned long long capacity_words() const { return R_; }
  size_t words_for_normals(size_t M) const;

 private:
  uint32_t *ring_ = nullptr;
  unsigned long long R_ = 0;  // power of two
  StreamState *st_ = nullptr;
  unsigned int *counts_ = nullptr;  // per-block accept counts
  unsigned long long *offsets_ = nullptr;
  size_t scratch_blocks_ = 0;
  hipStream_t side_ = nullptr;
  hipEvent_t ev_main_ = nullptr, ev_side_ = nullptr;
  bool prefetch_pending_ = false;
  int ensure_scratch(size_t nblocks);
  // chunked producer state
  bool par_ = false;
  unsigned long long W_ = 0;  // chunk words (power of two, >= MT_SEQ)
  int K_ = 0;                 // chunks per launch / seed lead
  int parts_ = 8;             // workgroups sharing each chunk's seed jump
  uint32_t *seeds_ = nullptr; // [2K][624]
  uint64_t *polys_ = nullptr; // x^(2^l W) mod P, l = 0..log2 K
  ChunkPlan *plan_ = nullptr;
  int seed_chunks(unsigned long long pos, hipStream_t s);
  int produce_chunks(unsigned long long ahead, hipStream_t s);
};

}  // namespace kg
