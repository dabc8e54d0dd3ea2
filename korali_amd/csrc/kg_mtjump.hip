// kg_mtjump.hip — jump-ahead for the GSL mt19937 stream (host side).
//
// The reference draws a generation's λ·N normals from ONE sequential
// mt19937 stream (univariate/normal/normal.cpp.base:32-35); at C4 (N=512,
// λ=65536) that is ~85 M words per generation, far more than one
// workgroup's recurrence can produce in time.  mt19937 is linear over GF(2)
// with a degree-19937 characteristic polynomial P, so the stream is cut
// into chunks of W words at fixed positions and every chunk is produced by
// its own workgroup from a start window obtained by jumping:
//
//   s_{n+J} = XOR_{i : c_i = 1} s_{n+i}      for all n >= 1,
//   c(x)    = x^J mod P(x)                    (deg c < 19937).
//
// (s_n = untempered words; the identity holds for every full word of the
// recurrence's 19937-bit state, and for the one word whose low 31 bits are
// outside that state only those low bits may differ — they never reach an
// output.)  P is recovered once per process by Berlekamp-Massey from 2x19937
// output bits; x^(2^e) mod P by repeated squaring.  This file is the host
// half (and a host reference of the jump for tests); the device kernels are
// in kg_rng.hip.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "kg_rng.hpp"

namespace kg {

namespace {

using Poly = std::vector<uint64_t>;  // bit i = coefficient of x^i

inline int bit(const Poly &p, int i) { return (int)((p[(size_t)i >> 6] >> (i & 63)) & 1u); }
inline void flip(Poly &p, int i) { p[(size_t)i >> 6] ^= 1ULL << (i & 63); }

// 64 bits of p starting at bit offset `off` (bits past the end read as 0)
inline uint64_t window64(const Poly &p, size_t off) {
  const size_t q = off >> 6, r = off & 63;
  const uint64_t lo = q < p.size() ? p[q] : 0, hi = (q + 1) < p.size() ? p[q + 1] : 0;
  return r ? (lo >> r) | (hi << (64 - r)) : lo;
}

// dst ^= src << sh  (dst sized to hold the result)
void xor_shifted(Poly &dst, const Poly &src, size_t sh) {
  const size_t q = sh >> 6, r = sh & 63;
  for (size_t w = 0; w < src.size(); w++) {
    if (!src[w]) continue;
    if (w + q < dst.size()) dst[w + q] ^= src[w] << r;
    if (r && w + q + 1 < dst.size()) dst[w + q + 1] ^= src[w] >> (64 - r);
  }
}

// Berlekamp-Massey over GF(2): the shortest LFSR generating s; returns the
// characteristic polynomial x^L C(1/x).
Poly berlekamp_massey(const std::vector<uint8_t> &s, int &Lout) {
  const size_t n = s.size(), words = (n + 64) / 64 + 1;
  Poly sr(words, 0);  // reversed sequence: bit k = s[n-1-k]
  for (size_t k = 0; k < n; k++)
    if (s[n - 1 - k]) sr[k >> 6] |= 1ULL << (k & 63);
  Poly C(words, 0), B(words, 0), T;
  C[0] = B[0] = 1;
  int L = 0;
  size_t m = 1;
  for (size_t i = 0; i < n; i++) {
    // d = sum_{j=0..L} C_j s[i-j]  (C_0 = 1); s[i-j] = sr bit (n-1-i+j)
    uint64_t acc = 0;
    const size_t base = n - 1 - i;
    for (size_t w = 0; w * 64 <= (size_t)L; w++) acc ^= C[w] & window64(sr, base + 64 * w);
    if ((size_t)L % 64 != 63) {
      // bits above L in the last word of C are zero, nothing to mask
    }
    const int d = __builtin_parityll(acc);
    if (!d) {
      m++;
    } else if (2 * L <= (int)i) {
      T = C;
      xor_shifted(C, B, m);
      L = (int)i + 1 - L;
      B = T;
      m = 1;
    } else {
      xor_shifted(C, B, m);
      m++;
    }
  }
  Poly P((MT_L + 64) / 64, 0);
  for (int k = 0; k <= L; k++)
    if (bit(C, L - k)) flip(P, k);
  Lout = L;
  return P;
}

// r mod P for deg r < 2L (in place; r sized for 2L bits)
void reduce(Poly &r, const Poly &P, int L) {
  const int top = (int)r.size() * 64 - 1;
  for (int d = top; d >= L; d--)
    if (bit(r, d)) xor_shifted(r, P, (size_t)(d - L));
}

Poly sqr_mod(const Poly &a, const Poly &P, int L) {
  Poly r(2 * a.size(), 0);
  for (size_t w = 0; w < a.size(); w++) {
    uint64_t x = a[w];
    for (int h = 0; h < 2; h++) {
      uint64_t v = (x >> (32 * h)) & 0xffffffffULL, o = 0;
      for (int b = 0; b < 32; b++) o |= ((v >> b) & 1ULL) << (2 * b);
      r[2 * w + h] = o;
    }
  }
  reduce(r, P, L);
  r.resize(a.size());
  return r;
}

Poly mul_mod(const Poly &a, const Poly &b, const Poly &P, int L) {
  Poly r(2 * a.size(), 0);
  for (int i = 0; i < L; i++)
    if (bit(a, i)) xor_shifted(r, b, (size_t)i);
  reduce(r, P, L);
  r.resize(a.size());
  return r;
}

struct MtPolys {
  Poly P;
  int L = 0;
  std::vector<Poly> pow2;  // x^(2^e) mod P
};

MtPolys &mt_polys() {
  static MtPolys mp;
  static std::once_flag once;
  std::call_once(once, [] {
    // untempered words of an arbitrary seed; bit 0 of the generated words
    std::vector<uint32_t> s(MT_N + 2 * MT_L + 128);
    s[0] = 5489u;
    for (int i = 1; i < MT_N; i++) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + (uint32_t)i;
    for (size_t j = MT_N; j < s.size(); j++) s[j] = mt_next(s[j - 624], s[j - 623], s[j - 227]);
    std::vector<uint8_t> bits(2 * MT_L + 64);
    for (size_t k = 0; k < bits.size(); k++) bits[k] = (uint8_t)(s[MT_N + k] & 1u);
    mp.P = berlekamp_massey(bits, mp.L);
    Poly x((MT_L + 64) / 64, 0);
    x[0] = 2;  // x^1
    mp.pow2.push_back(x);
  });
  return mp;
}

const Poly &pow2_poly(int e) {
  MtPolys &mp = mt_polys();
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  while ((int)mp.pow2.size() <= e) mp.pow2.push_back(sqr_mod(mp.pow2.back(), mp.P, mp.L));
  return mp.pow2[(size_t)e];
}

}  // namespace

int mt_poly_degree() { return mt_polys().L; }

int mt_jump_poly_pow2(int e, uint64_t *out) {
  if (mt_polys().L != MT_L) {
    set_error("mt19937 minimal polynomial: unexpected degree " + std::to_string(mt_polys().L));
    return 1;
  }
  const Poly &p = pow2_poly(e);
  std::fill(out, out + MT_POLY_WORDS, 0ULL);
  std::copy(p.begin(), p.begin() + std::min(p.size(), (size_t)MT_POLY_WORDS), out);
  return 0;
}

int mt_jump_host(const uint32_t *window, unsigned long long J, uint32_t *out) {
  MtPolys &mp = mt_polys();
  if (mp.L != MT_L) {
    set_error("mt19937 minimal polynomial: unexpected degree");
    return 1;
  }
  // c = x^J mod P by the binary expansion of J
  Poly c((MT_L + 64) / 64, 0);
  c[0] = 1;
  for (int e = 0; e < 64; e++)
    if ((J >> e) & 1ULL) c = mul_mod(c, pow2_poly(e), mp.P, mp.L);
  std::vector<uint32_t> seq(MT_N + MT_L - 1);
  std::copy(window, window + MT_N, seq.begin());
  for (size_t j = MT_N; j < seq.size(); j++) seq[j] = mt_next(seq[j - 624], seq[j - 623], seq[j - 227]);
  for (int m = 0; m < MT_N; m++) {
    uint32_t acc = 0;
    for (int i = 0; i < MT_L; i++)
      if (bit(c, i)) acc ^= seq[(size_t)m + i];
    out[m] = acc;
  }
  return 0;
}

}  // namespace kg

extern "C" int kg_debug_mt_jump(const uint32_t *window624, uint64_t distance, uint32_t *out624) {
  if (!window624 || !out624) {
    kg::set_error("kg_debug_mt_jump: null argument");
    return 1;
  }
  return kg::mt_jump_host(window624, distance, out624);
}
