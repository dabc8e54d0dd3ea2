// kg_eigen.hip — GSL-faithful symmetric eigensolver on one CDNA4 workgroup.
//
// Replaces CMAES::updateEigensystem + CMAES::eigen (CMAES.cpp.base:869-938),
// i.e. gsl_eigen_symmv + gsl_eigen_symmv_sort(GSL_EIGEN_SORT_ABS_ASC).  The
// eigenvector SIGNS of LAPACK-style solvers differ from GSL in 2-6 columns
// per generation and every sign flip changes the next population, so this
// kernel replays GSL 2.6's exact arithmetic:
//
//   A  Householder tridiagonalisation (linalg/symmtd.c) with gslcblas
//      dnrm2 / dsymv / dsyr2 operation order; A lives in LDS (row stride
//      N+1: conflict-free column and row sweeps) when N <= 128.
//   B  symmtd_unpack: Q = prod H_i (householder_hm), Q kept transposed in
//      LDS, one column per thread.
//   C  implicit-shift QR (eigen/qrstep.c): the Givens chase is inherently
//      serial and runs on lane 0 of wave 0; the rotations of step t are
//      applied row-parallel by waves 1..15 while lane 0 chases step t+1
//      (double-buffered gc/gs, one barrier per QR step).
//   D  ABS_ASC selection sort (parallel arg-min per position) and the
//      updateEigensystem write-back (keep the old B, D if min eval <= 0).
//
// Every +,-,*,/,sqrt is IEEE correctly rounded on gfx950 and the file is
// compiled with -ffp-contract=off, so the result equals the oracle bit for
// bit.
#include "kg_eigen.hpp"

namespace kg {

namespace {

__device__ __attribute__((unused)) inline double readlane_d(double x, int l) {
  const long long v = __double_as_longlong(x);
  int lo = (int)(v & 0xffffffffLL), hi = (int)(v >> 32);
  lo = __builtin_amdgcn_readlane(lo, l);
  hi = __builtin_amdgcn_readlane(hi, l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__host__ __device__ inline uint32_t hiw(double x) { return (uint32_t)(__builtin_bit_cast(unsigned long long, x) >> 32); }
__host__ __device__ inline uint32_t low(double x) {
  return (uint32_t)(__builtin_bit_cast(unsigned long long, x) & 0xffffffffULL);
}
__host__ __device__ inline double sethi(double x, uint32_t h) {
  return __builtin_bit_cast(double, ((unsigned long long)h << 32) | (unsigned long long)low(x));
}

// fdlibm __ieee754_hypot (glibc < 2.35), SURVEY.md Appendix A
__host__ __device__ double hypot_fdlibm(double x, double y) {
  double a, b, t1, t2, y1, y2, w;
  int32_t j, k, ha, hb;
  ha = (int32_t)(hiw(x) & 0x7fffffff);
  hb = (int32_t)(hiw(y) & 0x7fffffff);
  if (hb > ha) {
    a = y;
    b = x;
    j = ha;
    ha = hb;
    hb = j;
  } else {
    a = x;
    b = y;
  }
  a = sethi(a, (uint32_t)ha);
  b = sethi(b, (uint32_t)hb);
  if ((ha - hb) > 0x3c00000) return a + b;
  k = 0;
  if (ha > 0x5f300000) {
    if (ha >= 0x7ff00000) {
      w = a + b;
      if (((ha & 0xfffff) | low(a)) == 0) w = a;
      if (((hb ^ 0x7ff00000) | low(b)) == 0) w = b;
      return w;
    }
    ha -= 0x25800000;
    hb -= 0x25800000;
    k += 600;
    a = sethi(a, (uint32_t)ha);
    b = sethi(b, (uint32_t)hb);
  }
  if (hb < 0x20b00000) {
    if (hb <= 0x000fffff) {
      if ((hb | (int32_t)low(b)) == 0) return a;
      t1 = sethi(0.0, 0x7fd00000);
      b *= t1;
      a *= t1;
      k -= 1022;
    } else {
      ha += 0x25800000;
      hb += 0x25800000;
      k -= 600;
      a = sethi(a, (uint32_t)ha);
      b = sethi(b, (uint32_t)hb);
    }
  }
  w = a - b;
  if (w > b) {
    t1 = sethi(0.0, (uint32_t)ha);
    t2 = a - t1;
    w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
  } else {
    a = a + a;
    y1 = sethi(0.0, (uint32_t)hb);
    y2 = b - y1;
    t1 = sethi(0.0, (uint32_t)(ha + 0x00100000));
    t2 = a - t1;
    w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
  }
  if (k != 0) {
    t1 = sethi(1.0, hiw(1.0) + ((uint32_t)k << 20));
    return t1 * w;
  }
  return w;
}

constexpr double EPS = 2.2204460492503131e-16;
constexpr double DMIN = 2.2250738585072014e-308;

__host__ __device__ inline void chop_small(int n, const double *d, double *sd) {
  double d_i = d[0];
  for (int i = 0; i + 1 < n; i++) {
    const double sd_i = sd[i], d_ip1 = d[i + 1];
    if (fabs(sd_i) < EPS * (fabs(d_i) + fabs(d_ip1))) sd[i] = 0.0;
    d_i = d_ip1;
  }
}

__host__ __device__ inline void create_givens(double a, double b, double &c, double &s) {
  if (b == 0) {
    c = 1;
    s = 0;
  } else if (fabs(b) > fabs(a)) {
    const double t = -a / b;
    const double s1 = 1.0 / sqrt(1 + t * t);
    s = s1;
    c = s1 * t;
  } else {
    const double t = -b / a;
    const double c1 = 1.0 / sqrt(1 + t * t);
    c = c1;
    s = c1 * t;
  }
}

// eigen/qrstep.c qrstep on d[0..n), sd[0..n-1)
__host__ __device__ void qrstep(int n, double *d, double *sd, double *gc, double *gs) {
  double x, z, ak, bk, zk, ap, bp, aq, bq;
  double mu;
  {
    const double ta = d[n - 2], tb = d[n - 1], tab = sd[n - 2];
    const double dt = (ta - tb) / 2.0;
    if (dt > 0)
      mu = tb - tab * (tab / (dt + hypot_fdlibm(dt, tab)));
    else if (dt == 0)
      mu = tb - fabs(tab);
    else
      mu = tb + tab * (tab / ((-dt) + hypot_fdlibm(dt, tab)));
  }
  if (EPS * fabs(mu) > (fabs(d[0]) + fabs(sd[0]))) mu = 0;
  x = d[0] - mu;
  z = sd[0];
  ak = 0;
  bk = 0;
  zk = 0;
  ap = d[0];
  bp = sd[0];
  aq = d[1];
  if (n == 2) {
    double c, s;
    create_givens(x, z, c, s);
    gc[0] = c;
    gs[0] = s;
    const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
    const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
    const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
    d[0] = ap1;
    sd[0] = bp1;
    d[1] = aq1;
    return;
  }
  bq = sd[1];
  // d[k+2], sd[k+2] read at step k were never written by this chase yet:
  // load them one step ahead so LDS latency stays off the critical path
  double dn = d[n - 1 < 2 ? n - 1 : 2], sdn = sd[n - 2 < 2 ? n - 2 : 2];
  int k;
  for (k = 0; k < n - 1; k++) {
    const double dpf = d[(k + 3 < n - 1) ? k + 3 : n - 1];  // unconditional loads (unused past the end)
    const double sdpf = sd[(k + 3 < n - 2) ? k + 3 : n - 2];
    double c, s;
    create_givens(x, z, c, s);
    gc[k] = c;
    gs[k] = s;
    const double bk1 = c * bk - s * zk;
    const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
    const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
    const double zp1 = -s * bq;
    const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
    const double bq1 = c * bq;
    ak = ap1;
    bk = bp1;
    zk = zp1;
    ap = aq1;
    bp = bq1;
    if (k < n - 2) aq = dn;
    if (k < n - 3) bq = sdn;
    dn = dpf;
    sdn = sdpf;
    d[k] = ak;
    if (k > 0) sd[k - 1] = bk1;
    if (k < n - 2) sd[k + 1] = bp;
    x = bk;
    z = zk;
  }
  d[k] = ap;
  sd[k - 1] = bk;
}

}  // namespace

// Dynamic LDS: [matrix region N*(N+1) doubles if lds_mats] + vectors.
// Vectors (doubles): x N, d N, sd N, tau N, gc 2N, gs 2N, ev N, scal 16; ints
// perm N, misc 8.
// ------------------------------------------------------------------------
// Phase A: Householder tridiagonalisation (gsl_linalg_symmtd_decomp).
// Outputs: Householder vectors H (row i = column i of A below the
// diagonal), tau, diagonal d and sub-diagonal sd of the tridiagonal form.
template <bool kLds>
__global__ void __launch_bounds__(1024) k_tridiag(int N, const double *__restrict__ C, double *gA, double *gH,
                                                  double *tauOut, double *dOut, double *sdOut,
                                                  unsigned long long *trace) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wid = tid >> 6;
  const int lda = N + 1;
  double *M = kLds ? smem : gA;
  double *vb = kLds ? smem + (size_t)N * lda : smem;
  double *x = vb, *scal = vb + N;
  double *sv = vb + N + 16;  // staged addends of a serial chain (wave 0); t2 of dsymv
  double *tv = sv + (N > 64 ? N : 64);  // tau * v_r, contiguous (dsymv)
  double *vv = tv + N;       // v_r with v_0 = 1, contiguous (dsymv)
  unsigned long long acc_t[4] = {0, 0, 0, 0}, tmark = 0;
#define KG_MARK() \
  if (trace && tid == 0) tmark = __builtin_amdgcn_s_memtime();
#define KG_ACC(k) \
  if (trace && tid == 0) acc_t[k] += __builtin_amdgcn_s_memtime() - tmark;

  // symmetrise from the lower triangle (CMAES.cpp.base:908-913)
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, j = idx % N;
    M[i * lda + j] = (j <= i) ? C[i * N + j] : C[j * N + i];
  }
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    const int n = N - i - 1;
    double *v = M + (size_t)(i + 1) * lda + i;        // stride lda
    double *m = M + (size_t)(i + 1) * lda + (i + 1);  // lda
    KG_MARK()
    if (wid == 0) {
      // gslcblas dnrm2 over v[1..n-1]: prefix max in parallel, the ssq
      // recurrence sequentially on uniform registers (every lane the same)
      double scale_carry = 0.0, ssq = 1.0;
      for (int base = 1; base < n; base += 64) {
        const int r = base + lane;
        const double a_ = fabs(v[(size_t)min(r, n - 1) * lda]);
        const double a = (r < n) ? a_ : 0.0;
        double pm = a;
        for (int off = 1; off < 64; off <<= 1) {
          const double t = __shfl_up(pm, off, 64);
          if (lane >= off) pm = fmax(pm, t);
        }
        double before = __shfl_up(pm, 1, 64);
        if (lane == 0) before = 0.0;
        before = fmax(before, scale_carry);
        int type = 0;
        double q = 0.0;
        if (r < n && a != 0.0) {
          if (before < a) {
            type = 1;
            q = before / a;
          } else {
            type = 2;
            q = a / before;
          }
        }
        // addends precomputed lane-parallel; zero elements add +0.0, which
        // leaves ssq (>= 1) unchanged.  The serial recurrence then runs on
        // values staged in LDS, 8 in flight, new-maximum lanes (a handful
        // per vector) taking the rescaling branch.
        const double tq = (type == 2) ? q * q : 0.0;
        const unsigned long long m1 = __ballot(type == 1);
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        sv[lane] = (type == 1) ? q : tq;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int l0 = 0; l0 < cnt; l0 += 8) {
          double t[8];
#pragma unroll
          for (int u = 0; u < 8; u++) t[u] = sv[l0 + u];  // lanes past n staged +0.0
          const unsigned bits = (unsigned)((m1 >> l0) & 0xffULL);
          if (bits == 0) {
#pragma unroll
            for (int u = 0; u < 8; u++) ssq += t[u];
          } else {
#pragma unroll
            for (int u = 0; u < 8; u++) {
              if ((bits >> u) & 1u)
                ssq = 1.0 + ssq * t[u] * t[u];
              else
                ssq += t[u];
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        scale_carry = fmax(scale_carry, readlane_d(pm, 63));
      }
      if (lane == 0) {
        double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
        int branch = 0;
        const double xnorm = (n - 1 == 1) ? fabs(v[lda]) : scale_carry * sqrt(ssq);
        if (xnorm != 0) {
          const double alpha = v[0];
          beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fdlibm(alpha, xnorm);
          tau_i = (beta - alpha) / beta;
          const double s = alpha - beta;
          if (fabs(s) > DMIN) {
            f1 = 1.0 / s;
            branch = 1;
          } else {
            f1 = EPS / s;
            f2 = 1.0 / EPS;
            branch = 2;
          }
        }
        scal[0] = tau_i;
        scal[1] = f1;
        scal[2] = f2;
        scal[3] = beta;
        scal[4] = (double)branch;
        tauOut[i] = tau_i;
      }
    }
    __syncthreads();
    KG_ACC(0)
    const double tau_i = scal[0];
    const int branch = (int)scal[4];
    if (branch != 0) {
      const double f1 = scal[1], f2 = scal[2];
      for (int r = 1 + tid; r < n; r += nt) {
        double t = v[(size_t)r * lda] * f1;
        if (branch == 2) t = t * f2;
        v[(size_t)r * lda] = t;
      }
      if (tid == 0) v[0] = scal[3];
    }
    __syncthreads();
    if (tau_i == 0.0) continue;
    KG_MARK()
    // x = tau * m * v (dsymv RowMajor Lower, beta = 0), v0 := 1
    for (int r = tid; r < n; r += nt) {
      const double vr = (r == 0) ? 1.0 : v[(size_t)r * lda];
      vv[r] = vr;
      tv[r] = tau_i * vr;
    }
    __syncthreads();
    // The two sequential chains of output j run on different waves (all four
    // SIMDs busy), products formed inline, 8 at a time, loads unconditional:
    //   acc_j: rows r = n-1 .. j+1 (descending) of (tau v_r) m[r][j]   (thread j)
    //   t2_j : cols q = 0 .. j-1 of v_q m[j][q]                        (thread 128 + j)
    // then x_j = (acc_j + (tau v_j) m[j][j]) + tau t2_j.
    double *t2b = sv;  // t2 of every j (sv holds max(N, 64) doubles)
    const int half = (nt / 2) & ~63;
    if (tid < half) {
      for (int j = tid; j < n; j += half) {
        double acc = 0.0;
        int r = n - 1;
        const double *mc = m + j;
        for (; r - 7 > j; r -= 8) {
          double p[8];
#pragma unroll
          for (int u = 0; u < 8; u++) p[u] = tv[r - u] * mc[(size_t)(r - u) * lda];
#pragma unroll
          for (int u = 0; u < 8; u++) acc += p[u];
        }
        for (; r > j; r--) acc += tv[r] * mc[(size_t)r * lda];
        x[j] = acc;
      }
    } else {
      for (int j = tid - half; j < n; j += nt - half) {
        const double *mj = m + (size_t)j * lda;
        double t2 = 0.0;
        int q = 0;
        for (; q + 8 <= j; q += 8) {
          double p[8];
#pragma unroll
          for (int u = 0; u < 8; u++) p[u] = vv[q + u] * mj[q + u];
#pragma unroll
          for (int u = 0; u < 8; u++) t2 += p[u];
        }
        for (; q < j; q++) t2 += vv[q] * mj[q];
        t2b[j] = t2;
      }
    }
    __syncthreads();
    for (int j = tid; j < n; j += nt) {
      double acc = x[j];
      acc += tv[j] * m[(size_t)j * lda + j];
      acc += tau_i * t2b[j];
      x[j] = acc;
    }
    __syncthreads();
    KG_ACC(1)
    KG_MARK()
    if (wid == 0) {
      // xv = sum x[r] v[r] sequentially (products lane-parallel, staged in
      // LDS, 8 in flight; +0.0 padding is exact); alpha = -(tau/2) xv
      double xv = 0.0;
      for (int base = 0; base < n; base += 64) {
        const int r = base + lane, rc = min(r, n - 1);
        const double p_ = x[rc] * vv[rc];
        sv[lane] = (r < n) ? p_ : 0.0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        for (int l0 = 0; l0 < cnt; l0 += 8) {
          double t[8];
#pragma unroll
          for (int u = 0; u < 8; u++) t[u] = sv[l0 + u];
#pragma unroll
          for (int u = 0; u < 8; u++) xv += t[u];
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) scal[5] = -(tau_i / 2.0) * xv;
    }
    __syncthreads();
    {
      const double alpha = scal[5];
      for (int r = tid; r < n; r += nt) x[r] += alpha * ((r == 0) ? 1.0 : v[(size_t)r * lda]);
    }
    __syncthreads();
    KG_ACC(2)
    KG_MARK()
    // dsyr2 RowMajor Lower, alpha = -1
    for (int r = wid; r < n; r += (nt >> 6)) {
      const double vr = (r == 0) ? 1.0 : v[(size_t)r * lda];
      const double tmp1 = -1.0 * vr, tmp2 = -1.0 * x[r];
      for (int j = lane; j <= r; j += 64) {
        const double vj = (j == 0) ? 1.0 : v[(size_t)j * lda];
        m[(size_t)r * lda + j] += tmp1 * x[j] + tmp2 * vj;
      }
    }
    __syncthreads();
    KG_ACC(3)
  }
  // Householder vectors, diag / sub-diagonal
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, r = idx % N;
    if (i + 2 < N && r < N - i - 1) gH[(size_t)i * N + r] = M[(size_t)(i + 1 + r) * lda + i];
  }
  for (int i = tid; i < N; i += nt) {
    dOut[i] = M[(size_t)i * lda + i];
    if (i + 1 < N) sdOut[i] = M[(size_t)(i + 1) * lda + i];
  }
  if (trace && tid == 0)
    for (int k = 0; k < 4; k++) trace[k] += acc_t[k];
#undef KG_MARK
#undef KG_ACC
}

// Phase B: Q = H_0 ... H_{N-3} (gsl_linalg_symmtd_unpack via
// householder_hm), built transposed (Qt[col][row]) and stored to gQt.
template <bool kLds>
__global__ void __launch_bounds__(1024) k_unpack(int N, const double *__restrict__ gH,
                                                 const double *__restrict__ tau, double *gQt) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lda = N + 1;
  double *M = kLds ? smem : gQt;
  double *h = kLds ? smem + (size_t)N * lda : smem;
  for (int idx = tid; idx < N * lda; idx += nt) {
    const int c = idx / lda, r = idx % lda;
    M[idx] = (r < N && c == r) ? 1.0 : 0.0;
  }
  __syncthreads();
  double *wsh = h + N;  // w_j = col_j . h (phase 1 result)
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int i = N - 3; i >= 0; i--) {
    const double ti = tau[i];
    if (ti == 0.0) continue;  // householder_hm returns early
    const int n = N - (i + 1);
    for (int r = tid; r < n; r += nt) h[r] = gH[(size_t)i * N + r];
    __syncthreads();
    // phase 1: w_j = sum_r Q[i+1+r][i+1+j] h[r], one ordered chain per j
    for (int j = tid; j < n; j += nt) {
      const double *col = M + (size_t)(i + 1 + j) * lda + (i + 1);  // Q[i+1+r][i+1+j], r = 0..n-1
      double wj = col[0];
      for (int r0 = 1; r0 < n; r0 += 16) {
        double p[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const int r = min(r0 + u, n - 1);
          const double pr = col[r] * h[r];
          p[u] = (r0 + u < n) ? pr : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; u++) wj += p[u];  // +0.0 padding is exact (see k_tridiag)
      }
      wsh[j] = wj;
    }
    __syncthreads();
    // phase 2 (every wave): Q[.][j] -= tau h w_j, element-parallel
    for (int j = wid; j < n; j += nw) {
      double *col = M + (size_t)(i + 1 + j) * lda + (i + 1);
      const double wj = wsh[j];
      for (int r = lane; r < n; r += 64) col[r] = (r == 0) ? col[0] - ti * wj : col[r] - ti * h[r] * wj;
    }
    __syncthreads();
  }
  if (kLds)
    for (int idx = tid; idx < N * lda; idx += nt) gQt[idx] = M[idx];
}

// ------------------------------------------------------------------------
// Phases A and B for N > 128 (the matrix no longer fits one CU's LDS):
// many workgroups, each holding a few FULL rows of the symmetric matrix in
// LDS (rows round-robin, row r on workgroup r % P).  Symmetric storage makes
// every gslcblas chain of a row local to its owner:
//   dsymv  x_j = (sum_{c desc} (tau v_c) m[j][c] + (tau v_j) m[j][j]) + tau sum_{c asc} v_c m[j][c]
//          (column j of the lower triangle is row j of the upper one);
//   dsyr2  m[a][b] += (-v_a) x_b + (-x_a) v_b with a >= b, applied to both
//          (a,b) and (b,a), so the two copies stay bit-identical.
// Per Householder step two in-launch hand-offs (R2 granules): the pivot
// row's owner broadcasts (tau, v); every owner publishes its x_j and every
// workgroup gathers the whole x (xv is then recomputed redundantly).  Every
// step has slots of its own (no slot is ever rewritten within a launch, so
// no workgroup can miss a value however far the others run ahead; tau = 0
// steps skip the x exchange).
constexpr int TMW_TPB = 256;
constexpr int TMW_MAXP = 64;

__host__ __device__ inline int tmw_rows(int N) { return (N + TMW_MAXP - 1) / TMW_MAXP; }
__host__ __device__ inline int tmw_groups(int N) { return (N + tmw_rows(N) - 1) / tmw_rows(N); }
size_t tmw_lds_bytes(int N) {
  return ((size_t)tmw_rows(N) * (N + 1) + 3 * (size_t)N + 64 + 16 + 2 * 16) * sizeof(double);
}
// comm buffer (u64 words): v granules [N][2(N+1)] (tau in element N), x
// granules [N][2N], abort word (+ pad to 16 bytes)
size_t tmw_comm_words(int N) { return 2 * (size_t)N * (N + 1) + 2 * (size_t)N * N + 2; }

__global__ void __launch_bounds__(TMW_TPB) k_tridiag_mw(int N, const double *__restrict__ C, double *gH,
                                                        double *tauOut, double *dOut, double *sdOut,
                                                        unsigned long long *comm, unsigned int *errors) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x;
  const int P = gridDim.x, g = blockIdx.x, RW = tmw_rows(N), lda = N + 1;
  double *M = smem;                     // local row k = global row g + k P
  double *vloc = M + (size_t)RW * lda;  // v with v_0 = 1
  double *tv = vloc + N;                // tau v
  double *xl = tv + N;                  // x
  double *sv = xl + N;                  // 64: staged chain addends
  double *scal = sv + 64;               // 16 scalars
  double *accb = scal + 16;             // 16: dsymv acc per local row
  double *t2b = accb + 16;              // 16: dsymv t2 per local row
  unsigned long long *gv = comm, *gx = comm + 2 * (size_t)N * (N + 1);
  unsigned long long *abortw = gx + 2 * (size_t)N * N;

  for (int idx = tid; idx < RW * N; idx += nt) {
    const int k = idx / N, c = idx % N, r = g + k * P;
    if (r < N) M[(size_t)k * lda + c] = (c <= r) ? C[(size_t)r * N + c] : C[(size_t)c * N + r];
  }
  const int maxRow = g + ((N - 1 - g) / P) * P;  // largest row owned
  __syncthreads();
  for (int i = 0; i + 2 < N; i++) {
    if (maxRow < i) break;  // nothing left to own or to update
    const int n = N - i - 1;
    const unsigned tag = (unsigned)i + 1u;
    unsigned long long *gvp = gv + (size_t)i * 2 * (N + 1), *gxp = gx + (size_t)i * 2 * N;
    if (i % P == g) {
      // ---- pivot row i: Householder vector of v = row i, columns i+1.. (== column i below the diagonal)
      double *v = M + (size_t)(i / P) * lda + i + 1;
      if (wid == 0) {
        double scale_carry = 0.0, ssq = 1.0;  // gslcblas dnrm2 over v[1..n-1] (see k_tridiag)
        for (int base = 1; base < n; base += 64) {
          const int r = base + lane;
          const double a_ = fabs(v[min(r, n - 1)]);
          const double a = (r < n) ? a_ : 0.0;
          double pm = a;
          for (int off = 1; off < 64; off <<= 1) {
            const double t = __shfl_up(pm, off, 64);
            if (lane >= off) pm = fmax(pm, t);
          }
          double before = __shfl_up(pm, 1, 64);
          if (lane == 0) before = 0.0;
          before = fmax(before, scale_carry);
          int type = 0;
          double q = 0.0;
          if (r < n && a != 0.0) {
            if (before < a) {
              type = 1;
              q = before / a;
            } else {
              type = 2;
              q = a / before;
            }
          }
          const double tq = (type == 2) ? q * q : 0.0;
          const unsigned long long m1 = __ballot(type == 1);
          const int cnt = (n - base) < 64 ? (n - base) : 64;
          sv[lane] = (type == 1) ? q : tq;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          for (int l0 = 0; l0 < cnt; l0 += 8) {
            double t[8];
#pragma unroll
            for (int u = 0; u < 8; u++) t[u] = sv[l0 + u];
            const unsigned bits = (unsigned)((m1 >> l0) & 0xffULL);
            if (bits == 0) {
#pragma unroll
              for (int u = 0; u < 8; u++) ssq += t[u];
            } else {
#pragma unroll
              for (int u = 0; u < 8; u++) {
                if ((bits >> u) & 1u)
                  ssq = 1.0 + ssq * t[u] * t[u];
                else
                  ssq += t[u];
              }
            }
          }
          __builtin_amdgcn_wave_barrier();
          scale_carry = fmax(scale_carry, readlane_d(pm, 63));
        }
        if (lane == 0) {
          double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
          int branch = 0;
          const double xnorm = (n - 1 == 1) ? fabs(v[1]) : scale_carry * sqrt(ssq);
          if (xnorm != 0) {
            const double alpha = v[0];
            beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fdlibm(alpha, xnorm);
            tau_i = (beta - alpha) / beta;
            const double s = alpha - beta;
            if (fabs(s) > DMIN) {
              f1 = 1.0 / s;
              branch = 1;
            } else {
              f1 = EPS / s;
              f2 = 1.0 / EPS;
              branch = 2;
            }
          }
          scal[0] = tau_i;
          scal[1] = f1;
          scal[2] = f2;
          scal[3] = beta;
          scal[4] = (double)branch;
          tauOut[i] = tau_i;
        }
      }
      __syncthreads();
      const int branch = (int)scal[4];
      if (branch != 0) {
        const double f1 = scal[1], f2 = scal[2];
        for (int r = 1 + tid; r < n; r += nt) {
          double t = v[r] * f1;
          if (branch == 2) t = t * f2;
          v[r] = t;
        }
      }
      __syncthreads();
      if (branch != 0 && tid == 0) v[0] = scal[3];
      __syncthreads();
      for (int r = tid; r < n; r += nt) {
        gH[(size_t)i * N + r] = v[r];
        const double vr = (r == 0) ? 1.0 : v[r];
        vloc[r] = vr;
        put_granule_dbl(gvp + 2 * r, tag, vr);
      }
      if (tid == 0) put_granule_dbl(gvp + 2 * N, tag, scal[0]);
    } else {
      // (v_0..v_{n-1}, tau) from the pivot's owner; tau lands in vloc[n]
      const bool ok = poll_granule_dbls(gvp, n + 1, N, tag, vloc, abortw, errors);
      if (__syncthreads_or(!ok)) return;
      if (tid == 0) scal[0] = vloc[n];
    }
    __syncthreads();
    const double tau_i = scal[0];
    if (tau_i == 0.0) continue;  // householder_transform gave tau = 0: no update
    for (int r = tid; r < n; r += nt) tv[r] = tau_i * vloc[r];
    __syncthreads();
    // ---- dsymv chains of the owned active rows (rows i+1..N-1)
    if (wid < 2 && lane < RW) {
      const int r = g + lane * P;
      if (r > i && r < N) {
        const double *row = M + (size_t)lane * lda;
        const int jr = r - i - 1;
        if (wid == 0) {
          double acc = 0.0;  // columns c = N-1 .. r+1, descending
          int c = N - 1;
          for (; c - 7 > r; c -= 8) {
            double p[8];
#pragma unroll
            for (int u = 0; u < 8; u++) p[u] = tv[c - u - i - 1] * row[c - u];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += p[u];
          }
          for (; c > r; c--) acc += tv[c - i - 1] * row[c];
          accb[lane] = acc + tv[jr] * row[r];
        } else {
          double t2 = 0.0;  // columns c = i+1 .. r-1, ascending
          int c = i + 1;
          for (; c + 8 <= r; c += 8) {
            double p[8];
#pragma unroll
            for (int u = 0; u < 8; u++) p[u] = vloc[c + u - i - 1] * row[c + u];
#pragma unroll
            for (int u = 0; u < 8; u++) t2 += p[u];
          }
          for (; c < r; c++) t2 += vloc[c - i - 1] * row[c];
          t2b[lane] = t2;
        }
      }
    }
    __syncthreads();
    if (tid < RW) {
      const int r = g + tid * P;
      if (r > i && r < N) put_granule_dbl(gxp + 2 * (r - i - 1), tag, accb[tid] + tau_i * t2b[tid]);
    }
    {
      const bool ok = poll_granule_dbls(gxp, n, -1, tag, xl, abortw, errors);
      if (__syncthreads_or(!ok)) return;
    }
    // ---- xv = sum x_r v_r (sequential, staged) and alpha = -(tau/2) xv
    if (wid == 0) {
      double xv = 0.0;
      for (int base = 0; base < n; base += 64) {
        const int r = base + lane, rc = min(r, n - 1);
        const double p_ = xl[rc] * vloc[rc];
        sv[lane] = (r < n) ? p_ : 0.0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        for (int l0 = 0; l0 < cnt; l0 += 8) {
          double t[8];
#pragma unroll
          for (int u = 0; u < 8; u++) t[u] = sv[l0 + u];
#pragma unroll
          for (int u = 0; u < 8; u++) xv += t[u];
        }
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) scal[5] = -(tau_i / 2.0) * xv;
    }
    __syncthreads();
    {
      const double alpha = scal[5];
      for (int r = tid; r < n; r += nt) xl[r] += alpha * vloc[r];
    }
    __syncthreads();
    // ---- dsyr2 (alpha = -1) on the owned active rows, both triangles
    for (int idx = tid; idx < RW * n; idx += nt) {
      const int k = idx / n, jj = idx % n, r = g + k * P;
      if (r <= i || r >= N) continue;
      const int jr = r - i - 1;
      const int a = jr > jj ? jr : jj, b = jr > jj ? jj : jr;
      const double tmp1 = -1.0 * vloc[a], tmp2 = -1.0 * xl[a];
      M[(size_t)k * lda + i + 1 + jj] += tmp1 * xl[b] + tmp2 * vloc[b];
    }
    __syncthreads();
  }
  for (int k = tid; k < RW; k += nt) {
    const int r = g + k * P;
    if (r < N) {
      dOut[r] = M[(size_t)k * lda + r];
      if (r + 1 < N) sdOut[r] = M[(size_t)k * lda + r + 1];
    }
  }
}

// Phase B for N > 128: the columns of Q are independent under
// householder_hm, so workgroups own UMW_COLS columns each (Q^T rows in LDS)
// and apply all reflectors without talking to each other; the next
// reflector row streams into a second LDS buffer while the current one is
// applied.
constexpr int UMW_COLS = 4;
constexpr int UMW_TPB = 256;
__host__ __device__ inline int umw_groups(int N) { return (N + UMW_COLS - 1) / UMW_COLS; }
size_t umw_lds_bytes(int N) { return ((size_t)UMW_COLS * (N + 1) + 2 * (size_t)N + 16) * sizeof(double); }

__global__ void __launch_bounds__(UMW_TPB) k_unpack_mw(int N, const double *__restrict__ gH,
                                                       const double *__restrict__ tau, double *gQt) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x;
  const int P = gridDim.x, g = blockIdx.x, lda = N + 1;
  double *Q = smem;                              // local k = column g + k P of Q
  double *hb = Q + (size_t)UMW_COLS * lda;       // 2 x N
  double *w = hb + 2 * (size_t)N;                // UMW_COLS
  for (int idx = tid; idx < UMW_COLS * lda; idx += nt) {
    const int k = idx / lda, r = idx % lda;
    Q[idx] = (r < N && r == g + k * P) ? 1.0 : 0.0;
  }
  constexpr int PF = 4;  // prefetch registers per thread (N <= 1024)
  if (N >= 3)
    for (int r = tid; r < N - (N - 3) - 1; r += nt) hb[r] = gH[(size_t)(N - 3) * N + r];
  __syncthreads();
  int buf = 0;
  for (int i = N - 3; i >= 0; i--) {
    const int n = N - i - 1;
    const double ti = tau[i];
    const double *h = hb + (size_t)buf * N;
    double pf[PF];
    if (i > 0) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        const int r = tid + u * nt;
        pf[u] = (r < n + 1) ? gH[(size_t)(i - 1) * N + r] : 0.0;
      }
    }
    if (ti != 0.0) {
      if (wid == 0 && lane < UMW_COLS) {
        const int c = g + lane * P;
        if (c > i && c < N) {
          const double *col = Q + (size_t)lane * lda + (i + 1);
          double wj = col[0];
          int r = 1;
          for (; r + 8 <= n; r += 8) {
            double p[8];
#pragma unroll
            for (int u = 0; u < 8; u++) p[u] = col[r + u] * h[r + u];
#pragma unroll
            for (int u = 0; u < 8; u++) wj += p[u];
          }
          for (; r < n; r++) wj += col[r] * h[r];
          w[lane] = wj;
        }
      }
      __syncthreads();
      for (int idx = tid; idx < UMW_COLS * n; idx += nt) {
        const int k = idx / n, r = idx % n, c = g + k * P;
        if (c <= i || c >= N) continue;
        double *col = Q + (size_t)k * lda + (i + 1);
        const double wj = w[k];
        col[r] = (r == 0) ? col[0] - ti * wj : col[r] - ti * h[r] * wj;
      }
    }
    if (i > 0) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        const int r = tid + u * nt;
        if (r < n + 1) hb[(size_t)(buf ^ 1) * N + r] = pf[u];
      }
    }
    __syncthreads();
    buf ^= 1;
  }
  for (int idx = tid; idx < UMW_COLS * lda; idx += nt) {
    const int k = idx / lda, r = idx % lda, c = g + k * P;
    if (c < N) gQt[(size_t)c * lda + r] = Q[idx];
  }
}

// ------------------------------------------------------------------------
// Phase C: the implicit-shift QR chase (eigen/symmv.c main loop + qrstep)
// on the tridiagonal d/sd.  It only produces the rotation sequence: per QR
// step a header (a, n) and n-1 Givens pairs (c, s); then the ABS_ASC
// selection sort gives eval (sorted) and the column permutation.
struct EigRec {
  int *hdr;     // 2 per step: a, n
  double *cs;   // 2 per rotation
  int *meta;    // [0] steps [1] rotations [2] overflow/error
  double *eval; // N sorted eigenvalues
  int *perm;    // N: sorted column i = unsorted column perm[i]
};

EigenSolver::Rec::operator EigRec() const { return EigRec{hdr, cs, meta, eval, perm}; }

__host__ __device__ inline int qr_chase(int N, double *d, double *sd, EigRec r, int maxRot, double *gc, double *gs) {
  chop_small(N, d, sd);
  int b = N - 1, steps = 0, rot = 0, err = 0;
  while (b > 0) {
    if (sd[b - 1] == 0.0 || sd[b - 1] != sd[b - 1]) {  // == 0 or NaN
      b--;
      continue;
    }
    int a = b - 1;
    while (a > 0) {
      if (sd[a - 1] == 0.0) break;
      a--;
    }
    const int nb = b - a + 1;
    if (rot + nb - 1 > maxRot) {
      err = 1;
      break;
    }
    qrstep(nb, d + a, sd + a, gc, gs);
    for (int k = 0; k + 1 < nb; k++) {
      r.cs[2 * (rot + k)] = gc[k];
      r.cs[2 * (rot + k) + 1] = gs[k];
    }
    r.hdr[2 * steps] = a;
    r.hdr[2 * steps + 1] = nb;
    steps++;
    rot += nb - 1;
    chop_small(nb, d + a, sd + a);
  }
  // gsl_eigen_symmv_sort(ABS_ASC): selection sort, strict < on |e|
  for (int i = 0; i < N; i++) {
    r.eval[i] = d[i];
    r.perm[i] = i;
  }
  for (int i = 0; i + 1 < N; i++) {
    int k = i;
    double ek = r.eval[i];
    for (int j = i + 1; j < N; j++)
      if (fabs(r.eval[j]) < fabs(ek)) {
        k = j;
        ek = r.eval[j];
      }
    if (k != i) {
      const double t = r.eval[i];
      r.eval[i] = r.eval[k];
      r.eval[k] = t;
      const int p = r.perm[i];
      r.perm[i] = r.perm[k];
      r.perm[k] = p;
    }
  }
  r.meta[0] = steps;
  r.meta[1] = rot;
  r.meta[2] = err;
  return err;
}

// device variant of phase C: one lane (the chase is a strict dependency
// chain; see DESIGN.md for why the default runs it on the host core)
__global__ void __launch_bounds__(64) k_chase(int N, const double *__restrict__ dIn, const double *__restrict__ sdIn,
                                              EigRec r, int maxRot, double *work) {
  if (threadIdx.x != 0) return;
  double *d = work, *sd = work + N, *gc = work + 2 * N, *gs = work + 3 * N;
  for (int i = 0; i < N; i++) {
    d[i] = dIn[i];
    if (i + 1 < N) sd[i] = sdIn[i];
  }
  qr_chase(N, d, sd, r, maxRot, gc, gs);
}

// Phase C application + phase D write-back (CMAES::updateEigensystem).
// Row k of Q replays every Givens rotation in GSL's order:
//   (Q[k][a+i], Q[k][a+i+1]) <- (qi c - qj s, qi s + qj c)
// Rows are independent: workgroups own APPLY_ROWS rows each (their own
// LDS copy).  Along a row the rotations are a dependency chain, but QR step
// t+1 only needs the entries step t has finished: rotation i of step t+1
// touches columns a'+i, a'+i+1, final in step t after its rotation
// (a'-a)+i+1.  A team of APPLY_TEAM lanes per row therefore runs
// APPLY_TEAM consecutive steps at once in lockstep, lane s lagging lane s-1
// by 2 + (a_s - a_{s-1}) rotations -- for steps whose column range is
// nested in the previous one's (a_s >= a_{s-1}, a_s + nb_s <= a_{s-1} +
// nb_{s-1}); any other step starts a new group.  Every entry still sees the
// same operations in the same order, so the result is GSL's bit for bit.
constexpr int APPLY_TEAM = 16, APPLY_ROWS = 16, APPLY_TPB = APPLY_TEAM * APPLY_ROWS;

// x of lane l-1 (row_shr:1 within each 16-lane DPP row = one team; the
// team's lane 0 gets 0 and never uses it)
__device__ inline double dpp_shr1(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(v & 0xffffffffLL), 0x111, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), 0x111, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int APPLY_HCAP = 256;  // step headers per LDS chunk
// rotations per LDS chunk: up to 4096, what fits next to the rows (>= N - 1,
// one whole QR step, for every N the CMA-ES path accepts)
__host__ __device__ inline int apply_cap(int N) {
  const long long avail = 160LL * 1024 - (long long)N * (APPLY_ROWS + 1) * 8 - 8 * APPLY_HCAP - 16 - 512;
  const long long c = avail / 16;
  return (int)(c > 4096 ? 4096 : c);
}
__host__ __device__ inline size_t apply_lds_bytes(int N) {
  return (size_t)N * (APPLY_ROWS + 1) * sizeof(double) + 16 * (size_t)apply_cap(N) + 8 * APPLY_HCAP + 16;
}

__global__ void __launch_bounds__(APPLY_TPB) k_apply(int N, const double *__restrict__ gQt, EigRec r,
                                                     double *__restrict__ B, double *__restrict__ D, double *minEig,
                                                     double *maxEig, double *eigenFailures, unsigned int *errors,
                                                     unsigned long long *trace) {
  unsigned long long ngroups = 0, nunits = 0, tstart = __builtin_amdgcn_s_memtime();
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lda = N + 1;
  const int S = APPLY_ROWS + 1;                  // Lq[c * S + kl] = Q[k0 + kl][c]
  const int k0 = blockIdx.x * APPLY_ROWS;
  const int nrows = min(APPLY_ROWS, N - k0);
  double *Lq = smem;
  const int cap = apply_cap(N);
  double *csh = Lq + (size_t)N * S;              // cap (c, s) pairs
  int *hsh = (int *)(csh + 2 * (size_t)cap);      // APPLY_HCAP (a, nb)
  int *chunk = hsh + 2 * APPLY_HCAP;
  if (r.meta[2]) {
    if (tid == 0 && blockIdx.x == 0) atomicOr(errors, KG_ERR_EIGEN);
    return;
  }
  for (int idx = tid; idx < N * APPLY_ROWS; idx += APPLY_TPB) {
    const int c = idx / APPLY_ROWS, kl = idx % APPLY_ROWS;
    Lq[c * S + kl] = (kl < nrows) ? gQt[(size_t)c * lda + k0 + kl] : 0.0;
  }
  const int steps = r.meta[0];
  const int kl = tid / APPLY_TEAM, s = tid % APPLY_TEAM;
  const int lane = tid & 63;
  int t0 = 0, ro0 = 0;
  __syncthreads();
  while (t0 < steps) {
    const int hn = min(APPLY_HCAP, steps - t0);
    for (int idx = tid; idx < 2 * hn; idx += APPLY_TPB) hsh[idx] = r.hdr[2 * (size_t)t0 + idx];
    __syncthreads();
    if (tid < 64) {  // wave 0: the longest prefix of whole steps with <= cap rotations
      int base = 0, carry = 0, t1 = hn;
      for (; base < hn; base += 64) {
        const int t = base + lane;
        int v = (t < hn) ? hsh[2 * t + 1] - 1 : 0;
        for (int off = 1; off < 64; off <<= 1) {
          const int u = __shfl_up(v, off, 64);
          if (lane >= off) v += u;
        }
        const unsigned long long over = __ballot(t < hn && carry + v > cap);
        if (over) {
          t1 = base + __builtin_ctzll(over);
          carry += (t1 > base) ? __shfl(v, t1 - base - 1, 64) : 0;
          break;
        }
        carry += __shfl(v, 63, 64);
      }
      if (lane == 0) {
        chunk[0] = t1;
        chunk[1] = carry;
      }
    }
    __syncthreads();
    const int tn = chunk[0], nrot = chunk[1];
    for (int idx = tid; idx < 2 * nrot; idx += APPLY_TPB) csh[idx] = r.cs[2 * (size_t)ro0 + idx];
    __syncthreads();
    double *col = Lq + kl;  // col[c * S] = Q[k0 + kl][c]
    int t = 0, ro = 0;
    while (t < tn) {
      // group of up to APPLY_TEAM nested steps (uniform across the workgroup)
      int my_a = 0, my_nb = 0, my_d = -1, my_ro = 0;
      int pa = hsh[2 * t], pnb = hsh[2 * t + 1], pd = 0, pro = ro, T = pnb - 1, K = 1;
      if (s == 0) {
        my_a = pa;
        my_nb = pnb;
        my_d = 0;
        my_ro = pro;
      }
      while (K < APPLY_TEAM && t + K < tn) {
        const int a2 = hsh[2 * (t + K)], nb2 = hsh[2 * (t + K) + 1];
        if (a2 < pa || a2 + nb2 > pa + pnb) break;
        const int d2 = pd + 2 + (a2 - pa), ro2 = pro + pnb - 1;
        if (s == K) {
          my_a = a2;
          my_nb = nb2;
          my_d = d2;
          my_ro = ro2;
        }
        T = max(T, d2 + nb2 - 1);
        pa = a2;
        pnb = nb2;
        pd = d2;
        pro = ro2;
        K++;
      }
      // Systolic replay: lane s's qj at time tau is exactly the entry lane
      // s-1 finalised at tau-1 ("emit": its rotation output, or its carry
      // one unit after its last rotation), passed by a DPP row shift; lane 0
      // reads LDS (entries final since the previous group).  Every lane
      // also stores what it finalises, so LDS holds the group's result.
      const double *cs = csh + 2 * my_ro;
      const bool act = my_d >= 0 && kl < nrows;
      const int last = act ? my_nb - 1 : 0;  // i == last: emit the carry
      // branch-free body: every lane computes, selects keep the state, the
      // only predicated instruction is the store (issue slots, not latency,
      // bound this loop: one wave64 VALU op = 4 cycles)
      auto clampi = [&](int i1) { return i1 < 0 ? 0 : (i1 > last - 1 ? (last > 0 ? last - 1 : 0) : i1); };
      int ic = clampi(-my_d);
      double cN = cs[2 * ic], sN = cs[2 * ic + 1], qjN = col[(size_t)(my_a + ic + 1) * S];
      double qi = col[(size_t)my_a * S], emit = 0.0;
      T += 1;  // the carry unit of the slowest lane
      for (int tau = 0; tau < T; tau++) {
        const double vin = dpp_shr1(emit);
        const int i = tau - my_d;
        const double c = cN, sn = sN, qjl = qjN;
        ic = clampi(i + 1);
        cN = cs[2 * ic];
        sN = cs[2 * ic + 1];
        qjN = col[(size_t)(my_a + ic + 1) * S];
        qi = (s > 0 && i == -1) ? vin : qi;
        const double qj = (s == 0) ? qjl : vin;
        const double out = qi * c - qj * sn;
        const double qn = qi * sn + qj * c;
        const bool inrot = act && i >= 0 && i < last;
        const bool store = act && i >= 0 && i <= last;
        const double e = inrot ? out : qi;
        if (store) col[(size_t)(my_a + i) * S] = e;
        emit = store ? e : emit;
        qi = inrot ? qn : qi;
      }
      T -= 1;
      t += K;
      ro = pro + pnb - 1;
      ngroups++;
      nunits += T;
    }
    __syncthreads();
    t0 += tn;
    ro0 += nrot;
  }
  if (trace && tid == 0 && blockIdx.x == 0) {
    trace[4] += ngroups;
    trace[5] += nunits;
    trace[6] += steps;
    trace[7] += __builtin_amdgcn_s_memtime() - tstart;
  }
  // updateEigensystem: min/max eigenvalue; keep old B, D if min <= 0
  double mn = r.eval[0], mx = r.eval[0];
  for (int i = 1; i < N; i++) {
    mn = fmin(mn, r.eval[i]);
    mx = fmax(mx, r.eval[i]);
  }
  if (mn <= 0.0) {
    if (tid == 0 && blockIdx.x == 0) *eigenFailures += 1.0;
    return;
  }
  for (int idx = tid; idx < nrows * N; idx += APPLY_TPB) {
    const int kk = idx / N, e = idx % N;
    B[(size_t)(k0 + kk) * N + e] = Lq[(size_t)r.perm[e] * S + kk];
  }
  if (blockIdx.x == 0) {
    for (int i = tid; i < N; i += APPLY_TPB) D[i] = sqrt(r.eval[i]);
    if (tid == 0) {
      *minEig = mn;
      *maxEig = mx;
    }
  }
}

// diagonal covariance (CMAES::eigen diagonal branch): Q = I, eval = diag(C)
__global__ void __launch_bounds__(256) k_eigen_diag(int N, const double *__restrict__ C, double *B, double *D,
                                                    double *minEig, double *maxEig, double *eigenFailures) {
  __shared__ double mnmx[2];
  if (threadIdx.x == 0) {
    double mn = C[0], mx = C[0];
    for (int i = 1; i < N; i++) {
      const double v = C[(size_t)i * N + i];
      if (v < mn) mn = v;
      if (v > mx) mx = v;
    }
    mnmx[0] = mn;
    mnmx[1] = mx;
  }
  __syncthreads();
  if (mnmx[0] <= 0.0) {
    if (threadIdx.x == 0) *eigenFailures += 1.0;
    return;
  }
  for (int idx = threadIdx.x; idx < N * N; idx += blockDim.x) B[idx] = (idx / N == idx % N) ? 1.0 : 0.0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) D[i] = sqrt(C[(size_t)i * N + i]);
  if (threadIdx.x == 0) {
    *minEig = mnmx[0];
    *maxEig = mnmx[1];
  }
}

// ------------------------------------------------------------------------
// Orchestration
size_t eig_mat_bytes(int N) { return (size_t)N * (N + 1) * sizeof(double); }
size_t tridiag_vec_bytes(int N) { return (size_t)(3 * N + 16 + (N > 64 ? N : 64)) * sizeof(double); }
bool eig_use_lds(int N) { return eig_mat_bytes(N) + tridiag_vec_bytes(N) + 256 <= 160 * 1024; }

int EigenSolver::init(int N_, bool hostChase_) {
  N = N_;
  hostChase = hostChase_;
  maxRot = 64 * N * N + 4096;
  const size_t mat = (size_t)N * (N + 1);
  KG_HIP(hipMalloc(&gA, mat * sizeof(double)));
  KG_HIP(hipMalloc(&gH, (size_t)N * N * sizeof(double)));
  KG_HIP(hipMalloc(&gQt, mat * sizeof(double)));
  KG_HIP(hipMalloc(&gWork, mat * sizeof(double)));
  KG_HIP(hipMalloc(&tau, (size_t)N * sizeof(double)));
  KG_HIP(hipMalloc(&dsd, 2 * (size_t)N * sizeof(double)));
  KG_HIP(hipMalloc(&chaseWork, 4 * (size_t)N * sizeof(double)));
  KG_HIP(hipMalloc(&dev.hdr, 2 * (size_t)(maxRot + N) * sizeof(int)));
  KG_HIP(hipMalloc(&dev.cs, 2 * (size_t)maxRot * sizeof(double)));
  KG_HIP(hipMalloc(&dev.meta, 4 * sizeof(int)));
  KG_HIP(hipMalloc(&dev.eval, (size_t)N * sizeof(double)));
  KG_HIP(hipMalloc(&dev.perm, (size_t)N * sizeof(int)));
  KG_HIP(hipMemset(dev.meta, 0, 4 * sizeof(int)));
  if (hostChase) {
    KG_HIP(hipHostMalloc(&h_dsd, 2 * (size_t)N * sizeof(double), hipHostMallocDefault));
    KG_HIP(hipHostMalloc(&host.hdr, 2 * (size_t)(maxRot + N) * sizeof(int), hipHostMallocDefault));
    KG_HIP(hipHostMalloc(&host.cs, 2 * (size_t)maxRot * sizeof(double), hipHostMallocDefault));
    KG_HIP(hipHostMalloc(&host.meta, 4 * sizeof(int), hipHostMallocDefault));
    KG_HIP(hipHostMalloc(&host.eval, (size_t)N * sizeof(double), hipHostMallocDefault));
    KG_HIP(hipHostMalloc(&host.perm, (size_t)N * sizeof(int), hipHostMallocDefault));
    KG_HIP(hipEventCreateWithFlags(&ev_dsd, hipEventDisableTiming));
    hgc.resize(N);
    hgs.resize(N);
  } else {
    KG_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    KG_HIP(hipEventCreateWithFlags(&ev_dsd, hipEventDisableTiming));
    KG_HIP(hipEventCreateWithFlags(&ev_chase, hipEventDisableTiming));
  }
  lds = eig_use_lds(N);
  if (!lds) {
    KG_HIP(hipMalloc(&comm, tmw_comm_words(N) * sizeof(unsigned long long)));
    KG_HIP(hipFuncSetAttribute((const void *)k_tridiag_mw, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)tmw_lds_bytes(N)));
    KG_HIP(hipFuncSetAttribute((const void *)k_unpack_mw, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)umw_lds_bytes(N)));
  }
  const int attr = 160 * 1024;
  KG_HIP(hipFuncSetAttribute((const void *)k_tridiag<true>, hipFuncAttributeMaxDynamicSharedMemorySize, attr));
  KG_HIP(hipFuncSetAttribute((const void *)k_unpack<true>, hipFuncAttributeMaxDynamicSharedMemorySize, attr));
  KG_HIP(hipFuncSetAttribute((const void *)k_apply, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)apply_lds_bytes(N)));
  return 0;
}

EigenSolver::~EigenSolver() {
  for (void *p : {(void *)gA, (void *)gH, (void *)gQt, (void *)gWork, (void *)tau, (void *)dsd, (void *)chaseWork,
                  (void *)dev.hdr, (void *)dev.cs, (void *)dev.meta, (void *)dev.eval, (void *)dev.perm, (void *)comm})
    if (p) (void)hipFree(p);
  for (void *p : {(void *)h_dsd, (void *)host.hdr, (void *)host.cs, (void *)host.meta, (void *)host.eval,
                  (void *)host.perm})
    if (p) (void)hipHostFree(p);
  if (side) (void)hipStreamDestroy(side);
  if (ev_dsd) (void)hipEventDestroy(ev_dsd);
  if (ev_chase) (void)hipEventDestroy(ev_chase);
}

int EigenSolver::run(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
                     double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof, void *profCtx) {
  if (diagonal) {
    hipLaunchKernelGGL(k_eigen_diag, dim3(1), dim3(256), 0, s, N, C, B, D, minEig, maxEig, eigenFailures);
    KG_HIP(hipGetLastError());
    return 0;
  }
  const size_t matb = lds ? eig_mat_bytes(N) : 0;
  double *d = dsd, *sd = dsd + N;
  if (prof) prof(profCtx, "eigen_tridiag", 0);
  if (lds)
    hipLaunchKernelGGL(k_tridiag<true>, dim3(1), dim3(1024), matb + tridiag_vec_bytes(N), s, N, C, gA, gH, tau, d, sd,
                       trace);
  else {
    KG_HIP(hipMemsetAsync(comm, 0, tmw_comm_words(N) * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_tridiag_mw, dim3(tmw_groups(N)), dim3(TMW_TPB), tmw_lds_bytes(N), s, N, C, gH, tau, d, sd,
                       comm, errors);
  }
  KG_HIP(hipGetLastError());
  if (prof) prof(profCtx, "eigen_tridiag", 1);
  EigRec devRec = dev;
  if (hostChase) {
    KG_HIP(hipMemcpyAsync(h_dsd, dsd, 2 * (size_t)N * sizeof(double), hipMemcpyDeviceToHost, s));
    KG_HIP(hipEventRecord(ev_dsd, s));
  } else {
    KG_HIP(hipEventRecord(ev_dsd, s));
    KG_HIP(hipStreamWaitEvent(side, ev_dsd, 0));
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, side, N, d, sd, devRec, maxRot, chaseWork);
    KG_HIP(hipGetLastError());
    KG_HIP(hipEventRecord(ev_chase, side));
  }
  if (prof) prof(profCtx, "eigen_unpack", 0);
  if (lds)
    hipLaunchKernelGGL(k_unpack<true>, dim3(1), dim3(1024), matb + 2 * N * sizeof(double), s, N, gH, tau, gQt);
  else
    hipLaunchKernelGGL(k_unpack_mw, dim3(umw_groups(N)), dim3(UMW_TPB), umw_lds_bytes(N), s, N, gH, tau, gQt);
  KG_HIP(hipGetLastError());
  if (prof) prof(profCtx, "eigen_unpack", 1);
  if (hostChase) {
    // the GPU unpacks Q while this core runs the serial Givens chase
    KG_HIP(hipEventSynchronize(ev_dsd));
    if (prof) prof(profCtx, "eigen_chase_host", 2);
    EigRec hr = host;
    qr_chase(N, h_dsd, h_dsd + N, hr, maxRot, hgc.data(), hgs.data());
    if (prof) prof(profCtx, "eigen_chase_host", 3);
    const int steps = host.meta[0], rot = host.meta[1];
    KG_HIP(hipMemcpyAsync(dev.meta, host.meta, 4 * sizeof(int), hipMemcpyHostToDevice, s));
    KG_HIP(hipMemcpyAsync(dev.hdr, host.hdr, 2 * (size_t)steps * sizeof(int), hipMemcpyHostToDevice, s));
    if (rot) KG_HIP(hipMemcpyAsync(dev.cs, host.cs, 2 * (size_t)rot * sizeof(double), hipMemcpyHostToDevice, s));
    KG_HIP(hipMemcpyAsync(dev.eval, host.eval, (size_t)N * sizeof(double), hipMemcpyHostToDevice, s));
    KG_HIP(hipMemcpyAsync(dev.perm, host.perm, (size_t)N * sizeof(int), hipMemcpyHostToDevice, s));
  } else {
    KG_HIP(hipStreamWaitEvent(s, ev_chase, 0));
  }
  if (prof) prof(profCtx, "eigen_apply", 0);
  hipLaunchKernelGGL(k_apply, dim3((N + APPLY_ROWS - 1) / APPLY_ROWS), dim3(APPLY_TPB), apply_lds_bytes(N), s, N, gQt,
                     devRec, B, D, minEig, maxEig, eigenFailures, errors, trace);
  KG_HIP(hipGetLastError());
  if (prof) prof(profCtx, "eigen_apply", 1);
  return 0;
}

}  // namespace kg
