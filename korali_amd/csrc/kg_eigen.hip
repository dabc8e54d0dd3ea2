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
#include "kg_common.hpp"

namespace kg {

namespace {

__device__ inline double readlane_d(double x, int l) {
  const long long v = __double_as_longlong(x);
  int lo = (int)(v & 0xffffffffLL), hi = (int)(v >> 32);
  lo = __builtin_amdgcn_readlane(lo, l);
  hi = __builtin_amdgcn_readlane(hi, l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ inline uint32_t hiw(double x) { return (uint32_t)(__double_as_longlong(x) >> 32); }
__device__ inline uint32_t low(double x) { return (uint32_t)(__double_as_longlong(x) & 0xffffffffLL); }
__device__ inline double sethi(double x, uint32_t h) {
  return __longlong_as_double(((long long)h << 32) | (long long)low(x));
}

// fdlibm __ieee754_hypot (glibc < 2.35), SURVEY.md Appendix A
__device__ double hypot_fdlibm(double x, double y) {
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

__device__ inline void chop_small(int n, const double *d, double *sd) {
  double d_i = d[0];
  for (int i = 0; i + 1 < n; i++) {
    const double sd_i = sd[i], d_ip1 = d[i + 1];
    if (fabs(sd_i) < EPS * (fabs(d_i) + fabs(d_ip1))) sd[i] = 0.0;
    d_i = d_ip1;
  }
}

__device__ inline void create_givens(double a, double b, double &c, double &s) {
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
__device__ void qrstep(int n, double *d, double *sd, double *gc, double *gs) {
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
  double dn = d[min(2, n - 1)], sdn = sd[min(2, n - 2)];
  int k;
  for (k = 0; k < n - 1; k++) {
    const double dpf = d[min(k + 3, n - 1)];   // unconditional loads (values unused past the end)
    const double sdpf = sd[min(k + 3, n - 2)];
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
template <bool kLds>
__global__ void __launch_bounds__(1024) k_symmv(int N, int diagonal, const double *__restrict__ C, double *gA,
                                                double *gH, double *__restrict__ B, double *__restrict__ D,
                                                double *minEig, double *maxEig, double *eigenFailures,
                                                unsigned int *errors, unsigned long long *trace) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wid = tid >> 6;
  const int lda = N + 1;
  double *M = kLds ? smem : gA;  // A during phase A, Qt during B/C
  double *vb = kLds ? smem + (size_t)N * lda : smem;
#define KG_TRACE(i) \
  if (trace && tid == 0) trace[i] = __builtin_amdgcn_s_memtime();
  KG_TRACE(0)
  unsigned long long acc_t[6] = {0, 0, 0, 0, 0, 0}, tmark = 0, nrot = 0;
#define KG_MARK() \
  if (trace && tid == 0) tmark = __builtin_amdgcn_s_memtime();
#define KG_ACC(k) \
  if (trace && tid == 0) acc_t[k] += __builtin_amdgcn_s_memtime() - tmark;
  double *x = vb, *dv = vb + N, *sdv = vb + 2 * N, *tau = vb + 3 * N;
  double *gc = vb + 4 * N, *gs = vb + 6 * N, *ev = vb + 8 * N, *scal = vb + 9 * N;
  int *perm = (int *)(scal + 16);
  int *misc = perm + N;  // [0..1] a, [2..3] n per buffer, [4] fail

  if (diagonal) {
    // CMAES::eigen, diagonal branch: Q = I, diag = diag(M) (no sort)
    for (int i = tid; i < N; i += nt) ev[i] = C[i * N + i];
    __syncthreads();
    if (tid == 0) {
      double mn = ev[0], mx = ev[0];
      for (int i = 1; i < N; i++) {
        if (ev[i] < mn) mn = ev[i];
        if (ev[i] > mx) mx = ev[i];
      }
      scal[0] = mn;
      scal[1] = mx;
    }
    __syncthreads();
    if (scal[0] <= 0.0) {
      if (tid == 0) *eigenFailures += 1.0;
      return;
    }
    for (int idx = tid; idx < N * N; idx += nt) B[idx] = (idx / N == idx % N) ? 1.0 : 0.0;
    for (int i = tid; i < N; i += nt) D[i] = sqrt(ev[i]);
    if (tid == 0) {
      *minEig = scal[0];
      *maxEig = scal[1];
    }
    return;
  }

  // symmetrise from the lower triangle (CMAES.cpp.base:908-913)
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, j = idx % N;
    M[i * lda + j] = (j <= i) ? C[i * N + j] : C[j * N + i];
  }
  __syncthreads();

  if (N == 1) {
    if (tid == 0) {
      ev[0] = M[0];
      perm[0] = 0;
      scal[0] = ev[0];
      scal[1] = ev[0];
    }
    __syncthreads();
    if (tid == 0) {
      if (ev[0] <= 0.0)
        *eigenFailures += 1.0;
      else {
        B[0] = 1.0;
        D[0] = sqrt(ev[0]);
        *minEig = ev[0];
        *maxEig = ev[0];
      }
    }
    return;
  }

  // ---------------------------------------------------------- phase A
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
        // leaves ssq (>= 1) unchanged, so only new-maximum lanes branch
        const double tq = (type == 2) ? q * q : 0.0;
        const unsigned long long m1 = __ballot(type == 1);
        const int cnt = (n - base) < 64 ? (n - base) : 64;
#pragma unroll 8
        for (int l = 0; l < cnt; l++) {
          if ((m1 >> l) & 1ULL) {
            const double qq = readlane_d(q, l);
            ssq = 1.0 + ssq * qq * qq;
          } else {
            ssq += readlane_d(tq, l);
          }
        }
        scale_carry = fmax(scale_carry, readlane_d(pm, 63));
      }
      if (lane == 0) {
        double tau_i = 0.0, f1 = 1.0, f2 = 1.0, beta = 0.0;
        int branch = 0;
        double xnorm = (n - 1 == 1) ? fabs(v[lda]) : scale_carry * sqrt(ssq);
        if (n - 1 == 0) xnorm = 0.0;
        if (n > 1 && xnorm != 0) {
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
        tau[i] = tau_i;
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
    for (int j = tid; j < n; j += nt) {
      const double vj = (j == 0) ? 1.0 : v[(size_t)j * lda];
      // two sequential chains, loads and products issued 16 at a time:
      //   acc: rows r = n-1 .. j+1 (descending)      t2: cols ii = 0 .. j-1
      // Past its own length a chain adds +0.0, which is exact here (neither
      // running sum can be -0.0: both start at +0.0 under round-to-nearest).
      const int L1 = n - 1 - j, L2 = j, L = L1 > L2 ? L1 : L2;
      double acc = 0.0, t2 = 0.0;
      for (int q0 = 0; q0 < L; q0 += 16) {
        double p1[16], p2[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
          // unconditional loads from clamped (valid) addresses, then select:
          // keeps every LDS read of the chunk in flight at once
          const int q = q0 + u;
          const int r = max(n - 1 - q, 0), qc = min(q, n - 1);
          const double pa = (tau_i * v[(size_t)r * lda]) * m[(size_t)r * lda + j];
          const double vq = v[(size_t)qc * lda];
          const double pb = ((q == 0) ? 1.0 : vq) * m[(size_t)j * lda + qc];
          p1[u] = (q < L1) ? pa : 0.0;
          p2[u] = (q < L2) ? pb : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; u++) {
          acc += p1[u];
          t2 += p2[u];
        }
      }
      acc += (tau_i * vj) * m[(size_t)j * lda + j];
      acc += tau_i * t2;
      x[j] = acc;
    }
    __syncthreads();
    KG_ACC(1)
    KG_MARK()
    if (wid == 0) {
      // xv = sum x[r] v[r] sequentially; alpha = -(tau/2) xv
      double xv = 0.0;
      for (int base = 0; base < n; base += 64) {
        const int r = base + lane, rc = min(r, n - 1);
        const double p_ = x[rc] * ((rc == 0) ? 1.0 : v[(size_t)rc * lda]);
        const double p = (r < n) ? p_ : 0.0;
        const int cnt = (n - base) < 64 ? (n - base) : 64;
#pragma unroll 8
        for (int l = 0; l < cnt; l++) xv += readlane_d(p, l);
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
  // tau[N-2] is never set by the loop (GSL's tau has N-1 entries; the last
  // one is unused by unpack)
  // save Householder vectors to global, diag / subdiag to LDS
  for (int idx = tid; idx < N * N; idx += nt) {
    const int i = idx / N, r = idx % N;
    if (i + 2 < N && r < N - i - 1) gH[(size_t)i * N + r] = M[(size_t)(i + 1 + r) * lda + i];
  }
  for (int i = tid; i < N; i += nt) {
    dv[i] = M[(size_t)i * lda + i];
    if (i + 1 < N) sdv[i] = M[(size_t)(i + 1) * lda + i];
  }
  __syncthreads();

  KG_TRACE(1)
  // ---------------------------------------------------------- phase B
  // Qt[col][row] = Q[row][col] = I
  for (int idx = tid; idx < N * lda; idx += nt) {
    const int c = idx / lda, r = idx % lda;
    M[idx] = (r < N && c == r) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int i = N - 3; i >= 0; i--) {
    const double ti = tau[i];
    if (ti == 0.0) continue;  // householder_hm returns early
    const int n = N - (i + 1);
    for (int r = tid; r < n; r += nt) x[r] = gH[(size_t)i * N + r];
    __syncthreads();
    const double *h = x;
    for (int j = tid; j < n; j += nt) {
      double *col = M + (size_t)(i + 1 + j) * lda + (i + 1);  // Q[i+1+r][i+1+j], r = 0..n-1
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
        for (int u = 0; u < 16; u++) wj += p[u];  // +0.0 padding: wj is never -0.0 after col[0]+... (see dsymv)
      }
      col[0] = col[0] - ti * wj;
      for (int r = 1; r < n; r++) col[r] = col[r] - ti * h[r] * wj;
    }
    __syncthreads();
  }

  KG_TRACE(2)
  // ---------------------------------------------------------- phase C
  if (tid == 0) {
    chop_small(N, dv, sdv);
    misc[0] = misc[1] = 0;
    misc[2] = misc[3] = 0;
    misc[4] = N - 1;  // b
    misc[5] = 0;      // steps
  }
  __syncthreads();
  const int maxSteps = 64 * N + 1000;
  for (int step = 0;; step++) {
    const int buf = step & 1;
    if (tid == 0) {
      int b = misc[4];
      int nblk = -1;
      while (b > 0) {
        if (sdv[b - 1] == 0.0 || isnan(sdv[b - 1])) {
          b--;
          continue;
        }
        int a = b - 1;
        while (a > 0) {
          if (sdv[a - 1] == 0.0) break;
          a--;
        }
        nblk = b - a + 1;
        KG_MARK()
        qrstep(nblk, dv + a, sdv + a, gc + buf * N, gs + buf * N);
        chop_small(nblk, dv + a, sdv + a);
        KG_ACC(4)
        nrot += nblk - 1;
        misc[buf] = a;
        if (++misc[5] > maxSteps) {
          atomicOr(errors, KG_ERR_EIGEN);
          nblk = -1;
          b = 0;
        }
        break;
      }
      misc[4] = b;
      misc[2 + buf] = nblk;  // -1: converged
    } else if (tid >= 64 && step > 0 && !(trace && trace[15] == 1)) {
      const int pb = buf ^ 1;
      const int nblk = misc[2 + pb];
      if (nblk > 0) {
        const int a = misc[pb];
        const double *c_ = gc + pb * N, *s_ = gs + pb * N;
        for (int k = tid - 64; k < N; k += nt - 64) {
          double qi = M[(size_t)a * lda + k];
          for (int i = 0; i + 1 < nblk; i++) {
            const double c = c_[i], s = s_[i];
            const double qj = M[(size_t)(a + i + 1) * lda + k];
            M[(size_t)(a + i) * lda + k] = qi * c - qj * s;
            qi = qi * s + qj * c;
          }
          M[(size_t)(a + nblk - 1) * lda + k] = qi;
        }
      }
    }
    __syncthreads();
    if (misc[2 + buf] < 0) break;
  }

  KG_TRACE(3)
  if (trace && tid == 0) trace[6] = (unsigned long long)misc[5];
  // ---------------------------------------------------------- phase D
  for (int i = tid; i < N; i += nt) {
    ev[i] = dv[i];
    perm[i] = i;
  }
  __syncthreads();
  if (wid == 0) {
    for (int i = 0; i + 1 < N; i++) {
      // first index of min |e| over positions >= i (strict <, as GSL)
      double bv = INFINITY;
      int bi = 0x7fffffff;
      for (int j = i + lane; j < N; j += 64) {
        const double a = fabs(ev[j]);
        if (a < bv || (a == bv && j < bi)) {
          bv = a;
          bi = j;
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        if (ov < bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      // the arg-min must still honour 'strict <' against ev[i] itself
      if (lane == 0) {
        int k = i;
        if (fabs(ev[bi]) < fabs(ev[i])) k = bi;
        if (k != i) {
          const double t = ev[i];
          ev[i] = ev[k];
          ev[k] = t;
          const int p = perm[i];
          perm[i] = perm[k];
          perm[k] = p;
        }
      }
      // single wave: order lane 0's LDS updates before the next sweep
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) {
      double mn = ev[0], mx = ev[0];
      for (int i = 1; i < N; i++) {
        if (ev[i] < mn) mn = ev[i];
        if (ev[i] > mx) mx = ev[i];
      }
      scal[6] = mn;
      scal[7] = mx;
    }
  }
  __syncthreads();
  if (scal[6] <= 0.0) {
    if (tid == 0) *eigenFailures += 1.0;
    return;
  }
  for (int idx = tid; idx < N * N; idx += nt) {
    const int d = idx / N, e = idx % N;
    B[idx] = M[(size_t)perm[e] * lda + d];
  }
  for (int i = tid; i < N; i += nt) D[i] = sqrt(ev[i]);
  if (tid == 0) {
    *minEig = scal[6];
    *maxEig = scal[7];
  }
  KG_TRACE(4)
  if (trace && tid == 0) {
    for (int k = 0; k < 5; k++) trace[7 + k] = acc_t[k];
    trace[12] = nrot;
  }
#undef KG_TRACE
#undef KG_MARK
#undef KG_ACC
}

size_t symmv_lds_bytes(int N, bool lds_mats) {
  size_t v = (size_t)(9 * N + 16) * sizeof(double) + (size_t)(N + 8) * sizeof(int);
  if (lds_mats) v += (size_t)N * (N + 1) * sizeof(double);
  return (v + 15) & ~(size_t)15;
}

int launch_symmv(int N, int diagonal, const double *C, double *gA, double *gH, double *B, double *D, double *minEig,
                 double *maxEig, double *eigenFailures, unsigned int *errors, unsigned long long *trace,
                 hipStream_t s) {
  KG_CHECK(N >= 1 && N <= 960, "device eigensolver supports 1 <= N <= 960");
  const bool lds = (symmv_lds_bytes(N, true) <= 160 * 1024);
  const size_t bytes = symmv_lds_bytes(N, lds);
  static bool attr_set = false;
  if (!attr_set) {
    KG_HIP(hipFuncSetAttribute((const void *)k_symmv<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    KG_HIP(hipFuncSetAttribute((const void *)k_symmv<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  if (lds)
    hipLaunchKernelGGL(k_symmv<true>, dim3(1), dim3(1024), bytes, s, N, diagonal, C, gA, gH, B, D, minEig, maxEig,
                       eigenFailures, errors, trace);
  else
    hipLaunchKernelGGL(k_symmv<false>, dim3(1), dim3(1024), bytes, s, N, diagonal, C, gA, gH, B, D, minEig, maxEig,
                       eigenFailures, errors, trace);
  KG_HIP(hipGetLastError());
  return 0;
}

}  // namespace kg
