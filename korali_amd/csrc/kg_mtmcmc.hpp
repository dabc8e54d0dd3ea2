// kg_mtmcmc.hpp — host side of mTMCMC (TMCMC.cpp.base:383-681): the
// per-chain proposal construction and acceptance densities, on the host
// thread that drives the handle, as in the reference (N x N per chain:
// LU factorisation and inverse of the annealed Fisher information, its
// eigendecomposition, the boundary correction, the proposal covariance,
// Cholesky factors and Gaussian log-densities).  Same operation order as
// GSL 2.6's Level-2 routines and gslcblas, restated independently of the
// oracle (oracle/refcpu.c, which the product never links).  Part of the
// unity build korali_amd.hip (after kg_eigen.hip: hypot_fdlibm).
#pragma once
#include <cmath>
#include <cstring>
#include <vector>

namespace kg {
namespace mt {

// gsl_cdf_chisq_Pinv(0.68, N), N = 1..128 (tools/make_chi2_table.py)
constexpr double CHI2_068[128] = {
    0.988946481478023, 2.27886856637673, 3.505882355768179, 4.695422319122993,
  5.8608022596974125, 7.009169946950603, 8.144788668939585, 9.270418200246363,
  10.387958013319528, 11.498778181311328, 12.603903905356493, 13.704125276314006,
  14.800066067589455, 15.892228745155391, 16.98102499350416, 18.066797057367218,
  19.149833056062814, 20.230378223312684, 21.308643320753227, 22.38481104613223,
  23.459040989954513, 24.53147352253592, 25.602232880235793, 26.67142964341346,
  27.739162746301982, 28.805521122384825, 29.870585062847724, 30.934427346913328,
  31.997114189146984, 33.05870603866459, 34.119258257565306, 35.17882170015321,
  36.237443210107635, 37.29516604936419, 38.35203026982309, 39.40807303692524,
  40.46332891249609, 41.517830102949176, 42.571606677894444, 43.6246867633504,
  44.67709671307324, 45.728861260956485, 46.78000365699435, 47.83054578892401,
  48.880508291347134, 49.929910643870045, 50.97877125958297, 52.02710756501539,
  53.074936072549725, 54.122272446144436, 55.16913156110684, 56.215527558560616,
  57.26147389517232, 58.30698338863145, 59.35206825931891, 60.39674016854704,
  61.44101025370968, 62.48488916064193, 63.528387073455576, 64.57151374208671,
  65.61427850776624, 66.65669032660158, 67.69875779143783, 68.74048915214941,
  69.78189233449768, 70.82297495767644, 71.86374435065521, 72.90420756741935,
  73.9443714011968, 74.98424239775245, 76.0238268678238, 77.06313089876471,
  78.10216036545802, 79.14092094055236, 80.17941810407355, 81.21765715245671,
  82.2556432070412, 83.29338122206687, 84.33087599220691, 85.36813215966977,
  86.4051542208999, 87.44194653290452, 88.47851331923188, 89.51485867562381,
  90.55098657536443, 91.5869008743443, 92.62260531585866, 93.65810353515641,
  94.6933990637555, 95.72849533353936, 96.7633956806475, 97.79810334917329,
  98.83262149467973, 99.86695318754488, 100.90110141614619, 101.93506908989364,
  102.96885904212003, 104.00247403283672, 105.03591675136242, 106.06918981883199,
  107.10229579059188, 108.13523715848865, 109.1680163530559, 110.20063574560554,
  111.2330976502281, 112.26540432570714, 113.29755797735193, 114.32956075875305,
  115.36141477346426, 116.39312207661503, 117.4246846764566, 118.45610453584531,
  119.48738357366618, 120.5185236661994, 121.5495266484329, 122.58039431532332,
  123.6111284230079, 124.64173068996958, 125.67220279815764, 126.70254639406568,
  127.73276308976914, 128.76285446392407, 129.79282206272907, 130.82266740085166,
  131.85239196232124, 132.88199720138954, 133.91148454336053, 134.9408553853905,
};

inline double chi2inv_068(size_t N) { return (N >= 1 && N <= 128) ? CHI2_068[N - 1] : NAN; }

// gsl_linalg_cholesky_decomp (Level-2 form, gslcblas dgemv order) with the
// upper triangle mirrored; false (and the partial factor) at a
// non-positive pivot, as with GSL's error handler off
inline bool cholesky(size_t N, double *A) {
  for (size_t j = 0; j < N; ++j) {
    for (size_t r = j; j > 0 && r < N; r++) {
      double temp = 0.0;
      for (size_t i = 0; i < j; i++) temp += A[j * N + i] * A[r * N + i];
      A[r * N + j] += -1.0 * temp;
    }
    double ajj = A[j * N + j];
    if (ajj <= 0.0) return false;
    ajj = std::sqrt(ajj);
    const double f = 1.0 / ajj;
    for (size_t r = j; r < N; r++) A[r * N + j] *= f;
  }
  for (size_t j = 1; j < N; ++j)
    for (size_t i = 0; i < j; ++i) A[i * N + j] = A[j * N + i];
  return true;
}

// gslcblas dtrmv RowMajor Lower NoTrans NonUnit
inline void dtrmv_lower(size_t N, const double *L, double *x) {
  for (size_t i = N; i-- > 0;) {
    double temp = 0.0;
    for (size_t j = 0; j < i; j++) temp += x[j] * L[N * i + j];
    x[i] = temp + x[i] * L[N * i + i];
  }
}

// gslcblas dgemv RowMajor NoTrans, beta 1: y_i += alpha (sum_j A_ij x_j)
inline void dgemv_add(size_t N, double alpha, const double *A, const double *x, double *y) {
  for (size_t i = 0; i < N; i++) {
    double temp = 0.0;
    for (size_t j = 0; j < N; j++) temp += A[i * N + j] * x[j];
    y[i] += alpha * temp;
  }
}

// gsl_linalg_LU_decomp: partial pivoting by rows
inline void lu_decomp(size_t N, double *A, size_t *perm) {
  for (size_t i = 0; i < N; i++) perm[i] = i;
  for (size_t j = 0; j + 1 < N; j++) {
    double amax = std::fabs(A[j * N + j]);
    size_t ip = j;
    for (size_t i = j + 1; i < N; i++)
      if (std::fabs(A[i * N + j]) > amax) {
        amax = std::fabs(A[i * N + j]);
        ip = i;
      }
    if (ip != j) {
      for (size_t k = 0; k < N; k++) std::swap(A[j * N + k], A[ip * N + k]);
      std::swap(perm[j], perm[ip]);
    }
    const double ajj = A[j * N + j];
    if (ajj == 0.0) continue;
    for (size_t i = j + 1; i < N; i++) {
      const double aij = A[i * N + j] / ajj;
      A[i * N + j] = aij;
      for (size_t k = j + 1; k < N; k++) A[i * N + k] = A[i * N + k] - aij * A[j * N + k];
    }
  }
}

// gsl_linalg_LU_invert: each identity column through LU_svx (permutation
// v'_i = v_{p_i}, forward substitution with unit L, back substitution
// with U)
inline void lu_invert(size_t N, const double *LU, const size_t *perm, double *inv) {
  std::vector<double> x(N);
  for (size_t c = 0; c < N; c++) {
    for (size_t i = 0; i < N; i++) x[i] = (perm[i] == c) ? 1.0 : 0.0;
    for (size_t i = 1; i < N; i++) {
      double tmp = x[i];
      for (size_t j = 0; j < i; j++) tmp -= LU[i * N + j] * x[j];
      x[i] = tmp;
    }
    x[N - 1] = x[N - 1] / LU[(N - 1) * N + (N - 1)];
    for (size_t i = N - 1; i-- > 0;) {
      double tmp = x[i];
      for (size_t j = i + 1; j < N; j++) tmp -= LU[i * N + j] * x[j];
      x[i] = tmp / LU[i * N + i];
    }
    for (size_t i = 0; i < N; i++) inv[i * N + c] = x[i];
  }
}

// gslcblas dnrm2 (scaled sum of squares)
inline double dnrm2(size_t n, const double *x, size_t inc) {
  if (n == 0) return 0.0;
  if (n == 1) return std::fabs(x[0]);
  double scale = 0.0, ssq = 1.0;
  for (size_t i = 0; i < n; i++) {
    const double xi = x[i * inc];
    if (xi != 0.0) {
      const double ax = std::fabs(xi);
      if (scale < ax) {
        ssq = 1.0 + ssq * (scale / ax) * (scale / ax);
        scale = ax;
      } else {
        ssq += (ax / scale) * (ax / scale);
      }
    }
  }
  return scale * std::sqrt(ssq);
}

// gsl_eigen_symmv without sorting (TMCMC.cpp.base:468): Householder
// tridiagonalisation (symmtd), Q accumulated by householder_hm, implicit
// QR with Wilkinson shifts and Givens rotations applied to Q.
inline void symmv_unsorted(size_t N, double *A, double *eval, double *evec) {
  if (N == 1) {
    eval[0] = A[0];
    evec[0] = 1.0;
    return;
  }
  constexpr double EPS = 2.2204460492503131e-16, DMIN = 2.2250738585072014e-308;
  std::vector<double> tau(N, 0.0), d(N), sd(N), gc(N), gs(N);
  for (size_t i = 0; i + 2 < N; i++) {
    const size_t n = N - (i + 1);
    double *v = A + (i + 1) * N + i;  // column below the diagonal, stride N
    double ti = 0.0;
    // gsl_linalg_householder_transform
    if (n > 1) {
      const double xnorm = dnrm2(n - 1, v + N, N);
      if (xnorm != 0.0) {
        const double alpha = v[0];
        const double beta = -(alpha >= 0.0 ? 1.0 : -1.0) * hypot_fdlibm(alpha, xnorm);
        ti = (beta - alpha) / beta;
        const double s = alpha - beta;
        if (std::fabs(s) > DMIN) {
          const double f = 1.0 / s;
          for (size_t k = 1; k < n; k++) v[k * N] *= f;
        } else {
          const double f1 = EPS / s, f2 = 1.0 / EPS;
          for (size_t k = 1; k < n; k++) v[k * N] *= f1;
          for (size_t k = 1; k < n; k++) v[k * N] *= f2;
        }
        v[0] = beta;
      }
    }
    if (ti != 0.0) {
      double *m = A + (i + 1) * N + (i + 1);
      double *x = tau.data() + i;  // scratch of length n (tau[i..])
      const double ei = v[0];
      v[0] = 1.0;
      for (size_t r = 0; r < n; r++) x[r] = 0.0;
      for (size_t r = n; r-- > 0;) {  // dsymv Lower, alpha tau, beta 0
        const double t1 = ti * v[r * N];
        double t2 = 0.0;
        x[r] += t1 * m[r * N + r];
        for (size_t j = 0; j < r; j++) {
          x[j] += t1 * m[r * N + j];
          t2 += v[j * N] * m[r * N + j];
        }
        x[r] += ti * t2;
      }
      double xv = 0.0;
      for (size_t r = 0; r < n; r++) xv += x[r] * v[r * N];
      const double alpha = -(ti / 2.0) * xv;
      for (size_t r = 0; r < n; r++) x[r] += alpha * v[r * N];
      for (size_t r = 0; r < n; r++) {  // dsyr2 Lower, alpha -1
        const double a1 = -1.0 * v[r * N], a2 = -1.0 * x[r];
        for (size_t j = 0; j <= r; j++) m[r * N + j] += a1 * x[j] + a2 * v[j * N];
      }
      v[0] = ei;
    }
    tau[i] = ti;
  }
  // symmtd_unpack: Q = I, H_i applied for i = N-3 .. 0
  std::memset(evec, 0, sizeof(double) * N * N);
  for (size_t i = 0; i < N; i++) evec[i * N + i] = 1.0;
  for (size_t i = N - 2; i-- > 0;) {
    const double t = tau[i];
    if (t == 0.0) continue;
    const size_t n = N - (i + 1);
    const double *hv = A + (i + 1) * N + i;
    double *Q = evec + (i + 1) * N + (i + 1);
    for (size_t j = 0; j < n; j++) {
      double wj = Q[j];
      for (size_t r = 1; r < n; r++) wj += Q[r * N + j] * hv[r * N];
      Q[j] = Q[j] - t * wj;
      for (size_t r = 1; r < n; r++) Q[r * N + j] = Q[r * N + j] - t * hv[r * N] * wj;
    }
  }
  for (size_t i = 0; i < N; i++) d[i] = A[i * N + i];
  for (size_t i = 0; i + 1 < N; i++) sd[i] = A[(i + 1) * N + i];
  auto chop = [&](size_t n, const double *dd, double *ss) {
    double di = dd[0];
    for (size_t i = 0; i + 1 < n; i++) {
      const double dn = dd[i + 1];
      if (std::fabs(ss[i]) < EPS * (std::fabs(di) + std::fabs(dn))) ss[i] = 0.0;
      di = dn;
    }
  };
  auto givens = [](double a, double b, double &c, double &s) {
    if (b == 0) {
      c = 1;
      s = 0;
    } else if (std::fabs(b) > std::fabs(a)) {
      const double t = -a / b, s1 = 1.0 / std::sqrt(1 + t * t);
      s = s1;
      c = s1 * t;
    } else {
      const double t = -b / a, c1 = 1.0 / std::sqrt(1 + t * t);
      c = c1;
      s = c1 * t;
    }
  };
  chop(N, d.data(), sd.data());
  size_t b = N - 1;
  while (b > 0) {
    if (sd[b - 1] == 0.0 || std::isnan(sd[b - 1])) {
      b--;
      continue;
    }
    size_t a = b - 1;
    while (a > 0 && sd[a - 1] != 0.0) a--;
    const size_t n = b - a + 1;
    double *dd = d.data() + a, *ss = sd.data() + a;
    // qrstep with the trailing (Wilkinson) shift
    double mu;
    {
      const double ta = dd[n - 2], tb = dd[n - 1], tab = ss[n - 2], dt = (ta - tb) / 2.0;
      if (dt > 0)
        mu = tb - tab * (tab / (dt + hypot_fdlibm(dt, tab)));
      else if (dt == 0)
        mu = tb - std::fabs(tab);
      else
        mu = tb + tab * (tab / ((-dt) + hypot_fdlibm(dt, tab)));
    }
    if (EPS * std::fabs(mu) > (std::fabs(dd[0]) + std::fabs(ss[0]))) mu = 0;
    double x = dd[0] - mu, z = ss[0], ak = 0, bk = 0, zk = 0, ap = dd[0], bp = ss[0], aq = dd[1];
    if (n == 2) {
      double c, s;
      givens(x, z, c, s);
      gc[0] = c;
      gs[0] = s;
      const double ap1 = c * (c * ap - s * bp) + s * (s * aq - c * bp);
      const double bp1 = c * (s * ap + c * bp) - s * (s * bp + c * aq);
      const double aq1 = s * (s * ap + c * bp) + c * (s * bp + c * aq);
      dd[0] = ap1;
      ss[0] = bp1;
      dd[1] = aq1;
    } else {
      double bq = ss[1];
      size_t k = 0;
      for (; k < n - 1; k++) {
        double c, s;
        givens(x, z, c, s);
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
        if (k < n - 2) aq = dd[k + 2];
        if (k < n - 3) bq = ss[k + 2];
        dd[k] = ak;
        if (k > 0) ss[k - 1] = bk1;
        if (k < n - 2) ss[k + 1] = bp;
        x = bk;
        z = zk;
      }
      dd[k] = ap;
      ss[k - 1] = bk;
    }
    for (size_t k = 0; k + 1 < n; k++) {
      const double c = gc[k], s = gs[k];
      for (size_t r = 0; r < N; r++) {
        const double qi = evec[r * N + a + k], qj = evec[r * N + a + k + 1];
        evec[r * N + a + k] = qi * c - qj * s;
        evec[r * N + a + k + 1] = qi * s + qj * c;
      }
    }
    chop(n, dd, ss);
  }
  for (size_t i = 0; i < N; i++) eval[i] = d[i];
}

// gsl_ran_multivariate_gaussian_log_pdf with the lower Cholesky factor L
inline double mvn_log_pdf(size_t N, const double *x, const double *mu, const double *L) {
  std::vector<double> w(N);
  for (size_t i = 0; i < N; i++) w[i] = x[i] - mu[i];
  w[0] = w[0] / L[0];
  for (size_t i = 1; i < N; i++) {
    double tmp = w[i];
    for (size_t j = 0; j < i; j++) tmp -= L[i * N + j] * w[j];
    w[i] = tmp / L[i * N + i];
  }
  double quad = 0.0, logdet = 0.0;
  for (size_t i = 0; i < N; i++) quad += w[i] * w[i];
  for (size_t i = 0; i < N; i++) logdet += host_log_cr(L[i * N + i]);
  return -0.5 * quad - logdet - 0.5 * (double)N * host_log_cr(2.0 * 3.14159265358979323846);
}

}  // namespace mt
}  // namespace kg
