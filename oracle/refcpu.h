/*
 * refcpu — CPU ORACLE for the korali_amd CMA-ES / TMCMC generation path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * solver loops (JonathanLehner/korali @ 2025-02-26) and of the GSL 2.6 /
 * gslcblas algorithms they call.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the CPU
 * baseline.  The product path (korali_amd/) never links or calls it.
 *
 * Parity pinning: the restatement is checked bit-for-bit against the
 * reference's own committed generation files
 *   tests/python/plot/cmaes/gen000000{00..101}.json   (CMA-ES, N=10, lambda=32)
 *   tests/python/plot/tmcmc/gen0000000{0..7}.json     (TMCMC,  N=3,  P=50)
 * copied (trimmed) into tests/golden/.  The binomial BTPE branch (n*p >= 14)
 * is exercised by no fixture: parity unpinned for that branch only.
 *
 * Floating point: compile with -O2 -ffp-contract=off and no -mfma, matching
 * the reference release build (x86-64 baseline SSE2, no FMA).
 */
#ifndef KORALI_REFCPU_H
#define KORALI_REFCPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- GSL mt19937 (gsl_rng_default) ---------------- */
/* Memory layout equals GSL's mt_state_t on LP64: 624 x unsigned long + int
 * (+4 pad) = 5000 bytes, which is what Korali hex-encodes as "Range"
 * (distribution.cpp.base:10-30). */
typedef struct
{
  uint64_t mt[624];
  int32_t mti;
  int32_t pad;
} kr_rng;

void kr_rng_seed(kr_rng *r, uint64_t seed);
void kr_set_threads(int n);
unsigned long long kr_btpe_draws(void); /* binomial draws that took the BTPE branch so far */ /* OpenMP checker build: threads of the data-parallel loops */
uint32_t kr_rng_get(kr_rng *r);
double kr_rng_uniform(kr_rng *r);
double kr_rng_uniform_pos(kr_rng *r);
double kr_ran_gaussian(kr_rng *r, double sigma);
void kr_ran_gaussian_n(kr_rng *r, size_t n, double *out); /* n x (0 + gaussian(1)), stream order */
double kr_ran_flat(kr_rng *r, double a, double b);
unsigned int kr_ran_binomial(kr_rng *r, double p, unsigned int n);
void kr_ran_multinomial(kr_rng *r, size_t K, unsigned int N, const double *p, unsigned int *n);

/* ---------------- numerical kernels ---------------- */
double kr_hypot(double x, double y); /* fdlibm __ieee754_hypot (glibc < 2.35) */
double kr_dnrm2(size_t n, const double *x, size_t inc);
/* gsl_eigen_symmv + gsl_eigen_symmv_sort(ABS_ASC); A (row-major n x n) is
 * destroyed; evec row-major, column i = eigenvector i.  Returns #qrsteps. */
size_t kr_eigen_symmv(size_t n, double *A, double *eval, double *evec);
size_t kr_eigen_symmv_unsorted(size_t n, double *A, double *eval, double *evec);
void kr_symmtd_decomp(size_t N, double *A, double *tau); /* linalg/symmtd.c alone */
size_t kr_qr_chase(size_t N, double *d, double *sd, double *cs, size_t maxRot);
double kr_chi2inv_068(size_t n); /* gsl_cdf_chisq_Pinv(0.68, n), n <= 128 */
int kr_cholesky(size_t n, double *A); /* 0 ok, 1 not positive definite */
void kr_dtrmv_lower(size_t n, const double *L, double *x);
double kr_stats_mean(const double *x, size_t n);
double kr_stats_sd_m(const double *x, size_t n, double mean);

/* ---------------- objectives (examples/optimization/stochastic/_model) -- */
/* correctly-rounded cos / exp (double-double, one rounding) */
double kr_cos_cr(double x);
double kr_exp_cr(double x);
double kr_obj_negative_rosenbrock(const double *x, size_t n);
double kr_obj_negative_ackley(const double *x, size_t n);
double kr_obj_negative_sphere(const double *x, size_t n); /* -0.5*sum x^2 */
double kr_loglik_gaussian(const double *x, size_t n);     /* -0.5*sum x^2 */

/* ---------------- CMA-ES (CMAES.cpp.base) ---------------- */
typedef struct kr_cmaes kr_cmaes;
/* a sample's constraint values: out[c] for c < nc (Problem "Constraints") */
typedef void (*kr_constraint_fn)(const double *x, size_t N, double *out, size_t nc, void *ctx);
kr_cmaes *kr_cmaes_new(size_t N, size_t lambda, size_t mu);
void kr_cmaes_free(kr_cmaes *h);
/* named field access: returns a pointer to the double array / scalar and its
 * element count.  Integer-valued reference fields are kept as doubles except
 * "Sorting Index" (size_t array, use kr_cmaes_sorting_index). */
double *kr_cmaes_field(kr_cmaes *h, const char *name, size_t *len);
size_t *kr_cmaes_sorting_index(kr_cmaes *h);
kr_rng *kr_cmaes_rng(kr_cmaes *h, int which); /* 0 normal, 1 uniform */
void kr_cmaes_set_option(kr_cmaes *h, const char *name, double value);
void kr_cmaes_initialize(kr_cmaes *h);   /* setInitialConfiguration :14-184 */
void kr_cmaes_prepare(kr_cmaes *h);      /* prepareGeneration :439-492 */
void kr_cmaes_eigen_only(kr_cmaes *h);   /* updateEigensystem(C) :869-890 */
void kr_cmaes_sample_only(kr_cmaes *h);  /* draw loop of prepareGeneration */
void kr_cmaes_evaluate(kr_cmaes *h, int objective); /* 0 rosen 1 ackley 2 sphere */
void kr_cmaes_update(kr_cmaes *h, size_t generation); /* updateDistribution :547-688 */
/* whole generation (runGeneration :186-231) with a builtin objective */
void kr_cmaes_generation(kr_cmaes *h, size_t generation, int objective);
/* CCMA-ES (CMAES.cpp.base:315-437, :774-832) */
void kr_cmaes_set_constraints(kr_cmaes *h, size_t nc, size_t viabilityPopulationSize, size_t viabilityMuValue,
                              kr_constraint_fn fn, void *ctx);
void kr_cmaes_check_mean_and_set_regime(kr_cmaes *h);
void kr_cmaes_update_constraints(kr_cmaes *h, size_t generation);
void kr_cmaes_handle_constraints(kr_cmaes *h);
void kr_cmaes_ccmaes_prepare(kr_cmaes *h, size_t generation);
int kr_cmaes_constraint_error(kr_cmaes *h);

/* ---------------- TMCMC (TMCMC.cpp.base) ---------------- */
typedef struct kr_tmcmc kr_tmcmc;
kr_tmcmc *kr_tmcmc_new(size_t N, size_t P);
void kr_tmcmc_free(kr_tmcmc *h);
double *kr_tmcmc_field(kr_tmcmc *h, const char *name, size_t *len);
kr_rng *kr_tmcmc_rng(kr_tmcmc *h, int which); /* 0 multinomial 1 multivariate 2 uniform 3+k prior k */
void kr_tmcmc_set_option(kr_tmcmc *h, const char *name, double value);
void kr_tmcmc_set_prior_map(kr_tmcmc *h, const int *map);
void kr_tmcmc_set_per_generation_burn_in(kr_tmcmc *h, const double *v, size_t n); /* setBurnIn :781-789 */
void kr_tmcmc_initialize(kr_tmcmc *h);                   /* setInitialConfiguration :21-105 */
void kr_tmcmc_prepare(kr_tmcmc *h, size_t generation);   /* prepareGeneration :159-227 */
/* evaluate candidates with the builtin Gaussian likelihood + uniform priors */
void kr_tmcmc_evaluate(kr_tmcmc *h);
/* processCandidate for every chain in chain order (Sequential conduit) */
void kr_tmcmc_process_candidates(kr_tmcmc *h, size_t generation);
void kr_tmcmc_process_generation(kr_tmcmc *h);           /* :254-381 */
/* mTMCMC (set_option "Version" 1, "Step Size", "Domain Extension Factor"
 * before kr_tmcmc_initialize): calculateGradients + calculateProposals
 * :383-558 from every candidate's gradient (P x N) and Fisher information
 * (P x N x N); call after the evaluations, generations > 1 */
void kr_tmcmc_set_gradients(kr_tmcmc *h, const double *grad, const double *fim);
void kr_tmcmc_generation(kr_tmcmc *h, size_t generation);
/* nmsimplex min search (minSearch :712-779); returns #iterations */
size_t kr_tmcmc_minsearch(const double *loglike, size_t Ns, double exponent, double objCov, double *xmin, double *fmin);
double kr_tmcmc_cv2(double x, const double *loglike, size_t Ns, double exponent, double targetCOV);

#ifdef __cplusplus
}
#endif
#endif
