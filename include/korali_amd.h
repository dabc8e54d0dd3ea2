/*
 * korali_amd.h — C-ABI of the MI355X-native population-generation engine.
 *
 * This is the drop-in boundary for Korali's population-based solver
 * generation loop.  The reference calls GSL / gslcblas directly from its C++
 * solver modules; each entry point below replaces one of those solver
 * stages (reference paths relative to the korali root):
 *
 *   kg_cmaes_initialize   CMAES::setInitialConfiguration   CMAES.cpp.base:14-184
 *                         (initMuWeights :233-284, initCovariance :286-313)
 *   kg_cmaes_sample       CMAES::prepareGeneration         CMAES.cpp.base:439-492
 *                         (updateEigensystem/eigen :869-938, sampleSingle
 *                          :494-545, Optimizer::isSampleFeasible
 *                          optimizer.cpp.base:5-14, Normal::getRandomNumber
 *                          univariate/normal/normal.cpp.base:32-35)
 *   kg_cmaes_eval_builtin Optimization::evaluate → user objective
 *                         optimization.cpp.base:26-34, batched over λ
 *   kg_cmaes_get_candidates / kg_cmaes_set_fitness
 *                         KORALI_START/WAITALL/GET of CMAES::runGeneration
 *                         CMAES.cpp.base:204-224 (host-callback objectives)
 *   kg_cmaes_update       CMAES::updateDistribution        CMAES.cpp.base:547-688
 *                         (sort_index :940-950, adaptC :690-718,
 *                          updateSigma :720-761, numericalErrorTreatment :763-772)
 *   kg_cmaes_generation   CMAES::runGeneration             CMAES.cpp.base:186-231
 *   kg_cmaes_{get,set}_field / _{get,set}_rng
 *                         Module::getConfiguration / setConfiguration of the
 *                         solver state incl. RNG "Range" (distribution.cpp.base:10-62)
 *
 *   kg_tmcmc_*            TMCMC::runGeneration             TMCMC.cpp.base:107-157
 *
 * Conventions: every function returns 0 on success and non-zero on error;
 * kg_last_error() returns the message (thread-local).  No C++ exceptions or
 * torch types cross this boundary.  Host arrays are caller-owned and copied;
 * device buffers are owned by the handle.  Matrices are row-major doubles,
 * exactly as the reference stores them (std::vector<double> N*N).
 */
#ifndef KORALI_AMD_H
#define KORALI_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KG_ABI_VERSION 8

const char *kg_last_error(void);
int kg_abi_version(void);
int kg_device_count(int *count);

/* -------------------------------------------------------------- CMA-ES */
typedef struct kg_cmaes_s *kg_cmaes_t;

enum kg_mu_type { KG_MU_LOGARITHMIC = 0, KG_MU_LINEAR = 1, KG_MU_EQUAL = 2, KG_MU_PROPORTIONAL = 3 };
enum kg_objective { KG_OBJ_NEGATIVE_ROSENBROCK = 0, KG_OBJ_NEGATIVE_ACKLEY = 1, KG_OBJ_NEGATIVE_SPHERE = 2 };
/* Covariance rank-mu update: EXACT replays the reference's sequential
 * per-element summation (bit-faithful); MFMA sums y_k y_k^T on the FP64
 * matrix cores (v_mfma_f64_16x16x4f64), within 1e-12 relative. */
enum kg_cov_mode { KG_COV_EXACT = 0, KG_COV_MFMA = 1 };

typedef struct {
  size_t variable_count;  /* N  (CMAES "Variable Count") */
  size_t population_size; /* λ  ("Population Size") */
  size_t mu_value;        /* μ  ("Mu Value"; 0 → λ/2, CMAES.cpp.base:27) */
  int mu_type;            /* enum kg_mu_type ("Mu Type") */
  double initial_sigma_cumulation_factor; /* ≤0 → formula default */
  double initial_damp_factor;             /* ≤0 → formula default */
  double initial_cumulative_covariance;   /* ≤0 or >1 → formula default */
  int is_sigma_bounded;                   /* "Is Sigma Bounded" */
  int diagonal_covariance;                /* "Diagonal Covariance" */
  int mirrored_sampling;                  /* "Mirrored Sampling" (pairs z, -z; CMAES.cpp.base:461-491) */
  double max_infeasible_resamplings;      /* "Termination Criteria/Max Infeasible Resamplings" */
  const double *lower_bound;              /* N, may be NULL → -inf */
  const double *upper_bound;              /* N, may be NULL → +inf */
  const double *initial_value;            /* N, NaN → midpoint of bounds */
  const double *initial_std;              /* N, NaN → 0.3*(ub-lb) */
  const double *min_std_update;           /* N, may be NULL → 0 */
  uint64_t normal_seed;                   /* seed of the Normal generator (GSL mt19937) */
  uint64_t uniform_seed;                  /* seed of the Uniform generator */
  int cov_mode;                           /* enum kg_cov_mode */
  int device;                             /* HIP device ordinal */
  int store_bdz;                          /* also keep the BDZ matrix (state export) */
  int eigen_device_chase;                 /* 0: implicit-QR Givens recurrence on the calling host
                                             core, overlapped with the device unpack (default);
                                             1: on one device lane.  Identical results. */
  int shard_rank;                         /* population sharding: this rank's index */
  int shard_count;                        /* ranks sharing one population; 0 or 1 = unsharded */
  /* "Use Gradient Information" / "Gradient Step Size" (CMAES.cpp.base:82-87,
   * :611-621): the mean moves by sum_i w_i step / sqrt(N) g_(i) after the
   * weighted recombination; the samples' gradients come through
   * kg_cmaes_set_gradients (host-evaluated objectives only, unsharded) */
  int use_gradients;
  double gradient_step_size;
  /* "Granularity" of each variable (N, may be NULL → all 0 = continuous;
   * CMAES.cpp.base:44-50, :515-544, :834-867): samples are rounded to it,
   * discrete mutations drawn from the Uniform Generator, sigma follows the
   * masked path length; with or without Mirrored Sampling, sharded or not. */
  const double *granularity;
  /* CCMA-ES (Problem "Constraints"; CMAES.cpp.base:54-68, :132-170,
   * :315-437, :551-580, :724-731, :774-832).  constraint_count > 0: the
   * viability regime (viability_population_size samples, viability_mu_value
   * → half of it) until the mean satisfies every constraint; the constraint
   * values come from the callback of kg_cmaes_set_constraints.  The four
   * doubles below are then required (CMAES.config defaults: 1e6, 0.1818,
   * 0.1, 0.2).  Not with Mirrored Sampling, discrete variables or
   * sharding. */
  size_t constraint_count;
  size_t viability_population_size;
  size_t viability_mu_value;
  double max_covariance_matrix_corrections;
  double target_success_rate;
  double covariance_matrix_adaption_strength;
  double global_success_learning_rate;
} kg_cmaes_cfg;

int kg_cmaes_create(const kg_cmaes_cfg *cfg, kg_cmaes_t *out);

/* Constraint values of `rows` samples (row-major rows x N, host memory):
 * out[r * constraint_count + c] = constraint c at X[r] (Optimization::
 * evaluateConstraints, optimization.cpp.base:11-24: the reference runs
 * sample.run(_constraints[c]) for c in order).  ids[r] = the sample's index
 * in the population, or (size_t)-1 for the mean (checkMeanAndSetRegime).
 * Return 0, or nonzero to abort the generation (kg_last_error() then names
 * the callback). */
typedef int (*kg_constraint_fn)(const double *X, size_t rows, size_t N, const size_t *ids, double *out, void *ctx);
int kg_cmaes_set_constraints(kg_cmaes_t h, kg_constraint_fn fn, void *ctx);
/* CMAES::runGeneration up to the objective with constraints
 * (CMAES.cpp.base:190-196): checkMeanAndSetRegime, prepareGeneration,
 * updateConstraints and handleConstraints (covariance shrunk along the
 * constraint normals on the device, re-decomposed, the violating samples
 * redrawn from the Normal stream and re-evaluated).  Then evaluate the
 * current population (kg_cmaes_population_size rows) and kg_cmaes_update. */
int kg_cmaes_prepare_constrained(kg_cmaes_t h, size_t generation);
/* the current population / mu (CCMA-ES viability regime: the viability sizes) */
int kg_cmaes_population_size(kg_cmaes_t h, size_t *lambda, size_t *mu);
int kg_cmaes_destroy(kg_cmaes_t h);
int kg_cmaes_initialize(kg_cmaes_t h);
int kg_cmaes_sample(kg_cmaes_t h);
int kg_cmaes_eval_builtin(kg_cmaes_t h, int objective);
int kg_cmaes_get_candidates(kg_cmaes_t h, double *X, size_t ld);
int kg_cmaes_set_fitness(kg_cmaes_t h, const double *F);
/* Bayesian problems (F(x) = logPosterior, bayesian.cpp.base:79-84): like
 * kg_cmaes_set_fitness, but -inf (a candidate outside the prior's support)
 * is a valid value; NaN and +inf are still rejected.  Ties sort by index. */
int kg_cmaes_set_log_posterior(kg_cmaes_t h, const double *F);
/* the samples' "Gradient" (lambda x N, row i = sample i), with
 * use_gradients, after kg_cmaes_set_fitness and before kg_cmaes_update */
int kg_cmaes_set_gradients(kg_cmaes_t h, const double *G);
int kg_cmaes_update(kg_cmaes_t h, size_t generation);
/* One whole generation (CMAES::runGeneration).  The device work is enqueued
 * on the handle's stream, but the call itself BLOCKS the calling thread for
 * part of it: with the default host-side Givens chase (cfg eigen_device_chase = 0)
 * the thread waits for the generation's tridiagonal form and then runs the
 * implicit-QR chase itself (kg_eigen.hip EigenSolver::run), streaming the
 * rotations to the device; the call returns once the chase is done and the
 * rest of the generation is queued.  With the device chase (eigen_device_chase =
 * 1, bit-identical, slower) the call only enqueues. */
int kg_cmaes_generation(kg_cmaes_t h, size_t generation, int objective);
/* The next generation's first half ahead of time: the generator prefetch /
 * polar pass and the eigendecomposition's tridiagonalisation and unpack,
 * which touch only workspace (no state a result file holds), so a caller
 * can enqueue them before deciding whether that generation will run (the
 * engine does, before its termination check).  kg_cmaes_sample completes
 * it; without this call kg_cmaes_sample does both halves. */
int kg_cmaes_begin_sample(kg_cmaes_t h);
/* The termination scalars of the last kg_cmaes_update without a stream
 * synchronisation: the device publishes them (and the error flags) into
 * host-coherent memory at the end of the update; this spins until they
 * arrive.  out[] = Model Evaluation Count, Infeasible Sample Count, Maximum
 * Covariance Eigenvalue, Minimum Covariance Eigenvalue, Current Min Standard
 * Deviation, Current Max Standard Deviation, Best Ever Value, Current Best
 * Value, Previous Best Value.  Device-side errors are reported as by
 * kg_cmaes_synchronize.  (Experiment::run's check, experiment.cpp.base:56-99
 * + the generated CMAES/optimizer/solver checkTermination.) */
#define KG_TERMINATION_FIELDS 9
int kg_cmaes_wait_termination_fields(kg_cmaes_t h, double *out);
/* Population sharding over shard_count ranks (one handle per rank, state
 * replicated, λ % shard_count == 0).  kg_cmaes_sample and
 * kg_cmaes_eval_builtin then cover only rows [rank λ/S, (rank+1) λ/S) (with
 * finite bounds, discrete variables, Mirrored Sampling or a diagonal
 * covariance kg_cmaes_sample draws the whole population on every rank: the
 * redraw walk and the ±z pairs are sequential over it);
 * the caller all-gathers "Value Vector" (λ doubles, shards in rank order)
 * — with use_gradients also "Gradients" (λ x N doubles, each rank's rows set
 * by kg_cmaes_set_gradients, shards in rank order) — and then runs the
 * update protocol of the handle's covariance mode.
 *
 * cov_mode KG_COV_EXACT — the reference's summation order, every rank's state
 * bit-identical to the unsharded run (CMAES.cpp.base:603-609, :690-718 sum
 * mean and rank-μ over the selected rows in selection order):
 *   kg_cmaes_update_partial    replicated sort, best bookkeeping; this rank's
 *                              selected rows (ascending selection rank) packed
 *                              into block `rank` of "Shard Rows";
 *   kg_cmaes_shard_row_count   waits for the packing; *count = doubles per
 *                              rank block (0: nothing to exchange);
 *   caller                     in-place all-gather of "Shard Rows", *count
 *                              doubles per rank (skip when 0);
 *   kg_cmaes_update_rows       the μ selected rows in selection order on every
 *                              rank; mean and paths (replicated); the rank-μ
 *                              chains of this rank's share of the covariance's
 *                              lower triangle into "Shard Covariance" (packed,
 *                              entry d (d+1)/2 + e, INT64_MIN bits elsewhere);
 *   caller                     MAX all-reduce of "Shard Covariance" viewed as
 *                              int64 (every entry's owner's exact bits);
 *   kg_cmaes_update_finalize   covariance, σ.
 *
 * cov_mode KG_COV_MFMA — per-shard partial sums (within 1e-12 of the
 * sequential order): kg_cmaes_update_partial, sum all-reduce of "Shard
 * Partials", kg_cmaes_update_finalize.
 *
 * The sort and selection are replicated bit-exactly in both modes. */
int kg_cmaes_update_partial(kg_cmaes_t h, size_t generation);
int kg_cmaes_shard_row_count(kg_cmaes_t h, size_t *count);
int kg_cmaes_update_rows(kg_cmaes_t h, size_t generation);
int kg_cmaes_update_finalize(kg_cmaes_t h, size_t generation);
int kg_cmaes_synchronize(kg_cmaes_t h); /* waits and reports device-side errors */
/* named state fields, keys as in the reference's solver JSON
 * ("Sigma", "Covariance Matrix", "Current Mean", ...); sizes in doubles */
int kg_cmaes_field_size(kg_cmaes_t h, const char *name, size_t *n);
int kg_cmaes_get_field(kg_cmaes_t h, const char *name, double *out, size_t n);
int kg_cmaes_set_field(kg_cmaes_t h, const char *name, const double *in, size_t n);
/* several scalar fields with one device read (termination checks, logging) */
int kg_cmaes_get_fields(kg_cmaes_t h, const char *const *names, size_t count, double *out);
int kg_cmaes_get_sorting_index(kg_cmaes_t h, uint64_t *out);
/* GSL mt19937 state as Korali serialises it: 624 x uint64 words + int32 mti
 * + 4 pad bytes = 5000 bytes.  which: 0 Normal, 1 Uniform generator. */
int kg_cmaes_get_rng(kg_cmaes_t h, int which, void *state5000);
int kg_cmaes_set_rng(kg_cmaes_t h, int which, const void *state5000);
/* device pointer of a named buffer (zero-copy interop) and the HIP stream */
int kg_cmaes_device_ptr(kg_cmaes_t h, const char *name, void **ptr);
int kg_cmaes_stream(kg_cmaes_t h, void **stream);
/* kernel timing probe: average device time (ms) of the named kernel family
 * over the last generation(s) since the previous call, measured with HIP
 * events on the handle's stream; enable with kg_cmaes_profile(h, 1). */
int kg_cmaes_profile(kg_cmaes_t h, int enable);
int kg_cmaes_profile_read(kg_cmaes_t h, const char *stage, double *ms_total, size_t *count);
/* A stage bracketed by the caller (phase 0 = begin, 1 = end): an event pair
 * on the handle's stream, read back with kg_cmaes_profile_read -- the C++
 * engine's exchange steps (collectives enqueued on this stream) under
 * KORALI_AMD_EXCHANGE_PROFILE=1.  Returns 1 for an end without a begin. */
int kg_cmaes_profile_mark(kg_cmaes_t h, const char *stage, int phase);

/* ------------------------------------------------------------ testing */
/* Host reference of the mt19937 jump-ahead the chunked device producer
 * uses: out = the 624 untempered words `distance` positions after window624
 * (window624 = 624 consecutive untempered words of a GSL mt19937 stream,
 * not starting at the seeding word 0).  Runs on the host, no device needed. */
int kg_debug_mt_jump(const uint32_t *window624, uint64_t distance, uint32_t *out624);
/* The host core's tridiagonalisation (phase A of CMAES::eigen,
 * CMAES.cpp.base:896-938 → gsl_linalg_symmtd_decomp, run every generation
 * from prepareGeneration :441) on a given matrix: C row-major N x N (lower
 * triangle read); H (N x N): row i < N-2 = column i below the diagonal
 * (H[i][0] = sd[i], the reflector's entries after it), tau (N), d (N),
 * sd (N).  Runs on the host, no device needed. */
int kg_debug_host_tridiag(size_t N, const double *C, double *H, double *tau, double *d, double *sd);
/* The host core's Givens chase (phase C of the eigendecomposition, GSL
 * eigen/symmv.c + qrstep.c as kg_eigen.hip's qr_chase) on the tridiagonal
 * (d[N], sd[N-1]) reps times: sorted eigenvalues (ABS_ASC) and their
 * permutation, counts[3] = {QR steps, rotations, overflow}, the first cs_cap
 * rotation values (c, s pairs) and the mean wall time per chase.  fused
 * selects the sweep with the chop test folded in.  CPU only (no device code). */
int kg_debug_host_chase(size_t N, const double *d, const double *sd, int fused, size_t reps, double *eval, int *perm,
                        double *cs, size_t cs_cap, int *counts, double *ns_per_chase);
/* Host-only check of the TMCMC resampling (no device call): `reps`
 * consecutive gsl_ran_multinomial draws (K categories, N trials) from one
 * mt19937 seeded with `seed`, by the exact conditional-binomial walk
 * (n_exact) and by the interval-decided walk the handle uses (n_interval);
 * each array holds reps * K counts.  Replaces nothing in the reference
 * (TMCMC.cpp.base:303-309 draws through Multinomial::getSelections). */
int kg_debug_multinomial(uint64_t seed, size_t K, unsigned N, const double *p, size_t reps, unsigned *n_exact,
                         unsigned *n_interval);
/* The device CartPole (examples/learning/reinforcement/cartpole/_model/
 * cartpole.py: scipy dopri5 advance, restated in kg_vracer.hip) on given
 * forces: n trajectories from u0 (n x 4) at t = 0, `steps` advances each with
 * force[j * steps + k]; u_out (n x steps x 4) the state after every advance,
 * over (n x steps) 1 where the pole fell or the cart left the track, -1 where
 * the integration failed.  Runs on `device`. */
int kg_debug_cartpole(int device, const double *u0, const double *force, size_t n, size_t steps, double *u_out,
                      int *over);
/* kg_debug_cartpole from time t0[j] (NULL: 0) instead of 0, the time after
 * the last advance in t_out (n, may be NULL): one environment step at a time
 * on the device's dynamics (a host 'Environment Function' equal to the
 * CartPole kernel, tests/test_gpu_vracer_host_env.py). */
int kg_debug_cartpole_at(int device, const double *u0, const double *t0, const double *force, size_t n, size_t steps,
                         double *u_out, double *t_out, int *over);

/* --------------------------------------------------------------- TMCMC */
typedef struct kg_tmcmc_s *kg_tmcmc_t;

enum kg_likelihood { KG_LIK_GAUSSIAN = 0 }; /* -0.5*sum(x^2), model.py:32-37 */

typedef struct {
  size_t variable_count;  /* N */
  size_t population_size; /* P ("Population Size") */
  double max_chain_length;               /* "Max Chain Length" (>= 1) */
  double default_burn_in;                /* "Burn In" (TMCMC.config "Default Burn In", >= 0) */
  double target_cov;                     /* "Target Coefficient Of Variation" */
  double covariance_scaling;             /* "Covariance Scaling" */
  double min_annealing_exponent_update;  /* "Min Annealing Exponent Update" */
  double max_annealing_exponent_update;  /* "Max Annealing Exponent Update" */
  const double *prior_min;               /* N: Univariate/Uniform prior of each variable */
  const double *prior_max;               /* N */
  /* Korali draws variable d's generation-1 candidate from the distribution
   * object _k->_distributions[_variables[d]->_distributionIndex]
   * (TMCMC.cpp.base:218-220); variables that share a distribution share its
   * RNG.  prior_distribution[d] is that index (NULL: variable d uses
   * distribution d); prior_seeds[k] seeds distribution k. */
  const int *prior_distribution;         /* N or NULL */
  size_t distribution_count;             /* entries of prior_seeds (0: N) */
  const uint64_t *prior_seeds;
  uint64_t multinomial_seed, multivariate_seed, uniform_seed;
  int likelihood;                        /* enum kg_likelihood */
  int device;
  /* "Per Generation Burn In": entry k is the burn-in of generation k+2
   * (setBurnIn, TMCMC.cpp.base:781-789); NULL / 0 entries: Burn In only */
  const double *per_generation_burn_in;
  size_t per_generation_burn_in_count;
  /* chain sharding: shard_count ranks, one handle each,
   * state replicated; 0 = unsharded (kg_tmcmc_process), >= 1 = sharded
   * (the partial / exchange / finalize protocol below, also for one rank) */
  int shard_rank;
  int shard_count;
  /* "Version" (TMCMC.config): 0 TMCMC, 1 mTMCMC — gradient / Fisher
   * information proposals per chain (TMCMC.cpp.base:383-681), with the
   * reference's constraints (:48-83: Max Chain Length 1, Step Size >= 0,
   * Domain Extension Factor >= 0, Uniform priors) and this implementation's
   * (burn-in 0, unsharded, N <= 128, likelihoods set by the caller) */
  int version;
  double step_size;               /* "Step Size" (default 0.1) */
  double domain_extension_factor; /* "Domain Extension Factor" (default 0.2) */
  /* per variable, enum kg_prior_kind (prior_min / prior_max = the
   * distribution's two parameters as listed there).  Variables sharing a
   * distribution share its kind.  NULL: every prior Uniform.  mTMCMC:
   * Uniform only. */
  const int *prior_kind;
} kg_tmcmc_cfg;

enum kg_prior_kind {
  KG_PRIOR_UNIFORM = 0,     /* Minimum, Maximum (uniform.cpp.base) */
  KG_PRIOR_NORMAL = 1,      /* Mean, Standard Deviation (normal.cpp.base) */
  KG_PRIOR_EXPONENTIAL = 2, /* Location, Mean (exponential.cpp.base) */
  KG_PRIOR_LAPLACE = 3,     /* Mean, Width (laplace.cpp.base) */
  KG_PRIOR_CAUCHY = 4,      /* Location, Scale (cauchy.cpp.base) */
  KG_PRIOR_LOGNORMAL = 5    /* Mu, Sigma (logNormal.cpp.base) */
};

int kg_tmcmc_create(const kg_tmcmc_cfg *cfg, kg_tmcmc_t *out);
int kg_tmcmc_destroy(kg_tmcmc_t h);
/* one whole generation (TMCMC::runGeneration) with the builtin likelihood */
int kg_tmcmc_generation(kg_tmcmc_t h, size_t generation);
int kg_tmcmc_synchronize(kg_tmcmc_t h);
int kg_tmcmc_field_size(kg_tmcmc_t h, const char *name, size_t *n);
int kg_tmcmc_get_field(kg_tmcmc_t h, const char *name, double *out, size_t n);
int kg_tmcmc_set_field(kg_tmcmc_t h, const char *name, const double *in, size_t n);
/* which: 0 Multinomial, 1 Multivariate, 2 Uniform, 3+k prior distribution k */
int kg_tmcmc_get_rng(kg_tmcmc_t h, int which, void *state5000);
int kg_tmcmc_set_rng(kg_tmcmc_t h, int which, const void *state5000);
/* the stages of one generation:
 *   prepare  = (gen 1: setInitialConfiguration :21-105) + prepareGeneration :159-227;
 *              the first candidate of every started chain is pending evaluation
 *   evaluate = Bayesian::evaluate with the builtin likelihood (bayesian.cpp.base:24-84)
 *              of the pending candidates
 *   advance  = one step of every unfinished chain (runGeneration's WAITANY loop
 *              :112-144 + processCandidate :229-252): accept / reject, database
 *              entry past the burn-in, and the next candidate of chains with
 *              steps left, which become pending; *pending = their number.
 *              Chains run Chain Lengths[c] + Current Burn In steps, in the
 *              Sequential conduit's chain-major RNG order.
 *   process  = the remaining steps (builtin likelihood) + processGeneration :254-381 */
int kg_tmcmc_prepare(kg_tmcmc_t h, size_t generation);
int kg_tmcmc_evaluate(kg_tmcmc_t h);
int kg_tmcmc_advance(kg_tmcmc_t h, size_t generation, size_t *pending);
/* P flags: 1 where the chain's candidate awaits evaluation */
int kg_tmcmc_get_pending(kg_tmcmc_t h, unsigned char *mask);
int kg_tmcmc_process(kg_tmcmc_t h, size_t generation);
/* Chain sharding over shard_count ranks: each rank draws, evaluates and steps
 * only its contiguous share of the started chains (it counts the whole
 * Multivariate / Uniform streams, so positions stay global).  Then
 *   kg_tmcmc_process_partial  - remaining steps + packs the rank's database,
 *                               leader and candidate rows and its accepted
 *                               count into "Shard Exchange" (int64 words,
 *                               INT64_MIN where the rank owns nothing),
 *   caller                    - MAX all-reduce of "Shard Exchange" viewed as
 *                               int64 (exact bits of every owner), on the
 *                               handle's stream (kg_tmcmc_stream),
 *   kg_tmcmc_process_finalize - unpacks, then processGeneration :254-381
 *                               replicated: every rank's state stays
 *                               bit-identical to the unsharded run. */
int kg_tmcmc_process_partial(kg_tmcmc_t h, size_t generation);
int kg_tmcmc_process_finalize(kg_tmcmc_t h, size_t generation);
int kg_tmcmc_device_ptr(kg_tmcmc_t h, const char *name, void **ptr);
int kg_tmcmc_stream(kg_tmcmc_t h, void **stream);
/* host-callback likelihoods (KORALI_START/WAITANY of TMCMC::runGeneration
 * :114-144): kg_tmcmc_evaluate_prior forms the uniform log-priors of the
 * pending candidates on the device ("Chain Candidates LogPriors"; -inf prior
 * -> logLikelihood -inf, bayesian.cpp.base:56-77), then the host reads the
 * P x N candidates, runs the model for pending chains whose prior is finite
 * and hands both back with kg_tmcmc_set_evaluations (entries of chains that
 * are not pending are ignored), then calls kg_tmcmc_advance; repeat while
 * chains are pending, then kg_tmcmc_process. */
int kg_tmcmc_evaluate_prior(kg_tmcmc_t h);
int kg_tmcmc_get_candidates(kg_tmcmc_t h, double *X, size_t ld);
int kg_tmcmc_set_evaluations(kg_tmcmc_t h, const double *log_prior, const double *log_likelihood);
/* mTMCMC, generations > 1, after kg_tmcmc_set_evaluations:
 * calculateGradients + calculateProposals (TMCMC.cpp.base:383-558) from
 * every candidate's "logLikelihood Gradient" (P x N) and "Fisher
 * Information" (P x N x N, row-major), as Bayesian/Reference computes them
 * (reference.cpp.base:231-621); rows of chains whose candidate log-prior or
 * log-likelihood is not finite are not read.  Also forms the proposal
 * log-density ratios of the acceptance step (:634-677). */
int kg_tmcmc_set_gradients(kg_tmcmc_t h, const double *grad, const double *fisher);
int kg_tmcmc_profile(kg_tmcmc_t h, int enable);
int kg_tmcmc_profile_read(kg_tmcmc_t h, const char *stage, double *ms_total, size_t *count);

/* ---------------------------------------------------------------- VRACER
 * The VRACER agent with the continuous Normal
 * policy, its critic/policy network and the CartPole environment of
 * examples/learning/reinforcement/cartpole, all on the device:
 *
 *   kg_vracer_create              Agent::initialize + VRACER::initializeAgent
 *                                 agent.cpp.base:9-154, VRACER.cpp.base:10-63,
 *                                 continuous.cpp.base:9-93 (Normal transforms)
 *   kg_vracer_run_policy          VRACER::runPolicy              VRACER.cpp.base:183-205
 *   kg_vracer_environment_step    one action of every concurrent environment
 *                                 (continuous.cpp.base:95-150) + Agent::processEpisode
 *                                 of the episodes that ended (agent.cpp.base:376-572)
 *   kg_vracer_train_policy        VRACER::trainPolicy x updates  VRACER.cpp.base:65-181
 *                                 (generateMiniBatch :574-597, updateExperienceMetadata
 *                                 :599-735, DeepSupervisor::runGeneration, fAdam)
 *   kg_vracer_training_step       the body of Agent::trainingGeneration's loop
 *                                 (agent.cpp.base:176-235): environment step, then
 *                                 as many policy updates as Experiences Between
 *                                 Policy Updates allows
 *   kg_vracer_{get,set}_field / _scalar   replay memory, hyperparameters and agent
 *                                 state (the reference's serialized agent fields)
 * Float32 throughout, as the reference.  Hyperparameters are Korali's vector:
 * per layer [W (out x in, row-major), b]. */
typedef struct kg_vracer_s *kg_vracer_t;
typedef struct {
  size_t state_size, action_size;          /* Variables of Type State / Action */
  size_t hidden_size, hidden_layers;       /* Linear + Elementwise/Tanh hidden layers */
  size_t environments;                     /* Concurrent Environments */
  size_t environment_count;                /* Problem / Environment Count */
  size_t mini_batch_size;                  /* Mini Batch / Size */
  size_t replay_maximum_size, replay_start_size;   /* Experience Replay sizes */
  size_t max_episode_steps;                /* the environment's truncation length */
  double experiences_between_policy_updates;
  double discount_factor, learning_rate, importance_weight_truncation_level;
  double off_policy_cutoff_scale, off_policy_target, off_policy_annealing_rate, off_policy_refer_beta;
  int l2_regularization_enabled;
  double l2_regularization_importance;
  const double *initial_exploration_noise; /* action_size values */
  uint64_t seed;                           /* action-noise / mini-batch stream key */
  int device;
  int policy_distribution;                 /* Policy / Distribution: 0 Normal, 1 Clipped Normal */
  const double *action_lower_bounds, *action_upper_bounds;  /* action_size values (may be NULL for Normal) */
  int reward_rescaling;                    /* Reward / Rescaling / Enabled (environment_count <= 8) */
  int state_rescaling;                     /* State Rescaling / Enabled (state_size <= 8) */
  int host_environment;                    /* 1: a host 'Environment Function' feeds the steps
                                              (kg_vracer_host_*); any state_size, action_size <= 4;
                                              0: the device CartPole (4 states, 1 action) */
} kg_vracer_config;

int kg_vracer_create(const kg_vracer_config *cfg, kg_vracer_t *out);
int kg_vracer_destroy(kg_vracer_t h);
int kg_vracer_hyperparameter_count(kg_vracer_t h, size_t *n);
int kg_vracer_field_size(kg_vracer_t h, const char *name, size_t *elem_bytes, size_t *count);
int kg_vracer_get_field(kg_vracer_t h, const char *name, void *dst, size_t bytes);
int kg_vracer_set_field(kg_vracer_t h, const char *name, const void *src, size_t bytes);
int kg_vracer_get_scalar(kg_vracer_t h, const char *name, double *v);
int kg_vracer_set_scalar(kg_vracer_t h, const char *name, double v);
int kg_vracer_run_policy(kg_vracer_t h, const float *states, size_t n, float *out);
/* Use the given standard normals (environments x action_size) for the next
 * environment step's actions instead of the device stream (testing). */
int kg_vracer_set_action_noise(kg_vracer_t h, const float *noise, size_t n);
int kg_vracer_environment_step(kg_vracer_t h, size_t *new_experiences);
/* Agent::rescaleStates (agent.cpp.base:291-322): the replay memory's state
 * moments, every stored state rescaled; episodes launched from then on
 * scale their states with them.  kg_vracer_training_step calls it where the
 * reference does (agent.cpp.base:204-207). */
int kg_vracer_rescale_states(kg_vracer_t h);
int kg_vracer_train_policy(kg_vracer_t h, size_t updates);
/* the policy updates the experiences collected so far call for
 * (Agent::trainingGeneration, agent.cpp.base:201-231: State Rescaling at the
 * first update, then as many updates as Experiences Between Policy Updates
 * allows); kg_vracer_training_step = kg_vracer_environment_step + this */
int kg_vracer_train_pending(kg_vracer_t h, size_t *updates);
/* Host environments (a user 'Environment Function', run by the engine as a
 * coroutine per environment: reinforcementLearning.cpp.base:58-83,
 * :130-200, :276-340).  The device keeps the policy, the episode buffers and
 * the replay memory exactly as for the CartPole kernel; the transitions come
 * from the host:
 *   kg_vracer_host_launch   the first launch of every environment: its
 *                           initial state (E x S, raw: rescaled on the
 *                           device) and Environment Id (E);
 *   kg_vracer_host_act      the policy's action of every environment
 *                           (E x A, continuous.cpp.base:95-150), the
 *                           experience kept in the episode buffer;
 *   kg_vracer_host_feed     each environment's reward, state after the
 *                           action (E x S raw; an ended episode's last
 *                           state), termination (0 non terminal, 1 Terminal,
 *                           2 Truncated) and, for the ended ones, the next
 *                           launch's initial state (E x S) and Environment Id
 *                           (E); then Agent::processEpisode of the ended
 *                           episodes in environment order (agent.cpp.base:376-572).
 *                           Launches take sample ids in launch order. */
int kg_vracer_host_launch(kg_vracer_t h, const float *states, const int *env_ids);
int kg_vracer_host_act(kg_vracer_t h, float *actions);
int kg_vracer_host_feed(kg_vracer_t h, const float *rewards, const float *states, const int *terminations,
                        const float *next_states, const int *next_env_ids, size_t *new_experiences);
int kg_vracer_train_policy_minibatch(kg_vracer_t h, const uint32_t *sorted_ids, size_t count);
int kg_vracer_training_step(kg_vracer_t h, size_t *new_experiences, size_t *updates);
/* Agent::testingGeneration (agent.cpp.base:267-289) on the device CartPole:
 * one episode per entry, reset with seed sample_ids[j] * 1024 +
 * launch_ids[j] (env.py), actions = the policy's mode
 * (generateTestingAction, continuous.cpp.base:219-260: Normal mean, Clipped
 * Normal mean clipped), environment 0's reward, up to max_episode_steps;
 * rewards[j] = the episode's cumulative reward ("Testing Reward",
 * reinforcementLearning.cpp.base:207-255).  Uses the current
 * hyperparameters; replay memory and agent state are untouched. */
int kg_vracer_test_episodes(kg_vracer_t h, const uint64_t *sample_ids, const uint64_t *launch_ids, size_t n,
                            float *rewards);
/* The agent's whole training state in one binary file (replaces
 * Agent::serializeExperienceReplay / deserializeExperienceReplay,
 * agent.cpp.base:849-976, which write the replay memory to
 * <result path>/state.json): the replay memory, the concurrent environments'
 * episodes in flight, the policy, its Adam moments, the agent's scalars and
 * counters, plus user_bytes of the caller's own (the engine's session
 * counters).  kg_vracer_load_state needs a handle created with the same
 * configuration (the seed may differ: the saved one is restored) and
 * continues the saved run bit for bit. */
int kg_vracer_save_state(kg_vracer_t h, const char *path, const void *user, size_t user_bytes);
int kg_vracer_load_state(kg_vracer_t h, const char *path, void *user, size_t user_capacity, size_t *user_bytes);
int kg_vracer_synchronize(kg_vracer_t h);
int kg_vracer_stream(kg_vracer_t h, void **stream);
/* Stage timers (HIP events on the handle's stream): "environment_step",
 * "update", "gemm_rollout" (hidden-layer MFMA products of the rollout
 * forward), "gemm_update".  profile_read returns and resets a stage's total. */
int kg_vracer_profile(kg_vracer_t h, int enable);
int kg_vracer_profile_read(kg_vracer_t h, const char *stage, double *ms_total, size_t *count);

#ifdef __cplusplus
}
#endif
#endif /* KORALI_AMD_H */
