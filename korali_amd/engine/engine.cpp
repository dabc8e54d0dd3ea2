// engine.cpp — korali::Engine running CMA-ES / TMCMC experiments on the
// korali_amd C-ABI (include/korali_amd.h).
//
// Mirrors, for the solvers on this path, the reference's host side:
//   Engine::run                          source/engine.cpp:69-128
//   Experiment::initialize / run / saveState
//                                        source/modules/experiment/experiment.cpp.base:39-153, 165-251
//   Module::getModule (type strings)     source/modules/module.cpp:87-182
//   Distribution seeding / Range         source/modules/distribution/distribution.cpp.base:10-62
//   Optimization::evaluate               source/modules/problem/optimization/optimization.cpp.base:26-34
//   Bayesian::evaluate (+ Custom)        source/modules/problem/bayesian/bayesian.cpp.base:24-84
//   CMAES / TMCMC termination criteria   CMAES.config, optimizer.config, solver.config, TMCMC.config
// The generation loop itself (sampling, evaluation dispatch, update) runs on
// the device through kg_cmaes_* / kg_tmcmc_*; user functions are called
// from this thread in sample order (Sequential conduit semantics).
#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <exception>
#include <fstream>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <sstream>
#include <thread>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/korali_amd.h"
#include "distributed.hpp"
#include "korali.hpp"

namespace korali {

namespace {

[[noreturn]] void fail(const char *fmt, ...) {
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw KoraliError(std::string("[Korali] Error: ") + buf);
}

void check(int rc) {
  if (rc != 0) fail("%s", kg_last_error());
}

// A replicated evaluation under the Distributed conduit: `local` evaluates
// this rank's share into its block of `buf`, then every rank all-gathers
// `count` doubles per rank -- even a rank whose share threw, so no rank is
// left waiting in the bootstrap -- and one failure flag per rank; a failure
// anywhere is raised on every rank after the gathers (the failing rank's own
// error there, the others name it).
void replicatedGather(Collective &d, std::vector<double> &buf, size_t count, const std::function<void()> &local) {
  std::exception_ptr err;
  try {
    local();
  } catch (...) {
    err = std::current_exception();
  }
  if (count) d.allGatherHost(buf.data(), count);
  std::vector<double> flags((size_t)d.world, 0.0);
  flags[(size_t)d.rank] = err ? 1.0 : 0.0;
  d.allGatherHost(flags.data(), 1);
  if (err) std::rethrow_exception(err);
  for (int r = 0; r < d.world; r++)
    if (flags[(size_t)r] != 0.0) fail("rank %d failed while evaluating its share of the samples (see its error).", r);
}

// Module::getModule: whitespace removed, case-insensitive compare
std::string canon(const std::string &s) {
  std::string r;
  for (char c : s)
    if (!isspace((unsigned char)c)) r += (char)tolower((unsigned char)c);
  return r;
}

double num(Json &j, const char *key, double def) {
  if (!j.contains(key) || j[key].is_null()) j[key] = def;
  return j[key].getDouble();
}
// a mandatory numeric setting (generated setConfiguration, source_builders.py:72-75)
double mandatory(Json &j, const char *key, const char *module) {
  if (!j.contains(key) || j[key].is_null())
    fail(" + No value provided for mandatory setting: ['%s'] required by %s.\n", key, module);
  const double v = j[key].getDouble();
  if (!std::isfinite(v)) fail(" + Non-finite value provided for mandatory setting: ['%s'] required by %s.\n", key, module);
  return v;
}
bool flag(Json &j, const char *key, bool def) {
  if (!j.contains(key) || j[key].is_null()) j[key] = def;
  return j[key].getBool();
}
std::string str(Json &j, const char *key, const std::string &def) {
  if (!j.contains(key) || j[key].is_null()) j[key] = def;
  return j[key].getString();
}
unsigned long long uint(Json &j, const char *key, unsigned long long def) {
  if (!j.contains(key) || j[key].is_null()) j[key] = def;
  return j[key].getUInt();
}

std::string hexState(const unsigned char *b) {
  static const char *hx = "0123456789ABCDEF";
  std::string s(10000, '0');
  for (int i = 0; i < 5000; i++) {
    s[2 * i] = hx[b[i] >> 4];
    s[2 * i + 1] = hx[b[i] & 15];
  }
  return s;
}
bool parseHexState(const std::string &s, unsigned char *b) {
  if (s.size() != 10000) return false;
  auto v = [](char c) { return c >= 'a' ? c - 'a' + 10 : c >= 'A' ? c - 'A' + 10 : c - '0'; };
  for (int i = 0; i < 5000; i++) b[i] = (unsigned char)(v(s[2 * i]) * 16 + v(s[2 * i + 1]));
  return true;
}

// ------------------------------------------------------------- logging
struct Logger {
  int level = 2;  // Silent 0, Minimal 1, Normal 2, Detailed 3
  void set(const std::string &v) {
    const std::string c = canon(v);
    level = c == "silent" ? 0 : c == "minimal" ? 1 : c == "normal" ? 2 : c == "detailed" ? 3 : -1;
    if (level < 0) fail("Unrecognized verbosity level '%s'.", v.c_str());
  }
  void log(int l, const char *fmt, ...) const {
    if (level < l) return;
    va_list ap;
    va_start(ap, fmt);
    printf("[Korali] ");
    vprintf(fmt, ap);
    va_end(ap);
    fflush(stdout);
  }
};

// seed assignment in configuration order (distribution.cpp.base:32-43):
// a generator keeps its seed only when states are preserved
struct Seeder {
  unsigned long long counter;
  bool preserve;
  unsigned long long assign(Json &gen) {
    unsigned long long s = gen.contains("Random Seed") ? gen["Random Seed"].getUInt() : 0;
    if (s == 0 || !preserve) s = counter++;
    gen["Random Seed"] = s;
    return s;
  }
  // saved GSL state to restore (Preserve Random Number Generator States)
  bool range(Json &gen, unsigned char *state) {
    return preserve && gen.contains("Range") && gen["Range"].is_string() && parseHexState(gen["Range"].getString(), state);
  }
};

// ------------------------------------------------------------- conduits
// Host-callback dispatch (the Engine's "Conduit").  Sequential
// (conduit/sequential/sequential.cpp.base:80-92): the engine thread calls
// the user function for every sample in Sample Id order.  Concurrent
// (conduit/concurrent/concurrent.cpp.base:18-231 forks "Concurrent Jobs"
// worker processes and ships each sample's JSON through pipes): here that
// many threads of this process share the batch of one generation (CMA-ES)
// or of one chain round (TMCMC), the engine thread being one of them.
// Results land by Sample Id, so completion order never reaches the solver
// and a run is bit-identical to the Sequential one; of several failing
// samples the lowest Sample Id's error is raised, as in a Sequential run.
// User functions must be safe to call from several threads (Python
// callbacks take the GIL, which the engine releases while it runs).
class Conduit {
 public:
  explicit Conduit(size_t jobs) : jobs_(jobs < 1 ? 1 : jobs) {
    for (size_t t = 1; t < jobs_; t++) pool_.emplace_back([this] { serve(); });
  }
  ~Conduit() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    wake_.notify_all();
    for (auto &t : pool_) t.join();
  }
  Conduit(const Conduit &) = delete;
  Conduit &operator=(const Conduit &) = delete;

  // Distributed: the collectives among the ranks (null for Sequential /
  // Concurrent); every rank runs the engine on its own GPU
  std::unique_ptr<Collective> dist;

  void evaluateBatch(size_t n, const std::function<void(size_t)> &body) {
    if (pool_.empty() || n <= 1) {
      for (size_t i = 0; i < n; i++) body(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      body_ = &body;
      n_ = n;
      next_.store(0);
      busy_ = pool_.size();
      err_ = nullptr;
      errAt_ = n;
      batch_++;
    }
    wake_.notify_all();
    work();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return busy_ == 0; });
    body_ = nullptr;
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void work() {
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= n_) return;
      try {
        (*body_)(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(m_);
        if (i < errAt_) {
          errAt_ = i;
          err_ = std::current_exception();
        }
        next_.store(n_);  // hand out nothing more; lower ids are already running
      }
    }
  }
  void serve() {
    size_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        wake_.wait(g, [&] { return stop_ || batch_ != seen; });
        if (stop_) return;
        seen = batch_;
      }
      work();
      std::lock_guard<std::mutex> g(m_);
      if (--busy_ == 0) done_.notify_all();
    }
  }
  size_t jobs_;
  std::vector<std::thread> pool_;
  std::mutex m_;
  std::condition_variable wake_, done_;
  const std::function<void(size_t)> *body_ = nullptr;
  size_t n_ = 0, busy_ = 0, errAt_ = 0, batch_ = 0;
  std::atomic<size_t> next_{0};
  std::exception_ptr err_;
  bool stop_ = false;
};

// Engine::initialize (engine.cpp:39) + Conduit module defaults
std::unique_ptr<Conduit> makeConduit(Json &js) {
  Json &c = js["Conduit"];
  const std::string t = canon(str(c, "Type", "Sequential"));
  if (t == "sequential") return std::unique_ptr<Conduit>(new Conduit(1));
  if (t == "concurrent") {
    const double jobs = num(c, "Concurrent Jobs", 1);  // concurrent.config default
    if (!(jobs >= 1) || jobs != std::floor(jobs))  // concurrent.cpp.base:23
      fail("You need to define at least 1 concurrent job(s) for external models \n");
    return std::unique_ptr<Conduit>(new Conduit((size_t)jobs));
  }
  if (t == "distributed") {
    // distributed.config: Ranks Per Worker (default 1).  The reference farms
    // samples to worker teams (distributed.cpp.base:31-71); here each rank is
    // one engine on one GPU and the solver shards its population / chains, so
    // a team is always one rank.
    const double rpw = num(c, "Ranks Per Worker", 1);
    if (rpw != 1)
      fail("The Distributed conduit runs one rank per GPU: 'Ranks Per Worker' must be 1 (is %g).", rpw);
    const std::string tr = canon(str(c, "Transport", "RCCL"));
    if (tr != "rccl" && tr != "host") fail("Conduit 'Transport' must be 'RCCL' or 'Host'.");
    const double port = num(c, "Bootstrap Port", 0);
    std::unique_ptr<Conduit> cd(new Conduit(1));
    try {
      cd->dist = makeCollective(tr, (int)port);
    } catch (const std::exception &e) {
      fail("%s", e.what());
    }
    return cd;
  }
  fail("Unrecognized conduit type '%s' (Sequential, Concurrent or Distributed).", c["Type"].getString().c_str());
}

struct VariableSpec {
  std::string name;
  double lb, ub, iv, istd, minstd, granularity = 0.0;
  int dist = -1;
};

}  // namespace

// Bayesian::evaluate on the host (bayesian.cpp.base:24-84) for solvers that
// see a Bayesian problem through F(x) = logPosterior (CMA-ES MAP estimation):
// the log-prior of each variable's Univariate/Uniform or Univariate/Normal
// prior (uniform.cpp.base / normal.cpp.base getLogDensity), then the
// likelihood only where the prior is finite: a Custom 'Likelihood Model', or a
// Reference 'Computational Model' + likelihood model (likelihood.cpp).
struct BayesianEvaluator {
  struct Prior {
    int kind;          // enum kg_prior_kind
    double a, b, aux;  // the distribution's two parameters and its log-density constant
  };
  std::vector<Prior> priors;
  bool reference = false;
  size_t fn = 0;
  std::vector<double> referenceData;
  std::string likelihoodModel;

  BayesianEvaluator(Json &js, const std::string &type) {
    Json &pb = js["Problem"];
    reference = type == "bayesian/reference";
    if (reference) {
      if (!pb.contains("Computational Model") || !pb["Computational Model"].is_integer())
        fail("Problem 'Bayesian/Reference' requires a 'Computational Model' function.");
      fn = pb["Computational Model"].getUInt();
      if (pb.contains("Reference Data") && pb["Reference Data"].is_array())
        for (const Json &x : pb["Reference Data"].elements()) referenceData.push_back(x.getDouble());
      likelihoodModel = str(pb, "Likelihood Model", "");
      if (referenceData.empty()) fail("Bayesian (%s) problems require defining reference data.\n", likelihoodModel.c_str());
      if (!isReferenceLikelihoodModel(likelihoodModel)) fail("Bayesian problem (%s) not recognized.\n", likelihoodModel.c_str());
    } else {
      if (!pb.contains("Likelihood Model") || !pb["Likelihood Model"].is_integer())
        fail("Problem 'Bayesian/Custom' requires a 'Likelihood Model' function.");
      fn = pb["Likelihood Model"].getUInt();
    }
    Json &ds = js["Distributions"];
    for (size_t i = 0; i < js["Variables"].size(); i++) {  // Bayesian::initialize :6-22
      Json &v = js["Variables"][i];
      const std::string pn = v.contains("Prior Distribution") ? v["Prior Distribution"].getString() : "";
      int k = -1;
      for (size_t d = 0; d < ds.size(); d++)
        if (ds[d].contains("Name") && ds[d]["Name"].getString() == pn) k = (int)d;
      if (k < 0) fail("Did not find distribution %s, specified by variable %s\n", pn.c_str(), str(v, "Name", "").c_str());
      const std::string t = canon(ds[k]["Type"].getString());
      Prior p{};
      if (t == "univariate/uniform") {
        p.a = mandatory(ds[k], "Minimum", "Distributions");
        p.b = mandatory(ds[k], "Maximum", "Distributions");
        p.aux = p.b - p.a <= 0.0 ? NAN : -std::log(p.b - p.a);
      } else if (t == "univariate/normal") {
        p.kind = KG_PRIOR_NORMAL;
        p.a = mandatory(ds[k], "Mean", "Distributions");
        p.b = mandatory(ds[k], "Standard Deviation", "Distributions");
        if (!(p.b > 0.0)) fail("Incorrect Standard Deviation parameter of Normal distribution: %f.\n", p.b);
        p.aux = -0.5 * std::log(2 * M_PI) - std::log(p.b);
      } else if (t == "univariate/exponential") {  // exponential.cpp.base
        p.kind = KG_PRIOR_EXPONENTIAL;
        p.a = mandatory(ds[k], "Location", "Distributions");
        p.b = mandatory(ds[k], "Mean", "Distributions");
        p.aux = -std::log(p.b);
      } else if (t == "univariate/laplace") {  // laplace.cpp.base
        p.kind = KG_PRIOR_LAPLACE;
        p.a = mandatory(ds[k], "Mean", "Distributions");
        p.b = mandatory(ds[k], "Width", "Distributions");
        if (p.b <= 0.0) fail("Incorrect Width parameter of Laplace distribution: %f.\n", p.b);
        p.aux = -std::log(2. * p.b);
      } else if (t == "univariate/cauchy") {  // cauchy.cpp.base
        p.kind = KG_PRIOR_CAUCHY;
        p.a = mandatory(ds[k], "Location", "Distributions");
        p.b = mandatory(ds[k], "Scale", "Distributions");
        if (p.b <= 0) fail("Incorrect Scale parameter of Cauchy distribution: %f.\n", p.b);
        p.aux = -std::log(p.b * M_PI);
      } else if (t == "univariate/lognormal") {  // logNormal.cpp.base
        p.kind = KG_PRIOR_LOGNORMAL;
        p.a = mandatory(ds[k], "Mu", "Distributions");
        p.b = mandatory(ds[k], "Sigma", "Distributions");
        if (p.b <= 0.0) fail("Incorrect Sigma parameter of LogNormal distribution: %f.\n", p.b);
        p.aux = -0.5 * std::log(2 * M_PI) - std::log(p.b);
      } else {
        fail("Bayesian problems on this path support 'Univariate/Uniform', 'Univariate/Normal', "
             "'Univariate/Exponential', 'Univariate/Laplace', 'Univariate/Cauchy' and 'Univariate/LogNormal' priors "
             "(distribution '%s').",
             pn.c_str());
      }
      priors.push_back(p);
    }
  }

  // evaluateLogPosterior (:56-77); F(x) = logP(x) = logPosterior (:79-84)
  void evaluate(Sample &s, const std::vector<double> &x, size_t id) {
    double logPrior = 0.0;
    for (size_t i = 0; i < x.size(); i++) {
      const Prior &p = priors[i];
      switch (p.kind) {  // the distributions' getLogDensity
        case KG_PRIOR_NORMAL: {
          const double d = (x[i] - p.a) / p.b;
          logPrior += p.aux - 0.5 * d * d;
          break;
        }
        case KG_PRIOR_EXPONENTIAL:
          logPrior += x[i] - p.a < 0 ? -INFINITY : p.aux - (x[i] - p.a) / p.b;
          break;
        case KG_PRIOR_LAPLACE: logPrior += p.aux - std::fabs(x[i] - p.a) / p.b; break;
        case KG_PRIOR_CAUCHY: logPrior += p.aux - std::log(1. + (x[i] - p.a) * (x[i] - p.a) / (p.b * p.b)); break;
        case KG_PRIOR_LOGNORMAL: {
          if (x[i] <= 0) {
            logPrior += -INFINITY;
            break;
          }
          const double lx = std::log(x[i]), d = (lx - p.a) / p.b;
          logPrior += p.aux - lx - 0.5 * d * d;
          break;
        }
        default: logPrior += (x[i] >= p.a && x[i] <= p.b) ? p.aux : -INFINITY;
      }
    }
    s["logPrior"] = logPrior;
    if (logPrior == -INFINITY) {
      s["logLikelihood"] = -INFINITY;
      s["logPosterior"] = -INFINITY;
    } else {
      getFunction(fn)(s);
      if (reference) s["logLikelihood"] = referenceLoglikelihood(likelihoodModel, referenceData, s);
      if (!s.contains("logLikelihood")) fail("The likelihood model did not assign 'logLikelihood' for sample %zu.", id);
      const double ll = s["logLikelihood"].getDouble();
      if (std::isnan(ll)) fail("Sample %zu returned NaN logLikelihood evaluation.\n", id);
      s["logPosterior"] = logPrior + ll;
    }
    s["F(x)"] = s["logPosterior"];
    s["logP(x)"] = s["logPosterior"];
  }
};

Json bayesianEvaluate(Json &experiment, const std::vector<double> &x) {
  const std::string pt = canon(str(experiment["Problem"], "Type", ""));
  if (pt != "bayesian/custom" && pt != "bayesian/reference") fail("Not a Bayesian problem ('%s').", pt.c_str());
  BayesianEvaluator b(experiment, pt);
  if (x.size() != b.priors.size()) fail("Expected %zu parameters, got %zu.", b.priors.size(), x.size());
  Sample s;
  s["Parameters"] = x;
  s["Sample Id"] = 0ULL;
  b.evaluate(s, x, 0);
  return s._js;
}

// ------------------------------------------------------------ modules
struct SolverModule {
  Conduit *conduit = nullptr;  // the engine's sample dispatch (host callbacks)
  virtual ~SolverModule() = default;
  virtual void runGeneration(size_t gen) = 0;
  // criteria evaluated before generation `gen` (experiment.cpp.base:56)
  virtual void checkTermination(size_t gen, std::vector<std::string> &met) = 0;
  virtual void getConfiguration(Json &solver) = 0;
  virtual void finalize(Json &js) = 0;
  virtual void printAfter(const Logger &log) = 0;
  virtual std::string type() const = 0;
  // beside each result file, in its directory (VRACER: the training state)
  virtual void saveFiles(const std::string &dir) { (void)dir; }
};

namespace {

std::vector<VariableSpec> readVariables(Json &js) {
  std::vector<VariableSpec> vs;
  if (!js.contains("Variables") || js["Variables"].size() == 0) fail("No variables have been defined.");
  for (size_t i = 0; i < js["Variables"].size(); i++) {
    Json &v = js["Variables"][i];
    VariableSpec s;
    s.name = str(v, "Name", "X" + std::to_string(i));
    s.lb = num(v, "Lower Bound", -INFINITY);
    s.ub = num(v, "Upper Bound", INFINITY);
    s.iv = num(v, "Initial Value", NAN);
    s.istd = num(v, "Initial Standard Deviation", NAN);
    s.minstd = num(v, "Minimum Standard Deviation Update", 0.0);
    s.granularity = num(v, "Granularity", 0.0);
    vs.push_back(s);
  }
  return vs;
}

Json matrixJson(const std::vector<double> &a, size_t rows, size_t cols) {
  std::vector<Json> m;
  m.reserve(rows);
  for (size_t r = 0; r < rows; r++) m.emplace_back(std::vector<double>(a.begin() + r * cols, a.begin() + (r + 1) * cols));
  Json j = Json::array();
  for (auto &x : m) j.push_back(std::move(x));
  return j;
}

std::vector<double> flatten(Json &j) {
  std::vector<double> v;
  for (const auto &x : j.elements()) {
    if (x.is_array())
      for (const auto &y : x.elements()) v.push_back(y.getDouble());
    else
      v.push_back(x.getDouble());
  }
  return v;
}

// ------------------------------------------------ unrecognised settings
// Every generated Module::setConfiguration erases the keys it consumes and
// fails on whatever is left (source_builders.py:164-170, e.g. the generated
// CMAES.cpp:1781): a misspelt key is an error, not a silently applied
// default.  The accepted names are the reference's .config keys of the
// module and its parents (Configuration Settings, Termination Criteria,
// Internal Settings) plus this build's extension keys and the state keys it
// writes into result files.
using KeyList = std::initializer_list<const char *>;
const KeyList SOLVER_KEYS = {"Type", "Variable Count", "Model Evaluation Count", "Termination Criteria"};
const KeyList SOLVER_TERMINATION = {"Max Model Evaluations", "Max Generations"};
const KeyList OPTIMIZER_KEYS = {"Current Best Value", "Previous Best Value", "Best Ever Value", "Best Ever Variables"};
const KeyList OPTIMIZER_TERMINATION = {"Max Value", "Min Value Difference Threshold"};
const KeyList CMAES_KEYS = {
    // Configuration Settings (CMAES.config)
    "Population Size", "Mu Value", "Mu Type", "Initial Sigma Cumulation Factor", "Initial Damp Factor",
    "Use Gradient Information", "Gradient Step Size", "Is Sigma Bounded", "Initial Cumulative Covariance",
    "Diagonal Covariance", "Mirrored Sampling", "Viability Population Size", "Viability Mu Value",
    "Max Covariance Matrix Corrections", "Target Success Rate", "Covariance Matrix Adaption Strength",
    "Normal Vector Learning Rate", "Global Success Learning Rate",
    // Internal Settings
    "Normal Generator", "Uniform Generator", "Is Viability Regime", "Value Vector", "Gradients",
    "Current Population Size", "Current Mu Value", "Mu Weights", "Effective Mu", "Sigma Cumulation Factor",
    "Damp Factor", "Cumulative Covariance", "Chi Square Number", "Covariance Eigenvalue Evaluation Frequency", "Sigma",
    "Trace", "Sample Population", "Finished Sample Count", "Current Best Variables", "Previous Best Ever Value",
    "Sorting Index", "Covariance Matrix", "Auxiliar Covariance Matrix", "Covariance Eigenvector Matrix",
    "Auxiliar Covariance Eigenvector Matrix", "Axis Lengths", "Auxiliar Axis Lengths", "BDZ Matrix",
    "Auxiliar BDZ Matrix", "Current Mean", "Previous Mean", "Mean Update", "Evolution Path",
    "Conjugate Evolution Path", "Conjugate Evolution Path L2 Norm", "Infeasible Sample Count",
    "Maximum Diagonal Covariance Matrix Element", "Minimum Diagonal Covariance Matrix Element",
    "Maximum Covariance Eigenvalue", "Minimum Covariance Eigenvalue", "Is Eigensystem Updated",
    "Viability Indicator", "Has Constraints", "Covariance Matrix Adaption Factor", "Best Valid Sample",
    "Global Success Rate", "Viability Function Value", "Resampled Parameter Count",
    "Covariance Matrix Adaptation Count", "Viability Boundaries", "Viability Improvement",
    "Max Constraint Violation Count", "Sample Constraint Violation Counts", "Constraint Evaluations",
    "Normal Constraint Approximation", "Best Constraint Evaluations", "Has Discrete Variables", "Discrete Mutations",
    "Number Of Discrete Mutations", "Number Masking Matrix Entries", "Masking Matrix", "Masking Matrix Sigma",
    "Chi Square Number Discrete Mutations", "Current Min Standard Deviation", "Current Max Standard Deviation",
    "Constraint Evaluation Count",
    // extension (include/korali_amd.h)
    "Covariance Update"};
const KeyList CMAES_TERMINATION = {"Max Infeasible Resamplings", "Max Condition Covariance Matrix",
                                   "Min Standard Deviation", "Max Standard Deviation"};
const KeyList TMCMC_KEYS = {
    // Configuration Settings (TMCMC.config)
    "Version", "Population Size", "Max Chain Length", "Burn In", "Per Generation Burn In",
    "Target Coefficient Of Variation", "Covariance Scaling", "Min Annealing Exponent Update",
    "Max Annealing Exponent Update", "Step Size", "Domain Extension Factor",
    // Internal Settings
    "Multinomial Generator", "Multivariate Generator", "Uniform Generator", "Current Burn In",
    "Chain Pending Evaluation", "Chain Pending Gradient", "Chain Candidates", "Chain Candidates LogLikelihoods",
    "Chain Candidates LogPriors", "Chain Candidates Gradients", "Chain Candidates Errors",
    "Chain Candidates Covariance", "Chain Leaders", "Chain Leaders LogLikelihoods", "Chain Leaders LogPriors",
    "Chain Leaders Gradients", "Chain Leaders Errors", "Chain Leaders Covariance", "Finished Chains Count",
    "Current Chain Step", "Chain Lengths", "Coefficient Of Variation", "Chain Count", "Annealing Exponent",
    "Previous Annealing Exponent", "Num Finite Prior Evaluations", "Num Finite Likelihood Evaluations",
    "Accepted Samples Count", "LogEvidence", "Proposals Acceptance Rate", "Selection Acceptance Rate",
    "Covariance Matrix", "Max Loglikelihood", "Mean Theta", "Sample Database", "Sample LogLikelihood Database",
    "Sample LogPrior Database", "Sample Gradient Database", "Sample Error Database", "Sample Covariances Database",
    "Upper Extended Boundaries", "Lower Extended Boundaries", "Num LU Decomposition Failures Proposal",
    "Num Eigen Decomposition Failures Proposal", "Num Inversion Failures Proposal", "Num Negative Definite Proposals",
    "Num Cholesky Decomposition Failures Proposal", "Num Covariance Corrections",
    // state this build writes
    "Database Entries", "Num Selections"};
const KeyList TMCMC_TERMINATION = {"Target Annealing Exponent"};
// problems (optimization.config, bayesian/*.config) + the extension kernels
const KeyList OPTIMIZATION_KEYS = {"Type", "Num Objectives", "Objective Function", "Constraints",
                                   "Has Discrete Variables", "Objective Kernel"};
const KeyList BAYESIAN_CUSTOM_KEYS = {"Type", "Likelihood Model", "Likelihood Kernel"};
const KeyList BAYESIAN_REFERENCE_KEYS = {"Type", "Computational Model", "Reference Data", "Likelihood Model"};

void rejectProblemUnrecognised(Json &pb, const std::string &canonType);

bool inList(const std::string &k, std::initializer_list<KeyList> lists) {
  for (const KeyList &l : lists)
    for (const char *a : l)
      if (k == a) return true;
  return false;
}

void rejectUnrecognised(Json &mod, const char *moduleName, std::initializer_list<KeyList> keys,
                        std::initializer_list<KeyList> termination) {
  Json left = Json::object();
  for (const auto &kv : mod.items()) {
    if (kv.first == "Termination Criteria" && kv.second.is_object() && termination.size()) {
      for (const auto &tv : kv.second.items())
        if (!inList(tv.first, termination)) left["Termination Criteria"][tv.first] = tv.second;
      continue;
    }
    if (!inList(kv.first, keys)) left[kv.first] = kv.second;
  }
  if (left.size()) fail(" + Unrecognized settings for Korali module: %s: \n%s\n", moduleName, left.dump(2).c_str());
}

void rejectProblemUnrecognised(Json &pb, const std::string &pt) {
  if (pt == "optimization") rejectUnrecognised(pb, "Optimization", {OPTIMIZATION_KEYS}, {});
  else if (pt == "bayesian/custom") rejectUnrecognised(pb, "Custom", {BAYESIAN_CUSTOM_KEYS}, {});
  else if (pt == "bayesian/reference") rejectUnrecognised(pb, "Reference", {BAYESIAN_REFERENCE_KEYS}, {});
}

// ------------------------------------------------------------- sharding
// The GPU of a Distributed rank: "Device" if given, else LOCAL_RANK modulo
// the visible devices (torch.distributed.run's one process per GPU).
int solverDevice(Json &js, const Collective *dist) {
  if (js.contains("Device")) return (int)js["Device"].getInt();
  if (!dist) return 0;
  int n = 0;
  check(kg_device_count(&n));
  const char *lr = getenv("LOCAL_RANK");
  const int l = (lr && *lr) ? atoi(lr) : dist->rank;
  return n > 0 ? l % n : 0;
}

// a named device buffer of a solver handle, as the collectives see it
template <class H>
SolverBuffer solverBuffer(H h, const char *name, int (*ptr)(H, const char *, void **), int (*stream)(H, void **),
                          int (*get)(H, const char *, double *, size_t),
                          int (*set)(H, const char *, const double *, size_t)) {
  SolverBuffer b;
  b.devicePtr = [=]() {
    void *p = nullptr;
    check(ptr(h, name, &p));
    return p;
  };
  b.stream = [=]() {
    void *q = nullptr;
    check(stream(h, &q));
    return q;
  };
  b.get = [=](void *out, size_t bytes) { check(get(h, name, (double *)out, bytes / sizeof(double))); };
  b.set = [=](void *in, size_t bytes) { check(set(h, name, (const double *)in, bytes / sizeof(double))); };
  return b;
}

// ------------------------------------------------------------- CMA-ES
// CMAES.cpp.base on the device (kg_cmaes_*); state names as in CMAES.config
const char *CMAES_VECTORS[] = {"Current Mean", "Previous Mean", "Covariance Matrix", "Covariance Eigenvector Matrix",
                               "Axis Lengths", "Evolution Path", "Conjugate Evolution Path", "Mu Weights",
                               "Value Vector", "Best Ever Variables", "Current Best Variables"};
const char *CMAES_SCALARS[] = {"Sigma", "Trace", "Effective Mu", "Cumulative Covariance", "Sigma Cumulation Factor",
                               "Damp Factor", "Chi Square Number", "Conjugate Evolution Path L2 Norm",
                               "Best Ever Value", "Previous Best Ever Value", "Previous Best Value",
                               "Current Best Value", "Current Min Standard Deviation",
                               "Current Max Standard Deviation", "Maximum Diagonal Covariance Matrix Element",
                               "Minimum Diagonal Covariance Matrix Element", "Minimum Covariance Eigenvalue",
                               "Maximum Covariance Eigenvalue", "Infeasible Sample Count", "Model Evaluation Count"};
// CCMA-ES state (CMAES.config Internal Settings; written and restored with constraints)
const char *CMAES_CONSTRAINT_VECTORS[] = {"Viability Boundaries", "Sample Constraint Violation Counts",
                                          "Best Constraint Evaluations", "Constraint Evaluations",
                                          "Viability Indicator", "Normal Constraint Approximation"};
const char *CMAES_CONSTRAINT_SCALARS[] = {"Global Success Rate", "Resampled Parameter Count",
                                          "Constraint Evaluation Count", "Covariance Matrix Adaptation Count",
                                          "Max Constraint Violation Count"};
// discrete variables (CMAES.config; written and restored when some variable has a Granularity)
const char *CMAES_DISCRETE_VECTORS[] = {"Masking Matrix", "Masking Matrix Sigma"};
const char *CMAES_DISCRETE_SCALARS[] = {"Number Of Discrete Mutations", "Number Masking Matrix Entries",
                                        "Chi Square Number Discrete Mutations"};

struct CmaesModule : SolverModule {
  kg_cmaes_t h = nullptr;
  size_t N = 0, lam = 0, mu = 0;
  int objective = -1;  // builtin kernel, or -1: host function
  size_t fn = 0;
  std::unique_ptr<BayesianEvaluator> bayesian;  // Bayesian problems: F(x) = logPosterior
  std::vector<VariableSpec> vars;
  double maxGenerations, maxModelEvaluations, maxInfeasible, maxCondition, minStd, maxStd, maxValue, minValueDiff;
  Json *solverJs = nullptr;
  bool updated = false;  // kg_cmaes_update ran on this handle (its termination record exists)
  bool hasDiscrete = false;   // some variable has a Granularity (CMAES.cpp.base:44-50)
  bool useGradients = false;  // "Use Gradient Information" (CMAES.cpp.base:82-87, :199, :226, :611-621)
  // Distributed conduit: this rank samples / evaluates rows [r0, r1) of the
  // population; the fitness all-gather and the partial-sum all-reduce run
  // between kg_cmaes_update_partial and _finalize (include/korali_amd.h)
  Collective *dist = nullptr;
  size_t r0 = 0, r1 = 0;
  bool exactShards = true;  // the sharded update's protocol (include/korali_amd.h): exact order or partial sums
  bool exchangeProfile = false;  // KORALI_AMD_EXCHANGE_PROFILE=1: time the exchange collectives
  // Distributed CCMA-ES: the device state runs replicated (unsharded handle on
  // every rank: the viability regime changes the population size and the
  // resampling walk is sequential), the callbacks are split over the ranks
  // and their values all-gathered (distributed.cpp.base:73-129's worker role)
  bool replicated = false;
  std::vector<size_t> constraintFns;  // CCMA-ES (function table indices)
  size_t curGen = 0;

  ~CmaesModule() override {
    if (h) kg_cmaes_destroy(h);
  }

  CmaesModule(Json &js, Seeder &seeds, bool resume, Collective *dist_) : dist(dist_) {
    Json &sv = js["Solver"];
    Json &pb = js["Problem"];
    solverJs = &sv;
    const std::string pt = canon(str(pb, "Type", ""));
    if (pt != "optimization" && pt != "bayesian/custom" && pt != "bayesian/reference")
      fail("Solver CMAES requires a problem of type 'Optimization', 'Bayesian/Custom' or 'Bayesian/Reference' (is '%s').",
           pb["Type"].getString().c_str());
    rejectUnrecognised(sv, "CMAES", {SOLVER_KEYS, OPTIMIZER_KEYS, CMAES_KEYS},
                       {SOLVER_TERMINATION, OPTIMIZER_TERMINATION, CMAES_TERMINATION});
    rejectProblemUnrecognised(pb, pt);
    vars = readVariables(js);
    N = vars.size();
    lam = uint(sv, "Population Size", 0);
    if (lam <= 1) fail("'Population Size' must be larger 1.");
    mu = uint(sv, "Mu Value", 0);
    const std::string muType = str(sv, "Mu Type", "Logarithmic");
    const std::string mt = canon(muType);
    const int muTypeId = mt == "logarithmic" ? KG_MU_LOGARITHMIC
                         : mt == "linear"    ? KG_MU_LINEAR
                         : mt == "equal"     ? KG_MU_EQUAL
                         : mt == "proportional" ? KG_MU_PROPORTIONAL
                                                : -1;
    if (muTypeId < 0)
      fail("Invalid setting of Mu Type (%s) (Linear, Equal, Logarithmic, or Proportional accepted).", muType.c_str());
    const bool mirrored = flag(sv, "Mirrored Sampling", false);
    if (mirrored && uint(sv, "Population Size", 0) % 2 == 1)  // CMAES.cpp.base:89-92
      fail("Mirrored Sampling can only be applied with an even Sample Population (is %zu)",
           (size_t)uint(sv, "Population Size", 0));
    useGradients = flag(sv, "Use Gradient Information", false);
    const double gradientStep = num(sv, "Gradient Step Size", 0.01);
    if (useGradients && gradientStep <= 0.)  // CMAES.cpp.base:86
      fail("Gradient Step Size must be larger than 0.0 (is %f)", gradientStep);
    if (useGradients && (pt != "optimization" || pb.contains("Objective Kernel")))
      fail("'Use Gradient Information' needs an Optimization problem with an 'Objective Function' that sets "
           "'Gradient'.");
    // CCMA-ES: Problem "Constraints" = functions evaluated per sample in list
    // order (optimization.cpp.base:11-24)
    if (pt == "optimization" && pb.contains("Constraints"))
      for (size_t c = 0; c < pb["Constraints"].size(); c++) constraintFns.push_back(pb["Constraints"][c].getUInt());
    replicated = dist && !constraintFns.empty();
    if (!constraintFns.empty() && mirrored) fail("Mirrored Sampling not applicable to problems with constraints");
    if (dist && !replicated) {
      if (lam % (size_t)dist->world)
        fail("The Distributed conduit splits the population evenly: 'Population Size' (%zu) must be a multiple of "
             "the number of ranks (%d).",
             lam, dist->world);
      r0 = lam / dist->world * dist->rank;
      r1 = r0 + lam / dist->world;
    } else {
      r1 = lam;
    }
    Json &tc = sv["Termination Criteria"];
    maxGenerations = num(tc, "Max Generations", 1e10);
    maxModelEvaluations = num(tc, "Max Model Evaluations", 1e9);
    maxInfeasible = num(tc, "Max Infeasible Resamplings", INFINITY);
    maxCondition = num(tc, "Max Condition Covariance Matrix", INFINITY);
    minStd = num(tc, "Min Standard Deviation", -INFINITY);
    maxStd = num(tc, "Max Standard Deviation", INFINITY);
    maxValue = num(tc, "Max Value", INFINITY);
    minValueDiff = num(tc, "Min Value Difference Threshold", -INFINITY);

    if (pt != "optimization") {
      bayesian.reset(new BayesianEvaluator(js, pt));
    } else if (pb.contains("Objective Kernel")) {
      const std::string k = canon(pb["Objective Kernel"].getString());
      objective = (k == "negativerosenbrock" || k == "rosenbrock")   ? KG_OBJ_NEGATIVE_ROSENBROCK
                  : (k == "negativeackley" || k == "ackley")         ? KG_OBJ_NEGATIVE_ACKLEY
                  : (k == "negativesphere" || k == "sphere")         ? KG_OBJ_NEGATIVE_SPHERE
                                                                     : -2;
      if (objective == -2) fail("Unknown 'Objective Kernel' '%s'.", pb["Objective Kernel"].getString().c_str());
    } else {
      if (!pb.contains("Objective Function")) fail("Problem 'Optimization' requires an 'Objective Function'.");
      fn = pb["Objective Function"].getUInt();
    }

    std::vector<double> lb(N), ub(N), iv(N), istd(N), minstd(N), gran(N);
    for (size_t i = 0; i < N; i++) {
      gran[i] = vars[i].granularity;
      if (gran[i] < 0.0) fail("Negative granularity for variable '%s'.\n", vars[i].name.c_str());  // CMAES.cpp.base:48
      if (gran[i] > 0.0) hasDiscrete = true;
      lb[i] = vars[i].lb;
      ub[i] = vars[i].ub;
      iv[i] = vars[i].iv;
      istd[i] = vars[i].istd;
      minstd[i] = vars[i].minstd;
    }
    // generators in CMAES.config Internal Settings order: Normal, Uniform
    Json &gn = sv["Normal Generator"], &gu = sv["Uniform Generator"];
    gn["Type"] = "Univariate/Normal";
    gn["Mean"] = 0.0;
    gn["Standard Deviation"] = 1.0;
    gu["Type"] = "Univariate/Uniform";
    gu["Minimum"] = 0.0;
    gu["Maximum"] = 1.0;
    kg_cmaes_cfg c{};
    c.variable_count = N;
    c.population_size = lam;
    c.mu_value = mu;
    c.mu_type = muTypeId;
    c.initial_sigma_cumulation_factor = num(sv, "Initial Sigma Cumulation Factor", -1.0);
    c.initial_damp_factor = num(sv, "Initial Damp Factor", -1.0);
    c.initial_cumulative_covariance = num(sv, "Initial Cumulative Covariance", -1.0);
    c.is_sigma_bounded = flag(sv, "Is Sigma Bounded", false);
    c.diagonal_covariance = flag(sv, "Diagonal Covariance", false);
    c.mirrored_sampling = mirrored ? 1 : 0;
    c.use_gradients = useGradients ? 1 : 0;
    c.gradient_step_size = gradientStep;
    c.max_infeasible_resamplings = maxInfeasible;
    c.lower_bound = lb.data();
    c.upper_bound = ub.data();
    c.initial_value = iv.data();
    c.initial_std = istd.data();
    c.min_std_update = minstd.data();
    c.granularity = gran.data();
    c.normal_seed = seeds.assign(gn);
    c.uniform_seed = seeds.assign(gu);
    // Exact (default, also under the Distributed conduit): the reference's
    // summation order; a sharded run all-gathers the selected rows and splits
    // the rank-mu chains by covariance entry, bit-identical to an unsharded
    // run.  MFMA: the matrix cores (sharded: per-rank partial sums)
    const std::string cu = canon(str(sv, "Covariance Update", "Exact"));
    if (cu != "exact" && cu != "mfma") fail("'Covariance Update' must be 'Exact' or 'MFMA'.");
    c.cov_mode = cu == "mfma" ? KG_COV_MFMA : KG_COV_EXACT;
    exactShards = c.cov_mode == KG_COV_EXACT;
    c.device = solverDevice(js, dist);
    c.shard_rank = dist && !replicated ? dist->rank : 0;
    c.shard_count = dist && !replicated ? dist->world : 0;
    c.store_bdz = 0;
    c.eigen_device_chase = 0;
    c.constraint_count = constraintFns.size();
    c.viability_population_size = uint(sv, "Viability Population Size", 2);
    c.viability_mu_value = uint(sv, "Viability Mu Value", 0);
    c.max_covariance_matrix_corrections = num(sv, "Max Covariance Matrix Corrections", 1000000);
    c.target_success_rate = num(sv, "Target Success Rate", 0.1818);
    c.covariance_matrix_adaption_strength = num(sv, "Covariance Matrix Adaption Strength", 0.1);
    c.global_success_learning_rate = num(sv, "Global Success Learning Rate", 0.2);
    check(kg_cmaes_create(&c, &h));
    {
      const char *ep = getenv("KORALI_AMD_EXCHANGE_PROFILE");
      exchangeProfile = ep && *ep == '1';
    }
    if (!constraintFns.empty()) check(kg_cmaes_set_constraints(h, &CmaesModule::constraintCallback, this));
    if (mu == 0) mu = lam / 2;
    unsigned char st[5000];
    if (seeds.range(gn, st)) check(kg_cmaes_set_rng(h, 0, st));
    if (seeds.range(gu, st)) check(kg_cmaes_set_rng(h, 1, st));
    if (resume) restore(sv);
  }

  // CMAES::setConfiguration of a saved state (loadState + resume)
  void restore(Json &sv) {
    check(kg_cmaes_initialize(h));  // derived constants; saved state overrides
    for (const char *k : CMAES_VECTORS)
      if (sv.contains(k) && sv[k].is_array() && sv[k].size()) {
        std::vector<double> v = flatten(sv[k]);
        size_t n = 0;
        check(kg_cmaes_field_size(h, k, &n));
        if (v.size() == n) check(kg_cmaes_set_field(h, k, v.data(), n));
      }
    for (const char *k : CMAES_SCALARS)
      if (sv.contains(k) && sv[k].is_number()) {
        const double v = sv[k].getDouble();
        check(kg_cmaes_set_field(h, k, &v, 1));
      }
    if (!constraintFns.empty()) {
      if (sv.contains("Is Viability Regime")) {
        const double v = sv["Is Viability Regime"].getBool() ? 1.0 : 0.0;
        check(kg_cmaes_set_field(h, "Is Viability Regime", &v, 1));
      }
      for (const char *k : CMAES_CONSTRAINT_VECTORS)
        if (sv.contains(k) && sv[k].is_array()) {
          std::vector<double> v = flatten(sv[k]);
          size_t n = 0;
          check(kg_cmaes_field_size(h, k, &n));
          if (v.size() == n) check(kg_cmaes_set_field(h, k, v.data(), n));
        }
      for (const char *k : CMAES_CONSTRAINT_SCALARS)
        if (sv.contains(k) && sv[k].is_number()) {
          const double v = sv[k].getDouble();
          check(kg_cmaes_set_field(h, k, &v, 1));
        }
      size_t cur = 0;
      check(kg_cmaes_population_size(h, &cur, nullptr));
      lam = cur;
      r1 = lam;
    }
    if (hasDiscrete) {
      for (const char *k : CMAES_DISCRETE_VECTORS)
        if (sv.contains(k) && sv[k].is_array() && sv[k].size() == N) {
          std::vector<double> v = flatten(sv[k]);
          check(kg_cmaes_set_field(h, k, v.data(), N));
        }
      for (const char *k : CMAES_DISCRETE_SCALARS)
        if (sv.contains(k) && sv[k].is_number()) {
          const double v = sv[k].getDouble();
          check(kg_cmaes_set_field(h, k, &v, 1));
        }
    }
  }

  // Optimization::evaluateConstraints for a batch of samples (the mean: id -1),
  // through the conduit (Sequential, or the Concurrent pool)
  static int constraintCallback(const double *X, size_t rows, size_t N_, const size_t *ids, double *out, void *ctx) {
    auto *self = (CmaesModule *)ctx;
    const size_t nc = self->constraintFns.size();
    try {
      if (self->dist) {  // replicated: this rank's block of rows, then the all-gather
        Collective &d = *self->dist;
        const size_t per = (rows + d.world - 1) / d.world, a = std::min(rows, per * d.rank),
                     b = std::min(rows, a + per);
        std::vector<double> buf((size_t)d.world * per * nc, 0.0);
        replicatedGather(d, buf, per * nc, [&] {
          for (size_t r = a; r < b; r++)
            self->evaluateConstraints(X + r * N_, N_, buf.data() + ((size_t)d.rank * per + (r - a)) * nc);
        });
        std::copy(buf.begin(), buf.begin() + rows * nc, out);
        return 0;
      }
      self->conduit->evaluateBatch(rows, [&](size_t r) { self->evaluateConstraints(X + r * N_, N_, out + r * nc); });
    } catch (...) {
      self->pendingError = std::current_exception();
      return 1;
    }
    (void)ids;
    return 0;
  }
  // Optimization::evaluateConstraints for one sample (optimization.cpp.base:11-24)
  void evaluateConstraints(const double *x, size_t N_, double *out) {
    Sample s;
    s["Module"] = "Problem";
    s["Operation"] = "Evaluate Constraints";
    s["Sample Id"] = (unsigned long long)0;  // (as CMAES.cpp.base:326, :357, :398)
    s["Current Generation"] = (unsigned long long)curGen;
    s["Parameters"] = std::vector<double>(x, x + N_);
    for (size_t c = 0; c < constraintFns.size(); c++) {
      getFunction(constraintFns[c])(s);
      if (!s.contains("F(x)")) fail("The constraint function %zu did not assign 'F(x)'.", c);
      const double v = s["F(x)"].getDouble();
      if (!std::isfinite(v)) fail("Non finite value of constraint evaluation %lu detected: %f\n", (unsigned long)c, v);
      out[c] = v;
    }
  }
  std::exception_ptr pendingError;

  void runGeneration(size_t gen) override {
    curGen = gen;
    if (gen == 1) check(kg_cmaes_initialize(h));
    if (!constraintFns.empty()) {
      if (kg_cmaes_prepare_constrained(h, gen) != 0) {
        if (pendingError) {
          std::exception_ptr e = pendingError;
          pendingError = nullptr;
          std::rethrow_exception(e);
        }
        check(1);
      }
      size_t cur = 0;
      check(kg_cmaes_population_size(h, &cur, nullptr));
      lam = cur;
      r1 = lam;
    } else {
      check(kg_cmaes_sample(h));
    }
    if (objective >= 0) {
      check(kg_cmaes_eval_builtin(h, objective));
    } else if (replicated) {
      splitEvaluate(gen);
    } else if (dist) {
      hostEvaluate(gen, r0, r1);
    } else {
      // KORALI_START every sample, KORALI_WAITALL (CMAES.cpp.base:204-224)
      std::vector<double> X(lam * N), F(lam), G(useGradients ? lam * N : 0);
      check(kg_cmaes_get_candidates(h, X.data(), N));
      Function *f = bayesian ? nullptr : &getFunction(fn);
      conduit->evaluateBatch(lam, [&](size_t i) { evaluateSample(gen, i, X, F, G, f); });
      check(bayesian ? kg_cmaes_set_log_posterior(h, F.data()) : kg_cmaes_set_fitness(h, F.data()));
      if (useGradients) check(kg_cmaes_set_gradients(h, G.data()));
    }
    if (dist && !replicated) {
      // the exchange steps of the sharded update; with
      // KORALI_AMD_EXCHANGE_PROFILE=1 each is bracketed by stream events
      // (device time of the collective, "Exchange Milliseconds" in the results)
      auto mark = [&](const char *stage, int phase) {
        if (exchangeProfile) check(kg_cmaes_profile_mark(h, stage, phase));
      };
      mark("exchange_fitness", 0);
      dist->allGather(buffer("Value Vector"), r1 - r0);
      if (useGradients) dist->allGather(buffer("Gradients"), (r1 - r0) * N);
      mark("exchange_fitness", 1);
      check(kg_cmaes_update_partial(h, gen));
      size_t n = 0;
      if (exactShards) {
        // the selected rows to every rank, then the covariance entries' owners
        check(kg_cmaes_shard_row_count(h, &n));
        mark("exchange_rows", 0);
        if (n) dist->allGather(buffer("Shard Rows"), n);
        mark("exchange_rows", 1);
        check(kg_cmaes_update_rows(h, gen));
        check(kg_cmaes_field_size(h, "Shard Covariance", &n));
        mark("exchange_covariance", 0);
        dist->allReduceMaxI64(buffer("Shard Covariance"), n);
        mark("exchange_covariance", 1);
      } else {
        check(kg_cmaes_field_size(h, "Shard Partials", &n));
        mark("exchange_partials", 0);
        dist->allReduceSum(buffer("Shard Partials"), n);
        mark("exchange_partials", 1);
      }
      check(kg_cmaes_update_finalize(h, gen));
      updated = true;
      return;
    }
    check(kg_cmaes_update(h, gen));
    updated = true;
    // enqueue the next generation's first half (generator prefetch, the
    // eigendecomposition's tridiagonalisation and unpack: workspace only)
    // before the termination check, so the device never idles while the
    // host decides; device-side errors surface in checkTermination
    check(kg_cmaes_begin_sample(h));
  }

  SolverBuffer buffer(const char *name) {
    return solverBuffer<kg_cmaes_t>(h, name, kg_cmaes_device_ptr, kg_cmaes_stream, kg_cmaes_get_field,
                                    kg_cmaes_set_field);
  }

  // a rank's share of the host-evaluated population (the Distributed
  // conduit's worker role, distributed.cpp.base:73-129): rows [a, b) through
  // the objective / log-posterior, the other rows' values arrive with the
  // all-gather
  void hostEvaluate(size_t gen, size_t a, size_t b) {
    std::vector<double> X(lam * N), F(lam, 0.0), G(useGradients ? lam * N : 0, 0.0);
    check(kg_cmaes_get_candidates(h, X.data(), N));
    Function *f = bayesian ? nullptr : &getFunction(fn);
    for (size_t i = a; i < b; i++) evaluateSample(gen, i, X, F, G, f);
    check(bayesian ? kg_cmaes_set_log_posterior(h, F.data()) : kg_cmaes_set_fitness(h, F.data()));
    if (useGradients) check(kg_cmaes_set_gradients(h, G.data()));
  }

  // replicated device state (Distributed CCMA-ES): this rank's block of the
  // population through the objective, the values (and gradients) all-gathered
  // over the bootstrap, every rank then sets the whole population's
  void splitEvaluate(size_t gen) {
    const size_t W = dist->world, per = (lam + W - 1) / W, a = std::min(lam, per * dist->rank),
                 b = std::min(lam, a + per), gw = useGradients ? N : 0;
    std::vector<double> X(lam * N), F(lam, 0.0), G(lam * gw, 0.0);
    check(kg_cmaes_get_candidates(h, X.data(), N));
    Function *f = bayesian ? nullptr : &getFunction(fn);
    std::vector<double> buf(W * per * (1 + gw), 0.0);
    replicatedGather(*dist, buf, per * (1 + gw), [&] {
      for (size_t i = a; i < b; i++) evaluateSample(gen, i, X, F, G, f);
      for (size_t i = a; i < b; i++) {
        double *row = buf.data() + (dist->rank * per + (i - a)) * (1 + gw);
        row[0] = F[i];
        std::copy(G.begin() + i * gw, G.begin() + (i + 1) * gw, row + 1);
      }
    });
    for (size_t i = 0; i < lam; i++) {
      const double *row = buf.data() + i * (1 + gw);
      F[i] = row[0];
      std::copy(row + 1, row + 1 + gw, G.begin() + i * gw);
    }
    check(bayesian ? kg_cmaes_set_log_posterior(h, F.data()) : kg_cmaes_set_fitness(h, F.data()));
    if (useGradients) check(kg_cmaes_set_gradients(h, G.data()));
  }

  // one sample through the objective / log-posterior (CMAES.cpp.base:204-224;
  // with gradients Optimization::evaluateWithGradients, optimization.cpp.base:47-63)
  void evaluateSample(size_t gen, size_t i, const std::vector<double> &X, std::vector<double> &F,
                      std::vector<double> &G, Function *f) {
    Sample s;
    s["Module"] = "Problem";
    s["Operation"] = useGradients ? "Evaluate With Gradients" : "Evaluate";
    s["Sample Id"] = (unsigned long long)i;
    s["Current Generation"] = (unsigned long long)gen;
    std::vector<double> x(X.begin() + i * N, X.begin() + (i + 1) * N);
    s["Parameters"] = x;
    if (bayesian) {  // Bayesian::evaluate: -Inf outside the prior's support is a valid F(x)
      bayesian->evaluate(s, x, i);
      F[i] = s["F(x)"].getDouble();
      return;
    }
    (*f)(s);
    if (!s.contains("F(x)")) fail("The objective function did not assign 'F(x)' for sample %zu.", i);
    F[i] = s["F(x)"].getDouble();
    if (useGradients) {
      const std::vector<double> g = KORALI_GET(std::vector<double>, s, "Gradient");
      if (g.size() != N)
        fail("Size of sample's gradient evaluations vector (%lu) is different from the number of problem "
             "variables defined (%lu).\n",
             (unsigned long)g.size(), (unsigned long)N);
      if (!std::isfinite(F[i])) fail("Non finite value of function evaluation detected: %f\n", F[i]);
      for (size_t d = 0; d < N; d++) {
        if (!std::isfinite(g[d]))
          fail("Non finite value of gradient evaluation detected for variable %lu: %f\n", (unsigned long)d, g[d]);
        G[i * N + d] = g[d];
      }
    }
    if (!std::isfinite(F[i])) fail("Non finite value of function evaluation detected: %f\n", F[i]);
  }

  double field(const char *k) {
    double v;
    check(kg_cmaes_get_field(h, k, &v, 1));
    return v;
  }

  void checkTermination(size_t gen, std::vector<std::string> &met) override {
    static const char *names[] = {"Model Evaluation Count",         "Infeasible Sample Count",
                                  "Maximum Covariance Eigenvalue",  "Minimum Covariance Eigenvalue",
                                  "Current Min Standard Deviation", "Current Max Standard Deviation",
                                  "Best Ever Value",                "Current Best Value",
                                  "Previous Best Value"};
    double v[KG_TERMINATION_FIELDS];
    if (updated)  // published by the device at the end of the update, no stream synchronisation
      check(kg_cmaes_wait_termination_fields(h, v));
    else
      check(kg_cmaes_get_fields(h, names, KG_TERMINATION_FIELDS, v));
    if (gen > maxGenerations) met.push_back("Max Generations");
    if (maxModelEvaluations <= v[0]) met.push_back("Max Model Evaluations");
    if (gen <= 1) return;
    if (maxInfeasible > 0 && v[1] >= maxInfeasible) met.push_back("Max Infeasible Resamplings");
    if (v[2] >= maxCondition * v[3]) met.push_back("Max Condition Covariance Matrix");
    if (v[4] <= minStd) met.push_back("Min Standard Deviation");
    if (v[5] >= maxStd) met.push_back("Max Standard Deviation");
    if (v[6] > maxValue) met.push_back("Max Value");
    if (std::fabs(v[7] - v[8]) < minValueDiff) met.push_back("Min Value Difference Threshold");
  }

  void getConfiguration(Json &sv) override {
    for (const char *k : CMAES_VECTORS) {
      size_t n = 0;
      check(kg_cmaes_field_size(h, k, &n));
      std::vector<double> v(n);
      check(kg_cmaes_get_field(h, k, v.data(), n));
      sv[k] = v;
    }
    {
      constexpr size_t ns = sizeof(CMAES_SCALARS) / sizeof(CMAES_SCALARS[0]);
      double v[ns];
      check(kg_cmaes_get_fields(h, CMAES_SCALARS, ns, v));
      for (size_t i = 0; i < ns; i++) sv[CMAES_SCALARS[i]] = v[i];
    }
    if (!constraintFns.empty()) {
      sv["Has Constraints"] = true;
      sv["Is Viability Regime"] = field("Is Viability Regime") != 0.0;
      sv["Current Population Size"] = (unsigned long long)field("Current Population Size");
      sv["Current Mu Value"] = (unsigned long long)field("Current Mu Value");
      sv["Covariance Matrix Adaption Factor"] = field("Covariance Matrix Adaption Factor");
      sv["Normal Vector Learning Rate"] = field("Normal Vector Learning Rate");
      for (const char *k : CMAES_CONSTRAINT_VECTORS) {
        size_t n = 0;
        check(kg_cmaes_field_size(h, k, &n));
        std::vector<double> v(n);
        check(kg_cmaes_get_field(h, k, v.data(), n));
        const size_t nc = constraintFns.size();
        if (!strcmp(k, "Constraint Evaluations") || !strcmp(k, "Normal Constraint Approximation"))
          sv[k] = matrixJson(v, nc, n / nc);
        else if (!strcmp(k, "Viability Indicator")) {
          Json m = Json::array();
          for (size_t c = 0; c < nc; c++) {
            Json row = Json::array();
            for (size_t i = 0; i < n / nc; i++) row.push_back(v[c * (n / nc) + i] != 0.0);
            m.push_back(row);
          }
          sv[k] = m;
        } else
          sv[k] = v;
      }
      for (const char *k : CMAES_CONSTRAINT_SCALARS) sv[k] = field(k);
    }
    if (hasDiscrete) {
      sv["Has Discrete Variables"] = true;
      for (const char *k : CMAES_DISCRETE_VECTORS) {
        std::vector<double> v(N);
        check(kg_cmaes_get_field(h, k, v.data(), N));
        sv[k] = v;
      }
      for (const char *k : CMAES_DISCRETE_SCALARS) sv[k] = field(k);
      // updateDiscreteMutationMatrix clears them every update (:859): zero in every result file
      sv["Discrete Mutations"] = std::vector<double>(lam * N, 0.0);
    }
    {
      std::vector<double> X(lam * N);
      check(kg_cmaes_get_field(h, "Sample Population", X.data(), X.size()));
      sv["Sample Population"] = matrixJson(X, lam, N);
      std::vector<uint64_t> idx(lam);
      check(kg_cmaes_get_sorting_index(h, idx.data()));
      Json si = Json::array();
      for (auto i : idx) si.push_back((unsigned long long)i);
      sv["Sorting Index"] = si;
    }
    sv["Variable Count"] = (unsigned long long)N;
    sv["Mu Value"] = (unsigned long long)mu;
    unsigned char st[5000];
    check(kg_cmaes_get_rng(h, 0, st));
    sv["Normal Generator"]["Range"] = hexState(st);
    check(kg_cmaes_get_rng(h, 1, st));
    sv["Uniform Generator"]["Range"] = hexState(st);
  }

  void finalize(Json &js) override {
    if (exchangeProfile) {
      for (const char *st : {"exchange_fitness", "exchange_rows", "exchange_covariance", "exchange_partials"}) {
        double ms = 0;
        size_t cnt = 0;
        check(kg_cmaes_profile_read(h, st, &ms, &cnt));
        if (cnt) js["Results"]["Exchange Milliseconds"][st] = ms / (double)cnt;
      }
    }
    // CMAES::finalize (CMAES.cpp.base:994-999)
    js["Results"]["Best Sample"]["F(x)"] = field("Best Ever Value");
    std::vector<double> b(N);
    check(kg_cmaes_get_field(h, "Best Ever Variables", b.data(), N));
    js["Results"]["Best Sample"]["Parameters"] = b;
  }

  void printAfter(const Logger &log) override {
    log.log(2, "Sigma:                        %+6.3e\n", field("Sigma"));
    log.log(2, "Current Function Value: Max = %+6.3e - Best = %+6.3e\n", field("Current Best Value"),
            field("Best Ever Value"));
    log.log(2, "Diagonal Covariance:    Min = %+6.3e -  Max = %+6.3e\n",
            field("Minimum Diagonal Covariance Matrix Element"), field("Maximum Diagonal Covariance Matrix Element"));
    log.log(2, "Covariance Eigenvalues: Min = %+6.3e -  Max = %+6.3e\n", field("Minimum Covariance Eigenvalue"),
            field("Maximum Covariance Eigenvalue"));
  }

  std::string type() const override { return "Optimizer/CMAES"; }
};

// --------------------------------------------------------------- TMCMC
const char *TMCMC_VECTORS[] = {"Chain Leaders LogLikelihoods", "Chain Leaders LogPriors", "Chain Lengths",
                               "Mean Theta", "Covariance Matrix", "Chain Candidates LogLikelihoods",
                               "Chain Candidates LogPriors", "Sample LogLikelihood Database",
                               "Sample LogPrior Database", "Num Selections"};
const char *TMCMC_MATRICES[] = {"Chain Leaders", "Chain Candidates", "Sample Database"};
// mTMCMC state (TMCMC.config names), flattened per chain
const char *MTMCMC_VECTORS[] = {"Chain Leaders Errors",       "Chain Candidates Errors",     "Sample Error Database",
                                "Chain Leaders Gradients",    "Chain Candidates Gradients",  "Sample Gradient Database",
                                "Chain Leaders Covariance",   "Chain Candidates Covariance", "Sample Covariances Database",
                                "Upper Extended Boundaries",  "Lower Extended Boundaries"};
const char *TMCMC_SCALARS[] = {"Annealing Exponent", "Previous Annealing Exponent", "LogEvidence",
                               "Coefficient Of Variation", "Max Loglikelihood", "Chain Count",
                               "Accepted Samples Count", "Proposals Acceptance Rate", "Selection Acceptance Rate",
                               "Database Entries", "Model Evaluation Count", "Current Burn In"};

struct TmcmcModule : SolverModule {
  kg_tmcmc_t h = nullptr;
  size_t N = 0, P = 0, ndist = 0;
  bool builtin = false, reference = false, mtmcmc = false;
  size_t fn = 0;
  std::vector<double> referenceData;  // Bayesian/Reference
  std::string likelihoodModel;
  double maxGenerations, maxModelEvaluations, targetExponent;
  // Distributed conduit: this rank advances its share of the chains; the
  // exchange is one MAX all-reduce between kg_tmcmc_process_partial and
  // _finalize (include/korali_amd.h)
  Collective *dist = nullptr;
  // Distributed mTMCMC: the handle runs replicated (the gradient / Fisher
  // proposals are per chain but the handle's proposal stage is unsharded),
  // each round's likelihood evaluations are split over the ranks and their
  // values, gradients and Fisher matrices all-gathered
  bool replicated = false;

  ~TmcmcModule() override {
    if (h) kg_tmcmc_destroy(h);
  }

  TmcmcModule(Json &js, Seeder &seeds, std::vector<uint64_t> &distSeeds,
              std::vector<std::vector<unsigned char>> &distStates, bool resume, Collective *dist_)
      : dist(dist_) {
    Json &sv = js["Solver"];
    Json &pb = js["Problem"];
    const std::string pt = canon(str(pb, "Type", ""));
    if (pt != "bayesian/custom" && pt != "bayesian/reference")
      fail("The device TMCMC path supports problems of type 'Bayesian/Custom' and 'Bayesian/Reference' (is '%s').",
           pb["Type"].getString().c_str());
    rejectUnrecognised(sv, "TMCMC", {SOLVER_KEYS, TMCMC_KEYS}, {SOLVER_TERMINATION, TMCMC_TERMINATION});
    rejectProblemUnrecognised(pb, pt);
    reference = pt == "bayesian/reference";
    const std::string version = canon(str(sv, "Version", "TMCMC"));
    if (version != "tmcmc" && version != "mtmcmc")
      fail("Unrecognized value (%s) provided for mandatory setting: ['Version'] required by TMCMC.\n",
           sv["Version"].getString().c_str());
    mtmcmc = version == "mtmcmc";
    replicated = mtmcmc && dist;
    // TMCMC.cpp.base:48-55
    if (mtmcmc && !reference) fail("mTMCMC works only for problems of type 'Bayesian/Reference'\n");
    std::vector<VariableSpec> vars = readVariables(js);
    N = vars.size();
    P = uint(sv, "Population Size", 0);
    if (P < 2) fail("TMCMC 'Population Size' must be at least 2.");
    const double mcl = num(sv, "Max Chain Length", 1);
    if (mcl == 0) fail("Max Chain Length must be greater 0.");  // TMCMC.cpp.base:32
    const double burnIn = num(sv, "Burn In", 0);
    std::vector<double> perGenBurnIn;
    if (sv.contains("Per Generation Burn In") && sv["Per Generation Burn In"].is_array())
      perGenBurnIn = flatten(sv["Per Generation Burn In"]);
    const double covScaling = num(sv, "Covariance Scaling", 0.04);
    if (covScaling <= 0.0) fail("Covariance Scaling must be larger 0.0 (is %lf).\n", covScaling);
    Json &tc = sv["Termination Criteria"];
    maxGenerations = num(tc, "Max Generations", 1e10);
    maxModelEvaluations = num(tc, "Max Model Evaluations", 1e9);
    targetExponent = num(tc, "Target Annealing Exponent", 1.0);

    // priors: each variable's Univariate/Uniform or Univariate/Normal
    // distribution (Bayesian::evaluateLogPrior, bayesian.cpp.base:24-32)
    Json &ds = js["Distributions"];
    ndist = ds.size();
    std::vector<double> pmin(N), pmax(N);
    std::vector<int> pdist(N), pkind(N, 0);
    for (size_t i = 0; i < N; i++) {
      Json &v = js["Variables"][i];
      if (!v.contains("Prior Distribution")) fail("Variable '%s' has no 'Prior Distribution'.", vars[i].name.c_str());
      const std::string pn = v["Prior Distribution"].getString();
      int k = -1;
      for (size_t d = 0; d < ndist; d++)
        if (ds[d].contains("Name") && ds[d]["Name"].getString() == pn) k = (int)d;
      if (k < 0) fail("Did not find a distribution named '%s'.", pn.c_str());
      const std::string dt = canon(ds[k]["Type"].getString());
      if (dt != "univariate/uniform" && mtmcmc)
        fail("Only 'Univariate/Uniform' priors allowed (is %s).\n", ds[k]["Type"].getString().c_str());
      if (dt == "univariate/uniform") {
        pmin[i] = mandatory(ds[k], "Minimum", "Distributions");
        pmax[i] = mandatory(ds[k], "Maximum", "Distributions");
      } else {
        // the two parameters of each supported distribution and its
        // updateDistribution check (exponential.cpp.base has none: a Mean <= 0
        // is accepted, its log-density is then NaN / infinite as the reference's)
        struct Kind {
          const char *type, *a, *b, *what;
          int kind;
        };
        static const Kind kinds[] = {
            {"univariate/normal", "Mean", "Standard Deviation", "Standard Deviation parameter of Normal", KG_PRIOR_NORMAL},
            {"univariate/exponential", "Location", "Mean", nullptr, KG_PRIOR_EXPONENTIAL},
            {"univariate/laplace", "Mean", "Width", "Width parameter of Laplace", KG_PRIOR_LAPLACE},
            {"univariate/cauchy", "Location", "Scale", "Scale parameter of Cauchy", KG_PRIOR_CAUCHY},
            {"univariate/lognormal", "Mu", "Sigma", "Sigma parameter of LogNormal", KG_PRIOR_LOGNORMAL}};
        const Kind *kd = nullptr;
        for (const Kind &q : kinds)
          if (dt == q.type) kd = &q;
        if (!kd)
          fail("The device TMCMC path supports 'Univariate/Uniform', 'Univariate/Normal', 'Univariate/Exponential', "
               "'Univariate/Laplace', 'Univariate/Cauchy' and 'Univariate/LogNormal' priors (distribution '%s').",
               pn.c_str());
        pkind[i] = kd->kind;
        pmin[i] = mandatory(ds[k], kd->a, "Distributions");
        pmax[i] = mandatory(ds[k], kd->b, "Distributions");
        if (kd->what && !(pmax[i] > 0.0)) fail("Incorrect %s distribution: %f.\n", kd->what, pmax[i]);
      }
      pdist[i] = k;
    }
    if (reference) {
      // Reference::initialize (reference.cpp.base:17-23) + the model checks
      // of evaluateLoglikelihood (:25-44)
      if (!pb.contains("Computational Model") || !pb["Computational Model"].is_integer())
        fail("Problem 'Bayesian/Reference' requires a 'Computational Model' function.");
      fn = pb["Computational Model"].getUInt();
      if (pb.contains("Reference Data") && pb["Reference Data"].is_array()) referenceData = flatten(pb["Reference Data"]);
      likelihoodModel = str(pb, "Likelihood Model", "");
      if (referenceData.empty())
        fail("Bayesian (%s) problems require defining reference data.\n", likelihoodModel.c_str());
      if (!isReferenceLikelihoodModel(likelihoodModel))
        fail("Bayesian problem (%s) not recognized.\n", likelihoodModel.c_str());
    } else if (pb.contains("Likelihood Kernel")) {
      if (canon(pb["Likelihood Kernel"].getString()) != "gaussian")
        fail("Unknown 'Likelihood Kernel' '%s'.", pb["Likelihood Kernel"].getString().c_str());
      builtin = true;
    } else {
      if (!pb.contains("Likelihood Model")) fail("Problem 'Bayesian/Custom' requires a 'Likelihood Model'.");
      fn = pb["Likelihood Model"].getUInt();
    }
    // generators in TMCMC.config order: Multinomial, Multivariate, Uniform
    Json &gm = sv["Multinomial Generator"], &gv = sv["Multivariate Generator"], &gu = sv["Uniform Generator"];
    gm["Type"] = "Specific/Multinomial";
    gv["Type"] = "Multivariate/Normal";
    gu["Type"] = "Univariate/Uniform";
    gu["Minimum"] = 0.0;
    gu["Maximum"] = 1.0;
    kg_tmcmc_cfg c{};
    c.variable_count = N;
    c.population_size = P;
    c.max_chain_length = mcl;
    c.default_burn_in = burnIn;
    c.per_generation_burn_in = perGenBurnIn.empty() ? nullptr : perGenBurnIn.data();
    c.per_generation_burn_in_count = perGenBurnIn.size();
    c.target_cov = num(sv, "Target Coefficient Of Variation", 1.0);
    c.covariance_scaling = covScaling;
    c.min_annealing_exponent_update = num(sv, "Min Annealing Exponent Update", 1e-5);
    c.max_annealing_exponent_update = num(sv, "Max Annealing Exponent Update", 1.0);
    c.prior_min = pmin.data();
    c.prior_max = pmax.data();
    c.prior_distribution = pdist.data();
    c.prior_kind = pkind.data();
    c.distribution_count = ndist;
    c.prior_seeds = distSeeds.data();
    c.multinomial_seed = seeds.assign(gm);
    c.multivariate_seed = seeds.assign(gv);
    c.uniform_seed = seeds.assign(gu);
    c.likelihood = KG_LIK_GAUSSIAN;
    c.device = solverDevice(js, dist);
    c.shard_rank = dist && !replicated ? dist->rank : 0;
    c.shard_count = dist && !replicated ? dist->world : 0;
    c.version = mtmcmc ? 1 : 0;
    c.step_size = num(sv, "Step Size", 0.1);
    c.domain_extension_factor = num(sv, "Domain Extension Factor", 0.2);
    if (mtmcmc) {
      if (mcl != 1) fail("Current version of 'mTMCMC' supports only 'Max Chain Length' of 1 (BASIS).");
      if (c.step_size < 0.0) fail("Step Size lower than 0.0 (is %lf)\n", c.step_size);
      if (c.domain_extension_factor < 0.0)
        fail("Domain Extension Factor lower than 0.0 (is %lf)\n", c.domain_extension_factor);
    }
    check(kg_tmcmc_create(&c, &h));
    unsigned char st[5000];
    if (seeds.range(gm, st)) check(kg_tmcmc_set_rng(h, 0, st));
    if (seeds.range(gv, st)) check(kg_tmcmc_set_rng(h, 1, st));
    if (seeds.range(gu, st)) check(kg_tmcmc_set_rng(h, 2, st));
    for (size_t d = 0; d < ndist; d++)
      if (!distStates[d].empty()) check(kg_tmcmc_set_rng(h, 3 + (int)d, distStates[d].data()));
    if (resume) restore(sv);
  }

  void restore(Json &sv) {
    for (const char *k : TMCMC_VECTORS)
      if (sv.contains(k) && sv[k].is_array() && sv[k].size()) {
        std::vector<double> v = flatten(sv[k]);
        size_t n = 0;
        check(kg_tmcmc_field_size(h, k, &n));
        if (v.size() == n) check(kg_tmcmc_set_field(h, k, v.data(), n));
      }
    for (const char *k : TMCMC_MATRICES)
      if (sv.contains(k) && sv[k].is_array() && sv[k].size()) {
        std::vector<double> v = flatten(sv[k]);
        size_t n = 0;
        check(kg_tmcmc_field_size(h, k, &n));
        if (v.size() == n) check(kg_tmcmc_set_field(h, k, v.data(), n));
      }
    for (const char *k : TMCMC_SCALARS)
      if (sv.contains(k) && sv[k].is_number()) {
        const double v = sv[k].getDouble();
        check(kg_tmcmc_set_field(h, k, &v, 1));
      }
    if (mtmcmc)
      for (const char *k : MTMCMC_VECTORS)
        if (sv.contains(k) && sv[k].is_array() && sv[k].size()) {
          std::vector<double> v = flatten(sv[k]);
          size_t n = 0;
          check(kg_tmcmc_field_size(h, k, &n));
          if (v.size() == n) check(kg_tmcmc_set_field(h, k, v.data(), n));
        }
  }

  double field(const char *k) {
    double v;
    check(kg_tmcmc_get_field(h, k, &v, 1));
    return v;
  }

  void runGeneration(size_t gen) override {
    check(kg_tmcmc_prepare(h, gen));
    if (builtin) {
      check(kg_tmcmc_evaluate(h));
    } else {
      // runGeneration's WAITANY loop :112-144: every round evaluates the
      // pending candidate of each unfinished chain (Bayesian::evaluate per
      // sample, the likelihood model only where the prior is finite,
      // bayesian.cpp.base:56-77), then advances every chain one step
      std::vector<double> X(P * N), LP(P), LL(P);
      std::vector<unsigned char> pend(P);
      // mTMCMC (generations > 1): calculateGradients / calculateProposals
      // :383-558 from each finite sample's "logLikelihood Gradient" and
      // "Fisher Information" (Reference::evaluate*, from the model outputs
      // the evaluation stored in the sample)
      const bool grads = mtmcmc && gen > 1;
      std::vector<double> G(grads ? P * N : 0), FIM(grads ? P * N * N : 0);
      Function &f = getFunction(fn);
      for (size_t pending = 1; pending;) {
        check(kg_tmcmc_evaluate_prior(h));
        check(kg_tmcmc_get_pending(h, pend.data()));
        check(kg_tmcmc_get_candidates(h, X.data(), N));
        check(kg_tmcmc_get_field(h, "Chain Candidates LogPriors", LP.data(), P));
        std::vector<size_t> todo;
        for (size_t i = 0; i < P; i++) {
          LL[i] = -INFINITY;
          if (pend[i] && !(std::isinf(LP[i]) && LP[i] < 0)) todo.push_back(i);
        }
        auto evaluate = [&](size_t k) {
          const size_t i = todo[k];
          Sample s;
          s["Module"] = "Problem";
          s["Operation"] = "Evaluate";
          s["Sample Id"] = (unsigned long long)i;
          s["Current Generation"] = (unsigned long long)gen;
          s["Parameters"] = std::vector<double>(X.begin() + i * N, X.begin() + (i + 1) * N);
          f(s);
          if (reference) {
            // Reference::evaluateLoglikelihood: sample.run(_computationalModel), then the model
            s["logLikelihood"] = referenceLoglikelihood(likelihoodModel, referenceData, s);
            if (std::isnan(s["logLikelihood"].getDouble())) fail("Sample %zu returned NaN logLikelihood evaluation.\n", i);
          }
          if (!s.contains("logLikelihood")) fail("The likelihood model did not assign 'logLikelihood' for sample %zu.", i);
          LL[i] = s["logLikelihood"].getDouble();
          if (std::isnan(LL[i])) fail("Non finite value of log-likelihood detected: %f\n", LL[i]);
          if (grads && std::isfinite(LL[i]) && std::isfinite(LP[i])) {
            const auto g = referenceLoglikelihoodGradient(likelihoodModel, referenceData, s, N);
            const auto F = referenceFisherInformation(likelihoodModel, referenceData, s, N);
            std::copy(g.begin(), g.end(), G.begin() + i * N);
            std::copy(F.begin(), F.end(), FIM.begin() + i * N * N);
          }
        };
        if (replicated) {
          // this rank's block of the round's evaluations; rows of (logLikelihood,
          // gradient, Fisher information) all-gathered over the bootstrap
          const size_t W = dist->world, per = (todo.size() + W - 1) / W,
                       a = std::min(todo.size(), per * dist->rank), b = std::min(todo.size(), a + per),
                       gw = grads ? N + N * N : 0;
          std::vector<double> buf(W * per * (1 + gw), 0.0);
          replicatedGather(*dist, buf, per * (1 + gw), [&] {
            for (size_t k = a; k < b; k++) evaluate(k);
            for (size_t k = a; k < b; k++) {
              const size_t i = todo[k];
              double *row = buf.data() + (dist->rank * per + (k - a)) * (1 + gw);
              row[0] = LL[i];
              if (grads) {
                std::copy(G.begin() + i * N, G.begin() + (i + 1) * N, row + 1);
                std::copy(FIM.begin() + i * N * N, FIM.begin() + (i + 1) * N * N, row + 1 + N);
              }
            }
          });
          for (size_t k = 0; k < todo.size(); k++) {
            const size_t i = todo[k];
            const double *row = buf.data() + k * (1 + gw);
            LL[i] = row[0];
            if (grads) {
              std::copy(row + 1, row + 1 + N, G.begin() + i * N);
              std::copy(row + 1 + N, row + 1 + N + N * N, FIM.begin() + i * N * N);
            }
          }
        } else {
          conduit->evaluateBatch(todo.size(), evaluate);
        }
        check(kg_tmcmc_set_evaluations(h, LP.data(), LL.data()));
        if (grads) check(kg_tmcmc_set_gradients(h, G.data(), FIM.data()));
        check(kg_tmcmc_advance(h, gen, &pending));
      }
    }
    if (dist && !replicated) {
      check(kg_tmcmc_process_partial(h, gen));
      size_t n = 0;
      check(kg_tmcmc_field_size(h, "Shard Exchange", &n));
      dist->allReduceMaxI64(solverBuffer<kg_tmcmc_t>(h, "Shard Exchange", kg_tmcmc_device_ptr, kg_tmcmc_stream,
                                                     kg_tmcmc_get_field, kg_tmcmc_set_field),
                            n);
      check(kg_tmcmc_process_finalize(h, gen));
    } else {
      check(kg_tmcmc_process(h, gen));
    }
    check(kg_tmcmc_synchronize(h));
  }

  void checkTermination(size_t gen, std::vector<std::string> &met) override {
    if (gen > maxGenerations) met.push_back("Max Generations");
    if (maxModelEvaluations <= field("Model Evaluation Count")) met.push_back("Max Model Evaluations");
    if (field("Previous Annealing Exponent") >= targetExponent) met.push_back("Target Annealing Exponent");
  }

  void getConfiguration(Json &sv) override {
    for (const char *k : TMCMC_VECTORS) {
      size_t n = 0;
      check(kg_tmcmc_field_size(h, k, &n));
      std::vector<double> v(n);
      check(kg_tmcmc_get_field(h, k, v.data(), n));
      sv[k] = v;
    }
    for (const char *k : TMCMC_MATRICES) {
      size_t n = 0;
      check(kg_tmcmc_field_size(h, k, &n));
      std::vector<double> v(n);
      check(kg_tmcmc_get_field(h, k, v.data(), n));
      sv[k] = matrixJson(v, n / N, N);
    }
    for (const char *k : TMCMC_SCALARS) sv[k] = field(k);
    if (mtmcmc) {
      for (const char *k : MTMCMC_VECTORS) {
        size_t n = 0;
        check(kg_tmcmc_field_size(h, k, &n));
        std::vector<double> v(n);
        check(kg_tmcmc_get_field(h, k, v.data(), n));
        sv[k] = v;
      }
      sv["Num Covariance Corrections"] = field("Num Covariance Corrections");
    }
    unsigned char st[5000];
    check(kg_tmcmc_get_rng(h, 0, st));
    sv["Multinomial Generator"]["Range"] = hexState(st);
    check(kg_tmcmc_get_rng(h, 1, st));
    sv["Multivariate Generator"]["Range"] = hexState(st);
    check(kg_tmcmc_get_rng(h, 2, st));
    sv["Uniform Generator"]["Range"] = hexState(st);
  }

  void saveDistributions(Json &js) {
    unsigned char st[5000];
    for (size_t d = 0; d < ndist; d++) {
      check(kg_tmcmc_get_rng(h, 3 + (int)d, st));
      js["Distributions"][d]["Range"] = hexState(st);
    }
  }

  void finalize(Json &js) override {
    // TMCMC::finalize: the last generation's sample database is the posterior
    size_t n = 0;
    check(kg_tmcmc_field_size(h, "Sample Database", &n));
    std::vector<double> v(n);
    check(kg_tmcmc_get_field(h, "Sample Database", v.data(), n));
    js["Results"]["Sample Database"] = matrixJson(v, n / N, N);  // TMCMC.cpp.base:791-795 (the only key it writes)
  }

  void printAfter(const Logger &log) override {
    log.log(2, "Acceptance Rate (proposals / selections): (%.2f%% / %.2f%%)\n",
            100 * field("Proposals Acceptance Rate"), 100 * field("Selection Acceptance Rate"));
    log.log(2, "Coefficient of Variation: %.2f%%\n", 100.0 * field("Coefficient Of Variation"));
    log.log(2, "Annealing Exponent:       %.3e\n", field("Annealing Exponent"));
  }

  std::string type() const override { return "Sampler/TMCMC"; }
};

bool dirExists(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

}  // namespace

struct ExperimentState {
  std::unique_ptr<SolverModule> solver;
  Logger log;
  // seconds from the start of the last run's loop until each generation's
  // termination check returned (generationCompletionTimes; kept out of the
  // experiment's JSON, whose keys the reference's setConfiguration checks)
  std::vector<double> marks;
};

std::vector<double> generationCompletionTimes(const Experiment &e) { return e._state->marks; }

Experiment::Experiment() : _state(new ExperimentState()) {}

std::vector<std::vector<float>> Experiment::getEvaluation(const std::vector<std::vector<std::vector<float>>> &) {
  // experiment.cpp.base:219-229: only a Learner solver evaluates input batches
  fail("This solver does not support evaluation operations.\n");
}
Experiment::~Experiment() = default;
Experiment::Experiment(Experiment &&) noexcept = default;
Experiment &Experiment::operator=(Experiment &&) noexcept = default;

bool Experiment::loadState(const std::string &path) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  _js = Json::parse(ss.str());
  return true;
}

namespace {

void makeDirs(const std::string &path) {
  for (size_t p = 1; p <= path.size(); p++)
    if (p == path.size() || path[p] == '/') {
      const std::string d = path.substr(0, p);
      if (!dirExists(d)) mkdir(d.c_str(), 0775);
    }
}

std::string resultPath(Json &js) {
  std::string path = js["File Output"]["Path"].getString();
  if (path.empty()) path = ".";
  if (path[0] != '/') path = "./" + path;  // experiment.cpp.base:136
  return path;
}

void saveState(Json &js, size_t gen) {
  Json &fo = js["File Output"];
  const std::string path = resultPath(js);
  makeDirs(path);
  char name[64];
  if (fo["Use Multiple Files"].getBool())
    snprintf(name, sizeof(name), "gen%08zu.json", gen);
  else
    snprintf(name, sizeof(name), "genLatest.json");
  const std::string file = path + "/" + name;
  {
    std::ofstream out(file);
    if (!out) fail("Error trying to save result file: %s.\n", file.c_str());
    out << js.dump(2);
  }
  const std::string link_ = path + "/latest";
  remove(link_.c_str());
  if (link(file.c_str(), link_.c_str()) != 0) {
    // hard links unsupported: fall back to a copy
    std::ifstream src(file);
    std::ofstream dst(link_);
    dst << src.rdbuf();
  }
}

// ------------------------------------------------------------- VRACER
// Agent / Continuous / VRACER (agent.cpp.base, continuous.cpp.base,
// VRACER.cpp.base) on the device (kg_vracer_*): the environment is the
// device CartPole of examples/learning/reinforcement/cartpole, selected by
// the extension key Problem/"Environment Kernel" (a host "Environment
// Function" cannot run inside the device rollouts and fails loudly).
const KeyList AGENT_KEYS = {
    // agent.config Configuration Settings
    "Mode", "Testing", "Training", "Concurrent Environments", "Episodes Per Generation", "Mini Batch",
    "Time Sequence Length", "Learning Rate", "L2 Regularization", "Neural Network", "Discount Factor",
    "Importance Weight Truncation Level", "Experience Replay", "Experiences Between Policy Updates",
    "State Rescaling", "Reward", "Multi Agent Relationship", "Multi Agent Correlation", "Multi Agent Sampling",
    // continuous.config / VRACER.config
    "Policy", "Normal Generator", "Statistics",
    // Internal Settings
    "Action Lower Bounds", "Action Upper Bounds", "Current Episode", "Current Learning Rate", "Policy Update Count",
    "Current Sample ID", "Uniform Generator", "Experience Count", "Experience Count Per Environment",
    "Agent Count", "Action Shifts", "Action Scales"};
const KeyList AGENT_TERMINATION = {"Max Episodes", "Max Experiences", "Max Policy Updates"};
const KeyList RL_KEYS = {"Type", "Environment Function", "Environment Kernel", "Environment Count",
                         "Actions Between Policy Updates", "Agents Per Environment", "Policies Per Environment",
                         "Testing Frequency", "Policy Testing Episodes", "Custom Settings", "Max Episode Steps",
                         "State Vector Size", "Action Vector Size", "State Vector Indexes", "Action Vector Indexes"};

}  // namespace

Json vracerPolicyDescription(Json &js) {
  Json &sv = js["Solver"];
  const std::string dist = canon(str(sv["Policy"], "Distribution", "Normal"));
  const bool normalFamily = dist == "normal" || dist == "squashednormal" || dist == "clippednormal" ||
                            dist == "truncatednormal";
  const bool bounded = dist == "squashednormal" || dist == "beta" || dist == "clippednormal" || dist == "truncatednormal";
  if (!normalFamily && dist != "beta") fail("Unknown policy distribution '%s'.", sv["Policy"]["Distribution"].getString().c_str());
  std::vector<unsigned long long> sIdx, aIdx;
  std::vector<float> noise, lbs, ubs;
  for (size_t i = 0; i < js["Variables"].size(); i++) {
    Json &v = js["Variables"][i];
    const std::string t = canon(str(v, "Type", "State"));
    if (t == "state") sIdx.push_back(i);
    else if (t == "action") {
      aIdx.push_back(i);
      noise.push_back((float)num(v, "Initial Exploration Noise", -1.0));
      lbs.push_back((float)num(v, "Lower Bound", -INFINITY));
      ubs.push_back((float)num(v, "Upper Bound", INFINITY));
    }
  }
  const size_t A = aIdx.size();
  std::vector<float> shifts(A, 0.0f), scales(A, 0.0f), scaling(2 * A), shifting(2 * A);
  std::vector<std::string> masks(2 * A);
  for (size_t i = 0; i < A; i++) {
    if (bounded) {
      if (!std::isfinite(lbs[i]) || !std::isfinite(ubs[i]))
        fail("Provided bounds (%f, %f) for action variable %zu are non-finite, but the distribution (%s) is bounded.\n",
             lbs[i], ubs[i], i, sv["Policy"]["Distribution"].getString().c_str());
      shifts[i] = (ubs[i] + lbs[i]) * 0.5f;
      scales[i] = (ubs[i] - lbs[i]) * 0.5f;
    }
    if (noise[i] <= 0.0f)
      fail("Provided initial noise (%f) for action variable %llu is not defined or negative.\n", noise[i], aIdx[i]);
    scaling[i] = 1.0f, shifting[i] = shifts[i], masks[i] = "Identity";
    scaling[A + i] = 2.0f * noise[i], shifting[A + i] = 0.0f, masks[A + i] = normalFamily ? "Softplus" : "Sigmoid";
  }
  Json out;
  out["Problem"]["State Vector Size"] = (unsigned long long)sIdx.size();
  out["Problem"]["Action Vector Size"] = (unsigned long long)A;
  out["Problem"]["State Vector Indexes"] = sIdx;
  out["Problem"]["Action Vector Indexes"] = aIdx;
  out["Solver"]["Action Shifts"] = shifts;
  out["Solver"]["Action Scales"] = scales;
  out["Solver"]["Policy"]["Parameter Count"] = (unsigned long long)(2 * A);
  out["Solver"]["Policy"]["Parameter Scaling"] = scaling;
  out["Solver"]["Policy"]["Parameter Shifting"] = shifting;
  out["Solver"]["Policy"]["Parameter Transformation Masks"] = masks;
  // network: state -> [Linear (H), Tanh] x L -> Linear (value + policy parameters)
  std::vector<unsigned long long> sizes{(unsigned long long)sIdx.size()};
  Json &hl = sv["Neural Network"]["Hidden Layers"];
  for (size_t l = 0; 2 * l < hl.size(); l++) sizes.push_back(uint(hl[2 * l], "Output Channels", 0));
  sizes.push_back(1 + 2 * A);
  unsigned long long count = 0;
  for (size_t l = 0; l + 1 < sizes.size(); l++) count += sizes[l] * sizes[l + 1] + sizes[l + 1];
  out["Layer Sizes"] = sizes;
  out["Hyperparameter Count"] = count;
  return out;
}

std::vector<float> vracerInitialHyperparameters(const std::vector<size_t> &sizes, unsigned seed) {
  size_t n = 0;
  for (size_t l = 0; l + 1 < sizes.size(); l++) n += sizes[l] * sizes[l + 1] + sizes[l + 1];
  std::vector<float> theta(n);
  std::mt19937 mt(seed);
  std::uniform_real_distribution<float> U(-1.0f, 1.0f);
  size_t k = 0;
  for (size_t l = 0; l + 1 < sizes.size(); l++) {
    const size_t ic = sizes[l], oc = sizes[l + 1];
    const float scale = l + 2 == sizes.size() ? 0.001f : 1.0f;
    const float xav = std::sqrt(6.0f) / std::sqrt((float)(oc + ic));
    for (size_t i = 0; i < ic * oc; i++) theta[k++] = scale * xav * U(mt);
    for (size_t i = 0; i < oc; i++) theta[k++] = 0.0f;
  }
  return theta;
}

namespace {

// A user 'Environment Function' run as a coroutine (the reference's
// co_create / co_switch, reinforcementLearning.cpp.base:66-88, :282-298,
// :332-336): the function runs on a thread of its own and control passes
// back and forth at every Sample::update and when the function returns, so
// exactly one side runs at a time.  Abandoning a running function (its
// episode ended with Termination set but the function did not return, or the
// engine is leaving) makes its pending update() throw, which unwinds it.
class EnvCoroutine {
 public:
  Sample s;

  ~EnvCoroutine() { stop(); }
  bool finished() const { return done_; }

  // starts fn(s) and runs it up to its first update() (or its end)
  void launch(size_t fn) {
    stop();
    done_ = false, abort_ = false, err_ = nullptr, envTurn_ = true;
    s._yield = [this] { yieldToEngine(); };
    th_ = std::thread([this, fn] {
      try {
        getFunction(fn)(s);
      } catch (...) {
        std::lock_guard<std::mutex> g(m_);
        if (!abort_) err_ = std::current_exception();
      }
      std::lock_guard<std::mutex> g(m_);
      done_ = true, envTurn_ = false;
      cv_.notify_all();
    });
    waitEngineTurn();
  }

  // runs the function from its pending update() to the next one (or its end)
  void resume() {
    if (done_) fail("Resuming a finished agent\n");
    {
      std::lock_guard<std::mutex> g(m_);
      envTurn_ = true;
    }
    cv_.notify_all();
    waitEngineTurn();
  }

  // abandons a function still running (its pending update() throws) and joins
  void stop() {
    if (!th_.joinable()) return;
    {
      std::lock_guard<std::mutex> g(m_);
      if (!done_) abort_ = true, envTurn_ = true;
    }
    cv_.notify_all();
    th_.join();
  }

 private:
  void yieldToEngine() {  // the function's thread, inside Sample::update
    std::unique_lock<std::mutex> g(m_);
    if (abort_) throw KoraliError("[Korali] Error: the environment's episode was abandoned by the engine.");
    envTurn_ = false;
    cv_.notify_all();
    cv_.wait(g, [this] { return envTurn_; });
    if (abort_) throw KoraliError("[Korali] Error: the environment's episode was abandoned by the engine.");
  }
  void waitEngineTurn() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return !envTurn_; });
    if (err_) {
      std::exception_ptr e = err_;
      err_ = nullptr;
      std::rethrow_exception(e);
    }
  }
  std::thread th_;
  std::mutex m_;
  std::condition_variable cv_;
  bool envTurn_ = false, done_ = true, abort_ = false;
  std::exception_ptr err_;
};

// ReinforcementLearning::runEnvironment's checks of what the function returned
// (reinforcementLearning.cpp.base:343-392, one agent per environment)
void readEnvState(Sample &s, size_t S, float *out) {
  if (!s.contains("State") || !s["State"].is_array())
    fail("Agent state variable returned by the environment is not a vector.\n");
  Json &st = s["State"];
  if (st.size() != S) fail("Agents state vector %lu returned with the wrong size: %lu, expected: %lu.\n", 0ul,
                           (unsigned long)st.size(), (unsigned long)S);
  for (size_t j = 0; j < S; j++) {
    const float v = (float)st[j].getDouble();
    if (!std::isfinite(v)) fail("Agent %lu state variable %lu returned an invalid value: %f\n", 0ul, (unsigned long)j, v);
    out[j] = v;
  }
}
float readEnvReward(Sample &s) {
  if (!s.contains("Reward") || !s["Reward"].is_number()) fail("Agent reward variable returned by the environment is not a number.\n");
  const float r = (float)s["Reward"].getDouble();
  if (!std::isfinite(r)) fail("Agent %lu reward returned an invalid value: %f\n", 0ul, r);
  return r;
}
// 0 Non Terminal, 1 Terminal, 2 Truncated (__environmentWrapper's checks,
// reinforcementLearning.cpp.base:77-83)
int readEnvTermination(EnvCoroutine &c) {
  const std::string t = c.s.contains("Termination") && c.s["Termination"].is_string() ? c.s["Termination"].getString() : "";
  if (t == "Non Terminal") {
    if (c.finished())
      fail("Environment function terminated, but agent termination status (success or truncated) was not set.\n");
    return 0;
  }
  if (t == "Terminal") return 1;
  if (t == "Truncated") return 2;
  fail("Environment function terminated, but agent termination status (%s) is neither 'Terminal' nor 'Truncated'.\n",
       t.c_str());
}

struct VracerModule : SolverModule {
  size_t envIds = 1;  // Problem / Environment Count
  kg_vracer_t h = nullptr;
  double maxGenerations = 1e10;
  unsigned long long maxEpisodes = 0, maxExperiences = 0, maxPolicyUpdates = 0, episodesPerGeneration = 1,
                     averageDepth = 100;
  unsigned long long sessionEpisodes = 0, sessionGeneration = 1;
  std::vector<float> rewardHistory;
  float lastReward = 0.f, bestReward = -INFINITY, averageReward = 0.f;
  Json *solverJs = nullptr;
  Json description;  // vracerPolicyDescription: written into every result file
  bool testing = false, tested = false;  // Mode = Testing
  bool rewardRescaled = false;           // Reward / Rescaling / Enabled
  bool serialize = true;                 // Experience Replay / Serialize: the training state beside the results
  std::vector<uint64_t> testingIds;
  std::vector<float> testingReward;
  size_t nState = 4, nAction = 1, concurrent = 1;
  // a host 'Environment Function' (without 'Environment Kernel'): one
  // coroutine per concurrent environment
  bool hostEnv = false, clipped = false;
  size_t envFn = 0;
  Json customSettings = Json::object();
  std::vector<double> actLbs, actUbs;
  std::vector<std::unique_ptr<EnvCoroutine>> envs;
  unsigned long long nextSampleId = 0, nextLaunchId = 0;  // agent.cpp.base:186; reinforcementLearning.cpp.base:71

  ~VracerModule() override {
    envs.clear();  // (the functions unwind before the agent goes)
    if (h) kg_vracer_destroy(h);
  }

  VracerModule(Json &js, Seeder &seeds, bool resume) {
    Json &sv = js["Solver"];
    Json &pb = js["Problem"];
    solverJs = &sv;
    const std::string pt = canon(str(pb, "Type", ""));
    if (pt != "reinforcementlearning/continuous")
      fail("Solver VRACER requires a problem of type 'Reinforcement Learning / Continuous' (is '%s').",
           pb["Type"].getString().c_str());
    rejectUnrecognised(sv, "VRACER", {SOLVER_KEYS, AGENT_KEYS}, {SOLVER_TERMINATION, AGENT_TERMINATION});
    rejectUnrecognised(pb, "Continuous", {RL_KEYS}, {});
    const std::string mode = canon(str(sv, "Mode", "Training"));
    if (mode != "training" && mode != "testing") fail("'Mode' must be 'Training' or 'Testing'.");
    testing = mode == "testing";
    // Testing runs one generation of the policy the experiment holds; a
    // resumed training run loads <result path>/state.bin (below)
    if (testing) {
      Json &tj = sv["Testing"];
      if (tj.contains("Sample Ids"))
        for (size_t i = 0; i < tj["Sample Ids"].size(); i++) testingIds.push_back(tj["Sample Ids"][i].getUInt());
      if (testingIds.empty())
        fail("For testing, you need to indicate the sample ids to run in the ['Testing']['Sample Ids'] field.\n");
    }
    // the environment: the device CartPole ('Environment Kernel'), else the
    // user's 'Environment Function' on the host
    if (pb.contains("Environment Kernel")) {
      if (canon(pb["Environment Kernel"].getString()) != "cartpole")
        fail("Unknown 'Environment Kernel' '%s' (the device provides \"CartPole\").",
             pb["Environment Kernel"].getString().c_str());
    } else if (pb.contains("Environment Function")) {
      hostEnv = true;
      envFn = (size_t)pb["Environment Function"].getUInt();
      if (pb.contains("Custom Settings")) customSettings = pb["Custom Settings"];
    } else {
      fail(" + No value provided for mandatory setting: ['Environment Function'] required by reinforcementLearning.\n");
    }
    if (uint(pb, "Agents Per Environment", 1) != 1) fail("'Agents Per Environment' > 1 is not supported by the device path.");
    const unsigned long long envCount = uint(pb, "Environment Count", 1);
    envIds = (size_t)envCount;
    uint(pb, "Actions Between Policy Updates", 0);  // the device policy is always the current one
    // the episode buffer: env.py's maxSteps for the CartPole kernel; a host
    // function ends its episodes itself, up to this many steps
    const unsigned long long maxSteps = uint(pb, "Max Episode Steps", hostEnv ? 10000 : 500);
    // variables (reinforcementLearning.cpp.base:40-53; continuous.cpp.base:44-50)
    nState = 0, nAction = 0;
    std::vector<double> noises;
    if (!js.contains("Variables") || js["Variables"].size() == 0) fail("No variables have been defined.");
    for (size_t i = 0; i < js["Variables"].size(); i++) {
      Json &v = js["Variables"][i];
      const std::string t = canon(str(v, "Type", "State"));
      if (t == "state") nState++;
      else if (t == "action") {
        nAction++;
        const double noise = num(v, "Initial Exploration Noise", -1.0);
        if (noise <= 0.0)
          fail("Provided initial noise (%f) for action variable %zu is not defined or negative.\n", noise, i);
        const double lb = num(v, "Lower Bound", -INFINITY), ub = num(v, "Upper Bound", INFINITY);
        if (ub - lb <= 0.0) fail("Upper (%f) and Lower Bound (%f) of action variable %zu invalid.\n", ub, lb, i);
        noises.push_back(noise), actLbs.push_back(lb), actUbs.push_back(ub);
      } else fail("Variable %zu: unknown Type '%s' (State or Action).", i, v["Type"].getString().c_str());
    }
    if (nAction == 0) fail("No action variables have been defined.\n");
    if (nState == 0) fail("No state variables have been defined.\n");
    if (!hostEnv && (nState != 4 || nAction != 1))
      fail("The CartPole environment kernel has 4 state variables and 1 action variable (%zu / %zu given).", nState,
           nAction);
    if (nAction > 4) fail("The device policy supports up to 4 action variables (%zu given).", nAction);
    const std::string dist = canon(str(sv["Policy"], "Distribution", "Normal"));
    if (dist != "normal" && dist != "clippednormal")
      fail("Policy Distribution '%s' is not supported by the device path (Normal, Clipped Normal).",
           sv["Policy"]["Distribution"].getString().c_str());
    clipped = dist == "clippednormal";
    if (clipped)  // continuous.cpp.base:20-26
      for (size_t i = 0; i < nAction; i++)
        if (!(std::isfinite(actLbs[i]) && std::isfinite(actUbs[i])))
          fail("Provided bounds (%f, %f) for action variable %zu are non-finite, but the distribution (%s) is bounded.\n",
               actLbs[i], actUbs[i], i, sv["Policy"]["Distribution"].getString().c_str());
    if (uint(sv, "Time Sequence Length", 1) != 1) fail("'Time Sequence Length' > 1 is not supported by the device path.");
    const bool stateRescaling = flag(sv["State Rescaling"], "Enabled", false);
    const bool rewardRescaling = flag(sv["Reward"]["Rescaling"], "Enabled", false);
    if (envCount < 1) fail("'Environment Count' must be at least 1 (%llu given).", envCount);
    rewardRescaled = rewardRescaling;
    if (flag(sv["Reward"]["Outbound Penalization"], "Enabled", false))
      fail("Reward Outbound Penalization is not supported by the device path.");
    Json &nn = sv["Neural Network"];
    if (canon(str(nn, "Optimizer", "Adam")) != "adam")
      fail("Neural Network Optimizer '%s' is not supported by the device path (Adam).", nn["Optimizer"].getString().c_str());
    str(nn, "Engine", "Korali");
    // hidden layers: [Layer/Linear (H), Layer/Activation (Elementwise/Tanh)] x L
    if (!nn.contains("Hidden Layers") || nn["Hidden Layers"].size() == 0 || nn["Hidden Layers"].size() % 2)
      fail("'Neural Network' / 'Hidden Layers' must be pairs of Layer/Linear and Layer/Activation (Elementwise/Tanh).");
    size_t H = 0, L = nn["Hidden Layers"].size() / 2;
    for (size_t l = 0; l < L; l++) {
      Json &lin = nn["Hidden Layers"][2 * l];
      Json &act = nn["Hidden Layers"][2 * l + 1];
      if (canon(str(lin, "Type", "")) != "layer/linear" || canon(str(act, "Type", "")) != "layer/activation" ||
          canon(str(act, "Function", "")) != "elementwise/tanh")
        fail("Hidden layer pair %zu must be Layer/Linear followed by Layer/Activation with Elementwise/Tanh.", l);
      const size_t oc = (size_t)uint(lin, "Output Channels", 0);
      if (l == 0) H = oc;
      if (oc != H || H == 0)  // widths that are not multiples of 64 run zero-padded (kg_vracer.hip)
        fail("Hidden layers must share one width on the device path (layer %zu: %zu).", l, oc);
    }
    Json &er = sv["Experience Replay"];
    Json &op = er["Off Policy"];
    kg_vracer_config c{};
    c.state_size = nState, c.action_size = nAction, c.hidden_size = H, c.hidden_layers = L;
    c.host_environment = hostEnv ? 1 : 0;
    c.environments = concurrent = (size_t)uint(sv, "Concurrent Environments", 1);
    c.environment_count = (size_t)envCount;
    c.mini_batch_size = (size_t)uint(sv["Mini Batch"], "Size", 256);
    str(sv["Mini Batch"], "Strategy", "Uniform");
    size_t maxSize = (size_t)uint(er, "Maximum Size", 0), startSize = (size_t)uint(er, "Start Size", 0);
    if (maxSize == 0) maxSize = (size_t)(std::pow(2, 14) * std::sqrt(4.0 + 1.0));  // agent.cpp.base:37-38
    if (startSize == 0) startSize = maxSize;
    er["Maximum Size"] = (unsigned long long)maxSize, er["Start Size"] = (unsigned long long)startSize;
    serialize = flag(er, "Serialize", true);
    c.replay_maximum_size = maxSize, c.replay_start_size = startSize;
    c.max_episode_steps = (size_t)maxSteps;
    c.experiences_between_policy_updates = mandatory(sv, "Experiences Between Policy Updates", "VRACER");
    c.discount_factor = num(sv, "Discount Factor", 0.995);
    c.learning_rate = mandatory(sv, "Learning Rate", "VRACER");
    c.importance_weight_truncation_level = num(sv, "Importance Weight Truncation Level", 1.0);
    c.off_policy_cutoff_scale = num(op, "Cutoff Scale", 4.0);
    c.off_policy_target = num(op, "Target", 0.1);
    c.off_policy_annealing_rate = num(op, "Annealing Rate", 0.0);
    c.off_policy_refer_beta = num(op, "REFER Beta", 0.3);
    c.l2_regularization_enabled = flag(sv["L2 Regularization"], "Enabled", false) ? 1 : 0;
    c.l2_regularization_importance = num(sv["L2 Regularization"], "Importance", 1e-4);
    c.initial_exploration_noise = noises.data();
    c.policy_distribution = clipped ? 1 : 0;
    c.reward_rescaling = rewardRescaling ? 1 : 0;
    c.state_rescaling = stateRescaling ? 1 : 0;
    c.action_lower_bounds = actLbs.data(), c.action_upper_bounds = actUbs.data();
    c.seed = seeds.counter++;
    c.device = 0;
    episodesPerGeneration = uint(sv, "Episodes Per Generation", 1);
    averageDepth = uint(sv["Training"], "Average Depth", 100);
    Json &tc = sv["Termination Criteria"];
    maxGenerations = num(tc, "Max Generations", 1e10);
    maxEpisodes = uint(tc, "Max Episodes", 0);
    maxExperiences = uint(tc, "Max Experiences", 0);
    maxPolicyUpdates = uint(tc, "Max Policy Updates", 0);
    check(kg_vracer_create(&c, &h));
    // initial hyperparameters (linear.cpp.base:28-49): Xavier-scaled U(-1, 1)
    // weights, zero biases, output layer Weight Scaling 0.001 (VRACER.cpp.base:38).
    // The uniform stream is this build's (std::mt19937 seeded from the
    // experiment's seed counter), not GSL's: initial weights are not pinned.
    size_t n = 0;
    check(kg_vracer_hyperparameter_count(h, &n));
    std::vector<size_t> sizes{nState};
    for (size_t l = 0; l < L; l++) sizes.push_back(H);
    sizes.push_back(1 + 2 * nAction);
    std::vector<float> theta = vracerInitialHyperparameters(sizes, (unsigned)seeds.counter++);
    if (theta.size() != n) fail("VRACER: hyperparameter count mismatch (%zu vs the device's %zu).", theta.size(), n);
    description = vracerPolicyDescription(js);
    if (sv["Training"].contains("Current Policy") && sv["Training"]["Current Policy"].contains("Policy") &&
        sv["Training"]["Current Policy"]["Policy"].size() == n) {
      auto v = flatten(sv["Training"]["Current Policy"]["Policy"]);
      for (size_t i = 0; i < n; i++) theta[i] = (float)v[i];
    }
    if (testing) {
      // agent.cpp.base:139-153: the Testing policy (Testing / Current Policy,
      // else the training policy), the sample ids, one generation
      Json &tj = sv["Testing"];
      if (tj.contains("Current Policy") && tj["Current Policy"].contains("Policy") &&
          tj["Current Policy"]["Policy"].size() == n) {
        auto v = flatten(tj["Current Policy"]["Policy"]);
        for (size_t i = 0; i < n; i++) theta[i] = (float)v[i];
      }
    }
    check(kg_vracer_set_field(h, "hyperparameters", theta.data(), n * sizeof(float)));
    if (resume && !testing) {
      // Agent::deserializeExperienceReplay (agent.cpp.base:903-976) + the
      // training statistics the result file holds
      const std::string file = resultPath(js) + "/state.bin";
      unsigned long long blob[3] = {0, 1, 0};
      size_t got = 0;
      check(kg_vracer_load_state(h, file.c_str(), blob, sizeof blob, &got));
      if (got >= 2 * sizeof(unsigned long long)) sessionEpisodes = blob[0], sessionGeneration = blob[1];
      // a host environment's episodes in flight are not part of the state:
      // its environments launch afresh (the reference's agents in flight are
      // lost with the run as well), with the sample ids continuing
      if (got == sizeof blob) nextSampleId = blob[2];
      Json &tr = sv["Training"];
      if (tr.contains("Reward History"))
        for (size_t i = 0; i < tr["Reward History"].size(); i++)
          rewardHistory.push_back((float)tr["Reward History"][i].getDouble());
      lastReward = (float)num(tr, "Last Reward", 0.0);
      bestReward = (float)num(tr, "Best Reward", -INFINITY);
      averageReward = (float)num(tr, "Average Reward", 0.0);
    }
    if (testing) {
      // the agent's rescaling state as the experiment holds it (the reference
      // restores it with the policy, agent.cpp.base:1266-1274, and hands the
      // state moments to every testing agent, :279-280)
      Json &sr = sv["State Rescaling"];
      const size_t S = std::min<size_t>(nState, 8);  // (the device keeps 8 moments)
      if (sr.contains("Means") && sr["Means"].size() == nState && sr.contains("Sigmas") && sr["Sigmas"].size() == nState) {
        std::vector<float> m(8, 0.f), s(8, 1.f);
        for (size_t i = 0; i < S; i++) m[i] = (float)sr["Means"][i].getDouble(), s[i] = (float)sr["Sigmas"][i].getDouble();
        check(kg_vracer_set_field(h, "state_rescaling_means", m.data(), S * sizeof(float)));
        check(kg_vracer_set_field(h, "state_rescaling_sigmas", s.data(), S * sizeof(float)));
      }
      Json &rr = sv["Reward"]["Rescaling"];
      if (rewardRescaled && rr.contains("Sigma") && rr["Sigma"].size() == envIds) {
        std::vector<float> sg(envIds, 1.0f);
        for (size_t i = 0; i < envIds; i++) sg[i] = (float)rr["Sigma"][i].getDouble();
        check(kg_vracer_set_field(h, "reward_rescaling_sigma", sg.data(), envIds * sizeof(float)));
      }
    }
  }

  double scalar(const char *name) {
    double v = 0.0;
    check(kg_vracer_get_scalar(h, name, &v));
    return v;
  }

  // Agent::trainingGeneration (agent.cpp.base:162-265), or testingGeneration
  // (:267-289): one deterministic episode per testing sample id, launch ids
  // in launch order (a fresh environment per run, reinforcementLearning.cpp.base:67)
  // initializeEnvironment + the first runEnvironment of runTrainingEpisode /
  // runTestingEpisode (reinforcementLearning.cpp.base:90-130, :211-225,
  // :261-293): a new episode of the function up to its first state
  void launchEnv(EnvCoroutine &c, unsigned long long sampleId, bool training, float *state, int *envId) {
    c.stop();
    c.s._js = Json::object();
    c.s["Module"] = "Problem";
    c.s["Operation"] = training ? "Run Training Episode" : "Run Testing Episode";
    c.s["Sample Id"] = sampleId;
    c.s["Launch Id"] = nextLaunchId++;
    c.s["Mode"] = training ? "Training" : "Testing";
    c.s["Custom Settings"] = customSettings;
    c.s["Reward"] = 0.0;
    c.s["Termination"] = "Non Terminal";
    c.s["Environment Id"] = 0ull;
    c.launch(envFn);
    readEnvState(c.s, nState, state);
    if (readEnvTermination(c) != 0)  // (no action taken: the reference would send an empty episode)
      fail("Environment function terminated before its first 'update()': an episode needs at least one action.\n");
    if (!c.s["Environment Id"].is_number()) fail("'Environment Id' returned by the environment is not a number.\n");
    const unsigned long long id = c.s["Environment Id"].getUInt();
    if (id >= envIds)  // reinforcementLearning.cpp.base:131-134
      fail("Environment Id provided (%lu) exceeds the maximum environment count defined (>= %lu).\n",
           (unsigned long)id, (unsigned long)envIds);
    if (envId) *envId = (int)id;
  }

  // the first launch of every concurrent environment (agent.cpp.base:178-190)
  void launchHostEnvs() {
    const size_t E = concurrent;
    envs.clear();
    std::vector<float> st(E * nState);
    std::vector<int> ids(E);
    for (size_t e = 0; e < E; e++) {
      envs.emplace_back(new EnvCoroutine());
      launchEnv(*envs[e], nextSampleId++, true, st.data() + e * nState, ids.data() + e);
    }
    check(kg_vracer_host_launch(h, st.data(), ids.data()));
  }

  // one action of every environment (the CartPole kernel's
  // kg_vracer_environment_step with the transitions from the functions):
  // the policy's actions, each function run to its next update() (or its
  // end), ended episodes relaunched in environment order, then the device's
  // episode bookkeeping and replay-memory appends
  void hostEnvironmentStep() {
    const size_t E = envs.size(), S = nState, A = nAction;
    std::vector<float> act(E * A), rew(E), st(E * S), next(E * S, 0.f);
    std::vector<int> term(E), nextId(E, 0);
    check(kg_vracer_host_act(h, act.data()));
    for (size_t e = 0; e < E; e++) {
      EnvCoroutine &c = *envs[e];
      c.s["Action"] = std::vector<float>(act.begin() + e * A, act.begin() + (e + 1) * A);
      c.resume();
      readEnvState(c.s, S, st.data() + e * S);
      rew[e] = readEnvReward(c.s);
      term[e] = readEnvTermination(c);
    }
    for (size_t e = 0; e < E; e++)
      if (term[e]) launchEnv(*envs[e], nextSampleId++, true, next.data() + e * S, nextId.data() + e);
    size_t added = 0;
    check(kg_vracer_host_feed(h, rew.data(), st.data(), term.data(), next.data(), nextId.data(), &added));
  }

  // runTestingEpisode (reinforcementLearning.cpp.base:211-259) per testing
  // sample: the policy's mode (generateTestingAction, continuous.cpp.base:
  // 219-260) on the state rescaled with the agent's moments (:365-376)
  void hostTestingEpisodes() {
    const size_t S = nState, A = nAction, O = 1 + 2 * A, SM = std::min<size_t>(S, 8);
    std::vector<float> mean(S, 0.f), sdev(S, 1.f), st(S), out(O);
    check(kg_vracer_get_field(h, "state_rescaling_means", mean.data(), SM * sizeof(float)));
    check(kg_vracer_get_field(h, "state_rescaling_sigmas", sdev.data(), SM * sizeof(float)));
    testingReward.assign(testingIds.size(), 0.f);
    nextLaunchId = 0;
    for (size_t j = 0; j < testingIds.size(); j++) {
      EnvCoroutine c;
      launchEnv(c, testingIds[j], false, st.data(), nullptr);
      float total = 0.f;
      for (;;) {
        for (size_t k = 0; k < S; k++) st[k] = (st[k] - mean[k]) / sdev[k];
        check(kg_vracer_run_policy(h, st.data(), 1, out.data()));
        std::vector<float> a(out.begin() + 1, out.begin() + 1 + A);
        if (clipped)
          for (size_t i = 0; i < A; i++) {
            if (a[i] >= (float)actUbs[i]) a[i] = (float)actUbs[i];
            if (a[i] <= (float)actLbs[i]) a[i] = (float)actLbs[i];
          }
        c.s["Action"] = a;
        c.resume();
        readEnvState(c.s, S, st.data());
        total += readEnvReward(c.s);
        if (readEnvTermination(c)) break;
      }
      testingReward[j] = total;
    }
  }

  void runGeneration(size_t) override {
    if (testing) {
      if (hostEnv) {
        hostTestingEpisodes();
        tested = true;
        return;
      }
      std::vector<uint64_t> lid(testingIds.size());
      for (size_t i = 0; i < lid.size(); i++) lid[i] = i;
      testingReward.assign(testingIds.size(), 0.f);
      check(kg_vracer_test_episodes(h, testingIds.data(), lid.data(), testingIds.size(), testingReward.data()));
      tested = true;
      return;
    }
    if (hostEnv && envs.empty()) launchHostEnvs();
    while (sessionEpisodes < episodesPerGeneration * sessionGeneration) {
      size_t added = 0, updates = 0;
      if (hostEnv) {
        hostEnvironmentStep();
        check(kg_vracer_train_pending(h, &updates));
      } else {
        check(kg_vracer_training_step(h, &added, &updates));
      }
      const size_t finished = (size_t)scalar("step_episodes");
      if (finished) {
        std::vector<float> r(finished);
        check(kg_vracer_get_field(h, "finished_rewards", r.data(), finished * sizeof(float)));
        for (float x : r) {
          rewardHistory.push_back(x);
          lastReward = x;
          bestReward = std::max(bestReward, x);
        }
        sessionEpisodes += finished;
      }
    }
    const size_t n = rewardHistory.size(), d = (size_t)std::min<unsigned long long>(averageDepth, n);
    averageReward = 0.f;
    for (size_t i = n - d; i < n; i++) averageReward += rewardHistory[i];
    if (d) averageReward /= (float)d;
    sessionGeneration++;
  }

  void checkTermination(size_t gen, std::vector<std::string> &met) override {
    if (testing) {  // Max Generations = the current generation + 1 (agent.cpp.base:141-142)
      if (tested) met.push_back("Max Generations");
      return;
    }
    if ((double)gen > maxGenerations) met.push_back("Max Generations");
    if (gen == 1) return;
    if (maxEpisodes > 0 && scalar("current_episode") >= (double)maxEpisodes) met.push_back("Max Episodes");
    if (maxExperiences > 0 && scalar("experience_count") >= (double)maxExperiences) met.push_back("Max Experiences");
    if (maxPolicyUpdates > 0 && scalar("policy_update_count") >= (double)maxPolicyUpdates)
      met.push_back("Max Policy Updates");
  }

  void getConfiguration(Json &sv) override {
    if (testing) {
      sv["Testing"]["Reward"] = std::vector<double>(testingReward.begin(), testingReward.end());
      return;
    }
    sv["Current Episode"] = (unsigned long long)scalar("current_episode");
    // the next launch's sample id (agent.cpp.base:186)
    sv["Current Sample ID"] = hostEnv ? nextSampleId : (unsigned long long)(scalar("current_sample_id") + (double)concurrent);
    sv["Experience Count"] = (unsigned long long)scalar("experience_count");
    sv["Policy Update Count"] = (unsigned long long)scalar("policy_update_count");
    sv["Current Learning Rate"] = scalar("learning_rate");
    sv["Experience Replay"]["Off Policy"]["Count"] = (unsigned long long)scalar("off_policy_count");
    sv["Experience Replay"]["Off Policy"]["Ratio"] = scalar("off_policy_ratio");
    sv["Experience Replay"]["Off Policy"]["Current Cutoff"] = scalar("off_policy_cutoff");
    sv["Experience Replay"]["Off Policy"]["REFER Beta"] = scalar("refer_beta");
    sv["Training"]["Reward History"] = std::vector<double>(rewardHistory.begin(), rewardHistory.end());
    sv["Training"]["Average Reward"] = (double)averageReward;
    sv["Training"]["Last Reward"] = (double)lastReward;
    sv["Training"]["Best Reward"] = (double)bestReward;
    size_t n = 0;
    check(kg_vracer_hyperparameter_count(h, &n));
    std::vector<float> theta(n);
    check(kg_vracer_get_field(h, "hyperparameters", theta.data(), n * sizeof(float)));
    sv["Training"]["Current Policy"]["Policy"] = std::vector<double>(theta.begin(), theta.end());
    {  // agent.config:311-320 (per environment id, Environment Count entries)
      if (rewardRescaled) {
        std::vector<float> sig(envIds), sum(envIds);
        check(kg_vracer_get_field(h, "reward_rescaling_sigma", sig.data(), envIds * sizeof(float)));
        check(kg_vracer_get_field(h, "reward_rescaling_sum", sum.data(), envIds * sizeof(float)));
        sv["Reward"]["Rescaling"]["Sigma"] = std::vector<double>(sig.begin(), sig.end());
        sv["Reward"]["Rescaling"]["Sum Squared Rewards"] = std::vector<double>(sum.begin(), sum.end());
      } else {
        // the sigmas stay 1 without rescaling (agent.cpp.base:97, :557-563);
        // the squared-reward sums only feed them, and the device keeps them
        // only when rescaling is enabled, so that key is left out
        sv["Reward"]["Rescaling"]["Sigma"] = std::vector<double>(envIds, 1.0);
      }
      // agent.config:326-335 (the device keeps the moments of up to 8 state
      // variables: State Rescaling needs S <= 8; without it they are 0 / 1)
      const size_t SM = std::min<size_t>(nState, 8);
      std::vector<float> sm(nState, 0.f), ss(nState, 1.f);
      check(kg_vracer_get_field(h, "state_rescaling_means", sm.data(), SM * sizeof(float)));
      check(kg_vracer_get_field(h, "state_rescaling_sigmas", ss.data(), SM * sizeof(float)));
      sv["State Rescaling"]["Means"] = std::vector<double>(sm.begin(), sm.end());
      sv["State Rescaling"]["Sigmas"] = std::vector<double>(ss.begin(), ss.end());
    }
    Json &ds = description["Solver"];
    sv["Action Shifts"] = ds["Action Shifts"];
    sv["Action Scales"] = ds["Action Scales"];
    for (const char *k : {"Parameter Count", "Parameter Scaling", "Parameter Shifting", "Parameter Transformation Masks"})
      sv["Policy"][k] = ds["Policy"][k];
  }

  void finalize(Json &) override {}

  // Agent::serializeExperienceReplay (agent.cpp.base:849-901) each time the
  // results are written (training runs with Experience Replay / Serialize)
  void saveFiles(const std::string &dir) override {
    if (testing || !serialize) return;
    const unsigned long long blob[3] = {sessionEpisodes, sessionGeneration, nextSampleId};
    check(kg_vracer_save_state(h, (dir + "/state.bin").c_str(), blob, sizeof blob));
  }

  void printAfter(const Logger &log) override {
    if (testing) {  // agent.cpp.base:1038-1045
      log.log(1, "Testing Results:\n");
      for (size_t i = 0; i < testingIds.size(); i++) {
        log.log(1, " + Sample %llu:\n", (unsigned long long)testingIds[i]);
        log.log(1, "   + (Average) Cumulative Reward            %f\n", testingReward[i]);
      }
      return;
    }
    log.log(2, "Experience Replay Statistics:\n");
    log.log(2, " + Experience Memory Size:      %.0f/%.0f\n", scalar("size"),
            (*solverJs)["Experience Replay"]["Maximum Size"].getDouble());
    log.log(2, " + Total Episodes Count:        %.0f\n", scalar("current_episode"));
    log.log(2, " + Total Experience Count:      %.0f\n", scalar("experience_count"));
    log.log(2, "Off-Policy Statistics:\n");
    log.log(2, " + Count (Ratio/Target):        %.0f (%.3f)\n", scalar("off_policy_count"), scalar("off_policy_ratio"));
    log.log(2, " + REFER Beta Factor:           %f\n", scalar("refer_beta"));
    log.log(2, "Training Statistics:\n");
    log.log(2, " + Policy Update Count:         %.0f\n", scalar("policy_update_count"));
    log.log(2, " + Latest Reward:               %f\n", lastReward);
    log.log(2, " + %zu-Episode Average Reward:  %f\n", (size_t)averageDepth, averageReward);
    log.log(2, " + Best Reward:                 %f\n", bestReward);
  }

  std::string type() const override { return "Agent/Continuous/VRACER"; }
};

// KORALI_AMD_RUN_PHASES=1: the wall time of each phase of a run on stderr
// (the engine's fixed cost outside the generation loop)
struct PhaseClock {
  bool on = getenv("KORALI_AMD_RUN_PHASES") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string text;
  void mark(const char *phase) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    char b[96];
    snprintf(b, sizeof(b), " %s=%.3fms", phase, std::chrono::duration<double, std::milli>(n - t).count());
    text += b;
    t = n;
  }
  ~PhaseClock() {
    if (on) fprintf(stderr, "[korali_amd run phases]%s\n", text.c_str());
  }
};

void runExperiment(Experiment &e, Conduit &conduit) {
  PhaseClock clk;
  Json &js = e._js;
  ExperimentState &st = *e._state;
  // experiment.config Module Defaults
  num(js, "Random Seed", 0);
  flag(js, "Preserve Random Number Generator States", false);
  Json &fo = js["File Output"];
  flag(fo, "Enabled", true);
  str(fo, "Path", "_korali_result");
  uint(fo, "Frequency", 1);
  flag(fo, "Use Multiple Files", true);
  Json &co = js["Console Output"];
  st.log.set(str(co, "Verbosity", "Normal"));
  // Distributed: every rank holds the same solver state; rank 0 alone
  // prints and writes result files (the reference's engine rank)
  const bool rootRank = !conduit.dist || conduit.dist->rank == 0;
  if (!rootRank) st.log.level = 0;
  const unsigned long long consoleFreq = uint(co, "Frequency", 1);
  flag(js, "Store Sample Information", false);
  if (!js.contains("Current Generation")) js["Current Generation"] = 0ULL;
  if (!js.contains("Distributions")) js["Distributions"] = Json::array();
  size_t gen = (size_t)js["Current Generation"].getUInt();
  const bool resume = gen > 0;
  if (resume && js.contains("Is Finished") && js["Is Finished"].getBool()) {
    // a finished experiment continues only if a termination limit was raised
  }
  js["Is Finished"] = false;
  // Experiment::setSeed: 0 -> time
  if (!resume && js["Random Seed"].getUInt() == 0)
    js["Random Seed"] = (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::high_resolution_clock::now().time_since_epoch())
                            .count();
  Seeder seeds{js["Random Seed"].getUInt(), js["Preserve Random Number Generator States"].getBool()};
  // distributions first (experiment.cpp:255-340), in order
  std::vector<uint64_t> distSeeds;
  std::vector<std::vector<unsigned char>> distStates;
  for (size_t d = 0; d < js["Distributions"].size(); d++) {
    Json &dj = js["Distributions"][d];
    distSeeds.push_back(seeds.assign(dj));
    std::vector<unsigned char> stt(5000);
    if (seeds.range(dj, stt.data()))
      distStates.push_back(stt);
    else
      distStates.emplace_back();
  }
  Json &sv = js["Solver"];
  if (!sv.contains("Type")) fail("No solver type specified ('Solver' / 'Type').");
  const std::string stype = canon(sv["Type"].getString());
  TmcmcModule *tm = nullptr;
  Collective *dist = conduit.dist.get();
  // the solver goes with the run, failed or not: its device handle, and a
  // host environment's coroutines, which must unwind while the caller (the
  // Python binding) has the GIL released
  struct SolverRelease {
    ExperimentState &st;
    ~SolverRelease() { st.solver.reset(); }
  } release{st};
  if (stype == "optimizer/cmaes" || stype == "cmaes") {
    st.solver.reset(new CmaesModule(js, seeds, resume, dist));
  } else if (stype == "sampler/tmcmc" || stype == "tmcmc") {
    tm = new TmcmcModule(js, seeds, distSeeds, distStates, resume, dist);
    st.solver.reset(tm);
  } else if (stype == "agent/continuous/vracer" || stype == "vracer") {
    // the device rollouts + update of one learner have no exchange step:
    // several GPUs run independent replicas
    if (dist)
      fail("Agent/Continuous/VRACER does not shard across ranks: run one experiment per GPU with the Sequential "
           "conduit (independent replicas).");
    st.solver.reset(new VracerModule(js, seeds, resume));
  } else {
    fail("Unrecognized solver type '%s' (the device path provides Optimizer/CMAES, Sampler/TMCMC and "
         "Agent/Continuous/VRACER).",
         sv["Type"].getString().c_str());
  }
  clk.mark("setup");
  js["Random Seed"] = seeds.counter;
  SolverModule &solver = *st.solver;
  solver.conduit = &conduit;
  const bool fileOut = fo["Enabled"].getBool() && rootRank;
  const size_t fileFreq = (size_t)fo["Frequency"].getUInt();
  auto save = [&]() {
    js["Current Generation"] = (unsigned long long)gen;
    solver.getConfiguration(sv);
    if (tm) tm->saveDistributions(js);
    saveState(js, gen);
    solver.saveFiles(resultPath(js));
  };
  const auto t0 = std::chrono::steady_clock::now();
  if (gen == 0 && fileOut) save();
  clk.mark("save0");
  gen++;
  std::vector<std::string> met;
  // marks[i]: seconds from the start of the loop until generation i (1-based
  // from the first generation of this run) had completed, i.e. until its
  // termination check returned; marks[0] is the loop's first check
  std::vector<double> marks;
  for (;;) {
    met.clear();
    solver.checkTermination(gen, met);
    marks.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    if (!met.empty()) break;
    if (consoleFreq > 0 && gen % consoleFreq == 0) {
      st.log.log(1, "--------------------------------------------------------------------\n");
      st.log.log(1, "Current Generation: #%zu\n", gen);
    }
    const auto g0 = std::chrono::steady_clock::now();
    solver.runGeneration(gen);
    // (a peer's failure aborts this rank's collectives: their results are void)
    if (conduit.dist && conduit.dist->failed()) fail("Another rank of the Distributed conduit failed.");
    const auto g1 = std::chrono::steady_clock::now();
    if (consoleFreq > 0 && gen % consoleFreq == 0) {
      // printAfter reads solver state from the device: only when it prints
      if (st.log.level >= 2) solver.printAfter(st.log);
      st.log.log(3, "Experiment: 0 - Generation Time: %.3fs\n", std::chrono::duration<double>(g1 - g0).count());
    }
    if (fileOut && fileFreq > 0 && gen % fileFreq == 0) save();
    gen++;
  }
  const auto t1 = std::chrono::steady_clock::now();
  clk.mark("loop");
  gen--;
  js["Is Finished"] = true;
  solver.finalize(js);
  js["Current Generation"] = (unsigned long long)gen;
  st.marks = marks;
  solver.getConfiguration(sv);
  clk.mark("state");
  if (tm) tm->saveDistributions(js);
  if (fileOut) {
    saveState(js, gen);
    solver.saveFiles(resultPath(js));
  }
  if (conduit.dist) conduit.dist->barrier();  // no rank leaves before the others finished
  clk.mark("files");
  st.log.log(1, "--------------------------------------------------------------------\n");
  st.log.log(1, "%s finished correctly.\n", solver.type().c_str());
  for (const auto &m : met) st.log.log(2, "Termination Criterion Met: %s\n", m.c_str());
  st.log.log(2, "Final Generation: %zu\n", gen);
  st.log.log(2, "Elapsed Time: %.3fs\n", std::chrono::duration<double>(t1 - t0).count());
  st.solver.reset();  // release the device handle
  clk.mark("release");
}

}  // namespace

// Engine::run (engine.cpp:69-128): the conduit lives for the whole run
void Engine::run(Experiment &e) {
  std::unique_ptr<Conduit> c = makeConduit(_js);
  runExperiment(e, *c);
}

void Engine::run(std::vector<Experiment> &es) {
  std::unique_ptr<Conduit> c = makeConduit(_js);
  for (auto &e : es) runExperiment(e, *c);
}

void Engine::run(const std::vector<Experiment *> &es) {
  std::unique_ptr<Conduit> c = makeConduit(_js);
  for (auto *e : es) runExperiment(*e, *c);
}

void conduitEvaluate(size_t jobs, size_t n, const std::function<void(size_t)> &body) {
  Conduit c(jobs);
  c.evaluateBatch(n, body);
}

}  // namespace korali
