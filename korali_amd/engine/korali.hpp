// korali.hpp — the korali::Engine / korali::Experiment / korali::Sample API
// (reference: source/korali.hpp:25-31, source/engine.hpp, source/modules/
// experiment/experiment.hpp.base, source/sample/sample.hpp:25-191) on top of
// the korali_amd C-ABI.  Existing problem definitions compile unchanged:
//
//   #include <korali.hpp>
//   void model(korali::Sample &s) { auto x = KORALI_GET(std::vector<double>, s, "Parameters"); s["F(x)"] = ...; }
//   void direct(korali::Sample &k) { float x = k["Parameters"][0]; k["F(x)"] = -0.5 * x * x; }
//   korali::Engine k; korali::Experiment e;
//   e["Problem"]["Type"] = "Optimization";
//   e["Problem"]["Objective Function"] = &model;
//   e["Solver"]["Type"] = "Optimizer/CMAES"; ...
//   k.run(e);
//
// Solvers on this path: "Optimizer/CMAES" and "Sampler/TMCMC" (Version
// "TMCMC").  Problems: "Optimization" and "Bayesian/Custom".  Extension keys
// (optional, no existing key changes meaning):
//   Problem / "Objective Kernel":  "Negative Rosenbrock" | "Negative Ackley" |
//                                  "Negative Sphere"  (batched on the device)
//   Problem / "Likelihood Kernel": "Gaussian"         (-0.5 |x|^2, on the device)
//   Solver  / "Covariance Update": "Exact" (default) | "MFMA"
//   "Device": HIP device ordinal of the experiment
#pragma once

#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "json.hpp"

namespace korali {

// thrown for every configuration or runtime error (KORALI_LOG_ERROR)
class KoraliError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// KORALI_GET(TYPE, SAMPLE, KEY, ...): typed read of a (nested) sample entry,
// failing with the reference's messages (sample.hpp:25-26, :115-131)
#define KORALI_GET(TYPE, SAMPLE, ...) (SAMPLE).template get<TYPE>(__FILE__, __LINE__, __VA_ARGS__)

class Sample {
 public:
  Json &operator[](const std::string &key) { return _js[key]; }
  Json &operator[](size_t key) { return _js[key]; }
  bool contains(const std::string &key) const { return _js.contains(key); }
  // Sample::update (sample.cpp:31-34) hands control back to the engine.  A
  // reinforcement-learning environment function runs as a coroutine
  // (reinforcementLearning.cpp.base:58-83): there update() returns once the
  // engine has set the next "Action".  CMA-ES and TMCMC samples run to
  // completion on the evaluating thread: no handler, a no-op.
  void update() {
    if (_yield) _yield();
  }
  std::function<void()> _yield;  // set by the engine for coroutine samples

  template <typename T, typename... Key>
  T get(const char *fileName, int lineNumber, const Key &...key) {
    const Json *j = &_js;
    std::string path;
    if (!walk(j, path, key...))
      fail(fileName, lineNumber, "Requesting non existing value " + path + " from sample.\n");
    try {
      return j->template get<T>();
    } catch (const std::exception &e) {
      fail(fileName, lineNumber,
           "Missing or incorrect value " + path + " for the sample.\n + Cause: " + std::string(e.what()) + "\n");
    }
  }

  Json _js;

 private:
  static bool step(const Json *&j, std::string &path, const std::string &k) {
    path += "[\"" + k + "\"]";
    if (!j->contains(k)) return false;
    j = &j->at(k);
    return true;
  }
  static bool step(const Json *&j, std::string &path, const char *k) { return step(j, path, std::string(k)); }
  template <typename I, typename = typename std::enable_if<std::is_integral<I>::value>::type>
  static bool step(const Json *&j, std::string &path, I idx) {
    path += "[" + std::to_string((long long)idx) + "]";
    if (!j->is_array() || (size_t)idx >= j->size()) return false;
    j = &j->at((size_t)idx);
    return true;
  }
  static bool walk(const Json *&, std::string &) { return true; }
  template <typename K, typename... Rest>
  static bool walk(const Json *&j, std::string &path, const K &k, const Rest &...rest) {
    return step(j, path, k) && walk(j, path, rest...);
  }
  [[noreturn]] static void fail(const char *fileName, int lineNumber, const std::string &msg) {
    // Logger::logError (logger.cpp:83-99): message + " + From file:line\n"
    throw KoraliError(msg + " + From " + fileName + ":" + std::to_string(lineNumber) + "\n");
  }
};

struct ExperimentState;  // solver module + bookkeeping (engine.cpp)

class Experiment {
 public:
  Experiment();
  ~Experiment();
  Experiment(const Experiment &) = delete;
  Experiment &operator=(const Experiment &) = delete;
  Experiment(Experiment &&) noexcept;
  Experiment &operator=(Experiment &&) noexcept;

  Json &operator[](const std::string &key) { return _js[key]; }
  // Experiment::loadState (experiment.cpp.base:150-153): the full JSON of a
  // result file; a following run() resumes from it bit for bit.
  bool loadState(const std::string &path);
  // Experiment::getEvaluation (experiment.cpp.base:219-229): only learner
  // solvers evaluate batches; CMA-ES and TMCMC raise the reference's error
  std::vector<std::vector<float>> getEvaluation(const std::vector<std::vector<std::vector<float>>> &inputBatch);

  Json _js;
  std::unique_ptr<ExperimentState> _state;
};

// Engine (source/engine.hpp): its own JSON holds the conduit,
//   k["Conduit"]["Type"] = "Sequential" (default) | "Concurrent" | "Distributed";
//   k["Conduit"]["Concurrent Jobs"] = n   (Concurrent: n evaluation threads)
//   Distributed (one process per GPU, launched by torch.distributed.run or
//   any launcher that sets RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT /
//   LOCAL_RANK): the CMA-ES population or the TMCMC chains are sharded over
//   the ranks, every rank ends with the same solver state, rank 0 writes the
//   results.  k["Conduit"]["Transport"] = "RCCL" (default) | "Host";
//   k["Conduit"]["Bootstrap Port"] = p (default MASTER_PORT + 1);
//   k["Conduit"]["Ranks Per Worker"] must be 1.
class Engine {
 public:
  Json &operator[](const std::string &key) { return _js[key]; }
  void run(Experiment &e);
  void run(std::vector<Experiment> &es);
  void run(const std::vector<Experiment *> &es);
  Json _js;
};

// The conduit's batch dispatch on its own (tests): body(i) for i < n on
// `jobs` threads, the lowest failing index's exception rethrown.
void conduitEvaluate(size_t jobs, size_t n, const std::function<void(size_t)> &body);

// The Distributed conduit's collectives on host data (tests): rank / world
// from RANK / WORLD_SIZE, the "Host" transport's TCP bootstrap on `port`.
// gathered = every rank's `block` in rank order, summed = the element-wise
// sum over ranks, maxed = the element-wise MAX of the int64 bit patterns.
struct CollectiveCheck {
  int rank = 0, world = 1;
  std::vector<double> gathered, summed, maxed;
  bool peerFailed = false;
};
// failRank >= 0: that rank throws; the others return once their watchdog
// reports the failure (peerFailed)
CollectiveCheck collectiveSelfTest(int port, const std::vector<double> &block, int failRank = -1);

// Bayesian/Reference likelihood models (likelihood.cpp,
// reference.cpp.base:25-229): the log-likelihood of reference data y given the
// entries a computational model wrote into s; throws KoraliError like
// KORALI_LOG_ERROR on malformed entries.
double referenceLoglikelihood(const std::string &model, const std::vector<double> &y, Sample &s);
bool isReferenceLikelihoodModel(const std::string &model);
std::vector<double> referenceLoglikelihoodGradient(const std::string &model, const std::vector<double> &y, Sample &s,
                                                   size_t nth);
std::vector<double> referenceFisherInformation(const std::string &model, const std::vector<double> &y, Sample &s,
                                               size_t nth);
// Bayesian::evaluate of one parameter vector under an experiment's Problem /
// Distributions / Variables (the host evaluation CMA-ES uses on Bayesian
// problems); returns the sample's JSON (logPrior, logLikelihood, F(x), ...)
Json bayesianEvaluate(Json &experiment, const std::vector<double> &x);

// The continuous agent's policy description from an experiment's Variables
// and Solver (continuous.cpp.base:9-60 initializeAgent; agent.cpp.base:37-90):
// Problem vector sizes / indexes, Action Shifts / Scales, Policy/Parameter
// Count / Scaling / Shifting / Transformation Masks, the network's layer
// widths (state, hidden..., 1 + parameter count) and its hyperparameter
// count.  Written into VRACER result files; pinned by the reference's
// tests/python/rlview/abf2d_vracer* files.
Json vracerPolicyDescription(Json &experiment);
// the last run's generation completion marks: marks[0] = the loop's first
// termination check, marks[i] = when generation i's check returned (seconds
// from the start of the loop; timing hook, not part of the experiment state)
std::vector<double> generationCompletionTimes(const Experiment &e);
// Initial hyperparameters ([W (out x in), b] per layer, linear.cpp.base:28-49):
// Xavier-scaled U(-1, 1) weights (the output layer x 0.001,
// VRACER.cpp.base:38), zero biases; std::mt19937(seed) uniforms.
std::vector<float> vracerInitialHyperparameters(const std::vector<size_t> &sizes, unsigned seed);

}  // namespace korali
