// korali.hpp — the korali::Engine / korali::Experiment / korali::Sample API
// (reference: source/korali.hpp:25-31, source/engine.hpp, source/modules/
// experiment/experiment.hpp.base, source/sample/sample.hpp:25-191) on top of
// the korali_amd C-ABI.  Existing problem definitions compile unchanged:
//
//   #include <korali.hpp>
//   void model(korali::Sample &s) { auto x = KORALI_GET(std::vector<double>, s, "Parameters"); s["F(x)"] = ...; }
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

#include <memory>
#include <string>
#include <vector>

#include "json.hpp"

namespace korali {

// KORALI_GET(TYPE, SAMPLE, KEY): typed read of a sample entry (sample.hpp:25)
#define KORALI_GET(TYPE, SAMPLE, KEY) ((SAMPLE)[KEY].template get<TYPE>())

class Sample {
 public:
  Json &operator[](const std::string &key) { return _js[key]; }
  bool contains(const std::string &key) const { return _js.contains(key); }
  Json _js;
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

  Json _js;
  std::unique_ptr<ExperimentState> _state;
};

// Engine (source/engine.hpp): its own JSON holds the conduit,
//   k["Conduit"]["Type"] = "Sequential" (default) | "Concurrent";
//   k["Conduit"]["Concurrent Jobs"] = n   (Concurrent: n evaluation threads)
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

// Bayesian/Reference likelihood models (likelihood.cpp,
// reference.cpp.base:25-229): the log-likelihood of reference data y given the
// entries a computational model wrote into s; throws KoraliError like
// KORALI_LOG_ERROR on malformed entries.
double referenceLoglikelihood(const std::string &model, const std::vector<double> &y, Sample &s);
bool isReferenceLikelihoodModel(const std::string &model);
// Bayesian::evaluate of one parameter vector under an experiment's Problem /
// Distributions / Variables (the host evaluation CMA-ES uses on Bayesian
// problems); returns the sample's JSON (logPrior, logLikelihood, F(x), ...)
Json bayesianEvaluate(Json &experiment, const std::vector<double> &x);

// thrown for every configuration or runtime error (KORALI_LOG_ERROR)
class KoraliError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

}  // namespace korali
