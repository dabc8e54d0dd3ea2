// A C++ problem definition written in the reference's own idioms, built
// against this package's korali.hpp / libkorali_engine.so unchanged:
//   examples/features/running.cxx/_model/direct.hpp (float x = k["Parameters"][0]),
//   examples/features/running.cxx/run-cmaes-direct.cpp (auto e = korali::Experiment(); &direct),
//   source/sample/sample.hpp:25-26 (variadic KORALI_GET), sample.cpp:31-34 (update),
//   experiment.cpp.base:219-229 (getEvaluation), generated CMAES.cpp:1781 (unknown keys).
//
//   reference_idioms cpu   checks that need no GPU (exit 0 = pass)
//   reference_idioms gpu   also runs run-cmaes-direct's experiment
#include <korali.hpp>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

void direct(korali::Sample &k)
{
  float x = k["Parameters"][0];
  k["F(x)"] = -0.5 * x * x;
}

static int failures = 0;
#define EXPECT(cond, what)                                      \
  do {                                                          \
    if (!(cond)) {                                              \
      fprintf(stderr, "FAIL: %s (%s:%d)\n", what, __FILE__, __LINE__); \
      failures++;                                               \
    }                                                           \
  } while (0)

template <typename F>
static std::string errorOf(F f)
{
  try {
    f();
  } catch (const korali::KoraliError &e) {
    return e.what();
  } catch (const std::exception &e) {
    return std::string("non-Korali exception: ") + e.what();
  }
  return "";
}

static void cpuChecks()
{
  // implicit JSON conversions and the model function itself
  korali::Sample s;
  s["Parameters"] = std::vector<double>{3.0, -1.5};
  direct(s);
  double f = s["F(x)"];
  EXPECT(f == -4.5, "direct(): F(x) = -0.5 x^2 through implicit conversions");
  std::vector<double> p = s["Parameters"];
  EXPECT(p.size() == 2 && p[1] == -1.5, "std::vector<double> p = s[\"Parameters\"]");
  size_t n = s["Parameters"].size();
  EXPECT(n == 2, "size()");

  // variadic KORALI_GET over nested keys and indices
  s["Solver"]["Internal"]["Values"] = std::vector<double>{1.0, 2.0, 7.0};
  double v = KORALI_GET(double, s, "Solver", "Internal", "Values", 2);
  EXPECT(v == 7.0, "KORALI_GET(double, s, \"Solver\", \"Internal\", \"Values\", 2)");
  auto x = KORALI_GET(std::vector<double>, s, "Parameters");
  EXPECT(x.size() == 2, "KORALI_GET(std::vector<double>, s, \"Parameters\")");
  std::string e1 = errorOf([&] { (void)KORALI_GET(double, s, "Solver", "Missing"); });
  EXPECT(e1.find("Requesting non existing value [\"Solver\"][\"Missing\"] from sample.") != std::string::npos,
         "KORALI_GET of a missing path fails with the reference's message");
  std::string e2 = errorOf([&] { (void)KORALI_GET(std::vector<double>, s, "F(x)"); });
  EXPECT(e2.find("Missing or incorrect value [\"F(x)\"] for the sample.") != std::string::npos,
         "KORALI_GET of a wrongly typed value fails with the reference's message");
  s.update();  // no messages to hand over on this path

  // getEvaluation: not a learner solver
  auto e = korali::Experiment();
  std::string e3 = errorOf([&] { e.getEvaluation({{{1.0f}}}); });
  EXPECT(e3.find("This solver does not support evaluation operations.") != std::string::npos, "getEvaluation error");

  // a misspelt solver key is rejected before anything runs
  auto k = korali::Engine();
  auto bad = korali::Experiment();
  bad["Problem"]["Type"] = "Optimization";
  bad["Problem"]["Objective Function"] = &direct;
  bad["Variables"][0]["Name"] = "X";
  bad["Variables"][0]["Lower Bound"] = -10.0;
  bad["Variables"][0]["Upper Bound"] = +10.0;
  bad["Solver"]["Type"] = "Optimizer/CMAES";
  bad["Solver"]["Populaton Size"] = 32;  // sic
  bad["File Output"]["Enabled"] = false;
  bad["Console Output"]["Verbosity"] = "Silent";
  std::string e4 = errorOf([&] { k.run(bad); });
  EXPECT(e4.find("Unrecognized settings for Korali module: CMAES") != std::string::npos &&
             e4.find("Populaton Size") != std::string::npos,
         "misspelt solver key raises KoraliError");
  auto bad2 = korali::Experiment();
  bad2["Problem"]["Type"] = "Optimization";
  bad2["Problem"]["Objective Function"] = &direct;
  bad2["Variables"][0]["Name"] = "X";
  bad2["Solver"]["Type"] = "Optimizer/CMAES";
  bad2["Solver"]["Population Size"] = 32;
  bad2["Solver"]["Termination Criteria"]["Max Generation"] = 10;  // sic
  bad2["File Output"]["Enabled"] = false;
  bad2["Console Output"]["Verbosity"] = "Silent";
  std::string e5 = errorOf([&] { k.run(bad2); });
  EXPECT(e5.find("Unrecognized settings for Korali module: CMAES") != std::string::npos &&
             e5.find("Max Generation") != std::string::npos,
         "misspelt termination criterion raises KoraliError");
}

static void gpuRun()
{
  // examples/features/running.cxx/run-cmaes-direct.cpp, File Output off
  auto e = korali::Experiment();
  e["Problem"]["Type"] = "Optimization";
  e["Problem"]["Objective Function"] = &direct;

  e["Variables"][0]["Name"] = "X";
  e["Variables"][0]["Lower Bound"] = -10.0;
  e["Variables"][0]["Upper Bound"] = +10.0;

  e["Solver"]["Type"] = "Optimizer/CMAES";
  e["Solver"]["Population Size"] = 32;
  e["Solver"]["Termination Criteria"]["Min Value Difference Threshold"] = 1e-7;
  e["Solver"]["Termination Criteria"]["Max Generations"] = 100;
  e["Random Seed"] = 0xC0FFEE;
  e["File Output"]["Enabled"] = false;
  e["Console Output"]["Verbosity"] = "Silent";

  auto k = korali::Engine();
  k.run(e);

  double best = e["Results"]["Best Sample"]["F(x)"];
  double xbest = e["Results"]["Best Sample"]["Parameters"][0];
  EXPECT(best <= 0.0 && best > -1e-6, "CMA-ES maximises -0.5 x^2 to ~0");
  EXPECT(std::fabs(xbest) < 1e-3, "argmax x ~ 0");
  size_t gen = e["Current Generation"];
  EXPECT(gen >= 2 && gen <= 101, "ran until a termination criterion");
}

int main(int argc, char *argv[])
{
  const bool gpu = argc > 1 && !strcmp(argv[1], "gpu");
  cpuChecks();
  if (gpu) gpuRun();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("REFERENCE_IDIOMS PASS (%s)\n", gpu ? "cpu+gpu" : "cpu");
  return 0;
}
