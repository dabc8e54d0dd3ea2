// CPU baseline variant (ii) of BASELINE.md §2 — TEST / MEASUREMENT
// INFRASTRUCTURE ONLY (run by bench.py's cpu_baseline leg, never by the
// product): the oracle's CMA-ES loop (refcpu.c, built against the system
// libm) with every sample dispatched the way Korali's Sequential conduit
// does it (conduit/sequential/sequential.cpp.base: one Sample JSON per
// candidate, "Module"/"Operation"/"Sample Id"/"Parameters" written, the
// model called on it, "F(x)" read back; Optimization::evaluate,
// optimization.cpp.base:25-36), using this repo's korali::Json.
//
//   dispatch_baseline N lambda warmup min_generations seconds
// prints one JSON line: generations, seconds, generations/s.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../korali_amd/engine/json.hpp"

extern "C" {
#include "refcpu.h"
}

// examples/optimization/stochastic/_model/model.py:23-34 on the sample
static void model(korali::Json &s) {
  std::vector<double> x = s["Parameters"];
  s["F(x)"] = kr_obj_negative_rosenbrock(x.data(), x.size());
}

int main(int argc, char **argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s N lambda warmup min_generations seconds\n", argv[0]);
    return 2;
  }
  const size_t N = std::strtoul(argv[1], nullptr, 10), lam = std::strtoul(argv[2], nullptr, 10);
  const long warm = std::atol(argv[3]), gmin = std::atol(argv[4]);
  const double budget = std::atof(argv[5]);
  kr_cmaes *h = kr_cmaes_new(N, lam, lam / 2);
  size_t n = 0;
  double *iv = kr_cmaes_field(h, "Initial Value", &n), *is = kr_cmaes_field(h, "Initial Standard Deviation", &n);
  for (size_t d = 0; d < N; d++) iv[d] = 0.0, is[d] = 1.0;
  kr_rng_seed(kr_cmaes_rng(h, 0), 1337);
  kr_rng_seed(kr_cmaes_rng(h, 1), 1338);
  auto generation = [&](size_t gen) {
    if (gen == 1) kr_cmaes_initialize(h);
    kr_cmaes_prepare(h);
    size_t m = 0;
    const double *X = kr_cmaes_field(h, "Sample Population", &m);
    double *F = kr_cmaes_field(h, "Value Vector", &m);
    for (size_t i = 0; i < lam; i++) {
      korali::Json s;
      s["Module"] = "Problem";
      s["Operation"] = "Evaluate";
      s["Sample Id"] = (unsigned long long)i;
      s["Parameters"] = std::vector<double>(X + i * N, X + (i + 1) * N);
      model(s);
      F[i] = s["F(x)"].getDouble();
    }
    kr_cmaes_update(h, gen);
  };
  size_t g = 0;
  for (long w = 0; w < warm; w++) generation(++g);
  const auto t0 = std::chrono::steady_clock::now();
  long k = 0;
  double el = 0.0;
  for (;;) {
    generation(++g);
    k++;
    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if ((k >= gmin && el > budget) || el > 4 * budget) break;
  }
  std::printf("{\"generations\": %ld, \"seconds\": %.6f, \"generations_per_sec\": %.6f}\n", k, el, k / el);
  kr_cmaes_free(h);
  return 0;
}
