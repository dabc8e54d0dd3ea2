// Phase times of the host tridiagonalisation (kg_host_tridiag.cpp built with
// KG_HT_PHASES) on a Wishart matrix: build and run on the box's core,
//   g++ -O3 -std=c++17 -pthread -ffp-contract=off -fno-math-errno -Wno-psabi -DKG_HT_PHASES \
//       -I korali_amd/csrc -o tools/host_tridiag_phases tools/host_tridiag_phases.cpp \
//       korali_amd/csrc/kg_host_tridiag.cpp
//   tools/host_tridiag_phases 128 400
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <x86intrin.h>

#include "kg_host_tridiag.hpp"

unsigned long long kg_ht_phases[8];

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 128, reps = argc > 2 ? atoi(argv[2]) : 200;
  std::mt19937_64 g(N);
  std::normal_distribution<double> nd;
  std::vector<double> Y((size_t)N * 2 * N), C((size_t)N * N);
  for (auto &y : Y) y = nd(g);
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) {
      double s = 0;
      for (int k = 0; k < 2 * N; k++) s += Y[(size_t)i * 2 * N + k] * Y[(size_t)j * 2 * N + k];
      C[(size_t)i * N + j] = s / (2 * N);
    }
  kg::HostTridiag h;
  h.init(N);
  std::vector<double> H((size_t)N * N), tau(N), d(N), sd(N);
  for (int k = 0; k < 5; k++) h.run(C.data(), N, H.data(), tau.data(), d.data(), sd.data());
  for (auto &p : kg_ht_phases) p = 0;
  const unsigned long long c0 = __rdtsc();
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; k++) h.run(C.data(), N, H.data(), tau.data(), d.data(), sd.data());
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
  const double tsc = (double)(__rdtsc() - c0) / reps, per_us = tsc / us;
  static const char *nm[6] = {"copy C", "column i", "dnrm2", "scalars+v", "row pass", "x.v, w"};
  printf("N=%d: %.1f us per tridiagonalisation (TSC %.0f MHz)", N, us, per_us);
  double acc = 0;
  for (int k = 0; k < 6; k++) {
    const double p = kg_ht_phases[k] / (double)reps / per_us;
    acc += p;
    printf(" | %s %.1f", nm[k], p);
  }
  printf(" | rest %.1f\n", us - acc);
  return 0;
}
