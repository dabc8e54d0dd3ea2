// kg_eigen.hpp — GSL-faithful symmetric eigensolver (gsl_eigen_symmv +
// gsl_eigen_symmv_sort ABS_ASC) for CMAES::updateEigensystem.
#pragma once

#include <vector>

#include "kg_common.hpp"
#include "kg_host_tridiag.hpp"

namespace kg {

struct EigRec;

// profiling callback: phase 0/1 = begin/end of a device stage (events on the
// stream), 2/3 = begin/end of a host stage (wall clock)
typedef void (*ProfileFn)(void *ctx, const char *stage, int phase);

class EigenSolver {
 public:
  ~EigenSolver();
  void drain();  // waits for the side stream (device chase)
  // hostChase: run the serial implicit-QR Givens recurrence on the calling
  // host core (overlapped with the device unpack); otherwise on one lane.
  int init(int N, bool hostChase);
  int run(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
          double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof, void *profCtx);
  // run = run_begin (tridiagonalisation, unpack: workspace only) + run_finish
  int run_begin(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
          double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof, void *profCtx);
  int run_finish(const double *C, int diagonal, double *B, double *D, double *minEig, double *maxEig,
          double *eigenFailures, unsigned int *errors, hipStream_t s, ProfileFn prof, void *profCtx);
  bool begun = false;
  // the caller changed C after run_begin: the next run() starts over
  // (phase A again; a host hand-off is published again under a new sequence)
  void invalidate() { begun = false; }
  // C reaches the host core for the tridiagonalisation (tri == 6): run_begin
  // only publishes C, so a caller may issue it as soon as C is final
  bool host_tridiag() const { return tri == 6; }
  int t1flags = 0;  // KORALI_AMD_T1_FLAGS: experiment switches of k_tridiag_1wg
  bool sqDpp = true;  // k_tridiag_sq's scalar chains on registers / DPP broadcasts (KORALI_AMD_SQ_DPP=0: LDS-streamed)
  unsigned long long *trace = nullptr;  // optional device counters (k_tridiag sub-phases)
  // QR steps / Givens rotations of the last host chase (diagnostics)
  void last_counts(int &steps, int &rotations) const {
    steps = (hostChase && host.meta) ? host.meta[0] : -1;
    rotations = (hostChase && host.meta) ? host.meta[1] : -1;
  }
  bool hostChase = true;
  int tridiag_kind() const { return tri; }  // (diagnostics)
  // host-core tridiagonalisation (tri == 6): wall time of the last one (ms)
  double last_host_tridiag_ms = 0.0;

 private:
  int N = 0, maxRot = 0;
  bool lds = true;
  int tri = 0;  // tridiagonalisation kernel: 0 k_tridiag (LDS), 1 k_tridiag_1wg, 2 k_tridiag_mw, 3 k_tridiag_1wg2, 4 k_tridiag_sq, 5 k_tridiag_mw2, 6 host core
  int launch_unpack(hipStream_t s, ProfileFn prof, void *profCtx);
  // tri == 6: C's lower triangle reaches the host through host-coherent
  // memory (k_publish_c), the host writes the reflectors + tau back
  // (k_fetch_h copies them to gH / tau ahead of the unpack)
  HostTridiag htri;
  double *h_C = nullptr, *d_C_map = nullptr, *h_H = nullptr, *d_H_map = nullptr;
  int ldc = 0;  // row stride of h_C (even: 16-byte rows)
  unsigned int *pubDone = nullptr;  // k_publish_c's workgroup counter (device memory)
  unsigned long long cSeq = 0, pubSeq = 0;  // sequence of the C hand-off the host waits for; publications so far
  double *gA = nullptr, *gH = nullptr, *gQt = nullptr, *gWork = nullptr, *tau = nullptr, *dsd = nullptr,
         *chaseWork = nullptr;
  unsigned long long *comm = nullptr;  // in-launch hand-off granules (N > 128 tridiagonalisation)
  struct Rec {
    int *hdr = nullptr;
    double *cs = nullptr;
    int *meta = nullptr;
    double *eval = nullptr;
    int *perm = nullptr;
    operator EigRec() const;
  } dev, host, hmap;  // hmap: device aliases of the host-coherent chase buffers
  unsigned long long *hprog = nullptr, *dprog = nullptr;  // streamed-chase progress word (host / device view)
  unsigned long long chaseSeq = 0;
  unsigned long long *dprogDev = nullptr;  // fetcher -> apply progress word (device memory)
  double *h_dsd = nullptr, *d_dsd_map = nullptr;  // host-coherent d/sd and its device alias
  unsigned long long dsdSeq = 0;
  std::vector<double> hgc, hgs;
  hipStream_t side = nullptr;
  hipEvent_t ev_dsd = nullptr, ev_chase = nullptr;
};

}  // namespace kg
