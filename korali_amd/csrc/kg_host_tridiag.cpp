// kg_host_tridiag.cpp — phase A of CMAES::eigen (CMAES.cpp.base:896-938:
// gsl_eigen_symmv → gsl_linalg_symmtd_decomp, GSL 2.6 linalg/symmtd.c with
// gslcblas dnrm2 / dsymv / ddot / daxpy / dsyr2) on one host core.
//
// Why the host core: the decomposition's arithmetic order is fixed by the
// bit-exactness contract (the eigenvector signs steer the next population),
// so each Householder step is three ordered FP64 chains (dnrm2, the dsymv row
// sums, x·v) plus a dozen dependent scalar operations (hypot, τ, 1/s).  On
// gfx950 a dependent FP64 add costs 14 shader cycles and a workgroup barrier
// ~1 µs; the one-workgroup kernel (k_tridiag_sq) measured 0.43 ms at N = 128,
// two thirds of it per-step fixed latency (profiles/r5/eigen_trace_c2.txt).
// A host core adds in 3-4 cycles at ~5 GHz and keeps eight ordered chains in
// flight per AVX-512 instruction, so the same operations in the same order
// take tens of µs.  The device keeps every stage whose work is parallel (the
// unpack of Q, the rotation replay, the draw, the update).
//
// Operation order (pinned by oracle/refcpu.c symmtd_decomp, which reproduces
// the reference's 99 committed eigensystems bit for bit):
//   householder_transform: dnrm2 of v[1..n-1] (gslcblas scaled ssq, in
//     order), β = -sign(α)·hypot(α, ‖x‖) (fdlibm), τ = (β-α)/β, v *= 1/(α-β);
//   dsymv (RowMajor, Lower, alpha τ): x[c] = Σ_{r = n-1 .. c} (τ v_r) m_rc
//     (descending r, the diagonal last), + τ·Σ_{k<c} v_k m_ck (ascending k);
//   xv = Σ x_r v_r (ascending), α' = -(τ/2)·xv, x += α' v;
//   dsyr2 (Lower, alpha -1): m_rj += (-v_r) x_j + (-x_r) v_j.
// Vectorisation never reorders an element's operations: SIMD lanes are
// different output elements.
//
// Layout and schedule: the lower triangle only, row r at a 64-byte aligned
// offset (length rounded up to 8), so the active submatrix fits the core's
// L1 after the first steps.  Step i's dsyr2 is deferred and fused into step
// i+1's dsymv: one descending pass over rows of 8 per step reads each 8x8
// tile once, applies the pending rank-2 update, adds the tile's rows to the
// column sums x (descending r, per column) and, after an in-register
// transpose, to the eight rows' dot chains (ascending k, per row).  Only
// column i+1, which the next Householder vector needs first, is updated
// ahead of the pass.
//
// Compiled by the host compiler (g++) with -ffp-contract=off (no FMA), -O3.
// The body (kg_host_tridiag_body.inc) is compiled three times, for AVX-512F,
// AVX2 and baseline SSE2, and the widest the core supports is called
// (KORALI_AMD_HOST_TRIDIAG_ISA = avx512 | avx2 | sse2 forces one).  No
// variant uses FMA, so all three produce the same bits.
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/file.h>
#include <unistd.h>
#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "kg_host_tridiag.hpp"

#define KGI __attribute__((always_inline)) inline

// KG_HT_PHASES (tools/host_tridiag_phases.cpp): time-stamp counters per phase
// into kg_ht_phases[]: 0 the copy of C, 1 column i with the pending update,
// 2 dnrm2, 3 the Householder scalars and v, 4 the fused row pass, 5 x.v and w
#ifdef KG_HT_PHASES
#include <x86intrin.h>
extern unsigned long long kg_ht_phases[8];
#define KG_HT_T(v) const unsigned long long v = __rdtsc()
#define KG_HT_ACC(k, v) kg_ht_phases[k] += __rdtsc() - (v)
#else
#define KG_HT_T(v)
#define KG_HT_ACC(k, v)
#endif

namespace kg {

namespace ht_avx512 {
#pragma GCC push_options
#pragma GCC target("avx512f")
#include "kg_host_tridiag_body.inc"
#pragma GCC pop_options
}  // namespace ht_avx512

namespace ht_avx2 {
#pragma GCC push_options
#pragma GCC target("avx2")
#include "kg_host_tridiag_body.inc"
#pragma GCC pop_options
}  // namespace ht_avx2

namespace ht_sse2 {
#include "kg_host_tridiag_body.inc"
}  // namespace ht_sse2

namespace {
typedef void (*TridiagFn)(HostTridiag &, const double *, int, double *, double *, double *, double *);
typedef void (*PassFn)(const HtMtJob &, int);
int isa_level() {  // 2 avx512, 1 avx2, 0 sse2
  const char *e = std::getenv("KORALI_AMD_HOST_TRIDIAG_ISA");
  const bool has512 = __builtin_cpu_supports("avx512f"), has2 = __builtin_cpu_supports("avx2");
  if (e && !std::strcmp(e, "sse2")) return 0;
  if (e && !std::strcmp(e, "avx2") && has2) return 1;
  if (has512 && !(e && !std::strcmp(e, "avx2"))) return 2;
  return has2 ? 1 : 0;
}
TridiagFn pick_isa() {
  static const TridiagFn f[3] = {ht_sse2::tridiag_run, ht_avx2::tridiag_run, ht_avx512::tridiag_run};
  return f[isa_level()];
}
PassFn pick_pass() {
  static const PassFn f[3] = {ht_sse2::mt_pass, ht_avx2::mt_pass, ht_avx512::mt_pass};
  return f[isa_level()];
}

// ---- helper threads of the multi-threaded pass
// CPUs for the helpers: the calling thread's L3 domain first (its siblings in
// /sys .../cache/index3/shared_cpu_list), one per physical core, within the
// process's affinity mask; then the rest of the mask.  Empty: no pinning.
std::vector<int> parse_cpu_list(const std::string &s) {
  std::vector<int> out;
  size_t i = 0;
  while (i < s.size()) {
    char *end = nullptr;
    const long a = std::strtol(s.c_str() + i, &end, 10);
    if (end == s.c_str() + i) break;
    long b = a;
    i = end - s.c_str();
    if (i < s.size() && s[i] == '-') {
      b = std::strtol(s.c_str() + i + 1, &end, 10);
      i = end - s.c_str();
    }
    for (long c = a; c <= b; c++) out.push_back((int)c);
    while (i < s.size() && (s[i] == ',' || s[i] == '\n' || s[i] == ' ')) i++;
  }
  return out;
}
std::string read_text(const std::string &path) {
  std::string out;
  if (FILE *f = std::fopen(path.c_str(), "r")) {
    char buf[4096];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
    std::fclose(f);
  }
  return out;
}
// A core is claimed with an advisory lock on /tmp/korali_amd_core_<cpu>.lock
// (released by the kernel when the process ends): the ranks of one node, and
// several solvers of one process, pin their helpers to disjoint cores.
bool claim_cpu(int cpu, std::vector<int> &fds) {
  const std::string path = "/tmp/korali_amd_core_" + std::to_string(cpu) + ".lock";
  const int fd = open(path.c_str(), O_CREAT | O_RDWR | O_CLOEXEC, 0666);
  if (fd < 0) return true;  // (no lock directory: no coordination)
  if (flock(fd, LOCK_EX | LOCK_NB)) {
    close(fd);
    return false;
  }
  fds.push_back(fd);
  return true;
}
// Per-CPU busy fraction over a short window from /proc/stat (empty when it is
// unreadable): on a shared host, cores another process keeps busy make slow
// helpers (a spinning helper preempted stalls every step of the pass).
std::vector<double> cpu_busy(int window_ms) {
  auto sample = [](std::vector<std::pair<unsigned long long, unsigned long long>> &v) {
    v.assign(CPU_SETSIZE, {0, 0});
    std::string t = read_text("/proc/stat");
    size_t i = 0;
    while ((i = t.find("\ncpu", i)) != std::string::npos) {
      i += 4;
      if (i >= t.size() || t[i] < '0' || t[i] > '9') continue;
      char *end = nullptr;
      const long c = std::strtol(t.c_str() + i, &end, 10);
      unsigned long long f[8] = {0}, tot = 0;
      const char *q = end;
      for (int k = 0; k < 8; k++) {
        f[k] = std::strtoull(q, &end, 10);
        if (end == q) break;
        q = end;
        tot += f[k];
      }
      if (c >= 0 && c < CPU_SETSIZE) v[c] = {tot, f[3] + f[4]};  // (idle + iowait)
    }
  };
  std::vector<std::pair<unsigned long long, unsigned long long>> a, b;
  sample(a);
  std::this_thread::sleep_for(std::chrono::milliseconds(window_ms));
  sample(b);
  std::vector<double> busy(CPU_SETSIZE, 0.0);
  bool any = false;
  for (int c = 0; c < CPU_SETSIZE; c++) {
    const unsigned long long dt = b[c].first - a[c].first, di = b[c].second - a[c].second;
    if (dt == 0) continue;
    any = true;
    busy[c] = 1.0 - (double)di / (double)dt;
  }
  if (!any) busy.clear();
  return busy;
}
std::vector<int> helper_cpus(int want, std::vector<int> &fds) {
  std::vector<int> out;
  cpu_set_t mask;
  if (want <= 0 || sched_getaffinity(0, sizeof mask, &mask)) return out;
  // KORALI_AMD_HOST_TRIDIAG_BUSY_MS=<ms>: idle cores first within each
  // candidate list (stable: topology order among equally idle ones), from a
  // /proc/stat window of that length.  Off by default: the window is paid at
  // every handle creation (20 ms against a 20-generation C2 run's ~11 ms),
  // /proc/stat counts in 10 ms ticks, and a same-box C4 A/B showed no gain.
  const char *bm = std::getenv("KORALI_AMD_HOST_TRIDIAG_BUSY_MS");
  const int window = bm ? std::atoi(bm) : 0;
  const std::vector<double> busy = window > 0 ? cpu_busy(window) : std::vector<double>();
  if (std::getenv("KORALI_AMD_HOST_TRIDIAG_VERBOSE") && !busy.empty()) {
    int nb = 0, n = 0;
    for (int c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &mask)) n++, nb += busy[c] > 0.25;
    std::fprintf(stderr, "[host tridiag] %d of %d allowed cpus busy over the probe window\n", nb, n);
  }
  auto by_idle = [&](std::vector<int> v) {
    if (!busy.empty())
      std::stable_sort(v.begin(), v.end(), [&](int x, int y) {
        const bool bx = x >= 0 && x < (int)busy.size() && busy[x] > 0.25;
        const bool by = y >= 0 && y < (int)busy.size() && busy[y] > 0.25;
        return bx < by;
      });
    return v;
  };
  const int me = sched_getcpu();
  const std::string sys = "/sys/devices/system/cpu/cpu";
  std::set<int> used;  // physical cores taken (their SMT siblings too)
  auto take_core = [&](int c) {
    for (int s : parse_cpu_list(read_text(sys + std::to_string(c) + "/topology/thread_siblings_list"))) used.insert(s);
    used.insert(c);
  };
  if (me >= 0) take_core(me);
  auto consider = [&](const std::vector<int> &cands) {
    for (int c : cands) {
      if ((int)out.size() >= want) return;
      if (c < 0 || c >= CPU_SETSIZE || !CPU_ISSET(c, &mask) || used.count(c)) continue;
      take_core(c);
      if (!claim_cpu(c, fds)) continue;
      out.push_back(c);
    }
  };
  if (me >= 0) consider(by_idle(parse_cpu_list(read_text(sys + std::to_string(me) + "/cache/index3/shared_cpu_list"))));
  std::vector<int> all;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &mask)) all.push_back(c);
  consider(by_idle(all));
  return out;
}
}  // namespace

struct HostTridiagPool {
  int P = 1;
  PassFn fn = nullptr;
  // the two blocked copies of the lower triangle and the step vectors (see
  // mt_pass); vectors padded to whole blocks + 16, zero past N
  int N = 0, NB = 0, L = 0;
  std::vector<double *> colblk, rowblk;
  double *vecs = nullptr;
  double *vec(int k) const { return vecs + (size_t)k * L; }
  std::vector<int> lockFds;  // the claimed helper cores (claim_cpu)
  HtMtJob job;
  std::vector<std::thread> th;
  alignas(64) std::atomic<unsigned> epoch{0};
  alignas(64) std::atomic<unsigned> done{0};
  alignas(64) std::atomic<int> awake{0};
  std::atomic<bool> quit{false};
  long spin_us = 3000;  // KORALI_AMD_HOST_TRIDIAG_SPIN_US
  std::mutex mu;
  std::condition_variable cv;

  void helper(int t, int cpu) {
    if (cpu >= 0) {
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(cpu, &one);
      (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
    }
    unsigned seen = 0;
    auto last = std::chrono::steady_clock::now();  // end of the last phase this thread worked on
    for (;;) {
      unsigned e;
      unsigned spins = 0;
      while ((e = epoch.load(std::memory_order_acquire)) == seen) {
        _mm_pause();
        // between decompositions the helpers keep spinning for spin_us (a
        // futex wake-up of a core in a deep idle state took longer than the
        // covariance's way to the host: measured 90 -> 300 us tridiagonal),
        // then sleep until the next wake()
        if ((++spins & 1023) == 0 && !awake.load(std::memory_order_relaxed) &&
            std::chrono::steady_clock::now() - last > std::chrono::microseconds(spin_us)) {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] {
            return epoch.load(std::memory_order_acquire) != seen || awake.load(std::memory_order_relaxed) ||
                   quit.load(std::memory_order_relaxed);
          });
          last = std::chrono::steady_clock::now();
        }
        if (quit.load(std::memory_order_relaxed)) return;
      }
      seen = e;
      if (quit.load(std::memory_order_relaxed)) return;
      fn(job, t);
      done.fetch_add(1, std::memory_order_release);
      last = std::chrono::steady_clock::now();
    }
  }
  // every thread (the caller as thread 0) runs fn(job, t); returns when all are done
  void phase() {
    done.store(0, std::memory_order_relaxed);
    epoch.fetch_add(1, std::memory_order_release);
    fn(job, 0);
    while (done.load(std::memory_order_acquire) != (unsigned)(P - 1)) _mm_pause();
  }
  void set_awake(int a) {
    {
      std::lock_guard<std::mutex> lk(mu);
      awake.store(a, std::memory_order_relaxed);
    }
    if (a) cv.notify_all();
  }
  ~HostTridiagPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit.store(true);
    }
    cv.notify_all();
    epoch.fetch_add(1, std::memory_order_release);
    for (auto &t : th) t.join();
    for (double *p : colblk) std::free(p);
    for (double *p : rowblk) std::free(p);
    std::free(vecs);
    for (int fd : lockFds) close(fd);
  }
};


namespace {
// The multi-threaded decomposition: tridiag_run's steps (the body file) in
// the same order, the two matrix passes of each step split over the pool
// (mt_pass: column and row blocks), the O(N) work between them on the
// calling thread.  Column i+1's entries, which the next Householder vector
// needs first, come from the column block that owns them (nextcol) plus the
// step's own rank-2 update, exactly as the single-core pass updates column i
// ahead of its row pass.
void run_mt(HostTridiag &w, const double *C, int ldc, double *H, double *tau, double *d, double *sd) {
  HostTridiagPool &p = *w.pool;
  const int N = w.N;
  double *v = p.vec(0), *pv = p.vec(1), *x = p.vec(2), *px = p.vec(3), *npv = p.vec(4), *npx = p.vec(5),
         *t1 = p.vec(6), *colsum = p.vec(7), *rowsum = p.vec(8), *nextcol = p.vec(9), *colb = p.vec(10);
  for (int k = 0; k < 11; k++) std::memset(p.vec(k), 0, (size_t)p.L * sizeof(double));
  p.set_awake(1);
  HtMtJob &J = p.job;
  J = HtMtJob();
  J.N = N, J.P = p.P, J.colblk = p.colblk.data(), J.rowblk = p.rowblk.data();
  J.kind = 1, J.C = C, J.ldc = ldc;
  p.phase();
  J.kind = 0;
  J.colsum = colsum, J.rowsum = rowsum, J.nextcol = nextcol;
  bool pending = false;
  for (int i = 0; i + 2 < N; i++) {
    const int o = i + 1, n = N - o;
    for (int r = i; r < N; r++) {  // column i with the pending update: the Householder input
      double m = i == 0 ? C[(size_t)r * ldc] : nextcol[r];
      if (pending) m += npv[r] * px[i] + npx[r] * pv[i];
      colb[r] = m;
    }
    d[i] = colb[i];
    double *hrow = H + (size_t)i * N;
    double ti = 0.0;
    const double xnorm = ht_sse2::dnrm2(n - 1, colb + o + 1);
    if (xnorm != 0.0) {  // gsl_linalg_householder_transform
      const double alpha = colb[o];
      const double beta = -(alpha >= 0.0 ? 1.0 : -1.0) * ht_sse2::hypot_fd(alpha, xnorm);
      ti = (beta - alpha) / beta;
      const double s = alpha - beta;
      if (std::fabs(s) > 2.2250738585072014e-308) {
        const double f = 1.0 / s;
        for (int c = o + 1; c < N; c++) v[c] = colb[c] * f;
      } else {
        const double eps = 2.2204460492503131e-16, f1 = eps / s, f2 = 1.0 / eps;
        for (int c = o + 1; c < N; c++) v[c] = (colb[c] * f1) * f2;
      }
      v[o] = 1.0;
      hrow[0] = beta;
      for (int r = 1; r < n; r++) hrow[r] = v[o + r];
      sd[i] = beta;
    } else {
      for (int r = 0; r < n; r++) hrow[r] = colb[o + r];
      sd[i] = colb[o];
    }
    tau[i] = ti;
    for (int c = 0; c < o; c++) v[c] = 0.0;  // lanes below the submatrix
    J.o = o, J.pv = pv, J.px = px, J.npv = npv, J.npx = npx, J.v = v, J.t1 = t1;
    J.nextCol = i + 3 < N;  // the next step's column o
    J.syr2 = pending;
    if (ti != 0.0) {
      for (int r = o; r < N; r++) t1[r] = ti * v[r];
      J.symv = 1;
      p.phase();
      for (int c = o; c < N; c++) x[c] = colsum[c] + ti * rowsum[c];
      double xv = 0.0;
      for (int c = o; c < N; c++) xv += x[c] * v[c];
      const double alpha = -(ti / 2.0) * xv;
      for (int c = o; c < N; c++) x[c] += alpha * v[c];
      for (int c = 0; c < o; c++) x[c] = 0.0;
      for (int c = 0; c < p.L; c++) {
        npv[c] = -1.0 * v[c];
        npx[c] = -1.0 * x[c];
      }
      std::swap(pv, v);
      std::swap(px, x);
      pending = true;
    } else {
      J.symv = 0;
      p.phase();  // (the pending update alone, and the next column)
      pending = false;
    }
  }
  if (N >= 2) {  // the last 2 x 2: from the column blocks, with the pending update
    auto at = [&](int r, int c) { return p.colblk[c / 8][(size_t)(r - (c & ~7)) * 8 + (c & 7)]; };
    double m[2][2];
    for (int r = N - 2; r < N; r++)
      for (int c = N - 2; c <= r; c++) {
        double q = N > 2 ? at(r, c) : C[(size_t)r * ldc + c];
        if (pending) q += npv[r] * px[c] + npx[r] * pv[c];
        m[r - (N - 2)][c - (N - 2)] = q;
      }
    d[N - 2] = m[0][0];
    sd[N - 2] = m[1][0];
    d[N - 1] = m[1][1];
  }
  p.set_awake(0);
}

int pool_init(HostTridiag &w, int P) {
  HostTridiagPool *p = new HostTridiagPool();
  w.pool = p;
  const int N = w.N;
  p->P = P, p->N = N, p->NB = (N + 7) / 8, p->L = p->NB * 8 + 16;
  p->fn = pick_pass();
  if (const char *e = std::getenv("KORALI_AMD_HOST_TRIDIAG_SPIN_US")) p->spin_us = std::atol(e);
  for (int c = 0; c < p->NB; c++) {
    p->colblk.push_back((double *)std::aligned_alloc(64, (size_t)(N - 8 * c) * 64));
    const int kn = 8 * c + 8 < N ? 8 * c + 8 : N;
    p->rowblk.push_back((double *)std::aligned_alloc(64, (size_t)kn * 64));
    if (!p->colblk.back() || !p->rowblk.back()) return 1;
  }
  p->vecs = (double *)std::aligned_alloc(64, (size_t)11 * p->L * sizeof(double));
  if (!p->vecs) return 1;
  // helpers pinned one per physical core next to the caller (unpinned, they
  // measured 3-5x slower on the box: the scheduler spreads them over CCDs);
  // fewer free cores than asked: fewer helpers (none: the single-core pass)
  const bool pin = !std::getenv("KORALI_AMD_HOST_TRIDIAG_NOPIN");
  const std::vector<int> cpus = helper_cpus(pin ? P - 1 : 0, p->lockFds);
  if (pin) p->P = P = 1 + (int)cpus.size();
  if (std::getenv("KORALI_AMD_HOST_TRIDIAG_VERBOSE")) {
    std::fprintf(stderr, "[host tridiag] caller on cpu %d, %d helper(s) on cpus", sched_getcpu(), P - 1);
    for (int c : cpus) std::fprintf(stderr, " %d", c);
    std::fprintf(stderr, "\n");
  }
  if (P == 1) return 0;
  for (int t = 1; t < P; t++) {
    const int cpu = pin ? cpus[t - 1] : -1;
    p->th.emplace_back([p, t, cpu] { p->helper(t, cpu); });
  }
  return 0;
}
}  // namespace

int HostTridiag::init(int N_) {
  release();
  N = N_;
  const int R = (N + 7) & ~7;  // rows incl. zero padding up to a whole block
  const int L = R + 16;
  size_t tot = 0;
  for (int r = 0; r < R; r++) tot += (size_t)((r + 8) & ~7);
  const size_t vec = (size_t)L, nvec = 8;
  mem = (double *)std::aligned_alloc(64, (tot + nvec * vec) * sizeof(double));
  row = (double **)std::malloc(sizeof(double *) * (R > 0 ? R : 1));
  if (!mem || !row) {
    release();
    return 1;
  }
  std::memset(mem, 0, (tot + nvec * vec) * sizeof(double));
  size_t off = 0;
  for (int r = 0; r < R; r++) {
    row[r] = mem + off;
    off += (size_t)((r + 8) & ~7);
  }
  double *p = mem + tot;
  v[0] = p;
  v[1] = p + vec;
  x[0] = p + 2 * vec;
  x[1] = p + 3 * vec;
  nv = p + 4 * vec;
  nx = p + 5 * vec;
  colb = p + 6 * vec;
  t1 = p + 7 * vec;
  // threads: KORALI_AMD_HOST_TRIDIAG_THREADS, else 6 from N = 256 up, 4 from
  // N = 128 (box, round 6: N = 512 4.16 -> 1.50 ms, 256 0.60 -> 0.33, 128
  // 0.099 -> 0.079; more threads than that gained nothing within the box's
  // 16-CPU share) and 1 below
  threads = N >= 256 ? 6 : (N >= 128 ? 4 : 1);
  if (const char *e = std::getenv("KORALI_AMD_HOST_TRIDIAG_THREADS")) threads = std::atoi(e);
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  if (threads > (N + 7) / 8) threads = (N + 7) / 8;
  if (threads > 1 && N >= 8 && pool_init(*this, threads)) {
    release();
    return 1;
  }
  if (pool && pool->P == 1) {  // no helper core could be claimed
    delete pool;
    pool = nullptr;
  }
  threads = pool ? pool->P : 1;
  return 0;
}

void HostTridiag::release() {
  delete pool;
  pool = nullptr;
  std::free(mem);
  std::free(row);
  mem = nullptr;
  row = nullptr;
}

void HostTridiag::wake() {
  if (pool) pool->set_awake(1);
}

void HostTridiag::run(const double *C, int ldc, double *H, double *tau, double *d, double *sd) {
  if (N == 1) {
    d[0] = C[0];
    return;
  }
  if (pool) {
    run_mt(*this, C, ldc, H, tau, d, sd);
    return;
  }
  static const TridiagFn fn = pick_isa();
  fn(*this, C, ldc, H, tau, d, sd);
}

}  // namespace kg
