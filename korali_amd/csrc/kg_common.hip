// kg_common.hip — error plumbing, double-double constant tables, ABI info.
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/korali_amd.h"
#include "kg_common.hpp"

namespace kg {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }
const char *last_error() { return g_last_error.c_str(); }

__constant__ dd_tables c_dd_tab;

// 1/q as an (unevaluated) double-double: hi = fl(1/q), lo = fl((1 - hi*q)/q)
// with the residual 1 - hi*q exact via fma.
static void dd_recip(double q, double &hi, double &lo) {
  hi = 1.0 / q;
  const double r = -std::fma(hi, q, -1.0);
  lo = r / q;
}

static dd_tables make_tables() {
  dd_tables t;
  for (int j = 0; j < 22; j++) dd_recip(2.0 * j + 1.0, t.inv_odd_hi[j], t.inv_odd_lo[j]);
  t.inv_int_hi[0] = t.inv_int_lo[0] = 0.0;
  for (int j = 1; j < 15; j++) dd_recip((double)j, t.inv_int_hi[j], t.inv_int_lo[j]);
  return t;
}

static const dd_tables &host_tables() {
  static const dd_tables t = make_tables();
  return t;
}

void upload_dd_tables() {
  static std::once_flag once;
  static bool ok = false;
  std::call_once(once, [] {
    const dd_tables &t = host_tables();
    ok = hipMemcpyToSymbol(HIP_SYMBOL(c_dd_tab), &t, sizeof(t)) == hipSuccess;
  });
  (void)ok;
}

// ------------------------------------------------- device block / stream cache
namespace {
struct DeviceCache {
  std::mutex mu;
  std::unordered_map<void *, std::pair<int, size_t>> live;  // block -> (device, rounded bytes)
  std::multimap<std::pair<int, size_t>, void *> idle;
  std::map<int, std::vector<hipStream_t>> streams;
  std::unordered_map<void *, std::pair<unsigned, size_t>> hostLive;  // pinned block -> (flags, bytes)
  std::multimap<std::pair<unsigned, size_t>, void *> hostIdle;
  size_t idleBytes = 0;
  size_t cap = [] {
    const char *e = getenv("KORALI_AMD_DEVICE_CACHE_MB");
    return (e && *e ? (size_t)strtoull(e, nullptr, 10) : (size_t)8192) << 20;
  }();
  void drop_idle() {  // under mu
    for (auto &kv : idle) (void)hipFree(kv.second);
    idle.clear();
    for (auto &kv : hostIdle) (void)hipHostFree(kv.second);
    hostIdle.clear();
    idleBytes = 0;
  }
};
// never destroyed: blocks may be released from other static destructors
DeviceCache &device_cache() {
  static auto *c = new DeviceCache();
  return *c;
}
}  // namespace

hipError_t dev_alloc(void **p, size_t bytes) {
  const size_t rb = ((bytes ? bytes : 1) + 511) & ~(size_t)511;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  DeviceCache &c = device_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.idle.find({dev, rb});
  if (it != c.idle.end()) {
    *p = it->second;
    c.idle.erase(it);
    c.idleBytes -= rb;
  } else {
    e = hipMalloc(p, rb);
    if (e == hipErrorOutOfMemory && !c.idle.empty()) {
      (void)hipGetLastError();
      c.drop_idle();
      e = hipMalloc(p, rb);
    }
    if (e != hipSuccess) return e;
  }
  c.live[*p] = {dev, rb};
  return hipSuccess;
}

void dev_release(void *p, hipStream_t drain) {
  if (!p) return;
  if (drain) (void)hipStreamSynchronize(drain);
  DeviceCache &c = device_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.live.find(p);
  if (it == c.live.end()) {  // not one of ours
    (void)hipFree(p);
    return;
  }
  const auto key = it->second;
  c.live.erase(it);
  if (c.idleBytes + key.second > c.cap) {
    (void)hipFree(p);
    return;
  }
  c.idle.emplace(key, p);
  c.idleBytes += key.second;
}

hipError_t host_alloc(void **p, size_t bytes, unsigned flags) {
  const size_t rb = ((bytes ? bytes : 1) + 511) & ~(size_t)511;
  DeviceCache &c = device_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.hostIdle.find({flags, rb});
  if (it != c.hostIdle.end()) {
    *p = it->second;
    c.hostIdle.erase(it);
    c.idleBytes -= rb;
    memset(*p, 0, rb);
  } else {
    hipError_t e = hipHostMalloc(p, rb, flags);
    if (e == hipErrorOutOfMemory && !c.hostIdle.empty()) {
      (void)hipGetLastError();
      c.drop_idle();
      e = hipHostMalloc(p, rb, flags);
    }
    if (e != hipSuccess) return e;
  }
  c.hostLive[*p] = {flags, rb};
  return hipSuccess;
}

void host_release(void *p) {
  if (!p) return;
  DeviceCache &c = device_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.hostLive.find(p);
  if (it == c.hostLive.end()) {
    (void)hipHostFree(p);
    return;
  }
  const auto key = it->second;
  c.hostLive.erase(it);
  if (c.idleBytes + key.second > c.cap) {
    (void)hipHostFree(p);
    return;
  }
  c.hostIdle.emplace(key, p);
  c.idleBytes += key.second;
}

hipError_t stream_acquire(hipStream_t *s) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  DeviceCache &c = device_cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto &v = c.streams[dev];
    if (c.cap && !v.empty()) {
      *s = v.back();
      v.pop_back();
      return hipSuccess;
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

void stream_release(hipStream_t s) {
  if (!s) return;
  (void)hipStreamSynchronize(s);
  int dev = 0;
  DeviceCache &c = device_cache();
  if (!c.cap || hipGetDevice(&dev) != hipSuccess) {
    (void)hipStreamDestroy(s);
    return;
  }
  std::lock_guard<std::mutex> lk(c.mu);
  c.streams[dev].push_back(s);
}

double host_log_cr(double x) {
  if (!(x > 0.0) || std::isinf(x)) return std::log(x);
  if (x == 1.0) return 0.0;
  if (x < 2.2250738585072014e-308) return std::log(x);
  const dd r = dd_log_tab(x, host_tables());
  return r.hi + r.lo;
}

// KORALI_AMD_SEGV_MAPS=1 (diagnostics of faults inside other libraries,
// e.g. under a profiler): on SIGSEGV write the faulting address, the native
// backtrace and /proc/self/maps to stderr (so every frame resolves to a
// library + offset), then die with the default action.  Async-signal-safe
// calls only (write, open, read; backtrace is preloaded at install time).
static void segv_diag(int sig, siginfo_t *si, void *) {
  char buf[4096];
  int n = snprintf(buf, sizeof buf, "\n[korali_amd SIGSEGV diagnostics] fault address %p\nbacktrace:\n", si ? si->si_addr : nullptr);
  (void)!write(2, buf, (size_t)n);
  void *bt[64];
  const int nb = backtrace(bt, 64);
  backtrace_symbols_fd(bt, nb, 2);
  const char mh[] = "/proc/self/maps:\n";
  (void)!write(2, mh, sizeof mh - 1);
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd >= 0) {
    ssize_t k;
    while ((k = read(fd, buf, sizeof buf)) > 0) (void)!write(2, buf, (size_t)k);
    close(fd);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}
__attribute__((constructor)) static void install_segv_diag() {
  const char *e = getenv("KORALI_AMD_SEGV_MAPS");
  if (!e || *e != '1') return;
  void *warm[2];
  (void)backtrace(warm, 2);  // (loads libgcc's unwinder outside the handler)
  struct sigaction sa {};
  sa.sa_sigaction = segv_diag;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, nullptr);
}

}  // namespace kg

extern "C" {
const char *kg_last_error(void) { return kg::last_error(); }
int kg_abi_version(void) { return KG_ABI_VERSION; }
int kg_device_count(int *count) {
  KG_HIP(hipGetDeviceCount(count));
  return 0;
}
}
