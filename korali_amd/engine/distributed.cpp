// distributed.cpp — collectives of the Distributed conduit (distributed.hpp):
// a TCP bootstrap among the ranks of one node, an RCCL transport (librccl
// loaded at run time) and a host-staged transport.
#include "distributed.hpp"
#include "korali.hpp"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <cstring>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace korali {

namespace {

[[noreturn]] void dfail(const std::string &msg) {
  throw std::runtime_error("[Korali] Distributed conduit: " + msg);
}

int envInt(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

void sendAll(int fd, const void *p, size_t n) {
  const char *c = (const char *)p;
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) dfail("bootstrap connection lost while sending");
    c += k, n -= (size_t)k;
  }
}

void recvAll(int fd, void *p, size_t n) {
  char *c = (char *)p;
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) dfail("bootstrap connection lost while receiving");
    c += k, n -= (size_t)k;
  }
}

// Star of TCP connections rooted at rank 0 (the rendezvous of every
// transport; the Host transport also moves its data over it).
class Bootstrap {
 public:
  int rank, world;
  std::vector<int> peers;  // root: socket of each rank (index = rank); others: [0] = root
  Bootstrap(int rank_, int world_, int port) : rank(rank_), world(world_) {
    if (world <= 1) return;
    const char *addr = getenv("MASTER_ADDR");
    const std::string host = (addr && *addr) ? addr : "127.0.0.1";
    if (rank == 0) {
      const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
      if (ls < 0) dfail("socket() failed");
      const int one = 1;
      setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      sockaddr_in sa{};
      sa.sin_family = AF_INET;
      sa.sin_addr.s_addr = htonl(INADDR_ANY);
      sa.sin_port = htons((uint16_t)port);
      if (::bind(ls, (sockaddr *)&sa, sizeof(sa)) != 0) dfail("cannot bind the bootstrap port " + std::to_string(port));
      if (::listen(ls, world) != 0) dfail("listen() failed");
      peers.assign(world, -1);
      for (int k = 1; k < world; k++) {
        const int fd = ::accept(ls, nullptr, nullptr);
        if (fd < 0) dfail("accept() failed");
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        int32_t r = -1;
        recvAll(fd, &r, sizeof(r));
        if (r <= 0 || r >= world || peers[r] >= 0) dfail("bootstrap: unexpected rank " + std::to_string(r));
        peers[r] = fd;
      }
      ::close(ls);
    } else {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
        dfail("cannot resolve MASTER_ADDR '" + host + "'");
      const auto t0 = std::chrono::steady_clock::now();
      int fd = -1;
      for (;;) {
        fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
        if (fd >= 0) ::close(fd);
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
          dfail("rank " + std::to_string(rank) + " could not reach the bootstrap at " + host + ":" +
                std::to_string(port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
      freeaddrinfo(res);
      const int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      const int32_t r = rank;
      sendAll(fd, &r, sizeof(r));
      peers.assign(1, fd);
    }
  }
  ~Bootstrap() {
    for (int fd : peers)
      if (fd >= 0) ::close(fd);
  }
  // root: buf (world * bytes) <- every rank's block; then everyone gets buf
  void gatherToAll(void *buf, size_t bytes) {
    char *b = (char *)buf;
    if (rank == 0) {
      for (int k = 1; k < world; k++) recvAll(peers[k], b + (size_t)k * bytes, bytes);
      for (int k = 1; k < world; k++) sendAll(peers[k], b, (size_t)world * bytes);
    } else {
      sendAll(peers[0], b + (size_t)rank * bytes, bytes);
      recvAll(peers[0], b, (size_t)world * bytes);
    }
  }
  // root combines every rank's array in rank order, everyone gets the result
  template <class T, class Op>
  void reduceToAll(T *v, size_t n, Op op) {
    if (rank == 0) {
      std::vector<T> in(n);
      for (int k = 1; k < world; k++) {
        recvAll(peers[k], in.data(), n * sizeof(T));
        for (size_t i = 0; i < n; i++) v[i] = op(v[i], in[i]);
      }
      for (int k = 1; k < world; k++) sendAll(peers[k], v, n * sizeof(T));
    } else {
      sendAll(peers[0], v, n * sizeof(T));
      recvAll(peers[0], v, n * sizeof(T));
    }
  }
  void barrier() {
    char c = 0;
    if (world <= 1) return;
    if (rank == 0) {
      for (int k = 1; k < world; k++) recvAll(peers[k], &c, 1);
      for (int k = 1; k < world; k++) sendAll(peers[k], &c, 1);
    } else {
      sendAll(peers[0], &c, 1);
      recvAll(peers[0], &c, 1);
    }
  }
};

// Abort channel: a second star of TCP connections (bootstrap port + 1)
// watched by a thread of every rank.  A rank that leaves on an exception
// sends 'A' (the root relays it to every other rank), one that finishes
// sends 'B'; a connection closed without 'B' (the process died) counts as
// 'A'.  On 'A' the rank's transport is aborted (RCCL: ncclCommAbort, which
// ends the collective kernels waiting for the failed rank; Host: the
// bootstrap sockets are shut down, which ends a blocked recv) and every
// later collective or engine check throws.  The reference's MPI conduit gets
// the same from MPI_Abort on a worker error.
class Watchdog {
 public:
  Watchdog(int rank, int world, int port, std::function<void()> onAbort)
      : links_(rank, world, port), onAbort_(std::move(onAbort)) {
    if (world > 1) th_ = std::thread([this] { run(); });
  }
  ~Watchdog() { close(std::uncaught_exceptions() > 0); }
  bool aborted() const { return aborted_.load(); }
  // leave: 'A' when failing, else 'B'; joins the watcher
  void close(bool failing) {
    if (closed_.exchange(true)) return;
    stop_ = true;
    const char c = failing ? 'A' : 'B';
    for (size_t k = 0; k < links_.peers.size(); k++)
      if (links_.peers[k] >= 0) (void)::send(links_.peers[k], &c, 1, MSG_NOSIGNAL);
    if (th_.joinable()) th_.join();
  }

 private:
  Bootstrap links_;
  std::function<void()> onAbort_;
  std::thread th_;
  std::atomic<bool> stop_{false}, aborted_{false}, closed_{false};
  void trigger(int from) {
    if (aborted_.exchange(true)) return;
    const char c = 'A';
    if (links_.rank == 0)  // relay to every other rank
      for (size_t k = 1; k < links_.peers.size(); k++)
        if ((int)k != from && links_.peers[k] >= 0) (void)::send(links_.peers[k], &c, 1, MSG_NOSIGNAL);
    if (onAbort_) onAbort_();
  }
  void run() {
    std::vector<pollfd> fds;
    std::vector<int> who;
    for (size_t k = 0; k < links_.peers.size(); k++)
      if (links_.peers[k] >= 0) {
        fds.push_back({links_.peers[k], POLLIN, 0});
        who.push_back(links_.rank == 0 ? (int)k : 0);
      }
    while (!stop_) {
      if (::poll(fds.data(), fds.size(), 100) <= 0) continue;
      for (size_t i = 0; i < fds.size(); i++) {
        if (fds[i].fd < 0 || !fds[i].revents) continue;
        char c = 0;
        const ssize_t k = ::recv(fds[i].fd, &c, 1, 0);
        if (k == 1 && c == 'B') {
          fds[i].fd = -1;  // that rank finished: its close is not a failure
          continue;
        }
        fds[i].fd = -1;
        trigger(who[i]);
      }
    }
  }
};

class HostCollective : public Collective {
 public:
  Bootstrap boot;
  Watchdog dog;
  HostCollective(int r, int w, int port)
      : boot(r, w, port), dog(r, w, port + 1, [this] {
          for (int fd : boot.peers)
            if (fd >= 0) ::shutdown(fd, SHUT_RDWR);  // a blocked recv returns: the collective throws
        }) {
    rank = r;
    world = w;
  }
  std::string transport() const override { return "Host"; }
  bool failed() const override { return dog.aborted(); }
  void allGather(const SolverBuffer &b, size_t count) override {
    std::vector<double> v((size_t)world * count);
    b.get(v.data(), v.size() * sizeof(double));
    boot.gatherToAll(v.data(), count * sizeof(double));
    b.set(v.data(), v.size() * sizeof(double));
  }
  void allGatherHost(double *buf, size_t count) override { boot.gatherToAll(buf, count * sizeof(double)); }
  void allReduceSum(const SolverBuffer &b, size_t n) override {
    std::vector<double> v(n);
    b.get(v.data(), n * sizeof(double));
    boot.reduceToAll(v.data(), n, [](double a, double c) { return a + c; });
    b.set(v.data(), n * sizeof(double));
  }
  void allReduceMaxI64(const SolverBuffer &b, size_t n) override {
    std::vector<int64_t> v(n);
    b.get(v.data(), n * sizeof(int64_t));
    boot.reduceToAll(v.data(), n, [](int64_t a, int64_t c) { return a > c ? a : c; });
    b.set(v.data(), n * sizeof(int64_t));
  }
  void barrier() override { boot.barrier(); }
};

// the RCCL C API as librccl exports it (rccl.h: ncclUniqueId is 128 opaque
// bytes; ncclFloat64 = 8, ncclInt64 = 4; ncclSum = 0, ncclMax = 2)
struct NcclId {
  char internal[128];
};
typedef int (*GetUniqueIdFn)(NcclId *);
typedef int (*CommInitRankFn)(void **, int, NcclId, int);
typedef int (*AllGatherFn)(const void *, void *, size_t, int, void *, void *);
typedef int (*AllReduceFn)(const void *, void *, size_t, int, int, void *, void *);
typedef int (*CommDestroyFn)(void *);
typedef int (*CommAbortFn)(void *);
typedef const char *(*ErrorStringFn)(int);

class RcclCollective : public Collective {
 public:
  Bootstrap boot;
  void *lib = nullptr, *comm = nullptr;
  GetUniqueIdFn getUniqueId = nullptr;
  CommInitRankFn commInitRank = nullptr;
  AllGatherFn allGatherFn = nullptr;
  AllReduceFn allReduceFn = nullptr;
  CommDestroyFn commDestroy = nullptr;
  CommAbortFn commAbort = nullptr;
  ErrorStringFn errorString = nullptr;
  // commMu guards `comm` and the in-flight count; it is never held across an
  // RCCL call, so the watchdog's abort can always run.  A call that is in
  // flight when the abort fires (e.g. blocked in the lazy connection set-up
  // to the failed peer) is what ncclCommAbort exists to unblock: the abort
  // then runs outside the lock, concurrently with it, the call returns an
  // error and the rank leaves through check().
  std::mutex commMu;
  int inFlight = 0;
  bool commAborted = false;
  std::unique_ptr<Watchdog> dog;

  RcclCollective(int r, int w, int port) : boot(r, w, port) {
    rank = r;
    world = w;
    for (const char *n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((lib = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!lib) dfail("the RCCL transport needs librccl.so (ROCm), which could not be loaded");
    getUniqueId = (GetUniqueIdFn)dlsym(lib, "ncclGetUniqueId");
    commInitRank = (CommInitRankFn)dlsym(lib, "ncclCommInitRank");
    allGatherFn = (AllGatherFn)dlsym(lib, "ncclAllGather");
    allReduceFn = (AllReduceFn)dlsym(lib, "ncclAllReduce");
    commDestroy = (CommDestroyFn)dlsym(lib, "ncclCommDestroy");
    errorString = (ErrorStringFn)dlsym(lib, "ncclGetErrorString");
    commAbort = (CommAbortFn)dlsym(lib, "ncclCommAbort");
    if (!getUniqueId || !commInitRank || !allGatherFn || !allReduceFn || !commDestroy || !errorString || !commAbort)
      dfail("librccl.so lacks an nccl* entry point");
    dog.reset(new Watchdog(r, w, port + 1, [this] { abortComm(); }));
  }
  // the watchdog's abort: marks the communicator aborted (no new call can
  // take it) and aborts it -- under the lock when nothing is in flight,
  // outside it when a call is (that call is unblocked by it)
  void abortComm() {
    void *c = nullptr;
    {
      std::lock_guard<std::mutex> g(commMu);
      if (!comm || commAborted) return;
      commAborted = true;
      if (inFlight == 0) {
        commAbort(comm);
        return;
      }
      c = comm;
    }
    commAbort(c);
  }
  ~RcclCollective() override {
    const bool failing = std::uncaught_exceptions() > 0;
    dog->close(failing);  // (tells the other ranks first; joins the watchdog)
    std::lock_guard<std::mutex> g(commMu);
    if (comm && !commAborted) (failing ? commAbort : commDestroy)(comm);
  }
  std::string transport() const override { return "RCCL"; }
  bool failed() const override { return dog->aborted(); }
  void check(int rc, const char *what) {
    if (dog->aborted()) dfail("another rank failed; this rank's collectives were aborted");
    if (rc != 0) dfail(std::string(what) + ": " + errorString(rc));
  }
  // the communicator is created at the first collective, after the solver
  // handle has selected its GPU (RCCL binds the calling thread's device)
  void ensureComm() {
    if (dog->aborted()) dfail("another rank failed; this rank's collectives were aborted");
    {
      std::lock_guard<std::mutex> g(commMu);
      if (comm) return;
    }
    NcclId id{};
    if (rank == 0) check(getUniqueId(&id), "ncclGetUniqueId");
    std::vector<NcclId> all((size_t)world);
    all[(size_t)rank] = id;
    boot.gatherToAll(all.data(), sizeof(NcclId));  // (only the root's entry is used)
    void *c = nullptr;
    check(commInitRank(&c, world, all[0], rank), "ncclCommInitRank");
    bool late = false;
    {
      std::lock_guard<std::mutex> g(commMu);
      late = dog->aborted();
      if (!late) comm = c;
    }
    if (late) {  // the abort fired while the communicator was being created: it never saw this one
      commAbort(c);
      dfail("another rank failed; this rank's collectives were aborted");
    }
  }
  // takes the communicator under the lock (counted in flight), runs the RCCL
  // call without it
  template <class F>
  void enqueue(F &&call, const char *what) {
    ensureComm();
    void *c = nullptr;
    {
      std::lock_guard<std::mutex> g(commMu);
      if (!comm || commAborted || dog->aborted()) dfail("another rank failed; this rank's collectives were aborted");
      c = comm;
      inFlight++;
    }
    const int rc = call(c);
    {
      std::lock_guard<std::mutex> g(commMu);
      inFlight--;
    }
    check(rc, what);
  }
  void allGather(const SolverBuffer &b, size_t count) override {
    double *p = (double *)b.devicePtr();
    void *s = b.stream();
    enqueue([&](void *c) { return allGatherFn(p + (size_t)rank * count, p, count, 8 /* ncclFloat64 */, c, s); },
            "ncclAllGather");
  }
  void allGatherHost(double *buf, size_t count) override {
    if (dog->aborted()) dfail("another rank failed; this rank's collectives were aborted");
    boot.gatherToAll(buf, count * sizeof(double));
  }
  void allReduceSum(const SolverBuffer &b, size_t n) override {
    void *p = b.devicePtr(), *s = b.stream();
    enqueue([&](void *c) { return allReduceFn(p, p, n, 8 /* ncclFloat64 */, 0 /* ncclSum */, c, s); }, "ncclAllReduce");
  }
  void allReduceMaxI64(const SolverBuffer &b, size_t n) override {
    void *p = b.devicePtr(), *s = b.stream();
    enqueue([&](void *c) { return allReduceFn(p, p, n, 4 /* ncclInt64 */, 2 /* ncclMax */, c, s); }, "ncclAllReduce");
  }
  void barrier() override { boot.barrier(); }
};

}  // namespace

std::unique_ptr<Collective> makeCollective(const std::string &transport, int port) {
  const int world = envInt("WORLD_SIZE", 1), rank = envInt("RANK", 0);
  if (world < 1 || rank < 0 || rank >= world)
    dfail("RANK / WORLD_SIZE are inconsistent (" + std::to_string(rank) + " / " + std::to_string(world) + ")");
  if (port <= 0) port = envInt("MASTER_PORT", 29500) + 1;
  if (transport == "rccl") return std::unique_ptr<Collective>(new RcclCollective(rank, world, port));
  if (transport == "host") return std::unique_ptr<Collective>(new HostCollective(rank, world, port));
  dfail("'Transport' must be 'RCCL' or 'Host'");
}

CollectiveCheck collectiveSelfTest(int port, const std::vector<double> &block, int failRank) {
  std::unique_ptr<Collective> c = makeCollective("host", port);
  CollectiveCheck r;
  r.rank = c->rank;
  r.world = c->world;
  if (failRank >= 0) {
    // failure propagation: rank failRank throws (its collective leaves with
    // 'A'); every other rank waits for its watchdog to report it
    if (c->rank == failRank) dfail("rank " + std::to_string(failRank) + " failed on purpose");
    const auto t0 = std::chrono::steady_clock::now();
    while (!c->failed()) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) dfail("the peer failure was not reported");
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    r.peerFailed = true;
    return r;
  }
  const size_t n = block.size();
  auto hostBuffer = [](std::vector<double> &v) {
    SolverBuffer b;
    b.get = [&v](void *out, size_t bytes) { memcpy(out, v.data(), bytes); };
    b.set = [&v](void *in, size_t bytes) { memcpy(v.data(), in, bytes); };
    return b;
  };
  r.gathered.assign((size_t)c->world * n, 0.0);
  std::copy(block.begin(), block.end(), r.gathered.begin() + (size_t)c->rank * n);
  c->allGather(hostBuffer(r.gathered), n);
  r.summed = block;
  c->allReduceSum(hostBuffer(r.summed), n);
  r.maxed = block;
  c->allReduceMaxI64(hostBuffer(r.maxed), n);
  c->barrier();
  return r;
}

}  // namespace korali
