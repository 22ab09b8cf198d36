// Native front end: HTTP/1.1 server for the API's hot routes with no Python on the request path
// (SURVEY §7.5 hard part 2: "p50 is dominated by the host stack"; the reference serves these
// through Flask, RO/Flaskr/routes.py:29-50,89-127,365-383), and — when given an upstream port — the
// service's MAIN port: every other request is relayed unchanged to the Python (ASGI) app.
//
//  * POST /api/predict_eta, /predict: answered in the reactor (below).
//  * POST /api/optimize_route, /route, /api/request_route: parsed requests go to the GPU's route
//    service (csrc/route_service.hip: K5 + K6 + batched A* + native assembly, byte-identical to
//    the FastAPI handler); the connection is parked until its job comes back through the
//    reactor's eventfd.  A request whose semantics the native path does not mirror comes back as
//    a fallback and is relayed to the Python app.
//  * anything else: relayed to the upstream ASGI server over a per-connection keep-alive
//    connection; a streamed (chunked) answer such as the SSE feed turns the connection into a
//    byte tunnel for the rest of its life.
//
// Design (one process, MI355X-first):
//  * R reactor threads, each with its own SO_REUSEPORT listening socket (the kernel spreads
//    connections), its own epoll set, HIP stream and pinned (mapped) record/output buffers.
//  * Natural batching: every epoll wake-up parses ALL complete requests that arrived on all ready
//    connections (native JSON -> 16-byte EtaRecords, csrc/runtime/rt_core.h — the same code as the
//    batched /predict path), then issues ONE zero-copy launch of the fused featurize+MLP kernel
//    (K1+K2 read the records from pinned host memory and write minutes back over PCIe), one
//    stream sync, and formats every response with the CPython-exact formatter.  An idle server
//    answers a lone request after one launch; under load, batches grow with concurrency.
//  * Semantics follow the FastAPI handlers (api/app.py): non-JSON content type or malformed JSON
//    on /api/predict_eta reads as {} (Flask get_json(silent=True)); a JSON array (or {"items": []})
//    on /predict is a batch answered as {"predictions": [...]}; per-item errors -> 400 for single
//    requests, {"error": ...} entries in batches.  GET /api/ping is answered natively; everything
//    else is relayed to the upstream app (404 when the front end runs without one).
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "native_model.h"
#include "ops.h"
#include "route_service.h"
#include "runtime/history_db.h"
#include "runtime/rt_core.h"

namespace rt {

namespace {

using rtc::EtaRecord;
using rtc::Stamp;

struct Shared;

struct ServerCfg {
  int port = 0, threads = 1, device = 0, slot = 0, max_batch = 1 << 20;
  int persist_cap = 1024;              // rounds of up to this many rows use the resident scorer
  double persist_idle_ms = 20.0;       // (0 = off); it exits after this long without a request
  double persist_life_ms = 50.0;       // ... or after this long resident (then relaunched)
  std::vector<std::string> cors_exact;
  bool cors_vercel = true;
  int upstream_port = 0;               // Python app for everything not answered natively (0 = none)
  RouteService* routes = nullptr;      // this reactor's GPU's route service (nullptr = relay routes)
  Shared* sh = nullptr;                // the server's models, scorers and GPU health
  std::string history_db;              // the store's SQLite file: history / locations answered natively
  std::shared_ptr<const rrec::RecordGraph> record_graph;   // compact route records' graph (history detail)
};

// GPU health of one reactor slot: consecutive launch failures quarantine the GPU; a
// quarantined GPU gets one probe round every probe_ms and is restored by a success.  `fault` is the
// ROUTEST_FAULT=gpu_fail[@slot] injection hook (launches on the slot fail without running).
struct SlotHealth {
  std::atomic<int> consec{0};
  std::atomic<bool> quarantined{false};
  std::atomic<long long> failures{0}, rounds{0}, quarantines{0};
  std::atomic<long long> probe_at_ms{0};
  std::atomic<bool> fault{false};
  std::atomic<bool> hang{false};       // ROUTEST_FAULT=gpu_hang@<slot>: each launch first runs a kernel
                                       // that waits on a host flag (the watchdog's test)
  std::atomic<long long> timeouts{0};  // rounds abandoned at the deadline (ROUTEST_GPU_DEADLINE_MS)
};

// Fault hook of the latency watchdog: one wave that waits until the host releases it (or at most
// max_ticks of the 100 MHz wall clock), so the launch behind it on the same stream misses its
// deadline.  Reads only; every wave reaches the exit condition.
__global__ __launch_bounds__(64) void hang_kernel(const int* release, long long max_ticks) {
  const long long t0 = wall_clock64();
  // (also bounded by iterations: ~3.4 us per sleep at 2.4 GHz, 2M of them ~7 s, whatever the
  // wall clock's rate)
  for (int it = 0; it < 2000000 && __hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
                   wall_clock64() - t0 < max_ticks;
       ++it)
    __builtin_amdgcn_s_sleep(127);
}

inline long long mono_ms() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (long long)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

// Server-wide state the reactors and route services share.
struct Shared {
  std::vector<int> devices;                                // per slot
  std::mutex model_mu;
  std::vector<std::shared_ptr<const NativeModel>> models;  // per slot (hot-swapped under model_mu)
  std::atomic<uint64_t> epoch{0};
  std::vector<PersistentScorer*> scorers;                  // per slot (nullptr: none)
  std::vector<std::unique_ptr<std::mutex>> scorer_mus;
  std::vector<std::unique_ptr<SlotHealth>> health;
  int quarantine_after = 3;
  long long probe_ms = 30000;
  double deadline_ms = 500.0;          // ROUTEST_GPU_DEADLINE_MS: a round not done by then is abandoned
  double trace_ms = -1.0;              // ROUTEST_ROUTE_TRACE_MS: log slow / missed rounds (watchdog rehearsal)
  int* hang_release = nullptr;         // pinned host flag of the gpu_hang fault hook (1 = release)
  int* hang_release_d = nullptr;
  // the model each resident scorer was created on: its blob stays allocated while the scorer lives
  std::vector<std::shared_ptr<const NativeModel>> scorer_models;
  int slots() const { return (int)devices.size(); }
  std::vector<std::shared_ptr<const NativeModel>> snapshot() {
    std::lock_guard<std::mutex> lk(model_mu);
    return models;
  }
  std::shared_ptr<const NativeModel> model(int g) {
    std::lock_guard<std::mutex> lk(model_mu);
    return models[g];
  }
  bool usable(int g) {
    SlotHealth& h = *health[g];
    if (!h.quarantined.load(std::memory_order_relaxed)) return true;
    const long long now = mono_ms();
    long long due = h.probe_at_ms.load();
    return now >= due && h.probe_at_ms.compare_exchange_strong(due, now + probe_ms);   // one probe per period
  }
  void fail(int g) {
    SlotHealth& h = *health[g];
    h.failures.fetch_add(1);
    if (h.consec.fetch_add(1) + 1 >= quarantine_after && !h.quarantined.exchange(true)) {
      h.quarantines.fetch_add(1);
      h.probe_at_ms.store(mono_ms() + probe_ms);
    }
  }
  // a round that missed its deadline: the GPU is quarantined at once (its queue may hold a hung
  // kernel; rounds fail over to the other GPUs / the CPU), and re-probed after probe_ms
  void timed_out(int g) {
    SlotHealth& h = *health[g];
    h.failures.fetch_add(1);
    h.timeouts.fetch_add(1);
    h.consec.fetch_add(1);
    if (!h.quarantined.exchange(true)) h.quarantines.fetch_add(1);
    h.probe_at_ms.store(mono_ms() + probe_ms);
  }
  void ok(int g) {
    SlotHealth& h = *health[g];
    h.rounds.fetch_add(1, std::memory_order_relaxed);
    h.consec.store(0, std::memory_order_relaxed);
    if (h.quarantined.load(std::memory_order_relaxed)) h.quarantined.store(false);
  }
  // Micro-cache of the app's GET /api/health and GET /metrics answers (ROUTEST_FRONT_CACHE_MS,
  // default 250; 0 = relay every one): a probe or scrape served from the last answer while it is
  // younger than the TTL, or while one relay refreshes it (stale-while-revalidate), so at most one
  // such request per TTL crosses into the single Python process.  Both answers are snapshots of
  // process state anyway (uptime, counters); only requests WITHOUT an Origin header use the cache
  // (the app's CORS headers depend on it).
  struct CacheEnt {
    std::string resp;                  // full HTTP response bytes (status line .. body)
    long long t_ms = -1;
    uint64_t sig = 0;                  // state_sig() when stored: a hot swap or a quarantine change
    bool inflight = false;             // invalidates it at once
  };
  uint64_t state_sig() const {
    uint64_t v = epoch.load(std::memory_order_relaxed) * 0x9E3779B97F4A7C15ull;
    for (const auto& h : health)
      v = v * 1000003ull + (uint64_t)h->quarantines.load(std::memory_order_relaxed) * 2 +
          (h->quarantined.load(std::memory_order_relaxed) ? 1 : 0);
    return v;
  }
  std::mutex rc_mu;
  CacheEnt rc[2];
  long long rc_ttl_ms = 250;
  // park the slot's resident scorer (before a normal launch that may share its hardware queue)
  void park(int g) {
    if (g < 0 || g >= (int)scorers.size()) return;
    std::lock_guard<std::mutex> lk(*scorer_mus[g]);
    if (scorers[g] != nullptr) pscore_park(scorers[g]);
  }
};

struct Conn {
  int fd = -1;
  uint64_t gen = 0;      // distinguishes a reused fd from the connection a late job belongs to
  std::string in, out;
  size_t out_off = 0;
  bool close_after = false;
  int npending = 0;      // requests of this connection waiting for the batch launch
  bool async = false;    // a route job or a relayed request is in flight: answers stay in order
  // relay to the upstream app
  int up = -1;
  std::string up_out, up_in;
  size_t up_off = 0;
  bool up_head = false;  // the relayed request was HEAD (no response body)
  bool up_wait = false;  // a relayed request's answer is outstanding (async also covers route jobs)
  bool tunnel = false;   // streamed upstream answer: bytes flow both ways unparsed from now on
  int cache_slot = -1;   // the relayed request refreshes Shared::rc[cache_slot]
  long long up_used_ms = 0;   // last request written to / answer read from the upstream connection
};

// A route job's reactor-side context.
class Reactor;
struct JobTag {
  Reactor* reactor;
  int fd;
  uint64_t gen;
  bool keep_alive;
  std::string origin;
  std::string raw;       // the whole HTTP request, for the relay if the job falls back
};

// One parsed prediction request waiting for the batch launch.
struct Pending {
  int fd;
  size_t first = 0, count = 0;         // record range in this round's batch
  std::vector<Stamp> stamps;
  std::vector<std::string> errs;
  bool batch = false, keep_alive = true;
  std::string origin;
};

struct Stats {
  std::atomic<long long> requests{0}, predictions{0}, launches{0}, errors{0}, resident{0}, fallbacks{0},
      wire8{0}, route_requests{0}, route_fallbacks{0}, relayed{0}, failovers{0}, cpu_rounds{0}, history{0},
      cached{0}, timeouts{0};
};

inline Stamp now_local() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  struct tm lt;
  time_t t = ts.tv_sec;
  localtime_r(&t, &lt);
  Stamp s;
  s.secs = rtc::days_from_civil(lt.tm_year + 1900, (unsigned)lt.tm_mon + 1, (unsigned)lt.tm_mday) * 86400 +
           lt.tm_hour * 3600 + lt.tm_min * 60 + lt.tm_sec;
  s.us = (int32_t)(ts.tv_nsec / 1000);
  return s;
}

inline bool ieq(const char* a, size_t n, const char* b) {
  if (std::strlen(b) != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return false;
  return true;
}

class Reactor {
 public:
  Reactor(const ServerCfg& cfg, Stats& st, std::atomic<bool>& stop) : cfg_(cfg), st_(st), stop_(stop) {}
  int device() const { return cfg_.device; }

  bool init(std::string& err) {
    lfd_ = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)cfg_.port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind_any_) a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(lfd_, (sockaddr*)&a, sizeof a) != 0 || listen(lfd_, 4096) != 0) {
      err = std::string("bind/listen: ") + std::strerror(errno);
      return false;
    }
    ep_ = epoll_create1(0);
    wake_ = eventfd(0, EFD_NONBLOCK);
    add(lfd_);
    add(wake_);
    return true;
  }

  void set_bind_any(bool v) { bind_any_ = v; }
  void set_routes(RouteService* r) { cfg_.routes = r; }
  int wake_fd() const { return wake_; }

  // called on the route service's worker thread
  void job_done(RouteJob* j) {
    {
      std::lock_guard<std::mutex> lk(done_mu_);
      done_.push_back(j);
    }
    uint64_t one = 1;
    (void)!write(wake_, &one, 8);
  }
  // many at once: one lock and one wake-up
  void jobs_done(const std::vector<RouteJob*>& js) {
    if (js.empty()) return;
    {
      std::lock_guard<std::mutex> lk(done_mu_);
      done_.insert(done_.end(), js.begin(), js.end());
    }
    uint64_t one = 1;
    (void)!write(wake_, &one, 8);
  }

  void run() {
    if (hipSetDevice(cfg_.device) != hipSuccess) return;
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return;
    cap_ = cfg_.max_batch;
    // portable + mapped: a round can be re-run on another GPU when this one is quarantined
    const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
    if (hipHostMalloc((void**)&h_rec_, (size_t)cap_ * 16, fl) != hipSuccess ||
        hipHostMalloc((void**)&h_rec8_, (size_t)cap_ * 8, fl) != hipSuccess ||
        hipHostMalloc((void**)&h_out_, (size_t)cap_ * 4, fl) != hipSuccess)
      return;
    if (hipHostGetDevicePointer(&d_rec_, h_rec_, 0) != hipSuccess ||
        hipHostGetDevicePointer(&d_rec8_, h_rec8_, 0) != hipSuccess ||
        hipHostGetDevicePointer((void**)&d_out_, h_out_, 0) != hipSuccess)
      return;
    (void)alloc_round(spare_);         // the latency watchdog's spare round buffers
    streams_[cfg_.device] = stream_;
    // ROUTEST_HANG_ARM=1 (the watchdog rehearsal): the gpu_hang hook's isolated streams exist from
    // the start, so arming the fault later creates no hardware queue
    if (const char* v = std::getenv("ROUTEST_HANG_ARM"))
      if (std::string(v) == "1")
        for (int g = 0; g < cfg_.sh->slots(); ++g) {
          hipStream_t hs;
          if (hipSetDevice(cfg_.sh->devices[g]) == hipSuccess && isolated_stream(cfg_.sh->devices[g], &hs) == hipSuccess)
            streams_[-1 - g] = hs;
        }
    (void)hipSetDevice(cfg_.device);

    epoll_event evs[256];
    while (!stop_.load(std::memory_order_relaxed) || inflight_ > 0) {
      const int n = epoll_wait(ep_, evs, 256, 100);
      for (int i = 0; i < n; ++i) {
        const int fd = evs[i].data.fd;
        if (fd == lfd_) { if (!stop_.load(std::memory_order_relaxed)) accept_all(); continue; }
        if (fd == wake_) { uint64_t v; (void)!read(wake_, &v, 8); drain_done(); continue; }
        auto ui = up2c_.find(fd);
        if (ui != up2c_.end()) {
          auto ci = conns_.find(ui->second);
          if (ci != conns_.end()) on_upstream(ci->second, evs[i].events);
          continue;
        }
        auto it = conns_.find(fd);
        if (it == conns_.end()) continue;
        if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) on_readable(it->second);
        if (evs[i].events & EPOLLOUT) flush(it->second);
      }
      run_batch();
      for (int fd : to_close_) close_conn(fd);
      to_close_.clear();
      if (stop_.load(std::memory_order_relaxed) && n == 0) drain_done();
    }
    for (auto& kv : conns_) {
      if (kv.second.up >= 0) close(kv.second.up);
      close(kv.first);
    }
    conns_.clear();
    close(lfd_);
    close(ep_);
    close(wake_);
    (void)hipHostFree(h_rec_);
    (void)hipHostFree(h_rec8_);
    (void)hipHostFree(h_out_);
    for (auto& kv : streams_) {
      (void)hipSetDevice(kv.first >= 0 ? kv.first : cfg_.sh->devices[-1 - kv.first]);
      (void)hipStreamDestroy(kv.second);
    }
    for (auto& kv : events_) {
      (void)hipSetDevice(kv.first >= 0 ? kv.first : cfg_.sh->devices[-1 - kv.first]);
      (void)hipEventDestroy(kv.second);
    }
    reap_retired(true);
    for (void* p : {(void*)spare_.rec, (void*)spare_.rec8, (void*)spare_.out})
      if (p) (void)hipHostFree(p);
    (void)hipSetDevice(cfg_.device);
  }

 private:
  ServerCfg cfg_;                      // per-reactor copy: device + blob of its GPU
  Stats& st_;
  std::atomic<bool>& stop_;
  bool bind_any_ = false;
  int lfd_ = -1, ep_ = -1, wake_ = -1;
  hipStream_t stream_{};
  EtaRecord* h_rec_ = nullptr;
  rtc::Wire8* h_rec8_ = nullptr;       // the same round as 8-byte wire records, when exact
  float* h_out_ = nullptr;
  void* d_rec_ = nullptr;
  void* d_rec8_ = nullptr;
  float* d_out_ = nullptr;
  int cap_ = 0;
  size_t nrec_ = 0;
  std::unordered_map<int, hipStream_t> streams_;        // per device (failover launches)
  std::unordered_map<int, hipEvent_t> events_;          // per device: the round's completion
  // rounds abandoned at the deadline: their stream, buffers, workspace and model stay allocated
  // until their kernels drain (checked every round; released at shutdown after the hang flag)
  struct Retired {
    int dev;
    hipEvent_t ev;
    hipStream_t st;
    void *rec, *rec8, *out, *ws;
    std::shared_ptr<const NativeModel> model;
  };
  std::vector<Retired> retired_;
  rth::HistoryDb hdb_;                                  // this reactor's connection to the store
  bool hdb_tried_ = false;
  std::unordered_map<int, ModelWs> ws_;                 // per stream key (device, or the gpu_hang stream)
  uint64_t next_gen_ = 1;
  std::unordered_map<int, Conn> conns_;
  std::unordered_map<int, int> up2c_;  // upstream fd -> client fd
  std::vector<Pending> pending_;
  std::vector<int> to_close_;
  std::mutex done_mu_;
  std::vector<RouteJob*> done_;
  int inflight_ = 0;                   // route jobs submitted and not yet drained

  void add(int fd, uint32_t ev = EPOLLIN) {
    epoll_event e{};
    e.events = ev;
    e.data.fd = fd;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
  }

  void accept_all() {
    while (true) {
      const int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      Conn c;
      c.fd = fd;
      c.gen = next_gen_++;
      conns_[fd] = std::move(c);
      add(fd);
    }
  }

  void close_conn(int fd) {
    auto it = conns_.find(fd);
    if (it == conns_.end()) return;
    if (it->second.up >= 0) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, it->second.up, nullptr);
      up2c_.erase(it->second.up);
      close(it->second.up);
    }
    conns_.erase(it);
    epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
  }

  void on_readable(Conn& c) {
    char buf[65536];
    bool eof = false;
    while (true) {
      const ssize_t r = read(c.fd, buf, sizeof buf);
      if (r > 0) {
        c.in.append(buf, (size_t)r);
        if (c.in.size() > (256u << 20)) { to_close_.push_back(c.fd); return; }
        continue;
      }
      if (r == 0) { eof = true; break; }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      to_close_.push_back(c.fd);
      return;
    }
    if (c.tunnel) {                    // streamed upstream answer: forward the client's bytes raw
      c.up_out += c.in;
      c.in.clear();
      flush_up(c);
      if (eof) to_close_.push_back(c.fd);
      return;
    }
    if (eof) {
      // half-closed client: answer what is already complete, then close
      if (!c.async) parse_requests(c);
      if (c.async) { c.close_after = true; return; }
      if (c.out.size() > c.out_off) flush(c);
      to_close_.push_back(c.fd);
      return;
    }
    if (!c.async) parse_requests(c);
    if (c.out.size() > c.out_off) flush(c);   // immediate answers (errors, ping, 100-continue)
  }

  // Parse every complete request buffered on c (pipelining allowed); stops at an async request.
  void parse_requests(Conn& c) {
    while (!c.async && !c.tunnel) {
      const size_t hend = c.in.find("\r\n\r\n");
      if (hend == std::string::npos) {
        if (c.in.size() > 65536) { respond(c, 431, "{\"error\":\"headers too large\"}", "", true); }
        return;
      }
      const char* p = c.in.data();
      const size_t sp1 = c.in.find(' ');
      const size_t sp2 = sp1 == std::string::npos ? sp1 : c.in.find(' ', sp1 + 1);
      const size_t eol = c.in.find("\r\n");
      if (sp1 == std::string::npos || sp2 == std::string::npos || sp2 > eol) {
        respond(c, 400, "{\"error\":\"bad request line\"}", "", true);
        c.in.clear();
        return;
      }
      const std::string method(p, sp1);
      std::string path(p + sp1 + 1, sp2 - sp1 - 1);
      const size_t qm = path.find('?');
      if (qm != std::string::npos) path.resize(qm);
      const bool http10 = c.in.compare(sp2 + 1, 8, "HTTP/1.0") == 0;
      size_t clen = 0;
      bool json = false, keep = !http10, expect100 = false, chunked = false;
      std::string origin;
      size_t ls = eol + 2;
      while (ls < hend) {
        const size_t le = c.in.find("\r\n", ls);
        const size_t colon = c.in.find(':', ls);
        if (colon != std::string::npos && colon < le) {
          const char* k = p + ls;
          const size_t kn = colon - ls;
          size_t vs = colon + 1;
          while (vs < le && (p[vs] == ' ' || p[vs] == '\t')) ++vs;
          const std::string v(p + vs, le - vs);
          if (ieq(k, kn, "content-length")) clen = (size_t)std::strtoull(v.c_str(), nullptr, 10);
          else if (ieq(k, kn, "content-type")) {
            std::string lv = v;
            for (auto& ch : lv) ch = (char)std::tolower((unsigned char)ch);
            json = lv.find("json") != std::string::npos;
          } else if (ieq(k, kn, "connection")) {
            std::string lv = v;
            for (auto& ch : lv) ch = (char)std::tolower((unsigned char)ch);
            if (lv.find("close") != std::string::npos) keep = false;
            if (lv.find("keep-alive") != std::string::npos) keep = true;
          } else if (ieq(k, kn, "expect")) {
            expect100 = v.size() >= 3 && v.compare(0, 3, "100") == 0;
          } else if (ieq(k, kn, "transfer-encoding")) {
            chunked = true;
          } else if (ieq(k, kn, "origin")) {
            origin = v;
          }
        }
        ls = le + 2;
      }
      if (chunked) {
        if (cfg_.upstream_port > 0) {      // the Python app decodes chunked bodies: relay raw
          start_tunnel(c);
          return;
        }
        respond(c, 411, "{\"error\":\"chunked bodies are not supported; send Content-Length\"}", origin, true);
        c.in.clear();
        return;
      }
      if (clen > (256u << 20)) {
        respond(c, 413, "{\"error\":\"body too large\"}", origin, true);
        c.in.clear();
        return;
      }
      if (c.in.size() < hend + 4 + clen) {
        if (expect100 && c.in.size() == hend + 4) {
          if (c.npending > 0) run_batch();
          c.out += "HTTP/1.1 100 Continue\r\n\r\n";
          flush(c);
        }
        return;   // body not complete yet
      }
      std::string raw = c.in.substr(0, hend + 4 + clen);
      std::string body = c.in.substr(hend + 4, clen);
      c.in.erase(0, hend + 4 + clen);
      st_.requests.fetch_add(1, std::memory_order_relaxed);
      handle(c, method, path, body, json, keep, origin, raw);
      if (c.close_after) return;
    }
  }

  bool cors_ok(const std::string& o) const {
    if (o.empty()) return false;
    for (const auto& e : cfg_.cors_exact)
      if (e == o) return true;
    const std::string suf = ".vercel.app";
    return cfg_.cors_vercel && o.compare(0, 8, "https://") == 0 && o.size() > suf.size() + 8 &&
           o.compare(o.size() - suf.size(), suf.size(), suf) == 0;
  }

  void respond(Conn& c, int code, const std::string& body, const std::string& origin, bool close_after) {
    if (c.npending > 0) run_batch();   // HTTP/1.1 pipelining: answers leave in request order
    const char* reason = code == 200 ? "OK" : code == 204 ? "No Content" : code == 400 ? "Bad Request" : code == 404 ? "Not Found"
                         : code == 405 ? "Method Not Allowed" : code == 411 ? "Length Required"
                         : code == 413 ? "Payload Too Large" : code == 431 ? "Request Header Fields Too Large"
                         : code == 502 ? "Bad Gateway" : code == 503 ? "Service Unavailable" : "Error";
    char head[256];
    const int hn = code == 204 ? std::snprintf(head, sizeof head, "HTTP/1.1 204 No Content\r\n")
                               : std::snprintf(head, sizeof head,
                                               "HTTP/1.1 %d %s\r\ncontent-type: application/json\r\ncontent-length: %zu\r\n",
                                               code, reason, body.size());
    c.out.append(head, (size_t)hn);
    if (cors_ok(origin)) {
      c.out += "access-control-allow-origin: ";
      c.out += origin;
      c.out += "\r\naccess-control-allow-credentials: true\r\nvary: Origin\r\n";
    }
    if (close_after) c.out += "connection: close\r\n";
    c.out += "\r\n";
    c.out += body;
    if (close_after) c.close_after = true;
    if (code >= 400) st_.errors.fetch_add(1, std::memory_order_relaxed);
  }

  void handle(Conn& c, const std::string& method, const std::string& path, const std::string& body,
              bool json, bool keep, const std::string& origin, std::string& raw) {
    if (method == "OPTIONS") {
      if (c.npending > 0) run_batch();
      std::string h = "HTTP/1.1 200 OK\r\ncontent-length: 0\r\naccess-control-allow-methods: GET, POST, OPTIONS\r\n"
                      "access-control-allow-headers: *\r\n";
      if (cors_ok(origin)) h += "access-control-allow-origin: " + origin + "\r\naccess-control-allow-credentials: true\r\n";
      c.out += h + "\r\n";
      return;
    }
    if (path == "/api/ping" && method == "GET") {             // RO/Flaskr/routes.py:129-131
      respond(c, 200, "{\"ok\":true,\"service\":\"route-optimizer\"}", origin, !keep);
      return;
    }
    const bool is_opt = path == "/api/optimize_route" || path == "/route", is_req = path == "/api/request_route";
    if ((is_opt || is_req) && method == "POST" && cfg_.routes != nullptr) {
      if (c.npending > 0) run_batch();           // earlier predictions of this connection first
      auto* tag = new JobTag{this, c.fd, c.gen, keep, origin, std::move(raw)};
      auto* j = new RouteJob();
      j->body = body;
      j->json_ok = json;
      j->request_route = is_req;
      j->tag = tag;
      c.async = true;
      ++inflight_;
      st_.route_requests.fetch_add(1, std::memory_order_relaxed);
      if (!cfg_.routes->submit(j)) {             // the service is stopping: the app answers
        j->fallback = true;
        job_done(j);
      }
      return;
    }
    if (!cfg_.history_db.empty() && (method == "GET" || method == "DELETE") && answer_history(c, method, path, keep, origin, raw))
      return;
    const bool is_pe = path == "/api/predict_eta", is_p = path == "/predict";
    // a model family the native path does not serve (after a hot swap): the app answers
    const bool no_model = (is_pe || is_p) && method == "POST" && cfg_.sh->model(cfg_.slot) == nullptr;
    if (!(is_pe || is_p) || method != "POST" || no_model) {
      if (cfg_.upstream_port > 0) {
        const int slot = (method == "GET" && origin.empty() && cfg_.sh->rc_ttl_ms > 0)
                             ? (path == "/api/health" ? 0 : (path == "/metrics" ? 1 : -1)) : -1;
        if (slot >= 0) {
          Shared& sh = *cfg_.sh;
          std::unique_lock<std::mutex> lk(sh.rc_mu);
          Shared::CacheEnt& e = sh.rc[slot];
          const long long now = mono_ms();
          if (e.t_ms >= 0 && e.sig == sh.state_sig() && (now - e.t_ms < sh.rc_ttl_ms || e.inflight)) {
            if (c.npending > 0) { lk.unlock(); run_batch(); lk.lock(); }
            c.out += e.resp;
            lk.unlock();
            st_.cached.fetch_add(1, std::memory_order_relaxed);
            if (!keep) c.close_after = true;
            return;
          }
          if (!e.inflight) {
            e.inflight = true;
            c.cache_slot = slot;
          }
        }
        relay(c, raw, method == "HEAD");
        return;
      }
      if (!is_pe && !is_p) respond(c, 404, "{\"detail\":\"Not Found\"}", origin, !keep);
      else if (no_model) respond(c, 503, "{\"error\":\"model unavailable\"}", origin, !keep);
      else respond(c, 405, "{\"detail\":\"Method Not Allowed\"}", origin, !keep);
      return;
    }
    // body -> items
    rtj::Value root;
    bool parsed = false;
    std::string perr;
    if (json) {
      try {
        root = rtj::Parser(body.data(), body.size()).parse();
        parsed = true;
      } catch (const std::exception& e) {
        perr = e.what();
      }
    }
    Pending pd;
    pd.fd = c.fd;
    pd.keep_alive = keep;
    pd.origin = origin;
    std::vector<const rtj::Value*> items;
    rtj::Value empty;
    empty.kind = rtj::Value::Obj;
    if (is_p && parsed && root.kind == rtj::Value::Arr) {
      pd.batch = true;
      for (const auto& v : root.arr) items.push_back(&v);
    } else if (is_p && parsed && root.kind == rtj::Value::Obj && root.get("items") &&
               root.get("items")->kind == rtj::Value::Arr) {
      pd.batch = true;
      for (const auto& v : root.get("items")->arr) items.push_back(&v);
    } else if (is_p && json && !parsed && body.find_first_not_of(" \t\r\n") != std::string::npos &&
               body[body.find_first_not_of(" \t\r\n")] == '[') {
      std::string o = "{\"error\":\"";
      for (char ch : perr) { if (ch == '"' || ch == '\\') o += '\\'; if ((unsigned char)ch >= 0x20) o += ch; }
      respond(c, 400, o + "\"}", origin, !keep);
      return;
    } else {
      items.push_back(parsed && root.kind == rtj::Value::Obj ? &root : &empty);   // silent -> {}
    }
    if (nrec_ + items.size() > (size_t)cap_) run_batch();   // flush before overflowing the buffer
    if (items.size() > (size_t)cap_) {
      respond(c, 413, "{\"error\":\"batch larger than the server's max_batch\"}", origin, !keep);
      return;
    }
    const Stamp now = now_local();
    pd.first = nrec_;
    pd.count = items.size();
    pd.stamps.resize(items.size());
    pd.errs.resize(items.size());
    for (size_t i = 0; i < items.size(); ++i) {
      EtaRecord r{};
      pd.errs[i] = rtc::pack_item(*items[i], now, r, pd.stamps[i]);
      h_rec_[nrec_ + i] = r;
    }
    nrec_ += items.size();
    if (!pd.batch && !pd.errs[0].empty()) {   // single request with bad input: answer now
      nrec_ -= items.size();
      std::string o = "{\"error\":\"invalid input: ";
      for (char ch : pd.errs[0]) { if (ch == '"' || ch == '\\') o += '\\'; if ((unsigned char)ch >= 0x20) o += ch; }
      respond(c, 400, o + "\"}", origin, !keep);
      return;
    }
    ++c.npending;
    pending_.push_back(std::move(pd));
  }

  // History list / detail / delete and locations straight from the store's SQLite database
  // (csrc/runtime/history_db.h, byte-identical to the app); false: not answered here (relay).
  bool answer_history(Conn& c, const std::string& method, const std::string& path, bool keep,
                      const std::string& origin, const std::string& raw) {
    const bool list = path == "/api/history" && method == "GET";
    const bool item = path.size() > 13 && path.compare(0, 13, "/api/history/") == 0 && path.find('/', 13) == std::string::npos;
    const bool locs = path == "/api/locations" && method == "GET";
    if (!list && !item && !locs) return false;
    if (!hdb_tried_) {
      hdb_tried_ = true;
      std::string err;
      (void)hdb_.open(cfg_.history_db, err);
      hdb_.set_graph(cfg_.record_graph);
    }
    if (!hdb_.ok()) return false;
    rth::Reply r;
    if (list) {
      // the raw query string of the request line; percent-encoded or repeated params -> the app
      const size_t le = raw.find("\r\n");
      const std::string line = raw.substr(0, le);
      const size_t qm = line.find('?');
      const size_t sp = line.rfind(' ');
      std::string q = (qm != std::string::npos && sp != std::string::npos && sp > qm) ? line.substr(qm + 1, sp - qm - 1) : "";
      if (q.find('%') != std::string::npos || q.find('+') != std::string::npos) return false;
      std::string lim;
      int found = 0;
      size_t b = 0;
      while (b <= q.size() && !q.empty()) {
        size_t e = q.find('&', b);
        if (e == std::string::npos) e = q.size();
        const std::string kv = q.substr(b, e - b);
        if (kv.compare(0, 6, "limit=") == 0) { lim = kv.substr(6); ++found; }
        else if (kv == "limit") { lim.clear(); ++found; }
        b = e + 1;
      }
      if (found > 1) return false;
      r = hdb_.history(found ? lim.c_str() : nullptr);
    } else if (item) {
      const std::string id = path.substr(13);
      if (id.find('%') != std::string::npos) return false;
      r = method == "GET" ? hdb_.detail(id) : hdb_.del(id);
    } else {
      r = hdb_.locations();
    }
    if (r.fallback) return false;
    st_.history.fetch_add(1, std::memory_order_relaxed);
    if (c.npending > 0) run_batch();
    respond(c, r.status, r.body, origin, !keep);
    return true;
  }

  // ---------------------------------------------------------------- route jobs coming back
  void drain_done() {
    std::vector<RouteJob*> jobs;
    {
      std::lock_guard<std::mutex> lk(done_mu_);
      jobs.swap(done_);
    }
    for (RouteJob* j : jobs) {
      --inflight_;
      JobTag* t = static_cast<JobTag*>(j->tag);
      auto it = conns_.find(t->fd);
      if (it != conns_.end() && it->second.gen == t->gen) {
        Conn& c = it->second;
        c.async = false;
        if (j->fallback) {
          st_.route_fallbacks.fetch_add(1, std::memory_order_relaxed);
          if (cfg_.upstream_port > 0) {
            relay(c, t->raw, false);
          } else {
            respond(c, 503, "{\"error\":\"request not supported by the native route path\"}", t->origin,
                    !t->keep_alive);
          }
        } else {
          respond(c, j->status, j->out, t->origin, !t->keep_alive);
        }
        if (!c.async) {
          flush(c);
          if (!c.close_after && !c.tunnel) {
            parse_requests(c);                 // requests that arrived while the job ran
            if (c.out.size() > c.out_off) flush(c);
          }
        }
      }
      delete t;
      delete j;
    }
  }

  // ---------------------------------------------------------------- relay to the Python app
  bool connect_up(Conn& c) {
    if (c.up >= 0) return true;
    const int u = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK, 0);
    if (u < 0) return false;
    int one = 1;
    setsockopt(u, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)cfg_.upstream_port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(u, (sockaddr*)&a, sizeof a) != 0 && errno != EINPROGRESS) {
      close(u);
      return false;
    }
    c.up = u;
    c.up_in.clear();
    c.up_out.clear();
    c.up_off = 0;
    up2c_[u] = c.fd;
    add(u, EPOLLIN | EPOLLOUT);
    return true;
  }

  // uvicorn closes a keep-alive connection after 5 idle seconds; a request written as that close
  // crosses it would come back as a 502, so an upstream connection idle for 2 s is replaced first
  // (with most relays answered from the micro-cache, client connections idle upstream for long)
  bool connect_fresh_up(Conn& c) {
    const long long now = mono_ms();
    if (c.up >= 0 && !c.tunnel && now - c.up_used_ms > 2000) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, c.up, nullptr);
      up2c_.erase(c.up);
      close(c.up);
      c.up = -1;
    }
    c.up_used_ms = now;
    return connect_up(c);
  }

  void relay(Conn& c, const std::string& raw, bool head) {
    if (c.npending > 0) run_batch();
    flush(c);
    if (!connect_fresh_up(c)) {
      respond(c, 502, "{\"error\":\"upstream app unavailable\"}", "", true);
      flush(c);
      return;
    }
    st_.relayed.fetch_add(1, std::memory_order_relaxed);
    c.up_out += raw;
    c.up_head = head;
    c.up_wait = true;
    c.async = true;
    flush_up(c);
  }

  // chunked request bodies (and anything after them) go to the app as raw bytes
  void start_tunnel(Conn& c) {
    if (c.npending > 0) run_batch();
    flush(c);
    if (!connect_fresh_up(c)) {
      respond(c, 502, "{\"error\":\"upstream app unavailable\"}", "", true);
      flush(c);
      return;
    }
    c.tunnel = true;
    c.up_out += c.in;
    c.in.clear();
    flush_up(c);
  }

  void flush_up(Conn& c) {
    if (c.up < 0) return;
    while (c.up_off < c.up_out.size()) {
      const ssize_t w = write(c.up, c.up_out.data() + c.up_off, c.up_out.size() - c.up_off);
      if (w > 0) { c.up_off += (size_t)w; continue; }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOTCONN)) return;   // EPOLLOUT resumes
      upstream_closed(c);
      return;
    }
    c.up_out.clear();
    c.up_off = 0;
  }

  // a cacheable relay ended: store its answer (a complete 200) or just clear the refresh flag
  void cache_done(Conn& c, const std::string* resp, size_t n) {
    Shared& sh = *cfg_.sh;
    std::lock_guard<std::mutex> lk(sh.rc_mu);
    Shared::CacheEnt& e = sh.rc[c.cache_slot];
    if (resp != nullptr && resp->compare(0, 9, "HTTP/1.1 ") == 0 &&
        resp->find("\r\nconnection: close", 0) > n) {      // (an answer that closes is not reused)
      e.resp.assign(*resp, 0, n);
      e.t_ms = mono_ms();
      e.sig = sh.state_sig();
    }
    e.inflight = false;
    c.cache_slot = -1;
  }

  void upstream_closed(Conn& c) {
    if (c.cache_slot >= 0) cache_done(c, nullptr, 0);
    if (c.up < 0) return;
    epoll_ctl(ep_, EPOLL_CTL_DEL, c.up, nullptr);
    up2c_.erase(c.up);
    close(c.up);
    c.up = -1;
    if (c.tunnel) {                    // the stream ended: deliver what is left, then close
      if (!c.up_in.empty()) { c.out += c.up_in; c.up_in.clear(); }
      c.close_after = true;
      flush(c);
      return;
    }
    if (c.up_wait) {                   // no (complete) answer came back
      c.up_wait = false;
      if (!c.up_in.empty() && c.up_in.find("\r\n\r\n") != std::string::npos && !c.up_in.empty()) {
        c.out += c.up_in;              // read-until-close body
        c.up_in.clear();
        c.close_after = true;
      } else {
        c.async = false;
        respond(c, 502, "{\"error\":\"upstream app closed the connection\"}", "", true);
      }
      flush(c);
    }
  }

  void on_upstream(Conn& c, uint32_t events) {
    if (events & EPOLLOUT) {
      flush_up(c);
      if (c.up >= 0 && c.up_out.empty()) {
        epoll_event e{};
        e.events = EPOLLIN;
        e.data.fd = c.up;
        epoll_ctl(ep_, EPOLL_CTL_MOD, c.up, &e);
      }
    }
    if (c.up < 0 || !(events & (EPOLLIN | EPOLLHUP | EPOLLERR))) return;
    char buf[65536];
    bool eof = false;
    while (true) {
      const ssize_t r = read(c.up, buf, sizeof buf);
      if (r > 0) { c.up_in.append(buf, (size_t)r); continue; }
      if (r == 0) { eof = true; break; }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      eof = true;
      break;
    }
    if (c.tunnel) {
      c.out += c.up_in;
      c.up_in.clear();
      flush(c);
    } else {
      parse_upstream(c);
    }
    if (eof) upstream_closed(c);
  }

  // one relayed response: status line + headers + (content-length | chunked -> tunnel | none)
  void parse_upstream(Conn& c) {
    while (c.up_wait && !c.up_in.empty()) {
      const size_t hend = c.up_in.find("\r\n\r\n");
      if (hend == std::string::npos) return;
      int code = 0;
      if (c.up_in.size() > 12) code = std::atoi(c.up_in.c_str() + 9);
      if (code >= 100 && code < 200) {         // interim (100 Continue): the client had its own
        c.up_in.erase(0, hend + 4);
        continue;
      }
      size_t clen = 0;
      bool has_len = false, chunked = false;
      size_t ls = c.up_in.find("\r\n") + 2;
      while (ls < hend) {
        const size_t le = c.up_in.find("\r\n", ls);
        const size_t colon = c.up_in.find(':', ls);
        if (colon != std::string::npos && colon < le) {
          const char* k = c.up_in.data() + ls;
          const size_t kn = colon - ls;
          size_t vs = colon + 1;
          while (vs < le && c.up_in[vs] == ' ') ++vs;
          if (ieq(k, kn, "content-length")) {
            clen = (size_t)std::strtoull(c.up_in.c_str() + vs, nullptr, 10);
            has_len = true;
          } else if (ieq(k, kn, "transfer-encoding")) {
            chunked = true;
          }
        }
        ls = le + 2;
      }
      const bool no_body = c.up_head || code == 204 || code == 304;
      if (chunked && !no_body) {       // streamed answer (SSE): tunnel from here on
        c.tunnel = true;
        c.up_wait = false;
        c.async = false;
        c.out += c.up_in;
        c.up_in.clear();
        c.up_out += c.in;              // anything the client already sent follows raw
        c.in.clear();
        flush_up(c);
        flush(c);
        return;
      }
      if (!has_len && !no_body) return;          // body until close (upstream_closed delivers it)
      const size_t total = hend + 4 + (no_body ? 0 : clen);
      if (c.up_in.size() < total) return;
      if (c.cache_slot >= 0) cache_done(c, code == 200 && has_len ? &c.up_in : nullptr, total);
      c.out.append(c.up_in, 0, total);
      c.up_in.erase(0, total);
      c.up_wait = false;
      c.async = false;
      c.up_used_ms = mono_ms();
      flush(c);
      if (!c.close_after) {
        parse_requests(c);                       // requests that arrived meanwhile
        if (c.out.size() > c.out_off) flush(c);
      }
    }
  }

  // One round on GPU slot g's device with that slot's model (zero-copy: records and minutes stay
  // in this reactor's portable pinned buffers).
  // Latency watchdog (SURVEY §5.3 "a watchdog on batch latency"): the round's completion event is
  // polled against the deadline instead of an unbounded stream synchronize.
  hipError_t wait_deadline(hipStream_t st, hipEvent_t ev, double deadline_ms) {
    hipError_t e = hipEventRecord(ev, st);
    if (e != hipSuccess) return e;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0;; ++i) {
      e = hipEventQuery(ev);
      if (e != hipErrorNotReady) return e;
      if (deadline_ms > 0 && (i & 15) == 15 &&
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > deadline_ms)
        return hipErrorLaunchTimeOut;
      if (i > 4096) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }

  // free the buffers of abandoned rounds whose kernels have drained (all: wait for them, bounded)
  void reap_retired(bool all) {
    for (size_t i = 0; i < retired_.size();) {
      Retired& r = retired_[i];
      (void)hipSetDevice(r.dev);
      hipError_t q = hipEventQuery(r.ev);
      if (all && q == hipErrorNotReady) {
        const auto t0 = std::chrono::steady_clock::now();
        while ((q = hipEventQuery(r.ev)) == hipErrorNotReady &&
               std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (q == hipErrorNotReady) { ++i; continue; }
      (void)hipEventDestroy(r.ev);
      if (r.st) (void)hipStreamDestroy(r.st);
      if (spare_.rec == nullptr && !all) {           // the drained set is the next spare
        spare_.rec = (EtaRecord*)r.rec;
        spare_.rec8 = (rtc::Wire8*)r.rec8;
        spare_.out = (float*)r.out;
      } else {
        (void)hipHostFree(r.rec);
        (void)hipHostFree(r.rec8);
        (void)hipHostFree(r.out);
      }
      if (r.ws) (void)hipFree(r.ws);
      retired_[i] = std::move(retired_.back());
      retired_.pop_back();
    }
    (void)hipSetDevice(cfg_.device);
  }

  // a round on `dev` missed its deadline: its kernel may still run and write this reactor's
  // buffers, so they, the stream and the workspace are retired and the round continues on fresh
  // ones (records copied over)
  // the round buffers (pinned, mapped): the spare set is allocated up front, so an abandoned round
  // swaps to it without allocating while a kernel may hang on the GPU; a drained retired set
  // becomes the next spare
  struct RoundBufs {
    EtaRecord* rec = nullptr;
    rtc::Wire8* rec8 = nullptr;
    float* out = nullptr;
  };
  RoundBufs spare_;
  bool alloc_round(RoundBufs& b) {
    const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
    if (hipHostMalloc((void**)&b.rec, (size_t)cap_ * 16, fl) == hipSuccess &&
        hipHostMalloc((void**)&b.rec8, (size_t)cap_ * 8, fl) == hipSuccess &&
        hipHostMalloc((void**)&b.out, (size_t)cap_ * 4, fl) == hipSuccess)
      return true;
    for (void* p : {(void*)b.rec, (void*)b.rec8, (void*)b.out})
      if (p) (void)hipHostFree(p);
    b = RoundBufs();
    return false;
  }

  bool retire_round(int dev, int skey, hipStream_t st, hipEvent_t ev, std::shared_ptr<const NativeModel> m) {
    if (spare_.rec == nullptr && !alloc_round(spare_)) return false;   // (the slot is quarantined anyway)
    EtaRecord* nr = spare_.rec;
    rtc::Wire8* n8 = spare_.rec8;
    float* no = spare_.out;
    void *dr = nullptr, *d8 = nullptr;
    float* dout = nullptr;
    if (hipHostGetDevicePointer(&dr, nr, 0) != hipSuccess || hipHostGetDevicePointer(&d8, n8, 0) != hipSuccess ||
        hipHostGetDevicePointer((void**)&dout, no, 0) != hipSuccess)
      return false;
    spare_ = RoundBufs();
    std::memcpy(nr, h_rec_, nrec_ * sizeof(EtaRecord));
    // an isolated (gpu_hang) stream is kept and reused: creating another hardware queue while a
    // kernel hangs on one can wait for it
    const bool keep_stream = skey < 0;
    Retired r{dev, ev, keep_stream ? nullptr : st, h_rec_, h_rec8_, h_out_, nullptr, std::move(m)};
    ModelWs& w = ws_[skey];
    r.ws = w.p;
    w.p = nullptr;
    w.bytes = 0;
    retired_.push_back(std::move(r));
    if (!keep_stream) streams_.erase(skey);
    events_.erase(skey);
    h_rec_ = nr;
    h_rec8_ = n8;
    h_out_ = no;
    d_rec_ = dr;
    d_rec8_ = d8;
    d_out_ = dout;
    if (dev == cfg_.device) stream_ = nullptr;
    return true;
  }

  hipError_t launch_on(int g, const std::shared_ptr<const NativeModel>& mp) {
    const NativeModel& m = *mp;
    Shared& sh = *cfg_.sh;
    if (sh.health[g]->fault.load(std::memory_order_relaxed)) return hipErrorLaunchFailure;   // injected
    const int dev = sh.devices[g];
    if (hipSetDevice(dev) != hipSuccess) return hipErrorInvalidDevice;
    if (!retired_.empty()) reap_retired(false);
    (void)hipSetDevice(dev);
    // a slot under the gpu_hang fault hook runs on a stream of its own (key -1 - g), on a hardware
    // queue of its own
    const bool hang = sh.health[g]->hang.load(std::memory_order_relaxed) && sh.hang_release_d != nullptr;
    const int skey = hang ? -1 - g : dev;
    hipStream_t st;
    auto it = streams_.find(skey);
    if (it == streams_.end()) {
      if ((hang ? isolated_stream(dev, &st) : hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess) {
        (void)hipSetDevice(cfg_.device);
        return hipErrorOutOfMemory;
      }
      streams_[skey] = st;
    } else {
      st = it->second;
    }
    hipEvent_t ev;
    auto ei = events_.find(skey);
    if (ei == events_.end()) {
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipSetDevice(cfg_.device);
        return hipErrorOutOfMemory;
      }
      events_[skey] = ev;
    } else {
      ev = ei->second;
    }
    sh.park(g);                        // keep a hardware queue the resident scorer may share free
    if (hang) hipLaunchKernelGGL(hang_kernel, dim3(1), dim3(64), 0, st, sh.hang_release_d, 500000000ll);   // <= 5 s
    // 8-byte wire records whenever the round is exactly representable and the model reads them
    // (csrc/runtime/rt_core.h pack_wire8), else 16-byte
    const bool w8 = m.takes_wire8() && rtc::pack_wire8(h_rec_, nrec_, h_rec8_);
    if (w8) st_.wire8.fetch_add(1, std::memory_order_relaxed);
    hipError_t e = m.predict(w8 ? d_rec8_ : d_rec_, w8 ? 8 : 16, d_out_, (int)nrec_, st, ws_[skey]);
    const auto tw = std::chrono::steady_clock::now();
    if (e == hipSuccess) e = wait_deadline(st, ev, sh.deadline_ms);
    if (sh.trace_ms >= 0) {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
      if (ms > sh.trace_ms || e == hipErrorLaunchTimeOut)
        std::fprintf(stderr, "[predict slot %d on slot %d t=%.3f] %s %.1f ms (%zu rows)\n", cfg_.slot, g,
                     std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(),
                     e == hipErrorLaunchTimeOut ? "DEADLINE after" : "wait", ms, nrec_);
    }
    if (e == hipErrorLaunchTimeOut) {
      sh.timed_out(g);
      st_.timeouts.fetch_add(1, std::memory_order_relaxed);
      if (!retire_round(dev, skey, st, ev, mp)) e = hipErrorOutOfMemory;
    }
    (void)hipSetDevice(cfg_.device);
    return e;
  }

  // Score this round: the own GPU's resident scorer, else a launch on the own GPU, else on the other
  // healthy GPUs in turn (failover), else the model's fp32 CPU forward.  false: nothing answered.
  bool score_round() {
    Shared& sh = *cfg_.sh;
    const int S = sh.slots(), own = cfg_.slot;
    auto models = sh.snapshot();       // this round keeps its models alive across a hot swap
    const NativeModel* m0 = models[own].get();
    if (m0 != nullptr && m0->mlp3_blob() != nullptr && !sh.health[own]->fault.load(std::memory_order_relaxed) &&
        !sh.health[own]->quarantined.load(std::memory_order_relaxed)) {
      std::lock_guard<std::mutex> lk(*sh.scorer_mus[own]);
      PersistentScorer* ps = sh.scorers[own];
      if (ps != nullptr && (int)nrec_ <= pscore_cap(ps) && !pscore_broken(ps)) {
        // small round: the resident kernel (no dispatch, weights already in LDS, no stream sync)
        std::memcpy(pscore_records(ps), h_rec_, nrec_ * sizeof(EtaRecord));
        if (pscore_run(ps, (int)nrec_, 200.0) == hipSuccess) {
          std::memcpy(h_out_, pscore_out(ps), nrec_ * sizeof(float));
          st_.resident.fetch_add(1, std::memory_order_relaxed);
          st_.launches.fetch_add(1, std::memory_order_relaxed);
          sh.ok(own);
          return true;
        }
        st_.fallbacks.fetch_add(1, std::memory_order_relaxed);
      }
    }
    for (int k = 0; k < S; ++k) {
      const int g = (own + k) % S;
      if (models[g] == nullptr || !sh.usable(g)) continue;
      st_.launches.fetch_add(1, std::memory_order_relaxed);
      const hipError_t e = launch_on(g, models[g]);
      if (e == hipSuccess) {
        sh.ok(g);
        if (g != own) st_.failovers.fetch_add(1, std::memory_order_relaxed);
        return true;
      }
      if (e != hipErrorLaunchTimeOut) sh.fail(g);    // (a timeout quarantined the slot already)
    }
    if (m0 != nullptr && m0->cpu_predict(h_rec_, h_out_, (int)nrec_)) {
      st_.cpu_rounds.fetch_add(1, std::memory_order_relaxed);
      return true;
    }
    return false;
  }

  void run_batch() {
    if (pending_.empty()) return;
    if (nrec_ > 0) {
      if (!score_round()) {
        std::vector<Pending> failed;
        failed.swap(pending_);
        nrec_ = 0;
        for (auto& pd : failed) {
          auto it = conns_.find(pd.fd);
          if (it == conns_.end()) continue;
          --it->second.npending;
          respond(it->second, 503, "{\"error\":\"model unavailable\"}", pd.origin, !pd.keep_alive);
          flush(it->second);
        }
        return;
      }
    }
    std::vector<Pending> done;
    done.swap(pending_);                 // respond() below may re-enter run_batch: keep it empty
    nrec_ = 0;                           // h_out_ stays valid until the next launch
    for (auto& pd : done) {
      auto it = conns_.find(pd.fd);
      if (it == conns_.end()) continue;
      --it->second.npending;
      std::string o;
      o.reserve(pd.count * 96 + 32);
      long long ok = 0;
      if (pd.batch) o += "{\"predictions\":[";
      for (size_t i = 0; i < pd.count; ++i) {
        if (i) o += ',';
        rtc::format_one(o, (double)h_out_[pd.first + i], pd.stamps[i].secs, pd.stamps[i].us,
                        pd.stamps[i].has_tz, pd.stamps[i].tz_sec, pd.errs[i]);
        ok += pd.errs[i].empty();
      }
      if (pd.batch) o += "]}";
      st_.predictions.fetch_add(ok, std::memory_order_relaxed);
      respond(it->second, 200, o, pd.origin, !pd.keep_alive);
      flush(it->second);
    }
  }

  void flush(Conn& c) {
    while (c.out_off < c.out.size()) {
      const ssize_t w = write(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off);
      if (w > 0) { c.out_off += (size_t)w; continue; }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        epoll_event e{};
        e.events = EPOLLIN | EPOLLOUT;
        e.data.fd = c.fd;
        epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &e);
        return;
      }
      to_close_.push_back(c.fd);
      return;
    }
    c.out.clear();
    c.out_off = 0;
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.fd = c.fd;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &e);
    if (c.close_after && !c.async) to_close_.push_back(c.fd);
  }
};

struct Server {
  ServerCfg cfg;
  Stats stats;
  Shared sh;
  std::atomic<bool> stop{false};
  std::vector<std::unique_ptr<Reactor>> reactors;
  std::vector<std::thread> threads;
  std::vector<std::unique_ptr<RouteService>> routes;      // one per GPU
  std::shared_mutex routes_mu;                             // guards routes_open (failover lambdas)
  bool routes_open = false;                                // set once every service exists
  std::shared_ptr<AltScorerState> alt = std::make_shared<AltScorerState>();   // "alternatives" scorer
  ~Server() {
    if (sh.hang_release) *(volatile int*)sh.hang_release = 1;   // release any gpu_hang kernel
    {
      std::unique_lock<std::shared_mutex> lk(routes_mu);     // waits out failovers in flight
      routes_open = false;
    }
    routes.clear();                                          // joins the route workers
    for (PersistentScorer* p : sh.scorers)                   // stop + wait for the resident kernels
      if (p) pscore_destroy(p);
    if (sh.hang_release) (void)hipHostFree(sh.hang_release);
  }
};

// (re)create slot g's resident scorer for its current model (mlp3 only); caller holds its mutex
void stop_scorer(Server* s, int g) {
  Shared& sh = s->sh;
  if (sh.scorers[g] != nullptr) pscore_destroy(sh.scorers[g]);   // waits for the resident kernel
  sh.scorers[g] = nullptr;
  sh.scorer_models[g] = nullptr;     // the blob it staged from may go now
}

void restart_scorer(Server* s, int g) {
  Shared& sh = s->sh;
  stop_scorer(s, g);
  if (!(s->cfg.persist_idle_ms > 0 && s->cfg.persist_cap > 0)) return;
  auto m = sh.model(g);
  if (m == nullptr || m->mlp3_blob() == nullptr) return;
  hipError_t e = hipSuccess;
  sh.scorers[g] = pscore_create(sh.devices[g], m->mlp3_blob(), m->H, *m->mlp3_norm(), s->cfg.persist_cap,
                                s->cfg.persist_idle_ms, s->cfg.persist_life_ms, &e);   // nullptr: normal launches
  if (sh.scorers[g] != nullptr) sh.scorer_models[g] = m;   // keeps the blob alive as long as the scorer
}

std::mutex g_srv_mu;
std::vector<Server*> g_servers;

}  // namespace

int64_t native_server_start(int port, int threads, const std::vector<int>& devices,
                            const std::vector<std::shared_ptr<const NativeModel>>& models, int max_batch,
                            const std::vector<std::string>& cors, bool cors_vercel, bool bind_any, int upstream_port,
                            const std::vector<RouteServiceCfg>& routes, const std::string& history_db,
                            std::string& err) {
  if (devices.empty() || devices.size() != models.size() || (!routes.empty() && routes.size() != devices.size())) {
    err = "devices/models/routes mismatch";
    return -1;
  }
  auto* s = new Server();
  s->cfg.port = port;
  s->cfg.threads = threads < 1 ? 1 : threads;
  s->cfg.max_batch = max_batch;
  s->cfg.cors_exact = cors;
  s->cfg.cors_vercel = cors_vercel;
  s->cfg.upstream_port = upstream_port;
  s->cfg.sh = &s->sh;
  s->cfg.history_db = history_db;
  if (const char* v = std::getenv("ROUTEST_PERSIST_IDLE_MS")) s->cfg.persist_idle_ms = std::atof(v);
  if (const char* v = std::getenv("ROUTEST_PERSIST_CAP")) s->cfg.persist_cap = std::atoi(v);
  if (const char* v = std::getenv("ROUTEST_PERSIST_LIFE_MS")) s->cfg.persist_life_ms = std::atof(v);
  Shared& sh = s->sh;
  if (const char* v = std::getenv("ROUTEST_QUARANTINE_AFTER")) sh.quarantine_after = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("ROUTEST_QUARANTINE_PROBE_MS")) sh.probe_ms = std::max(1ll, std::atoll(v));
  if (const char* v = std::getenv("ROUTEST_FRONT_CACHE_MS")) sh.rc_ttl_ms = std::max(0ll, std::atoll(v));
  sh.devices = devices;
  sh.models = models;
  sh.epoch = 1;
  for (size_t g = 0; g < devices.size(); ++g) {
    sh.health.push_back(std::make_unique<SlotHealth>());
    sh.scorers.push_back(nullptr);
    sh.scorer_models.push_back(nullptr);
    sh.scorer_mus.push_back(std::make_unique<std::mutex>());
  }
  if (const char* v = std::getenv("ROUTEST_GPU_DEADLINE_MS")) sh.deadline_ms = std::atof(v);
  if (const char* v = std::getenv("ROUTEST_ROUTE_TRACE_MS")) sh.trace_ms = std::atof(v);
  if (hipHostMalloc((void**)&sh.hang_release, sizeof(int), hipHostMallocMapped | hipHostMallocPortable) == hipSuccess) {
    *(volatile int*)sh.hang_release = 1;
    if (hipHostGetDevicePointer((void**)&sh.hang_release_d, sh.hang_release, 0) != hipSuccess) sh.hang_release_d = nullptr;
  } else {
    sh.hang_release = nullptr;
  }
  // ROUTEST_FAULT=gpu_fail (every slot) | gpu_fail@<slot>: launches on the slot fail (fault injection)
  if (const char* v = std::getenv("ROUTEST_FAULT")) {
    std::string f = v;
    size_t b = 0;
    while (b <= f.size()) {
      size_t e = f.find(',', b);
      if (e == std::string::npos) e = f.size();
      std::string t = f.substr(b, e - b);
      while (!t.empty() && t.front() == ' ') t.erase(t.begin());
      while (!t.empty() && t.back() == ' ') t.pop_back();
      if (t == "gpu_fail") {
        for (auto& h : sh.health) h->fault = true;
      } else if (t.rfind("gpu_fail@", 0) == 0) {
        const int g = std::atoi(t.c_str() + 9);
        if (g >= 0 && g < (int)sh.health.size()) sh.health[g]->fault = true;
      } else if (t.rfind("gpu_hang@", 0) == 0 && sh.hang_release_d) {   // the watchdog's test hook
        const int g = std::atoi(t.c_str() + 9);
        if (g >= 0 && g < (int)sh.health.size()) {
          sh.health[g]->hang = true;
          *(volatile int*)sh.hang_release = 0;
        }
      }
      b = e + 1;
    }
  }
  for (size_t g = 0; g < devices.size(); ++g) {
    std::lock_guard<std::mutex> lk(*sh.scorer_mus[g]);
    restart_scorer(s, (int)g);
  }
  // one view of the road graph for every route service's compact records and every reactor's
  // history reader (the same arrays: the services' configs point at the provider's tensors)
  if (!routes.empty() && routes[0].provider == 1 && routes[0].h_length != nullptr && routes[0].glat != nullptr) {
    auto rg = std::make_shared<rrec::RecordGraph>();
    const RouteServiceCfg& r0 = routes[0];
    rg->own_names = r0.names;
    rg->build(r0.N, r0.glat, r0.glon, r0.h_indptr, r0.h_indices, r0.h_length, r0.h_edge_name, &rg->own_names);
    if (rg->ok()) s->cfg.record_graph = rg;
  }
  for (int i = 0; i < s->cfg.threads; ++i) {
    ServerCfg rc = s->cfg;                       // reactors are spread round-robin over the GPUs
    const size_t g = (size_t)i % devices.size();
    rc.device = devices[g];
    rc.slot = (int)g;
    auto r = std::make_unique<Reactor>(rc, s->stats, s->stop);
    r->set_bind_any(bind_any);
    if (!r->init(err)) {
      delete s;
      return -1;
    }
    s->reactors.push_back(std::move(r));
  }
  // one route service per GPU; a finished job goes back to the reactor that parsed it
  s->routes.reserve(routes.size());
  for (size_t g = 0; g < routes.size(); ++g) {
    RouteServiceCfg rc = routes[g];
    rc.record_graph = s->cfg.record_graph;
    Shared* shp = &s->sh;
    const int slot = (int)g;
    rc.eta_model = [shp, slot]() { return shp->model(slot); };
    rc.park_scorer = [shp, slot]() { shp->park(slot); };
    rc.alt = s->alt;
    // watchdog: a flush past the deadline quarantines this GPU and its jobs go to the next GPU's
    // route service that is not itself broken
    rc.on_timeout = [shp, slot]() { shp->timed_out(slot); };
    rc.slot = slot;
    rc.failover = [s, slot](RouteJob* j) {
      // (shared lock: the list is published once every service exists, and ~Server closes it
      // before the services are destroyed — a late failover then relays instead of submitting
      // into a drained or deleted service)
      std::shared_lock<std::shared_mutex> lk(s->routes_mu);
      if (!s->routes_open) return false;
      const int n = (int)s->routes.size();
      if (j->hops >= n - 1) return false;      // every other service has had it: to the app
      for (int k = 1; k < n; ++k) {
        RouteService* r = s->routes[(size_t)((slot + k) % n)].get();
        if (r != nullptr && !r->broken()) {
          ++j->hops;
          if (r->submit(j)) return true;
          --j->hops;
        }
      }
      return false;
    };
    rc.hang_fault = [shp, slot]() { return shp->health[slot]->hang.load(std::memory_order_relaxed); };
    rc.hang_release_d = shp->hang_release_d;
    s->routes.push_back(std::make_unique<RouteService>(rc, [](RouteJob* j) {
      static_cast<JobTag*>(j->tag)->reactor->job_done(j);
    }));
    s->routes.back()->set_done_batch([](std::vector<RouteJob*>& js) {
      // grouped by the reactor that parsed each job (a flush's jobs come from all of them)
      std::vector<std::pair<Reactor*, std::vector<RouteJob*>>> by;
      for (RouteJob* j : js) {
        Reactor* r = static_cast<JobTag*>(j->tag)->reactor;
        auto it = std::find_if(by.begin(), by.end(), [r](const auto& p) { return p.first == r; });
        if (it == by.end()) by.push_back({r, {j}});
        else it->second.push_back(j);
      }
      for (auto& [r, v] : by) r->jobs_done(v);
    });
  }
  {
    std::unique_lock<std::shared_mutex> lk(s->routes_mu);
    s->routes_open = true;
  }
  if (!s->routes.empty())
    for (int i = 0; i < s->cfg.threads; ++i) s->reactors[i]->set_routes(s->routes[(size_t)i % devices.size()].get());
  for (auto& r : s->reactors) s->threads.emplace_back([rp = r.get()]() { rp->run(); });
  std::lock_guard<std::mutex> lk(g_srv_mu);
  g_servers.push_back(s);
  return (int64_t)g_servers.size() - 1;
}

// Hot swap: the reactors pick the new models up at their next round (rounds in flight finish on the
// old ones, which are freed with their last reference); the resident scorers restart on the new
// weights.  Returns the new epoch, or -1.
int64_t native_server_set_models(int64_t h, const std::vector<std::shared_ptr<const NativeModel>>& models,
                                 std::string& err) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  if (h < 0 || h >= (int64_t)g_servers.size() || !g_servers[h]) {
    err = "no such server";
    return -1;
  }
  Server* s = g_servers[h];
  if (models.size() != s->sh.devices.size()) {
    err = "one model per GPU slot";
    return -1;
  }
  // the resident scorers stage weights from their model's blob: stop them first (each also holds
  // its model, so a scorer can never outlive the blob), then swap, then start them on the new ones
  for (size_t g = 0; g < models.size(); ++g) {
    std::lock_guard<std::mutex> sl(*s->sh.scorer_mus[g]);
    stop_scorer(s, (int)g);
  }
  uint64_t ep;
  {
    std::lock_guard<std::mutex> ml(s->sh.model_mu);
    s->sh.models = models;
    ep = s->sh.epoch.fetch_add(1) + 1;
  }
  for (size_t g = 0; g < models.size(); ++g) {
    std::lock_guard<std::mutex> sl(*s->sh.scorer_mus[g]);
    restart_scorer(s, (int)g);
  }
  return (int64_t)ep;
}

// fault injection per slot (tests; ROUTEST_FAULT=gpu_fail@<slot> at start)
bool native_server_set_fault(int64_t h, int slot, bool on) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  if (h < 0 || h >= (int64_t)g_servers.size() || !g_servers[h]) return false;
  Server* s = g_servers[h];
  if (slot < 0 || slot >= (int)s->sh.health.size()) return false;
  s->sh.health[slot]->fault = on;
  return true;
}

// the latency watchdog's fault hook per slot: launches on it first run a kernel that waits on a
// host flag (released when no slot hangs any more, and at shutdown)
bool native_server_set_hang(int64_t h, int slot, bool on) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  if (h < 0 || h >= (int64_t)g_servers.size() || !g_servers[h]) return false;
  Server* s = g_servers[h];
  if (slot < 0 || slot >= (int)s->sh.health.size() || !s->sh.hang_release) return false;
  s->sh.health[slot]->hang = on;
  bool any = false;
  for (auto& x : s->sh.health) any |= x->hang.load();
  *(volatile int*)s->sh.hang_release = any ? 0 : 1;
  return true;
}

// the GCN scorer's node delays for "alternatives" requests (empty: none -> the app answers them)
bool native_server_set_scorer(int64_t h, std::vector<double> delay, int kind, const std::string& engine) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  if (h < 0 || h >= (int64_t)g_servers.size() || !g_servers[h]) return false;
  Server* s = g_servers[h];
  std::lock_guard<std::mutex> lk2(s->alt->mu);
  s->alt->delay = delay.empty() ? nullptr : std::make_shared<const std::vector<double>>(std::move(delay));
  s->alt->kind = kind;
  s->alt->engine = engine;
  return true;
}

// per slot: device, quarantined, consecutive failures, failures, rounds, quarantines, fault, model
std::vector<std::vector<std::string>> native_server_health(int64_t h, uint64_t& epoch) {
  std::vector<std::vector<std::string>> out;
  std::lock_guard<std::mutex> lk(g_srv_mu);
  if (h < 0 || h >= (int64_t)g_servers.size() || !g_servers[h]) return out;
  Server* s = g_servers[h];
  epoch = s->sh.epoch.load();
  auto models = s->sh.snapshot();
  for (size_t g = 0; g < s->sh.devices.size(); ++g) {
    const SlotHealth& x = *s->sh.health[g];
    out.push_back({std::to_string(s->sh.devices[g]), x.quarantined.load() ? "1" : "0", std::to_string(x.consec.load()),
                   std::to_string(x.failures.load()), std::to_string(x.rounds.load()),
                   std::to_string(x.quarantines.load()), x.fault.load() ? "1" : "0",
                   models[g] ? models[g]->describe() : std::string("none"), std::to_string(x.timeouts.load()),
                   x.hang.load() ? "1" : "0"});
  }
  return out;
}

void native_server_stop(int64_t h) {
  Server* s = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_srv_mu);
    if (h < 0 || h >= (int64_t)g_servers.size()) return;
    s = g_servers[h];
    g_servers[h] = nullptr;
  }
  if (!s) return;
  if (s->sh.hang_release) *(volatile int*)s->sh.hang_release = 1;   // release any gpu_hang kernel first
  s->stop.store(true);
  for (auto& r : s->reactors) {
    uint64_t one = 1;
    (void)!write(r->wake_fd(), &one, 8);
  }
  for (auto& t : s->threads) t.join();
  delete s;
}

std::vector<long long> native_server_stats(int64_t h) {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  if (h < 0 || h >= (int64_t)g_servers.size() || !g_servers[h]) return std::vector<long long>(41, 0);
  Server* s = g_servers[h];
  std::vector<long long> v = {s->stats.requests.load(), s->stats.predictions.load(), s->stats.launches.load(),
                              s->stats.errors.load(), s->stats.resident.load(), s->stats.fallbacks.load(),
                              s->stats.wire8.load(), s->stats.route_requests.load(),
                              s->stats.route_fallbacks.load(), s->stats.relayed.load()};
  std::vector<long long> rs(18, 0);
  for (auto& r : s->routes) {
    const auto x = r->stats();
    for (size_t i = 0; i < rs.size() && i < x.size(); ++i) rs[i] += x[i];
  }
  v.insert(v.end(), rs.begin(), rs.end());
  v.push_back(s->stats.failovers.load());
  v.push_back(s->stats.cpu_rounds.load());
  v.push_back(s->stats.history.load());
  v.push_back(s->stats.cached.load());
  std::vector<long long> rx(4, 0);        // route service stats past the first 18
  for (auto& r : s->routes) {
    const auto x = r->stats();
    for (size_t i = 0; i < rx.size() && 18 + i < x.size(); ++i) rx[i] += x[18 + i];
  }
  v.insert(v.end(), rx.begin(), rx.end());
  v.push_back(s->stats.timeouts.load());
  std::vector<long long> rr(4, 0);        // compact route records: rows, bytes; GPU-thread collect / handoff us
  for (auto& r : s->routes) {
    const auto x = r->stats();
    for (size_t i = 0; i < rr.size() && 22 + i < x.size(); ++i) rr[i] += x[22 + i];
  }
  v.insert(v.end(), rr.begin(), rr.end());
  return v;
}

}  // namespace rt
