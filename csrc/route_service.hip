// Native route service: /api/optimize_route, /route and /api/request_route answered without Python
// (reference RO/Flaskr/routes.py:29-50,89-127 -> RO/Flaskr/utils.py:10-201; Python equivalent
// routest_amd/routing/route_batcher.py + optimizer.py + api/app.py _optimize).
//
// One worker thread per GPU pulls the requests the native front end's reactors parsed off their
// sockets, and flushes them together (batch_max requests or timeout_us after the first):
//   1. parse + validate every request (csrc/runtime/route_core.h RouteReq; unusual inputs are
//      handed back for the Python app);
//   2. ONE K5 + ONE K6 launch for every multi-stop request of the flush (csrc/route_kernels.hip);
//      only the trips and, for infeasible requests, the depot row of D come back to the host;
//   3. road-graph provider: every waypoint snapped (NodeGrid), the flush's unique legs searched on
//      the CCH (csrc/cch.hip, under each request's routing context) or by the batched A*
//      (csrc/astar.hip), and the found paths COMPACTED on the GPU into one flat array before the
//      copy-out (a leg row is max_path ints; a path is ~200);
//   4. responses assembled on the assembly thread (route_core.h: byte-identical to the FastAPI
//      handler) while the GPU stage runs the next flush;
//   5. use_ml_eta: one fused featurize+MLP launch (K1+K2) for the flush's ETA records;
//   6. persistence of /api/optimize_route results on a thread of its own: every flush waiting is
//      group-committed in one SQLite transaction into the database file the Python store reads
//      (reference routes.py:119-125, best effort); WAL checkpoints run on a fourth thread;
//   7. completed jobs go back to their reactors (eventfd wake-up), which write the bytes -- a
//      persisted job only after its commit.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <list>
#include <mutex>
#include <queue>
#include <random>
#include <memory>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>

#include "common.h"
#include "ops.h"
#include "route_service.h"
#include "runtime/alternatives.h"
#include "runtime/sqlite_lite.h"

namespace rt {

namespace {

// one block per found path: copy its nodes from the (Q, max_path) rows into the flat array
__global__ void compact_paths_kernel(const int* __restrict__ rows, int max_path, const int* __restrict__ len,
                                     const int* __restrict__ status, const long long* __restrict__ off, int Q,
                                     int* __restrict__ flat) {
  const int q = blockIdx.x;
  if (q >= Q || status[q] != 0) return;
  const int n = min(len[q], max_path);
  const long long o = off[q];
  for (int i = threadIdx.x; i < n; i += blockDim.x) flat[o + i] = rows[(size_t)q * max_path + i];
}

// the watchdog's fault hook (ROUTEST_FAULT=gpu_hang@<slot>): one wave waiting on a host flag, at
// most max_ticks of the 100 MHz wall clock; reads only, every wave reaches the exit condition
__global__ __launch_bounds__(64) void route_hang_kernel(const int* release, long long max_ticks) {
  const long long t0 = wall_clock64();
  // (also bounded by iterations: ~3.4 us per sleep at 2.4 GHz, 2M of them ~7 s, whatever the
  // wall clock's rate)
  for (int it = 0; it < 2000000 && __hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
                   wall_clock64() - t0 < max_ticks;
       ++it)
    __builtin_amdgcn_s_sleep(127);
}

// Queue-local copies: the flush's host <-> device transfers run as a small kernel on the flush's own
// stream (mapped pinned host memory, read / written by the GPU over PCIe) instead of on the copy
// engines.  The SDMA queues are shared by every stream of the process: a copy queued behind a
// kernel that never finishes (a hung GPU slot; the watchdog rehearsal's gpu_hang hook) blocked the
// OTHER slot's copies behind it for the hang's whole duration (r6 trace: the healthy slot's matrix
// stage missed its 300 ms deadline waiting on its own tiny H2D copies).  On the compute queue a
// flush's copies wait only for its own stream.  16-byte vector body, byte tail; 2-D for the depot rows.
__global__ __launch_bounds__(256) void route_copy_kernel(unsigned char* __restrict__ dst,
                                                         const unsigned char* __restrict__ src, size_t bytes) {
  const size_t nv = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0 ? bytes / 16 : 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride)
    reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(src)[i];
  for (size_t i = nv * 16 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < bytes; i += stride) dst[i] = src[i];
}
__global__ __launch_bounds__(256) void route_copy2d_kernel(unsigned char* __restrict__ dst, size_t dpitch,
                                                           const unsigned char* __restrict__ src, size_t spitch,
                                                           size_t width, size_t height) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < width * height; i += stride) {
    const size_t r = i / width, c = i - r * width;
    dst[r * dpitch + c] = src[r * spitch + c];
  }
}
std::atomic<bool>& qcopy_same_va() {
  static std::atomic<bool> ok{true};
  return ok;
}
hipError_t qcopy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  if (!qcopy_same_va().load(std::memory_order_relaxed)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s);
  const size_t blocks = std::min<size_t>(1024, (bytes / 16 + 255) / 256 + 1);
  hipLaunchKernelGGL(route_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (unsigned char*)dst,
                     (const unsigned char*)src, bytes);
  return hipGetLastError();
}
hipError_t qcopy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                   hipStream_t s) {
  if (width == 0 || height == 0) return hipSuccess;
  if (!qcopy_same_va().load(std::memory_order_relaxed))
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDefault, s);
  const size_t blocks = std::min<size_t>(1024, (width * height + 255) / 256);
  hipLaunchKernelGGL(route_copy2d_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (unsigned char*)dst, dpitch,
                     (const unsigned char*)src, spitch, width, height);
  return hipGetLastError();
}

// Growable buffers of the service's flushes.  A buffer outgrown while serving is not freed at
// once: hipFree / hipHostFree wait for the whole device, i.e. for every other service's and
// reactor's kernels on this GPU (a hung one included) — it is kept until the service ends (the
// geometric growth bounds the extra memory by the final size).
template <class T>
struct DevBuf {
  T* d = nullptr;
  size_t n = 0;
  std::vector<T*> old;
  hipError_t need(size_t k) {
    if (k <= n) return hipSuccess;
    const size_t m = std::max(k, n * 3 / 2);
    if (d) old.push_back(d);
    d = nullptr;
    n = 0;
    hipError_t e = hipMalloc((void**)&d, m * sizeof(T));
    if (e == hipSuccess) n = m;
    return e;
  }
  ~DevBuf() {
    if (d) (void)hipFree(d);
    for (T* p : old) (void)hipFree(p);
  }
};
template <class T>
struct HostBuf {
  T* h = nullptr;
  size_t n = 0;
  std::vector<T*> old;
  hipError_t need(size_t k) {
    if (k <= n) return hipSuccess;
    const size_t m = std::max(k, n * 3 / 2);
    if (h) old.push_back(h);
    h = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc((void**)&h, m * sizeof(T), hipHostMallocMapped | hipHostMallocPortable);
    if (e == hipSuccess) {
      n = m;
      void* dp = nullptr;      // the GPU sees it at the same address (qcopy); else copies take the DMA path
      if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess || dp != (void*)h) qcopy_same_va().store(false);
    }
    return e;
  }
  ~HostBuf() {
    if (h) (void)hipHostFree(h);
    for (T* p : old) (void)hipHostFree(p);
  }
};

inline rtc::Stamp local_now(int64_t skew_s = 0) {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  struct tm lt;
  time_t t = ts.tv_sec + (time_t)skew_s;
  localtime_r(&t, &lt);
  rtc::Stamp s;
  s.secs = rtc::days_from_civil(lt.tm_year + 1900, (unsigned)lt.tm_mon + 1, (unsigned)lt.tm_mday) * 86400 +
           lt.tm_hour * 3600 + lt.tm_min * 60 + lt.tm_sec;
  s.us = (int32_t)(ts.tv_nsec / 1000);
  return s;
}

// datetime.now(timezone.utc).isoformat() (store.py _now_iso)
inline std::string utc_now_iso() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  rtc::Stamp tz;
  tz.has_tz = true;
  tz.tz_sec = 0;
  return rtc::isoformat((int64_t)ts.tv_sec, ts.tv_nsec / 1000, tz);
}

// Row ids of the persisted requests/results: time-ordered UUIDs (RFC 9562 version 7: 48-bit Unix
// milliseconds, a 12-bit sequence within the millisecond, 62 random bits).  Both tables are keyed
// by TEXT ids with B-tree indexes (and route_results by request_id too): random v4 ids dirtied one
// random index leaf per row per index in every group commit, time-ordered ones append — the same
// opaque 36-character ids to every client (the reference's are Postgres v4 uuids).
struct RowId {
  std::mt19937_64 g{std::random_device{}() ^ ((uint64_t)std::random_device{}() << 32)};
  uint64_t last_ms = 0;
  uint32_t seq = 0;
  std::string next() {
    uint64_t ms = (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                      std::chrono::system_clock::now().time_since_epoch())
                      .count();
    if (ms <= last_ms) {                // same (or an earlier) millisecond: keep the order
      ms = last_ms;
      if (++seq > 0xFFF) {
        ++ms;
        seq = 0;
      }
    } else {
      seq = (uint32_t)(g() & 0x3FF);    // a random start, room to count up in the millisecond
    }
    last_ms = ms;
    const uint64_t a = (ms << 16) | 0x7000ULL | (seq & 0xFFF);                       // version 7
    const uint64_t b = (g() & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;        // variant 10
    char s[37];
    std::snprintf(s, sizeof s, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xFFFF),
                  (unsigned)(a & 0xFFFF), (unsigned)(b >> 48), (unsigned long long)(b & 0xFFFFFFFFFFFFULL));
    return s;
  }
};

// Exact host search for the rare leg both GPU stages gave up on (graph.py _exact_fallback):
// Dijkstra from s stopping when t is settled.
bool host_dijkstra(const int* indptr, const int* indices, const float* cost, int N, int s, int t, int max_path,
                   float& out_cost, std::vector<int32_t>& path) {
  std::vector<double> dist((size_t)N, INFINITY);
  std::vector<int32_t> par((size_t)N, -1);
  using QE = std::pair<double, int>;
  std::priority_queue<QE, std::vector<QE>, std::greater<QE>> pq;
  dist[s] = 0.0;
  pq.push({0.0, s});
  while (!pq.empty()) {
    auto [d, v] = pq.top();
    pq.pop();
    if (d > dist[v]) continue;
    if (v == t) break;
    for (int e = indptr[v]; e < indptr[v + 1]; ++e) {
      const int w = indices[e];
      const double nd = d + (double)cost[e];
      if (nd < dist[w]) {
        dist[w] = nd;
        par[w] = v;
        pq.push({nd, w});
      }
    }
  }
  if (!std::isfinite(dist[t])) return false;
  path.clear();
  for (int v = t; v != -1; v = par[v]) {
    path.push_back(v);
    if ((int)path.size() > max_path) return false;
    if (v == s) break;
  }
  std::reverse(path.begin(), path.end());
  out_cost = (float)dist[t];
  return true;
}

}  // namespace

// One flush in flight between the two stages: its jobs and the legs its responses are built from.
struct Batch {
  std::vector<RouteJob*> jobs;
  std::vector<std::shared_ptr<CchMetricDev>> metrics;   // per routing-context group (CCH)
  std::vector<std::shared_ptr<const std::vector<float>>> host_cost;   // their edge costs on the host
  std::vector<rtr::Leg> legs;
  std::vector<std::vector<int32_t>> host_paths;
  std::vector<int32_t> flat;                 // found paths, compacted (Leg::path points in here)
  std::vector<int32_t> flat_e;               // their hop edges (CCH; Leg::edges points in here)
  std::unordered_map<uint64_t, int> leg_index;
  bool failed = false;
  // "alternatives" jobs of the flush: the scorer snapshot they use
  std::shared_ptr<const std::vector<double>> alt_delay;
  int alt_kind = 0;
  std::string alt_engine;
  std::vector<RouteJob*> save;               // jobs whose rows the persistence thread writes
};

inline double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct RouteService::Impl {
  RouteServiceCfg cfg;
  std::function<void(RouteJob*)> done;
  // chunks per parallel_chunks call: cfg.chunk_threads, a 1/k share of the process's CPU pool when
  // k route services run per GPU (profiles/route_pipelines_r6ax.md: two services' full fan-outs
  // oversubscribed the box's CPU share and raised the no-store p99 from 15 to 34 ms)
  unsigned chunk_threads() const { return (unsigned)(cfg.chunk_threads < 1 ? 1 : cfg.chunk_threads); }
  std::function<void(std::vector<RouteJob*>&)> done_many;
  void done_all(std::vector<RouteJob*>& js) {
    if (js.empty()) return;
    if (done_many) {
      done_many(js);
    } else {
      for (RouteJob* j : js) done(j);
    }
  }
  std::mutex mu;
  std::condition_variable cv;
  std::deque<RouteJob*> q;
  bool stop = false;
  std::thread th, th_asm;
  hipStream_t stream{}, stream_asm{};
  rtr::NodeGrid grid;
  // GPU stage -> assembly stage hand-off (at most 2 flushes waiting: the GPU runs ahead by one)
  std::mutex amu;
  std::condition_variable acv;
  std::deque<Batch*> aq;
  bool gpu_done = false;
  // statistics
  std::atomic<long long> n_legs_reused{0};
  std::atomic<long long> n_jobs{0}, n_flushes{0}, n_fallback{0}, n_legs{0}, n_host_legs{0}, n_persisted{0},
      n_escalated{0};
  // stage times (us): parse, trips (K5+K6), snap, A*, copy-out, assembly, ETA, persistence
  std::atomic<long long> t_stage[8] = {};
  // GPU thread waits (us): collecting a flush after its first job, handing it to a full assembly queue
  std::atomic<long long> t_collect_us{0}, t_handoff_us{0};
  void add_t(int k, double t0) {
    const long long dt = (long long)(now_us() - t0);
    t_stage[k].fetch_add(dt, std::memory_order_relaxed);
    if (trace_ms >= 0 && dt > trace_ms * 1e3) {   // a stage that alone outlasts the trace threshold
      static const char* const names[8] = {"parse", "trips", "snap", "astar", "copyout", "assemble", "eta", "persist"};
      trace("stage %s took %.1f ms", names[k], dt * 1e-3);
    }
  }
  // K5 / K6 buffers
  HostBuf<double> h_lat, h_lon, h_dem, h_cap, h_maxd, h_row0;
  HostBuf<int> h_npts, h_visit, h_trip, h_ntrips, h_status;
  DevBuf<double> d_lat, d_lon, d_dem, d_cap, d_maxd, d_D;
  DevBuf<int> d_npts, d_visit, d_trip, d_ntrips, d_status;
  // A* buffers
  HostBuf<int> h_src, h_dst, h_len, h_st, h_qidx, h_flat, h_flat_e;
  HostBuf<float> h_cost;
  HostBuf<long long> h_off;
  DevBuf<int> d_src, d_dst, d_len, d_st, d_path, d_qidx, d_flat, d_iters, d_edge, d_flat_e;
  DevBuf<float> d_cost;
  DevBuf<long long> d_off;
  // CCH
  CchScratch csc;
  // the matrix stage's chains (kept for the multi-stop legs), the tag of its matrix call and each
  // multi-stop job's row in it; the flush's metrics as device views (one per context group) and the
  // group of every request row / leg, so ONE launch sequence serves all the flush's contexts
  CchScratch msc;
  uint64_t mtag = 0;
  std::unordered_map<const RouteJob*, int> jrow;
  HostBuf<CchMView> h_mv;
  DevBuf<CchMView> d_mv;
  HostBuf<int> h_rowg, h_lgrp;
  DevBuf<int> d_rowg, d_lgrp;
  HostBuf<int> h_lr, h_li, h_lj;
  DevBuf<int> d_lr, d_li, d_lj;
  HostBuf<int> h_pts, h_npts2;
  HostBuf<float> h_met;
  DevBuf<int> d_pts, d_npts2;
  DevBuf<float> d_msec, d_mmet, d_met;
  // host copies of metrics' edge costs (maneuver durations, exact host fallback): LRU by key
  std::mutex hc_mu;
  HostBuf<float> h_hcost;                  // pinned staging of host_costs' copy
  std::list<std::pair<uint64_t, std::shared_ptr<const std::vector<float>>>> hc_lru;
  std::unordered_map<uint64_t, decltype(hc_lru)::iterator> hc_index;
  static constexpr size_t HC_MAX = 64;
  std::atomic<long long> n_ctx_built{0};
  std::atomic<long long> t_ctx_us{0};
  // Routing contexts off the flush's critical path (CCH): a job whose context is not customized
  // yet waits here while the router's background builder customizes it; the rest of its flush
  // proceeds.  The build's listener puts the jobs back at the head of the queue.
  bool async_ctx = true;
  int listener = 0;
  std::mutex wmu;
  std::unordered_map<uint64_t, std::vector<RouteJob*>> waiting;
  std::atomic<long long> n_deferred{0}, t_wait_us{0}, n_prefetch{0};
  // latency watchdog: every wait on the flush's GPU work is bounded (ROUTEST_ROUTE_DEADLINE_MS)
  double deadline_ms = 2000.0;
  // the deadline of the current flush's waits: deadline_ms scaled with its work (a healthy
  // flush of oversized requests — NM up to 4096 stops, or a context built synchronously — must not
  // read as a hung GPU and quarantine the slot)
  std::atomic<double> flush_deadline_ms{2000.0};
  std::atomic<bool> broken{false};
  hipEvent_t ev_gpu{}, ev_asm{};
  hipStream_t hang_stream{};              // the gpu_hang fault hook's stream (own hardware queue)
  std::atomic<long long> n_failed_over{0};
  std::atomic<long long> n_records{0}, n_record_bytes{0};
  bool fail_fault = false;                 // ROUTEST_FAULT=route_fail (test hook)

  // ROUTEST_ROUTE_TRACE_MS=<ms>: every wait on the GPU longer than that, every deadline, hand-off and
  // recovery is logged to stderr with the slot and a steady-clock time stamp (the watchdog rehearsal's
  // timeline: which wait of which slot stalled, and on what)
  double trace_ms = -1.0;
  void trace(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
    if (trace_ms < 0) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    std::fprintf(stderr, "[route slot %d t=%.3f] %s\n", cfg.slot,
                 std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(), buf);
  }
  hipError_t sync(hipStream_t s, hipEvent_t ev, const char* what = "") {
    hipError_t e = hipEventRecord(ev, s);
    if (e != hipSuccess) return e;
    const auto t0 = std::chrono::steady_clock::now();
    auto waited = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    for (int i = 0;; ++i) {
      e = hipEventQuery(ev);
      if (e != hipErrorNotReady) {
        if (trace_ms >= 0 && waited() > trace_ms) trace("wait %s %.1f ms", what, waited());
        return e;
      }
      const double dl = flush_deadline_ms.load(std::memory_order_relaxed);
      if (dl > 0 && (i & 15) == 15 && waited() > dl) {
        trace("DEADLINE in %s after %.1f ms", what, waited());
        if (!broken.exchange(true) && cfg.on_timeout) cfg.on_timeout();
        return hipErrorLaunchTimeOut;
      }
      if (i > 4096) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  // the work that missed the deadline has drained: the service's buffers are its own again
  bool drained() {
    return (!ev_gpu || hipEventQuery(ev_gpu) != hipErrorNotReady) && (!ev_asm || hipEventQuery(ev_asm) != hipErrorNotReady);
  }
  // jobs of a failed / abandoned flush: to another GPU's route service, else relayed to the app
  void hand_off(std::vector<RouteJob*>& jobs) {
    for (RouteJob* j : jobs) {
      if (!j->fallback && !j->status && cfg.failover) {
        j->plan = rtr::Plan();
        j->calls.clear();
        j->nodes.clear();
        j->group = 0;
        j->alt_pairs.clear();
        j->alt_vias.clear();
        j->alt_legs.clear();
        j->alt_paths.clear();
        j->alt_edges.clear();
        j->alt_json.clear();
        j->asmb = rtr::Assembled();
        if (cfg.failover(j)) {
          n_failed_over.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        trace("no other route service takes the job (hops %d): relayed to the app", j->hops);
      }
      if (!j->status) j->fallback = true;
      finish(j);
      done(j);
    }
    jobs.clear();
  }
  // prefetch of the next week-hour: (weather, congestion) of requests routed at "now" -> last seen
  std::unordered_map<int, double> seen_now;
  int prefetched_wh = -1;
  int64_t clock_skew_s = 0;
  std::unordered_set<int> prefetched;      // pairs already queued for prefetched_wh
  int prefetch_min = 10;
  // ETA
  HostBuf<rtc::EtaRecord> h_rec;
  HostBuf<float> h_eta;
  ModelWs eta_ws;
  DevBuf<rtc::EtaRecord> d_rec;
  DevBuf<float> d_eta;
  // store
  rtsql::Api sql;
  void* db = nullptr;
  void* st_req = nullptr;
  void* st_res = nullptr;
  void *st_begin = nullptr, *st_commit = nullptr, *st_rollback = nullptr, *st_undo = nullptr;
  RowId uuid;
  // assembly -> persistence hand-off (group commit) and the background WAL checkpointer
  std::thread th_persist, th_ckpt;
  std::mutex pmu;
  std::condition_variable pcv;
  std::deque<std::vector<RouteJob*>> pq;
  bool asm_done = false;
  std::mutex cmu;
  std::condition_variable ccv;
  long long commits = 0;
  bool ck_stop = false;

  rtr::CoordCache coord_cache;             // graph nodes' "[lon,lat]" strings (graph provider)
  std::vector<double> edge_heading;        // per road edge: rtr::hop_heading (graph provider)
  // compact route records (runtime/route_record.h): the graph view persisted rows are encoded
  // against — the server's shared one, or this service's own over the tables above
  std::shared_ptr<const rrec::RecordGraph> rg;
  const rtr::CoordCache* ccache() const {
    if (rg) return rg->cc;
    return coord_cache.ofs.empty() ? nullptr : &coord_cache;
  }
  const double* headings() const {
    if (rg) return rg->heading;
    return edge_heading.empty() ? nullptr : edge_heading.data();
  }

  void open_store() {
    if (cfg.sqlite_path.empty()) return;
    std::string err;
    if (!sql.load(err)) return;
    if (sql.open_v2(cfg.sqlite_path.c_str(), &db, rtsql::OPEN_READWRITE | rtsql::OPEN_URI | rtsql::OPEN_NOMUTEX,
                    nullptr) != rtsql::OK) {
      if (db) sql.close(db);
      db = nullptr;
      return;
    }
    sql.wait_on_locks(db);
    sql.exec(db, "PRAGMA journal_mode=WAL", nullptr, nullptr, nullptr);
    // WAL + NORMAL: a commit appends to the WAL without an fsync (the WAL is synced at checkpoints);
    // FULL would fsync every flush's commit
    sql.exec(db, "PRAGMA synchronous=NORMAL", nullptr, nullptr, nullptr);
    // no foreign-key checks on THIS connection: it inserts each result right after its request in
    // one transaction, so the reference holds by construction and the parent lookup per result row
    // is pure cost; deletes (ON DELETE CASCADE) happen on the app's / history reader's connections,
    // which enforce the keys
    sql.exec(db, "PRAGMA foreign_keys=OFF", nullptr, nullptr, nullptr);
    sql.exec(db, "PRAGMA cache_size=-65536", nullptr, nullptr, nullptr);       // 64 MB page cache
    sql.exec(db, "PRAGMA wal_autocheckpoint=0", nullptr, nullptr, nullptr);   // ckpt_loop checkpoints
    sql.exec(db, "PRAGMA temp_store=MEMORY", nullptr, nullptr, nullptr);      // statement journals in RAM
    const char* q1 = "INSERT INTO route_requests(id,origin_id,stops,request_time,status,engine,vehicle_id,driver_age)"
                     " VALUES(?,?,?,?,?,?,?,?)";
    const char* q2 = "INSERT INTO route_results(id,request_id,optimized_order,total_distance,total_duration,legs,"
                     "geometry,eta_minutes_ml,eta_completion_time_ml,created_at) VALUES(?,?,?,?,?,?,?,?,?,?)";
    const std::pair<const char*, void**> stmts[] = {
        {q1, &st_req},         {q2, &st_res},          {"BEGIN", &st_begin}, {"COMMIT", &st_commit},
        {"ROLLBACK", &st_rollback}, {"DELETE FROM route_requests WHERE id=?", &st_undo}};
    bool ok = true;
    for (const auto& [text, st] : stmts) ok = ok && sql.prepare_v2(db, text, -1, st, nullptr) == rtsql::OK;
    if (!ok) {
      for (const auto& [text, st] : stmts) {
        if (*st) sql.finalize(*st);
        *st = nullptr;
      }
      sql.close(db);
      db = nullptr;
    }
  }

  // bind a JSON value like Python's sqlite3 adapter binds the corresponding object; false for
  // objects sqlite3 cannot bind (list / dict raise -> the persist fails, best effort)
  bool bind_value(void* st, int i, const rtj::Value* v) {
    if (!v || v->kind == rtj::Value::Null) return sql.bind_null(st, i) == rtsql::OK;
    switch (v->kind) {
      case rtj::Value::Bool: return sql.bind_int64(st, i, v->b ? 1 : 0) == rtsql::OK;
      case rtj::Value::Str: return sql.bind_text(st, i, v->str.data(), (int)v->str.size(), rtsql::TRANSIENT) == rtsql::OK;
      case rtj::Value::Num:
        if (v->is_int && std::fabs(v->num) < 9.0e15) return sql.bind_int64(st, i, (long long)v->num) == rtsql::OK;
        return sql.bind_double(st, i, v->num) == rtsql::OK;
      default: return false;
    }
  }
  // SQLITE_STATIC: every bound string outlives its statement's step (the row texts of a route are
  // ~100 KB of GeoJSON; a transient binding copied each once more)
  bool bind_text(void* st, int i, const std::string& s) {
    return sql.bind_text(st, i, s.data(), (int)s.size(), rtsql::STATIC) == rtsql::OK;
  }
  bool bind_text(void* st, int i, const char* literal) {      // string literals only (static storage)
    return sql.bind_text(st, i, literal, (int)std::strlen(literal), rtsql::STATIC) == rtsql::OK;
  }
  bool bind_text(void* st, int i, std::string&&) = delete;    // a temporary would dangle

  // the row texts of a job (store.py build_rows): the stops JSON and, for a route without a compact
  // record, the geometry object — built on the assembly stage's threads, so the single persistence
  // thread (SQLite's one writer) only binds and steps.  A graph route's legs and geometry are its
  // record (j->rec, encoded in assemble_all): ~1-3 KB instead of ~37 KB of text, rebuilt
  // byte-identically by the history readers.  false: a meta / stops shape the Python adapter would
  // refuse (persist fails)
  static bool prep_persist(RouteJob* j) {
    const rtj::Value* root = j->req.root;
    const rtj::Value* meta = root->get("meta");
    if (meta && meta->truthy() && meta->kind != rtj::Value::Obj) return false;   // .get on a non-dict
    if (meta && !meta->truthy()) meta = nullptr;
    std::string& stops = j->p_stops;
    stops = "{\"destination_ids\":";
    const rtj::Value* ids = meta ? meta->get("destination_ids") : nullptr;
    if (ids && ids->truthy()) { if (!rtr::put_value(stops, *ids)) return false; }
    else stops += "[]";
    stops += ",\"destination_points\":";
    if (!rtr::put_value(stops, *root->get("destination_points"))) return false;
    stops += '}';
    std::string& geom = j->p_geom;
    geom.clear();
    if (j->rec.empty()) {
      geom.reserve(j->asmb.coords.size() + 40);
      geom = "{\"type\":\"LineString\",\"coordinates\":";
      geom += j->asmb.coords;
      geom += '}';
    }
    j->p_ok = true;
    return true;
  }

  // one request row at parameter offset b (route_requests: 8 columns) / its result row (10)
  bool bind_req_row(void* st, int b, RouteJob* j, const std::string& rid, const std::string& now) {
    const rtj::Value* root = j->req.root;
    const rtj::Value* meta = root->get("meta");
    if (meta && !meta->truthy()) meta = nullptr;
    const rtj::Value* drv = root->get("driver_details");
    if (drv && !drv->truthy()) drv = nullptr;
    const rtj::Value* ue = root->get("use_ml_eta");
    return bind_text(st, b + 1, rid) && bind_value(st, b + 2, meta ? meta->get("origin_id") : nullptr) &&
           bind_text(st, b + 3, j->p_stops) && bind_text(st, b + 4, now) && bind_text(st, b + 5, "completed") &&
           bind_text(st, b + 6, (ue && ue->truthy()) ? "ml" : "default") &&
           bind_value(st, b + 7, drv ? drv->get("driver_name") : nullptr) &&
           bind_value(st, b + 8, drv ? drv->get("driver_age") : nullptr);
  }
  bool bind_res_row(void* st, int b, RouteJob* j, const std::string& rid, const std::string& res_id,
                    const std::string& now) {
    const rtr::Assembled& a = j->asmb;
    bool ok = bind_text(st, b + 1, res_id) && bind_text(st, b + 2, rid) && bind_text(st, b + 3, a.order) &&
              sql.bind_double(st, b + 4, rtr::py_round(a.dist, 2)) == rtsql::OK &&
              sql.bind_double(st, b + 5, rtr::py_round(a.dur, 2)) == rtsql::OK &&
              (j->rec.empty() ? bind_text(st, b + 6, a.segments) && bind_text(st, b + 7, j->p_geom)
                              : sql.bind_blob(st, b + 6, j->rec.data(), (int)j->rec.size(), rtsql::STATIC) == rtsql::OK &&
                                    sql.bind_null(st, b + 7) == rtsql::OK);
    if (ok && !j->eta_iso.empty()) {
      ok = sql.bind_double(st, b + 8, (double)j->eta_min) == rtsql::OK && bind_text(st, b + 9, j->eta_iso);
    } else if (ok) {
      ok = sql.bind_null(st, b + 8) == rtsql::OK && sql.bind_null(st, b + 9) == rtsql::OK;
    }
    return ok && bind_text(st, b + 10, now);
  }

  std::string persist_one(RouteJob* j, const std::string& now) {
    if (!j->p_ok) return "";
    const std::string rid = uuid.next();
    sql.reset(st_req);
    sql.clear_bindings(st_req);
    if (!bind_req_row(st_req, 0, j, rid, now) || sql.step(st_req) != rtsql::DONE) {
      sql.reset(st_req);
      return "";
    }
    sql.reset(st_req);
    sql.reset(st_res);
    sql.clear_bindings(st_res);
    const std::string res_id = uuid.next();
    if (!bind_res_row(st_res, 0, j, rid, res_id, now) || sql.step(st_res) != rtsql::DONE) {
      // per-request semantics of SQLiteStore without a savepoint per request (a savepoint's
      // statement journal copied every page the request touched: 2x the row cost): a failed
      // result insert removes the request row it belongs to; a failed statement itself is
      // atomic, so a failed request insert left nothing behind
      sql.reset(st_res);
      undo_request(rid);
      return "";
    }
    sql.reset(st_res);
    return rid;
  }
  void undo_request(const std::string& rid) {
    sql.reset(st_undo);
    sql.clear_bindings(st_undo);
    if (bind_text(st_undo, 1, rid)) (void)sql.step(st_undo);
    sql.reset(st_undo);
  }

  // Multi-row INSERTs: n requests' rows in one statement per table (prepared on first use per n).
  // SQLite's per-statement work (VM start, cursor seek to the tables' and indexes' right edges —
  // the time-ordered ids append) is paid once per n rows instead of once per row.
  std::unordered_map<int, std::pair<void*, void*>> st_multi;
  std::pair<void*, void*> multi_stmts(int n) {
    auto it = st_multi.find(n);
    if (it != st_multi.end()) return it->second;
    std::string q1 = "INSERT INTO route_requests(id,origin_id,stops,request_time,status,engine,vehicle_id,driver_age) VALUES";
    std::string q2 = "INSERT INTO route_results(id,request_id,optimized_order,total_distance,total_duration,legs,"
                     "geometry,eta_minutes_ml,eta_completion_time_ml,created_at) VALUES";
    for (int k = 0; k < n; ++k) {
      q1 += k ? ",(?,?,?,?,?,?,?,?)" : "(?,?,?,?,?,?,?,?)";
      q2 += k ? ",(?,?,?,?,?,?,?,?,?,?)" : "(?,?,?,?,?,?,?,?,?,?)";
    }
    void *a = nullptr, *b = nullptr;
    if (sql.prepare_v2(db, q1.c_str(), -1, &a, nullptr) != rtsql::OK ||
        sql.prepare_v2(db, q2.c_str(), -1, &b, nullptr) != rtsql::OK) {
      if (a) sql.finalize(a);
      if (b) sql.finalize(b);
      a = b = nullptr;
    }
    st_multi[n] = {a, b};
    return {a, b};
  }
  static constexpr int MULTI_ROWS = 32;
  // rows of `js` (all p_ok) in multi-row statements; a chunk whose statement fails is redone row by
  // row (a failed statement inserts nothing; a failed results statement removes its requests first)
  void persist_chunked(std::vector<RouteJob*>& js, const std::string& now) {
    std::vector<std::string> rids, resids;
    for (size_t i = 0; i < js.size(); i += MULTI_ROWS) {
      const int n = (int)std::min<size_t>(MULTI_ROWS, js.size() - i);
      auto one_by_one = [&] {
        for (int k = 0; k < n; ++k) js[i + k]->request_id = persist_one(js[i + k], now);
      };
      const auto [sq, sr] = n >= 4 ? multi_stmts(n) : std::pair<void*, void*>{nullptr, nullptr};
      if (sq == nullptr || sr == nullptr) {
        one_by_one();
        continue;
      }
      rids.assign(n, std::string());
      resids.assign(n, std::string());
      bool ok = true;
      sql.reset(sq);
      for (int k = 0; k < n && ok; ++k) {
        rids[k] = uuid.next();
        ok = bind_req_row(sq, 8 * k, js[i + k], rids[k], now);
      }
      ok = ok && sql.step(sq) == rtsql::DONE;
      sql.reset(sq);
      if (!ok) {
        one_by_one();
        continue;
      }
      sql.reset(sr);
      for (int k = 0; k < n && ok; ++k) {
        resids[k] = uuid.next();
        ok = bind_res_row(sr, 10 * k, js[i + k], rids[k], resids[k], now);
      }
      ok = ok && sql.step(sr) == rtsql::DONE;
      sql.reset(sr);
      if (!ok) {
        for (int k = 0; k < n; ++k) undo_request(rids[k]);
        one_by_one();
        continue;
      }
      for (int k = 0; k < n; ++k) js[i + k]->request_id = rids[k];
    }
  }

  void run() {
    if (hipSetDevice(cfg.device) != hipSuccess) return;
    // the query stream at the highest priority: the router's background context builds (lowest
    // priority, csrc/cch.hip builder_loop) never delay a flush's launches
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, greatest) != hipSuccess) {
      (void)hipGetLastError();
      if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return;
    }
    if (const char* v = std::getenv("ROUTEST_CCH_ASYNC")) async_ctx = std::string(v) != "0";
    if (const char* v = std::getenv("ROUTEST_ROUTE_DEADLINE_MS")) deadline_ms = std::atof(v);
    flush_deadline_ms.store(deadline_ms);
    if (const char* v = std::getenv("ROUTEST_ROUTE_TRACE_MS")) trace_ms = std::atof(v);
    // ROUTEST_FAULT=route_fail: every flush of every service fails (not a timeout) — the hop limit
    // of the failover must end each job at the app
    if (const char* v = std::getenv("ROUTEST_FAULT")) fail_fault = std::string(v).find("route_fail") != std::string::npos;
    if (hipEventCreateWithFlags(&ev_gpu, hipEventDisableTiming) != hipSuccess) ev_gpu = nullptr;
    if (const char* v = std::getenv("ROUTEST_CCH_PREFETCH_MIN")) prefetch_min = std::atoi(v);
    // rehearsal knob (bench/route_context_bench.py): shifts the clock "now" routing contexts are
    // resolved with, so an hour boundary can be crossed on demand
    if (const char* v = std::getenv("ROUTEST_ROUTE_CLOCK_SKEW_S")) clock_skew_s = std::atoll(v);
    if (cfg.cch != nullptr && cfg.cch_contexts && async_ctx) {
      listener = cfg.cch->add_build_listener([this](uint64_t key, bool ok) { on_built(key, ok); });
      cfg.cch->start_builders();         // their allocations at startup, not mid-serving
    }
    if (std::getenv("ROUTEST_ROUTE_PREWARM") == nullptr || std::string(std::getenv("ROUTEST_ROUTE_PREWARM")) != "0")
      prewarm();
    if (const char* v = std::getenv("ROUTEST_HANG_ARM"))      // the watchdog rehearsal: see native_server.hip
      if (std::string(v) == "1" && isolated_stream(cfg.device, &hang_stream) != hipSuccess) hang_stream = nullptr;
    th_asm = std::thread([this] { asm_loop(); });
    while (true) {
      auto* b = new Batch();
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (stop && q.empty()) { delete b; break; }
        // collect: up to batch_max, or timeout_us after the OLDEST queued job's arrival — jobs that
        // queued during the previous flush's GPU stage have waited long enough already (timing the
        // window from this wake-up added up to timeout_us to every flush of a busy service)
        const double t_wake = now_us();
        static const bool from_wake = [] {   // ROUTEST_ROUTE_COLLECT=wake: the round-5 window (A/B)
          const char* v = std::getenv("ROUTEST_ROUTE_COLLECT");
          return v && std::string(v) == "wake";
        }();
        const double t_open = from_wake ? t_wake : q.front()->t_enq_us;
        const auto deadline = std::chrono::steady_clock::time_point(std::chrono::duration_cast<std::chrono::steady_clock::duration>(
            std::chrono::duration<double, std::micro>(t_open + cfg.timeout_us)));
        while ((int)q.size() < cfg.batch_max && !stop && std::chrono::steady_clock::now() < deadline) {
          if (cv.wait_until(lk, deadline) == std::cv_status::timeout) break;
        }
        t_collect_us.fetch_add((long long)(now_us() - t_wake), std::memory_order_relaxed);
        const size_t take = std::min<size_t>(q.size(), (size_t)cfg.batch_max);
        b->jobs.assign(q.begin(), q.begin() + take);
        q.erase(q.begin(), q.begin() + take);
      }
      if (broken.load()) {
        if (drained()) {
          trace("drained: serving again");
          broken.store(false);      // the late work finished: buffers and streams usable again
        } else {
          trace("broken: handing %zu jobs off", b->jobs.size());
          hand_off(b->jobs);
          delete b;
          continue;
        }
      }
      // gpu_hang fault hook: this flush's GPU work goes to a stream on a hardware queue of its own,
      // behind a kernel that waits on the host flag (abandoned, not destroyed, if it hangs)
      hipStream_t main_stream = stream;
      if (cfg.hang_fault && cfg.hang_release_d && cfg.hang_fault()) {
        if (!hang_stream && isolated_stream(cfg.device, &hang_stream) != hipSuccess) hang_stream = nullptr;
        if (hang_stream) {
          stream = hang_stream;
          hipLaunchKernelGGL(route_hang_kernel, dim3(1), dim3(64), 0, stream, cfg.hang_release_d, 500000000ll);
        }
      }
      gpu_stage(*b);
      stream = main_stream;         // (the hang stream is reused once drained: see drained())
      if (fail_fault && !b->jobs.empty()) b->failed = true;
      if (b->failed) {              // a GPU error or the deadline: another GPU's service answers
        trace("flush of %zu jobs failed: handing off", b->jobs.size());
        hand_off(b->jobs);
        delete b;
        continue;
      }
      if (b->jobs.empty()) {        // every job of the flush is waiting for its routing context
        delete b;
        continue;
      }
      const double t_h = now_us();
      std::unique_lock<std::mutex> lk(amu);
      acv.wait(lk, [&] { return aq.size() < 2; });
      t_handoff_us.fetch_add((long long)(now_us() - t_h), std::memory_order_relaxed);
      aq.push_back(b);
      acv.notify_all();
    }
    // stopping: no more requeues; jobs still waiting for a context go to the app
    if (listener) cfg.cch->remove_build_listener(listener);
    std::vector<RouteJob*> left;
    {
      std::lock_guard<std::mutex> lk(wmu);
      for (auto& kv : waiting) left.insert(left.end(), kv.second.begin(), kv.second.end());
      waiting.clear();
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      left.insert(left.end(), q.begin(), q.end());
      q.clear();
    }
    for (RouteJob* j : left) {
      j->fallback = true;
      finish(j);
      done(j);
    }
    {
      std::lock_guard<std::mutex> lk(amu);
      gpu_done = true;
    }
    acv.notify_all();
    th_asm.join();
    (void)hipStreamDestroy(stream);
    if (ev_gpu) (void)hipEventDestroy(ev_gpu);
  }

  void asm_loop() {
    if (hipSetDevice(cfg.device) != hipSuccess) return;
    if (hipStreamCreateWithFlags(&stream_asm, hipStreamNonBlocking) != hipSuccess) return;
    if (hipEventCreateWithFlags(&ev_asm, hipEventDisableTiming) != hipSuccess) ev_asm = nullptr;
    open_store();
    th_persist = std::thread([this] { persist_loop(); });
    while (true) {
      Batch* b = nullptr;
      {
        std::unique_lock<std::mutex> lk(amu);
        acv.wait(lk, [&] { return gpu_done || !aq.empty(); });
        if (aq.empty()) break;
        b = aq.front();
        aq.pop_front();
        acv.notify_all();
      }
      asm_stage(*b);
      n_flushes.fetch_add(1, std::memory_order_relaxed);
      // jobs that persist nothing answer now; the others after their group commit
      std::vector<RouteJob*> save = std::move(b->save);
      std::vector<RouteJob*> now_done;
      {
        const std::unordered_set<RouteJob*> saving(save.begin(), save.end());
        for (RouteJob* j : b->jobs)
          if (!saving.count(j)) {
            finish(j);
            now_done.push_back(j);
          }
      }
      done_all(now_done);
      delete b;
      if (!save.empty()) {
        std::unique_lock<std::mutex> lk(pmu);
        pcv.wait(lk, [&] { return pq.size() < 8; });     // back-pressure on a stalled disk
        pq.push_back(std::move(save));
        pcv.notify_all();
      }
    }
    {
      std::lock_guard<std::mutex> lk(pmu);
      asm_done = true;
    }
    pcv.notify_all();
    th_persist.join();
    for (auto& kv : st_multi) {
      if (kv.second.first) sql.finalize(kv.second.first);
      if (kv.second.second) sql.finalize(kv.second.second);
    }
    st_multi.clear();
    for (void* st : {st_req, st_res, st_begin, st_commit, st_rollback, st_undo})
      if (st) sql.finalize(st);
    if (db) sql.close(db);
    (void)hipStreamDestroy(stream_asm);
    if (ev_asm) (void)hipEventDestroy(ev_asm);
  }

  void fail_all(std::vector<RouteJob*>& jobs, const char* msg) {
    for (RouteJob* j : jobs) {
      if (j->fallback || j->status) continue;
      j->status = 503;
      j->out = rtr::error_body(msg);
    }
  }

  bool plan_multi(std::vector<RouteJob*>& jobs) {
    std::vector<RouteJob*> m;
    for (RouteJob* j : jobs)
      if (!j->fallback && j->req.error.empty() && j->req.dst.size() > 1) m.push_back(j);
    if (m.empty()) return true;
    const int R = (int)m.size();
    int NM = 1;
    for (RouteJob* j : m) NM = std::max(NM, (int)j->req.dst.size() + 1);
    if (NM > 4096) {   // beyond the greedy kernel's LDS scan: CPU greedy for those (never in the UI)
      for (RouteJob* j : m) j->fallback = true;
      return true;
    }
    const size_t RN = (size_t)R * NM;
    if (h_lat.need(RN) || h_lon.need(RN) || h_dem.need(RN) || h_npts.need(R) || h_cap.need(R) || h_maxd.need(R) ||
        h_visit.need(RN) || h_trip.need(RN) || h_ntrips.need(R) || h_status.need(R) || h_row0.need(RN) ||
        d_lat.need(RN) || d_lon.need(RN) || d_dem.need(RN) || d_npts.need(R) || d_cap.need(R) || d_maxd.need(R) ||
        d_D.need(RN * NM) || d_visit.need(RN) || d_trip.need(RN) || d_ntrips.need(R) || d_status.need(R))
      return false;
    for (int k = 0; k < R; ++k) {
      const rtr::RouteReq& r = m[k]->req;
      const int n = (int)r.dst.size() + 1;
      double* la = h_lat.h + (size_t)k * NM;
      double* lo = h_lon.h + (size_t)k * NM;
      double* de = h_dem.h + (size_t)k * NM;
      std::fill(la, la + NM, 0.0);
      std::fill(lo, lo + NM, 0.0);
      std::fill(de, de + NM, 0.0);
      la[0] = r.src.lat;
      lo[0] = r.src.lon;
      for (int i = 1; i < n; ++i) {
        la[i] = r.dst[i - 1].lat;
        lo[i] = r.dst[i - 1].lon;
        de[i] = r.dst[i - 1].demand;
      }
      h_npts.h[k] = n;
      h_cap.h[k] = r.cap;
      h_maxd.h[k] = r.maxd;
    }
    hipError_t e = hipSuccess;
    auto cp = [&](void* d, const void* h, size_t b) {
      if (e == hipSuccess) e = qcopy(d, h, b, stream);
    };
    cp(d_lat.d, h_lat.h, RN * 8);
    cp(d_lon.d, h_lon.h, RN * 8);
    cp(d_dem.d, h_dem.h, RN * 8);
    cp(d_npts.d, h_npts.h, (size_t)R * 4);
    cp(d_cap.d, h_cap.h, (size_t)R * 8);
    cp(d_maxd.d, h_maxd.h, (size_t)R * 8);
    if (e == hipSuccess) e = launch_haversine_matrix(d_lat.d, d_lon.d, d_npts.d, R, NM, cfg.circuity, d_D.d, stream);
    if (e == hipSuccess)
      e = launch_greedy_cvrp(d_D.d, d_npts.d, d_dem.d, d_cap.d, d_maxd.d, R, NM, d_visit.d, d_trip.d, d_ntrips.d,
                             d_status.d, stream);
    auto back = [&](void* h, const void* d, size_t b) {
      if (e == hipSuccess) e = qcopy(h, d, b, stream);
    };
    back(h_visit.h, d_visit.d, RN * 4);
    back(h_trip.h, d_trip.d, RN * 4);
    back(h_ntrips.h, d_ntrips.d, (size_t)R * 4);
    back(h_status.h, d_status.d, (size_t)R * 4);
    // the depot row of every D (the infeasible-stop order key) — the matrices stay on the GPU
    if (e == hipSuccess)
      e = qcopy2d(h_row0.h, (size_t)NM * 8, d_D.d, (size_t)NM * NM * 8, (size_t)NM * 8, (size_t)R, stream);
    if (e == hipSuccess) e = sync(stream, ev_gpu, "k5k6-matrix");
    if (e != hipSuccess) return false;
    for (int k = 0; k < R; ++k) {
      rtr::Plan& p = m[k]->plan;
      const int n = h_npts.h[k];
      const int* vis = h_visit.h + (size_t)k * NM;
      const int* tof = h_trip.h + (size_t)k * NM;
      if (h_status.h[k] != 0) {           // batched.py _unpack: unplaced stops by depot distance
        std::vector<char> placed(n, 0);
        for (int i = 0; i < NM && vis[i] >= 0; ++i) placed[vis[i]] = 1;
        std::vector<int> rest;
        for (int i = 1; i < n; ++i)
          if (!placed[i]) rest.push_back(i);
        const double* d0 = h_row0.h + (size_t)k * NM;
        std::stable_sort(rest.begin(), rest.end(), [&](int a, int b) { return d0[a] < d0[b]; });
        p.infeasible = true;
        for (int i : rest) p.infeasible_stops.push_back(i - 1);
        continue;
      }
      p.trips.assign(h_ntrips.h[k], std::vector<int>{0});
      for (int i = 0; i < NM && vis[i] >= 0; ++i) p.trips[tof[i]].push_back(vis[i]);
      for (auto& t : p.trips) t.push_back(0);
    }
    return true;
  }

  static uint64_t leg_key(int group, int s, int t) {
    return ((uint64_t)(uint32_t)group << 48) ^ ((uint64_t)(uint32_t)s << 24) ^ (uint64_t)(uint32_t)t;
  }

  // edge costs of a metric on the host (maneuver durations, exact host fallback): the copy the
  // customization left with the metric (shares its lifetime), else copied once here
  std::shared_ptr<const std::vector<float>> host_costs(const std::shared_ptr<CchMetricDev>& m) {
    if (m->host_cost.size() == (size_t)cfg.cch->topo().E) return {m, &m->host_cost};
    {
      std::lock_guard<std::mutex> lk(hc_mu);
      auto it = hc_index.find(m->key);
      if (it != hc_index.end()) {
        hc_lru.splice(hc_lru.begin(), hc_lru, it->second);     // most recently used
        return it->second->second;
      }
    }
    auto v = std::make_shared<std::vector<float>>((size_t)cfg.cch->topo().E);
    // (through the pinned staging buffer: the copy kernel writes device-visible host memory only)
    if (h_hcost.need(v->size()) != hipSuccess || qcopy(h_hcost.h, m->cost, v->size() * 4, stream) != hipSuccess ||
        sync(stream, ev_gpu, "host-costs") != hipSuccess)
      return nullptr;
    std::memcpy(v->data(), h_hcost.h, v->size() * 4);
    std::lock_guard<std::mutex> lk(hc_mu);
    if (hc_index.count(m->key)) return v;
    hc_lru.emplace_front(m->key, v);
    hc_index[m->key] = hc_lru.begin();
    while (hc_lru.size() > HC_MAX) {                            // evict the least recently used
      hc_index.erase(hc_lru.back().first);
      hc_lru.pop_back();
    }
    return v;
  }

  // Buffers sized up front for a full flush of dashboard-sized requests (batch_max requests of up to
  // 10 stops, MAX_STOPS of the UI): growing one mid-serving allocates while other GPU work is in
  // flight (a flush handed over from another GPU doubles this service's flush size at once).
  void prewarm() {
    const size_t R = (size_t)std::max(1, cfg.batch_max), NM = 11, RN = R * NM, Q = RN;
    const size_t MP = (size_t)std::max(1, cfg.max_path);
    bool ok = !(h_lat.need(RN) || h_lon.need(RN) || h_dem.need(RN) || h_npts.need(R) || h_cap.need(R) ||
                h_maxd.need(R) || h_visit.need(RN) || h_trip.need(RN) || h_ntrips.need(R) || h_status.need(R) ||
                h_row0.need(RN) || d_lat.need(RN) || d_lon.need(RN) || d_dem.need(RN) || d_npts.need(R) ||
                d_cap.need(R) || d_maxd.need(R) || d_D.need(RN * NM) || d_visit.need(RN) || d_trip.need(RN) ||
                d_ntrips.need(R) || d_status.need(R));
    ok = ok && !(h_src.need(Q) || h_dst.need(Q) || h_len.need(Q) || h_st.need(Q) || h_cost.need(Q) ||
                 h_off.need(Q) || d_src.need(Q) || d_dst.need(Q) || d_len.need(Q) || d_st.need(Q) ||
                 d_cost.need(Q) || d_off.need(Q) || d_path.need(Q * MP) || h_flat.need(Q * 256) ||
                 d_flat.need(Q * 256) || h_rec.need(R) || h_eta.need(R) || d_rec.need(R) || d_eta.need(R));
    if (cfg.cch != nullptr) {
      ok = ok && !(h_pts.need(RN) || h_npts2.need(R) || d_pts.need(RN) || d_npts2.need(R) || d_msec.need(RN * NM) ||
                   d_mmet.need(RN * NM) || h_met.need(Q) || d_met.need(Q) || d_edge.need(Q * MP) ||
                   h_flat_e.need(Q * 256) || d_flat_e.need(Q * 256) || h_lr.need(Q) || h_li.need(Q) || h_lj.need(Q) ||
                   d_lr.need(Q) || d_li.need(Q) || d_lj.need(Q) || h_rowg.need(R) || d_rowg.need(R) ||
                   h_lgrp.need(Q) || d_lgrp.need(Q) || h_mv.need(R) || d_mv.need(R) ||
                   h_hcost.need((size_t)cfg.cch->topo().E));
      const int S = cfg.cch->stride();
      msc.device = cfg.device;
      ok = ok && msc.ensure(RN * 2, std::max(Q, (RN * NM * 2 + CchGpu::MAX_ARCS - 1) / CchGpu::MAX_ARCS + 1), S,
                                CchGpu::MAX_ARCS) == hipSuccess;
    }
    if (!ok) (void)hipGetLastError();       // best effort: the flushes grow what is missing
  }

  // a context's background build finished: its waiting jobs go back to the head of the queue
  // (a failed build: they build it synchronously in their next flush, which reports the error)
  void on_built(uint64_t key, bool ok) {
    std::vector<RouteJob*> js;
    {
      std::lock_guard<std::mutex> lk(wmu);
      auto it = waiting.find(key);
      if (it == waiting.end()) return;
      js.swap(it->second);
      waiting.erase(it);
    }
    if (!ok)
      for (RouteJob* j : js) j->sync_ctx = true;
    {
      std::lock_guard<std::mutex> lk(mu);
      for (auto it = js.rbegin(); it != js.rend(); ++it) q.push_front(*it);
    }
    cv.notify_one();
  }

  // CCH: group the flush's jobs by routing context and get each metric.  A context that is not
  // customized yet does not stall the flush: its jobs leave the batch and wait for the router's
  // background build (on_built requeues them), the other groups proceed now.  Contexts of requests
  // routed at "now" are prefetched for the next week-hour shortly before the hour turns.
  bool cch_groups(Batch& b) {
    if (cfg.cch != nullptr) cfg.cch->note_queries();     // background builds now run paced
    const rtc::Stamp now = local_now(clock_skew_s);
    const int64_t days = (int64_t)std::floor((double)now.secs / 86400.0);
    const int64_t sec_of_day = now.secs - days * 86400;
    const int now_wh = (int)(((days + 3) % 7 + 7) % 7) * 24 + (int)(sec_of_day / 3600);
    const double t_now = now_us();
    std::unordered_map<uint64_t, int> gidx;
    std::vector<CchContext> ctxs;
    std::vector<char> sync;
    for (RouteJob* j : b.jobs) {
      if (j->fallback || !j->req.error.empty()) continue;
      CchContext c;
      uint64_t key = cfg.cch_fixed_key;
      if (cfg.cch_contexts) {
        c.weather = j->req.route_weather;
        c.congestion = j->req.route_congestion;
        c.weekhour = j->req.route_weekhour >= 0 ? j->req.route_weekhour : now_wh;
        key = c.key();
        if (j->req.route_weekhour < 0) seen_now[(c.weather & 0xFF) | (c.congestion << 8)] = t_now;
      }
      auto it = gidx.find(key);
      if (it == gidx.end()) {
        it = gidx.emplace(key, (int)ctxs.size()).first;
        ctxs.push_back(c);
        sync.push_back(0);
      }
      j->group = it->second;
      if (j->sync_ctx) sync[j->group] = 1;
    }
    // which groups are ready now
    std::vector<std::shared_ptr<CchMetricDev>> met(ctxs.size());
    std::vector<char> ready(ctxs.size(), 1);
    for (size_t g = 0; g < ctxs.size(); ++g) {
      if (!cfg.cch_contexts) {
        if (!cfg.cch->cached_metric(cfg.cch_fixed_key, met[g])) return false;
      } else if (async_ctx && !sync[g]) {
        ready[g] = cfg.cch->cached_metric(ctxs[g].key(), met[g]) ? 1 : 0;
      } else {
        const double t0 = now_us();
        bool fresh = false;
        if (cfg.cch->metric_for(ctxs[g], stream, met[g], &fresh) != hipSuccess) return false;
        if (fresh) {
          n_ctx_built.fetch_add(1, std::memory_order_relaxed);
          t_ctx_us.fetch_add((long long)(now_us() - t0), std::memory_order_relaxed);
        }
      }
    }
    // defer the jobs of groups still building; compact the ready groups
    std::vector<int> remap(ctxs.size(), -1);
    for (size_t g = 0; g < ctxs.size(); ++g)
      if (ready[g]) {
        remap[g] = (int)b.metrics.size();
        b.metrics.push_back(met[g]);
      }
    std::vector<CchContext> to_build;
    if (b.metrics.size() < ctxs.size()) {
      std::vector<RouteJob*> keep;
      keep.reserve(b.jobs.size());
      {
        std::lock_guard<std::mutex> lk(wmu);
        for (RouteJob* j : b.jobs) {
          if (j->fallback || !j->req.error.empty() || ready[j->group]) {
            keep.push_back(j);
            continue;
          }
          if (j->defer_t0 == 0.0) {
            j->defer_t0 = t_now;
            n_deferred.fetch_add(1, std::memory_order_relaxed);
          }
          waiting[ctxs[j->group].key()].push_back(j);
        }
      }
      b.jobs.swap(keep);
      for (size_t g = 0; g < ctxs.size(); ++g)
        if (!ready[g]) to_build.push_back(ctxs[g]);
    }
    for (RouteJob* j : b.jobs) {
      if (j->fallback || !j->req.error.empty()) continue;
      j->group = remap[j->group];
      if (j->defer_t0 > 0.0) {
        t_wait_us.fetch_add((long long)(t_now - j->defer_t0), std::memory_order_relaxed);
        j->defer_t0 = -1.0;                      // counted once
      }
    }
    // (no lock held: a context finished meanwhile notifies on this thread)
    for (const CchContext& c : to_build) cfg.cch->request_build(c, true);
    // the next week-hour of the contexts seen at "now" during the last hour, before it begins
    const int min_in_hour = (int)((sec_of_day % 3600) / 60);
    const int next_wh = (now_wh + 1) % 168;
    if (cfg.cch_contexts && async_ctx && prefetch_min > 0 && min_in_hour >= 60 - prefetch_min) {
      if (prefetched_wh != next_wh) {
        prefetched_wh = next_wh;
        prefetched.clear();
      }
      for (auto it = seen_now.begin(); it != seen_now.end();) {
        if (t_now - it->second > 3600e6) { it = seen_now.erase(it); continue; }
        if (!prefetched.insert(it->first).second) { ++it; continue; }     // queued for next_wh already
        CchContext c;
        c.weather = it->first & 0xFF;
        c.congestion = it->first >> 8;
        c.weekhour = next_wh;
        cfg.cch->request_build(c, false);
        n_prefetch.fetch_add(1, std::memory_order_relaxed);
        ++it;
      }
    }
    b.host_cost.assign(b.metrics.size(), nullptr);
    for (size_t g = 0; g < b.metrics.size(); ++g) {
      b.host_cost[g] = host_costs(b.metrics[g]);
      if (!b.host_cost[g]) return false;
    }
    // the flush's metrics as device views for the multi-context launches (b.metrics keeps them alive
    // until the flush is done)
    const size_t G = b.metrics.size();
    if (G > 0) {
      if (h_mv.need(G) || d_mv.need(G)) return false;
      for (size_t g = 0; g < G; ++g) h_mv.h[g] = CchGpu::view(*b.metrics[g]);
      if (qcopy(d_mv.d, h_mv.h, G * sizeof(CchMView), stream) != hipSuccess) return false;
    }
    return true;
  }

  // CCH: road-metre matrices of every multi-stop job, then the greedy (K6) over them — the same
  // kernel as the haversine path, on road distances.  The jobs of all context groups are ONE set of
  // rows (grouped, a common row width) with each row's group: one upload, one matrix launch sequence
  // over every row (the sweep / meet kernels read the row's metric from the flush's views), one
  // greedy launch, one read-back and one wait — a flush spread over 64 routing contexts costs what
  // a single-context flush of the same size costs.
  bool plan_multi_road(Batch& b) {
    jrow.clear();
    mtag = 0;
    const int G = (int)b.metrics.size();
    std::vector<std::vector<RouteJob*>> byg(G);
    int NM = 1;
    for (RouteJob* j : b.jobs)
      if (!j->fallback && j->req.error.empty() && j->req.dst.size() > 1 && j->group >= 0 && j->group < G) {
        if ((int)j->req.dst.size() + 1 > 4096) {
          j->fallback = true;
          continue;
        }
        byg[j->group].push_back(j);
        NM = std::max(NM, (int)j->req.dst.size() + 1);
      }
    std::vector<RouteJob*> m;                  // all rows, grouped
    std::vector<int> r0(G + 1, 0);
    for (int g = 0; g < G; ++g) {
      r0[g] = (int)m.size();
      m.insert(m.end(), byg[g].begin(), byg[g].end());
    }
    r0[G] = (int)m.size();
    if (m.empty()) return true;
    const int R = (int)m.size();
    const size_t RN = (size_t)R * NM;
    if (h_pts.need(RN) || h_npts2.need(R) || h_dem.need(RN) || h_cap.need(R) || h_maxd.need(R) || h_visit.need(RN) ||
        h_trip.need(RN) || h_ntrips.need(R) || h_status.need(R) || h_row0.need(RN) || d_pts.need(RN) ||
        d_npts2.need(R) || d_dem.need(RN) || d_cap.need(R) || d_maxd.need(R) || d_D.need(RN * NM) ||
        d_msec.need(RN * NM) || d_mmet.need(RN * NM) || d_visit.need(RN) || d_trip.need(RN) || d_ntrips.need(R) ||
        d_status.need(R) || h_rowg.need(R) || d_rowg.need(R))
      return false;
    for (int g = 0; g < G; ++g)
      for (int k = r0[g]; k < r0[g + 1]; ++k) h_rowg.h[k] = g;
    rtc::parallel_chunks((size_t)R, 64, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t k = lo; k < hi; ++k) {
        const rtr::RouteReq& r = m[k]->req;
        const int n = (int)r.dst.size() + 1;
        int* pt = h_pts.h + k * NM;
        double* de = h_dem.h + k * NM;
        std::fill(pt, pt + NM, 0);
        std::fill(de, de + NM, 0.0);
        pt[0] = grid.nearest(r.src.lat, r.src.lon, cfg.snap_c);
        for (int i = 1; i < n; ++i) {
          pt[i] = grid.nearest(r.dst[i - 1].lat, r.dst[i - 1].lon, cfg.snap_c);
          de[i] = r.dst[i - 1].demand;
        }
        h_npts2.h[k] = n;
        h_cap.h[k] = r.cap;
        h_maxd.h[k] = r.maxd;
      }
    });
    hipError_t e = hipSuccess;
    auto cp = [&](void* d, const void* h, size_t bytes) {
      if (e == hipSuccess) e = qcopy(d, h, bytes, stream);
    };
    cp(d_pts.d, h_pts.h, RN * 4);
    cp(d_npts2.d, h_npts2.h, (size_t)R * 4);
    cp(d_dem.d, h_dem.h, RN * 8);
    cp(d_cap.d, h_cap.h, (size_t)R * 8);
    cp(d_maxd.d, h_maxd.h, (size_t)R * 8);
    cp(d_rowg.d, h_rowg.h, (size_t)R * 4);
    if (e == hipSuccess)
      e = cfg.cch->matrix_multi(d_mv.d, d_rowg.d, d_pts.d, d_npts2.d, R, NM, d_msec.d, d_mmet.d, d_D.d, msc, stream);
    mtag = e == hipSuccess ? msc.chain_tag : 0;
    for (int k = 0; k < R; ++k) jrow[m[k]] = k;
    if (e == hipSuccess)
      e = launch_greedy_cvrp(d_D.d, d_npts2.d, d_dem.d, d_cap.d, d_maxd.d, R, NM, d_visit.d, d_trip.d, d_ntrips.d,
                             d_status.d, stream);
    auto back = [&](void* h, const void* d, size_t bytes) {
      if (e == hipSuccess) e = qcopy(h, d, bytes, stream);
    };
    back(h_visit.h, d_visit.d, RN * 4);
    back(h_trip.h, d_trip.d, RN * 4);
    back(h_ntrips.h, d_ntrips.d, (size_t)R * 4);
    back(h_status.h, d_status.d, (size_t)R * 4);
    if (e == hipSuccess)
      e = qcopy2d(h_row0.h, (size_t)NM * 8, d_D.d, (size_t)NM * NM * 8, (size_t)NM * 8, (size_t)R, stream);
    if (e == hipSuccess) e = sync(stream, ev_gpu, "cch-matrix+greedy");
    if (e != hipSuccess) return false;
    for (int k = 0; k < R; ++k) unpack_plan(m[k], h_npts2.h[k], NM, k);
    return true;
  }

  // K6 output of request k -> its Plan (trips, or the infeasible stops by depot distance)
  void unpack_plan(RouteJob* j, int n, int NM, int k) {
    rtr::Plan& p = j->plan;
    const int* vis = h_visit.h + (size_t)k * NM;
    const int* tof = h_trip.h + (size_t)k * NM;
    if (h_status.h[k] != 0) {           // batched.py _unpack: unplaced stops by depot distance
      std::vector<char> placed(n, 0);
      for (int i = 0; i < NM && vis[i] >= 0; ++i) placed[vis[i]] = 1;
      std::vector<int> rest;
      for (int i = 1; i < n; ++i)
        if (!placed[i]) rest.push_back(i);
      const double* d0 = h_row0.h + (size_t)k * NM;
      std::stable_sort(rest.begin(), rest.end(), [&](int a, int c) { return d0[a] < d0[c]; });
      p.infeasible = true;
      for (int i : rest) p.infeasible_stops.push_back(i - 1);
      return;
    }
    p.trips.assign(h_ntrips.h[k], std::vector<int>{0});
    for (int i = 0; i < NM && vis[i] >= 0; ++i) p.trips[tof[i]].push_back(vis[i]);
    for (auto& t : p.trips) t.push_back(0);
  }

  // CCH legs: every unique (context, s, t) leg of the flush, one route call per context group
  // (sweep + meet + unpack launches), then the same path compaction / copy-out as the A* path
  bool search_legs_cch(Batch& b) {
    std::vector<rtr::Leg>& legs = b.legs;
    std::unordered_map<uint64_t, int>& leg_index = b.leg_index;
    double t0 = now_us();
    std::vector<RouteJob*> g;
    for (RouteJob* j : b.jobs)
      if (!j->fallback && !j->calls.empty()) g.push_back(j);
    rtc::parallel_chunks(g.size(), 64, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        RouteJob* j = g[i];
        j->nodes.clear();
        for (const auto& c : j->calls)
          for (const auto& pt : c) j->nodes.push_back(grid.nearest(pt.second, pt.first, cfg.snap_c));
      }
    });
    add_t(2, t0);
    t0 = now_us();
    const int G = (int)b.metrics.size();
    std::vector<std::vector<std::pair<int, int>>> pairs(G);
    std::vector<int> order;                    // leg index -> (group, index in group) flattened
    // legs of a multi-stop job run between points of its group's matrix: their chains are reused
    // (meet + unpack only); every other leg (point-to-point jobs, alternatives' via legs) is routed
    std::vector<std::vector<std::array<int, 3>>> tri(G);      // (row, i, j) of each matrix-derived pair
    std::vector<std::vector<std::pair<int, int>>> rest(G);
    auto want = [&](int grp, int s, int t, int row, int i, int jj) {
      if (!leg_index.emplace(leg_key(grp, s, t), -1 - grp).second) return;
      if (row >= 0) {
        pairs[grp].emplace_back(s, t);
        tri[grp].push_back({row, i, jj});
      } else {
        rest[grp].emplace_back(s, t);
      }
    };
    for (RouteJob* j : g) {
      int row = -1;
      if (mtag != 0 && !j->plan.trips.empty()) {
        auto it = jrow.find(j);
        if (it != jrow.end()) row = it->second;
      }
      size_t off = 0;
      for (size_t ci = 0; ci < j->calls.size(); ++ci) {
        const auto& c = j->calls[ci];
        // call ci of a multi-stop job is trip ci: its points are the trip's point indices
        const bool from_trip = row >= 0 && ci < j->plan.trips.size() && j->plan.trips[ci].size() == c.size();
        for (size_t i = 0; i + 1 < c.size(); ++i)
          want(j->group, j->nodes[off + i], j->nodes[off + i + 1], from_trip ? row : -1,
               from_trip ? j->plan.trips[ci][i] : 0, from_trip ? j->plan.trips[ci][i + 1] : 0);
        off += c.size();
      }
    }
    // "alternatives": every unique leg (in order) gets its via nodes; s->w and w->t join the batch
    std::vector<RouteJob*> alt_jobs;
    for (RouteJob* j : g)
      if (j->req.alt_k > 0) alt_jobs.push_back(j);
    rtc::parallel_chunks(alt_jobs.size(), 1, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        RouteJob* j = alt_jobs[i];
        j->alt_pairs.clear();
        std::unordered_map<uint64_t, int> seen;
        size_t off = 0;
        for (const auto& c : j->calls) {
          for (size_t k = 0; k + 1 < c.size(); ++k) {
            const int s = j->nodes[off + k], t = j->nodes[off + k + 1];
            if (seen.emplace(((uint64_t)(uint32_t)s << 32) | (uint32_t)t, 0).second) j->alt_pairs.emplace_back(s, t);
          }
          off += c.size();
        }
        j->alt_vias.assign(j->alt_pairs.size(), {});
        for (size_t k = 0; k < j->alt_pairs.size(); ++k)
          j->alt_vias[k] = ralt::via_nodes(cfg.glat, cfg.glon, cfg.N, j->alt_pairs[k].first, j->alt_pairs[k].second,
                                           j->req.alt_k - 1);
      }
    });
    for (RouteJob* j : alt_jobs)
      for (size_t k = 0; k < j->alt_pairs.size(); ++k)
        for (int w : j->alt_vias[k]) {
          want(j->group, j->alt_pairs[k].first, w, -1, 0, 0);
          want(j->group, w, j->alt_pairs[k].second, -1, 0, 0);
        }
    // leg order: every group's matrix-derived legs (group order), then every other leg (group order)
    int QA = 0, QR = 0;
    for (int gi = 0; gi < G; ++gi) {
      QA += (int)pairs[gi].size();
      QR += (int)rest[gi].size();
    }
    const int Q = QA + QR;
    {
      int a = 0, r = QA;
      for (int gi = 0; gi < G; ++gi) {
        for (const auto& pr : pairs[gi]) leg_index[leg_key(gi, pr.first, pr.second)] = a++;
        for (const auto& pr : rest[gi]) leg_index[leg_key(gi, pr.first, pr.second)] = r++;
      }
    }
    legs.assign(Q, rtr::Leg());
    if (Q == 0) return true;
    n_legs.fetch_add(Q, std::memory_order_relaxed);
    const int MP = cfg.max_path;
    if (h_src.need(Q) || h_dst.need(Q) || h_len.need(Q) || h_st.need(Q) || h_cost.need(Q) || h_met.need(Q) ||
        h_off.need(Q) || d_src.need(Q) || d_dst.need(Q) || d_len.need(Q) || d_st.need(Q) || d_cost.need(Q) ||
        d_met.need(Q) || d_off.need(Q) || d_path.need((size_t)Q * MP) || d_edge.need((size_t)Q * MP) ||
        h_lgrp.need(Q) || d_lgrp.need(Q))
      return false;
    if (QA > 0 && (h_lr.need(QA) || h_li.need(QA) || h_lj.need(QA) || d_lr.need(QA) || d_li.need(QA) || d_lj.need(QA)))
      return false;
    {
      int a = 0, r = QA;
      for (int gi = 0; gi < G; ++gi) {
        for (size_t k = 0; k < pairs[gi].size(); ++k, ++a) {
          h_src.h[a] = pairs[gi][k].first;
          h_dst.h[a] = pairs[gi][k].second;
          h_lgrp.h[a] = gi;
          h_lr.h[a] = tri[gi][k][0];
          h_li.h[a] = tri[gi][k][1];
          h_lj.h[a] = tri[gi][k][2];
        }
        for (const auto& pr : rest[gi]) {
          h_src.h[r] = pr.first;
          h_dst.h[r] = pr.second;
          h_lgrp.h[r] = gi;
          ++r;
        }
      }
    }
    hipError_t e = qcopy(d_src.d, h_src.h, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(d_dst.d, h_dst.h, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(d_lgrp.d, h_lgrp.h, (size_t)Q * 4, stream);
    if (QA > 0) {
      if (e == hipSuccess) e = qcopy(d_lr.d, h_lr.h, (size_t)QA * 4, stream);
      if (e == hipSuccess) e = qcopy(d_li.d, h_li.h, (size_t)QA * 4, stream);
      if (e == hipSuccess) e = qcopy(d_lj.d, h_lj.h, (size_t)QA * 4, stream);
    }
    auto out_at = [&](int q) {
      CchRouteOut o;
      o.sec = d_cost.d + q;
      o.metres = d_met.d + q;
      o.status = d_st.d + q;
      o.len = d_len.d + q;
      o.path = d_path.d + (size_t)q * MP;
      o.edges = d_edge.d + (size_t)q * MP;
      o.max_path = MP;
      return o;
    };
    if (e == hipSuccess && QA > 0)
      e = cfg.cch->legs_from_matrix_multi(d_mv.d, d_lgrp.d, d_src.d, d_lr.d, d_li.d, d_lj.d, QA, mtag, out_at(0), msc,
                                          stream);
    if (e == hipSuccess && QR > 0)
      e = cfg.cch->route_multi(d_mv.d, d_lgrp.d + QA, d_src.d + QA, d_dst.d + QA, QR, out_at(QA), csc, stream);
    n_legs_reused.fetch_add(QA, std::memory_order_relaxed);
    if (e == hipSuccess) e = qcopy(h_st.h, d_st.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(h_len.h, d_len.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(h_cost.h, d_cost.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(h_met.h, d_met.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = sync(stream, ev_gpu, "cch-legs");
    add_t(3, t0);
    t0 = now_us();
    if (e != hipSuccess) return false;
    long long total = 0;
    for (int i = 0; i < Q; ++i) {
      h_off.h[i] = total;
      if (h_st.h[i] == 0) total += std::min(h_len.h[i], MP);
    }
    if (total > 0) {
      if (h_flat.need((size_t)total) || d_flat.need((size_t)total)) return false;
      e = qcopy(d_off.d, h_off.h, (size_t)Q * 8, stream);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(compact_paths_kernel, dim3(Q), dim3(256), 0, stream, d_path.d, MP, d_len.d, d_st.d, d_off.d,
                           Q, d_flat.d);
        e = hipGetLastError();
      }
      // the hops' road edges the same way (maneuvers look them up instead of scanning adjacency)
      if (e == hipSuccess && (h_flat_e.need((size_t)total) || d_flat_e.need((size_t)total))) e = hipErrorOutOfMemory;
      if (e == hipSuccess) {
        hipLaunchKernelGGL(compact_paths_kernel, dim3(Q), dim3(256), 0, stream, d_edge.d, MP, d_len.d, d_st.d, d_off.d,
                           Q, d_flat_e.d);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = qcopy(h_flat.h, d_flat.d, (size_t)total * 4, stream);
      if (e == hipSuccess) e = qcopy(h_flat_e.h, d_flat_e.d, (size_t)total * 4, stream);
      if (e == hipSuccess) e = sync(stream, ev_gpu, "cch-paths");
      if (e != hipSuccess) return false;
      b.flat.assign(h_flat.h, h_flat.h + total);
      b.flat_e.assign(h_flat_e.h, h_flat_e.h + total);
    }
    add_t(4, t0);
    // legs the GPU could not return (status 4: longer than max_path / unpack stack): exact on the host
    int nbad = 0;
    for (int i = 0; i < Q; ++i) nbad += h_st.h[i] == 4;
    b.host_paths.resize(Q);
    for (int i = 0; i < Q; ++i) {
        const int gi = h_lgrp.h[i];
        rtr::Leg& L = legs[i];
        if (h_st.h[i] == 0) {
          L.sec = h_cost.h[i];
          L.metres = h_met.h[i];
          L.len = std::min(h_len.h[i], MP);
          L.path = b.flat.data() + h_off.h[i];
          L.edges = b.flat_e.data() + h_off.h[i];
        } else if (h_st.h[i] == 4 && nbad <= 1024 && cfg.h_indptr != nullptr) {
          const std::vector<float>& hc = *b.host_cost[gi];
          float c;
          if (host_dijkstra(cfg.h_indptr, cfg.h_indices, hc.data(), cfg.N, h_src.h[i], h_dst.h[i], 1 << 22, c,
                            b.host_paths[i])) {
            L.sec = c;
            float met = 0.f;
            const auto& p = b.host_paths[i];
            for (size_t k = 0; k + 1 < p.size(); ++k) {
              int32_t best = -1;
              for (int32_t ee = cfg.h_indptr[p[k]]; ee < cfg.h_indptr[p[k] + 1]; ++ee)
                if (cfg.h_indices[ee] == p[k + 1] && (best < 0 || hc[ee] < hc[best])) best = ee;
              if (best >= 0) met += cfg.h_length[best];
            }
            L.metres = met;
            L.len = (int)p.size();
            L.path = p.data();
            n_host_legs.fetch_add(1, std::memory_order_relaxed);
          }
        }
      }
    return true;
  }

  // graph provider: snap, search every unique leg of the flush once, fill the batch's legs
  bool search_legs(Batch& b) {
    std::vector<RouteJob*>& jobs = b.jobs;
    std::vector<rtr::Leg>& legs = b.legs;
    std::vector<std::vector<int32_t>>& host_paths = b.host_paths;
    std::unordered_map<uint64_t, int>& leg_index = b.leg_index;
    double t0 = now_us();
    std::vector<RouteJob*> g;
    for (RouteJob* j : jobs)
      if (!j->fallback && !j->calls.empty()) g.push_back(j);
    rtc::parallel_chunks(g.size(), 64, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        RouteJob* j = g[i];
        j->nodes.clear();
        for (const auto& c : j->calls)
          for (const auto& pt : c) j->nodes.push_back(grid.nearest(pt.second, pt.first, cfg.snap_c));
      }
    });
    add_t(2, t0);
    t0 = now_us();
    std::vector<std::pair<int, int>> pairs;
    for (RouteJob* j : g) {
      size_t off = 0;
      for (const auto& c : j->calls) {
        for (size_t i = 0; i + 1 < c.size(); ++i) {
          const uint64_t key = ((uint64_t)(uint32_t)j->nodes[off + i] << 32) | (uint32_t)j->nodes[off + i + 1];
          if (leg_index.emplace(key, (int)pairs.size()).second) pairs.emplace_back(j->nodes[off + i], j->nodes[off + i + 1]);
        }
        off += c.size();
      }
    }
    const int Q = (int)pairs.size();
    legs.assign(Q, rtr::Leg());
    if (Q == 0) return true;
    n_legs.fetch_add(Q, std::memory_order_relaxed);
    const int MP = cfg.max_path;
    if (h_src.need(Q) || h_dst.need(Q) || h_len.need(Q) || h_st.need(Q) || h_cost.need(Q) || h_off.need(Q) ||
        h_qidx.need(Q) || d_src.need(Q) || d_dst.need(Q) || d_len.need(Q) || d_st.need(Q) || d_cost.need(Q) ||
        d_off.need(Q) || d_qidx.need(Q + 1) || d_iters.need(Q) || d_path.need((size_t)Q * MP))
      return false;
    for (int i = 0; i < Q; ++i) {
      h_src.h[i] = pairs[i].first;
      h_dst.h[i] = pairs[i].second;
    }
    hipError_t e = qcopy(d_src.d, h_src.h, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(d_dst.d, h_dst.h, (size_t)Q * 4, stream);
    // the tiered search (csrc/astar.hip): interactive flushes (few thousand legs) skip the lane tier
    // (routing/graph.py BatchedAstar.run calls the same function)
    AstarGraphDev gd;
    gd.indptr = cfg.indptr;
    gd.indices = cfg.indices;
    gd.cost = cfg.cost;
    gd.lat = cfg.lat32;
    gd.lon = cfg.lon32;
    gd.N = cfg.N;
    gd.inv_vmax = cfg.inv_vmax;
    gd.lm = cfg.lm;
    gd.K = cfg.K;
    AstarOut ao;
    ao.cost = d_cost.d;
    ao.len = d_len.d;
    ao.status = d_st.d;
    ao.path = d_path.d;
    ao.max_path = MP;
    ao.iters = d_iters.d;
    AstarPlan pl;
    pl.max_iters = cfg.max_iters;
    pl.lane_pops = cfg.lane_pops;
    pl.wave_only_below = cfg.wave_only_below;
    pl.delta = cfg.wave_delta;
    pl.lane_max_m = cfg.lane_max_m;
    AstarRunStats rs;
    if (e == hipSuccess)
      e = astar_search(gd, d_src.d, d_dst.d, Q, cfg.lane_ws.slots > 0 ? &cfg.lane_ws : nullptr,
                       cfg.wave_ws.slots > 0 ? &cfg.wave_ws : nullptr, cfg.big_ws.slots > 0 ? &cfg.big_ws : nullptr,
                       ao, pl, d_qidx.d, stream, &rs, cfg.arena.base ? &cfg.arena : nullptr);
    n_escalated.fetch_add(rs.escalated, std::memory_order_relaxed);
    if (e == hipSuccess) e = qcopy(h_st.h, d_st.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = sync(stream, ev_gpu, "astar");
    add_t(3, t0);
    t0 = now_us();
    if (e == hipSuccess) e = qcopy(h_len.h, d_len.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = qcopy(h_cost.h, d_cost.d, (size_t)Q * 4, stream);
    if (e == hipSuccess) e = sync(stream, ev_gpu, "astar-escalate");
    if (e != hipSuccess) return false;
    long long total = 0;
    for (int i = 0; i < Q; ++i) {
      h_off.h[i] = total;
      if (h_st.h[i] == 0) total += std::min(h_len.h[i], MP);
    }
    if (total > 0) {
      if (h_flat.need((size_t)total) || d_flat.need((size_t)total)) return false;
      e = qcopy(d_off.d, h_off.h, (size_t)Q * 8, stream);
      if (e == hipSuccess) {
        hipLaunchKernelGGL(compact_paths_kernel, dim3(Q), dim3(256), 0, stream, d_path.d, MP, d_len.d, d_st.d, d_off.d,
                           Q, d_flat.d);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = qcopy(h_flat.h, d_flat.d, (size_t)total * 4, stream);
      if (e == hipSuccess) e = sync(stream, ev_gpu, "astar-paths");
      if (e != hipSuccess) return false;
      b.flat.assign(h_flat.h, h_flat.h + total);     // the next flush reuses the pinned buffer
    }
    add_t(4, t0);
    // searches both GPU stages gave up on (status 2 / 3): exact on the host, like graph.py
    int nbad = 0;
    for (int i = 0; i < Q; ++i) nbad += (h_st.h[i] == 2 || h_st.h[i] == 3);
    host_paths.resize(Q);
    for (int i = 0; i < Q; ++i) {
      rtr::Leg& L = legs[i];
      if (h_st.h[i] == 0) {
        L.sec = h_cost.h[i];
        L.len = std::min(h_len.h[i], MP);
        L.path = b.flat.data() + h_off.h[i];
      } else if ((h_st.h[i] == 2 || h_st.h[i] == 3) && nbad <= 1024 && cfg.h_indptr != nullptr) {
        float c;
        if (host_dijkstra(cfg.h_indptr, cfg.h_indices, cfg.h_cost, cfg.N, pairs[i].first, pairs[i].second, MP, c,
                          host_paths[i])) {
          L.sec = c;
          L.len = (int)host_paths[i].size();
          L.path = host_paths[i].data();
          n_host_legs.fetch_add(1, std::memory_order_relaxed);
        }
      }
    }
    return true;
  }

  // "alternatives": per unique leg, the candidates (time-shortest path, then s->w->t per via node
  // when both parts were found), the scorer's values, the pick, and the response block — exactly
  // routing/alternatives.py AlternativeLegs.choose + optimize_with_alternatives
  void choose_alternatives(Batch& b, RouteJob* j) {
    const std::vector<rtr::Leg>& legs = b.legs;
    const double* delay = b.alt_delay->data();
    const size_t P = j->alt_pairs.size();
    struct Cand {
      double sec, met;
      const int32_t* p1;
      int n1;
      const int32_t* p2;   // second part (from its node 1 on), or nullptr
      int n2;
      const int32_t* e1;   // hop edges of the parts (nullptr: unknown, looked up on the host)
      const int32_t* e2;
    };
    auto leg = [&](int s, int t) -> const rtr::Leg* {
      auto it = b.leg_index.find(leg_key(j->group, s, t));
      return it == b.leg_index.end() || it->second < 0 ? nullptr : &legs[it->second];
    };
    std::vector<std::vector<Cand>> cands(P);
    size_t total = 0;
    for (size_t k = 0; k < P; ++k) {
      const int s = j->alt_pairs[k].first, t = j->alt_pairs[k].second;
      const rtr::Leg* d = leg(s, t);
      if (d && d->len > 0) cands[k].push_back({d->sec, d->metres, d->path, d->len, nullptr, 0, d->edges, nullptr});
      for (int w : j->alt_vias[k]) {
        const rtr::Leg* a = leg(s, w);
        const rtr::Leg* c = leg(w, t);
        if (a && c && a->len > 0 && c->len > 0)
          cands[k].push_back({a->sec + c->sec, a->metres + c->metres, a->path, a->len, c->path + 1, c->len - 1,
                              a->edges, c->edges});
      }
      total += cands[k].size();
    }
    (void)total;
    j->alt_legs.assign(P, rtr::Leg());
    j->alt_paths.assign(P, {});
    j->alt_edges.assign(P, {});
    std::string o = ",\"alternatives\":{\"k\":";
    rtr::put_int(o, j->req.alt_k);
    o += ",\"scorer\":";
    rtr::put_str(o, b.alt_engine);
    o += ",\"legs\":[";
    std::vector<int32_t> tmp;
    for (size_t k = 0; k < P; ++k) {
      if (k) o += ',';
      o += "{\"from_node\":";
      rtr::put_int(o, j->alt_pairs[k].first);
      o += ",\"to_node\":";
      rtr::put_int(o, j->alt_pairs[k].second);
      o += ",\"candidates\":";
      rtr::put_int(o, (long long)cands[k].size());
      if (cands[k].empty()) {
        o += '}';
        continue;       // Leg stays "not found": the assembly reports it like a plain request
      }
      std::vector<double> sc(cands[k].size());
      for (size_t c = 0; c < cands[k].size(); ++c) {
        const Cand& x = cands[k][c];
        tmp.assign(x.p1, x.p1 + x.n1);
        if (x.p2) tmp.insert(tmp.end(), x.p2, x.p2 + x.n2);
        sc[c] = ralt::candidate_score(cfg.glat, cfg.glon, delay, tmp.data(), tmp.size(), x.sec, b.alt_kind);
      }
      const int best = ralt::argmin_score(sc);
      const Cand& x = cands[k][best];
      std::vector<int32_t>& own = j->alt_paths[k];
      own.assign(x.p1, x.p1 + x.n1);
      if (x.p2) own.insert(own.end(), x.p2, x.p2 + x.n2);
      rtr::Leg& L = j->alt_legs[k];
      L.sec = x.sec;
      L.metres = x.met;
      L.path = own.data();
      L.len = (int)own.size();
      if (x.e1 && (x.p2 == nullptr || x.e2)) {
        std::vector<int32_t>& oe = j->alt_edges[k];
        oe.assign(x.e1, x.e1 + (x.n1 - 1));
        if (x.p2) oe.insert(oe.end(), x.e2, x.e2 + x.n2);     // the second part's hops: n2 of them
        L.edges = oe.data();
      }
      o += ",\"chosen\":";
      rtr::put_int(o, best);
      o += ",\"scores\":[";
      for (size_t c = 0; c < sc.size(); ++c) {
        if (c) o += ',';
        rtr::put_float(o, sc[c]);
      }
      o += "],\"seconds\":[";
      for (size_t c = 0; c < cands[k].size(); ++c) {
        if (c) o += ',';
        rtr::put_float(o, cands[k][c].sec);
      }
      o += "]}";
    }
    o += "]}";
    j->alt_json = std::move(o);
  }

  void assemble_all(Batch& b) {
    std::vector<RouteJob*>& jobs = b.jobs;
    const std::vector<rtr::Leg>& legs = b.legs;
    const std::unordered_map<uint64_t, int>& leg_index = b.leg_index;
    rtc::parallel_chunks(jobs.size(), 8, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        RouteJob* j = jobs[i];
        if (j->fallback || j->status) continue;
        if (j->req.alt_k > 0) choose_alternatives(b, j);
        std::vector<rtr::Dir> dirs(j->calls.size());
        std::string perr;
        size_t off = 0;
        // the compact record of a route that will be persisted (graph provider, no alternatives)
        bool want_rec = rg != nullptr && db != nullptr && !j->request_route && j->req.alt_k == 0 &&
                        cfg.provider == 1 && !j->calls.empty();
        rrec::Writer rw;
        std::vector<uint64_t> durs;
        std::vector<uint32_t> per_leg;
        j->rec.clear();
        for (size_t k = 0; k < j->calls.size() && perr.empty(); ++k) {
          if (cfg.provider == 0) {
            rtr::haversine_directions(j->calls[k], j->req.profile, cfg.circuity, cfg.step_m, dirs[k]);
          } else {
            std::vector<const rtr::Leg*> lp;
            for (size_t t = 0; t + 1 < j->calls[k].size(); ++t) {
              const int s0 = j->nodes[off + t], s1 = j->nodes[off + t + 1];
              if (j->req.alt_k > 0) {        // the pair's chosen candidate
                size_t a = 0;
                while (j->alt_pairs[a].first != s0 || j->alt_pairs[a].second != s1) ++a;
                lp.push_back(&j->alt_legs[a]);
                continue;
              }
              const uint64_t key = cfg.cch ? leg_key(j->group, s0, s1)
                                           : (((uint64_t)(uint32_t)s0 << 32) | (uint32_t)s1);
              lp.push_back(&legs[leg_index.at(key)]);
            }
            rtr::GraphHost gh;
            const rtr::GraphHost* ghp = nullptr;
            if (cfg.cch && cfg.h_length != nullptr) {
              gh.indptr = cfg.h_indptr;
              gh.indices = cfg.h_indices;
              gh.length = cfg.h_length;
              gh.cost = b.host_cost[j->group]->data();
              gh.edge_name = cfg.h_edge_name;
              gh.names = &cfg.names;
              gh.edge_heading = headings();
              ghp = &gh;
            }
            if (k == 0 && want_rec) rrec::begin(rw, *rg, ghp != nullptr, j->req.profile, j->calls.size());
            durs.clear();
            per_leg.clear();
            rtr::StepDurs sd;
            sd.out = &durs;
            sd.per_leg = &per_leg;
            perr = rtr::graph_directions(j->calls[k], j->nodes.data() + off, lp, j->req.profile, cfg.glat, cfg.glon,
                                         dirs[k], ghp, want_rec && ghp ? &sd : nullptr);
            off += j->calls[k].size();
            if (want_rec && perr.empty())
              want_rec = !sd.bad && rrec::add_call(rw, *rg, ghp, j->calls[k], lp, durs, per_leg);
          }
        }
        if (!perr.empty()) j->req.error = perr;
        if (want_rec && perr.empty()) {
          j->rec = std::move(rw.b);
          n_records.fetch_add(1, std::memory_order_relaxed);
          n_record_bytes.fetch_add((long long)j->rec.size(), std::memory_order_relaxed);
        }
        if (!rtr::assemble(j->req, j->plan, dirs, cfg.engine, j->asmb, ccache()))
          j->fallback = true;
        else if (j->req.alt_k > 0 && j->asmb.ok) j->asmb.body += j->alt_json;
      }
    });
  }

  bool run_eta(std::vector<RouteJob*>& jobs) {
    std::vector<RouteJob*> m;
    for (RouteJob* j : jobs)
      if (!j->fallback && !j->status && j->asmb.ok && j->req.use_ml_eta && j->req.eta_ok) m.push_back(j);
    if (m.empty()) return true;
    std::shared_ptr<const NativeModel> model = cfg.eta_model ? cfg.eta_model() : nullptr;
    if (model == nullptr) {          // the served model is one the native path does not run: the app answers
      for (RouteJob* j : m) j->fallback = true;
      return true;
    }
    const int n = (int)m.size();
    if (h_rec.need(n) || h_eta.need(n) || d_rec.need(n) || d_eta.need(n)) return false;
    const rtc::Stamp now = local_now();
    for (int k = 0; k < n; ++k) {
      RouteJob* j = m[k];
      j->now = now;
      rtc::EtaRecord& r = h_rec.h[k];
      r.distance_m = (float)j->asmb.dist;
      r.driver_age = (float)j->req.eta_age;
      r.wallclock_s = (int32_t)(now.secs - rtc::EPOCH2020_DAYS * 86400);
      r.weather = j->req.eta_weather;
      r.traffic = j->req.eta_traffic;
      r.pad = 0;
    }
    hipError_t e = qcopy(d_rec.d, h_rec.h, (size_t)n * 16, stream_asm);
    if (e == hipSuccess) e = model->predict(d_rec.d, 16, d_eta.d, n, stream_asm, eta_ws);
    if (e == hipSuccess) e = qcopy(h_eta.h, d_eta.d, (size_t)n * 4, stream_asm);
    if (e == hipSuccess) e = sync(stream_asm, ev_asm, "eta");
    // a failed GPU round: the model's fp32 CPU forward (same fallback as the reactors), into a
    // buffer of its own (a round past the deadline may still write h_eta later)
    std::vector<float> cpu_eta;
    const float* eta = h_eta.h;
    if (e != hipSuccess) {
      cpu_eta.resize((size_t)n);
      std::vector<rtc::EtaRecord> rec(h_rec.h, h_rec.h + n);
      if (!model->cpu_predict(rec.data(), cpu_eta.data(), n)) return false;
      eta = cpu_eta.data();
    }
    for (int k = 0; k < n; ++k) {
      RouteJob* j = m[k];
      const double mins = (double)eta[k];
      // EtaService.finish: pickup + timedelta(minutes) — raises (-> no ETA fields) when out of range
      if (!std::isfinite(mins) || std::fabs(mins) > 1.4e9) continue;
      std::string tmp;
      rtc::format_one(tmp, mins, now.secs, now.us, false, 0, "");
      // {"eta_minutes_ml":X,"eta_completion_time_ml":"..."}: keep the iso text
      const size_t a = tmp.find("\"eta_completion_time_ml\":\"");
      if (a == std::string::npos) continue;
      const size_t b0 = a + 26;
      j->eta_iso = tmp.substr(b0, tmp.size() - 2 - b0);
      j->eta_min = eta[k];
    }
    return true;
  }

  // the request body -> j->root / j->req, once (a job back from waiting for its routing context,
  // or handed over from another GPU's service, is parsed already)
  static void parse_job(RouteJob* j) {
    if (j->parsed) return;
    j->parsed = true;
    bool parsed = false;
    if (j->json_ok && !j->body.empty()) {
      try {
        j->root = rtj::Parser(j->body.data(), j->body.size()).parse();
        parsed = true;
      } catch (const std::exception&) {
      }
    }
    if (j->request_route && (!j->json_ok || (!parsed && !j->body.empty()))) {
      j->fallback = true;
      return;
    }
    static const rtj::Value empty = [] { rtj::Value v; v.kind = rtj::Value::Obj; return v; }();
    const rtj::Value* rootp = parsed ? &j->root : (j->request_route ? nullptr : &empty);
    if (!j->request_route && parsed && j->root.kind != rtj::Value::Obj) rootp = &empty;
    j->req = rtr::parse_route_request(rootp);
    if (j->req.fallback) j->fallback = true;
  }

  // GPU stage: parse, trips (K5 + K6), snapping + the batched A* (graph provider)
  void gpu_stage(Batch& b) {
    std::vector<RouteJob*>& jobs = b.jobs;
    long long fresh_jobs = 0;
    for (RouteJob* j : jobs) fresh_jobs += !j->parsed;
    n_jobs.fetch_add(fresh_jobs, std::memory_order_relaxed);   // (submitted unparsed: none normally)
    double t0 = now_us();
    // (jobs are parsed on the submitting reactor thread, RouteService::submit; this catches any
    // that were not)
    rtc::parallel_chunks(jobs.size(), 32, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) parse_job(jobs[i]);
    });
    // "alternatives" need the road graph through the CCH and a published scorer; else the app
    bool any_alt = false;
    for (RouteJob* j : jobs) any_alt |= !j->fallback && j->req.alt_k > 0;
    if (any_alt) {
      if (cfg.alt && cfg.provider == 1 && cfg.cch != nullptr) b.alt_delay = cfg.alt->get(b.alt_kind, b.alt_engine);
      const bool ok = b.alt_delay != nullptr && (int)b.alt_delay->size() == cfg.N;
      for (RouteJob* j : jobs)
        if (!j->fallback && j->req.alt_k > 0 && (!ok || !j->req.error.empty())) j->fallback = !ok || j->fallback;
    }
    add_t(0, t0);
    {
      double pairs = 0.0;
      bool sync_build = false;
      for (RouteJob* j : jobs) {
        if (j->fallback) continue;
        const double n = (double)j->req.dst.size() + 1.0;
        pairs += n * n;
        sync_build |= j->sync_ctx;
      }
      // ~2 M matrix pairs ride on the base deadline; a synchronous context build gets 30 s more
      flush_deadline_ms.store(deadline_ms <= 0 ? deadline_ms
                                               : deadline_ms * (1.0 + pairs / 2.0e6) + (sync_build ? 30000.0 : 0.0));
    }
    if (cfg.park_scorer) cfg.park_scorer();
    t0 = now_us();
    if (cfg.provider == 1 && cfg.cch != nullptr) {
      // road graph through the CCH: contexts -> road matrices + greedy -> legs
      if (!cch_groups(b) || !plan_multi_road(b)) {
        b.failed = true;
        return;
      }
      add_t(1, t0);
      for (RouteJob* j : jobs)
        if (!j->fallback) rtr::directions_calls(j->req, j->plan, j->calls);
      if (!search_legs_cch(b)) b.failed = true;
      return;
    }
    if (!plan_multi(jobs)) { b.failed = true; return; }
    add_t(1, t0);
    for (RouteJob* j : jobs)
      if (!j->fallback) rtr::directions_calls(j->req, j->plan, j->calls);
    if (cfg.provider == 1 && !search_legs(b)) b.failed = true;
  }

  // assembly stage: GeoJSON, ETA, persistence, response bytes
  void asm_stage(Batch& b) {
    std::vector<RouteJob*>& jobs = b.jobs;
    if (b.failed) return;
    double t0 = now_us();
    assemble_all(b);
    add_t(5, t0);
    t0 = now_us();
    if (!run_eta(jobs)) {
      for (RouteJob* j : jobs) j->eta_iso.clear();
    }
    add_t(6, t0);
    // persistence (optimize_route / route only; request_route never persists) is the persistence
    // thread's: it group-commits these with whatever else is waiting
    for (RouteJob* j : jobs)
      if (db && !j->fallback && !j->status && j->asmb.ok && !j->request_route) b.save.push_back(j);
    t0 = now_us();
    rtc::parallel_chunks(b.save.size(), 16, chunk_threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) prep_persist(b.save[i]);
    });
    add_t(7, t0);
  }

  // the response bytes of a job whose assembly (and persistence, if any) is done
  void finish(RouteJob* j) {
    if (j->fallback) { n_fallback.fetch_add(1, std::memory_order_relaxed); return; }
    if (j->status) return;
    if (!j->asmb.ok) {
      j->status = (j->request_route && cfg.compat200) ? 200 : 400;
      j->out = rtr::error_body(j->asmb.error.empty() ? j->req.error : j->asmb.error);
      return;
    }
    j->status = 200;
    j->out = std::move(j->asmb.body);
    if (!j->eta_iso.empty()) {
      j->out += ",\"eta_minutes_ml\":";
      rtr::put_float(j->out, (double)j->eta_min);
      j->out += ",\"eta_completion_time_ml\":";
      rtr::put_str(j->out, j->eta_iso);
    }
    if (!j->request_id.empty()) {
      j->out += ",\"request_id\":";
      rtr::put_str(j->out, j->request_id);
      j->out += ",\"saved\":true";
    }
    j->out += "}}";
  }

  // Group commit: every flush waiting when the thread wakes goes into ONE transaction (a failed
  // insert removes only its own request's rows, persist_one -- SQLiteStore's per-request
  // semantics).  A response leaves only after its commit, so a client that reads its request_id
  // back (/api/history/<id>) finds it.
  void persist_group(std::vector<std::vector<RouteJob*>>& groups) {
    const std::string now = utc_now_iso();
    const bool tx = step_once(st_begin);
    std::vector<RouteJob*> js;
    for (auto& g : groups)
      for (RouteJob* j : g) {
        j->request_id.clear();
        if (j->p_ok) js.push_back(j);
      }
    persist_chunked(js, now);
    if (tx && !step_once(st_commit)) {
      step_once(st_rollback);      // nothing of the group was stored
      for (auto& g : groups)
        for (RouteJob* j : g) j->request_id.clear();
    }
    for (auto& g : groups)
      for (RouteJob* j : g)
        if (!j->request_id.empty()) n_persisted.fetch_add(1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(cmu);
      ++commits;
    }
    ccv.notify_one();
  }

  bool step_once(void* st) {
    const int rc = sql.step(st);
    sql.reset(st);
    return rc == rtsql::DONE;
  }

  void persist_loop() {
    if (db) th_ckpt = std::thread([this] { ckpt_loop(); });
    while (true) {
      std::vector<std::vector<RouteJob*>> groups;
      {
        std::unique_lock<std::mutex> lk(pmu);
        pcv.wait(lk, [&] { return asm_done || !pq.empty(); });
        if (pq.empty()) break;
        groups.assign(std::make_move_iterator(pq.begin()), std::make_move_iterator(pq.end()));
        pq.clear();
        pcv.notify_all();
      }
      const double t0 = now_us();
      persist_group(groups);
      add_t(7, t0);
      std::vector<RouteJob*> fin;
      for (auto& g : groups)
        for (RouteJob* j : g) {
          finish(j);
          fin.push_back(j);
        }
      done_all(fin);
    }
    if (th_ckpt.joinable()) {
      {
        std::lock_guard<std::mutex> lk(cmu);
        ck_stop = true;
      }
      ccv.notify_all();
      th_ckpt.join();
    }
  }

  // WAL checkpoints on a connection of their own: the writer runs with wal_autocheckpoint=0, so the
  // copy of WAL frames into the database file and its fsync (half of a commit's cost when the writer
  // checkpoints itself) stay off the response path.  PASSIVE never blocks the writer.
  void ckpt_loop() {
    void* cdb = nullptr;
    if (sql.open_v2(cfg.sqlite_path.c_str(), &cdb, rtsql::OPEN_READWRITE | rtsql::OPEN_URI | rtsql::OPEN_NOMUTEX,
                    nullptr) != rtsql::OK) {
      if (cdb) sql.close(cdb);
      return;
    }
    sql.wait_on_locks(cdb);
    sql.exec(cdb, "PRAGMA synchronous=NORMAL", nullptr, nullptr, nullptr);
    long long seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(cmu);
        ccv.wait(lk, [&] { return ck_stop || commits != seen; });
        if (commits == seen && ck_stop) break;
        seen = commits;
      }
      int log = 0, ck = 0;
      sql.wal_checkpoint_v2(cdb, nullptr, rtsql::CHECKPOINT_PASSIVE, &log, &ck);
      std::unique_lock<std::mutex> lk(cmu);     // at most one checkpoint per 20 ms
      ccv.wait_for(lk, std::chrono::milliseconds(20), [&] { return ck_stop; });
    }
    int log = 0, ck = 0;
    sql.wal_checkpoint_v2(cdb, nullptr, rtsql::CHECKPOINT_PASSIVE, &log, &ck);
    sql.close(cdb);
  }
};

RouteService::RouteService(const RouteServiceCfg& cfg, std::function<void(RouteJob*)> done) : p_(new Impl) {
  p_->cfg = cfg;
  p_->done = std::move(done);
  if (cfg.provider == 1 && cfg.glat != nullptr) {
    p_->grid.build(cfg.glat, cfg.glon, (size_t)cfg.N, cfg.snap_c);
    const auto& shared = cfg.record_graph;
    if (shared && shared->ok() && shared->N == cfg.N && shared->glat == cfg.glat && shared->indptr == cfg.h_indptr &&
        shared->length == cfg.h_length) {
      p_->rg = shared;                 // the server's view of this same graph (its tables too)
    } else {
      p_->coord_cache.build(cfg.glat, cfg.glon, (size_t)cfg.N);
      if (cfg.h_indptr != nullptr && cfg.h_indices != nullptr) {
        const int64_t E = cfg.h_indptr[cfg.N];
        p_->edge_heading.resize((size_t)E);
        for (int u = 0; u < cfg.N; ++u)
          for (int32_t e = cfg.h_indptr[u]; e < cfg.h_indptr[u + 1]; ++e)
            p_->edge_heading[(size_t)e] = rtr::hop_heading(cfg.glat, cfg.glon, u, cfg.h_indices[e]);
      }
      if (cfg.h_length != nullptr && cfg.h_indptr != nullptr && cfg.h_indices != nullptr) {
        auto g = std::make_shared<rrec::RecordGraph>();
        const Impl* ip = p_;
        g->build(cfg.N, cfg.glat, cfg.glon, cfg.h_indptr, cfg.h_indices, cfg.h_length, cfg.h_edge_name,
                 &ip->cfg.names, &ip->coord_cache, ip->edge_heading.empty() ? nullptr : ip->edge_heading.data());
        if (g->ok()) p_->rg = g;
      }
    }
  }
  p_->th = std::thread([this] { p_->run(); });
}

RouteService::~RouteService() {
  {
    std::lock_guard<std::mutex> lk(p_->mu);
    p_->stop = true;
  }
  p_->cv.notify_all();
  if (p_->th.joinable()) p_->th.join();
  delete p_;
}

void RouteService::set_done_batch(std::function<void(std::vector<RouteJob*>&)> done_many) {
  p_->done_many = std::move(done_many);
}

bool RouteService::submit(RouteJob* j) {
  if (!j->parsed) {             // on the submitting reactor's thread: off the flush's critical path
    p_->n_jobs.fetch_add(1, std::memory_order_relaxed);
    Impl::parse_job(j);
  }
  {
    std::lock_guard<std::mutex> lk(p_->mu);
    if (p_->stop) return false;   // the run loop may have drained its queue already
    j->t_enq_us = now_us();
    p_->q.push_back(j);
  }
  p_->cv.notify_one();
  return true;
}

std::vector<long long> RouteService::stats() const {
  std::vector<long long> v = {p_->n_jobs.load(), p_->n_flushes.load(), p_->n_fallback.load(), p_->n_legs.load(),
                              p_->n_host_legs.load(), p_->n_persisted.load()};
  for (int k = 0; k < 8; ++k) v.push_back(p_->t_stage[k].load());
  v.push_back(p_->n_escalated.load());     // A* searches rerun in the big tier
  v.push_back(p_->n_ctx_built.load());     // routing contexts customized by this service (CCH)
  v.push_back(p_->t_ctx_us.load());        // ... and their cost + customization time (us)
  v.push_back(p_->n_legs_reused.load());   // legs that reused their matrix chains (meet + unpack only)
  v.push_back(p_->n_deferred.load());      // jobs that waited for their context's background build
  v.push_back(p_->t_wait_us.load());       // ... their total wait (us)
  v.push_back(p_->n_prefetch.load());      // next-week-hour contexts queued ahead of time
  v.push_back(p_->n_failed_over.load());   // jobs handed to another GPU's route service
  v.push_back(p_->n_records.load());       // rows persisted as compact route records
  v.push_back(p_->n_record_bytes.load());  // ... and their record bytes
  v.push_back(p_->t_collect_us.load());    // GPU thread: collecting flushes (us)
  v.push_back(p_->t_handoff_us.load());    // GPU thread: waiting for the assembly queue (us)
  return v;
}

bool RouteService::broken() const { return p_->broken.load();
}

}  // namespace rt
