// GPU customizable contraction hierarchy (csrc/cch.hip): customization per routing context and
// batched elimination-tree queries.  Host preprocessing and the bit-identical CPU reference:
// csrc/runtime/cch.h.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <list>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <vector>

#include "common.h"
#include "runtime/cch.h"

namespace rt {

// Routing context: the ETA features an edge cost depends on besides the edge itself
// (routing/graph.py edge_records).  weather: features.py weather code (0..3, 255 unknown);
// congestion: city-wide traffic level 0..3 (Low, Medium, High, Jam) shifting every edge's level;
// weekhour: 0 = Monday 00:00 .. 167.
struct CchContext {
  int weather = 2, congestion = 1, weekhour = 9;
  float driver_age = 35.f;
  uint64_t key() const {
    return (uint64_t)(weather & 0xFF) | ((uint64_t)(congestion & 0xFF) << 8) | ((uint64_t)(weekhour & 0xFFFF) << 16);
  }
};

// One customized metric, kept on the device for as long as its context stays cached.
struct CchMetricDev {
  uint64_t key = 0;
  int device = 0;
  float* cost = nullptr;           // [E] the edge costs it was customized from
  int32_t* sub_up = nullptr;       // [2M] per arc: (first sub-arc, traversed down; second, up) | (-1, edge)
  int32_t* sub_dn = nullptr;
  float* len_up = nullptr;         // [M] metres of the path an arc stands for
  float* len_dn = nullptr;
  int32_t* cnt_up = nullptr;       // [M] road edges the arc stands for (cooperative unpack)
  int32_t* cnt_dn = nullptr;
  int32_t* f_ptr = nullptr;        // [N+1] kept forward arcs of rank r
  int32_t* b_ptr = nullptr;
  int4* f_rec = nullptr;           // {weight bits, head depth, arc id, 0}
  int4* b_rec = nullptr;
  int64_t kept_f = 0, kept_b = 0;
  double customize_ms = 0.0, cost_ms = 0.0;
  double basic_ms = 0.0, perfect_ms = 0.0, prune_ms = 0.0;   // device time per phase
  double alloc_ms = 0.0, hostcopy_ms = 0.0;                    // its device allocations; the host copy
  std::vector<float> host_cost;    // [E] the costs on the host (filled by customize before publishing)
  ~CchMetricDev();
};

// Per-caller query scratch (chains of every job + the pairs' shortcut-arc lists); grows on demand.
struct CchScratch {
  float* dist = nullptr;
  int32_t* pred = nullptr;
  int32_t* node = nullptr;
  size_t jobs_cap = 0;
  int32_t* jobs = nullptr;         // [2 * cap] (rank << 1 | dir)
  int32_t* arcs = nullptr;         // [pairs_cap * max_arcs]
  int32_t* narcs = nullptr;        // [pairs_cap]
  size_t pairs_cap = 0;
  int32_t* pj = nullptr;           // [2 * pj_cap] leg job indices (legs_from_matrix)
  size_t pj_cap = 0;
  uint64_t chain_tag = 0;          // the matrix() call whose chains are in dist/pred/node (0: none)
  int chain_nm = 0, chain_r = 0;
  int device = 0;
  std::vector<void*> old;          // outgrown buffers, freed with the scratch
  ~CchScratch();
  hipError_t ensure(size_t jobs, size_t pairs, int stride, int max_arcs);
};

// Device temporaries of one customization (the up/down arc weights with middles, the perfect
// pass's packed words, the prune counts, the scan's temp, the context-cost records and minutes).
struct CustScratch {
  unsigned long long *up64 = nullptr, *dn64 = nullptr;
  uint32_t *pup = nullptr, *pdn = nullptr;
  int32_t *fcnt = nullptr, *bcnt = nullptr;
  void* cub = nullptr;
  size_t cub_bytes = 0;
  void* rec_buf = nullptr;                         // context cost records [2E]
  float* min_buf = nullptr;                        // their minutes [2E]
  float* h_stage = nullptr;                        // pinned [E]: the costs' host copy lands here first
  int* tail_ctl = nullptr;                         // basic_tail_kernel: cursor, timed-out flag, done[level]
  unsigned long long* sup_buf = nullptr;           // dense fronts of one supernode level (build_supernodes)
};

// The device pointers of one metric that the query kernels read — an array of these plus a group
// index per request row / leg lets ONE launch sequence serve a flush spread over many routing
// contexts (the *_multi calls below).
struct CchMView {
  const int32_t* f_ptr;
  const int32_t* b_ptr;
  const int4* f_rec;
  const int4* b_rec;
  const float* len_up;
  const float* len_dn;
  const int32_t* sub_up;
  const int32_t* sub_dn;
  const int32_t* cnt_up;
  const int32_t* cnt_dn;
};

struct CchRouteOut {
  float* sec = nullptr;            // [Q] seconds (-1 when not found)
  float* metres = nullptr;         // [Q] metres of the chosen path
  int* status = nullptr;           // [Q] 0 found, 1 unreachable, 4 too long / unpack overflow
  int* len = nullptr;              // [Q] path nodes
  int* path = nullptr;             // [Q, max_path] node ids (nullptr: costs only)
  int* edges = nullptr;            // [Q, max_path] the road edge of each hop (optional; with path)
  int max_path = 0;
};

class CchGpu {
 public:
  // T: host topology (kept); length: [E] metres per original edge; road_class / base_traffic: [E]
  // per-edge class (0..3) and traffic level before the context's shift (routing/graph.py
  // edge_traffic with congestion 1), for on-device context costs.
  CchGpu(rcch::Topology T, const float* length, const uint8_t* road_class, const uint8_t* base_traffic, int device);
  ~CchGpu();
  const rcch::Topology& topo() const { return T_; }
  int device() const { return dev_; }
  int stride() const { return T_.max_depth + 1; }
  bool has_triangle_table() const { return d_tri != nullptr; }
  int64_t triangles() const { return n_tri; }
  int64_t basic_tasks() const { return n_btask_; }
  int basic_tail_levels() const { return n_tail_lev_; }   // top basic levels run by ONE persistent launch
  int perfect_tail_levels() const { return n_ptail_lev_; }  // top perfect depths run by ONE persistent launch
  int64_t perfect_tasks() const { return n_ptask_; }
  // supernodal customization of the etree's top (csrc/cch.hip build_supernodes; ROUTEST_CCH_DENSE)
  bool supernodal() const { return sup_on_; }
  int sup_fronts() const { return sup_fronts_; }
  int sup_nodes() const { return sup_nodes_; }
  int sup_levels() const { return (int)sup_lev_.size(); }
  int sup_blocks() const { return sup_blocks_; }
  int sparse_heights() const { return sparse_heights_; }
  int sparse_depths() const { return (int)rlev_nodes_.size(); }

  // ETA model used for context costs (the fused K1+K2 kernel's 32x32 blob on this device)
  void set_eta(const void* blob, int H, const NormParams& np, int variant, int num_cus);
  bool has_eta() const { return eta_blob_ != nullptr; }
  // edge costs (s) of a context into d_cost [E] on the device (routing/graph.py edge_costs)
  hipError_t context_costs(const CchContext& c, float* d_cost, hipStream_t s, CustScratch* cs = nullptr);

  // customize m from d_cost ([E] on this device; copied into m.cost)
  hipError_t customize(const float* d_cost, CchMetricDev& m, hipStream_t s, CustScratch* cs = nullptr);

  // the metric of a context: from the cache, else costs + customization now (LRU, `capacity`)
  hipError_t metric_for(const CchContext& c, hipStream_t s, std::shared_ptr<CchMetricDev>& out, bool* fresh = nullptr,
                        CustScratch* cs = nullptr);
  // a metric from caller-given costs under a caller-chosen key (tests, benches)
  hipError_t metric_from_costs(uint64_t key, const float* d_cost, hipStream_t s, std::shared_ptr<CchMetricDev>& out);
  // a cached metric by key (no build); false if absent
  bool cached_metric(uint64_t key, std::shared_ptr<CchMetricDev>& out);
  // LRU size: a fixed count (set_capacity), or — the default — as many metrics as fit an HBM budget
  // (set_cache_gb; ROUTEST_CCH_CACHE_GB, default 48 of the 288 GB), re-derived from each built
  // metric's device bytes
  void set_capacity(int n) {
    std::lock_guard<std::mutex> lk(mu_);
    capacity_ = n < 1 ? 1 : n;
    cache_gb_ = 0.0;
  }
  void set_cache_gb(double gb);
  double cache_gb() { std::lock_guard<std::mutex> lk(mu_); return cache_gb_; }
  int capacity() { std::lock_guard<std::mutex> lk(mu_); return capacity_; }
  int64_t metric_bytes() const { return metric_bytes_.load(); }
  int cached() { std::lock_guard<std::mutex> lk(mu_); return (int)cache_.size(); }

  // Asynchronous context builds, off every query path: a builder thread customizes queued contexts
  // on its own lowest-priority stream (query launches on higher-priority streams overtake it) and
  // tells the listeners (key, ok) when each is cached.  request_build is a no-op for a context
  // that is queued or building; for one already cached the listeners are told at once (on the
  // caller's thread: a caller must not hold a lock its listener takes).  urgent: ahead of queued
  // prefetches (a request waits for it).
  void request_build(const CchContext& c, bool urgent = true);
  void start_builders();
  int add_build_listener(std::function<void(uint64_t, bool)> cb);
  void remove_build_listener(int id);
  struct AsyncStats {
    long long queued = 0, built = 0, failed = 0;
    int pending = 0;
    double build_ms = 0.0, alloc_ms = 0.0, hostcopy_ms = 0.0;   // summed over the background builds
    long long paced = 0;                                          // of which paced (queries were running)
  };
  AsyncStats async_stats();
  // background builds launch wide levels in pieces of at most n workgroups (0: whole levels) —
  // while queries are being served (note_queries in the last 250 ms), or always; default
  // ROUTEST_CCH_BUILDER_MAX_WG
  void set_builder_pacing(int n, bool always = false) {
    builder_max_wg_.store(n < 0 ? 0 : n);
    pace_always_.store(always);
  }
  int builder_pacing() const { return builder_max_wg_.load(); }
  // a query flush ran now (the route services call this per flush): builds starting within the next
  // 250 ms are paced
  void note_queries() {
    query_us_.store(std::chrono::duration_cast<std::chrono::microseconds>(
                        std::chrono::steady_clock::now().time_since_epoch()).count(),
                    std::memory_order_relaxed);
  }
  bool serving_now() const {
    const long long now = std::chrono::duration_cast<std::chrono::microseconds>(
                              std::chrono::steady_clock::now().time_since_epoch()).count();
    return now - query_us_.load(std::memory_order_relaxed) < 250000;
  }

  // point-to-point: node ids on the device
  hipError_t route(const CchMetricDev& m, const int* d_src, const int* d_dst, int Q, const CchRouteOut& o,
                   CchScratch& sc, hipStream_t s);
  // many-to-many per request: pts [R][NM] node ids (n = npts[r] used), outputs [R][NM][NM] (any may
  // be nullptr): seconds, metres (f32; both required) and metres as f64 (the greedy kernel's matrix, K6)
  hipError_t matrix(const CchMetricDev& m, const int* d_pts, const int* d_npts, int R, int NM, float* d_sec,
                    float* d_met, double* d_D64, CchScratch& sc, hipStream_t s);
  // legs between points of the matrix() call whose chains are still in `sc` (tag = sc.chain_tag
  // right after it): leg q = (request r[q], point i[q] -> point j[q]) starting at node d_src[q];
  // meet + unpack only, no sweeps
  hipError_t legs_from_matrix(const CchMetricDev& m, const int* d_src, const int* d_r, const int* d_i, const int* d_j,
                              int Q, uint64_t tag, const CchRouteOut& o, CchScratch& sc, hipStream_t s);
  static constexpr int MAX_ARCS = 1024;   // shortcut arcs per path before unpacking

  // The same over several metrics at once: d_mv [G] views (view(m), on the device), d_grp the
  // metric of each leg (route, legs_from_matrix) or request row (matrix).  Bit-identical per leg to
  // the single-metric calls.
  static CchMView view(const CchMetricDev& m) {
    return CchMView{m.f_ptr, m.b_ptr, m.f_rec, m.b_rec, m.len_up, m.len_dn, m.sub_up, m.sub_dn, m.cnt_up, m.cnt_dn};
  }
  hipError_t route_multi(const CchMView* d_mv, const int* d_grp, const int* d_src, const int* d_dst, int Q,
                         const CchRouteOut& o, CchScratch& sc, hipStream_t s);
  hipError_t matrix_multi(const CchMView* d_mv, const int* d_row_grp, const int* d_pts, const int* d_npts, int R, int NM,
                          float* d_sec, float* d_met, double* d_D64, CchScratch& sc, hipStream_t s);
  hipError_t legs_from_matrix_multi(const CchMView* d_mv, const int* d_grp, const int* d_src, const int* d_r,
                                    const int* d_i, const int* d_j, int Q, uint64_t tag, const CchRouteOut& o,
                                    CchScratch& sc, hipStream_t s);

 private:
  // m: one metric; else mv + grp (group of item idx = grp[idx / gdiv])
  hipError_t route_impl(const CchMetricDev* m, const CchMView* mv, const int* grp, const int* d_src, const int* d_dst,
                        int Q, const CchRouteOut& o, CchScratch& sc, hipStream_t s);
  hipError_t matrix_impl(const CchMetricDev* m, const CchMView* mv, const int* grp, const int* d_pts, const int* d_npts,
                         int R, int NM, float* d_sec, float* d_met, double* d_D64, CchScratch& sc, hipStream_t s);
  hipError_t legs_impl(const CchMetricDev* m, const CchMView* mv, const int* grp, const int* d_src, const int* d_r,
                       const int* d_i, const int* d_j, int Q, uint64_t tag, const CchRouteOut& o, CchScratch& sc,
                       hipStream_t s);
  hipError_t launch_unpack(const CchMetricDev* m, const CchMView* mv, const int* grp, int Q, const int* d_src,
                           CchScratch& sc, const CchRouteOut& o, hipStream_t s);
  rcch::Topology T_;
  int dev_ = 0;
  // topology on the device
  int32_t *d_up_ptr = nullptr, *d_up_head = nullptr, *d_arc_lo = nullptr, *d_parent = nullptr, *d_depth = nullptr;
  int32_t *d_rank = nullptr, *d_node = nullptr, *d_edge_arc = nullptr;
  uint8_t* d_edge_dir = nullptr;
  float* d_length = nullptr;
  uint8_t *d_class = nullptr, *d_base_traffic = nullptr;
  int32_t *d_hnodes = nullptr, *d_dnodes = nullptr;
  int64_t *d_bofs = nullptr, *d_pofs = nullptr;    // work-item prefixes in level order
  int64_t* d_aofs = nullptr;                       // arc prefix in depth order (perfect pull)
  void* d_parc = nullptr;                          // per depth-ordered arc: csrc/cch.hip PArc
  std::vector<int64_t> bofs_, pofs_, aofs_;        // host copies (level boundaries)
  std::vector<int> plev_kmax_;                     // widest node (upward arcs) per depth level
  // triangle table (metric-independent): for the pair (i < j) of rank z's upward arcs, the arc id of
  // {head i, head j} at tri[tofs[z] + i(2k-i-1)/2 + j-i-1] — the customization's binary searches
  // done once per graph (nullptr when it would not fit the ROUTEST_CCH_TRI_GB budget)
  int64_t* d_tofs = nullptr;
  int32_t* d_tri = nullptr;
  int64_t n_tri = 0;
  // task tables of the customization (csrc/cch.hip build_tasks): 8-byte wave tasks in level order
  void build_tasks(const std::vector<int64_t>& tofs);
  void build_pull_records(const std::vector<int64_t>& tofs);
  void* d_btask = nullptr;
  void* d_ptask = nullptr;
  std::vector<int64_t> btask_ptr_, ptask_ptr_;
  int64_t n_btask_ = 0, n_ptask_ = 0;
  // the basic phase's narrow top (levels h_tail_ .. max_height, each <= ROUTEST_CCH_TAIL tasks):
  // basic_tail_kernel, d_tail_end_[l] = end of tail level l's tasks (relative to h_tail_'s first)
  int h_tail_ = -1, n_tail_lev_ = 0, tail_max_tasks_ = 0;
  int* d_tail_end_ = nullptr;
  // ... and of the perfect phase (depths 0 .. n_ptail_lev_ - 1): perfect_tail_kernel over their arcs
  int n_ptail_lev_ = 0, ptail_max_arcs_ = 0;
  int* d_ptail_end_ = nullptr;
  // supernodal top: the chains of at least ROUTEST_CCH_DENSE nodes and every ancestor chain are dense
  // fronts, customized level by level of the supernode tree (csrc/cch.hip sup_*_kernel); the rest of
  // the nodes keep the per-level kernels (basic: the task table without the fronts' nodes; perfect:
  // the pull over d_parc2, by depth below the nearest front)
  void build_supernodes(const std::vector<int64_t>& tofs);
  struct SupRange {
    int64_t off = 0, cnt = 0;
  };
  struct SupLevel {
    SupRange gather;
    std::vector<SupRange> panel;                 // basic, per block step: panels | the block below's trailing
    std::vector<SupRange> px, py;                // perfect, per block from the top: K x K | product, solve
  };
  bool sup_on_ = false;
  std::vector<uint8_t> sup_node_;                  // [N] rank in a dense front
  std::vector<SupLevel> sup_lev_;
  void* d_sup_sn = nullptr;                        // SupNode per front
  void* d_sup_work = nullptr;                      // SupWork lists of every launch
  int32_t* d_sup_fnode = nullptr;                  // the fronts' node lists
  int32_t* d_sup_farc = nullptr;                   // the fronts' arc tables
  int64_t sup_buf_entries_ = 0;                    // dense entries of the largest level
  int sup_fronts_ = 0, sup_nodes_ = 0, sup_blocks_ = 0, sparse_heights_ = 0;
  void* d_parc2 = nullptr;                         // PArc of the other nodes, by depth below their front
  std::vector<int64_t> rlev_aofs_;
  std::vector<int> rlev_nodes_, rlev_kmax_;
  std::vector<uint8_t> rlev_multi_;                // a node of the level has >= 2 arcs
  // customization temporaries: cs0_ for callers on their own streams (one at a time: mu_cust_),
  // one set per background builder (no lock: each builder owns its set)
  hipError_t alloc_scratch(CustScratch& x);
  void free_scratch(CustScratch& x);
  CustScratch cs0_;
  std::vector<std::unique_ptr<CustScratch>> bscr_;
  std::mutex mu_cust_;
  // contexts being built (metric_for: another caller of the same context waits for it; different
  // contexts build concurrently)
  std::mutex mu_inflight_;
  std::condition_variable cv_inflight_;
  std::unordered_set<uint64_t> inflight_;
  // ETA
  const void* eta_blob_ = nullptr;
  int eta_H_ = 0, eta_variant_ = -1, eta_cus_ = 256;
  NormParams eta_np_{};
  // context cache (LRU)
  std::mutex mu_;
  std::list<std::shared_ptr<CchMetricDev>> cache_;
  int capacity_ = 32;
  double cache_gb_ = 48.0;
  std::atomic<int64_t> metric_bytes_{0};
  void insert_cached(const std::shared_ptr<CchMetricDev>& m);   // LRU push_front + eviction
  std::atomic<uint64_t> tag_ctr_{0};
  // asynchronous builds
  void builder_loop(int idx);
  void start_builders_locked();
  void notify_built(uint64_t key, bool ok);
  std::vector<std::thread> bths_;                  // ROUTEST_CCH_BUILDERS threads (default 3)
  std::mutex bmu_;
  std::condition_variable bcv_;
  std::deque<CchContext> bq_;
  std::unordered_set<uint64_t> bpending_;          // queued or building
  bool bstop_ = false;
  std::mutex lmu_;                                 // held while listeners run (removal waits)
  std::vector<std::pair<int, std::function<void(uint64_t, bool)>>> listeners_;
  int next_listener_ = 1;
  std::atomic<long long> n_bqueued_{0}, n_bbuilt_{0}, n_bfailed_{0};
  std::atomic<long long> us_build_{0}, us_alloc_{0}, us_hostcopy_{0};
  std::atomic<long long> query_us_{-(1LL << 40)};
  std::atomic<bool> pace_always_{false};
  std::atomic<long long> n_paced_{0};              // background builds that ran paced
  // -1 until the constructor picks the default: ROUTEST_CCH_BUILDER_MAX_WG if set, else 512 on a
  // city-scale hierarchy (>= 20M shortcut arcs: the 1M-node city's builds otherwise raised the
  // cached requests' p99 1.7x; paced, 1.03x at 2-4x the build time) and whole levels below that
  std::atomic<int> builder_max_wg_{[] {
    const char* v = std::getenv("ROUTEST_CCH_BUILDER_MAX_WG");
    return v ? std::max(0, std::atoi(v)) : -1;
  }()};
};

}  // namespace rt
