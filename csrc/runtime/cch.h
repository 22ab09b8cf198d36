// Customizable contraction hierarchy (CCH) — host side.
//
// Replaces per-request road search (the reference's ORS directions + matrix calls,
// RO/Flaskr/utils.py:55-62,97-105,151-156) with a three-phase road router:
//
//   1. metric-INDEPENDENT preprocessing, once per graph (this file, host): a nested-dissection node
//      order (recursive geometric bisection with vertex separators), the chordal supergraph of the
//      road graph under that order (every node's upward neighbours form a clique), its elimination
//      tree (parent = lowest upward neighbour), node depths / heights and the level lists the
//      customization walks.  Everything is kept in RANK space: node r is the r-th contracted.
//   2. CUSTOMIZATION, once per metric (= per routing context: weather x traffic x week-hour):
//      basic (every arc gets the best path through lower nodes, bottom-up by etree height), then
//      perfect (best path through any node, top-down by etree depth) and pruning (an arc is kept
//      for queries only if its perfect weight equals its basic one — every shortest path then has
//      an up-down representation over kept arcs).  For unpacking each arc records the two sub-arcs
//      of its best lower triangle (first traversed downward, second upward) or its original edge,
//      and the metre length of the road path it stands for (the greedy's road-distance matrix).
//      GPU version: csrc/cch.hip (same tie rules, bit-identical results); this one is the CPU
//      reference and the same-box multi-thread CPU baseline.
//   3. QUERIES: elimination-tree search.  The forward search space of s is exactly its etree
//      ancestor chain; it is swept bottom-up once (no priority queue), distances indexed by etree
//      depth, and likewise the backward chain of t; the answer is the best common ancestor.
//      Many-to-many (the CVRP matrix) reuses each endpoint's chain for every pair.
//
// Tie rules shared with the GPU kernels (bit-identical answers):
//   * arc weights are (f32 weight, payload) pairs compared lexicographically; payload = middle node
//     rank z of a lower triangle (< 2^31) or 0x80000000 | original edge id — a triangle wins a tie
//     against an original edge, the lower z wins among triangles, the lower edge id among edges;
//   * sums are single f32 adds (no FMA); mins of the same candidate sets are order-independent;
//   * a chain sweep updates a label only on a strict improvement, sweeping from the deepest node
//     up, so the deepest predecessor wins a tie; the meeting node is the DEEPEST common ancestor
//     with the minimal sum.
#pragma once
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <future>
#include <limits>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

namespace rcch {

constexpr float INF = std::numeric_limits<float>::infinity();
constexpr uint32_t EDGE_FLAG = 0x80000000u;
constexpr uint32_t NO_PAYLOAD = 0xFFFFFFFFu;

inline uint64_t pack_w(float w, uint32_t payload) {
  uint32_t b;
  std::memcpy(&b, &w, 4);
  return ((uint64_t)b << 32) | payload;
}
inline float w_of(uint64_t p) {
  const uint32_t b = (uint32_t)(p >> 32);
  float w;
  std::memcpy(&w, &b, 4);
  return w;
}
constexpr uint64_t PACK_INF = 0x7F800000FFFFFFFFull;   // (+inf, no payload)

// ------------------------------------------------------------------------------------------------
// Persistent worker pool: run(n, fn) calls fn(i) for i in [0, n) over all workers (dynamic chunks)
// and returns when every call has finished.  Level-synchronous customization issues thousands of
// small rounds, so the workers are created once.
class Pool {
 public:
  explicit Pool(unsigned threads = 0) {
    unsigned t = threads ? threads : std::max(1u, std::thread::hardware_concurrency());
    for (unsigned k = 1; k < t; ++k) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return (unsigned)th_.size() + 1; }
  void run(size_t n, const std::function<void(size_t)>& fn, size_t grain = 1) {
    if (n == 0) return;
    if (th_.empty() || n <= grain) {
      for (size_t i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      grain_ = std::max<size_t>(1, grain);
      next_.store(0);
      busy_ = (unsigned)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    const auto* fn = fn_;
    while (true) {
      const size_t b = next_.fetch_add(grain_);
      if (b >= n_) break;
      const size_t e = std::min(n_, b + grain_);
      for (size_t i = b; i < e; ++i) (*fn)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0, grain_ = 1;
  std::atomic<size_t> next_{0};
  unsigned busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// ------------------------------------------------------------------------------------------------
// Metric-independent structure (rank space).
struct Topology {
  int N = 0;                       // nodes
  int64_t M = 0;                   // CCH arcs (lo < hi, undirected; two weights each)
  int64_t E = 0;                   // original directed edges
  std::vector<int32_t> rank;       // node id -> rank
  std::vector<int32_t> node;       // rank -> node id
  std::vector<int64_t> up_ptr;     // [N+1] arcs of lo = r: up_ptr[r] .. up_ptr[r+1]
  std::vector<int32_t> up_head;    // [M] hi rank (ascending within a lo: the first one is the parent)
  std::vector<int32_t> arc_lo;     // [M]
  std::vector<int64_t> dn_ptr;     // [N+1] lower neighbours of r (as arcs (z, r)), z ascending
  std::vector<int32_t> dn_tail;    // [M] z
  std::vector<int32_t> dn_arc;     // [M] arc id of (z, r)
  std::vector<int32_t> parent;     // [N] etree parent rank, -1 for a root
  std::vector<int32_t> depth;      // [N] etree depth (roots 0)
  std::vector<int32_t> height;     // [N] etree height (leaves 0)
  std::vector<int32_t> edge_arc;   // [E] arc of original edge e (-1: self loop)
  std::vector<uint8_t> edge_dir;   // [E] 0: travels lo -> hi (up), 1: hi -> lo (down)
  std::vector<int64_t> hlev_ptr;   // nodes by height: hlev_nodes[hlev_ptr[h] .. hlev_ptr[h+1])
  std::vector<int32_t> hlev_nodes;
  std::vector<int64_t> dlev_ptr;   // nodes by depth
  std::vector<int32_t> dlev_nodes;
  int max_depth = 0, max_height = 0, separator_top = 0;

  // arc id of {a, b} (any order), -1 if absent
  int64_t find_arc(int32_t a, int32_t b) const {
    if (a > b) std::swap(a, b);
    const int32_t* lo = up_head.data() + up_ptr[a];
    const int32_t* hi = up_head.data() + up_ptr[a + 1];
    const int32_t* p = std::lower_bound(lo, hi, b);
    return (p != hi && *p == b) ? (int64_t)(p - up_head.data()) : -1;
  }
};

// ------------------------------------------------------------------------------------------------
// Nested dissection order by recursive geometric bisection.  A region is split at the median of
// one of four projections (x, y, x+y, x-y); the vertex separator covers every cut edge (the smaller
// boundary side of the cut); the direction with the smallest separator wins.  Order of a region =
// order(part A) + order(part B) + separator (the separator ranks highest).
struct NDOptions {
  int leaf = 2;                 // regions this small are ordered as they are
  int parallel_min = 20000;     // regions this large recurse into their two halves concurrently
};

namespace detail {

struct NDCtx {
  int N;
  const int64_t* ptr;           // undirected, deduplicated adjacency
  const int32_t* adj;
  std::vector<double> x, y;
  std::vector<int32_t> mark;    // region stamp per node
  std::atomic<int32_t> stamp{1};
  NDOptions opt;
};

inline void nd_order(NDCtx& c, std::vector<int32_t> R, std::vector<int32_t>& out, int level, int* top_sep) {
  const size_t n = R.size();
  if ((int)n <= c.opt.leaf) {
    out.insert(out.end(), R.begin(), R.end());
    return;
  }
  const int32_t st = c.stamp.fetch_add(1);
  for (int32_t v : R) c.mark[v] = st;
  // connected components of the region: order each separately (no separator needed between them)
  {
    std::vector<int32_t> comp_of;
    std::vector<int32_t> seen_stack;
    const int32_t st2 = c.stamp.fetch_add(1);
    std::vector<std::vector<int32_t>> comps;
    for (int32_t v0 : R) {
      if (c.mark[v0] != st) continue;
      std::vector<int32_t> comp;
      seen_stack.clear();
      seen_stack.push_back(v0);
      c.mark[v0] = st2;
      while (!seen_stack.empty()) {
        const int32_t v = seen_stack.back();
        seen_stack.pop_back();
        comp.push_back(v);
        for (int64_t e = c.ptr[v]; e < c.ptr[v + 1]; ++e) {
          const int32_t u = c.adj[e];
          if (c.mark[u] == st) {
            c.mark[u] = st2;
            seen_stack.push_back(u);
          }
        }
      }
      comps.push_back(std::move(comp));
      if (comps.size() == 1 && comps[0].size() == n) break;
    }
    if (comps.size() > 1) {
      for (auto& cp : comps) nd_order(c, std::move(cp), out, level + 1, nullptr);
      return;
    }
    for (int32_t v : R) c.mark[v] = st;
  }
  // best of four directions
  static const double dirs[4][2] = {{1, 0}, {0, 1}, {0.7071067811865476, 0.7071067811865476},
                                    {0.7071067811865476, -0.7071067811865476}};
  std::vector<std::pair<double, int32_t>> key(n);
  std::vector<uint8_t> side_best, side(n);
  std::vector<int32_t> sep_best;
  size_t best = SIZE_MAX;
  std::vector<int32_t> pos_of;   // local index of node (valid for marked nodes)
  // local index via a map on the stamp array: store index in a side table
  std::vector<int32_t> local((size_t)0);
  // we need side per node: use a temporary global-indexed array only for this region's nodes
  thread_local std::vector<uint8_t> gside;
  if ((int)gside.size() < c.N) gside.assign(c.N, 0);
  for (int d = 0; d < 4; ++d) {
    for (size_t i = 0; i < n; ++i) key[i] = {c.x[R[i]] * dirs[d][0] + c.y[R[i]] * dirs[d][1], R[i]};
    const size_t half = n / 2;
    std::nth_element(key.begin(), key.begin() + half, key.end());
    for (size_t i = 0; i < n; ++i) gside[key[i].second] = i < half ? 0 : 1;
    std::vector<int32_t> b0, b1;
    for (int32_t v : R) {
      const uint8_t sv = gside[v];
      for (int64_t e = c.ptr[v]; e < c.ptr[v + 1]; ++e) {
        const int32_t u = c.adj[e];
        if (c.mark[u] == st && gside[u] != sv) {
          (sv ? b1 : b0).push_back(v);
          break;
        }
      }
    }
    std::vector<int32_t>& sep = b0.size() <= b1.size() ? b0 : b1;
    if (sep.size() < best) {
      best = sep.size();
      sep_best = sep;
      side_best.resize(n);
      for (size_t i = 0; i < n; ++i) side_best[i] = gside[R[i]];
    }
  }
  if (top_sep) *top_sep = (int)sep_best.size();
  // split: separator nodes leave their side
  const int32_t sst = c.stamp.fetch_add(1);
  for (int32_t v : sep_best) c.mark[v] = sst;
  std::vector<int32_t> A, B;
  A.reserve(n / 2 + 1);
  B.reserve(n / 2 + 1);
  for (size_t i = 0; i < n; ++i) {
    const int32_t v = R[i];
    if (c.mark[v] == sst) continue;
    (side_best[i] ? B : A).push_back(v);
  }
  if (A.empty() || B.empty()) {
    // degenerate split (e.g. all nodes at one point): no progress possible geometrically
    if (sep_best.empty() || sep_best.size() == n) {
      out.insert(out.end(), R.begin(), R.end());
      return;
    }
  }
  // separator order: along its own projection (a path in the etree)
  std::sort(sep_best.begin(), sep_best.end(), [&](int32_t a, int32_t b) {
    const double ka = c.x[a] + 0.5 * c.y[a], kb = c.x[b] + 0.5 * c.y[b];
    return ka < kb || (ka == kb && a < b);
  });
  R.clear();
  R.shrink_to_fit();
  if ((int)n >= c.opt.parallel_min) {
    std::vector<int32_t> oa;
    auto fut = std::async(std::launch::async, [&] { nd_order(c, std::move(A), oa, level + 1, nullptr); });
    std::vector<int32_t> ob;
    nd_order(c, std::move(B), ob, level + 1, nullptr);
    fut.get();
    out.insert(out.end(), oa.begin(), oa.end());
    out.insert(out.end(), ob.begin(), ob.end());
  } else {
    nd_order(c, std::move(A), out, level + 1, nullptr);
    nd_order(c, std::move(B), out, level + 1, nullptr);
  }
  out.insert(out.end(), sep_best.begin(), sep_best.end());
}

}  // namespace detail

// Build the topology.  indptr/indices: directed CSR (rows = source), lat/lon per node (degrees).
inline Topology build_topology(int N, const int32_t* indptr, const int32_t* indices, const double* lat,
                               const double* lon, const NDOptions& opt = NDOptions()) {
  Topology T;
  T.N = N;
  T.E = N > 0 ? indptr[N] : 0;
  // undirected, deduplicated adjacency (one-way streets still constrain the hierarchy both ways)
  std::vector<int64_t> uptr(N + 1, 0);
  std::vector<int32_t> uadj;
  {
    std::vector<std::vector<int32_t>> nb(N);
    for (int v = 0; v < N; ++v)
      for (int32_t e = indptr[v]; e < indptr[v + 1]; ++e) {
        const int32_t u = indices[e];
        if (u == v) continue;
        nb[v].push_back(u);
        nb[u].push_back(v);
      }
    for (int v = 0; v < N; ++v) {
      std::sort(nb[v].begin(), nb[v].end());
      nb[v].erase(std::unique(nb[v].begin(), nb[v].end()), nb[v].end());
      uptr[v + 1] = uptr[v] + (int64_t)nb[v].size();
    }
    uadj.resize(uptr[N]);
    for (int v = 0; v < N; ++v) std::copy(nb[v].begin(), nb[v].end(), uadj.begin() + uptr[v]);
  }
  // order
  detail::NDCtx c;
  c.N = N;
  c.ptr = uptr.data();
  c.adj = uadj.data();
  c.opt = opt;
  c.x.resize(N);
  c.y.resize(N);
  double mlat = 0.0;
  for (int v = 0; v < N; ++v) mlat += lat[v];
  mlat = N ? mlat / N : 0.0;
  const double cs = std::cos(mlat * 3.14159265358979323846 / 180.0);
  for (int v = 0; v < N; ++v) {
    c.x[v] = lon[v] * cs;
    c.y[v] = lat[v];
  }
  c.mark.assign(N, 0);
  std::vector<int32_t> all(N);
  std::iota(all.begin(), all.end(), 0);
  T.node.reserve(N);
  detail::nd_order(c, std::move(all), T.node, 0, &T.separator_top);
  T.rank.assign(N, -1);
  for (int r = 0; r < N; ++r) T.rank[T.node[r]] = r;
  // chordal completion along the order: merge each node's upward set minus its parent into the
  // parent's upward set (equivalent to making every upward set a clique)
  std::vector<std::vector<int32_t>> up(N);
  for (int v = 0; v < N; ++v) {
    const int32_t rv = T.rank[v];
    for (int64_t e = uptr[v]; e < uptr[v + 1]; ++e) {
      const int32_t ru = T.rank[uadj[e]];
      if (ru > rv) up[rv].push_back(ru);
    }
  }
  T.parent.assign(N, -1);
  for (int r = 0; r < N; ++r) {
    auto& u = up[r];
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    if (u.empty()) continue;
    const int32_t p = u[0];
    T.parent[r] = p;
    auto& pu = up[p];
    pu.insert(pu.end(), u.begin() + 1, u.end());
  }
  T.up_ptr.assign(N + 1, 0);
  for (int r = 0; r < N; ++r) T.up_ptr[r + 1] = T.up_ptr[r] + (int64_t)up[r].size();
  T.M = T.up_ptr[N];
  T.up_head.resize(T.M);
  T.arc_lo.resize(T.M);
  for (int r = 0; r < N; ++r) {
    std::copy(up[r].begin(), up[r].end(), T.up_head.begin() + T.up_ptr[r]);
    std::fill(T.arc_lo.begin() + T.up_ptr[r], T.arc_lo.begin() + T.up_ptr[r + 1], r);
    std::vector<int32_t>().swap(up[r]);
  }
  // downward lists (z ascending: arcs are visited in lo order)
  T.dn_ptr.assign(N + 1, 0);
  for (int64_t a = 0; a < T.M; ++a) T.dn_ptr[T.up_head[a] + 1]++;
  for (int r = 0; r < N; ++r) T.dn_ptr[r + 1] += T.dn_ptr[r];
  T.dn_tail.resize(T.M);
  T.dn_arc.resize(T.M);
  {
    std::vector<int64_t> fill(T.dn_ptr.begin(), T.dn_ptr.end() - 1);
    for (int64_t a = 0; a < T.M; ++a) {
      const int32_t h = T.up_head[a];
      T.dn_tail[fill[h]] = T.arc_lo[a];
      T.dn_arc[fill[h]] = (int32_t)a;
      ++fill[h];
    }
  }
  // depth (roots 0) and height (leaves 0)
  T.depth.assign(N, 0);
  for (int r = N - 1; r >= 0; --r) T.depth[r] = T.parent[r] < 0 ? 0 : T.depth[T.parent[r]] + 1;
  T.height.assign(N, 0);
  for (int r = 0; r < N; ++r)
    if (T.parent[r] >= 0) T.height[T.parent[r]] = std::max(T.height[T.parent[r]], T.height[r] + 1);
  T.max_depth = N ? *std::max_element(T.depth.begin(), T.depth.end()) : 0;
  T.max_height = N ? *std::max_element(T.height.begin(), T.height.end()) : 0;
  auto levels = [&](const std::vector<int32_t>& lv, int L, std::vector<int64_t>& ptr, std::vector<int32_t>& nodes) {
    ptr.assign(L + 2, 0);
    for (int r = 0; r < N; ++r) ptr[lv[r] + 1]++;
    for (int l = 0; l <= L; ++l) ptr[l + 1] += ptr[l];
    nodes.resize(N);
    std::vector<int64_t> f(ptr.begin(), ptr.end() - 1);
    for (int r = 0; r < N; ++r) nodes[f[lv[r]]++] = r;
  };
  levels(T.height, T.max_height, T.hlev_ptr, T.hlev_nodes);
  levels(T.depth, T.max_depth, T.dlev_ptr, T.dlev_nodes);
  // original edges -> arcs
  T.edge_arc.assign(T.E, -1);
  T.edge_dir.assign(T.E, 0);
  for (int v = 0; v < N; ++v)
    for (int32_t e = indptr[v]; e < indptr[v + 1]; ++e) {
      const int32_t u = indices[e];
      if (u == v) continue;
      const int32_t rv = T.rank[v], ru = T.rank[u];
      T.edge_arc[e] = (int32_t)T.find_arc(rv, ru);
      T.edge_dir[e] = rv < ru ? 0 : 1;
    }
  return T;
}

// ------------------------------------------------------------------------------------------------
// One customized metric.
struct Metric {
  std::vector<uint64_t> up, dn;    // basic (weight, payload): up = lo -> hi, dn = hi -> lo
  std::vector<int32_t> sub_up, sub_dn;   // [2M] (first traversed down, second traversed up) or (-1, edge)
  std::vector<float> len_up, len_dn;     // metres of the road path each arc stands for
  std::vector<float> pup, pdn;           // perfect weights
  // query graph: kept arcs by lo, forward (up weights) and backward (dn weights)
  std::vector<int64_t> f_ptr, b_ptr;     // [N+1]
  std::vector<int32_t> f_arc, b_arc;     // arc ids
  std::vector<float> f_w, b_w;           // their weights
  std::vector<int32_t> f_hd, b_hd;       // depth of the arc's hi end (the chain slot it relaxes)
  int64_t kept_f = 0, kept_b = 0;
};

// CPU customization: basic (pull over lower triangles, levels by height), lengths, perfect (pull over
// intermediate/upper triangles, levels by depth), pruning.  cost/length per original edge.
inline void customize(const Topology& T, const float* cost, const float* length, Metric& m, Pool& pool) {
  const int64_t M = T.M;
  m.up.assign(M, PACK_INF);
  m.dn.assign(M, PACK_INF);
  for (int64_t e = 0; e < T.E; ++e) {
    const int32_t a = T.edge_arc[e];
    if (a < 0) continue;
    const uint64_t p = pack_w(cost[e], EDGE_FLAG | (uint32_t)e);
    uint64_t& slot = T.edge_dir[e] ? m.dn[a] : m.up[a];
    if (p < slot) slot = p;
  }
  // basic: arcs of every node at height h depend only on arcs of its descendants (heights < h)
  for (int h = 0; h <= T.max_height; ++h) {
    const int64_t b = T.hlev_ptr[h], e = T.hlev_ptr[h + 1];
    pool.run((size_t)(e - b), [&](size_t i) {
      const int32_t u = T.hlev_nodes[b + i];
      const int64_t d0 = T.dn_ptr[u], d1 = T.dn_ptr[u + 1];
      for (int64_t a = T.up_ptr[u]; a < T.up_ptr[u + 1]; ++a) {
        const int32_t v = T.up_head[a];
        // lower triangles: z in down(u) ∩ down(v); arcs (z,u) and (z,v)
        int64_t i1 = d0, i2 = T.dn_ptr[v];
        const int64_t e2 = T.dn_ptr[v + 1];
        uint64_t bu = m.up[a], bd = m.dn[a];
        while (i1 < d1 && i2 < e2) {
          const int32_t z1 = T.dn_tail[i1], z2 = T.dn_tail[i2];
          if (z1 < z2) { ++i1; continue; }
          if (z2 < z1) { ++i2; continue; }
          const int32_t azu = T.dn_arc[i1], azv = T.dn_arc[i2];
          // u -> z -> v: u->z travels arc (z,u) downward, z->v travels (z,v) upward
          const float wu = w_of(m.dn[azu]) + w_of(m.up[azv]);
          // v -> z -> u
          const float wd = w_of(m.dn[azv]) + w_of(m.up[azu]);
          const uint64_t pu = pack_w(wu, (uint32_t)z1), pd = pack_w(wd, (uint32_t)z1);
          if (wu < INF && pu < bu) bu = pu;
          if (wd < INF && pd < bd) bd = pd;
          ++i1;
          ++i2;
        }
        m.up[a] = bu;
        m.dn[a] = bd;
      }
    }, 16);
  }
  // sub-arcs and lengths, bottom-up (sub-arcs are arcs of lower nodes)
  m.sub_up.assign(2 * M, -1);
  m.sub_dn.assign(2 * M, -1);
  m.len_up.assign(M, INF);
  m.len_dn.assign(M, INF);
  for (int h = 0; h <= T.max_height; ++h) {
    const int64_t b = T.hlev_ptr[h], e = T.hlev_ptr[h + 1];
    pool.run((size_t)(e - b), [&](size_t i) {
      const int32_t u = T.hlev_nodes[b + i];
      for (int64_t a = T.up_ptr[u]; a < T.up_ptr[u + 1]; ++a) {
        const int32_t v = T.up_head[a];
        for (int dir = 0; dir < 2; ++dir) {
          const uint64_t p = dir ? m.dn[a] : m.up[a];
          int32_t* sub = (dir ? m.sub_dn.data() : m.sub_up.data()) + 2 * a;
          float& len = dir ? m.len_dn[a] : m.len_up[a];
          const uint32_t pl = (uint32_t)p;
          if (w_of(p) == INF) continue;
          if (pl & EDGE_FLAG) {
            sub[0] = -1;
            sub[1] = (int32_t)(pl & ~EDGE_FLAG);
            len = length[sub[1]];
            continue;
          }
          const int32_t z = (int32_t)pl;
          const int32_t azu = (int32_t)T.find_arc(z, u), azv = (int32_t)T.find_arc(z, v);
          // up (u -> v): (z,u) down then (z,v) up;  down (v -> u): (z,v) down then (z,u) up
          sub[0] = dir ? azv : azu;
          sub[1] = dir ? azu : azv;
          len = m.len_dn[sub[0]] + m.len_up[sub[1]];
        }
      }
    }, 16);
  }
  // perfect: top-down by depth; for arc (x,y): candidates through every other upward neighbour z
  // of x (basic weights for x's own arcs, perfect ones for arcs between ancestors)
  m.pup.resize(M);
  m.pdn.resize(M);
  for (int64_t a = 0; a < M; ++a) {
    m.pup[a] = w_of(m.up[a]);
    m.pdn[a] = w_of(m.dn[a]);
  }
  for (int d = 0; d <= T.max_depth; ++d) {
    const int64_t b = T.dlev_ptr[d], e = T.dlev_ptr[d + 1];
    pool.run((size_t)(e - b), [&](size_t i) {
      const int32_t x = T.dlev_nodes[b + i];
      const int64_t a0 = T.up_ptr[x], a1 = T.up_ptr[x + 1];
      for (int64_t a = a0; a < a1; ++a) {
        const int32_t y = T.up_head[a];
        float bu = m.pup[a], bd = m.pdn[a];
        for (int64_t c = a0; c < a1; ++c) {
          if (c == a) continue;
          const int32_t z = T.up_head[c];
          const int64_t azy = T.find_arc(z, y);
          // x -> z (arc c up, basic), z -> y: arc {z,y} up if z < y else down
          const float xz = w_of(m.up[c]), zx = w_of(m.dn[c]);
          const float zy = z < y ? m.pup[azy] : m.pdn[azy];
          const float yz = z < y ? m.pdn[azy] : m.pup[azy];
          const float cu = xz + zy, cd = yz + zx;
          if (cu < bu) bu = cu;
          if (cd < bd) bd = cd;
        }
        m.pup[a] = bu;
        m.pdn[a] = bd;
      }
    }, 8);
  }
  // prune: keep an arc direction iff perfect == basic (and finite)
  const int N = T.N;
  m.f_ptr.assign(N + 1, 0);
  m.b_ptr.assign(N + 1, 0);
  for (int x = 0; x < N; ++x) {
    int64_t kf = 0, kb = 0;
    for (int64_t a = T.up_ptr[x]; a < T.up_ptr[x + 1]; ++a) {
      kf += m.pup[a] < INF && m.pup[a] == w_of(m.up[a]);
      kb += m.pdn[a] < INF && m.pdn[a] == w_of(m.dn[a]);
    }
    m.f_ptr[x + 1] = m.f_ptr[x] + kf;
    m.b_ptr[x + 1] = m.b_ptr[x] + kb;
  }
  m.kept_f = m.f_ptr[N];
  m.kept_b = m.b_ptr[N];
  m.f_arc.resize(m.kept_f);
  m.f_w.resize(m.kept_f);
  m.f_hd.resize(m.kept_f);
  m.b_arc.resize(m.kept_b);
  m.b_w.resize(m.kept_b);
  m.b_hd.resize(m.kept_b);
  pool.run((size_t)N, [&](size_t xi) {
    const int32_t x = (int32_t)xi;
    int64_t kf = m.f_ptr[x], kb = m.b_ptr[x];
    for (int64_t a = T.up_ptr[x]; a < T.up_ptr[x + 1]; ++a) {
      const int32_t hd = T.depth[T.up_head[a]];
      if (m.pup[a] < INF && m.pup[a] == w_of(m.up[a])) {
        m.f_arc[kf] = (int32_t)a;
        m.f_w[kf] = m.pup[a];
        m.f_hd[kf] = hd;
        ++kf;
      }
      if (m.pdn[a] < INF && m.pdn[a] == w_of(m.dn[a])) {
        m.b_arc[kb] = (int32_t)a;
        m.b_w[kb] = m.pdn[a];
        m.b_hd[kb] = hd;
        ++kb;
      }
    }
  }, 1024);
}

// ------------------------------------------------------------------------------------------------
// Queries.  A chain label per etree depth: (distance, arc that set it).
struct ChainScratch {
  std::vector<float> df, db;
  std::vector<int32_t> pf, pb;
  void ensure(int D) {
    if ((int)df.size() < D + 1) {
      df.assign(D + 1, INF);
      db.assign(D + 1, INF);
      pf.assign(D + 1, -1);
      pb.assign(D + 1, -1);
    }
  }
};

// sweep the chain of r (forward: up weights; backward: dn weights) into dist/pred by depth
inline void sweep(const Topology& T, const Metric& m, int32_t r, bool fwd, float* dist, int32_t* pred) {
  for (int d = 0; d <= T.depth[r]; ++d) {
    dist[d] = INF;
    pred[d] = -1;
  }
  dist[T.depth[r]] = 0.f;
  const std::vector<int64_t>& ptr = fwd ? m.f_ptr : m.b_ptr;
  const std::vector<int32_t>& arc = fwd ? m.f_arc : m.b_arc;
  const std::vector<float>& w = fwd ? m.f_w : m.b_w;
  const std::vector<int32_t>& hd = fwd ? m.f_hd : m.b_hd;
  for (int32_t x = r; x >= 0; x = T.parent[x]) {
    const float dx = dist[T.depth[x]];
    if (!(dx < INF)) continue;
    for (int64_t k = ptr[x]; k < ptr[x + 1]; ++k) {
      const float nd = dx + w[k];
      const int32_t slot = hd[k];
      if (nd < dist[slot]) {
        dist[slot] = nd;
        pred[slot] = arc[k];
      }
    }
  }
}

// the chain node (rank) at depth d of the chain of r (d <= depth[r])
inline int32_t chain_at(const Topology& T, int32_t r, int d) {
  while (T.depth[r] > d) r = T.parent[r];
  return r;
}

// Append the original-graph node ids of the path an arc stands for, traversed upward (lo -> hi,
// dir 0) or downward (hi -> lo, dir 1); the start node is NOT appended.
inline bool unpack_arc(const Topology& T, const Metric& m, int64_t a, int dir, std::vector<int32_t>& out,
                       size_t max_len) {
  // explicit stack of (arc, dir)
  std::vector<std::pair<int64_t, int>> st;
  st.emplace_back(a, dir);
  while (!st.empty()) {
    auto [x, d] = st.back();
    st.pop_back();
    const int32_t* sub = (d ? m.sub_dn.data() : m.sub_up.data()) + 2 * x;
    if (sub[0] < 0) {
      const int32_t lo = T.arc_lo[x], hi = T.up_head[x];
      out.push_back(T.node[d ? lo : hi]);
      if (out.size() > max_len) return false;
      continue;
    }
    // first sub[0] (traversed down) then sub[1] (traversed up): push in reverse
    st.emplace_back(sub[1], 0);
    st.emplace_back(sub[0], 1);
  }
  return true;
}

struct P2P {
  float sec = INF;
  float metres = INF;
  int status = 1;                 // 0 found, 1 unreachable, 4 path longer than max_path
  std::vector<int32_t> path;      // node ids, s .. t
};

// Point-to-point (node ids).  want_path: unpack to node ids.
inline void query(const Topology& T, const Metric& m, int32_t s_node, int32_t t_node, ChainScratch& cs, P2P& out,
                  bool want_path, size_t max_path = 1u << 20) {
  out = P2P();
  const int32_t s = T.rank[s_node], t = T.rank[t_node];
  cs.ensure(T.max_depth);
  sweep(T, m, s, true, cs.df.data(), cs.pf.data());
  sweep(T, m, t, false, cs.db.data(), cs.pb.data());
  // common ancestors: walk both chains to equal depth, then up together until they meet
  int32_t a = s, b = t;
  while (T.depth[a] > T.depth[b]) a = T.parent[a];
  while (T.depth[b] > T.depth[a]) b = T.parent[b];
  while (a != b && a >= 0 && b >= 0) {
    a = T.parent[a];
    b = T.parent[b];
  }
  if (a < 0 || a != b) return;    // different components
  float best = INF;
  int bestd = -1;
  for (int d = T.depth[a]; d >= 0; --d) {
    const float v = cs.df[d] + cs.db[d];
    if (v < best) {
      best = v;
      bestd = d;
    }
  }
  if (bestd < 0) return;
  out.sec = best;
  out.status = 0;
  // arc sequences: forward from the meeting node back to s, backward from it down to t
  const int32_t mnode = chain_at(T, a, bestd);
  std::vector<int64_t> fw, bw;
  float metres = 0.f;
  for (int32_t x = mnode; x != s;) {
    const int32_t arc = cs.pf[T.depth[x]];
    fw.push_back(arc);
    metres += m.len_up[arc];
    x = T.arc_lo[arc];
  }
  for (int32_t x = mnode; x != t;) {
    const int32_t arc = cs.pb[T.depth[x]];
    bw.push_back(arc);
    metres += m.len_dn[arc];
    x = T.arc_lo[arc];
  }
  out.metres = metres;
  if (!want_path) return;
  out.path.push_back(s_node);
  for (size_t i = fw.size(); i-- > 0;)
    if (!unpack_arc(T, m, fw[i], 0, out.path, max_path)) { out.status = 4; out.path.clear(); return; }
  for (size_t i = 0; i < bw.size(); ++i)
    if (!unpack_arc(T, m, bw[i], 1, out.path, max_path)) { out.status = 4; out.path.clear(); return; }
}

}  // namespace rcch
