// GPU customizable contraction hierarchy: per-context customization + batched elimination-tree
// queries (SURVEY K9 "edge costs precomputed per (graph, context) and cached"; replaces the
// per-request ORS directions / matrix calls of RO/Flaskr/utils.py:55-62,97-105,151-156).
//
// Preprocessing (node order, chordal supergraph, elimination tree, levels) is host C++
// (csrc/runtime/cch.h) and metric-independent.  Everything here is per metric, all on the device:
//
//  * context costs: 2E ETA records (edge traffic level shifted by the context's congestion, the
//    context's weather and week-hour) -> the fused featurize+MLP kernel (K1+K2) -> seconds per edge;
//  * basic customization, one launch per etree HEIGHT level: every node z of the level relaxes all
//    pairs (u, v) of its upward clique (lower triangle z of arc {u,v}) with a 64-bit atomicMin on a
//    (weight bits, middle node) word — ties resolve deterministically, exactly like the CPU
//    reference — and the same launch finalizes the level's own arcs (their best triangle's two
//    sub-arcs and the metre length they stand for).  Work items are FLATTENED over the level (a
//    binary search maps an item to its node), so the top of the hierarchy — one node per level with
//    a clique of hundreds — still spreads over the whole chip;
//  * perfect customization, one launch per etree DEPTH level, top-down: every ordered pair (a, c) of
//    a node's arcs tests the intermediate/upper triangle through head(c); 32-bit atomicMin on the
//    float bits;
//  * pruning: an arc direction is kept for queries iff its perfect weight equals its basic one;
//    kept arcs are compacted into 16-byte records {weight, head depth, arc id} per node (hipCUB scan).
//
// Queries (csrc/runtime/cch.h "elimination-tree search"): the forward search space of s is its
// etree ancestor chain, swept bottom-up once with labels in LDS indexed by depth (one wave per chain
// job; runs of consecutive ranks — the separators — are fetched 64 at a time, so pointer chasing is
// per run, not per node).  A meet kernel takes each pair's two chains (one wave per pair: LCA by
// binary search on the chains' node arrays, min over common depths, deepest tie) and lists the
// shortcut arcs of the chosen up-down path; an unpack kernel expands them to road nodes (one lane
// per pair, explicit DFS stack in LDS).  Many-to-many matrices reuse each point's two chains.
#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "cch_gpu.h"
#include "ops.h"
#include "runtime/rt_core.h"

namespace rt {

namespace {

using EtaRecordDev = rtc::EtaRecord;
constexpr unsigned long long PACK_INF_D = 0x7F800000FFFFFFFFull;
constexpr uint32_t EDGE_FLAG_D = 0x80000000u;
constexpr float F_INF = __builtin_inff();

__device__ __forceinline__ unsigned long long packw(float w, uint32_t p) {
  return ((unsigned long long)__float_as_uint(w) << 32) | p;
}
__device__ __forceinline__ float wof(unsigned long long p) { return __uint_as_float((uint32_t)(p >> 32)); }

// position of b in the sorted upward list of a (a < b), -1 if absent
__device__ __forceinline__ int find_arc_d(const int32_t* __restrict__ up_ptr, const int32_t* __restrict__ up_head,
                                          int a, int b) {
  int lo = up_ptr[a], hi = up_ptr[a + 1];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (up_head[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  return (lo < up_ptr[a + 1] && up_head[lo] == b) ? lo : -1;
}

// largest i in [lo, hi) with ofs[i] <= g  (per item, from global memory: staging the block's slice of
// ofs in LDS and searching that instead measured the same level-kernel times, r4x — the levels are
// bound by their gathers and atomics, not by this search)
__device__ __forceinline__ int item_owner(const int64_t* __restrict__ ofs, int lo, int hi, long long g) {
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (ofs[mid] <= g) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ void fill_u64_kernel(unsigned long long* __restrict__ p, long long n, unsigned long long v) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ void edge_scatter_kernel(const float* __restrict__ cost, const int32_t* __restrict__ edge_arc,
                                    const uint8_t* __restrict__ edge_dir, int E, unsigned long long* __restrict__ up,
                                    unsigned long long* __restrict__ dn) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int a = edge_arc[e];
  if (a < 0) return;
  atomicMin(edge_dir[e] ? dn + a : up + a, packw(cost[e], EDGE_FLAG_D | (uint32_t)e));
}

struct LevelArgs {
  const int32_t* up_ptr;
  const int32_t* up_head;
  const int32_t* nodes;    // level-ordered node list
  const int64_t* ofs;      // item prefix over that list
  int lo, hi;              // node index range of this level
  long long base, items;
  const int64_t* tofs;     // triangle table (nullptr: binary search instead)
  const int32_t* tri;
};

// arc {head i, head j} of a node's upward pair (i < j): the triangle table, else a binary search
__device__ __forceinline__ int pair_arc(const LevelArgs& L, int z, int k, int i, int j, int u, int v) {
  if (L.tri != nullptr) return L.tri[L.tofs[z] + (long long)i * (2 * k - i - 1) / 2 + (j - i - 1)];
  return find_arc_d(L.up_ptr, L.up_head, u, v);
}

// one-time triangle table: item g -> (rank z, pair q) -> arc of the pair's heads
__global__ void tri_build_kernel(const int32_t* __restrict__ up_ptr, const int32_t* __restrict__ up_head,
                                 const int64_t* __restrict__ tofs, int N, long long T, int32_t* __restrict__ tri) {
  for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < T; g += (long long)gridDim.x * blockDim.x) {
    const int z = item_owner(tofs, 0, N, g);
    const long long q = g - tofs[z];
    const int a0 = up_ptr[z];
    const int k = up_ptr[z + 1] - a0;
    const double kk = (double)(2 * k - 1);
    int i = (int)((kk - sqrt(kk * kk - 8.0 * (double)q)) * 0.5);
    if (i < 0) i = 0;
    auto row0 = [&](int r) { return (long long)r * (2 * k - r - 1) / 2; };
    while (i > 0 && row0(i) > q) --i;
    while (i + 1 < k && row0(i + 1) <= q) ++i;
    const int j = (int)(q - row0(i)) + i + 1;
    tri[g] = find_arc_d(up_ptr, up_head, up_head[a0 + i], up_head[a0 + j]);
  }
}

// Basic customization of one height level: items [0, k) of node z finalize arc k-th of z; items
// [k, k + k(k-1)/2) relax the lower triangle z of one pair of z's upward neighbours.
// SKIP: a candidate is sent to the atomic only if it beats the target's current value (a plain load;
// a stale value is only ever larger, so nothing that could win is skipped) — most of a target's
// candidates lose, and the 64-bit atomics were the level kernels' L2 traffic (round 5)
template <bool SKIP>
__global__ __launch_bounds__(256) void basic_level_kernel(LevelArgs L, unsigned long long* __restrict__ up,
                                                          unsigned long long* __restrict__ dn,
                                                          int32_t* __restrict__ sub_up, int32_t* __restrict__ sub_dn,
                                                          float* __restrict__ len_up, float* __restrict__ len_dn,
                                                          int32_t* __restrict__ cnt_up, int32_t* __restrict__ cnt_dn,
                                                          const float* __restrict__ length) {
  const long long gi = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (gi >= L.items) return;
  const long long g = L.base + gi;
  const int ni = item_owner(L.ofs, L.lo, L.hi, g);
  const int z = L.nodes[ni];
  const long long p = g - L.ofs[ni];
  const int a0 = L.up_ptr[z];
  const int k = L.up_ptr[z + 1] - a0;
  if (p < k) {
    // finalize arc a = (z, v): best triangle's sub-arcs + lengths (all lower arcs are final)
    const int a = a0 + (int)p;
    const int v = L.up_head[a];
#pragma unroll
    for (int dir = 0; dir < 2; ++dir) {
      const unsigned long long w = dir ? dn[a] : up[a];
      int32_t* sub = (dir ? sub_dn : sub_up) + 2 * (long long)a;
      float* len = dir ? len_dn : len_up;
      int32_t* cnt = dir ? cnt_dn : cnt_up;
      if (!(wof(w) < F_INF)) {
        sub[0] = -1;
        sub[1] = -1;
        len[a] = F_INF;
        cnt[a] = 0;
        continue;
      }
      const uint32_t pl = (uint32_t)w;
      if (pl & EDGE_FLAG_D) {
        const int e = (int)(pl & ~EDGE_FLAG_D);
        sub[0] = -1;
        sub[1] = e;
        len[a] = length[e];
        cnt[a] = 1;
        continue;
      }
      const int zz = (int)pl;
      const int azu = find_arc_d(L.up_ptr, L.up_head, zz, z), azv = find_arc_d(L.up_ptr, L.up_head, zz, v);
      const int s0 = dir ? azv : azu, s1 = dir ? azu : azv;
      sub[0] = s0;
      sub[1] = s1;
      len[a] = len_dn[s0] + len_up[s1];
      cnt[a] = cnt_dn[s0] + cnt_up[s1];     // road edges the arc stands for (cooperative unpack)
    }
    return;
  }
  // pair (i, j), i < j, row-major over i
  const long long q = p - k;
  const double kk = (double)(2 * k - 1);
  int i = (int)((kk - sqrt(kk * kk - 8.0 * (double)q)) * 0.5);
  if (i < 0) i = 0;
  auto row0 = [&](int r) { return (long long)r * (2 * k - r - 1) / 2; };
  while (i > 0 && row0(i) > q) --i;
  while (i + 1 < k && row0(i + 1) <= q) ++i;
  const int j = (int)(q - row0(i)) + i + 1;
  const int ai = a0 + i, aj = a0 + j;
  const int u = L.up_head[ai], v = L.up_head[aj];
  const int t = pair_arc(L, z, k, i, j, u, v);
  if (t < 0) return;   // cannot happen in a chordal completion
  // u -> z -> v: (z,u) traversed down, (z,v) up;  v -> z -> u: (z,v) down, (z,u) up
  const float wu = wof(dn[ai]) + wof(up[aj]);
  const float wd = wof(dn[aj]) + wof(up[ai]);
  if (wu < F_INF) {
    const unsigned long long pu = packw(wu, (uint32_t)z);
    if (!SKIP || pu < up[t]) atomicMin(up + t, pu);
  }
  if (wd < F_INF) {
    const unsigned long long pd = packw(wd, (uint32_t)z);
    if (!SKIP || pd < dn[t]) atomicMin(dn + t, pd);
  }
}

__global__ void perfect_init_kernel(const unsigned long long* __restrict__ up, const unsigned long long* __restrict__ dn,
                                    uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn, long long M) {
  for (long long a = blockIdx.x * (long long)blockDim.x + threadIdx.x; a < M; a += (long long)gridDim.x * blockDim.x) {
    pup[a] = (uint32_t)(up[a] >> 32);
    pdn[a] = (uint32_t)(dn[a] >> 32);
  }
}

// Perfect customization of one depth level: ordered pairs (c, a), a != c, of node x's arcs; the
// candidate for arc a = (x, y) goes through z = head(c): x -> z on c (basic), z -> y on {z, y}
// (perfect: an arc between two ancestors, finished by an earlier level).  Consecutive items share c
// and spread over a (different atomic targets).
template <bool SKIP>
__global__ __launch_bounds__(256) void perfect_level_kernel(LevelArgs L, const unsigned long long* __restrict__ up,
                                                            const unsigned long long* __restrict__ dn,
                                                            uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  const long long gi = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (gi >= L.items) return;
  const long long g = L.base + gi;
  const int ni = item_owner(L.ofs, L.lo, L.hi, g);
  const int x = L.nodes[ni];
  const long long p = g - L.ofs[ni];
  const int a0 = L.up_ptr[x];
  const int k = L.up_ptr[x + 1] - a0;
  const int c = (int)(p / (k - 1));
  const int r = (int)(p % (k - 1));
  const int a = r < c ? r : r + 1;
  const int ac = a0 + c, aa = a0 + a;
  const int y = L.up_head[aa], z = L.up_head[ac];
  const int lo = z < y ? z : y, hi = z < y ? y : z;
  // upward lists are sorted by head, so the pair's order is the heads' order
  const int azy = pair_arc(L, x, k, c < a ? c : a, c < a ? a : c, lo, hi);
  if (azy < 0) return;
  const float xz = wof(up[ac]), zx = wof(dn[ac]);
  const float zy = __uint_as_float(z < y ? pup[azy] : pdn[azy]);
  const float yz = __uint_as_float(z < y ? pdn[azy] : pup[azy]);
  const float cu = xz + zy, cd = yz + zx;
  if (cu < F_INF && (!SKIP || __float_as_uint(cu) < pup[aa])) atomicMin(pup + aa, __float_as_uint(cu));
  if (cd < F_INF && (!SKIP || __float_as_uint(cd) < pdn[aa])) atomicMin(pdn + aa, __float_as_uint(cd));
}

// Perfect customization as a PULL over one depth level (round 5): every arc a = (x, y) of the
// level's nodes takes the min over x's other arcs c of the candidate through z = head(c), and is
// written once with a plain store — the level owns its arcs, so no atomics and no per-item decode.
// Same candidate set and fp32 sums as the push kernel / the CPU reference (bit-identical).
struct PullArgs {
  const int32_t* up_ptr;
  const int32_t* up_head;
  const int32_t* nodes;    // depth-ordered node list
  const int64_t* aofs;     // arc prefix over that list
  int lo, hi;              // node index range of the level
  long long base, arcs;    // arc range of the level
  const int64_t* tofs;     // triangle table (required)
  const int32_t* tri;
  // per depth-ordered arc: everything the pull needs before its candidate loads, in one load —
  // instead of the binary search over the level's nodes (a level of thousands of nodes searched ~12
  // dependent steps per wave) and the dependent loads of the node's arc range, triangle offset and
  // the arc's head; nullptr: search
  const struct PArc* parc;
};

struct PArc {
  int64_t tb;        // tofs[x]: the node's triangle table offset
  int32_t a0;        // x's first upward arc
  int32_t y;         // the arc's head
  uint16_t k;        // x's upward arcs
  uint16_t ia;       // the arc's index among them
  int32_t pad;
};
static_assert(sizeof(PArc) == 24, "pull arc record");

__device__ __forceinline__ void pull_cand(const PullArgs& P, long long tb, int k, int a0, int ia, int ic, float xz_c,
                                          float zx_c, const uint32_t* __restrict__ pup, const uint32_t* __restrict__ pdn,
                                          int y, int z, float& bu, float& bd) {
  const int i = ic < ia ? ic : ia, j = ic < ia ? ia : ic;
  const int azy = P.tri[tb + (long long)i * (2 * k - i - 1) / 2 + (j - i - 1)];
  const float zy = __uint_as_float(z < y ? pup[azy] : pdn[azy]);
  const float yz = __uint_as_float(z < y ? pdn[azy] : pup[azy]);
  const float cu = xz_c + zy, cd = yz + zx_c;
  bu = cu < bu ? cu : bu;
  bd = cd < bd ? cd : bd;
}

// The wave's minimum over candidate chunks c_begin, c_begin + c_step, ... of arc (x -> y) = x's arc
// ia (x: arcs a0 .. a0 + k, triangle rows at tb): four 64-wide chunks of candidates per step, every
// stage's loads issued together (the serial tri -> weight chain of a high-degree node's ~22 chunks
// was the kernel's latency); bu / bd are reduced over the wave.
__device__ __forceinline__ void pull_arc_min(const PullArgs& P, long long tb, int a0, int k, int ia, int y, int c_begin,
                                             int c_step, int lane, const unsigned long long* __restrict__ up,
                                             const unsigned long long* __restrict__ dn, const uint32_t* __restrict__ pup,
                                             const uint32_t* __restrict__ pdn, float& bu, float& bd) {
  for (int c0 = c_begin; c0 < k; c0 += c_step) {
    int azy[4], z[4];
    unsigned long long wu[4], wd[4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ic = c0 + 64 * u + lane;
      ok[u] = ic < k && ic != ia;
      const int i = ic < ia ? ic : ia, j = ic < ia ? ia : ic;
      azy[u] = ok[u] ? P.tri[tb + (long long)i * (2 * k - i - 1) / 2 + (j - i - 1)] : 0;
      z[u] = ok[u] ? P.up_head[a0 + ic] : 0;
      wu[u] = ok[u] ? up[a0 + ic] : 0ull;
      wd[u] = ok[u] ? dn[a0 + ic] : 0ull;
    }
    uint32_t gu[4], gd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      gu[u] = ok[u] ? pup[azy[u]] : 0u;
      gd[u] = ok[u] ? pdn[azy[u]] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!ok[u]) continue;
      const float zy = __uint_as_float(z[u] < y ? gu[u] : gd[u]);
      const float yz = __uint_as_float(z[u] < y ? gd[u] : gu[u]);
      const float cu = wof(wu[u]) + zy, cd = yz + wof(wd[u]);
      bu = cu < bu ? cu : bu;
      bd = cd < bd ? cd : bd;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ou = __shfl_xor(bu, o), od = __shfl_xor(bd, o);
    bu = ou < bu ? ou : bu;
    bd = od < bd ? od : bd;
  }
}

// S waves per arc (4 / S arcs per workgroup), lanes over the node's other arcs, wave `part` of an
// arc taking candidate chunks part, part + S, ... (levels of high-degree nodes: the top separators,
// k up to ~1400 on the 1M-node city — one wave walked ~6 chunks of 256 candidates one after the
// other; split, each wave walks k / (256 S)).  The parts' minima meet in LDS (min is exact and
// order-free: bit-identical to one wave).
template <int S>
__global__ __launch_bounds__(256) void perfect_pull_wave_kernel(PullArgs P, const unsigned long long* __restrict__ up,
                                                                const unsigned long long* __restrict__ dn,
                                                                uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  static_assert(S == 1 || S == 2 || S == 4, "waves per arc");
  constexpr int APB = 4 / S;
  __shared__ float red[2][4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long g = (long long)blockIdx.x * APB + w / S;
  const int part = w % S;
  const bool active = g < P.arcs;
  float bu = F_INF, bd = F_INF;
  int aa = 0;
  if (active) {
    int a0, k, ia, y;
    long long tb;
    if (P.parc != nullptr) {
      const PArc pa = P.parc[P.base + g];
      tb = pa.tb;
      a0 = pa.a0;
      y = pa.y;
      k = pa.k;
      ia = pa.ia;
      aa = a0 + ia;
    } else {
      const int ni = item_owner(P.aofs, P.lo, P.hi, P.base + g);
      const int x = P.nodes[ni];
      a0 = P.up_ptr[x];
      k = P.up_ptr[x + 1] - a0;
      ia = (int)(P.base + g - P.aofs[ni]);
      aa = a0 + ia;
      y = P.up_head[aa];
      tb = P.tofs[x];
    }
    pull_arc_min(P, tb, a0, k, ia, y, 256 * part, 256 * S, lane, up, dn, pup, pdn, bu, bd);
  }
  if constexpr (S > 1) {
    if (lane == 0) {
      red[0][w] = bu;
      red[1][w] = bd;
    }
    __syncthreads();
    if (part != 0) return;
#pragma unroll
    for (int q = 1; q < S; ++q) {
      const float ou = red[0][w + q], od = red[1][w + q];
      bu = ou < bu ? ou : bu;
      bd = od < bd ? od : bd;
    }
  }
  if (active && lane == 0) {
    const float cu = __uint_as_float(pup[aa]), cd = __uint_as_float(pdn[aa]);
    if (bu < cu) pup[aa] = __float_as_uint(bu);
    if (bd < cd) pdn[aa] = __float_as_uint(bd);
  }
}

// one lane per arc, looping over the node's other arcs (levels of low-degree nodes)
__global__ __launch_bounds__(256) void perfect_pull_lane_kernel(PullArgs P, const unsigned long long* __restrict__ up,
                                                                const unsigned long long* __restrict__ dn,
                                                                uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= P.arcs) return;
  int a0, k, ia, y;
  long long tb;
  if (P.parc != nullptr) {
    const PArc pa = P.parc[P.base + g];
    tb = pa.tb;
    a0 = pa.a0;
    y = pa.y;
    k = pa.k;
    ia = pa.ia;
  } else {
    const int ni = item_owner(P.aofs, P.lo, P.hi, P.base + g);
    const int x = P.nodes[ni];
    a0 = P.up_ptr[x];
    k = P.up_ptr[x + 1] - a0;
    ia = (int)(P.base + g - P.aofs[ni]);
    y = P.up_head[a0 + ia];
    tb = P.tofs[x];
  }
  const int aa = a0 + ia;
  float bu = __uint_as_float(pup[aa]), bd = __uint_as_float(pdn[aa]);
  for (int ic = 0; ic < k; ++ic) {
    if (ic == ia) continue;
    const int ac = a0 + ic;
    pull_cand(P, tb, k, a0, ia, ic, wof(up[ac]), wof(dn[ac]), pup, pdn, y, P.up_head[ac], bu, bd);
  }
  pup[aa] = __float_as_uint(bu);
  pdn[aa] = __float_as_uint(bd);
}

// The narrow top of the perfect phase (depths 0 .. d_tail - 1, each <= ROUTEST_CCH_TAIL arcs: the
// top separators' chains) in ONE launch: a wave per arc at a time, taken in depth order from a global
// cursor, the same bounded relaxed-poll dependency wait and loop shape as basic_tail_kernel (below).
// ctl: [0] cursor, [1] timed out, [2 ..] done per depth.
__global__ __launch_bounds__(256) void perfect_tail_kernel(PullArgs P, int narcs, const int* __restrict__ lvl_end, int nlev,
                                                           int* __restrict__ ctl, long long max_ticks,
                                                           const unsigned long long* __restrict__ up,
                                                           const unsigned long long* __restrict__ dn,
                                                           uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  const int lane = threadIdx.x & 63;
  int* cursor = ctl;
  int* fail = ctl + 1;
  int* done = ctl + 2;
  int lev = 0, prev = -1;
  while (true) {
    int got = 0;
    if (lane == 0) {
      if (prev >= 0) __hip_atomic_fetch_add(done + prev, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      got = atomicAdd(cursor, 1);
    }
    const int ti = __builtin_amdgcn_readlane(got, 0);
    if (ti >= narcs) break;
    while (lev < nlev - 1 && ti >= lvl_end[lev]) ++lev;
    if (lev > 0) {
      int f = 0;
      if (lane == 0) {
        const int need = lvl_end[lev - 1] - (lev >= 2 ? lvl_end[lev - 2] : 0);
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(done + lev - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
          if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
              (long long)__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) {
            __hip_atomic_fetch_or(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            f = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
      }
      if (__builtin_amdgcn_readlane(f, 0)) break;
    }
    const PArc pa = P.parc[P.base + ti];
    const int aa = pa.a0 + pa.ia;
    float bu = F_INF, bd = F_INF;
    pull_arc_min(P, pa.tb, pa.a0, pa.k, pa.ia, pa.y, 0, 256, lane, up, dn, pup, pdn, bu, bd);
    if (lane == 0) {
      const float cu = __uint_as_float(pup[aa]), cd = __uint_as_float(pdn[aa]);
      if (bu < cu) pup[aa] = __float_as_uint(bu);
      if (bd < cd) pdn[aa] = __float_as_uint(bd);
    }
    prev = lev;
  }
}

// ---- task-table customization (round 5) ----
// A wave's work is one precomputed, metric-independent TASK (8 bytes, built once per graph in level
// order): {node, row/arc index, first column}; its 64 lanes take 64 consecutive columns.  That
// replaces the per-item chain of the flattened kernels (binary search for the item's node, node id,
// arc range, the pair decode by sqrt) — which made every wave a ~6-deep chain of dependent global
// loads — by one scalar load of the task and one of the node's arc range, and the lanes' loads are
// coalesced along a row of the triangle table.
struct CustTask {
  int32_t node;
  uint16_t row;      // basic: pair row i (ROW_FINAL: the node's own arcs); perfect: the target arc's index
  uint16_t col0;     // first column (c or j) of the wave's 64
};
constexpr uint16_t ROW_FINAL = 0xFFFF;

// A basic-customization task with its node's arc range and its triangle row's base folded in (24
// bytes): the wave's first load gives everything the triangle and weight loads need — the 8-byte
// task cost one more dependent round trip (the node's arc range and triangle offset) per level.
struct BasicTask {
  int64_t rowbase;   // pair rows: tofs[z] + i (2k - i - 1) / 2 - i - 1 (column j's triangle at rowbase + j)
  int32_t node;
  int32_t a0;        // z's first upward arc
  uint16_t k;        // z's upward arcs
  uint16_t row;      // pair row i, or ROW_FINAL
  uint16_t col0;     // first column of the wave's 64
  uint16_t pad;
};
static_assert(sizeof(BasicTask) == 24, "basic task layout");

// Basic customization of one height level, one task per wave: a pair row (i, j0 .. j0+63) of node
// z relaxes its lower triangles z of the arcs {head i, head j}; a ROW_FINAL task finalizes 64 of
// z's own arcs (best triangle's two sub-arcs, metres, road-edge counts).  Same math as
// basic_level_kernel (bit-identical).
template <bool SKIP>
__device__ __forceinline__ void basic_task_run(const BasicTask& T, int lane, const int32_t* __restrict__ up_ptr,
                                               const int32_t* __restrict__ up_head,
                                               const int32_t* __restrict__ tri, unsigned long long* __restrict__ up,
                                               unsigned long long* __restrict__ dn, int32_t* __restrict__ sub_up,
                                               int32_t* __restrict__ sub_dn, float* __restrict__ len_up,
                                               float* __restrict__ len_dn, int32_t* __restrict__ cnt_up,
                                               int32_t* __restrict__ cnt_dn, const float* __restrict__ length) {
  const int z = T.node;
  const int a0 = T.a0;
  const int k = T.k;
  if (T.row == ROW_FINAL) {
    const int p = T.col0 + lane;
    if (p >= k) return;
    const int a = a0 + p;
    const int v = up_head[a];
#pragma unroll
    for (int dir = 0; dir < 2; ++dir) {
      const unsigned long long w = dir ? dn[a] : up[a];
      int32_t* sub = (dir ? sub_dn : sub_up) + 2 * (long long)a;
      float* len = dir ? len_dn : len_up;
      int32_t* cnt = dir ? cnt_dn : cnt_up;
      if (!(wof(w) < F_INF)) {
        sub[0] = -1;
        sub[1] = -1;
        len[a] = F_INF;
        cnt[a] = 0;
        continue;
      }
      const uint32_t pl = (uint32_t)w;
      if (pl & EDGE_FLAG_D) {
        const int e = (int)(pl & ~EDGE_FLAG_D);
        sub[0] = -1;
        sub[1] = e;
        len[a] = length[e];
        cnt[a] = 1;
        continue;
      }
      const int zz = (int)pl;
      const int azu = find_arc_d(up_ptr, up_head, zz, z), azv = find_arc_d(up_ptr, up_head, zz, v);
      const int s0 = dir ? azv : azu, s1 = dir ? azu : azv;
      sub[0] = s0;
      sub[1] = s1;
      len[a] = len_dn[s0] + len_up[s1];
      cnt[a] = cnt_dn[s0] + cnt_up[s1];
    }
    return;
  }
  const int i = T.row;
  const int j = T.col0 + lane;
  if (j >= k) return;
  const int ai = a0 + i, aj = a0 + j;
  const int t = tri[T.rowbase + j];
  if (t < 0) return;
  const float wu = wof(dn[ai]) + wof(up[aj]);
  const float wd = wof(dn[aj]) + wof(up[ai]);
  if (wu < F_INF) {
    const unsigned long long pu = packw(wu, (uint32_t)z);
    if (!SKIP || pu < up[t]) atomicMin(up + t, pu);
  }
  if (wd < F_INF) {
    const unsigned long long pd = packw(wd, (uint32_t)z);
    if (!SKIP || pd < dn[t]) atomicMin(dn + t, pd);
  }
}

template <bool SKIP>
__global__ __launch_bounds__(256) void basic_task_kernel(const BasicTask* __restrict__ tasks, long long ntask,
                                                         const int32_t* __restrict__ up_ptr,
                                                         const int32_t* __restrict__ up_head,
                                                         const int64_t* __restrict__ tofs, const int32_t* __restrict__ tri,
                                                         unsigned long long* __restrict__ up,
                                                         unsigned long long* __restrict__ dn, int32_t* __restrict__ sub_up,
                                                         int32_t* __restrict__ sub_dn, float* __restrict__ len_up,
                                                         float* __restrict__ len_dn, int32_t* __restrict__ cnt_up,
                                                         int32_t* __restrict__ cnt_dn, const float* __restrict__ length) {
  const long long ti = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ti >= ntask) return;
  (void)tofs;
  basic_task_run<SKIP>(tasks[ti], threadIdx.x & 63, up_ptr, up_head, tri, up, dn, sub_up, sub_dn, len_up, len_dn,
                       cnt_up, cnt_dn, length);
}

// The narrow top of the basic phase in ONE launch (round 6): the levels
// [h_tail, max_height] each hold few tasks (the top separator's chain: one node per level), and as
// separate kernels each cost a dependent launch (~2.6 us) plus its ramp, ~12 us per level in all
// (profiles/cch_customize_r5.md).  Here every WAVE is an independent worker: lane 0 takes the next
// task index from a global cursor (tasks in level order), and before a task of tail level l > 0 waits
// until every task of level l - 1 is done (done[l - 1] == its task count), polling with RELAXED
// agent-scope loads and one acquire fence after (an acquire poll invalidates the XCD's L2 on every
// iteration); finishing a task is a release increment of done[l].  Deadlock-free without co-residency:
// a waiting wave only waits for tasks taken earlier, by running waves, down to level 0, whose
// predecessors ran in earlier launches.  Every wait is bounded by wall clock (s_memrealtime, 100 MHz):
// on expiry ctl[1] is set, every wave leaves, and the host reports the customization failed.
// The loop's exits test wave-uniform values, and lane 0's release of one task and fetch of the next
// are ONE block before the loop's work: lane-0 code on both sides of the back edge lets the AMDGPU
// structurizer split the loop per lane, which livelocked the r5t work-queue probe
// (tools/probes/kernel_chain_probe.hip).  ctl: [0] cursor, [1] timed out, [2 ..] done per tail level.
template <bool SKIP>
__global__ __launch_bounds__(256) void basic_tail_kernel(const BasicTask* __restrict__ tasks, int ntask,
                                                         const int* __restrict__ lvl_end, int nlev,
                                                         int* __restrict__ ctl, long long max_ticks,
                                                         const int32_t* __restrict__ up_ptr,
                                                         const int32_t* __restrict__ up_head,
                                                         const int32_t* __restrict__ tri,
                                                         unsigned long long* __restrict__ up,
                                                         unsigned long long* __restrict__ dn, int32_t* __restrict__ sub_up,
                                                         int32_t* __restrict__ sub_dn, float* __restrict__ len_up,
                                                         float* __restrict__ len_dn, int32_t* __restrict__ cnt_up,
                                                         int32_t* __restrict__ cnt_dn, const float* __restrict__ length) {
  const int lane = threadIdx.x & 63;
  int* cursor = ctl;
  int* fail = ctl + 1;
  int* done = ctl + 2;
  int lev = 0;             // tail level of the wave's current task (task indices only grow)
  int prev = -1;           // tail level of the task finished in the previous iteration
  while (true) {
    int got = 0;
    if (lane == 0) {
      if (prev >= 0) __hip_atomic_fetch_add(done + prev, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      got = atomicAdd(cursor, 1);
    }
    const int ti = __builtin_amdgcn_readlane(got, 0);
    if (ti >= ntask) break;
    while (lev < nlev - 1 && ti >= lvl_end[lev]) ++lev;
    if (lev > 0) {
      int f = 0;
      if (lane == 0) {
        const int need = lvl_end[lev - 1] - (lev >= 2 ? lvl_end[lev - 2] : 0);
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(done + lev - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
          if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
              (long long)__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) {
            __hip_atomic_fetch_or(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            f = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
      }
      if (__builtin_amdgcn_readlane(f, 0)) break;
    }
    basic_task_run<SKIP>(tasks[ti], lane, up_ptr, up_head, tri, up, dn, sub_up, sub_dn, len_up, len_dn, cnt_up,
                         cnt_dn, length);
    prev = lev;
  }
}

// Perfect customization of one depth level, one task per wave: target arc a = (x, y) of node x
// and 64 of x's other arcs c as candidates (through z = head(c)); the wave's min goes to the
// target with one atomicMin (only if it beats the current value) — 64x fewer atomics than the
// push kernel, and no serial loop over c as in the one-wave-per-arc pull.
__global__ __launch_bounds__(256) void perfect_task_kernel(const CustTask* __restrict__ tasks, long long ntask,
                                                           const int32_t* __restrict__ up_ptr,
                                                           const int32_t* __restrict__ up_head,
                                                           const int64_t* __restrict__ tofs,
                                                           const int32_t* __restrict__ tri,
                                                           const unsigned long long* __restrict__ up,
                                                           const unsigned long long* __restrict__ dn,
                                                           uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  const long long ti = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ti >= ntask) return;
  const int lane = threadIdx.x & 63;
  const CustTask T = tasks[ti];
  const int x = T.node;
  const int a0 = up_ptr[x];
  const int k = up_ptr[x + 1] - a0;
  const int ia = T.row;
  const int aa = a0 + ia;
  const int y = up_head[aa];
  const int ic = T.col0 + lane;
  float bu = F_INF, bd = F_INF;
  if (ic < k && ic != ia) {
    const int ac = a0 + ic;
    const int z = up_head[ac];
    const int i = ic < ia ? ic : ia, j = ic < ia ? ia : ic;
    const int azy = tri[tofs[x] + (long long)i * (2 * k - i - 1) / 2 + (j - i - 1)];
    const float zy = __uint_as_float(z < y ? pup[azy] : pdn[azy]);
    const float yz = __uint_as_float(z < y ? pdn[azy] : pup[azy]);
    bu = wof(up[ac]) + zy;
    bd = yz + wof(dn[ac]);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ou = __shfl_xor(bu, o), od = __shfl_xor(bd, o);
    bu = ou < bu ? ou : bu;
    bd = od < bd ? od : bd;
  }
  if (lane == 0) {
    if (bu < F_INF && __float_as_uint(bu) < pup[aa]) atomicMin(pup + aa, __float_as_uint(bu));
    if (bd < F_INF && __float_as_uint(bd) < pdn[aa]) atomicMin(pdn + aa, __float_as_uint(bd));
  }
}

__device__ __forceinline__ bool kept(uint32_t p, unsigned long long b) {
  return __uint_as_float(p) < F_INF && p == (uint32_t)(b >> 32);
}

// Pruning, one wave per node: lanes over its arcs (coalesced), ballot counts and in-order
// positions (round 5; a thread per node walking its arcs serially took 1.5 ms per customization
// on the 100k graph)
__global__ __launch_bounds__(256) void prune_count_wave_kernel(const int32_t* __restrict__ up_ptr,
                                                               const uint32_t* __restrict__ pup,
                                                               const uint32_t* __restrict__ pdn,
                                                               const unsigned long long* __restrict__ up,
                                                               const unsigned long long* __restrict__ dn, int N,
                                                               int32_t* __restrict__ fcnt, int32_t* __restrict__ bcnt) {
  const int x = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (x >= N) return;
  int kf = 0, kb = 0;
  for (int a = up_ptr[x] + lane; a < up_ptr[x + 1]; a += 64) {
    kf += kept(pup[a], up[a]);
    kb += kept(pdn[a], dn[a]);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    kf += __shfl_xor(kf, o);
    kb += __shfl_xor(kb, o);
  }
  if (lane == 0) {
    fcnt[x] = kf;
    bcnt[x] = kb;
  }
}

__global__ __launch_bounds__(256) void prune_scatter_wave_kernel(
    const int32_t* __restrict__ up_ptr, const int32_t* __restrict__ up_head, const int32_t* __restrict__ depth,
    const uint32_t* __restrict__ pup, const uint32_t* __restrict__ pdn, const unsigned long long* __restrict__ up,
    const unsigned long long* __restrict__ dn, int N, const int32_t* __restrict__ f_ptr, const int32_t* __restrict__ b_ptr,
    int4* __restrict__ f_rec, int4* __restrict__ b_rec) {
  const int x = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (x >= N) return;
  int kf = f_ptr[x], kb = b_ptr[x];
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int a0 = up_ptr[x]; a0 < up_ptr[x + 1]; a0 += 64) {
    const int a = a0 + lane;
    const bool in = a < up_ptr[x + 1];
    const bool f = in && kept(pup[a], up[a]);
    const bool b = in && kept(pdn[a], dn[a]);
    const unsigned long long mf = __ballot(f), mb = __ballot(b);
    if (f || b) {
      const int hd = depth[up_head[a]];        // records in arc order, like the serial kernel
      if (f) f_rec[kf + __popcll(mf & below)] = make_int4((int)pup[a], hd, a, 0);
      if (b) b_rec[kb + __popcll(mb & below)] = make_int4((int)pdn[a], hd, a, 0);
    }
    kf += __popcll(mf);
    kb += __popcll(mb);
  }
}

// ---- supernodal customization of the top of the elimination tree (round 6) ----
// The top ~80 % of the etree levels are the nested-dissection separators: CHAINS of nodes (each the
// only child of the next), one etree level per node, so the per-level kernels above walk them one
// ~12 us level at a time (963 levels per phase on the 100k graph, profiles/cch_customize_r6.md).
// A chain with its upper set is a dense FRONT (chordality: every chain node's upward arcs lead into
// the chain above it or into the top node's upward set), and its customization is dense (min, +)
// elimination: basic = tropical Gaussian elimination of the chain's pivots (a triangle z of pair
// {u, v} is "pivot z updates D[u][v]"), perfect = tropical back substitution from the top.  Blocked
// 32 pivots at a time, a level of the supernode tree takes 2 (basic) / 3 (perfect) launches per
// block instead of one launch per node — and every candidate is the same single f32 add of the
// same two operands as in the per-level kernels (min is exact and order-free), so the results are
// bit-identical to them and to the CPU reference (csrc/runtime/cch.h).
// A front's D is row-major n x n over its nodes in rank order (chain c0 .. c0 + m - 1 first, then
// the top's upward set): D[i][j] = weight f_i -> f_j — basic: the packed (weight, middle) word,
// perfect: two f32 matrices (basic Db, perfect P) in the same bytes.  farc[i][j]: the arc of
// {f_i, f_j} (-1: none).  Entries between two upper-set nodes (U x U) are only ever TARGETS here
// (their arcs belong to an ancestor front): basic sends them with one atomicMin each at the end.
struct SupNode {
  int64_t dofs;      // first entry of the front in the level's dense buffer
  int64_t foff;      // first entry of its farc table
  int32_t c0, m, n;  // first chain rank, chain length, front size
  int32_t fnode;     // offset of its node list
};
struct SupWork {
  int32_t s, b, t0, t1;   // supernode, block (or row), tile indices
  SupNode sn;             // the front itself (one load per workgroup instead of two dependent ones)
};
constexpr int SUP_B = 32;      // pivots per block
constexpr int SUP_PJ = 32;     // basic panel: front columns per workgroup
constexpr int SUP_TT = 64;     // basic trailing update: 64 x 64 targets per workgroup
constexpr int SUP_G1Y = 32;    // perfect GEMM: 32 output columns per workgroup
constexpr int SUP_G1Z = 128;   // ... over at most 128 intermediate nodes (more: split, atomicMin)
constexpr int SUP_SJ = 64;     // perfect solve: front columns per workgroup

__device__ __forceinline__ unsigned long long sup_cand(unsigned long long a, unsigned long long b, uint32_t z) {
  const float w = wof(a) + wof(b);
  return w < F_INF ? packw(w, z) : PACK_INF_D;
}
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return b < a ? b : a; }

// farc of every front row (once per graph): a wave per row
__global__ __launch_bounds__(256) void sup_farc_kernel(const SupNode* __restrict__ sn, const SupWork* __restrict__ w,
                                                       long long nw, const int32_t* __restrict__ fnode,
                                                       const int32_t* __restrict__ up_ptr,
                                                       const int32_t* __restrict__ up_head, int32_t* __restrict__ farc) {
  const long long wi = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wi >= nw) return;
  const SupWork W = w[wi];
  const SupNode S = W.sn;
  const int i = W.b, n = S.n;
  const int fi = fnode[S.fnode + i];
  for (int j = threadIdx.x & 63; j < n; j += 64) {
    const int fj = fnode[S.fnode + j];
    farc[S.foff + (long long)i * n + j] = i == j ? -1 : find_arc_d(up_ptr, up_head, fi < fj ? fi : fj, fi < fj ? fj : fi);
  }
}

// basic: a front's rows from the arc weights (all lower levels are done; U x U starts at +inf), a
// workgroup per row.  An entry whose best triangle so far has a middle node (necessarily below the
// front: no pivot of it has run) also gets that triangle's finalization now — sub-arcs by binary
// search, metres, road edges — in SS / SL: the elimination only adds middles from the chain, so if
// the entry still has this middle at the end, the panel takes it from here (off its serial path).
__global__ __launch_bounds__(256) void sup_gather_basic_kernel(
    const SupNode* __restrict__ sn, const SupWork* __restrict__ w, const int32_t* __restrict__ fnode,
    const int32_t* __restrict__ farc, const unsigned long long* __restrict__ up, const unsigned long long* __restrict__ dn,
    const int32_t* __restrict__ up_ptr, const int32_t* __restrict__ up_head, const float* __restrict__ len_up,
    const float* __restrict__ len_dn, const int32_t* __restrict__ cnt_up, const int32_t* __restrict__ cnt_dn,
    unsigned long long* __restrict__ D, int2* __restrict__ SS, int2* __restrict__ SL) {
  const SupWork W = w[blockIdx.x];
  const SupNode S = W.sn;
  const int i = W.b, n = S.n;
  const long long r0 = S.dofs + (long long)i * n;
  const int32_t* fr = farc + S.foff + (long long)i * n;
  const int fi = fnode[S.fnode + i];
  for (int j = threadIdx.x; j < n; j += 256) {
    unsigned long long v = PACK_INF_D;
    if (i != j && (i < S.m || j < S.m)) {
      const int a = fr[j];
      if (a >= 0) {
        v = i < j ? up[a] : dn[a];
        const uint32_t pl = (uint32_t)v;
        if (wof(v) < F_INF && !(pl & EDGE_FLAG_D)) {
          const int zz = (int)pl, fj = fnode[S.fnode + j];
          const int lo = i < j ? fi : fj, hi = i < j ? fj : fi;
          const int azx = find_arc_d(up_ptr, up_head, zz, lo), azv = find_arc_d(up_ptr, up_head, zz, hi);
          const int s0 = i < j ? azx : azv, s1 = i < j ? azv : azx;
          SS[r0 + j] = make_int2(s0, s1);
          SL[r0 + j] = make_int2(__float_as_int(len_dn[s0] + len_up[s1]), cnt_dn[s0] + cnt_up[s1]);
        }
      }
    }
    D[r0 + j] = v;
  }
}

// basic, block b of a front: the 32 pivots K = [k0, k1) eliminated in the diagonal block and in the
// row / column panels of this workgroup's 32 front columns J (every workgroup of the front redoes
// the 32 x 32 diagonal block: no inter-workgroup dependency), then the rows of K are final: their
// arcs' weights go out, and they are FINALIZED (best triangle's sub-arcs, metres, road edges —
// basic_task_run's ROW_FINAL): a middle below the front from the gather's SS / SL, one in an earlier
// block from its (final) arcs, and one inside K row by row from LDS (it needs the lengths of an arc
// of K finalized just before).  1024 threads: one entry of each matrix per thread and pivot.
__device__ __forceinline__ void sup_panel_body(
    const SupWork& W, const int32_t* __restrict__ farc, unsigned long long* __restrict__ D, const int2* __restrict__ SS,
    const int2* __restrict__ SL, unsigned long long* __restrict__ up, unsigned long long* __restrict__ dn,
    int32_t* __restrict__ sub_up, int32_t* __restrict__ sub_dn, float* __restrict__ len_up, float* __restrict__ len_dn,
    int32_t* __restrict__ cnt_up, int32_t* __restrict__ cnt_dn, const float* __restrict__ length) {
  constexpr int B = SUP_B, J = SUP_PJ, W2 = SUP_B + SUP_PJ;
  static_assert(B == 32 && J == 32, "one entry of each matrix per thread");
  __shared__ unsigned long long Dk[B][B + 1];   // D[K][K]
  __shared__ unsigned long long R[B][J + 1];    // D[K][J]
  __shared__ unsigned long long C[J][B + 1];    // D[J][K]
  __shared__ int32_t FK[B][W2];                 // arcs of the rows of K: columns K | J
  __shared__ float lu[B][W2], ld[B][W2];        // their finalized metres
  __shared__ int32_t cu[B][W2], cd[B][W2];      // ... and road edges
  const SupNode S = W.sn;
  const int n = S.n, tid = threadIdx.x;
  const int k0 = W.b * B, k1 = min(k0 + B, S.m), kb = k1 - k0;
  const int j0 = k1 + W.t0 * J, nj = max(0, min(J, n - j0));
  const bool diag_writer = W.t0 == 0;
  unsigned long long* Df = D + S.dofs;
  const int32_t* F = farc + S.foff;
  const int ty = tid >> 5, tx = tid & 31;      // (row, column) of this thread's entry of each matrix
  Dk[ty][tx] = (ty < kb && tx < kb) ? Df[(long long)(k0 + ty) * n + k0 + tx] : PACK_INF_D;
  R[ty][tx] = (ty < kb && tx < nj) ? Df[(long long)(k0 + ty) * n + j0 + tx] : PACK_INF_D;
  C[ty][tx] = (tx < kb && ty < nj) ? Df[(long long)(j0 + ty) * n + k0 + tx] : PACK_INF_D;
  FK[ty][tx] = (ty < kb && tx < kb && tx > ty) ? F[(long long)(k0 + ty) * n + k0 + tx] : -1;
  FK[ty][B + tx] = (ty < kb && tx < nj) ? F[(long long)(k0 + ty) * n + j0 + tx] : -1;
  __syncthreads();
  // the block below K (K- = [k0 - 32, k0), its panels finished in the previous launch): its pivots'
  // candidates for this workgroup's entries.  That block's trailing update runs in the same launch
  // as this and leaves the rows and columns of K to here (left-looking for one block).
  if (W.b > 0) {
    const int km = k0 - B;                      // (every block but a front's last is full)
    __shared__ unsigned long long Ay[B][B + 1];   // D[K][K-]
    __shared__ unsigned long long Aj[J][B + 1];   // D[J][K-]
    __shared__ unsigned long long Bx[B][B + 1];   // D[K-][K]
    __shared__ unsigned long long Bj[B][J + 1];   // D[K-][J]
    Ay[ty][tx] = ty < kb ? Df[(long long)(k0 + ty) * n + km + tx] : PACK_INF_D;
    Aj[ty][tx] = ty < nj ? Df[(long long)(j0 + ty) * n + km + tx] : PACK_INF_D;
    Bx[ty][tx] = tx < kb ? Df[(long long)(km + ty) * n + k0 + tx] : PACK_INF_D;
    Bj[ty][tx] = tx < nj ? Df[(long long)(km + ty) * n + j0 + tx] : PACK_INF_D;
    __syncthreads();
    unsigned long long dk = Dk[ty][tx], rr = R[ty][tx], cc = C[ty][tx];
    const bool odk = ty < kb && tx < kb && ty != tx, orr = ty < kb && tx < nj, occ = ty < nj && tx < kb;
    for (int p = 0; p < B; ++p) {
      const uint32_t z = (uint32_t)(S.c0 + km + p);
      if (odk) dk = umin64(dk, sup_cand(Ay[ty][p], Bx[p][tx], z));
      if (orr) rr = umin64(rr, sup_cand(Ay[ty][p], Bj[p][tx], z));
      if (occ) cc = umin64(cc, sup_cand(Aj[ty][p], Bx[p][tx], z));
    }
    Dk[ty][tx] = dk;
    R[ty][tx] = rr;
    C[ty][tx] = cc;
    __syncthreads();
  }
  // pivot p: entries of rows / columns above p (row p and column p are final and only read)
  for (int p = 0; p < kb; ++p) {
    const uint32_t z = (uint32_t)(S.c0 + k0 + p);
    if (ty > p && tx > p && ty < kb && tx < kb && ty != tx) Dk[ty][tx] = umin64(Dk[ty][tx], sup_cand(Dk[ty][p], Dk[p][tx], z));
    if (ty > p && ty < kb && tx < nj) R[ty][tx] = umin64(R[ty][tx], sup_cand(Dk[ty][p], R[p][tx], z));
    if (tx > p && tx < kb && ty < nj) C[ty][tx] = umin64(C[ty][tx], sup_cand(C[ty][p], Dk[p][tx], z));
    __syncthreads();
  }
  if (ty < kb && tx < nj) {
    Df[(long long)(k0 + ty) * n + j0 + tx] = R[ty][tx];
    Df[(long long)(j0 + tx) * n + k0 + ty] = C[tx][ty];
    const int a = FK[ty][B + tx];
    if (a >= 0) {
      up[a] = R[ty][tx];
      dn[a] = C[tx][ty];
    }
  }
  if (diag_writer && ty < kb && tx < kb) {
    Df[(long long)(k0 + ty) * n + k0 + tx] = Dk[ty][tx];
    const int a = FK[ty][tx];
    if (a >= 0) {
      up[a] = Dk[ty][tx];
      dn[a] = Dk[tx][ty];
    }
  }
  // finalize the arcs (x, v), x in K, v in K above x (column v - k0) or in J (column B + j)
  const int zK = S.c0 + k0;     // rank of K's first pivot
  auto vfront = [&](int col) { return col < B ? k0 + col : j0 + col - B; };
  auto weight = [&](int x, int col, int dir) -> unsigned long long {
    if (col < B) return dir ? Dk[col][x] : Dk[x][col];
    return dir ? C[col - B][x] : R[x][col - B];
  };
  auto put = [&](int x, int col, int a, int dir, int s0, int s1, float L, int32_t Cn) {
    (dir ? ld : lu)[x][col] = L;
    (dir ? cd : cu)[x][col] = Cn;
    if (col >= B || diag_writer) {
      int32_t* sub = (dir ? sub_dn : sub_up) + 2 * (long long)a;
      sub[0] = s0;
      sub[1] = s1;
      (dir ? len_dn : len_up)[a] = L;
      (dir ? cnt_dn : cnt_up)[a] = Cn;
    }
  };
  // every entry whose middle is not in K, in two rounds of independent loads: (1) the gather's
  // finalization (middle below the front), a road edge's metres, or the sub-arcs through an earlier
  // block's node; (2) those sub-arcs' metres and road edges
  {
    constexpr int Q = B * W2 / 1024;
    int kind[Q][2], s0[Q][2], s1[Q][2];
    float L[Q][2];
    int32_t Cn[Q][2];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = tid + 1024 * q, x = e / W2, col = e % W2;
      const int a = FK[x][col];
#pragma unroll
      for (int dir = 0; dir < 2; ++dir) {
        kind[q][dir] = 0;
        if (a < 0) continue;
        const unsigned long long wt = weight(x, col, dir);
        const uint32_t pl = (uint32_t)wt;
        const int vf = vfront(col);
        if (!(wof(wt) < F_INF)) {
          kind[q][dir] = 1;
          s0[q][dir] = -1;
          s1[q][dir] = -1;
          L[q][dir] = F_INF;
          Cn[q][dir] = 0;
        } else if (pl & EDGE_FLAG_D) {
          const int ed = (int)(pl & ~EDGE_FLAG_D);
          kind[q][dir] = 1;
          s0[q][dir] = -1;
          s1[q][dir] = ed;
          L[q][dir] = length[ed];
          Cn[q][dir] = 1;
        } else if ((int)pl < S.c0) {           // below the front: the gather's
          const long long idx = dir ? (long long)vf * n + k0 + x : (long long)(k0 + x) * n + vf;
          const int2 ss = SS[S.dofs + idx], sl = SL[S.dofs + idx];
          kind[q][dir] = 1;
          s0[q][dir] = ss.x;
          s1[q][dir] = ss.y;
          L[q][dir] = __int_as_float(sl.x);
          Cn[q][dir] = sl.y;
        } else if ((int)pl < zK) {             // an earlier block of the chain
          const long long fz = (int)pl - S.c0;
          const int azx = F[fz * n + k0 + x], azv = F[fz * n + vf];
          kind[q][dir] = 2;
          s0[q][dir] = dir ? azv : azx;
          s1[q][dir] = dir ? azx : azv;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int dir = 0; dir < 2; ++dir)
        if (kind[q][dir] == 2) {
          L[q][dir] = len_dn[s0[q][dir]] + len_up[s1[q][dir]];
          Cn[q][dir] = cnt_dn[s0[q][dir]] + cnt_up[s1[q][dir]];
        }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = tid + 1024 * q, x = e / W2, col = e % W2;
#pragma unroll
      for (int dir = 0; dir < 2; ++dir)
        if (kind[q][dir]) put(x, col, FK[x][col], dir, s0[q][dir], s1[q][dir], L[q][dir], Cn[q][dir]);
    }
  }
  __syncthreads();
  for (int x = 1; x < kb; ++x) {
    if (tid < 2 * W2) {
      const int dir = tid / W2, col = tid % W2;
      const int a = FK[x][col];
      const unsigned long long wt = a >= 0 ? weight(x, col, dir) : PACK_INF_D;
      const uint32_t pl = (uint32_t)wt;
      const int zl = (int)pl - zK;
      if (wof(wt) < F_INF && !(pl & EDGE_FLAG_D) && zl >= 0) {
        // zl < x: row zl is final (the round above or an earlier row here); arc (z, x) is its column x
        const int azx = FK[zl][x], azv = FK[zl][col];
        if (dir == 0)
          put(x, col, a, 0, azx, azv, ld[zl][x] + lu[zl][col], cd[zl][x] + cu[zl][col]);
        else
          put(x, col, a, 1, azv, azx, ld[zl][col] + lu[zl][x], cd[zl][col] + cu[zl][x]);
      }
    }
    __syncthreads();
  }
}

// basic, block b: the trailing update of the front's targets above the next block up — for every
// (y, z), both past k1' (the end of the block above K; k1 for a front's last block), the best pivot p
// in K of D[y][p] + D[p][z] (ties: the lowest pivot = the smallest middle rank, as the packed
// atomicMin); the rows and columns of the block above K get theirs in its panel (same launch as this).
// U x U targets go to their arcs with one atomicMin after the last block.  1024 threads, 64 x 64
// targets, four per thread.
__device__ __forceinline__ void sup_trailing_body(const SupWork& W, const int32_t* __restrict__ farc,
                                                  unsigned long long* __restrict__ D, unsigned long long* __restrict__ up,
                                                  unsigned long long* __restrict__ dn) {
  constexpr int B = SUP_B, T = SUP_TT;
  __shared__ float A[T][B + 1];     // weights D[y][K]
  __shared__ float Bm[B][T + 1];    // weights D[K][z]
  const SupNode S = W.sn;
  const int n = S.n, m = S.m, tid = threadIdx.x;
  const int nb = (m + B - 1) / B;
  const int k0 = W.b * B, k1 = min(k0 + B, m), kb = k1 - k0;
  const int zr0 = W.b + 1 < nb ? min(k1 + B, m) : k1;
  const int y0 = zr0 + W.t0 * T, z0 = zr0 + W.t1 * T;
  unsigned long long* Df = D + S.dofs;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = tid + 1024 * h;
    {
      const int r = e / B, p = e % B;
      A[r][p] = (y0 + r < n && p < kb) ? wof(Df[(long long)(y0 + r) * n + k0 + p]) : F_INF;
    }
    {
      const int p = e / T, c = e % T;
      Bm[p][c] = (p < kb && z0 + c < n) ? wof(Df[(long long)(k0 + p) * n + z0 + c]) : F_INF;
    }
  }
  // the targets' current words, loaded now (their latency hides behind the loop below)
  const int ty = tid >> 4, tz = tid & 15;
  const int y = y0 + ty;
  unsigned long long old[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int z = z0 + tz + 16 * j;
    old[j] = (y < n && z < n && y != z) ? Df[(long long)y * n + z] : PACK_INF_D;
  }
  __syncthreads();
  float bw[4];
  int bp[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bw[j] = F_INF;
    bp[j] = 0;
  }
  for (int p = 0; p < kb; ++p) {
    const float a = A[ty][p];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float sum = a + Bm[p][tz + 16 * j];
      if (sum < bw[j]) {        // strict: the first (lowest) pivot keeps a tie
        bw[j] = sum;
        bp[j] = p;
      }
    }
  }
  const bool last = k1 == m;
  const int32_t* F = farc + S.foff;
  unsigned long long nv[4];
  int arc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int z = z0 + tz + 16 * j;
    const unsigned long long c = bw[j] < F_INF ? packw(bw[j], (uint32_t)(S.c0 + k0 + bp[j])) : PACK_INF_D;
    nv[j] = umin64(old[j], c);
    arc[j] = -1;
    if (y >= n || z >= n || y == z) continue;
    if (y >= m && z >= m && last) {
      if (nv[j] != PACK_INF_D) arc[j] = F[(long long)y * n + z];
    } else if (c < old[j]) {
      Df[(long long)y * n + z] = c;
    }
  }
  if (!last) return;
  unsigned long long cur[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int z = z0 + tz + 16 * j;
    cur[j] = arc[j] >= 0 ? (y < z ? up : dn)[arc[j]] : 0ull;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int z = z0 + tz + 16 * j;
    if (arc[j] >= 0 && nv[j] < cur[j]) atomicMin((y < z ? up : dn) + arc[j], nv[j]);
  }
}

// one launch per block step of the basic phase: the panels of block r of every front (work items
// with t1 < 0) beside the trailing updates of block r - 1 (1024 threads)
__global__ __launch_bounds__(1024) void sup_step_basic_kernel(
    const SupWork* __restrict__ w, const int32_t* __restrict__ farc, unsigned long long* __restrict__ D,
    const int2* __restrict__ SS, const int2* __restrict__ SL, unsigned long long* __restrict__ up,
    unsigned long long* __restrict__ dn, int32_t* __restrict__ sub_up, int32_t* __restrict__ sub_dn,
    float* __restrict__ len_up, float* __restrict__ len_dn, int32_t* __restrict__ cnt_up, int32_t* __restrict__ cnt_dn,
    const float* __restrict__ length) {
  const SupWork W = w[blockIdx.x];
  if (W.t1 < 0)
    sup_panel_body(W, farc, D, SS, SL, up, dn, sub_up, sub_dn, len_up, len_dn, cnt_up, cnt_dn, length);
  else
    sup_trailing_body(W, farc, D, up, dn);
}

// perfect: a front's basic weights (f32) of every pair with a chain node, and the perfect weights
// of U x U (final: an ancestor front's or an earlier level's); the diagonal is +inf (no candidate
// through the target's own head)
__global__ __launch_bounds__(256) void sup_gather_perfect_kernel(const SupNode* __restrict__ sn,
                                                                 const SupWork* __restrict__ w, long long nw,
                                                                 const int32_t* __restrict__ farc,
                                                                 const unsigned long long* __restrict__ up,
                                                                 const unsigned long long* __restrict__ dn,
                                                                 const uint32_t* __restrict__ pup,
                                                                 const uint32_t* __restrict__ pdn, float* __restrict__ D) {
  const long long wi = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wi >= nw) return;
  const SupWork W = w[wi];
  const SupNode S = W.sn;
  const int i = W.b, n = S.n;
  float* Db = D + 2 * S.dofs;
  float* P = Db + (long long)n * n;
  const int32_t* fr = farc + S.foff + (long long)i * n;
  for (int j = threadIdx.x & 63; j < n; j += 64) {
    float db = F_INF, p = F_INF;
    const int a = fr[j];
    if (i != j && a >= 0) {
      if (i < S.m || j < S.m) {
        db = wof(i < j ? up[a] : dn[a]);
        p = db;
      } else {
        p = __uint_as_float(i < j ? pup[a] : pdn[a]);
      }
    }
    Db[(long long)i * n + j] = db;
    P[(long long)i * n + j] = p;
  }
}

// perfect, block b (blocks from the top): the candidates through the final part above the next
// block up, F' = [k1', n) (k1' = the end of the block above K; the whole F = [k1, n) for a front's top
// block) — up: P[x][y] = min_z Db[x][z] + P[z][y], dn: P[y][x] = min_z P[y][z] + Db[z][x]  (x in K,
// y in F, z in F') — a (min, +) product, 32 x 32 outputs per workgroup over <= SUP_G1Z z (t1 = split
// << 1 | dir).  The block above K (z in [k1, k1')) is added by sup_solve_perfect_kernel: it is only
// final after that block's K x K kernel, which runs in the same launch as this (no data shared).
__device__ __forceinline__ void sup_gemm_body(const SupWork& W, float* __restrict__ D) {
  constexpr int B = SUP_B, ZC = 64;
  __shared__ float As[32][ZC + 1];
  __shared__ float Bs[ZC][33];
  const SupNode S = W.sn;
  const int n = S.n, tid = threadIdx.x;
  const int nb = (S.m + B - 1) / B;
  const int k0 = W.b * B, k1 = min(k0 + B, S.m), kb = k1 - k0;
  const int zlo = W.b + 1 < nb ? min(k1 + B, S.m) : k1;
  const int y0 = k1 + W.t0 * SUP_G1Y, ny = min(SUP_G1Y, n - y0);
  const int dir = W.t1 & 1, zs = W.t1 >> 1;
  const int zbeg = zlo + zs * SUP_G1Z, zend = min(zbeg + SUP_G1Z, n);
  const bool split = n - zlo > SUP_G1Z;
  float* Db = D + 2 * S.dofs;
  float* P = Db + (long long)n * n;
  const int r = tid >> 5, c = tid & 31;
  float best = F_INF;
  for (int zc = zbeg; zc < zend; zc += ZC) {
    const int nz = min(ZC, zend - zc);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + 1024 * h;
      {
        const int rr = e / ZC, q = e % ZC;
        float v = F_INF;
        if (q < nz) {
          if (dir == 0 && rr < kb) v = Db[(long long)(k0 + rr) * n + zc + q];
          if (dir == 1 && rr < ny) v = P[(long long)(y0 + rr) * n + zc + q];
        }
        As[rr][q] = v;
      }
      {
        const int q = e / 32, cc = e % 32;
        float v = F_INF;
        if (q < nz) {
          if (dir == 0 && cc < ny) v = P[(long long)(zc + q) * n + y0 + cc];
          if (dir == 1 && cc < kb) v = Db[(long long)(zc + q) * n + k0 + cc];
        }
        Bs[q][cc] = v;
      }
    }
    __syncthreads();
    for (int q = 0; q < nz; ++q) {
      const float sum = As[r][q] + Bs[q][c];
      best = sum < best ? sum : best;
    }
    __syncthreads();
  }
  if (!(best < F_INF)) return;
  long long idx;
  if (dir == 0) {
    if (r >= kb || c >= ny) return;
    idx = (long long)(k0 + r) * n + y0 + c;
  } else {
    if (r >= ny || c >= kb) return;
    idx = (long long)(y0 + r) * n + k0 + c;
  }
  if (split) atomicMin((uint32_t*)(P + idx), __float_as_uint(best));
  else if (best < P[idx]) P[idx] = best;
}

// perfect, block b: the rows of K against this workgroup's 64 columns y of F, top-down through K
// (candidates through z in K above x), then written out; and the F-part of the K x K targets through
// these 64 z (atomicMin into P[K][K], finished by sup_kk_body in the next launch).  1024 threads: two entries
// of each direction per thread and step.
__global__ __launch_bounds__(1024) void sup_solve_perfect_kernel(const SupNode* __restrict__ sn,
                                                                 const SupWork* __restrict__ w,
                                                                 const int32_t* __restrict__ farc, float* __restrict__ D,
                                                                 uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  constexpr int B = SUP_B, Y = SUP_SJ;
  static_assert(B * Y == 2048, "two entries per thread");
  __shared__ float Dk[B][B + 1];     // Db[K][K]
  __shared__ float PU[B][Y + 1];     // P[K][y]
  __shared__ float PD[Y][B + 1];     // P[y][K]
  __shared__ float DKT[B][Y + 1];    // Db[K][y]
  __shared__ float DTK[Y][B + 1];    // Db[y][K]
  const SupWork W = w[blockIdx.x];
  const SupNode S = W.sn;
  const int n = S.n, tid = threadIdx.x;
  const int k0 = W.b * B, k1 = min(k0 + B, S.m), kb = k1 - k0;
  const int y0 = k1 + W.t0 * Y, ny = min(Y, n - y0);
  float* Db = D + 2 * S.dofs;
  float* P = Db + (long long)n * n;
  {
    const int y = tid >> 5, x = tid & 31;
    Dk[y][x] = (y < kb && x < kb) ? Db[(long long)(k0 + y) * n + k0 + x] : F_INF;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int e = tid + 1024 * q;
    {
      const int x = e / Y, y = e % Y;
      const bool ok = x < kb && y < ny;
      PU[x][y] = ok ? P[(long long)(k0 + x) * n + y0 + y] : F_INF;
      DKT[x][y] = ok ? Db[(long long)(k0 + x) * n + y0 + y] : F_INF;
    }
    {
      const int y = e / B, x = e % B;
      const bool ok = x < kb && y < ny;
      PD[y][x] = ok ? P[(long long)(y0 + y) * n + k0 + x] : F_INF;
      DTK[y][x] = ok ? Db[(long long)(y0 + y) * n + k0 + x] : F_INF;
    }
  }
  __syncthreads();
  // the block above K, K' = [k1, k2) (finished in the previous launches: its rows by its solve, its
  // K' x K' by its K x K kernel): its candidates for this workgroup's entries (the product left it out)
  const int nbk = (S.m + B - 1) / B;
  if (W.b + 1 < nbk) {
    const int k2 = min(k1 + B, S.m), kb2 = k2 - k1;
    __shared__ float A2[B][B + 1];    // Db[K][K']
    __shared__ float E2[B][B + 1];    // Db[K'][K]
    __shared__ float B2[B][Y + 1];    // P[K'][y]
    __shared__ float C2[Y][B + 1];    // P[y][K']
    {
      const int y = tid >> 5, x = tid & 31;
      A2[y][x] = (y < kb && x < kb2) ? Db[(long long)(k0 + y) * n + k1 + x] : F_INF;
      E2[y][x] = (y < kb2 && x < kb) ? Db[(long long)(k1 + y) * n + k0 + x] : F_INF;
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + 1024 * q;
      {
        const int z = e / Y, y = e % Y;
        B2[z][y] = (z < kb2 && y < ny) ? P[(long long)(k1 + z) * n + y0 + y] : F_INF;
      }
      {
        const int y = e / B, z = e % B;
        C2[y][z] = (z < kb2 && y < ny) ? P[(long long)(y0 + y) * n + k1 + z] : F_INF;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + 1024 * q;
      {
        const int x = e / Y, y = e % Y;
        if (x < kb && y < ny) {
          float v = PU[x][y];
          for (int z = 0; z < kb2; ++z) {
            const float c = A2[x][z] + B2[z][y];
            v = c < v ? c : v;
          }
          PU[x][y] = v;
        }
      }
      {
        const int y = e / B, x = e % B;
        if (x < kb && y < ny) {
          float v = PD[y][x];
          for (int z = 0; z < kb2; ++z) {
            const float c = C2[y][z] + E2[z][x];
            v = c < v ? c : v;
          }
          PD[y][x] = v;
        }
      }
    }
    __syncthreads();
  }
  // top-down through K, four pivots z0 > z1 > z2 > z3 per barrier: every thread first finishes the
  // group's own entries of its column (u_i = P[z_i][y] through z_j, j < i) from LDS, then applies
  // all four to its entry (a group row stores its u).  A group row may be read while its owner
  // stores it: the value read is either the old one or the finished one, and u_i comes out the same
  // (its candidates are recomputed either way) — every candidate is the same single add as one pivot
  // per step, so the minima are bit-identical.
  for (int zt = kb - 1; zt >= 1; zt -= 4) {
    const int G = min(4, zt);                 // members zt, zt - 1, ..., zt - G + 1 (>= 1)
    const int zb = zt - G + 1;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = tid + 1024 * q;
      {
        const int x = e / Y, y = e % Y;
        if (x < zt && y < ny) {
          float u[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (i >= G) break;
            float v = PU[zt - i][y];
#pragma unroll
            for (int j = 0; j < i; ++j) {
              const float c = Dk[zt - i][zt - j] + u[j];
              v = c < v ? c : v;
            }
            u[i] = v;
          }
          if (x < zb) {
            float v = PU[x][y];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              if (i >= G) break;
              const float c = Dk[x][zt - i] + u[i];
              v = c < v ? c : v;
            }
            PU[x][y] = v;
          } else {
            PU[x][y] = u[zt - x];
          }
        }
      }
      {
        const int y = e / B, x = e % B;
        if (x < zt && y < ny) {
          float u[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (i >= G) break;
            float v = PD[y][zt - i];
#pragma unroll
            for (int j = 0; j < i; ++j) {
              const float c = u[j] + Dk[zt - j][zt - i];
              v = c < v ? c : v;
            }
            u[i] = v;
          }
          if (x < zb) {
            float v = PD[y][x];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              if (i >= G) break;
              const float c = u[i] + Dk[zt - i][x];
              v = c < v ? c : v;
            }
            PD[y][x] = v;
          } else {
            PD[y][x] = u[zt - x];
          }
        }
      }
    }
    __syncthreads();
  }
  const int32_t* F = farc + S.foff;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int e = tid + 1024 * q, x = e / Y, y = e % Y;
    if (x < kb && y < ny) {
      const long long iu = (long long)(k0 + x) * n + y0 + y;
      P[iu] = PU[x][y];
      P[(long long)(y0 + y) * n + k0 + x] = PD[y][x];
      const int a = F[iu];
      if (a >= 0) {
        pup[a] = __float_as_uint(PU[x][y]);
        pdn[a] = __float_as_uint(PD[y][x]);
      }
    }
  }
  {
    const int x = tid >> 5, y = tid & 31;
    if (x < y && y < kb) {
      float bu = F_INF, bd = F_INF;
      for (int q = 0; q < ny; ++q) {
        const float su = DKT[x][q] + PD[q][y];
        const float sd = PU[y][q] + DTK[q][x];
        bu = su < bu ? su : bu;
        bd = sd < bd ? sd : bd;
      }
      if (bu < F_INF) atomicMin((uint32_t*)(P + (long long)(k0 + x) * n + k0 + y), __float_as_uint(bu));
      if (bd < F_INF) atomicMin((uint32_t*)(P + (long long)(k0 + y) * n + k0 + x), __float_as_uint(bd));
    }
  }
}

// perfect, block b: the K x K targets top-down (x from the top of K: all of its candidates through
// z in K above x are final), one workgroup per front; 16 lanes per target split the z loop
__device__ __forceinline__ void sup_kk_body(const SupWork& W, const int32_t* __restrict__ farc, float* __restrict__ D,
                                            uint32_t* __restrict__ pup, uint32_t* __restrict__ pdn) {
  constexpr int B = SUP_B;
  __shared__ float Dk[B][B + 1];
  __shared__ float Pk[B][B + 1];
  const SupNode S = W.sn;
  const int n = S.n, tid = threadIdx.x;
  const int k0 = W.b * B, k1 = min(k0 + B, S.m), kb = k1 - k0;
  float* Db = D + 2 * S.dofs;
  float* P = Db + (long long)n * n;
  {
    const int y = tid >> 5, x = tid & 31;
    const bool ok = y < kb && x < kb;
    Dk[y][x] = ok ? Db[(long long)(k0 + y) * n + k0 + x] : F_INF;
    Pk[y][x] = ok ? P[(long long)(k0 + y) * n + k0 + x] : F_INF;
  }
  __syncthreads();
  const int g = tid >> 4, q = tid & 15;
  const int dir = g >> 5, y = g & 31;
  for (int x = kb - 2; x >= 0; --x) {
    float best = F_INF;
    if (y > x && y < kb)
      for (int z = x + 1 + q; z < kb; z += 16) {
        if (z == y) continue;
        const float s = dir == 0 ? Dk[x][z] + Pk[z][y] : Pk[y][z] + Dk[z][x];
        best = s < best ? s : best;
      }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float v = __shfl_xor(best, o);
      best = v < best ? v : best;
    }
    if (q == 0 && y > x && y < kb) {
      if (dir == 0) {
        if (best < Pk[x][y]) Pk[x][y] = best;
      } else {
        if (best < Pk[y][x]) Pk[y][x] = best;
      }
    }
    __syncthreads();
  }
  const int32_t* F = farc + S.foff;
  {
    const int x = tid >> 5, yy = tid & 31;
    if (x < kb && yy < kb) {
      const long long idx = (long long)(k0 + x) * n + k0 + yy;
      P[idx] = Pk[x][yy];
      if (x < yy) {
        const int a = F[idx];
        if (a >= 0) {
          pup[a] = __float_as_uint(Pk[x][yy]);
          pdn[a] = __float_as_uint(Pk[yy][x]);
        }
      }
    }
  }
}

// one launch per block step of the perfect phase: the K x K kernels of the blocks solved in the
// previous launch (work items with t0 < 0) beside the products of the next blocks down (1024 threads)
__global__ __launch_bounds__(1024) void sup_kk_gemm_perfect_kernel(const SupWork* __restrict__ w,
                                                                   const int32_t* __restrict__ farc,
                                                                   float* __restrict__ D, uint32_t* __restrict__ pup,
                                                                   uint32_t* __restrict__ pdn) {
  const SupWork W = w[blockIdx.x];
  if (W.t0 < 0) sup_kk_body(W, farc, D, pup, pdn);
  else sup_gemm_body(W, D);
}

// ---- context costs (routing/graph.py edge_records / edge_costs) ----
constexpr float L_REF_M = 10000.f;
constexpr int32_t MONDAY_2025_08_25 = 2063 * 86400;   // seconds since 2020-01-01 (a Monday)

__global__ void ctx_records_kernel(const uint8_t* __restrict__ base_traffic, int E, int weather, int congestion,
                                   int weekhour, float age, EtaRecordDev* __restrict__ rec) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  int lvl = (int)base_traffic[e] + congestion - 1;
  lvl = lvl < 0 ? 0 : (lvl > 3 ? 3 : lvl);
  // TRAFFIC_LEVELS (Low, Medium, High, Jam) -> features.py traffic codes (High 0, Jam 1, Low 2, Medium 3)
  const uint8_t code = (uint8_t)((0x01000302u >> (8 * lvl)) & 0xFF);
  EtaRecordDev r;
  r.distance_m = L_REF_M;
  r.driver_age = age;
  r.wallclock_s = MONDAY_2025_08_25 + weekhour * 3600;
  r.weather = (uint8_t)weather;
  r.traffic = code;
  r.pad = 0;
  rec[2 * (long long)e] = r;
  r.distance_m = 0.f;
  rec[2 * (long long)e + 1] = r;
}

__global__ void ctx_cost_kernel(const float* __restrict__ minutes, const float* __restrict__ length,
                                const uint8_t* __restrict__ road_class, int E, float* __restrict__ cost) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float k60 = (float)(60.0 / 10000.0);
  const float rate = (minutes[2 * (long long)e] - minutes[2 * (long long)e + 1]) * k60;
  const float cf[4] = {1.15f, 1.0f, 0.85f, 0.65f};
  const float sec = rate * length[e] * cf[road_class[e] & 3];
  const float floor_s = length[e] / (float)(130.0 / 3.6);
  cost[e] = sec > floor_s ? sec : floor_s;
}

// ---- queries ----

// One wave per chain job (rank << 1 | dir): sweep the etree ancestor chain bottom-up with labels in
// LDS by depth, then dump them (dist, pred arc) and the chain's node ranks to the job's scratch row.
//
// The chain is walked in runs of consecutive ranks (parent(x + i) == x + i + 1: the separators), up to
// 64 per run, whose headers (parent, record range) one coalesced load fetches; the next run's header
// is loaded while the current run is swept.  Inside a run, node i's first 256 kept-arc records (4 per lane) are
// loaded SWEEP_AHEAD nodes ahead, so the sequential label sweep waits on LDS, not on one global
// load per chain node (r4c profile: the sweep was 49.6 % of the CCH GPU time at ~25 us per chain).
constexpr int SWEEP_AHEAD = 3;
constexpr int SWEEP_RECS = 4;          // records per lane fetched ahead per chain node (256 per node)

typedef int sweep_v4i __attribute__((ext_vector_type(4)));

struct SweepRecs {
  sweep_v4i r[SWEEP_RECS];
};

// The record prefetch is issued as inline-asm loads the compiler does not track, and each use
// waits for its own loads with an explicit vmcnt (sweep_wait): compiler-tracked loads that stay in
// flight across the loop's back edge made it wait for all of them at the top of every iteration.
// Branch-free: lanes past the node's records load record 0 (always allocated) and are masked where
// the records are used, so every fetch issues exactly SWEEP_RECS loads.
__device__ __forceinline__ SweepRecs sweep_fetch(const int4* __restrict__ rec, int pb, int pe, int i, int L, int lane) {
  SweepRecs v;
  const int ii = i < 63 ? i : 63;
  const int b = __shfl(pb, ii);
  const int e = i < L ? __shfl(pe, ii) : b;
#pragma unroll
  for (int k = 0; k < SWEEP_RECS; ++k) {
    const int idx = b + lane + 64 * k;
    const int4* p = rec + (idx < e ? idx : 0);
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v.r[k]) : "v"(p));
  }
  return v;
}

// wait until the loads of the fetch issued `newer` fetches before the current one have landed
template <int NEWER>
__device__ __forceinline__ void sweep_wait(SweepRecs& q) {
  static_assert(NEWER * SWEEP_RECS <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(q.r[0]), "+v"(q.r[1]), "+v"(q.r[2]), "+v"(q.r[3]) : "n"(NEWER * SWEEP_RECS));
}

__device__ __forceinline__ void sweep_relax(float* sd, int32_t* sp, float dx, int w, int hd, int arc) {
  const float nd = dx + __int_as_float(w);
  if (nd < sd[hd]) {
    sd[hd] = nd;
    sp[hd] = arc;
  }
}

__global__ __launch_bounds__(64) void sweep_kernel(const int32_t* __restrict__ jobs, int J,
                                                   const int32_t* __restrict__ parent,
                                                   const int32_t* __restrict__ depth, int N,
                                                   const int32_t* __restrict__ f_ptr, const int4* __restrict__ f_rec,
                                                   const int32_t* __restrict__ b_ptr, const int4* __restrict__ b_rec,
                                                   int stride, float* __restrict__ out_dist,
                                                   int32_t* __restrict__ out_pred, int32_t* __restrict__ out_node,
                                                   const CchMView* __restrict__ mv, const int32_t* __restrict__ grp,
                                                   int gdiv) {
  extern __shared__ unsigned char smem[];
  float* sd = reinterpret_cast<float*>(smem);
  int32_t* sp = reinterpret_cast<int32_t*>(smem + (size_t)stride * 4);
  const int j = blockIdx.x;
  if (j >= J) return;
  const int lane = threadIdx.x;
  const int code = jobs[j];
  if (code < 0) return;                     // matrix padding
  const int r = code >> 1;
  const bool fwd = (code & 1) == 0;
  if (mv != nullptr) {                      // this job's metric (one job per workgroup: uniform)
    const CchMView& v = mv[grp[j / gdiv]];
    f_ptr = v.f_ptr;
    f_rec = v.f_rec;
    b_ptr = v.b_ptr;
    b_rec = v.b_rec;
  }
  const int32_t* __restrict__ ptr = fwd ? f_ptr : b_ptr;
  const int4* __restrict__ rec = fwd ? f_rec : b_rec;
  const int D = depth[r];
  for (int d = lane; d <= D; d += 64) {
    sd[d] = F_INF;
    sp[d] = -1;
  }
  __syncthreads();
  if (lane == 0) sd[D] = 0.f;
  __syncthreads();
  const size_t base = (size_t)j * stride;
  int x = r, d = D;
  // header of the run starting at x: parent and record range of x + lane
  int cand = x + lane;
  int par = cand < N ? parent[cand] : -2;
  int pb = cand < N ? ptr[cand] : 0;
  int pe = cand < N ? ptr[cand + 1] : 0;
  while (x >= 0 && d >= 0) {
    const unsigned long long cont = __ballot(cand < N && par == cand + 1);
    int L = (~cont == 0ull) ? 64 : (__builtin_ctzll(~cont) + 1);
    if (L > d + 1) L = d + 1;
    const int next = __shfl(par, L - 1);
    if (lane < L) out_node[base + (d - lane)] = x + lane;
    // the next run's header, in flight while this run is swept
    const int ncand = next + lane;
    const bool nin = next >= 0 && ncand < N;
    const int npar = nin ? parent[ncand] : -2;
    const int npb = nin ? ptr[ncand] : 0;
    const int npe = nin ? ptr[ncand + 1] : 0;
    // each node's records were requested three nodes earlier; named buffers, unrolled by four
    auto node = [&](int i, const SweepRecs& q) {
      if (i >= L) return;
      const float dx = sd[d - i];
      if (dx < F_INF) {
        // a node's kept arcs have distinct heads: the lanes' updates never collide
        const int b = __shfl(pb, i), e = __shfl(pe, i);
#pragma unroll
        for (int k = 0; k < SWEEP_RECS; ++k)
          if (b + lane + 64 * k < e) sweep_relax(sd, sp, dx, q.r[k].x, q.r[k].y, q.r[k].z);
        for (int k = b + 64 * SWEEP_RECS + lane; k < e; k += 64) {     // nodes with > 256 kept arcs
          const int4 rc = rec[k];
          sweep_relax(sd, sp, dx, rc.x, rc.y, rc.z);
        }
        __syncthreads();
      }
    };
    SweepRecs qa = sweep_fetch(rec, pb, pe, 0, L, lane);
    SweepRecs qb = sweep_fetch(rec, pb, pe, 1, L, lane);
    SweepRecs qc = sweep_fetch(rec, pb, pe, 2, L, lane);
    for (int i = 0; i < L; i += 4) {
      SweepRecs qd = sweep_fetch(rec, pb, pe, i + 3, L, lane);
      sweep_wait<3>(qa);
      node(i, qa);
      qa = sweep_fetch(rec, pb, pe, i + 4, L, lane);
      sweep_wait<3>(qb);
      node(i + 1, qb);
      qb = sweep_fetch(rec, pb, pe, i + 5, L, lane);
      sweep_wait<3>(qc);
      node(i + 2, qc);
      qc = sweep_fetch(rec, pb, pe, i + 6, L, lane);
      sweep_wait<3>(qd);
      node(i + 3, qd);
    }
    sweep_wait<0>(qa);          // drain the prefetch past the run's end before the buffers are reused
    sweep_wait<0>(qb);
    sweep_wait<0>(qc);
    x = next;
    d -= L;
    cand = ncand;
    par = npar;
    pb = npb;
    pe = npe;
  }
  __syncthreads();
  for (int dd = lane; dd <= D; dd += 64) {
    out_dist[base + dd] = sd[dd];
    out_pred[base + dd] = sp[dd];
  }
}

// One wave per pair: LCA depth, best common depth (min sum, deepest tie), metres along the chosen
// shortcut arcs (forward arcs from the meeting node down to s, then backward ones down to t), and —
// with `arcs` — the arc list in path order (arc << 1 | traversed-down).
__global__ __launch_bounds__(64) void meet_kernel(int P, const int32_t* __restrict__ pjf, const int32_t* __restrict__ pjb,
                                                  int jf0, int jb0, const int32_t* __restrict__ jobs, int stride,
                                                  const float* __restrict__ sdist, const int32_t* __restrict__ spred,
                                                  const int32_t* __restrict__ snode, const int32_t* __restrict__ depth,
                                                  const int32_t* __restrict__ arc_lo, const float* __restrict__ len_up,
                                                  const float* __restrict__ len_dn, float* __restrict__ out_sec,
                                                  float* __restrict__ out_met, int* __restrict__ out_status,
                                                  int32_t* __restrict__ arcs, int32_t* __restrict__ narcs, int max_arcs,
                                                  const CchMView* __restrict__ mv, const int32_t* __restrict__ grp,
                                                  int gdiv) {
  __shared__ int32_t fw[4096];
  const int q = blockIdx.x;
  if (q >= P) return;
  const int lane = threadIdx.x;
  if (mv != nullptr) {
    const CchMView& v = mv[grp[q / gdiv]];
    len_up = v.len_up;
    len_dn = v.len_dn;
  }
  const int jf = pjf ? pjf[q] : jf0 + 2 * q;
  const int jb = pjb ? pjb[q] : jb0 + 2 * q;
  if (jobs[jf] < 0 || jobs[jb] < 0) {       // a matrix padding point: nothing to meet
    if (threadIdx.x == 0) {
      if (out_sec) out_sec[q] = -1.f;
      if (out_met) out_met[q] = -1.f;
      if (out_status) out_status[q] = 1;
      if (narcs) narcs[q] = 0;
    }
    return;
  }
  const int s = jobs[jf] >> 1, t = jobs[jb] >> 1;
  const int ds = depth[s], dt = depth[t];
  const size_t bf = (size_t)jf * stride, bb = (size_t)jb * stride;
  int status = 1;
  float best = F_INF;
  int bestd = -1;
  if (snode[bf] == snode[bb]) {
    // chains agree on depths [0, L]
    int lo = 0, hi = ds < dt ? ds : dt;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (snode[bf + mid] == snode[bb + mid]) lo = mid;
      else hi = mid - 1;
    }
    const int L = lo;
    for (int d = lane; d <= L; d += 64) {
      const float v = sdist[bf + d] + sdist[bb + d];
      if (v < best || (v == best && d > bestd)) {
        best = v;
        bestd = d;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(best, o);
      const int od = __shfl_xor(bestd, o);
      if (ov < best || (ov == best && od > bestd)) {
        best = ov;
        bestd = od;
      }
    }
    if (best < F_INF) status = 0;
  }
  if (lane != 0) return;
  float met = 0.f;
  int n = 0;
  if (status == 0) {
    int nf = 0;
    for (int slot = bestd; slot != ds;) {
      const int a = spred[bf + slot];
      met += len_up[a];
      if (nf < 4096) fw[nf] = a;
      ++nf;
      slot = depth[arc_lo[a]];
    }
    if (arcs != nullptr) {
      int32_t* out = arcs + (size_t)q * max_arcs;
      if (nf > 4096 || nf > max_arcs) status = 4;
      for (int i = nf - 1; i >= 0 && status == 0; --i) out[n++] = fw[i] << 1;
      for (int slot = bestd; slot != dt && status == 0;) {
        const int a = spred[bb + slot];
        met += len_dn[a];
        if (n >= max_arcs) { status = 4; break; }
        out[n++] = (a << 1) | 1;
        slot = depth[arc_lo[a]];
      }
    } else {
      for (int slot = bestd; slot != dt;) {
        const int a = spred[bb + slot];
        met += len_dn[a];
        slot = depth[arc_lo[a]];
      }
    }
  }
  if (out_sec) out_sec[q] = status == 0 ? best : -1.f;
  if (out_met) out_met[q] = status == 0 ? met : -1.f;
  if (out_status) out_status[q] = status;
  if (narcs) narcs[q] = n;
}

// One lane per pair: expand the shortcut arcs to road node ids (DFS, first sub-arc first).
constexpr int UNPACK_STACK = 128;
__global__ __launch_bounds__(64) void unpack_kernel(int P, const int* __restrict__ src_node, const int32_t* __restrict__ arcs,
                                                    const int32_t* __restrict__ narcs, int max_arcs,
                                                    const int32_t* __restrict__ sub_up,
                                                    const int32_t* __restrict__ sub_dn,
                                                    const int32_t* __restrict__ arc_lo,
                                                    const int32_t* __restrict__ up_head,
                                                    const int32_t* __restrict__ node_of, int* __restrict__ status,
                                                    int* __restrict__ out_len, int* __restrict__ out_path, int max_path,
                                                    int min_arcs, int* __restrict__ out_edge,
                                                    const CchMView* __restrict__ mv, const int32_t* __restrict__ grp) {
  __shared__ int32_t stk[64 * UNPACK_STACK];
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= P) return;
  if (mv != nullptr) {
    const CchMView& v = mv[grp[q]];
    sub_up = v.sub_up;
    sub_dn = v.sub_dn;
  }
  int32_t* st = stk + threadIdx.x * UNPACK_STACK;
  if (status[q] != 0) {
    if (min_arcs < 0) out_len[q] = 0;
    return;
  }
  if (narcs[q] <= min_arcs && out_len[q] != -1) return;   // unpacked by unpack_coop_kernel
  int* out = out_path + (size_t)q * max_path;
  int n = 0;
  out[n++] = src_node[q];
  const int na = narcs[q];
  const int32_t* al = arcs + (size_t)q * max_arcs;
  bool ok = true;
  for (int k = 0; k < na && ok; ++k) {
    int sp = 0;
    st[sp++] = al[k];
    while (sp > 0) {
      const int code = st[--sp];
      const int a = code >> 1, dn = code & 1;
      const int32_t* sub = (dn ? sub_dn : sub_up) + 2 * (long long)a;
      const int s0 = sub[0];
      if (s0 < 0) {
        if (n >= max_path) { ok = false; break; }
        if (out_edge) out_edge[(size_t)q * max_path + n - 1] = sub[1];
        out[n++] = node_of[dn ? arc_lo[a] : up_head[a]];
        continue;
      }
      if (sp + 2 > UNPACK_STACK) { ok = false; break; }
      st[sp++] = sub[1] << 1;        // second: traversed up
      st[sp++] = (s0 << 1) | 1;      // first: traversed down (popped first)
    }
  }
  if (!ok) {
    status[q] = 4;
    out_len[q] = 0;
    return;
  }
  out_len[q] = n;
}

// Cooperative unpack: UNPACK_LANES lanes per pair share its path.  The arcs' road-edge counts
// (cnt_*, from the customization) give each shortcut arc its offset in the path, every lane takes a
// contiguous range of road edges, descends the shortcut tree once to its first edge (counts pick the
// branch), then walks the DFS for the rest of its range — ~depth + edges/UNPACK_LANES dependent
// loads per lane instead of one lane walking the whole path (the serial unpack's time was the
// longest path's DFS).  Pairs with more than UNPACK_MAX_ARCS shortcut arcs take the serial kernel.
constexpr int UNPACK_LANES = 16;
constexpr int UNPACK_MAX_ARCS = 256;
constexpr int UNPACK_SD = 64;                 // per-lane DFS stack (pending second sub-arcs)
__global__ __launch_bounds__(64) void unpack_coop_kernel(int P, const int* __restrict__ src_node,
                                                         const int32_t* __restrict__ arcs,
                                                         const int32_t* __restrict__ narcs, int max_arcs,
                                                         const int32_t* __restrict__ sub_up,
                                                         const int32_t* __restrict__ sub_dn,
                                                         const int32_t* __restrict__ cnt_up,
                                                         const int32_t* __restrict__ cnt_dn,
                                                         const int32_t* __restrict__ arc_lo,
                                                         const int32_t* __restrict__ up_head,
                                                         const int32_t* __restrict__ node_of, int* __restrict__ status,
                                                         int* __restrict__ out_len, int* __restrict__ out_path,
                                                         int max_path, int* __restrict__ out_edge,
                                                         const CchMView* __restrict__ mv,
                                                         const int32_t* __restrict__ grp) {
  constexpr int G = 64 / UNPACK_LANES;
  __shared__ int32_t offs[G][UNPACK_MAX_ARCS + 1];
  __shared__ int32_t stk[64 * UNPACK_SD];
  const int lane = threadIdx.x, g = lane / UNPACK_LANES, sl = lane % UNPACK_LANES;
  const int q = blockIdx.x * G + g;
  const bool active = q < P;
  if (mv != nullptr && active) {            // (per pair: the four pairs of a wave may differ)
    const CchMView& v = mv[grp[q]];
    sub_up = v.sub_up;
    sub_dn = v.sub_dn;
    cnt_up = v.cnt_up;
    cnt_dn = v.cnt_dn;
  }
  int st = active ? status[q] : 1;
  const int na = active && st == 0 ? narcs[q] : 0;
  const bool coop = active && st == 0 && na <= UNPACK_MAX_ARCS;   // longer arc lists: the serial kernel
  if (active && st != 0 && sl == 0) out_len[q] = 0;
  // exclusive prefix of the arcs' edge counts, UNPACK_LANES at a time
  const int32_t* al = arcs + (size_t)(active ? q : 0) * max_arcs;
  int carry = 0;
  for (int b = 0; b < (coop ? na : 0); b += UNPACK_LANES) {
    const int k = b + sl;
    int c = 0;
    if (k < na) {
      const int code = al[k];
      c = (code & 1) ? cnt_dn[code >> 1] : cnt_up[code >> 1];
    }
    int incl = c;
#pragma unroll
    for (int o = 1; o < UNPACK_LANES; o <<= 1) {
      const int y = __shfl_up(incl, o, UNPACK_LANES);
      if (sl >= o) incl += y;
    }
    if (k < na) offs[g][k] = carry + incl - c;
    carry += __shfl(incl, UNPACK_LANES - 1, UNPACK_LANES);
  }
  const int E = carry;                       // road edges of the path (uniform in the group)
  if (coop) {
    if (sl == 0) offs[g][na] = E;
    if (E + 1 > max_path) {
      if (sl == 0) {
        status[q] = 4;
        out_len[q] = 0;
      }
      st = 4;
    } else if (sl == 0) {
      out_len[q] = E + 1;
    }
  }
  __syncthreads();
  if (!coop || st != 0) return;
  int* out = out_path + (size_t)q * max_path;
  int* oe = out_edge ? out_edge + (size_t)q * max_path : nullptr;
  if (sl == 0) out[0] = src_node[q];
  const int per = (E + UNPACK_LANES - 1) / UNPACK_LANES;
  int e = sl * per;
  const int e1 = min(E, e + per);
  if (e >= e1) return;
  int32_t* sk = stk + lane * UNPACK_SD;
  // the arc holding edge e
  int lo = 0, hi = na - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (offs[g][mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  int k = lo;
  int r = e - offs[g][k];                  // edge index inside arc k
  int sp = 0;
  bool ok = true;
  int code = al[k];
  // descend to the r-th edge of `code`, keeping the pending second halves
  auto descend = [&](int c, int rr) -> int {
    while (true) {
      const int a = c >> 1, dn = c & 1;
      const int32_t* sub = (dn ? sub_dn : sub_up) + 2 * (long long)a;
      const int s0 = sub[0];
      if (s0 < 0) return c;                  // an original edge
      const int s1 = sub[1];
      const int first = (s0 << 1) | 1, second = s1 << 1;     // first traversed down, second up
      const int c0 = cnt_dn[s0];
      if (rr < c0) {
        if (sp >= UNPACK_SD) { ok = false; return c; }
        sk[sp++] = second;
        c = first;
      } else {
        rr -= c0;
        c = second;
      }
    }
  };
  int leaf = descend(code, r);
  while (ok) {
    const int a = leaf >> 1, dn = leaf & 1;
    out[e + 1] = node_of[dn ? arc_lo[a] : up_head[a]];
    if (oe) oe[e] = (dn ? sub_dn : sub_up)[2 * (long long)a + 1];    // a leaf arc's original edge
    if (++e >= e1) break;
    if (sp > 0) {
      leaf = descend(sk[--sp], 0);
    } else {
      ++k;                                   // next shortcut arc of the path
      leaf = descend(al[k], 0);
    }
  }
  if (!ok) out_len[q] = -1;                  // stack overflow: the serial kernel redoes the pair
}

// (node ids are range-checked by the callers; out-of-range ids are clamped, never dereferenced)
__global__ void route_jobs_kernel(const int* __restrict__ src, const int* __restrict__ dst, int Q,
                                  const int32_t* __restrict__ rank, int N, int32_t* __restrict__ jobs) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  int s = src[q], t = dst[q];
  s = (s < 0 || s >= N) ? 0 : s;
  t = (t < 0 || t >= N) ? 0 : t;
  jobs[2 * q] = rank[s] << 1;
  jobs[2 * q + 1] = (rank[t] << 1) | 1;
}

// legs from a matrix call's chains: job indices of (r, i) forward and (r, j) backward
__global__ void leg_pairs_kernel(int NM, const int* __restrict__ r, const int* __restrict__ i,
                                 const int* __restrict__ j, int Q, int R, int32_t* __restrict__ pjf,
                                 int32_t* __restrict__ pjb) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  int rr = r[q], ii = i[q], jj = j[q];
  rr = rr < 0 ? 0 : (rr >= R ? R - 1 : rr);       // clamped: the host checks the ranges
  ii = ii < 0 ? 0 : (ii >= NM ? NM - 1 : ii);
  jj = jj < 0 ? 0 : (jj >= NM ? NM - 1 : jj);
  pjf[q] = 2 * (rr * NM + ii);
  pjb[q] = 2 * (rr * NM + jj) + 1;
}

// matrix: jobs [R][NM][2] (forward, backward per point); pairs (r, i, j) for i != j
__global__ void matrix_jobs_kernel(const int* __restrict__ pts, const int* __restrict__ npts, int R, int NM,
                                   const int32_t* __restrict__ rank, int N, int32_t* __restrict__ jobs) {
  const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (g >= (long long)R * NM) return;
  const int r = (int)(g / NM), i = (int)(g % NM);
  if (i >= npts[r]) {                       // padding of a shorter request: no chain is swept
    jobs[2 * g] = -1;
    jobs[2 * g + 1] = -1;
    return;
  }
  int v = pts[g];
  if (v < 0 || v >= N) v = 0;
  jobs[2 * g] = rank[v] << 1;
  jobs[2 * g + 1] = (rank[v] << 1) | 1;
}

__global__ void matrix_pairs_kernel(const int* __restrict__ npts, int R, int NM, int32_t* __restrict__ pjf,
                                    int32_t* __restrict__ pjb) {
  const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (g >= (long long)R * NM * NM) return;
  const int r = (int)(g / ((long long)NM * NM));
  const int rem = (int)(g % ((long long)NM * NM));
  const int i = rem / NM, j = rem % NM;
  pjf[g] = 2 * (r * NM + i);
  pjb[g] = 2 * (r * NM + j) + 1;
}

__global__ void matrix_out_kernel(const int* __restrict__ npts, int R, int NM, float* __restrict__ sec,
                                  float* __restrict__ met, double* __restrict__ D64) {
  const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (g >= (long long)R * NM * NM) return;
  const int r = (int)(g / ((long long)NM * NM));
  const int rem = (int)(g % ((long long)NM * NM));
  const int i = rem / NM, j = rem % NM;
  const int n = npts[r];
  const bool diag = i == j;
  const bool out = i >= n || j >= n;
  float s = sec ? sec[g] : 0.f, m = met ? met[g] : 0.f;
  if (diag || out) s = m = 0.f;
  else {
    if (s < 0.f) s = F_INF;
    if (m < 0.f) m = F_INF;
  }
  if (sec) sec[g] = s;
  if (met) met[g] = m;
  if (D64) D64[g] = (double)m;
}

inline int blocks_for(long long n, int b) { return (int)((n + b - 1) / b); }

template <class T>
hipError_t dmalloc(T*& p, size_t n) {
  p = nullptr;
  if (n == 0) n = 1;
  return hipMalloc((void**)&p, n * sizeof(T));
}
template <class T>
hipError_t up_copy(T*& p, const T* h, size_t n) {
  hipError_t e = dmalloc(p, n);
  if (e == hipSuccess && n) e = hipMemcpy(p, h, n * sizeof(T), hipMemcpyHostToDevice);
  return e;
}
template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
CchMetricDev::~CchMetricDev() {
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(device);
  dfree(cost);
  dfree(sub_up);
  dfree(sub_dn);
  dfree(len_up);
  dfree(len_dn);
  dfree(cnt_up);
  dfree(cnt_dn);
  dfree(f_ptr);
  dfree(b_ptr);
  dfree(f_rec);
  dfree(b_rec);
  (void)hipSetDevice(cur);
}

CchScratch::~CchScratch() {
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(device);
  dfree(dist);
  dfree(pred);
  dfree(node);
  dfree(jobs);
  dfree(arcs);
  dfree(narcs);
  dfree(pj);
  for (void* p : old) (void)hipFree(p);
  (void)hipSetDevice(cur);
}

// (outgrown buffers are kept until the scratch dies: a hipFree would wait for the whole device)
hipError_t CchScratch::ensure(size_t J, size_t P, int stride, int max_arcs) {
  hipError_t e = hipSuccess;
  auto retire = [&](auto*& p) {
    if (p) old.push_back((void*)p);
    p = nullptr;
  };
  if (J > jobs_cap) {
    retire(dist);
    retire(pred);
    retire(node);
    retire(jobs);
    const size_t cap = std::max(J, jobs_cap * 3 / 2);
    if ((e = dmalloc(dist, cap * stride)) != hipSuccess) return e;
    if ((e = dmalloc(pred, cap * stride)) != hipSuccess) return e;
    if ((e = dmalloc(node, cap * stride)) != hipSuccess) return e;
    if ((e = dmalloc(jobs, cap)) != hipSuccess) return e;
    jobs_cap = cap;
  }
  if (P > pairs_cap) {
    retire(arcs);
    retire(narcs);
    const size_t cap = std::max(P, pairs_cap * 3 / 2);
    if ((e = dmalloc(arcs, cap * (size_t)max_arcs)) != hipSuccess) return e;
    if ((e = dmalloc(narcs, cap)) != hipSuccess) return e;
    pairs_cap = cap;
  }
  return e;
}

CchGpu::CchGpu(rcch::Topology T, const float* length, const uint8_t* road_class, const uint8_t* base_traffic,
               int device)
    : T_(std::move(T)), dev_(device) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (hipSetDevice(dev_) != hipSuccess) throw std::runtime_error("CchGpu: bad device");
  const int N = T_.N;
  const int64_t M = T_.M, E = T_.E;
  if (M >= (int64_t)1 << 31 || E >= (int64_t)1 << 31) throw std::runtime_error("CchGpu: graph too large");
  std::vector<int32_t> up_ptr32(N + 1);
  for (int r = 0; r <= N; ++r) up_ptr32[r] = (int32_t)T_.up_ptr[r];
  // level work prefixes: basic items per node = k(k+1)/2 (k finalize + k(k-1)/2 pairs), height
  // order; perfect items = k(k-1), depth order
  bofs_.assign(N + 1, 0);
  pofs_.assign(N + 1, 0);
  aofs_.assign(N + 1, 0);
  for (int i = 0; i < N; ++i) {
    const int64_t kb = T_.up_ptr[T_.hlev_nodes[i] + 1] - T_.up_ptr[T_.hlev_nodes[i]];
    bofs_[i + 1] = bofs_[i] + kb * (kb + 1) / 2;
    const int64_t kp = T_.up_ptr[T_.dlev_nodes[i] + 1] - T_.up_ptr[T_.dlev_nodes[i]];
    pofs_[i + 1] = pofs_[i] + kp * (kp - 1);
    aofs_[i + 1] = aofs_[i] + kp;
  }
  plev_kmax_.assign((size_t)T_.max_depth + 1, 0);
  for (int d = 0; d <= T_.max_depth; ++d)
    for (int64_t i = T_.dlev_ptr[d]; i < T_.dlev_ptr[d + 1]; ++i) {
      const int x = T_.dlev_nodes[i];
      plev_kmax_[d] = std::max(plev_kmax_[d], (int)(T_.up_ptr[x + 1] - T_.up_ptr[x]));
    }
  hipError_t e = hipSuccess;
  auto ck = [&](hipError_t x) {
    if (x != hipSuccess && e == hipSuccess) e = x;
  };
  ck(up_copy(d_up_ptr, up_ptr32.data(), N + 1));
  ck(up_copy(d_up_head, T_.up_head.data(), M));
  ck(up_copy(d_arc_lo, T_.arc_lo.data(), M));
  ck(up_copy(d_parent, T_.parent.data(), N));
  ck(up_copy(d_depth, T_.depth.data(), N));
  ck(up_copy(d_rank, T_.rank.data(), N));
  ck(up_copy(d_node, T_.node.data(), N));
  ck(up_copy(d_edge_arc, T_.edge_arc.data(), E));
  ck(up_copy(d_edge_dir, T_.edge_dir.data(), E));
  ck(up_copy(d_length, length, E));
  if (road_class) ck(up_copy(d_class, road_class, E));
  if (base_traffic) ck(up_copy(d_base_traffic, base_traffic, E));
  ck(up_copy(d_hnodes, T_.hlev_nodes.data(), N));
  ck(up_copy(d_dnodes, T_.dlev_nodes.data(), N));
  ck(up_copy(d_bofs, bofs_.data(), N + 1));
  ck(up_copy(d_pofs, pofs_.data(), N + 1));
  ck(up_copy(d_aofs, aofs_.data(), N + 1));

  ck(alloc_scratch(cs0_));
  if (builder_max_wg_.load() < 0) builder_max_wg_.store(M >= 20000000LL ? 512 : 0);
  // triangle table within ROUTEST_CCH_TRI_GB of HBM (default 48 — a 1M-node city needs ~38 GB of the 288; 0 disables)
  if (e == hipSuccess) {
    std::vector<int64_t> tofs(N + 1, 0);
    for (int z = 0; z < N; ++z) {
      const int64_t k = T_.up_ptr[z + 1] - T_.up_ptr[z];
      tofs[z + 1] = tofs[z] + k * (k - 1) / 2;
    }
    const char* env = std::getenv("ROUTEST_CCH_TRI_GB");
    const double budget = env ? std::atof(env) : 48.0;
    const int64_t T = tofs[N];
    if (T > 0 && (double)T * 4.0 <= budget * 1073741824.0 && T < ((int64_t)1 << 40)) {
      if (up_copy(d_tofs, tofs.data(), N + 1) == hipSuccess && dmalloc(d_tri, (size_t)T) == hipSuccess) {
        hipLaunchKernelGGL(tri_build_kernel, dim3((unsigned)std::min<int64_t>(65536, (T + 255) / 256)), dim3(256), 0, 0,
                           d_up_ptr, d_up_head, d_tofs, N, (long long)T, d_tri);
        if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess) {
          n_tri = T;
          build_supernodes(tofs);
          build_tasks(tofs);
          build_pull_records(tofs);
        } else {
          dfree(d_tri);
          dfree(d_tofs);
        }
      } else {
        (void)hipGetLastError();
        dfree(d_tri);
        dfree(d_tofs);
      }
    }
  }
  (void)hipSetDevice(cur);
  if (e != hipSuccess) throw std::runtime_error(std::string("CchGpu: ") + hipGetErrorString(e));
  if (const char* gb = std::getenv("ROUTEST_CCH_CACHE_GB")) cache_gb_ = std::atof(gb);
}

// The supernodal plan (metric-independent, once per graph).  A supernode is a maximal chain of ranks
// c0, c0 + 1, ... in which every node is the only child of the next; the chains of at least
// ROUTEST_CCH_DENSE nodes (default 8; 0: off) and all their ancestor chains are dense fronts, levelled
// by height in the tree of fronts.  Per level: the gather rows, and per block the panel / trailing
// (basic) and GEMM / solve / K x K (perfect) workgroup lists.  The nodes outside the fronts keep the
// per-level kernels: basic by etree height (their heights end far below the top), perfect by depth
// below their nearest front (all of their ancestors inside fronts are final by then).
void CchGpu::build_supernodes(const std::vector<int64_t>& tofs) {
  const char* v = std::getenv("ROUTEST_CCH_DENSE");
  const int S0 = v ? std::atoi(v) : 8;
  const int N = T_.N;
  if (S0 <= 0 || N < 2 || d_tri == nullptr) return;
  std::vector<int> nch(N, 0);
  for (int i = 0; i < N; ++i)
    if (T_.parent[i] >= 0) ++nch[T_.parent[i]];
  std::vector<int> sid(N), sc0, ssz;
  for (int i = 0; i < N; ++i) {
    if (!(i > 0 && T_.parent[i - 1] == i && nch[i] == 1)) {
      sc0.push_back(i);
      ssz.push_back(0);
    }
    sid[i] = (int)sc0.size() - 1;
    ++ssz.back();
  }
  const int NS = (int)sc0.size();
  std::vector<int> spar(NS, -1);
  for (int s = 0; s < NS; ++s) {
    const int p = T_.parent[sc0[s] + ssz[s] - 1];
    spar[s] = p >= 0 ? sid[p] : -1;
  }
  std::vector<uint8_t> dense(NS, 0);
  for (int s = 0; s < NS; ++s)
    if (ssz[s] >= S0)
      for (int q = s; q >= 0 && !dense[q]; q = spar[q]) dense[q] = 1;
  std::vector<int> lev(NS, 0);       // children precede parents (ranks grow upward)
  int L = 0;
  for (int s = 0; s < NS; ++s) {
    if (!dense[s]) continue;
    L = std::max(L, lev[s] + 1);
    if (spar[s] >= 0) lev[spar[s]] = std::max(lev[spar[s]], lev[s] + 1);
  }
  if (L == 0) return;
  // fronts: chain, then the top node's upward set; every chain arc must lead into the front
  std::vector<SupNode> sn;
  std::vector<int32_t> fnode;
  std::vector<std::vector<int>> by_lev(L);
  int64_t foff = 0;
  for (int s = 0; s < NS; ++s) {
    if (!dense[s]) continue;
    const int c0 = sc0[s], m = ssz[s], top = c0 + m - 1;
    const int64_t a0 = T_.up_ptr[top], a1 = T_.up_ptr[top + 1];
    const int64_t n = m + (a1 - a0);
    if (n > 32767) return;
    const int32_t* U0 = T_.up_head.data() + a0;
    const int32_t* U1 = T_.up_head.data() + a1;
    for (int i = 0; i < m; ++i)
      for (int64_t a = T_.up_ptr[c0 + i]; a < T_.up_ptr[c0 + i + 1]; ++a) {
        const int h = T_.up_head[a];
        if (!((h > c0 + i && h <= top) || std::binary_search(U0, U1, h))) {
          std::fprintf(stderr, "[cch] rank %d: arc to %d outside its front; supernodal customization off\n", c0 + i, h);
          return;
        }
      }
    by_lev[lev[s]].push_back((int)sn.size());
    sn.push_back(SupNode{0, foff, c0, m, (int32_t)n, (int32_t)fnode.size()});
    for (int i = 0; i < m; ++i) fnode.push_back(c0 + i);
    fnode.insert(fnode.end(), U0, U1);
    foff += n * n;
  }
  const auto cdiv = [](int64_t a, int64_t b) { return (a + b - 1) / b; };
  std::vector<SupWork> work;
  auto range_of = [&](int64_t from) { return SupRange{from, (int64_t)work.size() - from}; };
  // every front row (farc build)
  for (int f = 0; f < (int)sn.size(); ++f)
    for (int i = 0; i < sn[f].n; ++i) work.push_back(SupWork{f, i, 0, 0});
  const SupRange all_rows = range_of(0);
  // the trailing update of front f's block b: targets past the end of the block above it
  auto push_trail = [&](int f, int b) {
    const SupNode& S = sn[f];
    const int nb = (int)cdiv(S.m, SUP_B);
    const int k1 = std::min(SUP_B * (b + 1), S.m);
    const int zr0 = b + 1 < nb ? std::min(k1 + SUP_B, S.m) : k1;
    const int T = (int)cdiv(S.n - zr0, SUP_TT);
    for (int ty = 0; ty < T; ++ty)
      for (int tz = 0; tz < T; ++tz) work.push_back(SupWork{f, b, ty, tz});
  };
  std::vector<SupLevel> levs(L);
  int64_t buf = 0;
  int blocks = 0;
  for (int l = 0; l < L; ++l) {
    SupLevel& SL = levs[l];
    int64_t dofs = 0;
    int nbmax = 0;
    for (int f : by_lev[l]) {
      sn[f].dofs = dofs;
      dofs += (int64_t)sn[f].n * sn[f].n;
      nbmax = std::max(nbmax, (int)cdiv(sn[f].m, SUP_B));
    }
    buf = std::max(buf, dofs);
    blocks += nbmax;
    int64_t w0 = (int64_t)work.size();
    for (int f : by_lev[l])
      for (int i = 0; i < sn[f].n; ++i) work.push_back(SupWork{f, i, 0, 0});
    SL.gather = range_of(w0);
    for (int r = 0; r < nbmax; ++r) {
      // basic, step r: the panels of every front's block r (t1 = -1) beside the trailing updates of
      // its block r - 1 (sup_step_basic_kernel)
      w0 = (int64_t)work.size();
      for (int f : by_lev[l]) {
        const SupNode& S = sn[f];
        const int nb = (int)cdiv(S.m, SUP_B);
        if (nb > r) {
          const int k1 = std::min(SUP_B * (r + 1), S.m);
          const int nt = std::max<int64_t>(1, cdiv(S.n - k1, SUP_PJ));
          for (int t = 0; t < nt; ++t) work.push_back(SupWork{f, r, t, -1});
        }
        if (r >= 1 && nb > r - 1) push_trail(f, r - 1);
      }
      SL.panel.push_back(range_of(w0));
      // perfect, launch pair r: [the K x K kernels of the blocks solved at r - 1 | the products of
      // the r-th blocks from the top], then the r-th blocks' solves
      w0 = (int64_t)work.size();
      for (int f : by_lev[l]) {
        const SupNode& S = sn[f];
        const int nb = (int)cdiv(S.m, SUP_B);
        if (r >= 1 && nb > r - 1) work.push_back(SupWork{f, nb - r, -1, 0});
        if (nb <= r) continue;
        const int b = nb - 1 - r, k1 = std::min(SUP_B * (b + 1), S.m), nF = S.n - k1;
        const int zlo = b + 1 < nb ? std::min(k1 + SUP_B, S.m) : k1;
        if (nF <= 0 || S.n - zlo <= 0) continue;
        const int TY = (int)cdiv(nF, SUP_G1Y), Z = (int)cdiv(S.n - zlo, SUP_G1Z);
        for (int dir = 0; dir < 2; ++dir)
          for (int zs = 0; zs < Z; ++zs)
            for (int ty = 0; ty < TY; ++ty) work.push_back(SupWork{f, b, ty, (zs << 1) | dir});
      }
      SL.px.push_back(range_of(w0));
      w0 = (int64_t)work.size();
      for (int f : by_lev[l]) {
        const SupNode& S = sn[f];
        const int nb = (int)cdiv(S.m, SUP_B);
        if (nb <= r) continue;
        const int b = nb - 1 - r, k1 = std::min(SUP_B * (b + 1), S.m), nF = S.n - k1;
        for (int t = 0; t < (int)cdiv(nF, SUP_SJ); ++t) work.push_back(SupWork{f, b, t, 0});
      }
      SL.py.push_back(range_of(w0));
    }
    {
      const int64_t w1 = (int64_t)work.size();
      for (int f : by_lev[l]) {
        const int nb = (int)cdiv(sn[f].m, SUP_B);
        if (nb == nbmax) work.push_back(SupWork{f, 0, -1, 0});   // the last blocks' K x K
      }
      SL.px.push_back(range_of(w1));
      const int64_t w2 = (int64_t)work.size();
      for (int f : by_lev[l])
        if ((int)cdiv(sn[f].m, SUP_B) == nbmax) push_trail(f, nbmax - 1);   // the last blocks' trailing
      SL.panel.push_back(range_of(w2));
    }
  }
  for (SupWork& wk : work) wk.sn = sn[wk.s];
  // the other nodes: perfect by depth below their nearest front
  std::vector<uint8_t> node_in(N, 0);
  int nodes_in = 0;
  for (int i = 0; i < N; ++i)
    if (dense[sid[i]]) {
      node_in[i] = 1;
      ++nodes_in;
    }
  std::vector<int> rd(N, -1);
  int R = 0, hmax = -1;
  for (int x = N - 1; x >= 0; --x) {
    if (node_in[x]) continue;
    const int p = T_.parent[x];
    rd[x] = (p < 0 || node_in[p]) ? 0 : rd[p] + 1;
    R = std::max(R, rd[x] + 1);
    hmax = std::max(hmax, T_.height[x]);
  }
  std::vector<int64_t> rptr(R + 1, 0);
  for (int x = 0; x < N; ++x)
    if (rd[x] >= 0) ++rptr[rd[x] + 1];
  for (int d = 0; d < R; ++d) rptr[d + 1] += rptr[d];
  std::vector<int> order(rptr[R]);
  {
    std::vector<int64_t> pos(rptr.begin(), rptr.end() - 1);
    for (int x = 0; x < N; ++x)
      if (rd[x] >= 0) order[pos[rd[x]]++] = x;
  }
  std::vector<PArc> parc;
  std::vector<int64_t> raofs(R + 1, 0);
  std::vector<int> rnodes(R, 0), rkmax(R, 0);
  std::vector<uint8_t> rmulti(R, 0);
  for (int d = 0; d < R; ++d) {
    raofs[d] = (int64_t)parc.size();
    for (int64_t q = rptr[d]; q < rptr[d + 1]; ++q) {
      const int x = order[q];
      const int a0 = (int)T_.up_ptr[x], k = (int)(T_.up_ptr[x + 1] - T_.up_ptr[x]);
      if (k > 0xFFFF) return;
      ++rnodes[d];
      rkmax[d] = std::max(rkmax[d], k);
      if (k >= 2) rmulti[d] = 1;
      for (int ia = 0; ia < k; ++ia)
        parc.push_back(PArc{tofs[x], a0, (int32_t)T_.up_head[a0 + ia], (uint16_t)k, (uint16_t)ia, 0});
    }
  }
  raofs[R] = (int64_t)parc.size();
  // device copies; any failure leaves the plan off (nothing filtered yet)
  SupNode* dsn = nullptr;
  SupWork* dwk = nullptr;
  int32_t *dfn = nullptr, *dfa = nullptr;
  PArc* dpa = nullptr;
  bool ok = up_copy(dsn, sn.data(), sn.size()) == hipSuccess && up_copy(dwk, work.data(), work.size()) == hipSuccess &&
            up_copy(dfn, fnode.data(), fnode.size()) == hipSuccess && dmalloc(dfa, (size_t)foff) == hipSuccess &&
            up_copy(dpa, parc.data(), parc.size()) == hipSuccess && dmalloc(cs0_.sup_buf, 3 * (size_t)buf) == hipSuccess;
  if (ok) {
    hipLaunchKernelGGL(sup_farc_kernel, dim3((unsigned)cdiv(all_rows.cnt, 4)), dim3(256), 0, 0, dsn, dwk + all_rows.off,
                       (long long)all_rows.cnt, dfn, d_up_ptr, d_up_head, dfa);
    ok = hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess;
  }
  if (!ok) {
    (void)hipGetLastError();
    dfree(dsn);
    dfree(dwk);
    dfree(dfn);
    dfree(dfa);
    dfree(dpa);
    dfree(cs0_.sup_buf);
    std::fprintf(stderr, "[cch] supernodal plan: device allocation failed; per-level customization\n");
    return;
  }
  d_sup_sn = dsn;
  d_sup_work = dwk;
  d_sup_fnode = dfn;
  d_sup_farc = dfa;
  d_parc2 = dpa;
  sup_buf_entries_ = buf;
  sup_lev_ = std::move(levs);
  sup_node_ = std::move(node_in);
  rlev_aofs_ = std::move(raofs);
  rlev_nodes_ = std::move(rnodes);
  rlev_kmax_ = std::move(rkmax);
  rlev_multi_ = std::move(rmulti);
  sup_fronts_ = (int)sn.size();
  sup_nodes_ = nodes_in;
  sup_blocks_ = blocks;
  sparse_heights_ = hmax + 1;
  sup_on_ = true;
}

// the task tables of the task-table customization (metric-independent; level order)
// the perfect pull's per-arc records (ROUTEST_CCH_PARC=0: the binary search instead)
void CchGpu::build_pull_records(const std::vector<int64_t>& tofs) {
  if (const char* v = std::getenv("ROUTEST_CCH_PARC"))
    if (std::string(v) == "0") return;
  const int N = T_.N;
  std::vector<PArc> parc((size_t)aofs_[N]);
  for (int i = 0; i < N; ++i) {
    const int x = T_.dlev_nodes[i];
    const int a0 = (int)T_.up_ptr[x], k = (int)(T_.up_ptr[x + 1] - T_.up_ptr[x]);
    if (k > 0xFFFF) return;                   // (never on road graphs)
    for (int ia = 0; ia < k; ++ia)
      parc[(size_t)aofs_[i] + ia] = PArc{tofs[x], a0, (int32_t)T_.up_head[a0 + ia], (uint16_t)k, (uint16_t)ia, 0};
  }
  PArc* dp = nullptr;
  if (!parc.empty() && up_copy(dp, parc.data(), parc.size()) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  d_parc = dp;
  // the narrow top of the perfect phase: the longest prefix of depths with at most `thr` arcs each
  // (ROUTEST_CCH_TAIL as for the basic phase)
  const char* v = std::getenv("ROUTEST_CCH_TAIL");
  const int64_t thr = v && !sup_on_ ? std::atoll(v) : 0;
  int d = 0;
  while (thr > 0 && d < T_.max_depth && aofs_[T_.dlev_ptr[d + 1]] - aofs_[T_.dlev_ptr[d]] <= thr) ++d;
  if (d >= 2) {
    std::vector<int> ends;
    int64_t mx = 0;
    const int64_t base = aofs_[T_.dlev_ptr[0]];
    for (int l = 0; l < d; ++l) {
      ends.push_back((int)(aofs_[T_.dlev_ptr[l + 1]] - base));
      mx = std::max<int64_t>(mx, aofs_[T_.dlev_ptr[l + 1]] - aofs_[T_.dlev_ptr[l]]);
    }
    int* de = nullptr;
    if (up_copy(de, ends.data(), ends.size()) == hipSuccess) {
      d_ptail_end_ = de;
      n_ptail_lev_ = d;
      ptail_max_arcs_ = (int)mx;
    } else {
      (void)hipGetLastError();
    }
  }
}

void CchGpu::build_tasks(const std::vector<int64_t>& tofs) {
  if (const char* v = std::getenv("ROUTEST_CCH_TASKS"))
    if (std::string(v) == "0") return;
  const int N = T_.N;
  std::vector<BasicTask> bt;
  std::vector<CustTask> pt;
  btask_ptr_.assign(T_.max_height + 2, 0);
  for (int h = 0; h <= T_.max_height; ++h) {
    for (int64_t q = T_.hlev_ptr[h]; q < T_.hlev_ptr[h + 1]; ++q) {
      const int z = T_.hlev_nodes[q];
      if (sup_on_ && sup_node_[z]) continue;                // a dense front's (sup_panel_body)
      const int k = (int)(T_.up_ptr[z + 1] - T_.up_ptr[z]);
      if (k > 0xFFFE) { bt.clear(); pt.clear(); return; }   // (never on road graphs: k <= ~2k)
      const int a0 = (int)T_.up_ptr[z];
      for (int j0 = 0; j0 < k; j0 += 64)
        bt.push_back(BasicTask{0, z, a0, (uint16_t)k, ROW_FINAL, (uint16_t)j0, 0});
      for (int i = 0; i + 1 < k; ++i) {
        const int64_t rb = tofs[z] + (int64_t)i * (2 * k - i - 1) / 2 - i - 1;
        for (int j0 = i + 1; j0 < k; j0 += 64)
          bt.push_back(BasicTask{rb, z, a0, (uint16_t)k, (uint16_t)i, (uint16_t)j0, 0});
      }
    }
    btask_ptr_[h + 1] = (int64_t)bt.size();
  }
  ptask_ptr_.assign(T_.max_depth + 2, 0);
  const char* pv = std::getenv("ROUTEST_CCH_PERFECT");
  const bool want_p = pv && std::string(pv) == "tasks";       // (the pull kernels need no table)
  for (int d = 0; d <= T_.max_depth && want_p; ++d) {
    for (int64_t q = T_.dlev_ptr[d]; q < T_.dlev_ptr[d + 1]; ++q) {
      const int x = T_.dlev_nodes[q];
      const int k = (int)(T_.up_ptr[x + 1] - T_.up_ptr[x]);
      if (k < 2) continue;
      for (int a = 0; a < k; ++a)
        for (int c0 = 0; c0 < k; c0 += 64) pt.push_back(CustTask{x, (uint16_t)a, (uint16_t)c0});
    }
    ptask_ptr_[d + 1] = (int64_t)pt.size();
  }
  (void)N;
  // the narrow top of the basic phase: the longest suffix of levels with at most `thr` tasks each
  // (ROUTEST_CCH_TAIL=<tasks>; default 0: every level its own launch — run r6m: a 4096-task tail of
  // 500 levels made the basic phase 11.4 -> 39.7 ms, profiles/cch_customize_r6.md)
  {
    const char* v = std::getenv("ROUTEST_CCH_TAIL");
    const int64_t thr = v && !sup_on_ ? std::atoll(v) : 0;
    int h = T_.max_height + 1;
    while (thr > 0 && h > 1 && btask_ptr_[h] - btask_ptr_[h - 1] <= thr) --h;
    if (thr > 0 && h <= T_.max_height && !bt.empty()) {
      std::vector<int> ends;
      int64_t mx = 0;
      for (int l = h; l <= T_.max_height; ++l) {
        ends.push_back((int)(btask_ptr_[l + 1] - btask_ptr_[h]));
        mx = std::max<int64_t>(mx, btask_ptr_[l + 1] - btask_ptr_[l]);
      }
      int* d = nullptr;
      if (up_copy(d, ends.data(), ends.size()) == hipSuccess) {
        d_tail_end_ = d;
        h_tail_ = h;
        n_tail_lev_ = (int)ends.size();
        tail_max_tasks_ = (int)mx;
      } else {
        (void)hipGetLastError();
      }
    }
  }
  BasicTask* db = nullptr;
  CustTask* dp = nullptr;
  const bool ok = up_copy(db, bt.data(), bt.size()) == hipSuccess && up_copy(dp, pt.data(), pt.size()) == hipSuccess;
  d_btask = db;
  d_ptask = dp;
  if (!ok) {
    (void)hipGetLastError();
    dfree(d_btask);
    dfree(d_ptask);
    return;
  }
  n_btask_ = (int64_t)bt.size();
  n_ptask_ = (int64_t)pt.size();
}

CchGpu::~CchGpu() {
  {
    std::lock_guard<std::mutex> lk(bmu_);
    bstop_ = true;
    bq_.clear();
  }
  bcv_.notify_all();
  for (auto& t : bths_)
    if (t.joinable()) t.join();
  for (auto& x : bscr_) free_scratch(*x);
  {
    std::lock_guard<std::mutex> lk(mu_);
    cache_.clear();
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(dev_);
  dfree(d_up_ptr);
  dfree(d_up_head);
  dfree(d_arc_lo);
  dfree(d_parent);
  dfree(d_depth);
  dfree(d_rank);
  dfree(d_node);
  dfree(d_edge_arc);
  dfree(d_edge_dir);
  dfree(d_length);
  dfree(d_class);
  dfree(d_base_traffic);
  dfree(d_hnodes);
  dfree(d_dnodes);
  dfree(d_bofs);
  dfree(d_pofs);
  dfree(d_aofs);
  dfree(d_parc);
  dfree(d_tofs);
  dfree(d_tri);
  dfree(d_btask);
  dfree(d_ptask);
  dfree(d_tail_end_);
  dfree(d_ptail_end_);
  dfree(d_sup_sn);
  dfree(d_sup_work);
  dfree(d_sup_fnode);
  dfree(d_sup_farc);
  dfree(d_parc2);
  free_scratch(cs0_);
  (void)hipSetDevice(cur);
}

void CchGpu::set_eta(const void* blob, int H, const NormParams& np, int variant, int num_cus) {
  std::lock_guard<std::mutex> lk(mu_cust_);
  eta_blob_ = blob;
  eta_H_ = H;
  eta_np_ = np;
  eta_variant_ = variant;
  eta_cus_ = num_cus;
}

hipError_t CchGpu::alloc_scratch(CustScratch& x) {
  const int N = T_.N;
  const int64_t M = T_.M;
  hipError_t e = hipSuccess;
  auto ck = [&](hipError_t r) {
    if (r != hipSuccess && e == hipSuccess) e = r;
  };
  ck(dmalloc(x.up64, M));
  ck(dmalloc(x.dn64, M));
  ck(dmalloc(x.pup, M));
  ck(dmalloc(x.pdn, M));
  ck(dmalloc(x.fcnt, N));
  ck(dmalloc(x.bcnt, N));
  size_t tb = 0;
  ck(hipcub::DeviceScan::InclusiveSum(nullptr, tb, x.fcnt, x.fcnt, N));
  x.cub_bytes = tb;
  ck(hipMalloc(&x.cub, x.cub_bytes ? x.cub_bytes : 1));
  ck(hipHostMalloc((void**)&x.h_stage, (size_t)std::max<int64_t>(1, T_.E) * sizeof(float), hipHostMallocDefault));
  ck(dmalloc(x.tail_ctl, (size_t)T_.max_height + (size_t)T_.max_depth + 8));   // basic | perfect tail
  if (x.tail_ctl != nullptr)
    ck(hipMemset(x.tail_ctl, 0, ((size_t)T_.max_height + (size_t)T_.max_depth + 8) * sizeof(int)));
  if (sup_on_) ck(dmalloc(x.sup_buf, 3 * (size_t)sup_buf_entries_));   // D | SS | SL
  return e;
}

void CchGpu::free_scratch(CustScratch& x) {
  dfree(x.up64);
  dfree(x.dn64);
  dfree(x.pup);
  dfree(x.pdn);
  dfree(x.fcnt);
  dfree(x.bcnt);
  if (x.cub) (void)hipFree(x.cub);
  x.cub = nullptr;
  if (x.rec_buf) (void)hipFree(x.rec_buf);
  x.rec_buf = nullptr;
  dfree(x.min_buf);
  if (x.h_stage) (void)hipHostFree(x.h_stage);
  x.h_stage = nullptr;
  dfree(x.tail_ctl);
  dfree(x.sup_buf);
}

hipError_t CchGpu::context_costs(const CchContext& c, float* d_cost, hipStream_t s, CustScratch* cs) {
  if (eta_blob_ == nullptr || d_class == nullptr || d_base_traffic == nullptr) return hipErrorInvalidValue;
  const int E = (int)T_.E;
  hipError_t e = hipSuccess;
  std::unique_lock<std::mutex> lk(mu_cust_, std::defer_lock);
  if (cs == nullptr) lk.lock();
  CustScratch& X = cs ? *cs : cs0_;
  void*& rec_buf = X.rec_buf;
  float*& min_buf = X.min_buf;
  if (rec_buf == nullptr) {
    if ((e = hipMalloc(&rec_buf, (size_t)2 * E * sizeof(EtaRecordDev))) != hipSuccess) return e;
    if ((e = dmalloc(min_buf, (size_t)2 * E)) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(ctx_records_kernel, dim3(blocks_for(E, 256)), dim3(256), 0, s, d_base_traffic, E, c.weather,
                     c.congestion, c.weekhour, c.driver_age, (EtaRecordDev*)rec_buf);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  e = launch_eta_mlp3_fwd(rec_buf, min_buf, 2 * E, eta_blob_, eta_H_, eta_np_, eta_variant_, eta_cus_, s, 16);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ctx_cost_kernel, dim3(blocks_for(E, 256)), dim3(256), 0, s, min_buf, d_length, d_class, E, d_cost);
  e = hipGetLastError();
  // the shared temporaries are free again only once this stream has consumed them
  if (e == hipSuccess && cs == nullptr) e = hipStreamSynchronize(s);
  return e;
}

hipError_t CchGpu::customize(const float* d_cost, CchMetricDev& m, hipStream_t s, CustScratch* cs) {
  std::unique_lock<std::mutex> lk(mu_cust_, std::defer_lock);
  if (cs == nullptr) lk.lock();
  CustScratch& X = cs ? *cs : cs0_;
  // a background build while queries are served (or always, set_builder_pacing): paced launches
  const bool paced = cs != nullptr && builder_max_wg_.load() > 0 && (pace_always_.load() || serving_now());
  if (paced) n_paced_.fetch_add(1, std::memory_order_relaxed);
  auto t0 = std::chrono::steady_clock::now();
  const int N = T_.N;
  const int64_t M = T_.M, E = T_.E;
  m.device = dev_;
  hipError_t e = hipSuccess;
  auto ck = [&](hipError_t x) {
    if (x != hipSuccess && e == hipSuccess) e = x;
  };
  const auto ta = std::chrono::steady_clock::now();
  if (m.cost == nullptr) ck(dmalloc(m.cost, E));
  if (m.sub_up == nullptr) {
    ck(dmalloc(m.sub_up, 2 * M));
    ck(dmalloc(m.sub_dn, 2 * M));
    ck(dmalloc(m.len_up, M));
    ck(dmalloc(m.len_dn, M));
    ck(dmalloc(m.cnt_up, M));
    ck(dmalloc(m.cnt_dn, M));
    ck(dmalloc(m.f_ptr, N + 1));
    ck(dmalloc(m.b_ptr, N + 1));
  }
  m.alloc_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
  if (e != hipSuccess) return e;
  if (d_cost != m.cost) ck(hipMemcpyAsync(m.cost, d_cost, E * sizeof(float), hipMemcpyDeviceToDevice, s));
  static const bool skip = [] {
    const char* v = std::getenv("ROUTEST_CCH_SKIP");
    return !(v && std::string(v) == "0");
  }();
  // phase boundaries (basic / perfect / prune device times, reported with the metric)
  struct Events {
    hipEvent_t e[4] = {};
    Events() {
      for (auto& x : e)
        if (hipEventCreate(&x) != hipSuccess) x = nullptr;
    }
    ~Events() {
      for (auto& x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } evs;
  hipEvent_t* ev = evs.e;
  // the launch sequence from the weights' reset through the prune counts (ev: phase events, or
  // nullptr when captured into the graph probe below)
  auto core = [&](hipStream_t s, hipEvent_t* ev) {
    const int fill_blocks = (int)std::min<int64_t>(4096, (M + 255) / 256 + 1);
    hipLaunchKernelGGL(fill_u64_kernel, dim3(fill_blocks), dim3(256), 0, s, X.up64, (long long)M, PACK_INF_D);
    hipLaunchKernelGGL(fill_u64_kernel, dim3(fill_blocks), dim3(256), 0, s, X.dn64, (long long)M, PACK_INF_D);
    hipLaunchKernelGGL(edge_scatter_kernel, dim3(blocks_for(E, 256)), dim3(256), 0, s, m.cost, d_edge_arc, d_edge_dir,
                       (int)E, X.up64, X.dn64);
    ck(hipGetLastError());
    if (ev && ev[0]) (void)hipEventRecord(ev[0], s);
    const bool tasks = d_btask != nullptr && d_tri != nullptr;
    // basic, bottom-up by height: the task kernel when the task tables exist
    // (builder_max_wg_ > 0, the background builders: a wide level is launched in pieces of at most
    // max_wg workgroups, one after the other on the stream, so a build never has more than that many
    // workgroups of memory traffic in flight next to the flushes' query kernels)
    const int max_wg = paced ? std::max(0, builder_max_wg_.load(std::memory_order_relaxed)) : 0;
    const long long wave_cap = max_wg > 0 ? 4LL * max_wg : (1LL << 40);
    const bool tail = tasks && h_tail_ >= 0 && X.tail_ctl != nullptr;
    const int h_end = tail ? h_tail_ - 1 : T_.max_height;
    for (int h = 0; h <= h_end && e == hipSuccess && tasks; ++h) {
      const long long ntl = btask_ptr_[h + 1] - btask_ptr_[h];
      for (long long t0 = 0; t0 < ntl && e == hipSuccess; t0 += wave_cap) {
        const long long nt = std::min(wave_cap, ntl - t0);
        const BasicTask* tk = (const BasicTask*)d_btask + btask_ptr_[h] + t0;
        if (skip)
          hipLaunchKernelGGL(basic_task_kernel<true>, dim3((unsigned)((nt + 3) / 4)), dim3(256), 0, s, tk, nt, d_up_ptr,
                             d_up_head, d_tofs, d_tri, X.up64, X.dn64, m.sub_up, m.sub_dn, m.len_up, m.len_dn, m.cnt_up,
                             m.cnt_dn, d_length);
        else
          hipLaunchKernelGGL(basic_task_kernel<false>, dim3((unsigned)((nt + 3) / 4)), dim3(256), 0, s, tk, nt, d_up_ptr,
                             d_up_head, d_tofs, d_tri, X.up64, X.dn64, m.sub_up, m.sub_dn, m.len_up, m.len_dn, m.cnt_up,
                             m.cnt_dn, d_length);
        ck(hipGetLastError());
      }
    }
    if (tail && e == hipSuccess) {
      // the narrow top levels: one persistent launch (basic_tail_kernel), a wave per task at a time
      const int ntask = (int)(btask_ptr_[T_.max_height + 1] - btask_ptr_[h_tail_]);
      int blocks = std::max(1, std::min(256, (tail_max_tasks_ + 3) / 4));
      if (max_wg > 0) blocks = std::min(blocks, max_wg);
      const long long max_ticks = 100LL * 1000 * 1000;     // 1 s of the 100 MHz clock per wait
      ck(hipMemsetAsync(X.tail_ctl, 0, ((size_t)n_tail_lev_ + 2) * sizeof(int), s));
      const BasicTask* tk = (const BasicTask*)d_btask + btask_ptr_[h_tail_];
      if (skip)
        hipLaunchKernelGGL(basic_tail_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, tk, ntask, d_tail_end_,
                           n_tail_lev_, X.tail_ctl, max_ticks, d_up_ptr, d_up_head, d_tri, X.up64, X.dn64, m.sub_up,
                           m.sub_dn, m.len_up, m.len_dn, m.cnt_up, m.cnt_dn, d_length);
      else
        hipLaunchKernelGGL(basic_tail_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, tk, ntask, d_tail_end_,
                           n_tail_lev_, X.tail_ctl, max_ticks, d_up_ptr, d_up_head, d_tri, X.up64, X.dn64, m.sub_up,
                           m.sub_dn, m.len_up, m.len_dn, m.cnt_up, m.cnt_dn, d_length);
      ck(hipGetLastError());
    }
    for (int h = 0; h <= T_.max_height && e == hipSuccess && !tasks; ++h) {
      LevelArgs L{d_up_ptr, d_up_head, d_hnodes, d_bofs, (int)T_.hlev_ptr[h], (int)T_.hlev_ptr[h + 1], 0, 0, d_tofs, d_tri};
      if (L.lo >= L.hi) continue;
      L.base = bofs_[L.lo];
      L.items = bofs_[L.hi] - bofs_[L.lo];
      if (L.items <= 0) continue;
      if (skip)
        hipLaunchKernelGGL(basic_level_kernel<true>, dim3(blocks_for(L.items, 256)), dim3(256), 0, s, L, X.up64, X.dn64,
                           m.sub_up, m.sub_dn, m.len_up, m.len_dn, m.cnt_up, m.cnt_dn, d_length);
      else
        hipLaunchKernelGGL(basic_level_kernel<false>, dim3(blocks_for(L.items, 256)), dim3(256), 0, s, L, X.up64, X.dn64,
                           m.sub_up, m.sub_dn, m.len_up, m.len_dn, m.cnt_up, m.cnt_dn, d_length);
      ck(hipGetLastError());
    }
    // the dense fronts (build_supernodes), bottom-up by front level: gather, then per block of 32
    // pivots the panel and the trailing update (the task table above left their nodes out)
    const bool sup = sup_on_ && tasks;
    if (sup && X.sup_buf == nullptr) ck(hipErrorOutOfMemory);
    const SupNode* sup_sn = (const SupNode*)d_sup_sn;
    const SupWork* sup_wk = (const SupWork*)d_sup_work;
    int2* sup_ss = X.sup_buf ? (int2*)(X.sup_buf + sup_buf_entries_) : nullptr;       // gather's sub-arcs
    int2* sup_sl = X.sup_buf ? (int2*)(X.sup_buf + 2 * sup_buf_entries_) : nullptr;   // ... metres, edges
    for (size_t l = 0; sup && l < sup_lev_.size() && e == hipSuccess; ++l) {
      const SupLevel& SL = sup_lev_[l];
      hipLaunchKernelGGL(sup_gather_basic_kernel, dim3((unsigned)SL.gather.cnt), dim3(256), 0, s, sup_sn,
                         sup_wk + SL.gather.off, d_sup_fnode, d_sup_farc, X.up64, X.dn64, d_up_ptr, d_up_head, m.len_up,
                         m.len_dn, m.cnt_up, m.cnt_dn, X.sup_buf, sup_ss, sup_sl);
      for (size_t r = 0; r < SL.panel.size(); ++r)
        if (SL.panel[r].cnt > 0)
          hipLaunchKernelGGL(sup_step_basic_kernel, dim3((unsigned)SL.panel[r].cnt), dim3(1024), 0, s,
                             sup_wk + SL.panel[r].off, d_sup_farc, X.sup_buf, sup_ss, sup_sl, X.up64, X.dn64, m.sub_up,
                             m.sub_dn, m.len_up, m.len_dn, m.cnt_up, m.cnt_dn, d_length);
      ck(hipGetLastError());
    }
    if (ev && ev[1]) (void)hipEventRecord(ev[1], s);
    // perfect, top-down by depth
    hipLaunchKernelGGL(perfect_init_kernel, dim3(fill_blocks), dim3(256), 0, s, X.up64, X.dn64, X.pup, X.pdn, (long long)M);
    ck(hipGetLastError());
    // pull (default with the triangle table; ROUTEST_CCH_PERFECT=push: the atomic kernel)
    static const bool pull = [] {
      const char* v = std::getenv("ROUTEST_CCH_PERFECT");
      return !(v && std::string(v) == "push");
    }();
    // perfect: the pull kernels (measured faster than the perfect task kernel: 12.0 vs 15.3 ms on
    // the 100k graph, 227 vs 351 ms on the 1M city; ROUTEST_CCH_PERFECT=tasks selects it)
    static const bool env_ptasks = [] {
      const char* v = std::getenv("ROUTEST_CCH_PERFECT");
      return v && std::string(v) == "tasks";
    }();
    const bool ptasks = env_ptasks && d_ptask != nullptr && !sup;
    for (int d = 0; d <= T_.max_depth && e == hipSuccess && tasks && ptasks; ++d) {
      const long long nt = ptask_ptr_[d + 1] - ptask_ptr_[d];
      if (nt <= 0) continue;
      hipLaunchKernelGGL(perfect_task_kernel, dim3((unsigned)((nt + 3) / 4)), dim3(256), 0, s,
                         (const CustTask*)d_ptask + ptask_ptr_[d], nt, d_up_ptr, d_up_head, d_tofs, d_tri, X.up64, X.dn64,
                         X.pup, X.pdn);
      ck(hipGetLastError());
    }
    // the narrow top depths: one persistent launch (perfect_tail_kernel), a wave per arc at a time
    const bool ptail = !sup && !(tasks && ptasks) && pull && d_tri != nullptr && d_parc != nullptr && n_ptail_lev_ > 0 &&
                       X.tail_ctl != nullptr;
    if (ptail && e == hipSuccess) {
      int* pctl = X.tail_ctl + T_.max_height + 4;
      const int lo = (int)T_.dlev_ptr[0], hi = (int)T_.dlev_ptr[n_ptail_lev_];
      PullArgs P{d_up_ptr, d_up_head, d_dnodes, d_aofs, lo, hi, aofs_[lo], aofs_[hi] - aofs_[lo], d_tofs, d_tri,
                 (const PArc*)d_parc};
      int blocks = std::max(1, std::min(256, (ptail_max_arcs_ + 3) / 4));
      if (max_wg > 0) blocks = std::min(blocks, max_wg);
      ck(hipMemsetAsync(pctl, 0, ((size_t)n_ptail_lev_ + 2) * sizeof(int), s));
      hipLaunchKernelGGL(perfect_tail_kernel, dim3((unsigned)blocks), dim3(256), 0, s, P, (int)P.arcs, d_ptail_end_,
                         n_ptail_lev_, pctl, 100LL * 1000 * 1000, X.up64, X.dn64, X.pup, X.pdn);
      ck(hipGetLastError());
    }
    // one depth level of the pull (nodes: its node count; km: its widest node's arcs)
    auto pull_level = [&](PullArgs P, long long nodes, int km, int wave_km) {
      // mean degree of the level's nodes: wide nodes get a wave per arc, narrow ones a lane per arc —
      // or a level with a node of >= wave_km arcs (below the fronts: a lane looping over a ~200-arc
      // node's candidates was the level's time, 30-50 us, r6ah)
      const bool wave = P.arcs >= 24 * nodes || km >= wave_km;
      // waves per arc by the level's widest node (ROUTEST_CCH_PULL_SPLIT=0: one)
      static const bool split = !(std::getenv("ROUTEST_CCH_PULL_SPLIT") &&
                                  std::string(std::getenv("ROUTEST_CCH_PULL_SPLIT")) == "0");
      // (only where the level's arcs alone do not fill the GPU: 1M-city levels of thousands of wide
      // nodes are bound by their random gathers, and splitting them measured 1 % slower, r5z)
      const int S = (!split || P.arcs >= 8192) ? 1 : (km > 768 ? 4 : (km > 256 ? 2 : 1));
      const long long cap = wave ? std::max(1LL, wave_cap / S) : 64 * wave_cap;   // arcs per piece (see wave_cap)
      const long long arcs = P.arcs, base = P.base;
      for (long long a0 = 0; a0 < arcs && e == hipSuccess; a0 += cap) {
        P.base = base + a0;
        P.arcs = std::min(cap, arcs - a0);
        if (wave && S == 4)
          hipLaunchKernelGGL(perfect_pull_wave_kernel<4>, dim3((unsigned)P.arcs), dim3(256), 0, s, P, X.up64, X.dn64,
                             X.pup, X.pdn);
        else if (wave && S == 2)
          hipLaunchKernelGGL(perfect_pull_wave_kernel<2>, dim3((unsigned)((P.arcs + 1) / 2)), dim3(256), 0, s, P,
                             X.up64, X.dn64, X.pup, X.pdn);
        else if (wave)
          hipLaunchKernelGGL(perfect_pull_wave_kernel<1>, dim3((unsigned)((P.arcs + 3) / 4)), dim3(256), 0, s, P,
                             X.up64, X.dn64, X.pup, X.pdn);
        else
          hipLaunchKernelGGL(perfect_pull_lane_kernel, dim3(blocks_for(P.arcs, 256)), dim3(256), 0, s, P, X.up64,
                             X.dn64, X.pup, X.pdn);
        ck(hipGetLastError());
      }
    };
    for (int d = ptail ? n_ptail_lev_ : 0; d <= T_.max_depth && e == hipSuccess && !(tasks && ptasks) && pull && d_tri != nullptr && !sup; ++d) {
      const int lo = (int)T_.dlev_ptr[d], hi = (int)T_.dlev_ptr[d + 1];
      if (lo >= hi) continue;
      PullArgs P{d_up_ptr, d_up_head, d_dnodes, d_aofs, lo, hi, aofs_[lo], aofs_[hi] - aofs_[lo], d_tofs, d_tri,
                 (const PArc*)d_parc};
      if (P.arcs <= 0 || pofs_[hi] == pofs_[lo]) continue;       // no node of the level has two arcs
      pull_level(P, hi - lo, plev_kmax_[d], 1 << 30);
    }
    // the dense fronts top-down by front level (per block from the top: the (min, +) product through
    // the final part, the solve through K, the K x K targets), then the other nodes by depth below
    // their nearest front, pulled over d_parc2
    for (int l = (int)sup_lev_.size() - 1; sup && l >= 0 && e == hipSuccess; --l) {
      const SupLevel& SL = sup_lev_[l];
      float* Dp = (float*)X.sup_buf;
      hipLaunchKernelGGL(sup_gather_perfect_kernel, dim3(blocks_for(SL.gather.cnt, 4)), dim3(256), 0, s, sup_sn,
                         sup_wk + SL.gather.off, (long long)SL.gather.cnt, d_sup_farc, X.up64, X.dn64, X.pup, X.pdn, Dp);
      for (size_t r = 0; r < SL.px.size(); ++r) {
        if (SL.px[r].cnt > 0)
          hipLaunchKernelGGL(sup_kk_gemm_perfect_kernel, dim3((unsigned)SL.px[r].cnt), dim3(1024), 0, s,
                             sup_wk + SL.px[r].off, d_sup_farc, Dp, X.pup, X.pdn);
        if (r < SL.py.size() && SL.py[r].cnt > 0)
          hipLaunchKernelGGL(sup_solve_perfect_kernel, dim3((unsigned)SL.py[r].cnt), dim3(1024), 0, s, sup_sn,
                             sup_wk + SL.py[r].off, d_sup_farc, Dp, X.pup, X.pdn);
      }
      ck(hipGetLastError());
    }
    for (size_t d = 0; sup && d < rlev_nodes_.size() && e == hipSuccess; ++d) {
      if (!rlev_multi_[d]) continue;
      PullArgs P{d_up_ptr, d_up_head, nullptr, nullptr, 0, 0, rlev_aofs_[d], rlev_aofs_[d + 1] - rlev_aofs_[d], d_tofs,
                 d_tri, (const PArc*)d_parc2};
      static const int wave_km = [] {
        const char* v = std::getenv("ROUTEST_CCH_PULL_WAVE_K");
        return v ? std::atoi(v) : 64;
      }();
      pull_level(P, rlev_nodes_[d], rlev_kmax_[d], wave_km);
    }
    for (int d = 0; d <= T_.max_depth && e == hipSuccess && !(tasks && ptasks) && !(pull && d_tri != nullptr) && !sup; ++d) {
      LevelArgs L{d_up_ptr, d_up_head, d_dnodes, d_pofs, (int)T_.dlev_ptr[d], (int)T_.dlev_ptr[d + 1], 0, 0, d_tofs, d_tri};
      if (L.lo >= L.hi) continue;
      L.base = pofs_[L.lo];
      L.items = pofs_[L.hi] - pofs_[L.lo];
      if (L.items <= 0) continue;
      if (skip)
        hipLaunchKernelGGL(perfect_level_kernel<true>, dim3(blocks_for(L.items, 256)), dim3(256), 0, s, L, X.up64, X.dn64,
                           X.pup, X.pdn);
      else
        hipLaunchKernelGGL(perfect_level_kernel<false>, dim3(blocks_for(L.items, 256)), dim3(256), 0, s, L, X.up64, X.dn64,
                           X.pup, X.pdn);
      ck(hipGetLastError());
    }
    if (ev && ev[2]) (void)hipEventRecord(ev[2], s);
    // prune + compact
    hipLaunchKernelGGL(prune_count_wave_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, d_up_ptr, X.pup, X.pdn,
                       X.up64, X.dn64, N, X.fcnt, X.bcnt);
    ck(hipGetLastError());
  };
  core(s, ev);
  ck(hipMemsetAsync(m.f_ptr, 0, sizeof(int32_t), s));
  ck(hipMemsetAsync(m.b_ptr, 0, sizeof(int32_t), s));
  size_t tb = X.cub_bytes;
  ck(hipcub::DeviceScan::InclusiveSum(X.cub, tb, X.fcnt, m.f_ptr + 1, N, s));
  tb = X.cub_bytes;
  ck(hipcub::DeviceScan::InclusiveSum(X.cub, tb, X.bcnt, m.b_ptr + 1, N, s));
  int32_t tot[4] = {0, 0, 0, 0};
  ck(hipMemcpyAsync(&tot[0], m.f_ptr + N, 4, hipMemcpyDeviceToHost, s));
  ck(hipMemcpyAsync(&tot[1], m.b_ptr + N, 4, hipMemcpyDeviceToHost, s));
  if (X.tail_ctl != nullptr) {      // the tails' timed-out flags (zeroed at allocation; set only on expiry)
    ck(hipMemcpyAsync(&tot[2], X.tail_ctl + 1, 4, hipMemcpyDeviceToHost, s));
    ck(hipMemcpyAsync(&tot[3], X.tail_ctl + T_.max_height + 5, 4, hipMemcpyDeviceToHost, s));
  }
  ck(hipStreamSynchronize(s));
  if (e == hipSuccess && (tot[2] != 0 || tot[3] != 0)) {
    std::fprintf(stderr, "[cch] %s tail kernel: a level wait exceeded its bound; customization failed\n",
                 tot[2] ? "basic" : "perfect");
    e = hipErrorLaunchTimeOut;
  }
  if (e != hipSuccess) return e;
  if (tot[0] > m.kept_f || m.f_rec == nullptr) {
    dfree(m.f_rec);
    ck(dmalloc(m.f_rec, tot[0]));
  }
  if (tot[1] > m.kept_b || m.b_rec == nullptr) {
    dfree(m.b_rec);
    ck(dmalloc(m.b_rec, tot[1]));
  }
  m.kept_f = tot[0];
  m.kept_b = tot[1];
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(prune_scatter_wave_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, d_up_ptr, d_up_head,
                     d_depth, X.pup, X.pdn, X.up64, X.dn64, N, m.f_ptr, m.b_ptr, m.f_rec, m.b_rec);
  ck(hipGetLastError());
  if (ev[3]) (void)hipEventRecord(ev[3], s);
  ck(hipStreamSynchronize(s));
  m.customize_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  float ms = 0.f;
  if (ev[0] && ev[1] && hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) m.basic_ms = ms;
  if (ev[1] && ev[2] && hipEventElapsedTime(&ms, ev[1], ev[2]) == hipSuccess) m.perfect_ms = ms;
  if (ev[2] && ev[3] && hipEventElapsedTime(&ms, ev[2], ev[3]) == hipSuccess) m.prune_ms = ms;
  // diagnostics (ROUTEST_CCH_GRAPH_PROBE=n): the launch sequence above n times eagerly and n times
  // as one captured HIP graph on a private stream, to price the per-level dispatch gaps (the
  // replays recompute this metric's values in place: same inputs, same results)
  static const int probe = [] {
    const char* v = std::getenv("ROUTEST_CCH_GRAPH_PROBE");
    return v ? std::atoi(v) : 0;
  }();
  if (probe > 0 && e == hipSuccess) {
    hipStream_t ps = nullptr;
    hipEvent_t pa = nullptr, pb = nullptr;
    if (hipStreamCreateWithFlags(&ps, hipStreamNonBlocking) == hipSuccess && hipEventCreate(&pa) == hipSuccess &&
        hipEventCreate(&pb) == hipSuccess) {
      float eager = 0.f, graph = 0.f;
      (void)hipEventRecord(pa, ps);
      for (int r = 0; r < probe; ++r) core(ps, nullptr);
      (void)hipEventRecord(pb, ps);
      (void)hipEventSynchronize(pb);
      (void)hipEventElapsedTime(&eager, pa, pb);
      const auto tc = std::chrono::steady_clock::now();
      hipGraph_t g = nullptr;
      hipGraphExec_t ge = nullptr;
      size_t nodes = 0;
      if (hipStreamBeginCapture(ps, hipStreamCaptureModeThreadLocal) == hipSuccess) {
        core(ps, nullptr);
        if (hipStreamEndCapture(ps, &g) == hipSuccess && g != nullptr) {
          (void)hipGraphGetNodes(g, nullptr, &nodes);
          if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) ge = nullptr;
        }
      }
      const double inst_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count();
      if (ge != nullptr) {
        (void)hipGraphLaunch(ge, ps);             // (first replay uploads the graph)
        (void)hipStreamSynchronize(ps);
        (void)hipEventRecord(pa, ps);
        for (int r = 0; r < probe; ++r) (void)hipGraphLaunch(ge, ps);
        (void)hipEventRecord(pb, ps);
        (void)hipEventSynchronize(pb);
        (void)hipEventElapsedTime(&graph, pa, pb);
      }
      std::fprintf(stderr,
                   "[cch graph probe] %d runs: eager %.3f ms/run, graph %.3f ms/run (%zu nodes, capture+instantiate "
                   "%.1f ms)\n",
                   probe, eager / probe, ge ? graph / probe : -1.0, nodes, inst_ms);
      if (ge) (void)hipGraphExecDestroy(ge);
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
    }
    if (pa) (void)hipEventDestroy(pa);
    if (pb) (void)hipEventDestroy(pb);
    if (ps) (void)hipStreamDestroy(ps);
  }
  // the host copy of the costs (maneuver durations, the exact host fallback) is made here, on the
  // builder's stream, before the metric is published: a flush that first meets this context finds
  // it ready instead of copying E floats on its own critical path
  // (through the scratch's pinned stage: a pageable copy is staged by the runtime in pieces on the
  // copy engines the flushes' transfers use)
  const auto th = std::chrono::steady_clock::now();
  m.host_cost.resize((size_t)E);
  if (X.h_stage != nullptr) {
    ck(hipMemcpyAsync(X.h_stage, m.cost, (size_t)E * sizeof(float), hipMemcpyDeviceToHost, s));
    ck(hipStreamSynchronize(s));
    if (e == hipSuccess) std::memcpy(m.host_cost.data(), X.h_stage, (size_t)E * sizeof(float));
  } else {
    ck(hipMemcpyAsync(m.host_cost.data(), m.cost, (size_t)E * sizeof(float), hipMemcpyDeviceToHost, s));
    ck(hipStreamSynchronize(s));
  }
  if (e != hipSuccess) m.host_cost.clear();
  m.hostcopy_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th).count();
  return e;
}

hipError_t CchGpu::metric_from_costs(uint64_t key, const float* d_cost, hipStream_t s,
                                     std::shared_ptr<CchMetricDev>& out) {
  auto m = std::make_shared<CchMetricDev>();
  m->key = key;
  hipError_t e = customize(d_cost, *m, s);
  if (e != hipSuccess) return e;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = cache_.begin(); it != cache_.end(); ++it)
      if ((*it)->key == key) {
        cache_.erase(it);
        break;
      }
  }
  insert_cached(m);
  out = m;
  return hipSuccess;
}

// device bytes of one customized metric (what the LRU budget is divided by)
static int64_t metric_device_bytes(const CchMetricDev& m, int64_t N, int64_t M, int64_t E) {
  return E * 4 + M * (8 + 8 + 4 + 4 + 4 + 4) + (N + 1) * 8 + (m.kept_f + m.kept_b) * 16;
}

void CchGpu::insert_cached(const std::shared_ptr<CchMetricDev>& m) {
  const int64_t b = metric_device_bytes(*m, T_.N, T_.M, T_.E);
  metric_bytes_.store(b);
  std::lock_guard<std::mutex> lk(mu_);
  if (cache_gb_ > 0.0 && b > 0) capacity_ = (int)std::max<int64_t>(4, (int64_t)(cache_gb_ * 1073741824.0 / (double)b));
  cache_.push_front(m);
  while ((int)cache_.size() > capacity_) cache_.pop_back();
}

void CchGpu::set_cache_gb(double gb) {
  std::lock_guard<std::mutex> lk(mu_);
  cache_gb_ = gb > 0.0 ? gb : 0.0;
  const int64_t b = metric_bytes_.load();
  if (cache_gb_ > 0.0 && b > 0) capacity_ = (int)std::max<int64_t>(4, (int64_t)(cache_gb_ * 1073741824.0 / (double)b));
  while ((int)cache_.size() > capacity_) cache_.pop_back();
}

void CchGpu::request_build(const CchContext& c, bool urgent) {
  const uint64_t key = c.key();
  std::shared_ptr<CchMetricDev> m;
  if (cached_metric(key, m)) {
    notify_built(key, true);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(bmu_);
    if (bstop_ || !bpending_.insert(key).second) return;   // stopping, or already queued / building
    if (urgent) bq_.push_front(c);
    else bq_.push_back(c);
    start_builders_locked();
  }
  n_bqueued_.fetch_add(1, std::memory_order_relaxed);
  bcv_.notify_one();
}

// ROUTEST_CCH_BUILDERS concurrent builders (default 3), each with its own temporaries: a
// customization is a chain of dependent level launches that keeps a fraction of the GPU busy, so a
// burst of fresh contexts builds several at a time.  (caller holds bmu_)
void CchGpu::start_builders_locked() {
  if (!bths_.empty() || bstop_) return;
  static const int nb = [] {
    const char* v = std::getenv("ROUTEST_CCH_BUILDERS");
    const int k = v ? std::atoi(v) : 3;
    return k < 1 ? 1 : (k > 8 ? 8 : k);
  }();
  for (int i = 0; i < nb; ++i) bths_.emplace_back([this, i] { builder_loop(i); });
}

// the builders and their temporaries (device + pinned host allocations) now — a route service
// calls this at startup, so no allocation happens on the GPU while flushes are in flight
void CchGpu::start_builders() {
  std::lock_guard<std::mutex> lk(bmu_);
  start_builders_locked();
}

int CchGpu::add_build_listener(std::function<void(uint64_t, bool)> cb) {
  std::lock_guard<std::mutex> lk(lmu_);
  listeners_.emplace_back(next_listener_, std::move(cb));
  return next_listener_++;
}

void CchGpu::remove_build_listener(int id) {
  std::lock_guard<std::mutex> lk(lmu_);
  for (auto it = listeners_.begin(); it != listeners_.end(); ++it)
    if (it->first == id) {
      listeners_.erase(it);
      break;
    }
}

void CchGpu::notify_built(uint64_t key, bool ok) {
  std::lock_guard<std::mutex> lk(lmu_);
  for (auto& l : listeners_) l.second(key, ok);
}

CchGpu::AsyncStats CchGpu::async_stats() {
  AsyncStats a;
  a.queued = n_bqueued_.load();
  a.built = n_bbuilt_.load();
  a.failed = n_bfailed_.load();
  a.build_ms = us_build_.load() / 1e3;
  a.alloc_ms = us_alloc_.load() / 1e3;
  a.hostcopy_ms = us_hostcopy_.load() / 1e3;
  a.paced = n_paced_.load();
  std::lock_guard<std::mutex> lk(bmu_);
  a.pending = (int)bpending_.size();
  return a;
}

void CchGpu::builder_loop(int idx) {
  (void)idx;
  if (hipSetDevice(dev_) != hipSuccess) return;
  CustScratch* xs = nullptr;                // this builder's temporaries (freed by the destructor)
  {
    auto x = std::make_unique<CustScratch>();
    if (alloc_scratch(*x) == hipSuccess) {
      xs = x.get();
      std::lock_guard<std::mutex> lk(bmu_);
      bscr_.push_back(std::move(x));
    } else {
      free_scratch(*x);
      (void)hipGetLastError();              // builds below share cs0_ (under mu_cust_)
    }
  }
  hipStream_t s = nullptr;
  // The builder's kernels run on one CU in every ROUTEST_CCH_BUILDER_CU_SHARE (default 4: 64 of
  // the 256, spread over every XCD): a stream priority only orders dispatch, and the wide leaf
  // levels of a 1M-node customization otherwise fill every CU while the flushes' query kernels
  // wait for slots.  The customization is latency-bound (one dependent level after another), so
  // a quarter of the CUs costs it little.  1: all CUs, lowest priority.
  static const int share = [] {
    const char* v = std::getenv("ROUTEST_CCH_BUILDER_CU_SHARE");
    const int k = v ? std::atoi(v) : 4;
    return k < 1 ? 1 : k;
  }();
  if (share > 1) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_) != hipSuccess || cus <= 0) cus = 256;
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int c = share - 1; c < cus; c += share) mask[(size_t)c / 32] |= 1u << (c % 32);
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
      (void)hipGetLastError();
      s = nullptr;
    }
  }
  if (s == nullptr) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least) != hipSuccess) {
      (void)hipGetLastError();
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
    }
  }
  while (true) {
    CchContext c;
    {
      std::unique_lock<std::mutex> lk(bmu_);
      bcv_.wait(lk, [&] { return bstop_ || !bq_.empty(); });
      if (bstop_) break;
      c = bq_.front();
      bq_.pop_front();
    }
    std::shared_ptr<CchMetricDev> m;
    bool fresh = false;
    const auto tb = std::chrono::steady_clock::now();
    const bool ok = s != nullptr && metric_for(c, s, m, &fresh, xs) == hipSuccess;
    if (ok && fresh && m) {
      us_build_.fetch_add((long long)(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tb).count()));
      us_alloc_.fetch_add((long long)(m->alloc_ms * 1e3));
      us_hostcopy_.fetch_add((long long)(m->hostcopy_ms * 1e3));
    }
    if (!ok) (void)hipGetLastError();
    (ok ? n_bbuilt_ : n_bfailed_).fetch_add(1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(bmu_);
      bpending_.erase(c.key());
    }
    notify_built(c.key(), ok);
  }
  if (s) (void)hipStreamDestroy(s);
}

bool CchGpu::cached_metric(uint64_t key, std::shared_ptr<CchMetricDev>& out) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto it = cache_.begin(); it != cache_.end(); ++it)
    if ((*it)->key == key) {
      out = *it;
      cache_.splice(cache_.begin(), cache_, it);
      return true;
    }
  return false;
}

hipError_t CchGpu::metric_for(const CchContext& c, hipStream_t s, std::shared_ptr<CchMetricDev>& out, bool* fresh,
                              CustScratch* cs) {
  const uint64_t key = c.key();
  if (fresh) *fresh = false;
  auto lookup = [&]() -> bool { return cached_metric(key, out); };
  if (lookup()) return hipSuccess;
  {
    // a context another caller is building: wait for it, then hit; different contexts build
    // concurrently (each caller on its own stream and temporaries)
    std::unique_lock<std::mutex> lk(mu_inflight_);
    cv_inflight_.wait(lk, [&] { return inflight_.count(key) == 0; });
    if (lookup()) return hipSuccess;
    inflight_.insert(key);
  }
  struct Done {
    CchGpu* g;
    uint64_t k;
    ~Done() {
      {
        std::lock_guard<std::mutex> lk(g->mu_inflight_);
        g->inflight_.erase(k);
      }
      g->cv_inflight_.notify_all();
    }
  } done{this, key};
  auto m = std::make_shared<CchMetricDev>();
  m->key = key;
  m->device = dev_;
  const auto ta = std::chrono::steady_clock::now();
  hipError_t e = dmalloc(m->cost, T_.E);
  m->alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
  if (e != hipSuccess) return e;
  auto t0 = std::chrono::steady_clock::now();
  e = context_costs(c, m->cost, s, cs);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  m->cost_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  e = customize(m->cost, *m, s, cs);
  if (e != hipSuccess) return e;
  insert_cached(m);
  out = m;
  if (fresh) *fresh = true;
  return hipSuccess;
}

hipError_t CchGpu::launch_unpack(const CchMetricDev* m, const CchMView* mv, const int* grp, int Q, const int* d_src,
                                 CchScratch& sc, const CchRouteOut& o, hipStream_t s) {
  static const bool serial_only = [] {
    const char* v = std::getenv("ROUTEST_CCH_UNPACK");
    return v && std::string(v) == "serial";
  }();
  const int32_t* sub_up = m ? m->sub_up : nullptr;
  const int32_t* sub_dn = m ? m->sub_dn : nullptr;
  if (!serial_only) {
    constexpr int G = 64 / UNPACK_LANES;
    hipLaunchKernelGGL(unpack_coop_kernel, dim3((Q + G - 1) / G), dim3(64), 0, s, Q, d_src, sc.arcs, sc.narcs, MAX_ARCS,
                       sub_up, sub_dn, m ? m->cnt_up : nullptr, m ? m->cnt_dn : nullptr, d_arc_lo, d_up_head, d_node,
                       o.status, o.len, o.path, o.max_path, o.edges, mv, grp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(unpack_kernel, dim3(blocks_for(Q, 64)), dim3(64), 0, s, Q, d_src, sc.arcs, sc.narcs, MAX_ARCS,
                     sub_up, sub_dn, d_arc_lo, d_up_head, d_node, o.status, o.len, o.path, o.max_path,
                     serial_only ? -1 : UNPACK_MAX_ARCS, o.edges, mv, grp);
  return hipGetLastError();
}

hipError_t CchGpu::route_impl(const CchMetricDev* m, const CchMView* mv, const int* grp, const int* d_src,
                              const int* d_dst, int Q, const CchRouteOut& o, CchScratch& sc, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  const int S = stride();
  sc.device = dev_;
  sc.chain_tag = 0;
  hipError_t e = sc.ensure((size_t)2 * Q, (size_t)Q, S, MAX_ARCS);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(route_jobs_kernel, dim3(blocks_for(Q, 256)), dim3(256), 0, s, d_src, d_dst, Q, d_rank, T_.N,
                     sc.jobs);
  hipLaunchKernelGGL(sweep_kernel, dim3(2 * Q), dim3(64), (size_t)S * 8, s, sc.jobs, 2 * Q, d_parent, d_depth, T_.N,
                     m ? m->f_ptr : nullptr, m ? m->f_rec : nullptr, m ? m->b_ptr : nullptr, m ? m->b_rec : nullptr, S,
                     sc.dist, sc.pred, sc.node, mv, grp, 2);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(meet_kernel, dim3(Q), dim3(64), 0, s, Q, nullptr, nullptr, 0, 1, sc.jobs, S, sc.dist, sc.pred,
                     sc.node, d_depth, d_arc_lo, m ? m->len_up : nullptr, m ? m->len_dn : nullptr, o.sec, o.metres,
                     o.status, o.path ? sc.arcs : nullptr, o.path ? sc.narcs : nullptr, MAX_ARCS, mv, grp, 1);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (o.path != nullptr) e = launch_unpack(m, mv, grp, Q, d_src, sc, o, s);
  return e;
}

hipError_t CchGpu::route(const CchMetricDev& m, const int* d_src, const int* d_dst, int Q, const CchRouteOut& o,
                         CchScratch& sc, hipStream_t s) {
  return route_impl(&m, nullptr, nullptr, d_src, d_dst, Q, o, sc, s);
}

hipError_t CchGpu::route_multi(const CchMView* d_mv, const int* d_grp, const int* d_src, const int* d_dst, int Q,
                               const CchRouteOut& o, CchScratch& sc, hipStream_t s) {
  if (d_mv == nullptr || d_grp == nullptr) return hipErrorInvalidValue;
  return route_impl(nullptr, d_mv, d_grp, d_src, d_dst, Q, o, sc, s);
}

hipError_t CchGpu::matrix_impl(const CchMetricDev* m, const CchMView* mv, const int* grp, const int* d_pts,
                               const int* d_npts, int R, int NM, float* d_sec, float* d_met, double* d_D64,
                               CchScratch& sc, hipStream_t s) {
  if (R <= 0 || NM <= 0) return hipSuccess;
  if (d_sec == nullptr || d_met == nullptr) return hipErrorInvalidValue;   // the meet writes both
  const int S = stride();
  sc.device = dev_;
  const size_t J = (size_t)R * NM * 2, P = (size_t)R * NM * NM;
  // pair job indices live in the arcs buffer (2 ints per pair)
  hipError_t e = sc.ensure(J, (P * 2 + MAX_ARCS - 1) / MAX_ARCS + 1, S, MAX_ARCS);
  if (e != hipSuccess) return e;
  int32_t* pjf = sc.arcs;
  int32_t* pjb = sc.arcs + P;
  float* sec = d_sec;
  float* met = d_met;
  hipLaunchKernelGGL(matrix_jobs_kernel, dim3(blocks_for((long long)R * NM, 256)), dim3(256), 0, s, d_pts, d_npts, R, NM,
                     d_rank, T_.N, sc.jobs);
  hipLaunchKernelGGL(matrix_pairs_kernel, dim3(blocks_for((long long)P, 256)), dim3(256), 0, s, d_npts, R, NM, pjf, pjb);
  // (job 2(r NM + i) + dir and pair r NM^2 + i NM + j belong to request row r)
  hipLaunchKernelGGL(sweep_kernel, dim3((unsigned)J), dim3(64), (size_t)S * 8, s, sc.jobs, (int)J, d_parent, d_depth,
                     T_.N, m ? m->f_ptr : nullptr, m ? m->f_rec : nullptr, m ? m->b_ptr : nullptr,
                     m ? m->b_rec : nullptr, S, sc.dist, sc.pred, sc.node, mv, grp, 2 * NM);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(meet_kernel, dim3((unsigned)P), dim3(64), 0, s, (int)P, pjf, pjb, 0, 0, sc.jobs, S, sc.dist,
                     sc.pred, sc.node, d_depth, d_arc_lo, m ? m->len_up : nullptr, m ? m->len_dn : nullptr, sec, met,
                     nullptr, nullptr, nullptr, MAX_ARCS, mv, grp, NM * NM);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(matrix_out_kernel, dim3(blocks_for((long long)P, 256)), dim3(256), 0, s, d_npts, R, NM, sec, met,
                     d_D64);
  e = hipGetLastError();
  sc.chain_tag = e == hipSuccess ? ++tag_ctr_ : 0;
  sc.chain_nm = NM;
  sc.chain_r = R;
  return e;
}

hipError_t CchGpu::matrix(const CchMetricDev& m, const int* d_pts, const int* d_npts, int R, int NM, float* d_sec,
                          float* d_met, double* d_D64, CchScratch& sc, hipStream_t s) {
  return matrix_impl(&m, nullptr, nullptr, d_pts, d_npts, R, NM, d_sec, d_met, d_D64, sc, s);
}

hipError_t CchGpu::matrix_multi(const CchMView* d_mv, const int* d_row_grp, const int* d_pts, const int* d_npts, int R,
                                int NM, float* d_sec, float* d_met, double* d_D64, CchScratch& sc, hipStream_t s) {
  if (d_mv == nullptr || d_row_grp == nullptr) return hipErrorInvalidValue;
  return matrix_impl(nullptr, d_mv, d_row_grp, d_pts, d_npts, R, NM, d_sec, d_met, d_D64, sc, s);
}

hipError_t CchGpu::legs_impl(const CchMetricDev* m, const CchMView* mv, const int* grp, const int* d_src,
                             const int* d_r, const int* d_i, const int* d_j, int Q, uint64_t tag, const CchRouteOut& o,
                             CchScratch& sc, hipStream_t s) {
  if (Q <= 0) return hipSuccess;
  if (tag == 0 || tag != sc.chain_tag) return hipErrorInvalidValue;   // chains overwritten since
  const int S = stride();
  hipError_t e = sc.ensure(0, (size_t)Q, S, MAX_ARCS);
  if (e != hipSuccess) return e;
  if ((size_t)Q > sc.pj_cap) {
    if (sc.pj) sc.old.push_back((void*)sc.pj);
    sc.pj = nullptr;
    const size_t cap = std::max((size_t)Q, sc.pj_cap * 3 / 2);
    if ((e = dmalloc(sc.pj, 2 * cap)) != hipSuccess) return e;
    sc.pj_cap = cap;
  }
  int32_t* pjf = sc.pj;
  int32_t* pjb = sc.pj + sc.pj_cap;
  hipLaunchKernelGGL(leg_pairs_kernel, dim3(blocks_for(Q, 256)), dim3(256), 0, s, sc.chain_nm, d_r, d_i, d_j, Q,
                     sc.chain_r, pjf, pjb);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(meet_kernel, dim3(Q), dim3(64), 0, s, Q, pjf, pjb, 0, 0, sc.jobs, S, sc.dist, sc.pred, sc.node,
                     d_depth, d_arc_lo, m ? m->len_up : nullptr, m ? m->len_dn : nullptr, o.sec, o.metres, o.status,
                     o.path ? sc.arcs : nullptr, o.path ? sc.narcs : nullptr, MAX_ARCS, mv, grp, 1);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (o.path != nullptr) e = launch_unpack(m, mv, grp, Q, d_src, sc, o, s);
  return e;
}

hipError_t CchGpu::legs_from_matrix(const CchMetricDev& m, const int* d_src, const int* d_r, const int* d_i,
                                    const int* d_j, int Q, uint64_t tag, const CchRouteOut& o, CchScratch& sc,
                                    hipStream_t s) {
  return legs_impl(&m, nullptr, nullptr, d_src, d_r, d_i, d_j, Q, tag, o, sc, s);
}

hipError_t CchGpu::legs_from_matrix_multi(const CchMView* d_mv, const int* d_grp, const int* d_src, const int* d_r,
                                          const int* d_i, const int* d_j, int Q, uint64_t tag, const CchRouteOut& o,
                                          CchScratch& sc, hipStream_t s) {
  if (d_mv == nullptr || d_grp == nullptr) return hipErrorInvalidValue;
  return legs_impl(nullptr, d_mv, d_grp, d_src, d_r, d_i, d_j, Q, tag, o, sc, s);
}

}  // namespace rt
