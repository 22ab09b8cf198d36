// K9: batched point-to-point A* on a road graph with learned edge costs (north-star config 5).
// Conceptually replaces the reference's per-trip ORS directions calls (RO/Flaskr/utils.py:55-62,
// 151-156), which it issues one at a time over HTTPS.
//
// Per-search state is SPARSE: every search owns an open-addressing hash table of 16-byte entries
//   { key = node id, h = cached heuristic (NaN: not computed yet), w = g (f32) << 32 | closed | parent slot }
// sized to what the search may touch, not to the graph — workspace is O(slots x table), independent
// of N, so a 1M-node graph serves as many concurrent searches as a 10k-node one (the round-2 design
// kept a dense [slots, N] state plus a [slots, N] heuristic cache: 153 GB for 80k searches on a
// 100k-node graph, and no 1M-node graph fit at all).  Linear probing over a multiplicative hash
// (hslot); a relaxation's first probe is issued with the edge loads, like the dense word was.
// Parent pointers are table slots, so the path walk needs no probing; the reset list holds slots.
//
// Three tiers, each an AstarWs (tables + heap rows + reset lists), run by astar_search():
//   lane  — one LANE per query, an 8-ary lane heap (LaneHeap), `lane_pops` pops in small tables
//           (a few thousand entries): most legs finish here;
//   wave  — one WAVE per remaining query (table/heap overflow or pop budget spent), expanding a whole
//           f-band at once (label-correcting, exact) in medium tables; the launch is no longer as
//           long as the single longest search;
//   big   — searches that overflowed a medium table rerun in a few very large tables (>= 2N entries:
//           they cannot overflow);
// only searches that exceed max_iters fall back to the host.  Small batches (interactive flushes)
// skip the lane tier: one 64-lane wave per search fills the chip.
// Heuristic: max(great-circle distance x circuity / v_max, ALT landmark bound); edge costs are floored
// at length / v_max on the host, so both are admissible and consistent (ALT tables are shrunk by 1e-4
// against fp32 rounding).  Every search stops within max_iters pops (status 3), on overflow (2) or
// when the open set empties (1): the grid always drains.
#include <algorithm>
#include <chrono>
#include <cstdlib>

#include "common.h"
#include "ops.h"

namespace rt {

struct __align__(16) AEnt {
  unsigned key;              // node id, EMPTY = free
  float h;                   // cached heuristic, NaN = not computed
  unsigned long long w;      // g (f32 bits) << 32 | closed (bit 31) | parent slot (31 b)
};
constexpr unsigned EMPTY = 0xffffffffu;
constexpr unsigned long long W_INIT = ~0ull;    // the all-ones reset pattern: g unset (reads as +inf)
constexpr unsigned NOPAR = 0x7fffffffu;
constexpr unsigned CLOSEDB = 0x80000000u;

struct AstarArgs {
  const int* indptr;
  const int* indices;
  const float* cost;     // [E] seconds
  const float* lat;      // [N] degrees
  const float* lon;
  const int* src;        // [Q]
  const int* dst;
  AEnt* tab;             // [S][1 << tbits] per-search hash tables (all-ones when idle)
  unsigned long long* heap;  // [S][cap] lane heap / wave near+far lists
  int* touched;          // [S][(1 << tbits) / 2] table slots a search wrote (reset list)
  float* out_cost;       // [Q]
  int* out_len;          // [Q]
  int* out_status;       // [Q]
  int* out_path;         // [Q][max_path]
  int N, Q, q0, S, cap, tbits, max_path, max_iters;
  float inv_vmax;        // seconds per metre at v_max
  const float* lm;       // [N][2K] ALT landmark tables: d(L_k -> v), d(v -> L_k) (nullptr: off)
  int K;
  int* out_iters;        // [Q] pops (lane) / expansions (wave) per query (nullptr: not recorded)
};

// Growth arena of the wave tier (all-ones when idle; the bump counter is reset before each launch)
struct AstarArena {
  AEnt* base;
  unsigned long long n;      // entries
  unsigned long long* ctr;   // bump pointer (entries)
};

constexpr int KMAX = 32;
// diagnostics: the wave tier records f-band passes instead of expansions in out_iters
__constant__ int c_count_passes = 0;
__device__ __forceinline__ bool count_passes_flag() { return c_count_passes != 0; }
// edges relaxed per batch of independent loads (road-graph degrees are 2-6, mostly 4-5)
constexpr int RB = 4;

__device__ __forceinline__ float hdist(const AstarArgs& a, int v, float tlat, float tlon, float ctl) {
  const float k = 0.017453292519943295f;
  const float la = a.lat[v] * k;
  const float dphi = tlat - la, dl = (tlon - a.lon[v] * k);
  const float s1 = __sinf(0.5f * dphi), s2 = __sinf(0.5f * dl);
  const float hv = s1 * s1 + __cosf(la) * ctl * s2 * s2;
  // slightly shrunk so float rounding never makes h inadmissible
  return 0.999f * 2.f * 6371000.f * asinf(sqrtf(fminf(1.f, fmaxf(0.f, hv)))) * a.inv_vmax;
}

// ALT lower bound on d(v -> t): max_k max(d(L_k,t) - d(L_k,v), d(v,L_k) - d(t,L_k)).
template <int K>
__device__ __forceinline__ float halt(const AstarArgs& a, int v, const float (&ft)[KMAX],
                                      const float (&bt)[KMAX]) {
  const float4* row = reinterpret_cast<const float4*>(a.lm + (size_t)v * 2 * K);
  float best = 0.f;
#pragma unroll
  for (int q = 0; q < K / 2; ++q) {     // one float4 = (fwd_k, fwd_k+1, bwd_k, bwd_k+1)
    const float4 x = row[q];
    best = fmaxf(best, ft[2 * q] - x.x);
    best = fmaxf(best, ft[2 * q + 1] - x.y);
    best = fmaxf(best, x.z - bt[2 * q]);
    best = fmaxf(best, x.w - bt[2 * q + 1]);
  }
  return best * 0.9999f;
}

template <int K>
__device__ __forceinline__ void load_target_lm(const AstarArgs& a, int t, float (&ft)[KMAX], float (&bt)[KMAX]) {
  if constexpr (K > 0) {
    const float4* row = reinterpret_cast<const float4*>(a.lm + (size_t)t * 2 * K);
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
      const float4 x = row[i];
      ft[2 * i] = x.x;
      ft[2 * i + 1] = x.y;
      bt[2 * i] = x.z;
      bt[2 * i + 1] = x.w;
    }
  }
}

// Block hashing: the 8 ids of a group (u >> 3) share one 128-byte block of 8 entries, at offset u & 7,
// and the block is chosen by Fibonacci (multiplicative) hashing of the group; a collision moves to the
// next block at the same offset (probe stride 8).  So ids that are neighbours in the graph (row-major
// grids, Morton-ordered OSM) share cache lines like the dense state did, while blocks are scattered
// uniformly: each of the 8 offset columns is an ordinary linear-probing table over random blocks
// (expected probes <= 2.5 at the half-full limit).  Hashing that keeps whole id RUNS contiguous
// (identity on the low bits) clustered under wrap-around collisions and ran the wave tier 30x slower.
__device__ __forceinline__ unsigned hslot(unsigned u, int tbits) {
  return (((u >> 3) * 0x9E3779B1u) >> (35 - tbits) << 3) | (u & 7u);
}
constexpr unsigned PSTEP = 8;                       // probe stride (one block)
__device__ __forceinline__ AEnt ld_ent(const AEnt* p) {
  const uint4 x = *reinterpret_cast<const uint4*>(p);
  AEnt e;
  e.key = x.x;
  e.h = __uint_as_float(x.y);
  e.w = ((unsigned long long)x.w << 32) | x.z;
  return e;
}
__device__ __forceinline__ void st_ent(AEnt* p, unsigned key, float h, unsigned long long w) {
  *reinterpret_cast<uint4*>(p) = make_uint4(key, __float_as_uint(h), (unsigned)w, (unsigned)(w >> 32));
}
__device__ __forceinline__ void clr_ent(AEnt* p) {
  *reinterpret_cast<uint4*>(p) = make_uint4(~0u, ~0u, ~0u, ~0u);
}
__device__ __forceinline__ float w_g(unsigned long long w) {
  return w == W_INIT ? __int_as_float(0x7f800000) : __uint_as_float((unsigned)(w >> 32));
}
__device__ __forceinline__ unsigned w_par(unsigned long long w) { return (unsigned)w & NOPAR; }
__device__ __forceinline__ unsigned long long w_make(float g, unsigned par) {
  return ((unsigned long long)__float_as_uint(g) << 32) | par;
}
__device__ __forceinline__ unsigned long long hkey(float f, int v) {
  return ((unsigned long long)__float_as_uint(f) << 32) | (unsigned)v;   // f >= 0: monotone bits
}

// D-ary min-heap of 64-bit (f, node) keys in this lane's HBM row.  Every pop/push is a chain of
// DEPENDENT random loads (a lane walks its own heap), so the heap depth, not bandwidth, sets the
// per-pop time.  With the storage shifted by D-1 the D children of a node are one aligned block
// (D/2 independent 16-byte loads, one memory latency per level).  80k-leg launch
// (bench/astar_tail.py): binary 378 ms, 4-ary 311-323 ms, 8-ary (default) 303 ms;
// ROUTEST_ASTAR_ARITY=2|4|8 selects.
template <int D>
struct LaneHeap {
  static constexpr int OFF = D == 8 ? 7 : (D == 4 ? 3 : 0);
  unsigned long long* hp;
  __device__ explicit LaneHeap(unsigned long long* row) : hp(row + OFF) {}
  __device__ __forceinline__ void push(int& hn, unsigned long long key) {
    int i = hn++;
    while (i > 0) {
      const int p = (i - 1) / D;
      const unsigned long long pk = hp[p];
      if (pk <= key) break;
      hp[i] = pk;
      i = p;
    }
    hp[i] = key;
  }
  __device__ __forceinline__ unsigned long long top() const { return hp[0]; }
  // remove the root (already read with top()): move the last entry down
  __device__ __forceinline__ void pop(int& hn) {
    const unsigned long long last = hp[--hn];
    if (hn == 0) return;
    int i = 0;
    while (true) {
      const int c = D * i + 1;
      if (c >= hn) break;
      unsigned long long best;
      int bi;
      if constexpr (D == 4) {
        const ulonglong2* blk = reinterpret_cast<const ulonglong2*>(hp + c);   // 32-byte aligned
        const ulonglong2 x0 = blk[0], x1 = blk[1];
        const unsigned long long v0 = x0.x;
        const unsigned long long v1 = c + 1 < hn ? x0.y : ~0ull;
        const unsigned long long v2 = c + 2 < hn ? x1.x : ~0ull;
        const unsigned long long v3 = c + 3 < hn ? x1.y : ~0ull;
        const bool b1 = v1 < v0, b3 = v3 < v2;
        const unsigned long long m01 = b1 ? v1 : v0, m23 = b3 ? v3 : v2;
        const int i01 = b1 ? c + 1 : c, i23 = b3 ? c + 3 : c + 2;
        best = m23 < m01 ? m23 : m01;
        bi = m23 < m01 ? i23 : i01;
      } else if constexpr (D == 8) {
        const ulonglong2* blk = reinterpret_cast<const ulonglong2*>(hp + c);   // 64-byte aligned
        ulonglong2 x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = blk[q];
        best = x[0].x;
        bi = c;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
          const unsigned long long v = (j & 1) ? x[j >> 1].y : x[j >> 1].x;
          if (c + j < hn && v < best) { best = v; bi = c + j; }
        }
      } else {
        best = hp[c];
        bi = c;
        if (c + 1 < hn) {
          const unsigned long long c2 = hp[c + 1];
          if (c2 < best) { best = c2; ++bi; }
        }
      }
      if (best >= last) break;
      hp[i] = best;
      i = bi;
    }
    hp[i] = last;
  }
};

// Walk parent slots from t's slot pt to s; writes the path source-first.  Returns the length, or -1
// when it does not fit max_path.
__device__ __forceinline__ int write_path(const AstarArgs& a, const AEnt* tab, unsigned pt, int s, int q) {
  int* path = a.out_path + (size_t)q * a.max_path;
  int len = 0;
  unsigned p = pt;
  while (true) {
    if (len >= a.max_path) return -1;
    const AEnt e = ld_ent(tab + p);
    path[len++] = (int)e.key;
    if ((int)e.key == s) break;
    p = w_par(e.w);
  }
  for (int i = 0, j = len - 1; i < j; ++i, --j) {
    const int tmp = path[i];
    path[i] = path[j];
    path[j] = tmp;
  }
  return len;
}

// ---------------------------------------------------------------------------------------------
// Lane tier: one lane per query, a private table (no atomics), lazy-deletion heap of (f, node).
template <int K, int D>
__global__ __launch_bounds__(64) void astar_kernel(AstarArgs a, const int* __restrict__ qidx, int n) {
  // XCD-aware: workgroup b runs on XCD b % 8; give each XCD a contiguous range of queries
  const int lb = (int)(blockIdx.x % 8u) * (int)(gridDim.x / 8u) + (int)(blockIdx.x / 8u);
  const int slot = lb * blockDim.x + threadIdx.x;
  if (slot >= a.S || slot >= n) return;
  const int q = qidx != nullptr ? qidx[slot] : a.q0 + slot;
  const int tb = a.tbits;
  const unsigned mask = (1u << tb) - 1u;
  const int tcap = 1 << (tb - 1);
  AEnt* tab = a.tab + ((size_t)slot << tb);
  unsigned long long* heap = a.heap + (size_t)slot * a.cap;
  int* touched = a.touched + (size_t)slot * tcap;
  const int s = a.src[q], t = a.dst[q];
  const float k = 0.017453292519943295f;
  const float tlat = a.lat[t] * k, tlon = a.lon[t] * k, ctl = __cosf(tlat);
  float ft[KMAX], bt[KMAX];  // landmark distances of the target (registers: K is a constant)
  load_target_lm<K>(a, t, ft, bt);
  auto heur = [&](int v) {
    float hv = hdist(a, v, tlat, tlon, ctl);
    if constexpr (K > 0) hv = fmaxf(hv, halt<K>(a, v, ft, bt));
    return hv;
  };

  int hn = 0, nt = 0, status = 1;
  const int capq = a.cap - 16;         // room for the shifted storage and a full child block
  LaneHeap<D> hq(heap);
  {
    const unsigned ps = hslot((unsigned)s, tb);     // the table is empty
    const float hs = heur(s);
    st_ent(tab + ps, (unsigned)s, hs, w_make(0.f, NOPAR));
    touched[nt++] = (int)ps;
    hq.push(hn, hkey(hs, s));
  }
  unsigned pt = 0;
  int it = 0;
  for (; hn > 0; ++it) {
    if (it >= a.max_iters) { status = 3; break; }
    // pop min: the popped node's own loads (table entry, CSR row bounds) are issued BEFORE the
    // sift-down, so their latency overlaps the heap's dependent chain
    const unsigned long long top = hq.top();
    const int v = (int)(unsigned)(top & 0xffffffffu);
    unsigned pv = hslot((unsigned)v, tb);
    AEnt ev = ld_ent(tab + pv);
    const int e0 = a.indptr[v], e1 = a.indptr[v + 1];
    hq.pop(hn);
    for (unsigned n = 0; ev.key != (unsigned)v && n < (mask >> 3); ++n) {   // a pushed node is in the table
      pv = (pv + PSTEP) & mask;
      ev = ld_ent(tab + pv);
    }
    if (ev.key != (unsigned)v) { status = 2; break; }
    if ((unsigned)ev.w & CLOSEDB) continue;         // stale duplicate
    tab[pv].w = ev.w | CLOSEDB;
    if (v == t) { status = 0; pt = pv; break; }
    const float gv = w_g(ev.w);
    bool overflow = false;
    // relax in chunks of RB edges: all (target, cost) loads, then all first-probe entry loads, are
    // issued together — two round trips per chunk instead of two per edge
    for (int eb = e0; eb < e1 && !overflow; eb += RB) {
      int uu[RB];
      float cc[RB];
      unsigned pp[RB];
      AEnt ee[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const bool in = eb + j < e1;
        uu[j] = in ? a.indices[eb + j] : v;
        cc[j] = in ? a.cost[eb + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        pp[j] = hslot((unsigned)uu[j], tb);
        if (eb + j < e1) ee[j] = ld_ent(tab + pp[j]);
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        if (eb + j >= e1) continue;
        const unsigned u = (unsigned)uu[j];
        unsigned p = pp[j];
        AEnt e = ee[j];
        // an earlier edge of this chunk may have written this entry (same target, or an insert
        // into the slot this probe started at): re-read it
        bool stale = false;
#pragma unroll
        for (int i = 0; i < j; ++i) {
          if (eb + i >= e1) continue;
          if ((unsigned)uu[i] == u) { p = pp[i]; stale = true; }
          else if (pp[i] == p) stale = true;
        }
        if (stale) e = ld_ent(tab + p);
        // (an empty entry is always reachable: inserts stop at half the table)
        for (unsigned n = 0; e.key != u && e.key != EMPTY && n < (mask >> 3); ++n) {
          p = (p + PSTEP) & mask;
          e = ld_ent(tab + p);
        }
        if (e.key != u && e.key != EMPTY) { overflow = true; break; }
        pp[j] = p;
        const float ng = gv + cc[j];
        if (e.key == EMPTY) {                       // first touch
          if (nt >= tcap || hn >= capq) { overflow = true; break; }
          const float hu = heur((int)u);
          st_ent(tab + p, u, hu, w_make(ng, pv));
          touched[nt++] = (int)p;
          hq.push(hn, hkey(ng + hu, (int)u));
        } else {
          if (((unsigned)e.w & CLOSEDB) || !(ng < w_g(e.w))) continue;
          if (hn >= capq) { overflow = true; break; }
          tab[p].w = w_make(ng, pv);
          hq.push(hn, hkey(ng + e.h, (int)u));
        }
      }
    }
    if (overflow) { status = 2; break; }
  }
  int len = 0;
  float total = 0.f;
  if (status == 0) {
    total = w_g(tab[pt].w);
    len = write_path(a, tab, pt, s, q);
    if (len < 0) { status = 4; len = 0; }
  }
  if (a.out_iters) a.out_iters[q] = it;
  a.out_cost[q] = status == 0 ? total : -1.f;
  a.out_len[q] = len;
  a.out_status[q] = status;
  // reset the entries this search wrote (the table is all-ones again for the next query)
  for (int i = 0; i < nt; ++i) clr_ent(tab + touched[i]);
}

// ---------------------------------------------------------------------------------------------
// Wave tier: one WORKGROUP of NW waves (NW = 1, 2, 4 or 8; AstarPlan::wave_nw / retry_nw) per query.
// Its 64 * NW lanes expand a whole f-band at once:
//
//   near = open nodes with f = g + h < thr;  far = the other open nodes as (f, node) pairs
//   repeat: every lane takes a near node, relaxes its edges with a 64-bit atomicMin on the packed
//           (g << 32 | parent) word; an improved target goes to next-near if f < thr, else to far
//   when near empties: best = g(t); if min f over far >= best the search is optimal (admissible
//           h: every open node on a better path would have f < best); else thr = min f + delta and
//           the far entries below it become the next near set (entries with f >= best are dropped)
//
// Label-correcting (a node is re-expanded when its g improves; stale duplicates are harmless), so
// costs are exact.  The table is shared by the wave's lanes: a key is claimed with atomicCAS (the
// claimer records the slot for the reset), the state word is lowered with atomicMin, and plain
// loads only ever see older (larger) words, which at worst cost a redundant atomic.  The heap row
// holds near A | near B | far.
// (waves_per_eu 4: the compiler fits the kernel in 102 VGPRs instead of 136 with no scratch, so four
// searches per SIMD are resident instead of three; the tier is bound by dependent-load latency)
template <int K, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4, 8))) void astar_wave_kernel(AstarArgs a, const int* __restrict__ qidx, int T,
                                                        float delta, AstarArena ar) {
  const int w = blockIdx.x;
  if (w >= T || w >= a.S) return;
  const int q = qidx != nullptr ? qidx[w] : a.q0 + w;
  const int lane = threadIdx.x;                     // thread of the search's workgroup (NW waves)
  constexpr int NT = 64 * NW;
  // the search's table: the slot's own region first; GROWN (2x per step) into the arena when it
  // fills up — memory follows the search instead of a fixed worst case per slot
  int tb = a.tbits;
  unsigned mask = (1u << tb) - 1u;
  int tcap = 1 << (tb - 1);
  AEnt* tab = a.tab + ((size_t)w << tb);
  int* touched = a.touched + (size_t)w * tcap;
  bool in_arena = false;
  // the f-band lists (near A | near B | far) start in the slot's heap row and, like the table, move
  // into larger arena buffers when a band would not fit
  int* nearA = reinterpret_cast<int*>(a.heap + (size_t)w * a.cap);
  int ncapA = a.cap / 2, ncapB = a.cap / 2;         // ints per near list
  bool narA = false, narB = false;
  int* nearB = nearA + a.cap / 2;
  unsigned long long* far = a.heap + (size_t)w * a.cap + a.cap / 2;
  int FCAP = a.cap / 2;                             // (f, node) entries
  bool farena = false;
  __shared__ int s_next, s_far, s_touch, s_bad;
  __shared__ float s_red[NW];
  __shared__ int s_wcnt[NW];
  __shared__ unsigned long long s_off;
  const int s = a.src[q], t = a.dst[q];
  const float k = 0.017453292519943295f;
  const float tlat = a.lat[t] * k, tlon = a.lon[t] * k, ctl = __cosf(tlat);
  float ft[KMAX], bt[KMAX];
  load_target_lm<K>(a, t, ft, bt);
  auto heur = [&](int v) {
    float hv = hdist(a, v, tlat, tlon, ctl);
    if constexpr (K > 0) hv = fmaxf(hv, halt<K>(a, v, ft, bt));
    return hv;
  };
  auto bad = [&]() { return *reinterpret_cast<volatile int*>(&s_bad) != 0; };
  // slot of u, or -1 if absent (bounded: an empty entry is always reachable below the grow
  // threshold; past an overflow at most TS / 8 probes per offset column)
  auto find = [&](unsigned u) -> int {
    unsigned p = hslot(u, tb);
    for (unsigned n = 0; n <= (mask >> 3); ++n) {
      const unsigned key = __hip_atomic_load(&tab[p].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (key == u) return (int)p;
      if (key == EMPTY) return -1;
      p = (p + PSTEP) & mask;
    }
    return -1;
  };
  // find-or-insert u starting at slot p; -1 when its offset column is full
  auto acquire = [&](unsigned u, unsigned p, bool& claimed) -> int {
    claimed = false;
    for (unsigned n = 0; n <= (mask >> 3); ++n) {
      const unsigned key = __hip_atomic_load(&tab[p].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (key == u) return (int)p;
      if (key == EMPTY) {
        const unsigned old = atomicCAS(&tab[p].key, EMPTY, u);
        if (old == EMPTY) { claimed = true; return (int)p; }
        if (old == u) return (int)p;
      }
      p = (p + PSTEP) & mask;
    }
    return -1;
  };
  int pt = -1;                                      // t's slot once inserted (until the table grows)
  auto gbest = [&]() -> float {
    if (pt < 0) pt = find((unsigned)t);
    return pt < 0 ? __int_as_float(0x7f800000) : w_g(tab[pt].w);
  };
  // Arena allocation of `units` 16-byte entries (all lanes, uniform control flow); nullptr when
  // the arena is exhausted.  Everything allocated is restored to all-ones before the search ends.
  auto alloc = [&](unsigned long long units) -> AEnt* {
    __syncthreads();
    if (lane == 0) {
      const unsigned long long off = atomicAdd(ar.ctr, units);
      s_off = off + units <= ar.n ? off : ~0ull;
    }
    __syncthreads();
    return s_off == ~0ull ? nullptr : ar.base + s_off;
  };
  auto fill_ones = [&](void* p, long long bytes) {     // bytes % 16 == 0
    uint4* q = reinterpret_cast<uint4*>(p);
    for (long long i = lane; i < bytes / 16; i += NT) q[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
  };
  // a near list able to take `need` ints (its content is dead at the call)
  auto ensure_near = [&](int*& lst, int& cap, bool& inar, int need) -> bool {
    if (need <= cap) return true;
    int nc = cap * 2;
    while (nc < need) nc *= 2;
    nc = (nc + 3) & ~3;
    AEnt* p = alloc((unsigned long long)nc / 4);
    if (p == nullptr) return false;
    if (inar) fill_ones(lst, (long long)cap * 4);
    lst = reinterpret_cast<int*>(p);
    cap = nc;
    inar = true;
    __syncthreads();
    return true;
  };
  auto ensure_far = [&](int need) -> bool {
    if (need <= FCAP) return true;
    int nc = FCAP * 2;
    while (nc < need) nc *= 2;
    nc = (nc + 1) & ~1;
    AEnt* p = alloc((unsigned long long)nc / 2);
    if (p == nullptr) return false;
    unsigned long long* nf = reinterpret_cast<unsigned long long*>(p);
    const int nfar = s_far < FCAP ? s_far : FCAP;
    for (int i = lane; i < nfar; i += NT) nf[i] = far[i];
    __syncthreads();
    if (farena) fill_ones(far, (long long)FCAP * 8);
    far = nf;
    FCAP = nc;
    farena = true;
    __syncthreads();
    return true;
  };
  // Grow 2x into the arena (all lanes, at a point where no lane is inside a pass).  Entries are
  // re-inserted, the old slot -> new slot map is kept in the dead table's key fields to rewrite the
  // parent pointers, and the old table (and old reset list, if it was an arena one) is restored to
  // all-ones.  Returns false when the arena is exhausted (the search then overflows to the big tier).
  auto grow = [&]() -> bool {
    const int nb = tb + 1;
    const unsigned long long tsz = 1ull << nb, lsz = (tsz / 2 * 4 + 15) / 16;   // table + reset list
    AEnt* ntab = alloc(tsz + lsz);
    if (ntab == nullptr) return false;
    int* ntouch = reinterpret_cast<int*>(ntab + tsz);
    const unsigned nmask = (unsigned)tsz - 1u;
    const int nt = s_touch < tcap ? s_touch : tcap;
    for (int i = lane; i < nt; i += NT) {
      const int o = touched[i];
      const AEnt e = ld_ent(tab + o);
      unsigned p = hslot(e.key, nb);
      for (unsigned n = 0; n <= (nmask >> 3); ++n) {
        if (atomicCAS(&ntab[p].key, EMPTY, e.key) == EMPTY) break;
        p = (p + PSTEP) & nmask;
      }
      ntab[p].h = e.h;
      ntab[p].w = e.w;
      ntouch[i] = (int)p;
      tab[o].key = p;                               // old -> new slot (the old table is dead)
    }
    __syncthreads();
    for (int i = lane; i < nt; i += NT) {
      const int p = ntouch[i];
      const unsigned long long e = ntab[p].w;
      const unsigned par = w_par(e);
      if (par != NOPAR) ntab[p].w = (e & ~(unsigned long long)NOPAR) | tab[par].key;
    }
    __syncthreads();
    for (int i = lane; i < nt; i += NT) {
      clr_ent(tab + touched[i]);
      if (in_arena) touched[i] = -1;
    }
    __syncthreads();
    tab = ntab;
    touched = ntouch;
    tb = nb;
    mask = nmask;
    tcap = (int)(tsz / 2);
    in_arena = true;
    pt = -1;
    return true;
  };

  if (lane == 0) {
    const unsigned ps = hslot((unsigned)s, tb);
    st_ent(tab + ps, (unsigned)s, heur(s), w_make(0.f, NOPAR));
    touched[0] = (int)ps;
    nearA[0] = s;
    s_far = 0;
    s_touch = 1;
    s_bad = 0;
  }
  __syncthreads();
  // cur / nxt alias the two near lists (A, B) and swap every pass
  bool curA = true;
  int nnear = 1;
  float thr = heur(s) + delta;
  long long expanded = 0;
  int passes = 0;                                   // f-band passes (diagnostics: ROUTEST_ASTAR_COUNT_PASSES)
  int status = 1;
  while (true) {
    while (nnear > 0) {
      // keep the table at most half full after a pass (a pass inserts at most ~6 entries per
      // expanded node), growing 2x at a time while the arena lasts
      while (s_touch + 8 * nnear > tcap && ar.base != nullptr && tb + 1 <= 26) {
        if (!grow()) break;
      }
      if (ar.base != nullptr) {             // room for this pass's pushes (<= 8 per expansion)
        if (curA) ensure_near(nearB, ncapB, narB, 8 * nnear);
        else ensure_near(nearA, ncapA, narA, 8 * nnear);
        ensure_far(s_far + 8 * nnear);
      }
      int* cur = curA ? nearA : nearB;
      int* nxt = curA ? nearB : nearA;
      const int ncap_nxt = curA ? ncapB : ncapA;
      // every wave has read s_next (nnear) after the previous pass's / far split's barrier before
      // lane 0 clears it: without this barrier a fast wave 0 could zero it while a slower wave was
      // still about to read it, and the waves' band loops (and their barriers) would diverge
      if constexpr (NW > 1) __syncthreads();
      if (lane == 0) s_next = 0;
      __syncthreads();
      const float best = gbest();
      for (int i = lane; i < nnear; i += NT) {
        if (bad()) break;
        const int v = cur[i];
        // probe with whole-entry loads: the hit is the entry (no second dependent load)
        int pv = -1;
        AEnt ev;
        {
          unsigned p = hslot((unsigned)v, tb);
          for (unsigned n = 0; n <= (mask >> 3); ++n) {
            ev = ld_ent(tab + p);
            if (ev.key == (unsigned)v) { pv = (int)p; break; }
            if (ev.key == EMPTY) break;
            p = (p + PSTEP) & mask;
          }
        }
        if (pv < 0) continue;
        const float gv = w_g(ev.w);
        const float hv = ev.h == ev.h ? ev.h : heur(v);
        if (!(gv + hv < best)) continue;                 // cannot lead to a better path
        const int e0 = a.indptr[v], e1 = a.indptr[v + 1];
        for (int eb = e0; eb < e1; eb += RB) {
          // same batching as the lane tier: all (target, cost), then all first-probe entries
          int uu[RB];
          float cc[RB];
          unsigned pp[RB];
          unsigned long long seen[RB];
          bool hit[RB];
#pragma unroll
          for (int j = 0; j < RB; ++j) {
            const bool in = eb + j < e1;
            uu[j] = in ? a.indices[eb + j] : v;
            cc[j] = in ? a.cost[eb + j] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < RB; ++j) {
            pp[j] = hslot((unsigned)uu[j], tb);
            seen[j] = 0ull;
            hit[j] = false;
            if (eb + j < e1) {
              const AEnt x = ld_ent(tab + pp[j]);
              // known entry: its word and slot; empty or another key: unknown (probe + claim)
              hit[j] = x.key == (unsigned)uu[j];
              seen[j] = hit[j] ? x.w : W_INIT;
            }
          }
#pragma unroll
          for (int j = 0; j < RB; ++j) {
            if (eb + j >= e1) continue;
            const int u = uu[j];
            const float ng = gv + cc[j];
            const unsigned long long nw = w_make(ng, (unsigned)pv);
            // plain load first: most relaxations do not improve, and a 64-bit atomic costs far
            // more than a load
            if (nw >= seen[j]) continue;
            bool claimed = false;
            const int p = hit[j] ? (int)pp[j] : acquire((unsigned)u, pp[j], claimed);
            if (p < 0) { s_bad = 1; break; }
            if (claimed) {
              const int ti = atomicAdd(&s_touch, 1);
              if (ti < tcap) touched[ti] = p;
              else s_bad = 1;                        // (the reset then clears the whole table)
            }
            const unsigned long long old = atomicMin(&tab[p].w, nw);
            if (nw >= old) continue;
            float hu = tab[p].h;
            if (hu != hu) {
              hu = heur(u);
              tab[p].h = hu;
            }
            const float f = ng + hu;
            if (f < thr) {
              const int ni = atomicAdd(&s_next, 1);
              if (ni < ncap_nxt) nxt[ni] = u;
              else s_bad = 1;
            } else {
              const int fi = atomicAdd(&s_far, 1);
              if (fi < FCAP) far[fi] = hkey(f, u);
              else s_bad = 1;
            }
          }
        }
      }
      expanded += nnear;
      ++passes;
      __syncthreads();
      nnear = s_next < ncap_nxt ? s_next : ncap_nxt;
      curA = !curA;
      if (s_bad) { status = 2; break; }
      if (expanded > a.max_iters) { status = 3; break; }
    }
    if (status >= 2) break;
    // near band exhausted: optimal if no open node can beat best; else open the next band
    const float best = gbest();
    const int nfar = s_far < FCAP ? s_far : FCAP;
    float fmin = __int_as_float(0x7f800000);
    for (int i = lane; i < nfar; i += NT) {
      const float f = __uint_as_float((unsigned)(far[i] >> 32));
      if (f < best) fmin = fminf(fmin, f);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) fmin = fminf(fmin, __shfl_xor(fmin, o));
    if constexpr (NW > 1) {
      if ((lane & 63) == 0) s_red[lane >> 6] = fmin;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < NW; ++w) fmin = fminf(fmin, s_red[w]);
      __syncthreads();
    }
    if (!(fmin < best)) break;                        // done: best is optimal (or +inf: unreachable)
    thr = fmin + delta;
    // split far in place: f < thr -> near (cur), f < best -> keep (compacted), else drop.  A chunk of
    // 64 is read before any of its kept entries is written, and writes never pass reads.
    // the split refills cur (its content is dead): make room for every far entry
    if (ar.base != nullptr) {
      if (curA) ensure_near(nearA, ncapA, narA, nfar);
      else ensure_near(nearB, ncapB, narB, nfar);
    }
    int* cur = curA ? nearA : nearB;
    const int ncap_cur = curA ? ncapA : ncapB;
    if (lane == 0) {
      s_next = 0;
      s_far = 0;
    }
    __syncthreads();
    for (int i0 = 0; i0 < nfar; i0 += NT) {
      const int i = i0 + lane;
      const unsigned long long x = i < nfar ? far[i] : ~0ull;
      const float f = __uint_as_float((unsigned)(x >> 32));
      const bool to_near = i < nfar && f < thr;
      const bool keep = i < nfar && !to_near && f < best;
      const unsigned long long mk = __ballot(keep);
      int base = s_far;
      int total = __popcll(mk);
      if constexpr (NW > 1) {                       // kept entries in (wave, lane) order
        if ((lane & 63) == 0) s_wcnt[lane >> 6] = total;
        __syncthreads();
        total = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const int c = s_wcnt[w];
          if (w < (lane >> 6)) base += c;
          total += c;
        }
      }
      __syncthreads();
      if (keep) far[base + __popcll(mk & ((1ull << (lane & 63)) - 1))] = x;
      if (to_near) {
        const int ni = atomicAdd(&s_next, 1);
        if (ni < ncap_cur) cur[ni] = (int)(unsigned)(x & 0xffffffffu);
        else s_bad = 1;
      }
      if (lane == 0) s_far = base + total;
      __syncthreads();
    }
    nnear = s_next < ncap_cur ? s_next : ncap_cur;
    if (s_bad) { status = 2; break; }
  }
  __syncthreads();
  if (lane == 0) {
    const int ptt = find((unsigned)t);
    const float total = ptt < 0 ? __int_as_float(0x7f800000) : w_g(tab[ptt].w);
    int len = 0;
    if (status < 2) status = total < __int_as_float(0x7f800000) ? 0 : 1;
    if (status == 0) {
      len = write_path(a, tab, (unsigned)ptt, s, q);
      if (len < 0) { status = 4; len = 0; }
    }
    if (a.out_iters)
      a.out_iters[q] = count_passes_flag() ? passes : (int)(expanded < 0x7fffffff ? expanded : 0x7fffffff);
    a.out_cost[q] = status == 0 ? total : -1.f;
    a.out_len[q] = len;
    a.out_status[q] = status;
  }
  __syncthreads();
  const int nt = s_touch;
  if (nt <= tcap) {
    for (int i = lane; i < nt; i += NT) {
      clr_ent(tab + touched[i]);
      if (in_arena) touched[i] = -1;
    }
  } else {                                            // claims past the reset list: clear everything
    for (int i = lane; i <= (int)mask; i += NT) clr_ent(tab + i);
    if (in_arena)
      for (int i = lane; i < tcap; i += NT) touched[i] = -1;
  }
  if (narA) fill_ones(nearA, (long long)ncapA * 4);
  if (narB) fill_ones(nearB, (long long)ncapB * 4);
  if (farena) fill_ones(far, (long long)FCAP * 8);
}

// Ordered compaction: qidx = [i for i in range(Q) if (1 << status[i]) & want], count = len (one block;
// the order is the query order, so tier slots — and results under exact ties — are deterministic).
__global__ __launch_bounds__(1024) void astar_select_kernel(const int* __restrict__ status, int Q, int want,
                                                            int* __restrict__ qidx, int* __restrict__ count) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int i0 = 0; i0 < Q; i0 += 1024) {
    const int i = i0 + (int)threadIdx.x;
    const int sv = i < Q ? status[i] : -1;
    const bool f = sv >= 0 && sv < 31 && ((want >> sv) & 1);
    const unsigned long long m = __ballot(f);
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int k = 0; k < wv; ++k) off += wsum[k];
    if (f) qidx[off + __popcll(m & ((1ull << lane) - 1))] = i;
    __syncthreads();
    if (threadIdx.x == 0) {
      int sum = 0;
      for (int k = 0; k < 16; ++k) sum += wsum[k];
      base += sum;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

// The same compaction for the wave tier, ordered LONGEST FIRST: a stable counting sort on NBK buckets
// of log2(great-circle src-dst distance), descending.  One launch holds more searches than the chip
// has wave slots, and a search's f-band passes grow with the leg's length (bench/astar_passes.py:
// p50 235, max 1508 passes), so a long leg dispatched late ran alone at the end of the launch; issuing
// long legs first lets the short ones fill in behind them (longest-processing-time-first).  Stable
// within a bucket and independent of timing, so slots and tie results stay deterministic.
constexpr int NBK = 32;
__device__ __forceinline__ int lpt_bucket(const float* lat, const float* lon, int s, int t) {
  const float k = 0.017453292519943295f;
  const float la = lat[s] * k, lb = lat[t] * k;
  const float s1 = __sinf(0.5f * (lb - la)), s2 = __sinf(0.5f * (lon[t] - lon[s]) * k);
  const float hv = s1 * s1 + __cosf(la) * __cosf(lb) * s2 * s2;
  const float d = 2.f * 6371000.f * asinf(sqrtf(fminf(1.f, fmaxf(0.f, hv))));   // metres
  // two buckets per octave above 100 m, longest legs in bucket 0
  const int b = d > 100.f ? (int)(2.f * __log2f(d * 0.01f)) : 0;
  return NBK - 1 - (b < 0 ? 0 : (b > NBK - 1 ? NBK - 1 : b));
}

__global__ __launch_bounds__(1024) void astar_select_lpt_kernel(const int* __restrict__ status, int Q, int want,
                                                                const int* __restrict__ src,
                                                                const int* __restrict__ dst,
                                                                const float* __restrict__ lat,
                                                                const float* __restrict__ lon,
                                                                int* __restrict__ qidx, int* __restrict__ count) {
  __shared__ int hist[NBK];            // per-bucket counts, then running output offsets
  __shared__ int wcnt[16][NBK];        // this chunk's per-wave bucket counts
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < NBK) hist[threadIdx.x] = 0;
  __syncthreads();
  auto bucket_of = [&](int i) {
    const int sv = i < Q ? status[i] : -1;
    const bool f = sv >= 0 && sv < 31 && ((want >> sv) & 1);
    return f ? lpt_bucket(lat, lon, src[i], dst[i]) : -1;
  };
  for (int i0 = 0; i0 < Q; i0 += 1024) {
    const int b = bucket_of(i0 + (int)threadIdx.x);
    if (b >= 0) atomicAdd(&hist[b], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int k = 0; k < NBK; ++k) {
      const int c = hist[k];
      hist[k] = run;
      run += c;
    }
    *count = run;
  }
  __syncthreads();
  for (int i0 = 0; i0 < Q; i0 += 1024) {
    const int i = i0 + (int)threadIdx.x;
    const int b = bucket_of(i);
    for (int k = lane; k < NBK; k += 64) wcnt[wv][k] = 0;
    // lanes of this wave with the same bucket, one ballot per distinct bucket present
    unsigned long long same = 0;
    unsigned long long todo = __ballot(b >= 0);
    while (todo) {
      const int l0 = __ffsll((long long)todo) - 1;
      const int b0 = __shfl(b, l0);
      const unsigned long long m = __ballot(b == b0);
      if (b == b0) same = m;
      if (lane == l0) wcnt[wv][b0] = __popcll(m);
      todo &= ~m;
    }
    __syncthreads();
    if (b >= 0) {
      int off = hist[b] + __popcll(same & ((1ull << lane) - 1));
      for (int k = 0; k < wv; ++k) off += wcnt[k][b];
      qidx[off] = i;
    }
    __syncthreads();
    if (threadIdx.x < NBK) {
      int s = 0;
      for (int k = 0; k < 16; ++k) s += wcnt[k][threadIdx.x];
      hist[threadIdx.x] += s;
    }
    __syncthreads();
  }
}

// Lane/wave split by leg length: legs longer than `thr_m` (great circle) would spend the lane tier's
// whole pop budget and then start over in the wave tier, so they skip the lane tier (status 3 = "pop
// budget spent" routes them to the wave tier's selection); the short ones are compacted, in query
// order, into qidx for the lane tier.
__global__ __launch_bounds__(1024) void astar_split_kernel(const int* __restrict__ src, const int* __restrict__ dst,
                                                           const float* __restrict__ lat,
                                                           const float* __restrict__ lon, int Q, float thr_m,
                                                           int* __restrict__ status, int* __restrict__ qidx,
                                                           int* __restrict__ count) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const float k = 0.017453292519943295f;
  for (int i0 = 0; i0 < Q; i0 += 1024) {
    const int i = i0 + (int)threadIdx.x;
    bool f = false;
    if (i < Q) {
      const int s = src[i], t = dst[i];
      const float la = lat[s] * k, lb = lat[t] * k;
      const float s1 = __sinf(0.5f * (lb - la)), s2 = __sinf(0.5f * (lon[t] - lon[s]) * k);
      const float hv = s1 * s1 + __cosf(la) * __cosf(lb) * s2 * s2;
      const float d = 2.f * 6371000.f * asinf(sqrtf(fminf(1.f, fmaxf(0.f, hv))));
      f = d <= thr_m;
      if (!f) status[i] = 3;
    }
    const unsigned long long m = __ballot(f);
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int j = 0; j < wv; ++j) off += wsum[j];
    if (f) qidx[off + __popcll(m & ((1ull << lane) - 1))] = i;
    __syncthreads();
    if (threadIdx.x == 0) {
      int sum = 0;
      for (int j = 0; j < 16; ++j) sum += wsum[j];
      base += sum;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

static AstarArgs make_args(const AstarGraphDev& g, const int* src, const int* dst, int Q, int q0,
                           const AstarWs& ws, const AstarOut& o, int max_iters) {
  return AstarArgs{g.indptr, g.indices, g.cost, g.lat, g.lon, src, dst, (AEnt*)ws.tab,
                   (unsigned long long*)ws.heap, ws.touched, o.cost, o.len, o.status, o.path,
                   g.N, Q, q0, ws.slots, ws.cap, ws.tbits, o.max_path, max_iters, g.inv_vmax, g.lm, g.K,
                   o.iters};
}

bool astar_ws_ok(const AstarWs& ws, bool wave) {
  return ws.tab != nullptr && ws.heap != nullptr && ws.touched != nullptr && ws.slots > 0 && ws.tbits >= 6 &&
         ws.tbits <= 30 && ws.cap >= (wave ? 128 : 64) && ws.cap % 8 == 0;
}

hipError_t launch_astar_lane(const AstarGraphDev& g, const int* src, const int* dst, int Q, int q0,
                             const AstarWs& ws, const AstarOut& o, int max_iters, hipStream_t stream,
                             const int* qidx, int nq) {
  const int n = min(ws.slots, qidx != nullptr ? nq : Q - q0);
  if (n <= 0) return hipSuccess;
  if (g.lm != nullptr && g.K != 32 && g.K != 16 && g.K != 8) return hipErrorInvalidValue;
  if (!astar_ws_ok(ws, false)) return hipErrorInvalidValue;
  const AstarArgs a = make_args(g, src, dst, Q, q0, ws, o, max_iters);
  // one wavefront per workgroup (a wave runs as long as its longest search); grid rounded to a
  // multiple of 8 for the XCD-aware remap in the kernel (surplus lanes exit at the slot check)
  const dim3 grid(((n + 63) / 64 + 7) / 8 * 8), block(64);
  static const int arity = [] {
    const char* v = std::getenv("ROUTEST_ASTAR_ARITY");
    const int d = v != nullptr ? std::atoi(v) : 8;
    return (d == 2 || d == 4) ? d : 8;
  }();
#define RT_ASTAR_LANE(D)                                                                          \
  do {                                                                                            \
    if (g.lm == nullptr) hipLaunchKernelGGL((astar_kernel<0, D>), grid, block, 0, stream, a, qidx, n);     \
    else if (g.K == 8) hipLaunchKernelGGL((astar_kernel<8, D>), grid, block, 0, stream, a, qidx, n);       \
    else if (g.K == 16) hipLaunchKernelGGL((astar_kernel<16, D>), grid, block, 0, stream, a, qidx, n);     \
    else hipLaunchKernelGGL((astar_kernel<32, D>), grid, block, 0, stream, a, qidx, n);                    \
  } while (0)
  if (arity == 2) RT_ASTAR_LANE(2);
  else if (arity == 4) RT_ASTAR_LANE(4);
  else RT_ASTAR_LANE(8);
#undef RT_ASTAR_LANE
  return hipGetLastError();
}

hipError_t launch_astar_wave(const AstarGraphDev& g, const int* src, const int* dst, int Q, const int* qidx,
                             int q0, int T, const AstarWs& ws, const AstarOut& o, int max_iters, float delta,
                             hipStream_t stream, const AstarArenaBuf* arena, int nw) {
  const int n = T < ws.slots ? T : ws.slots;
  if (n <= 0) return hipSuccess;
  if (g.lm != nullptr && g.K != 32 && g.K != 16 && g.K != 8) return hipErrorInvalidValue;
  if (!astar_ws_ok(ws, true)) return hipErrorInvalidValue;
  if (qidx == nullptr && q0 + n > Q) return hipErrorInvalidValue;
  const AstarArgs a = make_args(g, src, dst, Q, q0, ws, o, max_iters);
  static const int count_passes = [] {
    const char* v = std::getenv("ROUTEST_ASTAR_COUNT_PASSES");
    return v != nullptr && std::atoi(v) != 0 ? 1 : 0;
  }();
  if (count_passes) {
    static bool set[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (!set[dev & 63]) {
      hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_count_passes), &count_passes, sizeof(int));
      if (e != hipSuccess) return e;
      set[dev & 63] = true;
    }
  }
  AstarArena ar{nullptr, 0, nullptr};
  if (arena != nullptr && arena->base != nullptr && arena->ctr != nullptr && arena->entries > 0) {
    // every search of the previous launch restored what it used: start the bump pointer over
    hipError_t e = hipMemsetAsync(arena->ctr, 0, sizeof(unsigned long long), stream);
    if (e != hipSuccess) return e;
    ar = AstarArena{(AEnt*)arena->base, arena->entries, arena->ctr};
  }
#define RT_ASTAR_WAVE(NWV)                                                                                   \
  do {                                                                                                       \
    const dim3 blk(64 * NWV);                                                                                \
    if (g.lm == nullptr) hipLaunchKernelGGL((astar_wave_kernel<0, NWV>), dim3(n), blk, 0, stream, a, qidx, n, delta, ar); \
    else if (g.K == 8) hipLaunchKernelGGL((astar_wave_kernel<8, NWV>), dim3(n), blk, 0, stream, a, qidx, n, delta, ar);  \
    else if (g.K == 16) hipLaunchKernelGGL((astar_wave_kernel<16, NWV>), dim3(n), blk, 0, stream, a, qidx, n, delta, ar); \
    else hipLaunchKernelGGL((astar_wave_kernel<32, NWV>), dim3(n), blk, 0, stream, a, qidx, n, delta, ar);             \
  } while (0)
  if (nw == 8) RT_ASTAR_WAVE(8);
  else if (nw == 4) RT_ASTAR_WAVE(4);
  else if (nw == 2) RT_ASTAR_WAVE(2);
  else if (nw == 1) RT_ASTAR_WAVE(1);
  else return hipErrorInvalidValue;
#undef RT_ASTAR_WAVE
  return hipGetLastError();
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// select (1 << status) & want into scratch[0..Q), count -> scratch[Q]; returns the count on the host
static hipError_t select_count(const int* status, int Q, int want, int* scratch, hipStream_t stream, int& count) {
  hipLaunchKernelGGL(astar_select_kernel, dim3(1), dim3(1024), 0, stream, status, Q, want, scratch, scratch + Q);
  hipError_t e = hipGetLastError();
  int h = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&h, scratch + Q, sizeof(int), hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  count = h;
  return e;
}

static hipError_t select_count_lpt(const AstarGraphDev& g, const int* src, const int* dst, const int* status, int Q,
                                   int want, int* scratch, hipStream_t stream, int& count) {
  hipLaunchKernelGGL(astar_select_lpt_kernel, dim3(1), dim3(1024), 0, stream, status, Q, want, src, dst, g.lat, g.lon,
                     scratch, scratch + Q);
  hipError_t e = hipGetLastError();
  int h = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&h, scratch + Q, sizeof(int), hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  count = h;
  return e;
}

hipError_t astar_search(const AstarGraphDev& g, const int* src, const int* dst, int Q, const AstarWs* lane,
                        const AstarWs* wave, const AstarWs* big, const AstarOut& o, const AstarPlan& pl,
                        int* scratch, hipStream_t stream, AstarRunStats* st, const AstarArenaBuf* arena) {
  AstarRunStats z{};
  AstarRunStats& S = st != nullptr ? *st : z;
  S = AstarRunStats{};
  if (Q <= 0) return hipSuccess;
  auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipSuccess;
  // waves per search: the plan's value, else the environment (read per call, so tests can switch
  // them); only 1, 2, 4 and 8 have kernel instantiations — anything else is an error, not a rounding
  auto waves = [](int v, const char* env, int dflt) {
    if (v != 0) return v;
    const char* s = std::getenv(env);
    return s != nullptr ? std::atoi(s) : dflt;
  };
  const int wave_nw = waves(pl.wave_nw, "ROUTEST_ASTAR_WAVE_WAVES", 1);
  const int big_nw = waves(pl.retry_nw, "ROUTEST_ASTAR_RETRY_WAVES", 4);
  auto nw_ok = [](int v) { return v == 1 || v == 2 || v == 4 || v == 8; };
  if (!nw_ok(wave_nw) || !nw_ok(big_nw)) return hipErrorInvalidValue;
  const bool use_wave = wave != nullptr && pl.lane_pops > 0;
  const bool use_lane = lane != nullptr && (!use_wave || Q >= pl.wave_only_below);
  if (!use_lane && !use_wave) return hipErrorInvalidValue;
  const int* qidx = nullptr;
  int T = 0;
  if (use_lane) {
    const int iters = use_wave ? std::min(pl.max_iters, pl.lane_pops) : pl.max_iters;
    // legs longer than ROUTEST_ASTAR_LANE_MAX_M metres (great circle; 0 = no split) skip the lane tier
    float lane_max_m = pl.lane_max_m;
    if (lane_max_m < 0.f) {
      const char* v = std::getenv("ROUTEST_ASTAR_LANE_MAX_M");
      lane_max_m = v != nullptr ? (float)std::atof(v) : 0.f;
    }
    if (use_wave && lane_max_m > 0.f) {
      int L = 0;
      hipLaunchKernelGGL(astar_split_kernel, dim3(1), dim3(1024), 0, stream, src, dst, g.lat, g.lon, Q, lane_max_m,
                         o.status, scratch, scratch + Q);
      e = hipGetLastError();
      if (e == hipSuccess) e = hipMemcpyAsync(&L, scratch + Q, sizeof(int), hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      for (int q0 = 0; q0 < L && e == hipSuccess; q0 += lane->slots)
        e = launch_astar_lane(g, src, dst, Q, 0, *lane, o, iters, stream, scratch + q0, std::min(lane->slots, L - q0));
      S.lane = L;
    } else {
      for (int q0 = 0; q0 < Q && e == hipSuccess; q0 += lane->slots)
        e = launch_astar_lane(g, src, dst, Q, q0, *lane, o, iters, stream);
      S.lane = Q;
    }
    if (e == hipSuccess && use_wave) {
      // pop budget spent (3) or the small table/heap overflowed (2): continue in the wave tier,
      // longest legs first (ROUTEST_ASTAR_LPT=0: query order)
      // Only when the growth arena holds every resident wave-tier search at the largest table it can
      // reach (2N entries): long searches first means the longest ones grow at the same time, and on
      // a 1M-node graph that exhausted the arena and sent 18k searches to the chunked retry (1M-node
      // local step 739 -> 1630 ms; 100k-node route step 150 -> 124.6 ms with it,
      // profiles/superseded/astar_lpt_arena_ab_r3aa.jsonl).  ROUTEST_ASTAR_LPT=0 | 1 forces it off | on.
      static const int lpt_env = [] {
        const char* v = std::getenv("ROUTEST_ASTAR_LPT");
        return v == nullptr ? -1 : (std::atoi(v) != 0 ? 1 : 0);
      }();
      bool lpt = lpt_env == 1;
      if (lpt_env < 0 && arena != nullptr && arena->base != nullptr) {
        int dev = 0, cus = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        // resident searches: 4 SIMDs x 4 waves per CU, nw waves per search
        const unsigned long long resident = (unsigned long long)cus * 16ull / (unsigned long long)wave_nw;
        lpt = arena->entries >= resident * 2ull * (unsigned long long)g.N;
      }
      if (lpt) e = select_count_lpt(g, src, dst, o.status, Q, (1 << 2) | (1 << 3), scratch, stream, T);
      else e = select_count(o.status, Q, (1 << 2) | (1 << 3), scratch, stream, T);
      qidx = scratch;
    }
    S.lane_ms = ms_since(t0);
  } else {
    T = Q;                                          // every query, identity order
  }
  t0 = std::chrono::steady_clock::now();
  if (use_wave) {
    S.wave = T;
    for (int i0 = 0; i0 < T && e == hipSuccess; i0 += wave->slots)
      e = launch_astar_wave(g, src, dst, Q, qidx != nullptr ? qidx + i0 : nullptr, i0, std::min(wave->slots, T - i0),
                            *wave, o, pl.max_iters, pl.delta, stream, arena, wave_nw);
  }
  // Searches that overflowed because one launch's searches shared the growth arena: rerun them in
  // the wave tier a chunk at a time (the arena restarts per launch), so each can grow into
  // ROUTEST_ASTAR_RETRY_ENTRIES (default 2^20) entries — on a 1M-node graph thousands of local legs
  // overflowed a 32k-search launch's share, and the few big-tier slots then ran them ~100 at a time
  // for seconds (profiles/superseded/astar_scale_1m_r3n.jsonl).  Only what overflows again goes to the big tier.
  bool wave_timed = false;
  // the reruns and the big tier hold the LARGE searches (f-bands of thousands of nodes): a workgroup
  // of ROUTEST_ASTAR_RETRY_WAVES (default 4; 1, 2, 8) waves per search instead of one wave
  if (e == hipSuccess && use_wave && arena != nullptr && arena->base != nullptr && arena->entries > 0) {
    static const unsigned long long per = [] {
      const char* v = std::getenv("ROUTEST_ASTAR_RETRY_ENTRIES");
      const long long x = v ? std::atoll(v) : (1ll << 20);
      return (unsigned long long)(x < 4096 ? 4096 : x);
    }();
    int R = 0;
    e = select_count(o.status, Q, 1 << 2, scratch, stream, R);
    S.wave_ms = ms_since(t0);
    wave_timed = true;
    t0 = std::chrono::steady_clock::now();
    S.retried = R;
    if (R > 0) {
      const unsigned long long c = arena->entries / per;
      const int chunk = (int)std::max<unsigned long long>(64, std::min<unsigned long long>((unsigned long long)wave->slots, c));
      for (int i0 = 0; i0 < R && e == hipSuccess; i0 += chunk)
        e = launch_astar_wave(g, src, dst, Q, scratch + i0, 0, std::min(chunk, R - i0), *wave, o, pl.max_iters,
                              pl.delta, stream, arena, big_nw);
    }
    S.retry_ms = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
  }
  if (e == hipSuccess && big != nullptr) {
    int E = 0;
    e = select_count(o.status, Q, 1 << 2, scratch, stream, E);
    if (!wave_timed) S.wave_ms = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    S.escalated = E;
    for (int i0 = 0; i0 < E && e == hipSuccess; i0 += big->slots)
      e = launch_astar_wave(g, src, dst, Q, scratch + i0, 0, std::min(big->slots, E - i0), *big, o, pl.max_iters,
                            pl.delta, stream, arena, big_nw);
    if (E > 0 && e == hipSuccess) e = hipStreamSynchronize(stream);
    S.big_ms = ms_since(t0);
  }
  return e;
}

}  // namespace rt
