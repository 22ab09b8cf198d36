// K9: batched point-to-point A* on a road graph with learned edge costs (north-star config 5).
// Conceptually replaces the reference's per-trip ORS directions calls (RO/Flaskr/utils.py:55-62,
// 151-156), which it issues one at a time over HTTPS.
//
// One LANE per query ("slot"): tens of thousands of independent searches in flight, each with
//   * dense per-slot state[N]: one 8-byte word (g as f32 | parent, closed bit) per node, so a
//     relaxation is one random access — 80k slots x 100k nodes = 64 GB, which 288 GB of HBM3E makes
//     the simple and fast choice (no hashing);
//   * an 8-ary min-heap (LaneHeap) of (f, node) 64-bit entries with lazy deletion (stale pops are
//     skipped via the closed bit; the heuristic is consistent, so a node's first pop is final);
//   * a touched list, so only the entries a search wrote are reset afterwards (no N-sized memset
//     per query).
// Launch time is set by the LONGEST search (one lane walks its own heap), so the heuristic matters
// most in the tail: 32 landmarks (vs 16) cut p99 pops 28k -> 12k and the 80k-leg launch 671 ->
// 444 ms (bench/astar_tail.py).
// Heuristic: max(great-circle distance x circuity / v_max, ALT landmark bound); edge costs are
// floored at length / v_max on the host, so both are admissible and consistent (ALT tables are
// shrunk by 1e-4 against fp32 rounding).  Every lane stops within max_iters pops (status 3), on heap
// or touched-list overflow (status 2) or when the open set empties (status 1): the grid always
// drains.  Paths are written target->source then reversed in place.
#include <cstdlib>

#include "common.h"
#include "ops.h"

namespace rt {

struct AstarArgs {
  const int* indptr;
  const int* indices;
  const float* cost;     // [E] seconds
  const float* lat;      // [N] degrees
  const float* lon;
  const int* src;        // [Q]
  const int* dst;
  unsigned long long* st;  // [S][N] packed per-node state: g (f32 bits, low) | parent (31 b) + closed (bit 63)
  unsigned long long* heap;  // [S][cap]
  int* touched;          // [S][cap]
  float* out_cost;       // [Q]
  int* out_len;          // [Q]
  int* out_status;       // [Q]
  int* out_path;         // [Q][max_path]
  int N, Q, q0, S, cap, max_path, max_iters;
  float inv_vmax;        // seconds per metre at v_max
  const float* lm;       // [N][2K] ALT landmark tables: d(L_k -> v), d(v -> L_k) (nullptr: off)
  int K;
  int* out_iters;        // [Q] heap pops per query (nullptr: not recorded)
};

constexpr int KMAX = 32;
// edges relaxed per batch of independent loads (road-graph degrees are 2-6, mostly 4-5); 80k-leg
// launch: RB 4 236 ms, 6 243 ms, 8 259 ms; evaluating the batch's heuristics together was neutral
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

// One 8-byte word per (slot, node): a relaxation reads g and the closed bit with ONE random access
// (the searches are bound by random HBM lines: 80k searches x dense 100k-node state = 64 GB).
__device__ __forceinline__ float st_g(unsigned long long w) { return __uint_as_float((unsigned)w); }
__device__ __forceinline__ unsigned st_p(unsigned long long w) { return (unsigned)(w >> 32); }
__device__ __forceinline__ unsigned long long st_make(float g, unsigned p) {
  return ((unsigned long long)p << 32) | __float_as_uint(g);
}
constexpr unsigned long long ST_INIT = 0x7fffffff7f800000ull;   // g = +inf, parent = none, open

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

template <int K, int D>
__global__ __launch_bounds__(256) void astar_kernel(AstarArgs a) {
  // XCD-aware: workgroup b runs on XCD b % 8; give each XCD a contiguous range of queries, so with
  // source-sorted queries one XCD's L2 serves one region of the graph (edges, costs, ALT rows)
  const int lb = (int)(blockIdx.x % 8u) * (int)(gridDim.x / 8u) + (int)(blockIdx.x / 8u);
  const int slot = lb * blockDim.x + threadIdx.x;
  const int q = a.q0 + slot;
  if (q >= a.Q || slot >= a.S) return;
  unsigned long long* st = a.st + (size_t)slot * a.N;
  unsigned long long* heap = a.heap + (size_t)slot * a.cap;
  int* touched = a.touched + (size_t)slot * a.cap;
  const int s = a.src[q], t = a.dst[q];
  const float k = 0.017453292519943295f;
  const float tlat = a.lat[t] * k, tlon = a.lon[t] * k, ctl = __cosf(tlat);
  const unsigned CLOSED = 0x80000000u;

  float ft[KMAX], bt[KMAX];  // landmark distances of the target (registers: K is a constant)
  if constexpr (K > 0) {
    const float4* row = reinterpret_cast<const float4*>(a.lm + (size_t)t * 2 * K);
#pragma unroll
    for (int q = 0; q < K / 2; ++q) {
      const float4 x = row[q];
      ft[2 * q] = x.x;
      ft[2 * q + 1] = x.y;
      bt[2 * q] = x.z;
      bt[2 * q + 1] = x.w;
    }
  }
  auto heur = [&](int v) {
    float hv = hdist(a, v, tlat, tlon, ctl);
    if constexpr (K > 0) hv = fmaxf(hv, halt<K>(a, v, ft, bt));
    return hv;
  };

  int hn = 0, nt = 0, status = 1;
  const int capq = a.cap - 16;         // room for the shifted storage and a full child block
  LaneHeap<D> hq(heap);
  st[s] = st_make(0.f, 0x7fffffffu);
  touched[nt++] = s;
  hq.push(hn, hkey(heur(s), s));
  int it = 0;
  for (; hn > 0; ++it) {
    if (it >= a.max_iters) { status = 3; break; }
    // pop min: the popped node's own loads (state word, CSR row bounds) are issued BEFORE the
    // sift-down, so their latency overlaps the heap's dependent chain
    const unsigned long long top = hq.top();
    const int v = (int)(unsigned)(top & 0xffffffffu);
    const unsigned long long wv = st[v];
    const int e0 = a.indptr[v], e1 = a.indptr[v + 1];
    hq.pop(hn);
    if (st_p(wv) & CLOSED) continue;     // stale duplicate
    st[v] = wv | ((unsigned long long)CLOSED << 32);
    if (v == t) { status = 0; break; }
    const float gv = st_g(wv);
    bool overflow = false;
    // relax in chunks of RB edges: all (target, cost) loads, then all target state loads, are
    // issued together — two round trips per chunk instead of two per edge
    for (int eb = e0; eb < e1 && !overflow; eb += RB) {
      int uu[RB];
      float cc[RB];
      unsigned long long wu[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const bool in = eb + j < e1;
        uu[j] = in ? a.indices[eb + j] : v;
        cc[j] = in ? a.cost[eb + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) wu[j] = eb + j < e1 ? st[uu[j]] : (ST_INIT | ((unsigned long long)CLOSED << 32));
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        if (eb + j >= e1 || (st_p(wu[j]) & CLOSED)) continue;
        const int u = uu[j];
        const float ng = gv + cc[j];
        float gu = st_g(wu[j]);
        bool fresh = gu == __int_as_float(0x7f800000);
#pragma unroll
        for (int i = 0; i < j; ++i)             // a repeated target within the chunk: its state
          if (uu[i] == u && eb + i < e1) {      // word may have been updated by edge i
            const unsigned long long w2 = st[u];
            gu = st_g(w2);
            fresh = gu == __int_as_float(0x7f800000);
          }
        if (ng < gu) {
          if (fresh) {                          // first touch
            if (nt >= capq) { overflow = true; break; }
            touched[nt++] = u;
          }
          st[u] = st_make(ng, (unsigned)v);
          if (hn >= capq) { overflow = true; break; }
          hq.push(hn, hkey(ng + heur(u), u));
        }
      }
    }
    if (overflow) { status = 2; break; }
  }
  int len = 0;
  float total = 0.f;
  if (status == 0) {
    total = st_g(st[t]);
    int* path = a.out_path + (size_t)q * a.max_path;
    int v = t;
    while (true) {
      if (len >= a.max_path) { status = 4; break; }
      path[len++] = v;
      if (v == s) break;
      v = (int)(st_p(st[v]) & 0x7fffffffu);
    }
    if (status == 0) {
      for (int i = 0, j = len - 1; i < j; ++i, --j) {
        const int tmp = path[i];
        path[i] = path[j];
        path[j] = tmp;
      }
    } else {
      len = 0;
    }
  }
  if (a.out_iters) a.out_iters[q] = it;
  a.out_cost[q] = status == 0 ? total : -1.f;
  a.out_len[q] = len;
  a.out_status[q] = status;
  // reset this slot's touched entries for the next batch
  for (int i = 0; i < nt; ++i) st[touched[i]] = ST_INIT;
}

// ---------------------------------------------------------------------------------------------
// Tail stage: ONE WAVE per query, for the few searches that exhaust the lane kernel's pop budget.
// The lane kernel's launch time is set by its longest search (a sequential chain of dependent HBM
// loads, ~7.6 us per pop); here the 64 lanes of a wave expand a whole f-band at once:
//
//   near = open nodes with f = g + h < thr;  far = the other open nodes as (f, node) pairs
//   repeat: every lane takes a near node, relaxes its edges with a 64-bit atomicMin on the packed
//           (g << 32 | parent) word; an improved target goes to next-near if f < thr, else to far
//   when near empties: best = g(t); if min f over far >= best the search is optimal (admissible
//           h: every open node on a better path would have f < best); else thr = min f + delta and
//           the far entries below it become the next near set (entries with f >= best are dropped)
//
// Label-correcting (a node is re-expanded when its g improves; stale duplicates are harmless), so
// costs are exact.  Per-slot memory is the lane kernel's: the state row (read in the swapped
// layout g << 32 | parent, for which the reset value ST_INIT is still "+inf"), the heap row split
// into near A | near B | far, and the touched list.
template <int K>
__global__ __launch_bounds__(64) void astar_wave_kernel(AstarArgs a, const int* __restrict__ qidx, int T,
                                                        float delta, float* __restrict__ hcache) {
  const int w = blockIdx.x;
  if (w >= T || w >= a.S) return;
  const int q = qidx[w];
  const int lane = threadIdx.x;
  unsigned long long* st = a.st + (size_t)w * a.N;
  int* nearA = reinterpret_cast<int*>(a.heap + (size_t)w * a.cap);
  const int NCAP = a.cap / 2;                       // ints per near list
  int* nearB = nearA + NCAP;
  unsigned long long* far = a.heap + (size_t)w * a.cap + a.cap / 2;
  const int FCAP = a.cap / 2;                       // (f, node) entries
  int* touched = a.touched + (size_t)w * a.cap;
  // per-slot heuristic cache: h(v) costs a 256-byte landmark row, and this stage re-reads it for
  // every relaxation and expansion (it was bandwidth-bound on those rows); the first toucher of a
  // node stores h, everyone else reads 4 bytes (NaN = not yet stored -> compute it)
  float* hc = hcache + (size_t)w * a.N;
  __shared__ int s_next, s_far, s_touch, s_bad;
  const int s = a.src[q], t = a.dst[q];
  const float k = 0.017453292519943295f;
  const float tlat = a.lat[t] * k, tlon = a.lon[t] * k, ctl = __cosf(tlat);
  float ft[KMAX], bt[KMAX];
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
  auto heur = [&](int v) {
    float hv = hdist(a, v, tlat, tlon, ctl);
    if constexpr (K > 0) hv = fmaxf(hv, halt<K>(a, v, ft, bt));
    return hv;
  };
  // (the reset word ST_INIT reads as a NaN g in this layout: map it to +inf)
  auto gof = [](unsigned long long x) {
    return x == ST_INIT ? __int_as_float(0x7f800000) : __uint_as_float((unsigned)(x >> 32));
  };
  auto pack = [](float g, unsigned p) { return ((unsigned long long)__float_as_uint(g) << 32) | p; };

  if (lane == 0) {
    hc[s] = heur(s);
    st[s] = pack(0.f, 0x7fffffffu);
    touched[0] = s;
    nearA[0] = s;
    s_far = 0;
    s_touch = 1;
    s_bad = 0;
  }
  __syncthreads();
  int* cur = nearA;
  int* nxt = nearB;
  int nnear = 1;
  float thr = heur(s) + delta;
  long long expanded = 0;
  int status = 1;
  while (true) {
    while (nnear > 0) {
      if (lane == 0) s_next = 0;
      __syncthreads();
      const float best = gof(st[t]);
      for (int i = lane; i < nnear; i += 64) {
        const int v = cur[i];
        const float gv = gof(st[v]);
        float hv = hc[v];
        if (hv != hv) hv = heur(v);
        if (!(gv + hv < best)) continue;                 // cannot lead to a better path
        const int e0 = a.indptr[v], e1 = a.indptr[v + 1];
        for (int eb = e0; eb < e1; eb += RB) {
          // same batching as the lane kernel: all (target, cost), then all target words, in flight
          int uu[RB];
          float cc[RB];
          unsigned long long seen[RB];
#pragma unroll
          for (int j = 0; j < RB; ++j) {
            const bool in = eb + j < e1;
            uu[j] = in ? a.indices[eb + j] : v;
            cc[j] = in ? a.cost[eb + j] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < RB; ++j) seen[j] = eb + j < e1 ? st[uu[j]] : 0ull;
#pragma unroll
          for (int j = 0; j < RB; ++j) {
            if (eb + j >= e1) continue;
            const int u = uu[j];
            const float ng = gv + cc[j];
            const unsigned long long nw = pack(ng, (unsigned)v);
            // plain load first: most relaxations do not improve, and a 64-bit atomic to HBM costs
            // far more than a load
            if (nw >= seen[j]) continue;
            const unsigned long long old = atomicMin(st + u, nw);
            if (nw >= old) continue;
            float hu;
            if (old == ST_INIT) {
              const int ti = atomicAdd(&s_touch, 1);
              if (ti < a.cap) touched[ti] = u;
              else s_bad = 1;
              hu = heur(u);
              hc[u] = hu;
            } else {
              hu = hc[u];
              if (hu != hu) hu = heur(u);
            }
            const float f = ng + hu;
            if (f < thr) {
              const int ni = atomicAdd(&s_next, 1);
              if (ni < NCAP) nxt[ni] = u;
              else s_bad = 1;
            } else {
              const int fi = atomicAdd(&s_far, 1);
              if (fi < FCAP) far[fi] = pack(f, (unsigned)u);
              else s_bad = 1;
            }
          }
        }
      }
      expanded += nnear;
      __syncthreads();
      nnear = s_next < NCAP ? s_next : NCAP;
      int* tmp = cur;
      cur = nxt;
      nxt = tmp;
      if (s_bad) { status = 2; break; }
      if (expanded > a.max_iters) { status = 3; break; }
    }
    if (status >= 2) break;
    // near band exhausted: optimal if no open node can beat best; else open the next band
    const float best = gof(st[t]);
    const int nfar = s_far < FCAP ? s_far : FCAP;
    float fmin = __int_as_float(0x7f800000);
    for (int i = lane; i < nfar; i += 64) {
      const float f = gof(far[i]);
      if (f < best) fmin = fminf(fmin, f);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) fmin = fminf(fmin, __shfl_xor(fmin, o));
    if (!(fmin < best)) break;                        // done: best is optimal (or +inf: unreachable)
    thr = fmin + delta;
    // split far in place: f < thr -> near (cur), f < best -> keep (compacted), else drop.  A chunk of
    // 64 is read before any of its kept entries is written, and writes never pass reads.
    if (lane == 0) {
      s_next = 0;
      s_far = 0;
    }
    __syncthreads();
    for (int i0 = 0; i0 < nfar; i0 += 64) {
      const int i = i0 + lane;
      const unsigned long long x = i < nfar ? far[i] : ~0ull;
      const float f = gof(x);
      const bool to_near = i < nfar && f < thr;
      const bool keep = i < nfar && !to_near && f < best;
      const unsigned long long mk = __ballot(keep);
      const int base = s_far;
      __syncthreads();
      if (keep) far[base + __popcll(mk & ((1ull << lane) - 1))] = x;
      if (to_near) {
        const int ni = atomicAdd(&s_next, 1);
        if (ni < NCAP) cur[ni] = (int)(unsigned)(x & 0xffffffffu);
        else s_bad = 1;
      }
      if (lane == 0) s_far = base + __popcll(mk);
      __syncthreads();
    }
    nnear = s_next < NCAP ? s_next : NCAP;
    if (s_bad) { status = 2; break; }
  }
  const float total = gof(st[t]);
  int len = 0;
  if (status < 2) status = total < __int_as_float(0x7f800000) ? 0 : 1;
  if (lane == 0) {
    if (status == 0) {
      int* path = a.out_path + (size_t)q * a.max_path;
      int v = t;
      while (true) {
        if (len >= a.max_path) { status = 4; break; }
        path[len++] = v;
        if (v == s) break;
        v = (int)((unsigned)st[v] & 0x7fffffffu);
      }
      if (status == 0) {
        for (int i = 0, j = len - 1; i < j; ++i, --j) {
          const int tmp = path[i];
          path[i] = path[j];
          path[j] = tmp;
        }
      } else {
        len = 0;
      }
    }
    if (a.out_iters) a.out_iters[q] = (int)(expanded < 0x7fffffff ? expanded : 0x7fffffff);
    a.out_cost[q] = status == 0 ? total : -1.f;
    a.out_len[q] = len;
    a.out_status[q] = status;
  }
  __syncthreads();
  const int nt = s_touch < a.cap ? s_touch : a.cap;
  for (int i = lane; i < nt; i += 64) {
    const int v = touched[i];
    st[v] = ST_INIT;
    hc[v] = __int_as_float(-1);                      // NaN: not cached
  }
}

hipError_t launch_astar_wave(const int* indptr, const int* indices, const float* cost, const float* lat,
                             const float* lon, const int* src, const int* dst, void* state, void* heap,
                             int* touched, float* out_cost, int* out_len, int* out_status, int* out_path,
                             int N, int Q, int slots, int cap, int max_path, int max_iters, float inv_vmax,
                             const float* lm, int K, const int* qidx, int T, float delta, float* hcache,
                             int hrows, hipStream_t stream, int* out_iters) {
  int n = T < slots ? T : slots;
  if (n > hrows) n = hrows;
  if (n <= 0) return hipSuccess;
  if (lm != nullptr && K != 32 && K != 16 && K != 8) return hipErrorInvalidValue;
  if (cap < 128) return hipErrorInvalidValue;
  AstarArgs a{indptr, indices, cost, lat, lon, src, dst, (unsigned long long*)state,
              (unsigned long long*)heap, touched, out_cost, out_len, out_status, out_path,
              N, Q, 0, slots, cap, max_path, max_iters, inv_vmax, lm, K, out_iters};
  if (lm == nullptr) hipLaunchKernelGGL(astar_wave_kernel<0>, dim3(n), dim3(64), 0, stream, a, qidx, n, delta, hcache);
  else if (K == 8) hipLaunchKernelGGL(astar_wave_kernel<8>, dim3(n), dim3(64), 0, stream, a, qidx, n, delta, hcache);
  else if (K == 16) hipLaunchKernelGGL(astar_wave_kernel<16>, dim3(n), dim3(64), 0, stream, a, qidx, n, delta, hcache);
  else hipLaunchKernelGGL(astar_wave_kernel<32>, dim3(n), dim3(64), 0, stream, a, qidx, n, delta, hcache);
  return hipGetLastError();
}

hipError_t launch_astar(const int* indptr, const int* indices, const float* cost, const float* lat,
                        const float* lon, const int* src, const int* dst, void* state,
                        void* heap, int* touched, float* out_cost, int* out_len, int* out_status,
                        int* out_path, int N, int Q, int q0, int slots, int cap, int max_path,
                        int max_iters, float inv_vmax, const float* lm, int K,
                        hipStream_t stream, int* out_iters) {
  const int n = min(slots, Q - q0);
  if (n <= 0) return hipSuccess;
  if (lm != nullptr && K != 32 && K != 16 && K != 8) return hipErrorInvalidValue;
  AstarArgs a{indptr, indices, cost, lat, lon, src, dst, (unsigned long long*)state,
              (unsigned long long*)heap, touched, out_cost, out_len, out_status, out_path,
              N, Q, q0, slots, cap, max_path, max_iters, inv_vmax, lm, K, out_iters};
  // one wavefront per workgroup (a wave runs as long as its longest search); grid rounded to a
  // multiple of 8 for the XCD-aware remap in the kernel (surplus lanes exit at the slot check)
  const dim3 grid(((n + 63) / 64 + 7) / 8 * 8), block(64);
  static const int arity = [] {
    const char* v = std::getenv("ROUTEST_ASTAR_ARITY");
    const int d = v != nullptr ? std::atoi(v) : 8;
    return (d == 2 || d == 4) ? d : 8;
  }();
  if (a.cap < 64) return hipErrorInvalidValue;
  if (arity == 2) {
    if (lm == nullptr) hipLaunchKernelGGL((astar_kernel<0, 2>), grid, block, 0, stream, a);
    else if (K == 8) hipLaunchKernelGGL((astar_kernel<8, 2>), grid, block, 0, stream, a);
    else if (K == 16) hipLaunchKernelGGL((astar_kernel<16, 2>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((astar_kernel<32, 2>), grid, block, 0, stream, a);
  } else if (arity == 8) {
    if (lm == nullptr) hipLaunchKernelGGL((astar_kernel<0, 8>), grid, block, 0, stream, a);
    else if (K == 8) hipLaunchKernelGGL((astar_kernel<8, 8>), grid, block, 0, stream, a);
    else if (K == 16) hipLaunchKernelGGL((astar_kernel<16, 8>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((astar_kernel<32, 8>), grid, block, 0, stream, a);
  } else {
    if (lm == nullptr) hipLaunchKernelGGL((astar_kernel<0, 4>), grid, block, 0, stream, a);
    else if (K == 8) hipLaunchKernelGGL((astar_kernel<8, 4>), grid, block, 0, stream, a);
    else if (K == 16) hipLaunchKernelGGL((astar_kernel<16, 4>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((astar_kernel<32, 4>), grid, block, 0, stream, a);
  }
  return hipGetLastError();
}

}  // namespace rt
