// K9: batched point-to-point A* on a road graph with learned edge costs (north-star config 5).
// Conceptually replaces the reference's per-trip ORS directions calls (RO/Flaskr/utils.py:55-62,
// 151-156), which it issues one at a time over HTTPS.
//
// One LANE per query ("slot"): tens of thousands of independent searches in flight, each with
//   * dense per-slot g[N] (f32) and parent[N] (i32; bit 31 = closed) arrays in HBM — 16k slots x
//     100k nodes = 13 GB, which 288 GB of HBM3E makes the simple and fast choice (no hashing);
//   * a binary min-heap of (f, node) 64-bit entries with lazy deletion (stale pops are skipped via
//     the closed bit; the heuristic is consistent, so a node's first pop is final);
//   * a touched list, so only the entries a search wrote are reset afterwards (no N-sized memset
//     per query).
// Heuristic: max(great-circle distance x circuity / v_max, ALT landmark bound); edge costs are
// floored at length / v_max on the host, so both are admissible and consistent (ALT tables are
// shrunk by 1e-4 against fp32 rounding).  Every lane stops within max_iters pops (status 3), on heap
// or touched-list overflow (status 2) or when the open set empties (status 1): the grid always
// drains.  Paths are written target->source then reversed in place.
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
  float* g;              // [S][N]
  int* parent;           // [S][N]
  unsigned long long* heap;  // [S][cap]
  int* touched;          // [S][cap]
  float* out_cost;       // [Q]
  int* out_len;          // [Q]
  int* out_status;       // [Q]
  int* out_path;         // [Q][max_path]
  int N, Q, q0, cap, max_path, max_iters;
  float inv_vmax;        // seconds per metre at v_max
  const float* lm;       // [N][2K] ALT landmark tables: d(L_k -> v), d(v -> L_k) (nullptr: off)
  int K;
};

constexpr int KMAX = 16;

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

__device__ __forceinline__ unsigned long long hkey(float f, int v) {
  return ((unsigned long long)__float_as_uint(f) << 32) | (unsigned)v;   // f >= 0: monotone bits
}

template <int K>
__global__ __launch_bounds__(256) void astar_kernel(AstarArgs a) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  const int q = a.q0 + slot;
  if (q >= a.Q) return;
  float* g = a.g + (size_t)slot * a.N;
  int* par = a.parent + (size_t)slot * a.N;
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
  g[s] = 0.f;
  par[s] = -1 & 0x7fffffff;
  touched[nt++] = s;
  heap[hn++] = hkey(heur(s), s);
  int it = 0;
  for (; hn > 0; ++it) {
    if (it >= a.max_iters) { status = 3; break; }
    // pop min
    const unsigned long long top = heap[0];
    const unsigned long long last = heap[--hn];
    if (hn > 0) {
      int i = 0;
      while (true) {
        int c = 2 * i + 1;
        if (c >= hn) break;
        unsigned long long cv = heap[c];
        if (c + 1 < hn) {
          const unsigned long long c2 = heap[c + 1];
          if (c2 < cv) { cv = c2; ++c; }
        }
        if (cv >= last) break;
        heap[i] = cv;
        i = c;
      }
      heap[i] = last;
    }
    const int v = (int)(unsigned)(top & 0xffffffffu);
    const unsigned pv = (unsigned)par[v];
    if (pv & CLOSED) continue;           // stale duplicate
    par[v] = (int)(pv | CLOSED);
    if (v == t) { status = 0; break; }
    const float gv = g[v];
    const int e1 = a.indptr[v + 1];
    bool overflow = false;
    for (int e = a.indptr[v]; e < e1; ++e) {
      const int u = a.indices[e];
      const unsigned pu = (unsigned)par[u];
      if (pu & CLOSED) continue;
      const float ng = gv + a.cost[e];
      const float gu = g[u];
      if (ng < gu) {
        if (gu == __int_as_float(0x7f800000)) {   // first touch
          if (nt >= a.cap) { overflow = true; break; }
          touched[nt++] = u;
        }
        g[u] = ng;
        par[u] = v;
        if (hn >= a.cap) { overflow = true; break; }
        // push + sift up
        unsigned long long key = hkey(ng + heur(u), u);
        int i = hn++;
        while (i > 0) {
          const int p = (i - 1) >> 1;
          const unsigned long long pk = heap[p];
          if (pk <= key) break;
          heap[i] = pk;
          i = p;
        }
        heap[i] = key;
      }
    }
    if (overflow) { status = 2; break; }
  }
  int len = 0;
  float total = 0.f;
  if (status == 0) {
    total = g[t];
    int* path = a.out_path + (size_t)q * a.max_path;
    int v = t;
    while (true) {
      if (len >= a.max_path) { status = 4; break; }
      path[len++] = v;
      if (v == s) break;
      v = (int)((unsigned)par[v] & 0x7fffffffu);
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
  a.out_cost[q] = status == 0 ? total : -1.f;
  a.out_len[q] = len;
  a.out_status[q] = status;
  // reset this slot's touched entries for the next batch
  const float inf = __int_as_float(0x7f800000);
  for (int i = 0; i < nt; ++i) {
    const int v = touched[i];
    g[v] = inf;
    par[v] = 0x7fffffff;
  }
}

hipError_t launch_astar(const int* indptr, const int* indices, const float* cost, const float* lat,
                        const float* lon, const int* src, const int* dst, float* g, int* parent,
                        void* heap, int* touched, float* out_cost, int* out_len, int* out_status,
                        int* out_path, int N, int Q, int q0, int slots, int cap, int max_path,
                        int max_iters, float inv_vmax, const float* lm, int K,
                        hipStream_t stream) {
  const int n = min(slots, Q - q0);
  if (n <= 0) return hipSuccess;
  if (lm != nullptr && K != 16 && K != 8) return hipErrorInvalidValue;
  AstarArgs a{indptr, indices, cost, lat, lon, src, dst, g, parent,
              (unsigned long long*)heap, touched, out_cost, out_len, out_status, out_path,
              N, Q, q0, cap, max_path, max_iters, inv_vmax, lm, K};
  // one wavefront per workgroup: with length-sorted queries each wave is homogeneous, and the
  // dispatcher's round-robin placement spreads short and long waves over all CUs (256-lane
  // workgroups would pile the longest searches onto a few CUs and leave a serial tail)
  const dim3 grid((n + 63) / 64), block(64);
  if (lm == nullptr) hipLaunchKernelGGL(astar_kernel<0>, grid, block, 0, stream, a);
  else if (K == 8) hipLaunchKernelGGL(astar_kernel<8>, grid, block, 0, stream, a);
  else hipLaunchKernelGGL(astar_kernel<16>, grid, block, 0, stream, a);
  return hipGetLastError();
}

}  // namespace rt
