// K4: tree-ensemble ETA inference (reference compatibility: its model is an XGBoost regressor,
// RO/Flaskr/ml.py:53 / RO/xgb_eta_model.pkl) with the K1 featurize fused in front.
//
// Thread per row: featurize the 16-byte record into the 12 raw R16 features, stage them in the
// thread's own LDS slot (so the per-node feature lookup x[f] with a runtime f is one ds_read, not a
// 12-way select or a scratch access), then walk every tree.  Nodes are 8 bytes (value/threshold,
// packed info) in breadth-first order, so the two children of a node are adjacent and the walk is
// one dependent 8-byte load per level; a 2-3 MB ensemble stays L2-resident per XCD.
#include "common.h"
#include "ops.h"

namespace rt {

struct ForestArgs {
  const int4* rec;
  const float* values;
  const unsigned* info;
  const int* roots;
  float* out;
  int B, T, M;
  float base;
  int le;                 // 1: x <= thr goes left (sklearn), 0: x < thr (XGBoost)
  int fmap[12];           // model feature j -> R16 column
};

__global__ __launch_bounds__(256) void forest_kernel(ForestArgs a) {
  __shared__ float xs[256][13];   // +1 pad: conflict-free per-thread rows
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.B) return;         // no block-wide barrier below: early exit is safe
  float raw[12];
  featurize_raw12(a.rec[row], raw);
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    float v = raw[0];
#pragma unroll
    for (int c = 1; c < 12; ++c) v = (a.fmap[j] == c) ? raw[c] : v;
    xs[threadIdx.x][j] = v;
  }
  float acc = a.base;
  for (int t = 0; t < a.T; ++t) {
    const int root = a.roots[t];
    int n = root;
    unsigned inf = a.info[n];
    int guard = 0;
    while (!(inf >> 31) && guard++ < 64) {
      const int f = (inf >> 24) & 63;
      const float v = xs[threadIdx.x][f < 12 ? f : 0];
      const float thr = a.values[n];
      bool left;
      if (v != v) left = (inf >> 30) & 1;
      else left = a.le ? (v <= thr) : (v < thr);
      n = root + (int)(inf & 0xFFFFFFu) + (left ? 0 : 1);
      if ((unsigned)n >= (unsigned)a.M) { n = root; break; }   // corrupt model: never read OOB
      inf = a.info[n];
    }
    acc += a.values[n];
  }
  a.out[row] = acc;
}

// ---------------------------------------------------------------------------------------------
// LDS-staged variant.  The ensemble is cut (on the host, at tree boundaries) into chunks of at
// most FOREST_LDS_NODES nodes.  One 1024-thread workgroup per CU: for each chunk it stages the
// chunk's nodes into LDS ONCE, then streams all of its row tiles through it (featurize the tile's
// records into the per-thread LDS feature rows, walk the chunk's trees, add the partial sum into
// the output row, which this workgroup owns for every chunk).  Each thread walks two trees at a time
// so the two dependent LDS-load chains overlap (4 walks per thread measured 298 vs 326 M preds/s:
// the union of four walks' depths per loop trip costs more than the extra overlap buys).  LDS: 96 KB nodes + 52 KB features.
constexpr int FOREST_LDS_NODES = 12288;
constexpr int FOREST_TPB = 1024;

__global__ __launch_bounds__(FOREST_TPB, 1) void forest_lds_kernel(ForestArgs a, const int* __restrict__ chunks,
                                                                    int nchunks) {
  __shared__ int2 nodes[FOREST_LDS_NODES];
  __shared__ float xs[FOREST_TPB][13];
  const int tid = threadIdx.x;
  const int ntiles = (a.B + FOREST_TPB - 1) / FOREST_TPB;
  for (int c = 0; c < nchunks; ++c) {
    const int t0 = chunks[2 * c], n0 = chunks[2 * c + 1];
    const int t1 = chunks[2 * c + 2], n1 = chunks[2 * c + 3];
    __syncthreads();                           // previous chunk fully consumed
    const int2* src = reinterpret_cast<const int2*>(a.values);   // (value, info) interleaved
    for (int i = tid; i < n1 - n0; i += FOREST_TPB) nodes[i] = src[n0 + i];
    __syncthreads();
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      const int row = tile * FOREST_TPB + tid;
      const bool live = row < a.B;
      if (live) {
        float raw[12];
        featurize_raw12(a.rec[row], raw);
#pragma unroll
        for (int j = 0; j < 12; ++j) {
          float v = raw[0];
#pragma unroll
          for (int q = 1; q < 12; ++q) v = (a.fmap[j] == q) ? raw[q] : v;
          xs[tid][j] = v;
        }
      }
      float acc = 0.f;
      if (live) {
        int t = t0;
        for (; t + 1 < t1; t += 2) {           // two independent walks in flight
          const int r0 = a.roots[t] - n0, r1 = a.roots[t + 1] - n0;
          int m0 = r0, m1 = r1;
          int2 d0 = nodes[m0], d1 = nodes[m1];
          int guard = 0;
          while ((d0.y >= 0 || d1.y >= 0) && guard++ < 64) {   // bit 31 set (negative) = leaf
            if (d0.y >= 0) {
              const unsigned inf = (unsigned)d0.y;
              const unsigned f = (inf >> 24) & 63;
              const float v = xs[tid][f < 12 ? f : 0];
              const float thr = __int_as_float(d0.x);
              const bool left = (v != v) ? ((inf >> 30) & 1) : (a.le ? (v <= thr) : (v < thr));
              m0 = r0 + (int)(inf & 0xFFFFFFu) + (left ? 0 : 1);
              d0 = nodes[m0 < n1 - n0 ? m0 : r0];
            }
            if (d1.y >= 0) {
              const unsigned inf = (unsigned)d1.y;
              const unsigned f = (inf >> 24) & 63;
              const float v = xs[tid][f < 12 ? f : 0];
              const float thr = __int_as_float(d1.x);
              const bool left = (v != v) ? ((inf >> 30) & 1) : (a.le ? (v <= thr) : (v < thr));
              m1 = r1 + (int)(inf & 0xFFFFFFu) + (left ? 0 : 1);
              d1 = nodes[m1 < n1 - n0 ? m1 : r1];
            }
          }
          acc += __int_as_float(d0.x);
          acc += __int_as_float(d1.x);
        }
        if (t < t1) {
          const int r0 = a.roots[t] - n0;
          int m0 = r0;
          int2 d0 = nodes[m0];
          int guard = 0;
          while (d0.y >= 0 && guard++ < 64) {
            const unsigned inf = (unsigned)d0.y;
            const unsigned f = (inf >> 24) & 63;
              const float v = xs[tid][f < 12 ? f : 0];
            const float thr = __int_as_float(d0.x);
            const bool left = (v != v) ? ((inf >> 30) & 1) : (a.le ? (v <= thr) : (v < thr));
            m0 = r0 + (int)(inf & 0xFFFFFFu) + (left ? 0 : 1);
            d0 = nodes[m0 < n1 - n0 ? m0 : r0];
          }
          acc += __int_as_float(d0.x);
        }
        a.out[row] = (c == 0 ? a.base : a.out[row]) + acc;
      }
    }
  }
}

hipError_t launch_forest(const void* rec, const float* values, const unsigned* info, const int* roots,
                         float* out, int B, int T, int M, float base, int le, const int* fmap,
                         hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  ForestArgs a{(const int4*)rec, values, info, roots, out, B, T, M, base, le, {}};
  for (int j = 0; j < 12; ++j) a.fmap[j] = fmap[j];
  hipLaunchKernelGGL(forest_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// nodes2: [M] int2 (value bits, info) interleaved; chunks: [nchunks+1][2] (first tree, first node)
hipError_t launch_forest_lds(const void* rec, const void* nodes2, const int* roots, const int* chunks,
                             int nchunks, float* out, int B, int T, int M, float base, int le,
                             const int* fmap, int num_cus, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  ForestArgs a{(const int4*)rec, (const float*)nodes2, nullptr, roots, out, B, T, M, base, le, {}};
  for (int j = 0; j < 12; ++j) a.fmap[j] = fmap[j];
  const int ntiles = (B + FOREST_TPB - 1) / FOREST_TPB;
  const int grid = ntiles < num_cus ? ntiles : num_cus;
  hipLaunchKernelGGL(forest_lds_kernel, dim3(grid), dim3(FOREST_TPB), 0, stream, a, chunks, nchunks);
  return hipGetLastError();
}

}  // namespace rt
