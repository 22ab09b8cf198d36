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

hipError_t launch_forest(const void* rec, const float* values, const unsigned* info, const int* roots,
                         float* out, int B, int T, int M, float base, int le, const int* fmap,
                         hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  ForestArgs a{(const int4*)rec, values, info, roots, out, B, T, M, base, le, {}};
  for (int j = 0; j < 12; ++j) a.fmap[j] = fmap[j];
  hipLaunchKernelGGL(forest_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace rt
