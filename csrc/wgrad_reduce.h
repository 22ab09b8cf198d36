// Deterministic split-K slab reduction shared by wgrad_reduce_kernel (wgrad.hip) and the one-rank
// fused reduce + AdamW of the H <= 256 trainer (reduce_adamw_kernel, eta_mlp_train.hip): both sum a
// workgroup's 64 bucket values with the same loads in the same order, so their gradients agree bit
// for bit.  A workgroup of 256 threads reduces RED_COLS float4 columns, RED_SL slice lanes per column.
#pragma once

#include "common.h"

namespace rt {

constexpr int RED_SL = 16, RED_COLS = 16;

// Up to three independent segments (slab regions with their own slice counts) in one launch:
// blocks [0, nb0) reduce segment 0, [nb0, nb01) segment 1, the rest segment 2.
struct RedSeg {
  const float* slab;
  long long slab_stride;
  float* G;
  int S, n;
  int perm_h;        // 0: slab and G share a layout; H: train_bwd_kernel<H>'s register-native dW2 slabs
  int fold_ld = 0;   // > 0: the float4 at column fold_col of every fold_ld-wide row holds partials of
  int fold_col = 0;  // ONE value (wgrad256's db2 per tile column): stored as (x + y + z + w, 0, 0, 0)
};

__device__ __forceinline__ int red_hperm(int u) { return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1); }

// G's index of slab element e (e % 4 == 0) and the stride of its 3 successors in the register-native
// layout of train_bwd_kernel<H> (eta_mlp_train.hip): accumulator tile (w, i, mt) = 1024 floats, lane
// l's registers 4q .. 4q+3 at q*256 + 4l — rows 32mt + 8q + 4(l >> 5) + j of bucket column
// hperm(32(2w+i) + (l & 31)); past H*H the [row][16] block of the db2 / zero columns.
__device__ __forceinline__ void native_to_bucket(int e, int H, int& g0, int& step) {
  const int LDG = H + 16, MT = H / 32;
  if (e >= H * H) {
    const int x = e - H * H;
    g0 = (x >> 4) * LDG + H + (x & 15);
    step = 1;
    return;
  }
  const int blk = e >> 10, rem = e & 1023, q = rem >> 8, l = (rem & 255) >> 2;
  const int wi = blk / MT, mt = blk - wi * MT;
  const int nc = red_hperm(32 * wi + (l & 31));
  g0 = (32 * mt + 8 * q + 4 * (l >> 5)) * LDG + nc;
  step = LDG;
}

using RedPart = float4[RED_SL][RED_COLS + 1];

// Sum over the S slices of segment sg's elements e .. e+3, e = (blk * RED_COLS + c) * 4, c = thread &
// (RED_COLS - 1).  Valid in the returned value for threads of slice lane 0 with e < n; part is the
// workgroup's LDS scratch (one barrier inside).
template <bool NTLOAD>
__device__ __forceinline__ float4 red_sum(const RedSeg& sg, int blk, RedPart& part) {
  const float* __restrict__ slab = sg.slab;
  const long long slab_stride = sg.slab_stride;
  const int S = sg.S, n = sg.n;
  const int c = threadIdx.x & (RED_COLS - 1), sl = threadIdx.x / RED_COLS;
  const int e = (blk * RED_COLS + c) * 4;
  const bool vec = (slab_stride % 4) == 0 && e + 4 <= n;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n) {
    if (vec) {
      f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
      auto ld = [&](int k) {
        const f32x4* q = reinterpret_cast<const f32x4*>(slab + (long long)k * slab_stride + e);
        if constexpr (NTLOAD) return __builtin_nontemporal_load(q);
        else return *q;
      };
      int s = sl;
      for (; s + 3 * RED_SL < S; s += 4 * RED_SL) {
        const f32x4 v0 = ld(s), v1 = ld(s + RED_SL), v2 = ld(s + 2 * RED_SL), v3 = ld(s + 3 * RED_SL);
        a4 += v0;
        a4 += v1;
        a4 += v2;
        a4 += v3;
      }
      for (; s < S; s += RED_SL) a4 += ld(s);
      acc = make_float4(a4[0], a4[1], a4[2], a4[3]);
    } else {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s = sl; s < S; s += RED_SL)
        for (int q = 0; q < 4 && e + q < n; ++q) t[q] += slab[(long long)s * slab_stride + e + q];
      acc = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
  part[sl][c] = acc;
  __syncthreads();
  float4 r = part[0][c];
  if (sl == 0 && e < n) {
    for (int k = 1; k < RED_SL; ++k) {
      const float4 v = part[k][c];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    if (sg.fold_ld > 0 && e % sg.fold_ld == sg.fold_col) r = make_float4(((r.x + r.y) + r.z) + r.w, 0.f, 0.f, 0.f);
  }
  return r;
}

}  // namespace rt
