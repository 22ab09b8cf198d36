// Per-wave 32-row tile building blocks of the 3-layer ETA MLP (shared by the inference kernel
// eta_mlp_fwd.hip and the training kernel eta_mlp_train.hip).
//
// Packed weight blob (host: routest_amd/ops/eta_mlp.py::pack_mlp3; device: eta_mlp_train.hip
// adamw_pack_kernel), all offsets multiples of 16 B:
//   [ w2p: (H/32)x(H/16)x64 lanes x 8 bf16 | w1p: (H/32)x64x8 bf16 | b1p | b2p | w3p (H f32 each,
//     accumulator-register order) | tail: b3, 0, 0, 0 (f32) ]
#pragma once
#include "common.h"

namespace rt {

template <int H>
struct Mlp3Layout {
  static constexpr int MT = H / 32;   // 32-row hidden tiles
  static constexpr int KS = H / 16;   // 16-deep k-steps over the hidden dim
  static constexpr size_t W2B = (size_t)H * H * 2;
  static constexpr size_t W1B = (size_t)H * 16 * 2;
  static constexpr size_t VB = (size_t)H * 4;
  static constexpr size_t TAIL = 16;
  static constexpr size_t BLOB = W2B + W1B + 3 * VB + TAIL;
};

inline size_t mlp3_blob_bytes(int H) { return (size_t)2 * H * H + 44 * (size_t)H + 16; }

template <int H>
struct Mlp3View {
  const bf16x8* w2p;
  const bf16x8* w1p;
  const f32x4* b1p;
  const f32x4* b2p;
  const f32x4* w3p;
  const float* tail;
  __device__ __forceinline__ explicit Mlp3View(const unsigned char* base) {
    using L = Mlp3Layout<H>;
    w2p = reinterpret_cast<const bf16x8*>(base);
    w1p = reinterpret_cast<const bf16x8*>(base + L::W2B);
    b1p = reinterpret_cast<const f32x4*>(base + L::W2B + L::W1B);
    b2p = b1p + H / 4;
    w3p = b2p + H / 4;
    tail = reinterpret_cast<const float*>(w3p + H / 4);
  }
};

// Cooperative global -> LDS copy of the whole blob (16 B per thread per step).
template <int H>
__device__ __forceinline__ void stage_blob(const unsigned char* __restrict__ blob, unsigned char* smem) {
  using L = Mlp3Layout<H>;
  const int4* src = reinterpret_cast<const int4*>(blob);
  int4* dst = reinterpret_cast<int4*>(smem);
  constexpr int N16 = (int)(L::BLOB / 16);
  for (int i = threadIdx.x; i < N16; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// 16 accumulator-order floats of a per-hidden vector for tile mt, lane half h.
__device__ __forceinline__ f32x16 load_vec16(const f32x4* v, int mt, int h) {
  f32x16 acc;
  const f32x4* p = v + (mt * 2 + h) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 t = p[q];
    acc[4 * q + 0] = t[0];
    acc[4 * q + 1] = t[1];
    acc[4 * q + 2] = t[2];
    acc[4 * q + 3] = t[3];
  }
  return acc;
}

// Layer 1: h1^T = relu(W1k f^T + b1) as bf16 B fragments h1[ks] (ks = 2*mt + s).
template <int H>
__device__ __forceinline__ void mlp3_layer1(const Mlp3View<H>& w, const bf16x8 xb, int lane, int h,
                                            bf16x8 (&h1)[H / 16]) {
#pragma unroll
  for (int mt = 0; mt < H / 32; ++mt) {
    f32x16 acc = load_vec16(w.b1p, mt, h);
    acc = mfma32(w.w1p[mt * 64 + lane], xb, acc);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) h1[2 * mt + s][j] = (__bf16)fmaxf(acc[8 * s + j], 0.f);
    }
  }
}

// Layer 2 pre-activation tile mt: z2^T[32mt .. 32mt+31][batch] = W2 h1^T + b2.
template <int H>
__device__ __forceinline__ f32x16 mlp3_layer2_tile(const Mlp3View<H>& w, const bf16x8 (&h1)[H / 16],
                                                   int mt, int lane, int h) {
  constexpr int KS = H / 16;
  f32x16 acc = load_vec16(w.b2p, mt, h);
  const bf16x8* wa = w.w2p + (size_t)mt * KS * 64 + lane;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) acc = mfma32(wa[ks * 64], h1[ks], acc);
  return acc;
}

}  // namespace rt
