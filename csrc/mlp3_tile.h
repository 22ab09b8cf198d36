// Per-wave 32-row tile building blocks of the 3-layer ETA MLP (shared by the inference kernel
// eta_mlp_fwd.hip and the training kernel eta_mlp_train.hip).
//
// Packed weight blob (host: routest_amd/ops/eta_mlp.py::pack_mlp3; device: eta_mlp_train.hip
// adamw_pack_kernel), all offsets multiples of 16 B:
//   [ w2p: (H/32)x(H/16)x64 lanes x 8 bf16 | w1p: (H/32)x64x8 bf16 | b1p | b2p | w3p (H f32 each,
//     accumulator-register order) | tail: b3, 0, 0, 0 (f32) ]
#pragma once
#include "lds_fill.h"
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
  lds_fill_block(smem, blob, (int)L::BLOB);
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

// The H/32 layer-1 A fragments of this lane (W1k incl. the b1 hi/lo columns): loaded once per
// kernel and kept in registers by persistent waves.
template <int H>
struct W1Frags {
  bf16x8 f[H / 32];
  __device__ __forceinline__ void load(const Mlp3View<H>& w, int lane) {
#pragma unroll
    for (int mt = 0; mt < H / 32; ++mt) f[mt] = w.w1p[mt * 64 + lane];
  }
};

// Layer 1: h1^T = relu(W1k f^T) (bias folded into k = 14, 15) as bf16 B fragments h1[ks].
template <int H>
__device__ __forceinline__ void mlp3_layer1(const W1Frags<H>& w1, const bf16x8 xb,
                                            bf16x8 (&h1)[H / 16]) {
#pragma unroll
  for (int mt = 0; mt < H / 32; ++mt) {
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    acc = mfma32(w1.f[mt], xb, acc);
    float a[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = acc[e];
    relu_cvt_bf16x8(a, &h1[2 * mt]);
    relu_cvt_bf16x8(a + 8, &h1[2 * mt + 1]);
  }
}

// Layer 2 over all hidden tiles with a 4-deep ring of A-fragment prefetches that runs across tile
// boundaries (fragment f = mt*KS + ks; loads for f+1..f+4 are in flight while f feeds the MFMA),
// so no MFMA waits on the LDS read issued just before it.  epi(mt, acc) consumes each finished
// 32-row pre-activation tile z2^T[32mt..32mt+31][batch].
//
// PIPE = true software-pipelines the epilogue: epi(mt - 1) is issued after the first MFMA group of
// tile mt, so its VALU work (relu, dot with w3, ...) can fill the issue slots inside this wave's
// own MFMA gaps instead of running while the SIMD's matrix core idles.
template <int H, bool PIN = false, bool PIPE = false, typename Epi>
__device__ __forceinline__ void mlp3_layer2(const Mlp3View<H>& w, const bf16x8 (&h1)[H / 16],
                                            int lane, int h, Epi&& epi) {
  constexpr int MT = H / 32, KS = H / 16, NF = MT * KS, D = 4;
  const bf16x8* wa = w.w2p + lane;
  bf16x8 r0 = wa[0 * 64], r1 = wa[1 * 64], r2 = wa[2 * 64], r3 = wa[3 * 64];
  f32x16 prev;
#pragma unroll 1
  for (int mt = 0; mt < MT; ++mt) {
    f32x16 acc = load_vec16(w.b2p, mt, h);
    const int base = mt * KS;
#pragma unroll
    for (int ks = 0; ks < KS; ks += D) {
      // consume r0..r3 (fragments base+ks .. +3), refill with base+ks+4 .. +7 (clamped in range)
      const bf16x8 c0 = r0, c1 = r1, c2 = r2, c3 = r3;
      const int nf = base + ks + D;
      r0 = wa[min(nf + 0, NF - 1) * 64];
      r1 = wa[min(nf + 1, NF - 1) * 64];
      r2 = wa[min(nf + 2, NF - 1) * 64];
      r3 = wa[min(nf + 3, NF - 1) * 64];
      acc = mfma32(c0, h1[ks + 0], acc);
      acc = mfma32(c1, h1[ks + 1], acc);
      acc = mfma32(c2, h1[ks + 2], acc);
      acc = mfma32(c3, h1[ks + 3], acc);
      // pin the order: the 4 refill reads issue BEFORE the 4 MFMAs that consume older fragments
      // (hipcc otherwise sinks each read next to its MFMA and waits lgkmcnt(0) on it)
      if constexpr (PIN) {
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
      if constexpr (PIPE) {
        if (ks == 0 && mt > 0) epi(mt - 1, prev);
      }
    }
    if constexpr (PIPE) prev = acc;
    else epi(mt, acc);
  }
  if constexpr (PIPE) epi(MT - 1, prev);
}

}  // namespace rt
