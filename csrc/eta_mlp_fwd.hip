// K1 + K2: fused ETA featurize + 3-layer MLP forward (bf16 MFMA, fp32 accumulate) for gfx950.
//
// Replaces the reference's per-request CPU path  dict -> pandas.DataFrame -> XGBRegressor.predict
// (RO/Flaskr/ml.py:35-53) with ONE launch over a batch of packed 16-byte request records:
//
//   y[b] = w3 . relu(W2 relu(W1 f(rec[b]) + b1) + b2) + b3        (w3/b3 carry the target scale)
//
// Work decomposition: each wave owns 32 batch rows at a time ("batch on the lane", common.h).
//   * featurize: lane (r, h) builds features 8h..8h+7 of row r directly as the bf16 B fragment
//   * layer 1  : H/32 MFMAs 32x32x16 (K = 12 features padded to 16; km/age hi/lo split uses pads)
//   * layer 2  : (H/32) x (H/16) MFMAs; the layer-1 accumulators ARE the B operands (no LDS trip)
//   * layer 3  : fused into the layer-2 epilogue: relu(acc) * w3 summed in registers, one
//                cross-half shuffle, one 128-B store per 32 rows.
// Weight fragments are pre-permuted on the host so every A-fragment fetch is one lane-linear,
// bank-conflict-free 16-byte read.
//
// Two variants:
//   LDSW = true : persistent grid (1 workgroup of 8 waves per CU); the whole packed weight blob
//                 (2H^2 + 44H bytes = 139 KiB at H = 256) is staged into LDS once per workgroup
//                 and re-used for every tile the workgroup processes.  At one ds_read_b128 per
//                 32-cycle MFMA the LDS stays well under its 256 B/clk/CU rate.
//   LDSW = false: weights read straight from global (L2-resident, lane-linear 1 KiB per wave
//                 instruction) — for small serving batches where staging 139 KiB per CU would
//                 dominate.
#include "common.h"
#include "ops.h"

namespace rt {

template <int H>
struct Mlp3Layout {
  static constexpr int MT = H / 32;   // 32-row hidden tiles
  static constexpr int KS = H / 16;   // 16-deep k-steps over the hidden dim
  static constexpr size_t W2B = (size_t)H * H * 2;
  static constexpr size_t W1B = (size_t)H * 16 * 2;
  static constexpr size_t VB = (size_t)H * 4;
  static constexpr size_t BLOB = W2B + W1B + 3 * VB;
};

template <int H, bool LDSW>
__global__ __launch_bounds__(LDSW ? 512 : 256, LDSW ? 2 : 1) void eta_mlp3_fwd_kernel(const int4* __restrict__ rec,
                                                              float* __restrict__ out, int B,
                                                              const unsigned char* __restrict__ blob,
                                                              NormParams np, float b3) {
  using L = Mlp3Layout<H>;
  constexpr int MT = L::MT, KS = L::KS;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const unsigned char* base = blob;
  if constexpr (LDSW) {
    const int4* src = reinterpret_cast<const int4*>(blob);
    int4* dst = reinterpret_cast<int4*>(smem);
    constexpr int N16 = (int)(L::BLOB / 16);
    for (int i = threadIdx.x; i < N16; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    base = smem;
  }
  const bf16x8* w2p = reinterpret_cast<const bf16x8*>(base);
  const bf16x8* w1p = reinterpret_cast<const bf16x8*>(base + L::W2B);
  const f32x4* b1p = reinterpret_cast<const f32x4*>(base + L::W2B + L::W1B);
  const f32x4* b2p = b1p + H / 4;
  const f32x4* w3p = b2p + H / 4;

  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int r = lane & 31;
  const int wpb = blockDim.x >> 6;
  const int ntiles = (B + 31) >> 5;
  const int stride = gridDim.x * wpb;

  for (int tile = blockIdx.x * wpb + (threadIdx.x >> 6); tile < ntiles; tile += stride) {
    const int row = tile * 32 + r;
    const int4 rc = row < B ? rec[row] : make_int4(0, 0, 0, 0);
    float f[8];
    featurize_f32(rc, h, np, f);
    const bf16x8 xb = to_bf16x8(f);

    // ---- layer 1: h1^T = relu(W1k x^T + b1), kept as bf16 B fragments ----
    bf16x8 h1[KS];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f32x16 acc;
      const f32x4* bp = b1p + (mt * 2 + h) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 bv = bp[q];
        acc[4 * q + 0] = bv[0];
        acc[4 * q + 1] = bv[1];
        acc[4 * q + 2] = bv[2];
        acc[4 * q + 3] = bv[3];
      }
      acc = mfma32(w1p[mt * 64 + lane], xb, acc);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) h1[2 * mt + s][j] = (__bf16)fmaxf(acc[8 * s + j], 0.f);
      }
    }

    // ---- layer 2 + fused layer 3 ----
    float ys = 0.f;
#pragma unroll 1
    for (int mt = 0; mt < MT; ++mt) {
      f32x16 acc;
      const f32x4* bp = b2p + (mt * 2 + h) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 bv = bp[q];
        acc[4 * q + 0] = bv[0];
        acc[4 * q + 1] = bv[1];
        acc[4 * q + 2] = bv[2];
        acc[4 * q + 3] = bv[3];
      }
      const bf16x8* wa = w2p + (size_t)mt * KS * 64 + lane;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = mfma32(wa[ks * 64], h1[ks], acc);
      const f32x4* wp = w3p + (mt * 2 + h) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 wv = wp[q];
        ys += fmaxf(acc[4 * q + 0], 0.f) * wv[0];
        ys += fmaxf(acc[4 * q + 1], 0.f) * wv[1];
        ys += fmaxf(acc[4 * q + 2], 0.f) * wv[2];
        ys += fmaxf(acc[4 * q + 3], 0.f) * wv[3];
      }
    }
    ys += __shfl_xor(ys, 32);
    if (h == 0 && row < B) out[row] = ys + b3;
  }
}

// K1 standalone: records -> raw R16 features [B, 12] fp32 (reference order; CPU parity tests and
// the autograd training path use it).
__global__ __launch_bounds__(256) void eta_featurize_kernel(const int4* __restrict__ rec,
                                                            float* __restrict__ out, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  float f[12];
  featurize_raw12(rec[i], f);
  float4* o = reinterpret_cast<float4*>(out + (size_t)i * 12);
  o[0] = make_float4(f[0], f[1], f[2], f[3]);
  o[1] = make_float4(f[4], f[5], f[6], f[7]);
  o[2] = make_float4(f[8], f[9], f[10], f[11]);
}

template <int H>
static hipError_t launch_fwd_h(const void* rec, float* out, int B, const void* blob,
                               const NormParams& np, float b3, int variant, int num_cus,
                               hipStream_t stream) {
  using L = Mlp3Layout<H>;
  const int ntiles = (B + 31) / 32;
  if (ntiles == 0) return hipSuccess;
  const bool lds_fits = L::BLOB <= 160 * 1024;
  bool use_lds = lds_fits && (variant == 1 || (variant < 0 && ntiles >= num_cus * 8 * 2));
  if (use_lds) {
    static bool attr_set[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (!attr_set[dev & 63]) {
      hipError_t e = hipFuncSetAttribute((const void*)eta_mlp3_fwd_kernel<H, true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::BLOB);
      if (e != hipSuccess) return e;
      attr_set[dev & 63] = true;
    }
    const int waves_needed = ntiles;
    int grid = (waves_needed + 7) / 8;
    if (grid > num_cus) grid = num_cus;
    hipLaunchKernelGGL((eta_mlp3_fwd_kernel<H, true>), dim3(grid), dim3(512), L::BLOB, stream,
                       (const int4*)rec, out, B, (const unsigned char*)blob, np, b3);
  } else {
    // 4 waves per workgroup, one tile per wave
    int grid = (ntiles + 3) / 4;
    hipLaunchKernelGGL((eta_mlp3_fwd_kernel<H, false>), dim3(grid), dim3(256), 0, stream,
                       (const int4*)rec, out, B, (const unsigned char*)blob, np, b3);
  }
  return hipGetLastError();
}

hipError_t launch_eta_mlp3_fwd(const void* rec, float* out, int B, const void* blob, int H,
                               const NormParams& np, float b3, int variant, int num_cus,
                               hipStream_t stream) {
  switch (H) {
    case 64: return launch_fwd_h<64>(rec, out, B, blob, np, b3, variant, num_cus, stream);
    case 128: return launch_fwd_h<128>(rec, out, B, blob, np, b3, variant, num_cus, stream);
    case 256: return launch_fwd_h<256>(rec, out, B, blob, np, b3, variant, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

size_t eta_mlp3_blob_bytes(int H) { return (size_t)2 * H * H + 44 * (size_t)H; }

hipError_t launch_eta_featurize(const void* rec, float* out, int B, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(eta_featurize_kernel, dim3((B + 255) / 256), dim3(256), 0, stream,
                     (const int4*)rec, out, B);
  return hipGetLastError();
}

}  // namespace rt
