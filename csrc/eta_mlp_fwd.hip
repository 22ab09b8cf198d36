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
#include "mlp3_tile.h"
#include "ops.h"

namespace rt {

// Record loads for the three wire formats (16-byte full, 8-byte compact, 6-byte bulk record).
// ``T`` is what a lane holds between the prefetching load and its use: raw loaded words only, so
// the prefetch is never waited on before the tile that consumes it.
template <int RB>
struct RecT;
template <>
struct RecT<16> {
  using T = int4;
  static __device__ __forceinline__ T zero() { return make_int4(0, 0, 0, 0); }
  static __device__ __forceinline__ T load(const void* p, int i) { return ((const int4*)p)[i]; }
  static __device__ __forceinline__ bf16x8 feat(const T& r, int h, const NormParams& np) {
    return featurize_bf16(r, h, np);
  }
};
template <>
struct RecT<8> {
  using T = int2;
  static __device__ __forceinline__ T zero() { return make_int2(0, 0); }
  static __device__ __forceinline__ T load(const void* p, int i) { return ((const int2*)p)[i]; }
  static __device__ __forceinline__ bf16x8 feat(const T& r, int h, const NormParams& np) {
    return featurize8_bf16(r, h, np);
  }
};
struct Rec6Words {
  unsigned a, b, c;
};
template <>
struct RecT<6> {
  // 6-byte rows are only 2-byte aligned: three u16 loads (one VMEM triple per 32-row tile,
  // ~4k MFMA cycles of work) rather than a dword load that would straddle rows
  using T = Rec6Words;
  static __device__ __forceinline__ T zero() { return {0u, 0u, 0u}; }
  static __device__ __forceinline__ T load(const void* p, int i) {
    const unsigned short* s = (const unsigned short*)p + 3 * (size_t)i;
    return {s[0], s[1], s[2]};
  }
  static __device__ __forceinline__ bf16x8 feat(const T& r, int h, const NormParams& np) {
    return featurize6_bf16(r.a | (r.b << 16), r.c, h, np);
  }
};

template <int H, bool LDSW, int TPB, bool PIN = false, int RB = 16, bool PIPE = false,
          bool PRIO = false>
__global__ __launch_bounds__(TPB, LDSW ? TPB / 256 : 1) void eta_mlp3_fwd_kernel(
    const void* __restrict__ rec, float* __restrict__ out, int B,
    const unsigned char* __restrict__ blob, NormParams np) {
  constexpr int KS = H / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const unsigned char* base = blob;
  if constexpr (LDSW) {
    stage_blob<H>(blob, smem);
    base = smem;
  }
  const Mlp3View<H> w(base);
  const float b3 = w.tail[0];
  W1Frags<H> w1;
  w1.load(w, threadIdx.x & 63);

  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int r = lane & 31;
  const int wpb = blockDim.x >> 6;
  const int ntiles = (B + 31) >> 5;
  const int stride = gridDim.x * wpb;
  if constexpr (PRIO) {
    // static priority for the second-dispatched half of the workgroup (MI355X_MICROARCH.md, "two
    // waves per SIMD" item 4): the younger wave of each SIMD stops losing every VALU arbitration
    if ((threadIdx.x >> 6) >= (TPB >> 7)) __builtin_amdgcn_s_setprio(1);
  }

  // records are prefetched one tile ahead: with zero-copy I/O they come straight from pinned host
  // memory over PCIe, and the next tile's load then overlaps this tile's ~4k MFMA cycles
  int tile = blockIdx.x * wpb + (threadIdx.x >> 6);
  using R = RecT<RB>;
  typename R::T rc_next = R::zero();
  if (tile < ntiles && tile * 32 + r < B) rc_next = R::load(rec, tile * 32 + r);
  for (; tile < ntiles; tile += stride) {
    const int row = tile * 32 + r;
    const typename R::T rc = rc_next;
    const int nrow = (tile + stride) * 32 + r;
    if (tile + stride < ntiles && nrow < B) rc_next = R::load(rec, nrow);
    const bf16x8 xb = R::feat(rc, h, np);

    bf16x8 h1[KS];
    mlp3_layer1<H>(w1, xb, h1);

    // layer 2 + fused layer 3 (relu(acc) . w3 reduced in registers)
    // (relu as v_max_i32, the dot with w3 on packed v_pk_fma_f32: 24 VALU ops per 16 units)
    f32x2 ys2 = {0.f, 0.f};
    mlp3_layer2<H, PIN, PIPE>(w, h1, lane, h, [&](int mt, const f32x16& acc) {
      const f32x16 w3 = load_vec16(w.w3p, mt, h);
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 a2 = {relu_f(acc[i]), relu_f(acc[i + 1])};
        const f32x2 w2 = {w3[i], w3[i + 1]};
        ys2 = __builtin_elementwise_fma(a2, w2, ys2);
      }
    });
    float ys = ys2[0] + ys2[1];
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

// Persistent LDS-staged launch: one workgroup of T threads per CU (139 KiB of LDS at H = 256).
template <int H, int T, bool PIN, int RB, bool PIPE = false, bool PRIO = false>
static hipError_t launch_lds(const void* rec, float* out, int B, const void* blob,
                             const NormParams& np, int num_cus, hipStream_t stream) {
  using L = Mlp3Layout<H>;
  static bool attr_set[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!attr_set[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)eta_mlp3_fwd_kernel<H, true, T, PIN, RB, PIPE, PRIO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::BLOB);
    if (e != hipSuccess) return e;
    attr_set[dev & 63] = true;
  }
  const int ntiles = (B + 31) / 32;
  int grid = (ntiles + T / 64 - 1) / (T / 64);
  if (grid > num_cus) grid = num_cus;
  hipLaunchKernelGGL((eta_mlp3_fwd_kernel<H, true, T, PIN, RB, PIPE, PRIO>), dim3(grid), dim3(T), L::BLOB,
                     stream, rec, out, B, (const unsigned char*)blob, np);
  return hipGetLastError();
}

template <int H, int RB>
static hipError_t launch_fwd_h(const void* rec, float* out, int B, const void* blob,
                               const NormParams& np, int variant, int num_cus, hipStream_t stream) {
  // variant: -1 auto, 0 global weights, LDS-staged: 1 = 512 thr, 2 = 768 thr, 3/4 = same + pinned
  // read/MFMA interleave (auto -> 3, the measured best), 5/6 = 3/4 + software-pipelined epilogue,
  // 7 = 5 + static priority for waves 4-7, 8 = 3 + priority
  using L = Mlp3Layout<H>;
  const int ntiles = (B + 31) / 32;
  if (ntiles == 0) return hipSuccess;
  const bool lds_fits = L::BLOB <= 160 * 1024;
  bool use_lds = lds_fits && (variant >= 1 || (variant < 0 && ntiles >= num_cus * 8 * 2));
  if (use_lds) {
    switch (variant) {
      case 2: return launch_lds<H, 768, false, RB>(rec, out, B, blob, np, num_cus, stream);
      case 1: return launch_lds<H, 512, false, RB>(rec, out, B, blob, np, num_cus, stream);
      case 4: return launch_lds<H, 768, true, RB>(rec, out, B, blob, np, num_cus, stream);
      case 5: return launch_lds<H, 512, true, RB, true>(rec, out, B, blob, np, num_cus, stream);
      case 6: return launch_lds<H, 768, true, RB, true>(rec, out, B, blob, np, num_cus, stream);
      case 7: return launch_lds<H, 512, true, RB, true, true>(rec, out, B, blob, np, num_cus, stream);
      case 8: return launch_lds<H, 512, true, RB, false, true>(rec, out, B, blob, np, num_cus, stream);
      default: return launch_lds<H, 512, true, RB>(rec, out, B, blob, np, num_cus, stream);
    }
  } else {
    // 4 waves per workgroup, one tile per wave
    int grid = (ntiles + 3) / 4;
    hipLaunchKernelGGL((eta_mlp3_fwd_kernel<H, false, 256, false, RB>), dim3(grid), dim3(256), 0,
                       stream, rec, out, B, (const unsigned char*)blob, np);
  }
  return hipGetLastError();
}

template <int RB>
static hipError_t launch_fwd_rb(const void* rec, float* out, int B, const void* blob, int H,
                                const NormParams& np, int variant, int num_cus, hipStream_t stream) {
  switch (H) {
    case 64: return launch_fwd_h<64, RB>(rec, out, B, blob, np, variant, num_cus, stream);
    case 128: return launch_fwd_h<128, RB>(rec, out, B, blob, np, variant, num_cus, stream);
    case 256: return launch_fwd_h<256, RB>(rec, out, B, blob, np, variant, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_eta_mlp3_fwd(const void* rec, float* out, int B, const void* blob, int H,
                               const NormParams& np, int variant, int num_cus, hipStream_t stream,
                               int rec_bytes) {
  switch (rec_bytes) {
    case 16: return launch_fwd_rb<16>(rec, out, B, blob, H, np, variant, num_cus, stream);
    case 8: return launch_fwd_rb<8>(rec, out, B, blob, H, np, variant, num_cus, stream);
    case 6: return launch_fwd_rb<6>(rec, out, B, blob, H, np, variant, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

size_t eta_mlp3_blob_bytes(int H) { return mlp3_blob_bytes(H); }

hipError_t launch_eta_featurize(const void* rec, float* out, int B, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(eta_featurize_kernel, dim3((B + 255) / 256), dim3(256), 0, stream,
                     (const int4*)rec, out, B);
  return hipGetLastError();
}

}  // namespace rt
