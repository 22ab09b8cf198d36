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
    // next-row index formed only once tile + stride < ntiles: (tile + stride) * 32 < B + 32 then
    // cannot overflow int (bindings.cpp bounds B)
    if (tile + stride < ntiles) {
      const int nrow = (tile + stride) * 32 + r;
      if (nrow < B) rc_next = R::load(rec, nrow);
    }
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

// ---------------------------------------------------------------------------------------------
// 16x16 MFMA form of K1+K2 (variant 16/17: NH = 2/4 batch halves of 16 rows per wave-tile).
//
// Same math as eta_mlp3_fwd_kernel, on v_mfma_f32_16x16x32_bf16 (layer 2) and
// v_mfma_f32_16x16x16_bf16 (layer 1) instead of 32x32x16.  The reason is the clock, not the
// cycle count: under the MI355X power limit, 16x16x32 MFMA loops hold a ~12-15 % higher clock
// than 32x32x16 loops at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS item 7).
//   * layer 1: lane (j, kq) of the B operand holds features 4kq..4kq+3 of batch row j (the
//     (kq & 1) half of the 32x32 kernel's lane-half kq >> 1); D of hidden tile t gives lane
//     (j, g) hidden units 16t + 4g .. +3 of row j
//   * the layer-2 B fragment of k-chunk c is [relu(D_2c) | relu(D_2c+1)] in bf16 — no shuffles;
//     the host packs W2's columns in that (permuted) k order (ops/eta_mlp.py pack_mlp3_16)
//   * each W2 A fragment read from LDS feeds NH MFMAs (NH batch halves), so NH = 2 moves the
//     same LDS bytes per FLOP as the 32x32 kernel and NH = 4 half of them
// Blob16: [ w2p: (H/16)x(H/32)x64 lanes x 8 bf16 | w1p: (H/16)x64 lanes x 4 bf16 | b2 (H f32) |
//           w3 (H f32, target scale folded) | tail: b3, 0, 0, 0 |
//           w3f: (H/32)x64 lanes x 8 bf16 — w3 as the A operand of a layer-3 MFMA (EPI = 3) ]
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int H>
struct Mlp3Layout16 {
  static constexpr int MT = H / 16;   // 16-row hidden tiles
  static constexpr int KC = H / 32;   // 32-deep k chunks
  static constexpr size_t W2B = (size_t)H * H * 2;
  static constexpr size_t W1B = (size_t)H * 16 * 2;
  static constexpr size_t W3F = (size_t)H * 32;          // layer-3 A fragments (EPI = 3)
  static constexpr size_t BLOB = W2B + W1B + 2 * (size_t)H * 4 + 16 + W3F;
};

size_t eta_mlp3_blob16_bytes(int H) { return (size_t)2 * H * H + 72 * (size_t)H + 16; }

// (pairwise: a 4-wide convertvector lowers to 4 single-element v_cvt_pk_bf16_f32 + 2 v_perm_b32)
__device__ __forceinline__ bf16x4 relu_cvt_bf16x4(const f32x4 v) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const i16x2 z = {0, 0};
  const bf16x2 lo = __builtin_convertvector(__builtin_shufflevector(v, v, 0, 1), bf16x2);
  const bf16x2 hi = __builtin_convertvector(__builtin_shufflevector(v, v, 2, 3), bf16x2);
  const i16x2 rl = __builtin_elementwise_max(__builtin_bit_cast(i16x2, lo), z);
  const i16x2 rh = __builtin_elementwise_max(__builtin_bit_cast(i16x2, hi), z);
  return __builtin_bit_cast(bf16x4, __builtin_shufflevector(rl, rh, 0, 1, 2, 3));
}

template <int H, int NH, int RB, int TPB = 512, int EPI = 0>
__global__ __launch_bounds__(TPB, 1) void eta_mlp3_fwd16_kernel(const void* __restrict__ rec,
                                                                 float* __restrict__ out, int B,
                                                                 const unsigned char* __restrict__ blob,
                                                                 NormParams np) {
  using L = Mlp3Layout16<H>;
  constexpr int MT = L::MT, KC = L::KC, NF = MT * KC, D = KC < 4 ? KC : 4, ROWS = 16 * NH;
  static_assert(L::W1B >= D * 1024, "the ring's over-read must stay inside the blob");
  (void)NF;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  lds_fill_block(smem, blob, (int)L::BLOB);
  const bf16x8* w2p = reinterpret_cast<const bf16x8*>(smem);
  const i16x4* w1p = reinterpret_cast<const i16x4*>(smem + L::W2B);
  const float* b2 = reinterpret_cast<const float*>(smem + L::W2B + L::W1B);
  const float* w3 = b2 + H;
  const float b3 = w3[H];
  const bf16x8* w3f = reinterpret_cast<const bf16x8*>(smem + L::W2B + L::W1B + 8 * (size_t)H + 16);

  const int lane = threadIdx.x & 63;
  const int j = lane & 15;
  const int kq = lane >> 4;
  // layer-1 A fragments: kept in registers, or (NH = 4, where 4 halves of h1 already take
  // 128 VGPRs) re-read from LDS per use
  constexpr bool W1REG = NH < 4;
  i16x4 w1[W1REG ? MT : 1];
  if constexpr (W1REG) {
#pragma unroll
    for (int t = 0; t < MT; ++t) w1[t] = w1p[t * 64 + lane];
  }

  const int wpb = blockDim.x >> 6;
  const int ntiles = (B + ROWS - 1) / ROWS;
  const int stride = gridDim.x * wpb;
  using R = RecT<RB>;
  int tile = blockIdx.x * wpb + (threadIdx.x >> 6);
  typename R::T rc_next[NH];
#pragma unroll
  for (int n = 0; n < NH; ++n) {
    const int row = tile * ROWS + 16 * n + j;
    rc_next[n] = (tile < ntiles && row < B) ? R::load(rec, row) : R::zero();
  }
  for (; tile < ntiles; tile += stride) {
    bf16x8 h1[NH][KC];
#pragma unroll
    for (int n = 0; n < NH; ++n) {
      const typename R::T rc = rc_next[n];
      if (tile + stride < ntiles) {   // (tile + stride) * ROWS < B + ROWS: no int overflow
        const int nrow = (tile + stride) * ROWS + 16 * n + j;
        if (nrow < B) rc_next[n] = R::load(rec, nrow);
      }
      const bf16x8 f8 = R::feat(rc, kq >> 1, np);
      const i16x4 xb = (kq & 1) ? __builtin_bit_cast(i16x4, __builtin_shufflevector(f8, f8, 4, 5, 6, 7))
                                : __builtin_bit_cast(i16x4, __builtin_shufflevector(f8, f8, 0, 1, 2, 3));
      // layer 1 (bias folded into k = 14, 15)
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const i16x4 wa0 = W1REG ? w1[W1REG ? 2 * c : 0] : w1p[(2 * c) * 64 + lane];
        const i16x4 wa1 = W1REG ? w1[W1REG ? 2 * c + 1 : 0] : w1p[(2 * c + 1) * 64 + lane];
        const f32x4 d0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa0, xb, z, 0, 0, 0);
        const f32x4 d1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa1, xb, z, 0, 0, 0);
        const bf16x4 r0 = relu_cvt_bf16x4(d0), r1 = relu_cvt_bf16x4(d1);
        h1[n][c] = __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    // layer 2 + fused layer 3; A fragments through a 4-deep prefetch ring across tiles
    float ys[NH][2];
#pragma unroll
    for (int n = 0; n < NH; ++n) ys[n][0] = ys[n][1] = 0.f;
    const bf16x8* wa = w2p + lane;
    bf16x8 ring[D];
#pragma unroll
    for (int d = 0; d < D; ++d) ring[d] = wa[d * 64];
    // EPI = 0: relu + w3 dot on packed v_pk_fma_f32 after each hidden tile's MFMAs.
    // EPI = 1: the same on scalar v_fma_f32 (a packed f32 FMA beside MFMAs costs ~5x its issue
    //          slot, MI355X_MICROARCH.md "price of one filler").
    // EPI = 2: scalar, and software-pipelined: hidden tile t-1's relu/dot is interleaved one VALU
    //          per MFMA gap into tile t's MFMA chain instead of stalling on t's last MFMA.
    // EPI = 3: layer 3 on MFMA: relu(z2) of hidden tiles 2tp, 2tp+1 packed to bf16 (2 VALU per
    //          output pair) is the B operand (k = 32 units, the w2p k order) of one 16x16x32 MFMA
    //          whose A operand is w3 broadcast over the 16 rows (w3f); every lane then holds its
    //          row's y — no w3 FMAs and no cross-lane reduction.
    constexpr int NC = KC / D;            // prefetch chunks per hidden tile
    f32x4 accp[NH];
#pragma unroll
    for (int n = 0; n < NH; ++n) accp[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 w3p = {0.f, 0.f, 0.f, 0.f};
    f32x4 y3[EPI == 3 ? NH : 1];
    bf16x4 hprev[EPI == 3 ? NH : 1];
    if constexpr (EPI == 3) {
#pragma unroll
      for (int n = 0; n < NH; ++n) y3[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    auto epi = [&](const f32x4& a, const f32x4& w, float (&y)[2]) {
      y[0] = __builtin_fmaf(relu_f(a[0]), w[0], y[0]);
      y[1] = __builtin_fmaf(relu_f(a[1]), w[1], y[1]);
      y[0] = __builtin_fmaf(relu_f(a[2]), w[2], y[0]);
      y[1] = __builtin_fmaf(relu_f(a[3]), w[3], y[1]);
    };
    constexpr int TUNROLL = EPI == 3 ? 2 : 1;   // EPI 3: tile parity static in each copy
#pragma unroll TUNROLL
    for (int t = 0; t < MT; ++t) {
      const f32x4 bias = *reinterpret_cast<const f32x4*>(b2 + 16 * t + 4 * kq);
      f32x4 acc[NH];
#pragma unroll
      for (int n = 0; n < NH; ++n) acc[n] = bias;
      const int base = t * KC;
#pragma unroll
      for (int c = 0; c < KC; c += D) {
        bf16x8 a[D];
        const int nf = base + c + D;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          a[d] = ring[d];
          ring[d] = wa[(nf + d) * 64];   // past the last fragment: reads w1p (in the blob), unused
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
          for (int n = 0; n < NH; ++n)
            acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[d], h1[n][c + d], acc[n], 0, 0, 0);
        }
        if constexpr (EPI == 2) {
          // previous tile's epilogue for the halves assigned to this chunk (zeros at t = 0)
          int nv = 0;
#pragma unroll
          for (int n = 0; n < NH; ++n)
            if (n % NC == c / D) { epi(accp[n], w3p, ys[n]); nv += 8; }
          __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
#pragma unroll
          for (int i = 0; i < D * NH; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (i < nv) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
          }
        } else {
          __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, D * NH, 0);
        }
      }
      if constexpr (EPI == 3) {
        if (t & 1) {
          const bf16x8 wf = w3f[(t >> 1) * 64 + lane];
#pragma unroll
          for (int n = 0; n < NH; ++n) {
            const bf16x4 hc = relu_cvt_bf16x4(acc[n]);
            const bf16x8 hb = __builtin_shufflevector(hprev[n], hc, 0, 1, 2, 3, 4, 5, 6, 7);
            y3[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, hb, y3[n], 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int n = 0; n < NH; ++n) hprev[n] = relu_cvt_bf16x4(acc[n]);
        }
        continue;
      }
      const f32x4 w3v = *reinterpret_cast<const f32x4*>(w3 + 16 * t + 4 * kq);
      if constexpr (EPI == 2) {
#pragma unroll
        for (int n = 0; n < NH; ++n) accp[n] = acc[n];
        w3p = w3v;
      } else if constexpr (EPI == 1) {
#pragma unroll
        for (int n = 0; n < NH; ++n) epi(acc[n], w3v, ys[n]);
      } else {
        // relu + dot with w3 straight into packed per-lane partial sums (4 v_max + 2 v_pk_fma)
        const f32x2 w3lo = {w3v[0], w3v[1]}, w3hi = {w3v[2], w3v[3]};
#pragma unroll
        for (int n = 0; n < NH; ++n) {
          const f32x2 lo = {relu_f(acc[n][0]), relu_f(acc[n][1])};
          const f32x2 hi = {relu_f(acc[n][2]), relu_f(acc[n][3])};
          f32x2 y2 = {ys[n][0], ys[n][1]};
          y2 = __builtin_elementwise_fma(lo, w3lo, y2);
          y2 = __builtin_elementwise_fma(hi, w3hi, y2);
          ys[n][0] = y2[0];
          ys[n][1] = y2[1];
        }
      }
    }
    if constexpr (EPI == 2) {
#pragma unroll
      for (int n = 0; n < NH; ++n) epi(accp[n], w3p, ys[n]);
    }
    // after the two xor-reductions every lane holds the sums of its row j for all halves; lane
    // group kq stores half n = kq, so one store instruction writes the tile's 16*NH rows as one
    // contiguous run (256 B at NH = 4: full-size posted PCIe writes for zero-copy minutes out)
    float mine = 0.f;
#pragma unroll
    for (int n = 0; n < NH; ++n) {
      float y;
      if constexpr (EPI == 3) {
        y = y3[n][0];                    // C[m][row]: the same y in every m (w3 broadcast)
      } else {
        y = ys[n][0] + ys[n][1];
        y += __shfl_xor(y, 16);
        y += __shfl_xor(y, 32);
      }
      mine = (kq == n) ? y : mine;
    }
    const int row = tile * ROWS + 16 * kq + j;
    if (kq < NH && row < B) out[row] = mine + b3;
  }
}

template <int H, int NH, int RB, int TPB = 512, int EPI = 0>
static hipError_t launch_fwd16(const void* rec, float* out, int B, const void* blob,
                               const NormParams& np, int num_cus, hipStream_t stream) {
  using L = Mlp3Layout16<H>;
  static bool attr_set[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!attr_set[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)eta_mlp3_fwd16_kernel<H, NH, RB, TPB, EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::BLOB);
    if (e != hipSuccess) return e;
    attr_set[dev & 63] = true;
  }
  const int ntiles = (B + 16 * NH - 1) / (16 * NH);
  if (ntiles == 0) return hipSuccess;
  int grid = (ntiles + TPB / 64 - 1) / (TPB / 64);
  if (grid > num_cus) grid = num_cus;
  hipLaunchKernelGGL((eta_mlp3_fwd16_kernel<H, NH, RB, TPB, EPI>), dim3(grid), dim3(TPB), L::BLOB, stream,
                     rec, out, B, (const unsigned char*)blob, np);
  return hipGetLastError();
}

template <int H, int RB>
static hipError_t launch_fwd16_nh(const void* rec, float* out, int B, const void* blob,
                                  const NormParams& np, int nh, int num_cus, hipStream_t stream) {
  switch (nh) {
    case 1: return launch_fwd16<H, 1, RB>(rec, out, B, blob, np, num_cus, stream);
    case 2: return launch_fwd16<H, 2, RB>(rec, out, B, blob, np, num_cus, stream);
    case 4: return launch_fwd16<H, 4, RB>(rec, out, B, blob, np, num_cus, stream);
    case 3: return launch_fwd16<H, 2, RB, 768>(rec, out, B, blob, np, num_cus, stream);   // 2 halves, 12 waves
    case 5: return launch_fwd16<H, 4, RB, 512, 1>(rec, out, B, blob, np, num_cus, stream);  // scalar-FMA epilogue
    case 6: return launch_fwd16<H, 4, RB, 512, 2>(rec, out, B, blob, np, num_cus, stream);  // + pipelined
    case 7: return launch_fwd16<H, 2, RB, 512, 2>(rec, out, B, blob, np, num_cus, stream);
    case 8: return launch_fwd16<H, 4, RB, 512, 3>(rec, out, B, blob, np, num_cus, stream);  // layer 3 on MFMA
    default: return hipErrorInvalidValue;
  }
}

template <int RB>
static hipError_t launch_fwd16_rb(const void* rec, float* out, int B, const void* blob, int H,
                                  const NormParams& np, int nh, int num_cus, hipStream_t stream) {
  switch (H) {
    case 64: return launch_fwd16_nh<64, RB>(rec, out, B, blob, np, nh, num_cus, stream);
    case 128: return launch_fwd16_nh<128, RB>(rec, out, B, blob, np, nh, num_cus, stream);
    case 256: return launch_fwd16_nh<256, RB>(rec, out, B, blob, np, nh, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_eta_mlp3_fwd16(const void* rec, float* out, int B, const void* blob16, int H,
                                 const NormParams& np, int nh, int num_cus, hipStream_t stream,
                                 int rec_bytes) {
  switch (rec_bytes) {
    case 16: return launch_fwd16_rb<16>(rec, out, B, blob16, H, np, nh, num_cus, stream);
    case 8: return launch_fwd16_rb<8>(rec, out, B, blob16, H, np, nh, num_cus, stream);
    case 6: return launch_fwd16_rb<6>(rec, out, B, blob16, H, np, nh, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}


hipError_t launch_eta_featurize(const void* rec, float* out, int B, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(eta_featurize_kernel, dim3((B + 255) / 256), dim3(256), 0, stream,
                     (const int4*)rec, out, B);
  return hipGetLastError();
}

}  // namespace rt
