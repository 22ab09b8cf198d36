// K3: data-parallel training of the 3-layer ETA MLP on gfx950 — fused forward/loss kernel,
// ReLU backward, and fused AdamW + MFMA-fragment re-pack.  (The reference has no training code at
// all: notebooks/.gitkeep; its feature schema is RO/Flaskr/ml.py:35-51.)
//
// One training step on a rank (routest_amd/train/fused.py::FusedMlp3Trainer):
//   1. eta_mlp3_train_fwd_kernel: featurize + layer 1 + ONE pass over layer 2 + layer 3 + MSE
//      gradient.  Layers 1 and 2 stream over k with all hidden-tile accumulators live; relu(z2) is
//      kept packed to bf16 in registers, so the dW3 | db3 partial needs only an exact MFMA transpose
//      per hidden tile (no second layer-2 pass).  dL/dz2 = dy * w3 * relu'(z2) is formed in-register
//      once y (hence dy) is known.  Emits xf [B,16] (the exact bf16 features, slot 14 := 1), the dz2
//      tile images (512 B per row, [32 rows][H hperm columns] with a XOR chunk swizzle), the per-row
//      squared errors and one dW3 | db3 row per workgroup.  Records and targets of the next tile are
//      copied into LDS before the tile's stores (vmcnt is in order: a load issued after the stores
//      waits for all of them).
//   2. train_bwd_kernel: dgrad dh1 = dz2 W2 against an LDS image of W2 in B-fragment order,
//      relu'(z1) from h1 recomputed on the layer-1 MFMA, dW2 | db2 from the dz2 tile read transposed
//      (ds_read_b64_tr_b16) and dW1 — one kernel, split-K over the batch, then one deterministic
//      slab reduction (wgrad_reduce).  Nothing but dz2 and xf crosses HBM between the two kernels
//      (round 2 moved dz2^T + dh1^T, 1 KB per row, and ran the dgrad in the forward).
//   3. ONE flat fp32 gradient bucket -> one RCCL all-reduce over xGMI.
//   4. adamw_pack_kernel: AdamW on the flat fp32 master params, writing back the training blob the
//      next forward stages into LDS and the backward's W2 fragment image — no host work, no sync, so
//      the whole step is capturable in a HIP graph.
//
// Training blob (TrainLayout): [ w2img | w1p | b1p | b2p | w3p | tail | w2frag ] where w2img holds
// W2 row-major in 512-byte rows (natural unit order both ways) with 8-byte chunk k of row R at chunk
// k ^ w2swz(R): layer 2's A operand, lane (r, h) of tile (mt, ks) reads row 32mt + r, units
// 16ks + 4h .. +3 and 16ks + 8 + 4h .. +3 (the permuted k order of the h1 B fragments) with two
// ds_read_b64 — w2swz is a bijection of R mod 32, so a 32-lane half hits 64 distinct banks (bank rule,
// cdna_hip_programming.md §2 / MI355X_MICROARCH.md §LDS).  w1p .. tail is the inference layout
// (mlp3_tile.h); w2frag (w2frag_index) is the backward's B-fragment image, lane-linear per fragment.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lds_fill.h"
#include "mlp3_tile.h"
#include "ops.h"
#include "wgrad_reduce.h"

namespace rt {

// Stored hidden-unit order of the saved activations h1a / h2a / dz2 / dz1 (and of the gradient bucket
// built from them): element j of fragment ks on lane half h is hidden unit
// u = 16ks + 8(j>>2) + 4h + (j&3); storing it at column c = 16ks + 8h + j (= u with bits 2 and 3
// swapped, an involution) makes each lane's 8 values ONE contiguous 16-byte store instead of two
// 8-byte ones — the forward's activation writes went 42 -> 29 us at 65k rows.  adamw_pack_kernel
// reads the bucket through hperm() and train/fused.py::grads_from_bucket mirrors it.
__host__ __device__ __forceinline__ int hperm(int u) { return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1); }

template <int H>
struct TrainLayout {
  static constexpr int ROWB = 512;                       // bytes per W2 image row (256 slots)
  static constexpr size_t W2B = (size_t)H * ROWB;
  static constexpr size_t W1B = (size_t)H * 16 * 2;
  static constexpr size_t VB = (size_t)H * 4;
  static constexpr size_t BLOB = W2B + W1B + 3 * VB + 16;   // what the forward stages into LDS
  static constexpr size_t W2F = (size_t)H * H * 2;             // + train_bwd_kernel's W2 B fragments
};

size_t eta_mlp3_train_blob_bytes(int H) { return (size_t)H * 512 + 44 * (size_t)H + 16 + (size_t)H * H * 2; }

// W2 B-fragment image of train_bwd_kernel (past the forward's blob): fragment (nb, ks), lane
// (n, h), element j = W2[u2][u1] with u1 = 32nb + n and u2 = 16ks + 8(j>>2) + 4h + (j&3) — the k
// order of the forward's dz2 fragments.  Returns the bf16 index.
// XOR swizzle of the 16-byte chunks of row r in the dz2 tile image (512-byte rows at H = 256):
// 16 consecutive rows' chunk c land on 16 different bank groups (row reads) and the 4 rows x 64 bytes
// of a transposed read's 32-lane half on 16 different ones (cdna_hip_programming.md T10 (b))
__host__ __device__ __forceinline__ int dz2swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

__host__ __device__ __forceinline__ size_t w2frag_index(int u2, int u1, int KS) {
  const int nb = u1 >> 5, n = u1 & 31, ks = u2 >> 4, r = u2 & 15;
  const int hh = (r >> 2) & 1, j = 4 * (r >> 3) + (r & 3);
  return (((size_t)nb * KS + ks) * 64 + n + 32 * hh) * 8 + j;
}

__host__ __device__ __forceinline__ int w2swz(int row) { return ((row & 3) << 3) | ((row >> 2) & 7); }
// byte offset of W2[row][col] in the image (natural order both ways; 8-byte chunks swizzled)
__host__ __device__ __forceinline__ int w2off(int row, int col) {
  return row * 512 + (((col >> 2) ^ w2swz(row)) << 3) + 2 * (col & 3);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ bf16x8 join4(const s16x4 lo, const s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// 8 waves per workgroup, 2 per SIMD (<= 256 VGPRs each).
constexpr int TRAIN_TPB = 512;

template <int H>
__global__ __launch_bounds__(TRAIN_TPB, 1) void eta_mlp3_train_fwd_kernel(
    const int4* __restrict__ rec, const float* __restrict__ target, int B,
    const unsigned char* __restrict__ blob, NormParams np, float gscale, __bf16* __restrict__ xf,
    float* __restrict__ w3slab, bf16x8* __restrict__ dz2r, float* __restrict__ sq_err,
    int* __restrict__ step_ctr) {
  using L = TrainLayout<H>;
  constexpr int MT = H / 32, KS = H / 16, LDA = H + 16, D = KS < 4 ? KS : 4;
  // device-side optimizer step counter (read by adamw_pack_kernel later on the same stream), so a
  // captured HIP graph replays with correct bias corrections / LR schedule
  if (step_ctr != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *step_ctr += 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  lds_fill_block(smem, blob, (int)L::BLOB);
  // the W2 image as an absolute LDS address: dynamic LDS starts at 0 in this kernel (it has no
  // static __shared__ data), and a literal base lets every fragment read use its lane register as
  // the address with the rest in the instruction's offset field (through the extern array's base,
  // which is a link-time symbol, the compiler inserted a v_add of that base before each read)
  typedef __attribute__((address_space(3))) const unsigned char lds_u8;
  lds_u8* img = (lds_u8*)(uintptr_t)0;
  const bf16x8* w1p = reinterpret_cast<const bf16x8*>(smem + L::W2B);
  const f32x4* b2p = reinterpret_cast<const f32x4*>(smem + L::W2B + L::W1B) + H / 4;
  const f32x4* w3p = b2p + H / 4;

  const int lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int ntiles = (B + 31) >> 5;
  const int stride = gridDim.x * wpb;
  // this wave's dW3 | db3 partial accumulates in LDS past the blob (nothing carried in registers
  // across tiles): [wpb][LDA] f32, one row per wave until the final barrier
  float* const w3part = reinterpret_cast<float*>(smem + L::BLOB) + (threadIdx.x >> 6) * LDA;
  // per-wave 32-float scratch past the partials: the tile's dy values, broadcast to the lanes
  float* const dyscr = reinterpret_cast<float*>(smem + L::BLOB) + wpb * LDA + (threadIdx.x >> 6) * 32;
  for (int c = lane; c < LDA; c += 64) w3part[c] = 0.f;

  // The next tile's records and targets are copied into LDS (global_load_lds) at the top of the
  // current tile, BEFORE its stores, and read back after a counted wait: a register load issued after
  // the stores waits for all of them (vmcnt is in order), and a register prefetch carried across the
  // loop got a vmcnt(0) from the compiler at the loop head — either way the store latency was exposed
  // once per tile (PMC r3k2: waves waiting 53% of their cycles).  Per wave: [2][32] records (16 B) +
  // [2][32] targets past the dy scratch; zeroed first so rows past B only ever see finite values.
  typedef __attribute__((address_space(3))) void lds_void_t;
  unsigned char* const pfb = smem + L::BLOB + (size_t)wpb * (LDA + 32) * 4 + (size_t)(threadIdx.x >> 6) * 1280;
  for (int i = lane; i < 80; i += 64) reinterpret_cast<int4*>(pfb)[i] = make_int4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // the zeros land before any DMA write
  auto prefetch = [&](int t, int pb) {      // pb: buffer 0/1; all lanes call, lanes < 32 load
    const int rw = t * 32 + lane;
    if (lane < 32 && rw < B) {
      __builtin_amdgcn_global_load_lds((const void*)(rec + rw), (lds_void_t*)(pfb + pb * 512), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(target + rw), (lds_void_t*)(pfb + 1024 + pb * 128), 4, 0, 0);
    }
  };
  int pbuf = 0;
  {
    const int tile0 = blockIdx.x * wpb + (threadIdx.x >> 6);
    if (tile0 < ntiles) prefetch(tile0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  for (int tile = blockIdx.x * wpb + (threadIdx.x >> 6); tile < ntiles; tile += stride) {
    // nothing is hoisted out of the tile loop: the LDS-resident weights (W1 fragments, biases)
    // and the lane-derived LDS addresses are re-derived per tile.  Hoisted, they exceed the
    // 256-VGPR budget and get spilled, and a scratch reload issued after the activation stores
    // waits for all of them (vmcnt is in order) — which stalled every tile on its own stores.
    __asm__ volatile("" ::: "memory");
    int lv = lane;
    __asm__ volatile("" : "+v"(lv));
    const int r = lv & 31, h = lv >> 5;
    const int row = tile * 32 + r;
    const bool valid = row < B;
    // this tile's copy was issued at the top of the previous tile, followed by that tile's KS + 2
    // stores (the dz2 chunks, the xf row, the squared error: a tile always has a valid row 0).  The
    // LDS reads are inline asm: through plain loads the compiler adds its own vmcnt(0) for the DMA
    int4 rc;
    float tgt;
    {
      const unsigned a_rc = (unsigned)(uintptr_t)(pfb + pbuf * 512) + 16u * r;
      const unsigned a_tg = (unsigned)(uintptr_t)(pfb + 1024 + pbuf * 128) + 4u * r;
      asm volatile("s_waitcnt vmcnt(%2)\n\tds_read_b128 %0, %3\n\tds_read_b32 %1, %4\n\ts_waitcnt lgkmcnt(0)"
                   : "=&v"(rc), "=&v"(tgt) : "n"(KS + 2), "v"(a_rc), "v"(a_tg) : "memory");
    }
    if (tile + stride < ntiles) prefetch(tile + stride, pbuf ^ 1);
    pbuf ^= 1;
    const bf16x8 xb = featurize_bf16(rc, h, np);
    if (valid)  // slots 14, 15 hold 1.0 (the b1 hi/lo inputs): dW1k[:,14] == db1
      *reinterpret_cast<bf16x8*>(xf + (size_t)row * 16 + 8 * h) = xb;

    // layers 1 and 2 streamed over k: all MT layer-2 accumulators stay live (the MFMAs of one k-step
    // are MT independent chains), and layer-1 tile m1 is computed right before the two k-steps that
    // consume it, so only 2 h1 fragments are ever live (the round-2 order held all of h1: 64 VGPRs)
    f32x16 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = load_vec16(b2p, mt, h);
    {
      // W2 fragment addresses as lane bases + immediates (a run-time or fully hoisted w2off() per
      // fragment costs VGPRs the compiler then spills): chunk (2ks + h) ^ w2swz(r) only depends on
      // ks & 7, ks >> 3 adds 256 B
      const int sw = w2swz(r);
      lds_u8* lrow = img + r * 512;
      constexpr int NX = KS < 8 ? KS : 8;      // distinct ks & 7 patterns (ks >> 3 adds 256 B)
      int xk[NX][2];
#pragma unroll
      for (int k = 0; k < NX; ++k)
#pragma unroll
        for (int t = 0; t < 2; ++t) xk[k][t] = 8 * ((4 * k + 2 * t + h) ^ sw);
      // the ks >= 8 half gets its own (opaque) offsets: with pm + xk + 256 the compiler merges the
      // reads of ks and ks + 8 into one ds_read2_b64 (offsets 0 / 256 B), which conflicts with
      // itself — 7.5 bank-conflict cycles per instruction (tools/probes/lds_pattern_probe.hip);
      // two plain ds_read_b64 of the same swizzle are conflict-free
      int xk8[NX][2];
#pragma unroll
      for (int k = 0; k < NX; ++k)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          xk8[k][t] = xk[k][t] + 256;
          __asm__ volatile("" : "+v"(xk8[k][t]));
        }
      // per-hidden-tile row bases, opaque: with lrow + mt * 16384 visible the compiler paired the reads
      // of two hidden tiles into ds_read2st64_b64, which conflicts with itself (1.5 conflict cycles
      // per LDS instruction, PMC r3k2)
      lds_u8* pmv[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        uintptr_t v = (uintptr_t)(lrow + mt * 16384);
        __asm__ volatile("" : "+v"(v));
        pmv[mt] = (lds_u8*)v;
      }
      // units 16ks + 4h + 0..3 and 16ks + 8 + 4h + 0..3 of hidden tile mt: the permuted k order of h1
      auto frag = [&](int mt, int ks) {
        lds_u8* pm = pmv[mt];
        const int* xo = (ks >> 3) ? xk8[ks & 7] : xk[ks & 7];
        const s16x4 lo = *reinterpret_cast<const lds_s16x4*>(pm + xo[0]);
        const s16x4 hi = *reinterpret_cast<const lds_s16x4*>(pm + xo[1]);
        return join4(lo, hi);
      };
      f32x16 zero;
#pragma unroll
      for (int e = 0; e < 16; ++e) zero[e] = 0.f;
#pragma unroll
      for (int m1 = 0; m1 < MT; ++m1) {
        __asm__ volatile("" ::: "memory");     // one layer-1 tile's reads at a time
        const f32x16 z = mfma32(w1p[m1 * 64 + lane], xb, zero);
        float zf[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) zf[e] = z[e];
        bf16x8 hk[2];
        relu_cvt_bf16x8(zf, &hk[0]);
        relu_cvt_bf16x8(zf + 8, &hk[1]);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma32(frag(mt, 2 * m1 + s2), hk[s2], acc[mt]);
      }
    }
    // (h1 is not stored: train_bwd_kernel recomputes it from xf on the same MFMA)
    // y (hence dy), the relu'(z2) bits and relu(z2) itself packed to bf16 in registers (h2p, the
    // same k order as the dz2 fragments below); accumulator layout: units in registers, rows on lanes
    bf16x8 h2p[KS];
    unsigned long long mask_lo = 0, mask_hi = 0;   // 16 relu'(z2) bits per hidden tile
    float ys = 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const f32x16 w3 = load_vec16(w3p, mt, h);
      unsigned mk = 0;
      float a[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        ys = __builtin_fmaf(relu_f(acc[mt][e]), w3[e], ys);
        mk |= (acc[mt][e] > 0.f ? 1u : 0u) << e;
        a[e] = acc[mt][e];
      }
      relu_cvt_bf16x8(a, &h2p[2 * mt]);
      relu_cvt_bf16x8(a + 8, &h2p[2 * mt + 1]);
      if (mt < 4) mask_lo |= (unsigned long long)mk << (16 * mt);
      else mask_hi |= (unsigned long long)mk << (16 * (mt - 4));
    }
    const float b3 = reinterpret_cast<const float*>(w3p + H / 4)[0];   // (per tile: not held in a VGPR)
    ys += __shfl_xor(ys, 32);
    const float y = ys + b3;
    const float diff = valid ? (y - tgt) : 0.f;
    const float dy = gscale * diff;
    // per-row squared error (no cross-lane reduction: its shuffle addresses were the values the
    // compiler spilled)
    if (valid && h == 0) sq_err[row] = diff * diff;

    // dW3 | db3 partial sum_r dy_r relu(z2[r, c]) on the TRANSPOSED tile: relu(z2) is exactly
    // transposed by TWO MFMAs per hidden tile against a permuted identity (B[k][n] = 1 iff element k
    // of this lane half holds unit n; every product is x * 1), which puts hidden unit 32mt + n on the
    // lanes and the tile's rows 8(e>>2) + 4h + (e&3) in the registers — so the row sum is 16 in-lane
    // FMAs and ONE cross-half add per hidden tile.  (Round 2 recomputed z2^T with 128 more MFMAs per
    // tile because relu(z2) did not fit next to the dgrad's operands; the dgrad now runs in
    // train_bwd_kernel.)  The rows' dy reach the lanes through a 128-byte LDS broadcast.
    {
      float* const dys = dyscr;                      // this wave's 32-float scratch
      // (both lane halves hold row r's dy — y came through the cross-half add — so both store it: the
      // same value to the same slot, and no exec-mask branch)
      dys[r] = dy;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float dyv[16];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const f32x4 t = reinterpret_cast<const f32x4*>(dys)[2 * q4 + h];   // rows 8q4 + 4h .. +3
#pragma unroll
        for (int j = 0; j < 4; ++j) dyv[4 * q4 + j] = t[j];
      }
      bf16x8 eye0, eye1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int u0 = (j & 3) + 8 * (j >> 2) + 4 * h;          // unit offset of k = 8h + j, K-step 0
        eye0[j] = (__bf16)(u0 == r ? 1.f : 0.f);
        eye1[j] = (__bf16)(u0 + 16 == r ? 1.f : 0.f);
      }
      f32x16 zero;
#pragma unroll
      for (int e = 0; e < 16; ++e) zero[e] = 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f32x16 tt = mfma32(h2p[2 * mt], eye0, zero);
        tt = mfma32(h2p[2 * mt + 1], eye1, tt);
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) t = __builtin_fmaf(dyv[e], tt[e], t);
        t += __shfl_xor(t, 32);
        // (kept under the branch: written by both halves — same value, same slot — the kernel spilled)
        if (h == 0) w3part[hperm(32 * mt + r)] += t;
      }
      // db3 = sum of dy over the rows (lanes of half 0 hold each row once)
      float d = h == 0 ? dy : 0.f;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) d += __shfl_xor(d, o);
      if (lv == 0) w3part[H] += d;
    }

    // dz2 = dy * w3 * relu'(z2): fragment 2mt + s element j is accumulator register 8s + j of
    // hidden tile mt, i.e. hidden units 16ks + 8(j>>2) + 4h + (j&3) (ks = 2mt + s) — contiguous in the
    // hperm column order.  Stored as a row-major [32 rows][H hperm columns] tile image, one 16-byte
    // chunk per lane and fragment at chunk (2ks + h) ^ dz2swz(row): train_bwd_kernel copies the image
    // into LDS as it is and reads it both row-wise (ds_read_b128, the dgrad's A operand) and
    // transposed (ds_read_b64_tr_b16, dW2's A operand), conflict-free both ways.  Rows past B carry
    // dy = 0.
    {
      typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
      typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
      bf16x8* const out = dz2r + (size_t)tile * KS * 64 + r * (KS * 2);
      const int fz = dz2swz(r) & (2 * KS - 1);     // (within the row for H < 256)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f32x16 w3 = load_vec16(w3p, mt, h);
        const unsigned mk = (unsigned)((mt < 4 ? mask_lo >> (16 * mt) : mask_hi >> (16 * (mt - 4))) & 0xffffu);
        // per output pair: two products, one v_cvt_pk_bf16_f32, and the pair's two mask bits
        // sign-extended (v_bfe_i32) into a 0xFFFF / 0xFFFF0000 mask
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          u32x4v dw;
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) {
            const int b = 8 * s + 2 * q2;
            const f32x2 pr = {dy * w3[b], dy * w3[b + 1]};
            const unsigned cw = __builtin_bit_cast(unsigned, __builtin_convertvector(pr, bf16x2v));
            const unsigned lo = (unsigned)(((int)(mk << (31 - b))) >> 31);
            const unsigned hi = (unsigned)(((int)(mk << (30 - b))) >> 31);
            dw[q2] = cw & ((lo & 0xFFFFu) | (hi & 0xFFFF0000u));
          }
          out[(2 * (2 * mt + s) + h) ^ fz] = __builtin_bit_cast(bf16x8, dw);
        }
      }
    }
  }

  // workgroup dW3 | db3 partial: the waves' rows summed in wave order (deterministic), one fp32
  // row of w3slab per workgroup; wgrad_reduce sums the rows into the bucket
  __syncthreads();
  const float* part = reinterpret_cast<const float*>(smem + L::BLOB);
  for (int c = threadIdx.x; c < LDA; c += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < wpb; ++k) acc += part[k * LDA + c];
    w3slab[(size_t)blockIdx.x * LDA + c] = acc;
  }
}

// acc += a x b with the accumulator pinned to AGPRs.  train_bwd_kernel's 256 dW2 accumulators fill
// the AGPR file; through the builtin, the register allocator parked them in VGPRs and copied every
// tile in and out of AGPRs around each MFMA (32 v_accvgpr moves per MFMA pair).  Only other MFMAs
// of the same shape read these registers inside the loop (SrcC = the previous D: no wait states);
// the epilogue reads them after the loop has ended.
__device__ __forceinline__ void mfma32_acc(f32x16& acc, const bf16x8 a, const bf16x8 b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// the same with a VGPR accumulator (the dgrad's, which VALU reads after the loop: the reader must
// first pass mfma_drain, the hazard recognizer does not see inline asm)
__device__ __forceinline__ void mfma32_vacc(f32x16& acc, const bf16x8 a, const bf16x8 b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// 24 wait states after the last inline-asm MFMA that wrote x, y, before VALU reads them (an XDL write
// followed by a VALU read of the same VGPRs needs up to 18); the operands tie the order
__device__ __forceinline__ void mfma_drain(f32x16& x, f32x16& y) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(x), "+v"(y));
}

// ---------------------------------------------------------------------------------------------
// The whole backward below dz2 in ONE kernel: dh1 = dz2 W2 (dgrad), dz1 = dh1 * relu'(z1),
// dW2 | db2 = dz2^T [h1 | 1] and dW1 = dz1^T x, K = batch, split over k-slices (one workgroup per
// CU; slice s takes every S-th 32-row tile, newest first, so it starts on tiles the forward wrote
// last, still in the last-level cache).  Inputs per row: the forward's dz2 tile image (512 B) and the
// 32-byte feature row — half the bytes of the round-2 pair dz2^T + dh1^T, and the forward no longer
// runs the dgrad or any transpose.
//
// One wave per SIMD (4 waves at H = 256, 512 registers each); wave w owns the hidden units
// u1 = 64w .. 64w + 63 of h1 (two 32-unit n-blocks), so per 32-row tile it:
//   * recomputes h1^T for its two n-blocks on the layer-1 MFMA (x as A, the w1p fragment as B:
//     units on the lanes, rows in the registers = the dW2 B operand, and relu'(z1) in the layout
//     of its own dh1^T tile) — no redundant layer-1 work across waves;
//   * runs the dgrad with dz2 as the A operand (row reads of the tile image: rows on the lanes) and
//     W2's column block as B, read from an LDS image of W2 in B-fragment order (ds_read_b128,
//     conflict-free): D = dh1 with the units on the lanes and the rows in the registers, i.e. dh1^T
//     in the dW1 A layout;
//   * reads the same tile image transposed (ds_read_b64_tr_b16) as dz2^T, the dW2 A operand, and
//     accumulates dW2 for all 256 z2 units x its 64 h1 units: 16 accumulator tiles = 256 AGPRs,
//     resident for the whole slice (inline-asm MFMAs pin them; the builtin MFMAs beside them are
//     compiled in VGPR form, tools/build_ext.py MFMA_VGPR);
//   * transposes x once for dW1's B operand.
// 71 MFMAs per wave and tile, no LDS writes: the dz2 tile (16 KB) is double-buffered in LDS by
// global_load_lds issued one tile ahead through inline asm (issued with the builtin, the compiler's
// LDS-DMA tracking put a vmcnt(0) before the first read of the CURRENT tile and serialised the
// prefetch), x rows arrive by plain loads one tile ahead, and one barrier per tile separates the
// stages; within a tile the fragments of hidden tile mt + 1 are read while mt's 8 MFMAs (four
// interleaved accumulation chains) run.  LDS = W2 image (H*H*2 B) + two dz2 tiles (2 * H * 64 B):
// exactly 160 KB at H = 256.  Measured at 1M rows: 377 us (profiles/train_kernel_stats_1m_r3_v3.csv).
// Partial sums of slice s go to slab[s]: dW2 in the register-native layout (one 16-byte store per
// lane and 4 accumulator registers; wgrad.hip native_to_bucket), dW1 in the bucket layout (hperm
// rows, train/fused.py); wgrad_reduce sums them in a fixed order (deterministic) into the bucket.
// PROF (ROUTEST_TRAIN_BWD_PROF=1, diagnostics only; 2-6 also drop one part of the work: 2 the
// fragment prefetch, 3 the dgrad MFMAs, 4 the dW2 MFMAs, 5 the next tile's staging, 6 db2): s_memtime per tile segment — [0] the loop-top
// wait + barrier, [1] staging issue + layer 1, [2] the hidden-tile loop, [3] dW1 — summed per wave
// into prof[wave][4] (scalar registers: the timed code keeps its VGPR allocation)
//
// NBW = 1 (the column split, small batches): workgroups work in PAIRS on the same k-slice, each
// owning half of the h1 units (wave w of half c: n-block 4c + w), so a slice's dW2 | dW1 partial is
// written by two workgroups into disjoint parts of ONE slab — half the slabs (and half the slab
// bytes written here and read back by wgrad_reduce) for the same number of workgroups.  Each
// workgroup loads only its half of the W2 fragment image, the dgrad needs no cross-workgroup sum
// (an h1 unit's dh1 is a full K = H dot product over z2 units), and the two dgrad chains of the one
// n-block split k into even / odd steps.  The pair shares an XCD (blocks b and b + 8: round-robin
// XCD dispatch), so the second read of each dz2 tile hits that XCD's L2.
template <int H, int PROF = 0, int NBW = 2>
__global__ __launch_bounds__(H, 1) void train_bwd_kernel(
    const __bf16* __restrict__ xf, int B, const unsigned char* __restrict__ blob,
    const bf16x8* __restrict__ dz2r, float* __restrict__ slab2, float* __restrict__ slab1,
    unsigned long long* __restrict__ prof = nullptr) {
  unsigned long long pt[4] = {0, 0, 0, 0}, tprev = 0;
  auto mark = [&](int seg) {
    if constexpr (PROF) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (seg >= 0) pt[seg] += t - tprev;
      tprev = t;
    }
  };
  using L = TrainLayout<H>;
  constexpr int MT = H / 32, KS = H / 16, LDG = H + 16, RBF = KS * 64;
  typedef __attribute__((address_space(3))) void lds_void_t;
  typedef __attribute__((address_space(3))) const unsigned char lds_u8c;
  typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  static_assert(NBW == 1 || NBW == 2, "n-blocks per wave");
  constexpr int NW = H / 64, NBL = NW * NBW;                 // waves; n-blocks of this workgroup
  bf16x8* const w2s = reinterpret_cast<bf16x8*>(smem);      // [NBL][KS][64] B fragments
  bf16x8* const rb = w2s + NBL * RBF;                        // [2][KS][64] dz2 fragments
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 31, h = lane >> 5;
  const int nw = NW;
  const int wsc = __builtin_amdgcn_readfirstlane(w);
  const int ntiles = (B + 31) >> 5;
  // the k-slice of this workgroup and its half (NBW = 1: blocks b and b + 8 form a pair)
  const int bid = (int)blockIdx.x;
  const int half = NBW == 2 ? 0 : (bid >> 3) & 1;
  const int slice = NBW == 2 ? bid : ((bid & 7) | ((bid >> 4) << 3));
  const int nb0 = (half * NW + wsc) * NBW;                    // this wave's first n-block (global)
  // slice s takes tiles s, s + S, s + 2S, ... in DESCENDING order: the forward wrote the tiles in
  // rounds of increasing index, so every slice starts on the most recently written tiles, which are
  // still in the 256 MB last-level cache, instead of half the slices streaming the oldest from HBM
  const int S = NBW == 2 ? (int)gridDim.x : (int)gridDim.x >> 1;
  const int nmine = slice < ntiles ? (ntiles - 1 - slice) / S + 1 : 0;
  auto tile_at = [&](int i) { return slice + (nmine - 1 - i) * S; };
  const int t0 = 0, t1 = nmine;                              // loop positions

  // the W2 B-fragment image (kept by adamw_pack_kernel past the forward's blob) into LDS, and the
  // first dz2 tile behind it
  const unsigned char* w2g = blob + L::BLOB + (size_t)half * NBL * KS * 1024;   // this half's blocks
  for (int c = w; c < NBL * KS; c += nw)
    __builtin_amdgcn_global_load_lds((const void*)(w2g + (size_t)c * 1024 + 16 * lane),
                                     (lds_void_t*)(w2s + c * 64), 16, 0, 0);
  // the per-tile dz2 copy is issued through inline asm: issued with the builtin, the compiler tracks
  // it as a pending LDS write and put a vmcnt(0) before the first LDS read of the CURRENT tile — the
  // next tile's copy was then waited for right after it was issued (the loop-top vmcnt(0) + barrier
  // is what orders it)
  auto stage = [&](int tile, int buf) {
    const bf16x8* src = dz2r + (size_t)tile * RBF;
    for (int c = w; c < KS; c += nw) {
      const unsigned ldst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(rb + buf * RBF + c * 64));
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src + c * 64 + lane), "s"(ldst) : "memory");
    }
  };
  const bf16x8* xg = reinterpret_cast<const bf16x8*>(xf);    // row r, half h = chunk 2r + h
  bf16x8 xn;
  if (t0 < t1) {
    stage(tile_at(t0), 0);
    xn = xg[(size_t)tile_at(t0) * 64 + 2 * col + h];
  }
  const bf16x8* w1p = reinterpret_cast<const bf16x8*>(blob + L::W2B);
  // this wave's W2 B-fragment blocks in the LDS image (absolute addresses: lane base + immediates)
  unsigned wb0[NBW];
  bf16x8 w1f[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    wb0[i] = (unsigned)(((w * NBW + i) * KS * 64 + lane) * 16);
    w1f[i] = w1p[(nb0 + i) * 64 + lane];
  }
  bf16x8 eye;
#pragma unroll
  for (int j = 0; j < 8; ++j) eye[j] = (__bf16)(8 * h + j == col ? 1.f : 0.f);   // x^T: B (k = 8h + j, n = col)
  // Addresses into a dz2 tile image ([32 rows][2KS chunks of 16 B], chunk c of row r at
  // c ^ dz2swz(r)): the swizzled fields and the compile-time parts occupy disjoint bits, so every read
  // is ONE lane base XOR a constant (checked exhaustively for H = 64/128/256 on the host):
  //   row read of k-step ks (the dgrad's A operand, chunk 2ks + h of row col):
  //       R0 ^ (32 (ks & 7) + 256 (ks >> 3))
  //   transposed read t of k-step s2 of hidden tile mt (dW2's A operand: rows 16s2 + 8t + 4(lane>>5)
  //   + 0..3, image columns 32mt + 16((lane>>4)&1) + 0..15):
  //       C0 ^ (64 (mt & 3) + 32 t + 8t RB2 + 256 (mt >> 2) + 16 RB2 s2)
  // and the buffer's base is OR-ed in (its bits lie above).  Two VGPRs instead of a 16-entry table.
  constexpr int RB2 = 2 * KS * 16;                          // bytes per image row
  constexpr int CM = 2 * KS - 1;                            // chunk mask (H < 256: fewer chunks)
  const unsigned R0 = col * RB2 + 16 * ((h ^ dz2swz(col)) & CM);
  unsigned C0;
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int row = 4 * (g >> 1) + q, chunk = 2 * (g & 1) + (p >> 1);
    C0 = row * RB2 + 16 * ((chunk ^ dz2swz(row)) & CM) + 8 * (p & 1);
  }
  f32x16 acc2[MT][NBW], acc1[NBW], zero;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    zero[e] = 0.f;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      acc1[i][e] = 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc2[mt][i][e] = 0.f;
    }
  }
  float db2[NBW];                      // sums of dz2 over the rows, units 32(nb0 + i) + col
#pragma unroll
  for (int i = 0; i < NBW; ++i) db2[i] = 0.f;
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  auto pack = [](const f32x16& v, int s, bool relu) {
    u32x4v o;
#pragma unroll
    for (int q2 = 0; q2 < 4; ++q2) {
      float x0 = v[8 * s + 2 * q2], x1 = v[8 * s + 2 * q2 + 1];
      if (relu) {
        x0 = relu_f(x0);
        x1 = relu_f(x1);
      }
      const f32x2 pr = {x0, x1};
      o[q2] = __builtin_bit_cast(unsigned, __builtin_convertvector(pr, bf16x2v));
    }
    return __builtin_bit_cast(bf16x8, o);
  };

  for (int it = t0; it < t1; ++it) {
    const int buf = (it - t0) & 1;
    mark(-1);
    // this wave's share of the tile (and, on the first pass, of the W2 image) has landed; after the
    // barrier every wave's share has, and every wave has finished reading the other buffer
    // (xn passes through the wait as an asm operand: read as a plain load result, the compiler put a
    // vmcnt(0) after the NEXT tile's loads below and serialised the whole prefetch)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(xn) :: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    mark(0);
    const bf16x8 x = xn;
    if (it + 1 < t1 && PROF != 5) {      // (PROF 5, diagnostics: no next-tile staging in flight)
      stage(tile_at(it + 1), buf ^ 1);
      xn = xg[(size_t)tile_at(it + 1) * 64 + 2 * col + h];
    }
    // the tile image as an absolute LDS address (dynamic LDS starts at 0: no static __shared__ here),
    // so every read is a lane base + an immediate offset
    // layer 1 for the two n-blocks: h1^T (units on the lanes, rows in the registers)
    bf16x8 h1t[NBW][2];
    // (relu on the packed bf16 pairs, v_pk_max_i16 — and relu'(z1) is read back off the same packed
    // values below: one wave per SIMD issues VALU at 4 cycles, and the per-element compare/select
    // mask this replaces was ~150 VALU per tile)
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const f32x16 hz = mfma32(x, w1f[i], zero);
      float zf[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) zf[e] = hz[e];
      relu_cvt_bf16x8(zf, &h1t[i][0]);
      relu_cvt_bf16x8(zf + 8, &h1t[i][1]);
    }
    f32x16 accd[2] = {zero, zero};
    mark(1);
    // dz2 fragments of hidden tile mt — the dgrad's row-read pair and dW2's two transposed k-steps —
    // are read one hidden tile ahead, the tile's 4 W2 B fragments at its start (the dW2 MFMAs run
    // while they arrive).  The bases pass through an empty asm per hidden tile, so the XORs are
    // formed where they are used instead of all being hoisted into live registers, and the memory
    // clobber keeps later tiles' reads from being hoisted to the top (both spilled).
    const unsigned tb0 = (unsigned)(NBL * RBF * 16 + buf * RBF * 16);
    unsigned rbase = tb0 | R0, tbase = tb0 | C0;
    struct AFrags {
      bf16x8 a0, a1, t[2];
    };
    auto lda = [&](int mt) {
      AFrags f;
      f.a0 = *(const lds_bf16x8*)(uintptr_t)(rbase ^ (32u * ((2 * mt) & 7) + 256u * ((2 * mt) >> 3)));
      f.a1 = *(const lds_bf16x8*)(uintptr_t)(rbase ^ (32u * ((2 * mt + 1) & 7) + 256u * ((2 * mt + 1) >> 3)));
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const unsigned k0 = 64u * (mt & 3) + 256u * (mt >> 2) + 16u * RB2 * s2;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(tbase ^ k0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(tbase ^ (k0 + 32u + 8u * RB2)));
        f.t[s2] = join4(lo, hi);
      }
      return f;
    };
    auto ldw = [&](int mt, bf16x8 (&wv)[NBW][2]) {
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        const lds_u8c* wf = (const lds_u8c*)(uintptr_t)(wb0[i] + 2048u * mt);
        wv[i][0] = *reinterpret_cast<const lds_bf16x8*>(wf);
        wv[i][1] = *reinterpret_cast<const lds_bf16x8*>(wf + 1024);
      }
    };
    AFrags cur = lda(0);
    bf16x8 wc[NBW][2];
    ldw(0, wc);
    // VALU-written MFMA operands (h1t, the zeroed accd) get their wait states before the first
    // inline-asm MFMA reads them
    if constexpr (NBW == 2)
      asm volatile("s_nop 4" : "+v"(h1t[0][0]), "+v"(h1t[0][1]), "+v"(h1t[1][0]), "+v"(h1t[1][1]),
                   "+v"(accd[0]), "+v"(accd[1]));
    else
      asm volatile("s_nop 4" : "+v"(h1t[0][0]), "+v"(h1t[0][1]), "+v"(accd[0]), "+v"(accd[1]));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      asm volatile("" : "+v"(rbase), "+v"(tbase));
      AFrags nxt = cur;
      bf16x8 wn[NBW][2];
      if (mt + 1 < MT && PROF != 2) {
        nxt = lda(mt + 1);
        ldw(mt + 1, wn);
      }
      asm volatile("" ::: "memory");
      // four independent accumulation chains interleaved (a dependent MFMA waits for its
      // predecessor's result): dW2 = dz2^T (lane m: the unit in image column 32mt + m, rows in the k
      // order of h1t) x h1^T, and the dgrad dh1^T(u1 block) += dz2 (rows on lanes) x W2[:, block]
      if constexpr (NBW == 2) {
        if (PROF != 4) {
          mfma32_acc(acc2[mt][0], cur.t[0], h1t[0][0]);
          mfma32_acc(acc2[mt][1], cur.t[0], h1t[1][0]);
        }
        if (PROF != 3) {
          mfma32_vacc(accd[0], cur.a0, wc[0][0]);
          mfma32_vacc(accd[1], cur.a0, wc[1][0]);
        }
        if (PROF != 4) {
          mfma32_acc(acc2[mt][0], cur.t[1], h1t[0][1]);
          mfma32_acc(acc2[mt][1], cur.t[1], h1t[1][1]);
        }
        if (PROF != 3) {
          mfma32_vacc(accd[0], cur.a1, wc[0][1]);
          mfma32_vacc(accd[1], cur.a1, wc[1][1]);
        }
      } else {
        // one n-block: the dgrad's k-steps alternate between two chains (summed after the loop), so
        // dependent MFMAs stay three or four issues apart
        mfma32_acc(acc2[mt][0], cur.t[0], h1t[0][0]);
        mfma32_vacc(accd[0], cur.a0, wc[0][0]);
        mfma32_vacc(accd[1], cur.a1, wc[0][1]);
        mfma32_acc(acc2[mt][0], cur.t[1], h1t[0][1]);
      }
      // db2 of this wave's own two z2 tiles (row sums of dz2^T): the wave index through readfirstlane
      // makes this a scalar branch (an exec-mask one through threadIdx; hidden-tile loop 4129 -> 4044
      // cycles per 32-row tile, profiles/train_bwd_segments_r4.md).  Computing it at every hidden tile
      // and selecting measured slower (4562); summing the pairs with v_dot2_f32_bf16 against (1, 1)
      // was faster (3937) but did not reproduce these sums (db2 off by 13-54 %, r4an) and is not used.
      if (mt / NBW == half * NW + wsc && PROF != 6) {      // (PROF 6, diagnostics: no db2 block)
        const u32x4v q0 = __builtin_bit_cast(u32x4v, cur.t[0]), q1 = __builtin_bit_cast(u32x4v, cur.t[1]);
        float sacc = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sacc += __uint_as_float(q0[q] << 16) + __uint_as_float(q0[q] & 0xFFFF0000u);
          sacc += __uint_as_float(q1[q] << 16) + __uint_as_float(q1[q] & 0xFFFF0000u);
        }
        db2[mt % NBW] += sacc;
      }
      if (PROF != 2) cur = nxt;
      if (mt + 1 < MT && PROF != 2) {
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
          wc[i][0] = wn[i][0];
          wc[i][1] = wn[i][1];
        }
      }
    }
    mfma_drain(accd[0], accd[1]);
    if constexpr (NBW == 1) {
#pragma unroll
      for (int e = 0; e < 16; ++e) accd[0][e] += accd[1][e];
    }
    mark(2);
    // dW1 += (dh1 * relu'(z1))^T x: x^T as the B operand (features on the lanes)
    const f32x16 xt = mfma32(x, eye, zero);
    const bf16x8 xb0 = pack(xt, 0, false), xb1 = pack(xt, 1, false);
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      // dz1 = dh1 * relu'(z1): a bf16 half survives where h1 = relu(z1) is nonzero.  Per packed pair
      // (h1 halves in [0, 0x7F80]): x = (w + 0x7FFF7FFF) & 0x80008000 flags the nonzero halves (no
      // carry crosses a half) and (x << 1) - (x >> 15) widens each flag to 0xFFFF
      u32x4v g0 = __builtin_bit_cast(u32x4v, pack(accd[i], 0, false));
      u32x4v g1 = __builtin_bit_cast(u32x4v, pack(accd[i], 1, false));
      const u32x4v hw0 = __builtin_bit_cast(u32x4v, h1t[i][0]), hw1 = __builtin_bit_cast(u32x4v, h1t[i][1]);
      auto nzmask = [](unsigned wv) {
        const unsigned xv = (wv + 0x7FFF7FFFu) & 0x80008000u;
        return (xv << 1) - (xv >> 15);
      };
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2) {
        g0[q2] &= nzmask(hw0[q2]);
        g1[q2] &= nzmask(hw1[q2]);
      }
      acc1[i] = mfma32(__builtin_bit_cast(bf16x8, g0), xb0, acc1[i]);
      acc1[i] = mfma32(__builtin_bit_cast(bf16x8, g1), xb1, acc1[i]);
    }
    if constexpr (PROF) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      mark(3);
    }
  }
  if constexpr (PROF) {
    if (lane == 0 && prof != nullptr)
      for (int k = 0; k < 4; ++k) prof[((size_t)bid * nw + w) * 4 + k] = pt[k];
  }
  // the last dW2 MFMAs were issued through inline asm, which the hazard recognizer does not see: give
  // them their 16 passes before the epilogue reads the accumulators
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  // dW2 partial in the REGISTER-NATIVE slab layout (train_slab2_index; wgrad_reduce maps it to the
  // bucket): accumulator tile (w, i, mt) is 1024 contiguous floats, registers 4q .. 4q+3 of lane l at
  // q*256 + 4l — one 16-byte store per lane and 4 registers, 1 KB per wave-instruction.  (Stored in
  // the bucket's [row][hperm col] order, the same partial took 4x the store instructions: one dword
  // per lane, 256 per wave, an issue-bound tail of ~256 KB per workgroup after the last tile.)
  float* o2 = slab2 + (size_t)slice * H * LDG;
  float* o1 = slab1 + (size_t)slice * H * 16;
#pragma unroll
  for (int i = 0; i < NBW; ++i)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f32x4* t = reinterpret_cast<f32x4*>(o2 + (size_t)(((nb0 + i) * MT + mt) * 1024)) + lane;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        t[64 * q] = (f32x4){acc2[mt][i][4 * q], acc2[mt][i][4 * q + 1], acc2[mt][i][4 * q + 2], acc2[mt][i][4 * q + 3]};
    }
  // D[m][n] of dW1: lane -> n = col, register e -> m = (e&3) + 8(e>>2) + 4h, rows in hperm order
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int mo = (e & 3) + 8 * (e >> 2) + 4 * h;
#pragma unroll
    for (int i = 0; i < NBW; ++i)
      if (col < 16) o1[(size_t)hperm(32 * (nb0 + i) + mo) * 16 + col] = acc1[i][e];
  }
  // db2 column (and the zero columns H+1 .. H+15) past the H*H native block, [bucket row][16]: both
  // lane halves hold rows of image column 32(nb0+i) + col (image column = bucket row)
  float* oc = o2 + (size_t)H * H;
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const float d = db2[i] + __shfl_xor(db2[i], 32);
    const int ur = 32 * (nb0 + i) + col;
    if (h == 0) oc[(size_t)ur * 16] = d;
    else
#pragma unroll
      for (int c = 1; c < 16; ++c) oc[(size_t)ur * 16 + c] = 0.f;
  }
}

// Flat parameter layout (fp32 master): W1[H][12] | b1[H] | W2[H][H] | b2[H] | w3[H] | b3
// Flat gradient bucket:                gW2a[H][H+16] | gW3a[H+16] | gW1a[H][16]
struct AdamWArgs {
  float lr, beta1, beta2, eps, wd;
  int warmup, total_steps;  // linear warmup then cosine decay to min_lr_ratio * lr (total > 0)
  float min_lr_ratio;
  int update;  // 0: only (re)pack the blob from P
};

__device__ __forceinline__ float sched_lr(const AdamWArgs& a, int t) {
  float lr = a.lr;
  if (a.warmup > 0 && t < a.warmup) lr *= (float)t / (float)a.warmup;
  if (a.total_steps > 0) {
    const float prog = fminf(1.f, (float)(t - a.warmup) / fmaxf(1.f, (float)(a.total_steps - a.warmup)));
    if (t > a.warmup)
      lr *= a.min_lr_ratio + (1.f - a.min_lr_ratio) * 0.5f * (1.f + cosf(3.14159265f * prog));
  }
  return lr;
}

// AdamW on one master parameter e (flat P order: W1 | b1 | W2 | b2 | W3 | b3; o / i its row /
// column) with gradient g, then its bf16 / f32 copies in the training blob (the forward's LDS image
// and the backward's W2 fragment image).  Shared by adamw_pack_kernel and the one-rank fused
// reduce + AdamW (reduce_adamw_kernel): the same fp32 operations in the same order.
template <int H>
__device__ __forceinline__ void adamw_param(int e, float g, bool decay, int o, int i, float* __restrict__ P,
                                            float* __restrict__ M, float* __restrict__ V,
                                            unsigned char* __restrict__ blob, const int* __restrict__ step,
                                            const AdamWArgs& a) {
  using L = TrainLayout<H>;
  constexpr int OFF_B1 = 12 * H, OFF_W2 = 13 * H, OFF_B2 = 13 * H + H * H, OFF_W3 = OFF_B2 + H,
                OFF_B3 = OFF_W3 + H;
  unsigned char* w2img = blob;
  __bf16* w1p = reinterpret_cast<__bf16*>(blob + L::W2B);
  float* b1p = reinterpret_cast<float*>(blob + L::W2B + L::W1B);
  float* b2p = b1p + H;
  float* w3p = b2p + H;
  float* tail = w3p + H;
  float p = P[e];
  if (a.update) {
    const int t = *step > 0 ? *step : 1;
    const float lr = sched_lr(a, t);
    const float bc1 = 1.f - powf(a.beta1, (float)t);
    const float bc2 = 1.f - powf(a.beta2, (float)t);
    if (decay) p -= lr * a.wd * p;
    const float m = a.beta1 * M[e] + (1.f - a.beta1) * g;
    const float v = a.beta2 * V[e] + (1.f - a.beta2) * g * g;
    M[e] = m;
    V[e] = v;
    p -= lr * (m / bc1) / (sqrtf(v / bc2) + a.eps);
    P[e] = p;
  }
  // ---- re-pack into the MFMA fragment blob ----
  if (e < OFF_B1) {
    const int mt = o >> 5, rr = o & 31;
    auto put = [&](int kappa) {
      const int ln = rr + 32 * (kappa >> 3);
      w1p[((size_t)(mt * 64 + ln)) * 8 + (kappa & 7)] = (__bf16)p;
    };
    put(i);
    if (i == 10) put(12);
    if (i == 11) put(13);
  } else if (e >= OFF_W2 && e < OFF_B2) {
    *reinterpret_cast<__bf16*>(w2img + w2off(o, i)) = (__bf16)p;   // natural order, swizzled chunks
    reinterpret_cast<__bf16*>(blob + L::BLOB)[w2frag_index(o, i, H / 16)] = (__bf16)p;
  } else if (e < OFF_B3) {
    const int mt = o >> 5, rr = o & 31;
    const int hh = (rr >> 2) & 1;
    const int ii = (rr & 3) + 4 * (rr >> 3);
    const int idx = (mt * 2 + hh) * 16 + ii;
    if (e < OFF_W2) {
      b1p[idx] = p;
      const __bf16 hi = (__bf16)p;
      const int ln = rr;  // k = 14, 15 live in lane half 1: lane = rr + 32
      w1p[((size_t)(mt * 64 + ln + 32)) * 8 + 6] = hi;
      w1p[((size_t)(mt * 64 + ln + 32)) * 8 + 7] = (__bf16)(p - (float)hi);
    } else if (e < OFF_W3) b2p[idx] = p;
    else w3p[idx] = p;
  } else {
    tail[0] = p;
  }
}

template <int H>
__global__ __launch_bounds__(256) void adamw_pack_kernel(float* __restrict__ P,
                                                         const float* __restrict__ G,
                                                         float* __restrict__ M, float* __restrict__ V,
                                                         unsigned char* __restrict__ blob,
                                                         const int* __restrict__ step, AdamWArgs a) {
  constexpr int OFF_B1 = 12 * H, OFF_W2 = 13 * H, OFF_B2 = 13 * H + H * H, OFF_W3 = OFF_B2 + H,
                OFF_B3 = OFF_W3 + H, N = OFF_B3 + 1;
  constexpr int LDG = H + 16;
  const float* gW2a = G;
  const float* gW3a = G + H * LDG;
  const float* gW1a = gW3a + LDG;

  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  float g = 0.f;
  bool decay = false;
  int o = 0, i = 0;
  if (e < OFF_B1) {
    o = e / 12;
    i = e - o * 12;
    g = gW1a[hperm(o) * 16 + i];          // dW1 rows at hperm positions (dz1 is stored so)
    if (i == 10) g += gW1a[hperm(o) * 16 + 12];
    if (i == 11) g += gW1a[hperm(o) * 16 + 13];
    decay = true;
  } else if (e < OFF_W2) {
    o = e - OFF_B1;
    g = gW1a[hperm(o) * 16 + 14];
  } else if (e < OFF_B2) {
    const int k = e - OFF_W2;
    o = k / H;
    i = k - o * H;
    g = gW2a[hperm(o) * LDG + hperm(i)];
    decay = true;
  } else if (e < OFF_W3) {
    o = e - OFF_B2;
    g = gW2a[hperm(o) * LDG + H];
  } else if (e < OFF_B3) {
    o = e - OFF_W3;
    g = gW3a[hperm(o)];
    decay = true;
  } else {
    g = gW3a[H];
  }
  adamw_param<H>(e, g, decay, o, i, P, M, V, blob, step, a);
}

// One-rank step tail: the slab reduction of wgrad_reduce (three segments: the register-native dW2|db2
// slabs -> gW2a, the dW1 slabs -> gW1a, the forward's dW3|db3 rows -> gW3a) and AdamW + re-pack of
// the parameters whose gradients the workgroup just summed, in one launch instead of two (the
// 64k-row step's 7.7 + 5.1 us, profiles/train_kernel_stats_64k_r5o.csv).  Only without gradient
// communication: an all-reduce must see the whole bucket first.  G is still written (checkpoints,
// tests, gradient norms read it).  The sums and the AdamW arithmetic are those of wgrad_reduce_kernel
// and adamw_pack_kernel, so both paths produce the same bits (tests/test_train_gpu.py).
template <int H>
__global__ __launch_bounds__(256) void reduce_adamw_kernel(RedSeg s0, RedSeg s1, RedSeg s2, int nb0, int nb01,
                                                           float* __restrict__ P, float* __restrict__ M,
                                                           float* __restrict__ V, unsigned char* __restrict__ blob,
                                                           const int* __restrict__ step, AdamWArgs a) {
  constexpr int OFF_B1 = 12 * H, OFF_W2 = 13 * H, OFF_B2 = 13 * H + H * H, OFF_W3 = OFF_B2 + H,
                OFF_B3 = OFF_W3 + H;
  constexpr int LDG = H + 16;
  const int bx = (int)blockIdx.x;
  const int seg = bx < nb0 ? 0 : (bx < nb01 ? 1 : 2);
  const RedSeg sg = seg == 0 ? s0 : (seg == 1 ? s1 : s2);
  const int blk = bx - (seg == 0 ? 0 : (seg == 1 ? nb0 : nb01));
  __shared__ RedPart part;
  __shared__ float sum[RED_COLS * 4];
  const float4 r = red_sum<false>(sg, blk, part);
  const int c = threadIdx.x & (RED_COLS - 1), sl = threadIdx.x / RED_COLS;
  if (sl == 0) {
    sum[4 * c] = r.x;
    sum[4 * c + 1] = r.y;
    sum[4 * c + 2] = r.z;
    sum[4 * c + 3] = r.w;
  }
  __syncthreads();
  // thread t < 64: bucket value t of the workgroup (slab element blk * 64 + t)
  const int t = threadIdx.x;
  const int x = blk * (RED_COLS * 4) + t;
  if (t >= RED_COLS * 4 || x >= sg.n) return;
  const float g = sum[t];
  int gi;
  if (seg == 0) {
    int g0, st;
    native_to_bucket(x & ~3, H, g0, st);
    gi = g0 + (x & 3) * st;
  } else {
    gi = x;
  }
  sg.G[gi] = g;
  int e = -1, o = 0, i = 0;
  bool decay = false;
  float gg = g;
  if (seg == 0) {                    // gW2a [H][LDG]: row hperm(o), column hperm(i) | H (db2) | zero pad
    const int row = gi / LDG, col = gi - row * LDG;
    o = red_hperm(row);
    if (col < H) {
      i = red_hperm(col);
      e = OFF_W2 + o * H + i;
      decay = true;
    } else if (col == H) {
      e = OFF_B2 + o;
    }
  } else if (seg == 1) {             // gW1a [H][16]: row hperm(o); cols 0..11 W1 (10 += 12, 11 += 13), 14 b1
    const int row = x >> 4, col = x & 15;
    o = red_hperm(row);
    if (col < 12) {
      i = col;
      e = o * 12 + col;
      if (col >= 10) gg = g + sum[t + 2];     // the same add as adamw_pack_kernel
      decay = true;
    } else if (col == 14) {
      e = OFF_B1 + o;
    }
  } else {                           // gW3a [LDG]: hperm(o) | H (db3)
    if (x < H) {
      o = red_hperm(x);
      e = OFF_W3 + o;
      decay = true;
    } else if (x == H) {
      e = OFF_B3;
    }
  }
  if (e >= 0) adamw_param<H>(e, gg, decay, o, i, P, M, V, blob, step, a);
}

// workgroups of the training forward (= rows of its dW3 slab): one per 8 row tiles, at most one
// per CU (the blob fills the LDS)
int train_fwd_grid(int B, int num_cus) {
  const int ntiles = (B + 31) / 32;
  const int g = (ntiles + TRAIN_TPB / 64 - 1) / (TRAIN_TPB / 64);
  return g < num_cus ? g : num_cus;
}

template <int H>
static hipError_t launch_train_fwd_h(const void* rec, const float* target, int B, const void* blob,
                                     const NormParams& np, float gscale, void* xf, float* w3slab, void* dz2r,
                                     float* sq_err, int* step_ctr, int num_cus,
                                     hipStream_t stream) {
  using L = TrainLayout<H>;
  constexpr int TPB = TRAIN_TPB;
  // the blob + the waves' dW3 partials [TPB / 64][H + 16] f32 + their dy scratch [TPB / 64][32]
  constexpr size_t LDS = L::BLOB + (size_t)(TPB / 64) * ((H + 16 + 32) * 4 + 1280);
  static_assert(LDS <= 160 * 1024, "training kernel LDS budget");
  static bool attr_set[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!attr_set[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)eta_mlp3_train_fwd_kernel<H>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
    if (e != hipSuccess) return e;
    // the kernel addresses its W2 image at absolute LDS address 0: only valid without static LDS
    hipFuncAttributes fa;
    e = hipFuncGetAttributes(&fa, (const void*)eta_mlp3_train_fwd_kernel<H>);
    if (e != hipSuccess) return e;
    if (fa.sharedSizeBytes != 0) return hipErrorInvalidConfiguration;
    attr_set[dev & 63] = true;
  }
  const int grid = train_fwd_grid(B, num_cus);
  if (grid < 1) return hipSuccess;
  hipLaunchKernelGGL(eta_mlp3_train_fwd_kernel<H>, dim3(grid), dim3(TPB), LDS, stream,
                     (const int4*)rec, target, B, (const unsigned char*)blob, np, gscale,
                     (__bf16*)xf, w3slab, (bf16x8*)dz2r, sq_err, step_ctr);
  return hipGetLastError();
}

hipError_t launch_eta_mlp3_train_fwd(const void* rec, const float* target, int B, const void* blob,
                                     int H, const NormParams& np, float gscale, void* xf,
                                     float* w3slab, void* dz2r,
                                     float* sq_err, int* step_ctr, int num_cus,
                                     hipStream_t stream) {
  switch (H) {
    case 64: return launch_train_fwd_h<64>(rec, target, B, blob, np, gscale, xf, w3slab, dz2r, sq_err, step_ctr, num_cus, stream);
    case 128: return launch_train_fwd_h<128>(rec, target, B, blob, np, gscale, xf, w3slab, dz2r, sq_err, step_ctr, num_cus, stream);
    case 256: return launch_train_fwd_h<256>(rec, target, B, blob, np, gscale, xf, w3slab, dz2r, sq_err, step_ctr, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

// k-slices of train_bwd_kernel: one workgroup per CU at most (its LDS is the whole 160 KB at
// H = 256), each slice a whole number of 32-row tiles, >= ROUTEST_TRAIN_WGRAD_TILES (default 8) of
// them so the W2 staging and the slab write are amortised
static int wgrad_min_tiles() {
  static const int min_tiles = [] {
    const char* v = std::getenv("ROUTEST_TRAIN_WGRAD_TILES");
    const int t = v ? std::atoi(v) : 8;
    return t < 1 ? 1 : t;
  }();
  return min_tiles;
}

// The column split (train_bwd_kernel NBW = 1) at H = 256 for batches up to
// ROUTEST_TRAIN_BWD_SPLIT_ROWS (default 262144; 0 disables): there the slab round trip is a large
// share of the step (64k rows: 75 MB written + read for ~18 GFLOP of backward), while at 1M rows the
// slabs are amortised and the full n-block width per wave is the faster loop.  A slab count that is
// a multiple of 8 selects it (pairs b, b + 8 on one XCD need the grid in whole 16s).
static bool bwd_split(int H, int B, int S) {
  static const long long rows = [] {
    const char* v = std::getenv("ROUTEST_TRAIN_BWD_SPLIT_ROWS");
    return v ? std::atoll(v) : 262144LL;
  }();
  return H == 256 && (long long)B <= rows && S >= 8 && S % 8 == 0;
}

int train_wgrad_slices(int B, int num_cus, int H) {
  const int ntiles = (B + 31) / 32;
  const int min_tiles = wgrad_min_tiles();
  if (H == 256) {
    int Sp = ntiles / min_tiles;
    if (Sp > num_cus / 2) Sp = num_cus / 2;
    Sp &= ~7;
    if (bwd_split(H, B, Sp)) return Sp;
  }
  int S = ntiles / min_tiles;
  if (S > num_cus) S = num_cus;
  return S < 1 ? 1 : S;
}

template <int H>
static hipError_t launch_train_bwd_h(const void* xf, int B, const void* blob, const void* dz2r, float* slab2,
                                     float* slab1, int S, hipStream_t stream) {
  constexpr size_t LDS = (size_t)H * H * 2 + (size_t)2 * H * 64;
  constexpr size_t LDS_SPLIT = (size_t)H * H + (size_t)2 * H * 64;       // half the W2 image
  static_assert(LDS <= 160 * 1024, "train_bwd_kernel LDS budget");
  static bool attr_set[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!attr_set[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)train_bwd_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)LDS);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)train_bwd_kernel<H, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)LDS_SPLIT);
    if (e != hipSuccess) return e;
    attr_set[dev & 63] = true;
  }
  static const bool prof = [] {
    const char* v = std::getenv("ROUTEST_TRAIN_BWD_PROF");
    return v != nullptr && std::atoi(v) != 0;
  }();
  if (prof) {   // diagnostics: per-segment s_memtime sums, printed per launch (synchronises)
    static bool attr_p[64] = {};
    if (!attr_p[dev & 63]) {
      hipError_t e = hipFuncSetAttribute((const void*)train_bwd_kernel<H, 1>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
      if (e != hipSuccess) return e;
      attr_p[dev & 63] = true;
    }
    const int nwv = H / 64;
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(unsigned long long) * 4 * S * nwv);
    if (e != hipSuccess) return e;
    static const int pmode = std::atoi(std::getenv("ROUTEST_TRAIN_BWD_PROF"));
#define RT_BWD_PMODE(P)                                                                                   \
    if (pmode == P) {                                                                                       \
      (void)hipFuncSetAttribute((const void*)train_bwd_kernel<H, P>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                (int)LDS);                                                                  \
      hipLaunchKernelGGL((train_bwd_kernel<H, P>), dim3(S), dim3(H), LDS, stream, (const __bf16*)xf, B,    \
                         (const unsigned char*)blob, (const bf16x8*)dz2r, slab2, slab1, d);                \
    } else
    RT_BWD_PMODE(2) RT_BWD_PMODE(3) RT_BWD_PMODE(4) RT_BWD_PMODE(5) RT_BWD_PMODE(6) {
#undef RT_BWD_PMODE
      hipLaunchKernelGGL((train_bwd_kernel<H, 1>), dim3(S), dim3(H), LDS, stream, (const __bf16*)xf, B,
                         (const unsigned char*)blob, (const bf16x8*)dz2r, slab2, slab1, d);
    }
    std::vector<unsigned long long> h((size_t)4 * S * nwv);
    e = hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(d);
    if (e != hipSuccess) return e;
    double sum[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < h.size(); ++i) sum[i % 4] += (double)h[i];
    const double tiles = (double)((B + 31) / 32) / S;
    std::fprintf(stderr, "[train_bwd prof] per wave-tile (s_memtime ticks): top %.0f  stage+layer1 %.0f  hidden-tile loop %.0f  dW1 %.0f  (tiles/slice %.1f)\n",
                 sum[0] / (S * nwv) / tiles, sum[1] / (S * nwv) / tiles, sum[2] / (S * nwv) / tiles,
                 sum[3] / (S * nwv) / tiles, tiles);
    return hipGetLastError();
  }
  if (bwd_split(H, B, S))      // S slabs, 2S workgroups (pairs b, b + 8)
    hipLaunchKernelGGL((train_bwd_kernel<H, 0, 1>), dim3(2 * S), dim3(H), LDS_SPLIT, stream, (const __bf16*)xf, B,
                       (const unsigned char*)blob, (const bf16x8*)dz2r, slab2, slab1, nullptr);
  else
    hipLaunchKernelGGL(train_bwd_kernel<H>, dim3(S), dim3(H), LDS, stream, (const __bf16*)xf, B,
                       (const unsigned char*)blob, (const bf16x8*)dz2r, slab2, slab1, nullptr);
  return hipGetLastError();
}

hipError_t launch_train_bwd(const void* xf, int B, const void* blob, int H, const void* dz2r, float* slab2,
                            float* slab1, int S, hipStream_t stream) {
  if (S < 1) return hipErrorInvalidValue;
  switch (H) {
    case 64: return launch_train_bwd_h<64>(xf, B, blob, dz2r, slab2, slab1, S, stream);
    case 128: return launch_train_bwd_h<128>(xf, B, blob, dz2r, slab2, slab1, S, stream);
    case 256: return launch_train_bwd_h<256>(xf, B, blob, dz2r, slab2, slab1, S, stream);
    default: return hipErrorInvalidValue;
  }
}

int mlp3_num_params(int H) { return H * H + 15 * H + 1; }
int mlp3_grad_bucket_floats(int H) { return H * (H + 16) + (H + 16) + 16 * H; }

hipError_t launch_adamw_pack(float* P, const float* G, float* M, float* V, void* blob,
                             const int* step, int H, float lr, float beta1, float beta2, float eps,
                             float wd, int warmup, int total_steps, float min_lr_ratio, int update,
                             hipStream_t stream) {
  AdamWArgs a{lr, beta1, beta2, eps, wd, warmup, total_steps, min_lr_ratio, update};
  const int N = mlp3_num_params(H);
  const dim3 grid((N + 255) / 256), block(256);
  switch (H) {
    case 64: hipLaunchKernelGGL(adamw_pack_kernel<64>, grid, block, 0, stream, P, G, M, V, (unsigned char*)blob, step, a); break;
    case 128: hipLaunchKernelGGL(adamw_pack_kernel<128>, grid, block, 0, stream, P, G, M, V, (unsigned char*)blob, step, a); break;
    case 256: hipLaunchKernelGGL(adamw_pack_kernel<256>, grid, block, 0, stream, P, G, M, V, (unsigned char*)blob, step, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_reduce_adamw(const float* slab2, int S2, long long stride2, const float* slab1, int S1,
                               long long stride1, const float* w3slab, int S3, long long stride3, float* G,
                               float* P, float* M, float* V, void* blob, const int* step, int H, float lr,
                               float beta1, float beta2, float eps, float wd, int warmup, int total_steps,
                               float min_lr_ratio, hipStream_t stream) {
  if (H != 64 && H != 128 && H != 256) return hipErrorInvalidValue;
  const int LDG = H + 16;
  if (stride2 < (long long)H * LDG || stride1 < 16LL * H || stride3 < LDG || S2 < 1 || S1 < 1 || S3 < 1)
    return hipErrorInvalidValue;
  AdamWArgs a{lr, beta1, beta2, eps, wd, warmup, total_steps, min_lr_ratio, 1};
  const RedSeg s0{slab2, stride2, G, S2, H * LDG, H};
  const RedSeg s1{slab1, stride1, G + H * LDG + LDG, S1, 16 * H, 0};
  const RedSeg s2{w3slab, stride3, G + H * LDG, S3, LDG, 0};
  const int per = 4 * RED_COLS;
  const int nb0 = (s0.n + per - 1) / per, nb1 = (s1.n + per - 1) / per, nb2 = (s2.n + per - 1) / per;
  const dim3 grid(nb0 + nb1 + nb2), block(256);
  unsigned char* b = (unsigned char*)blob;
  switch (H) {
    case 64: hipLaunchKernelGGL(reduce_adamw_kernel<64>, grid, block, 0, stream, s0, s1, s2, nb0, nb0 + nb1, P, M, V, b, step, a); break;
    case 128: hipLaunchKernelGGL(reduce_adamw_kernel<128>, grid, block, 0, stream, s0, s1, s2, nb0, nb0 + nb1, P, M, V, b, step, a); break;
    case 256: hipLaunchKernelGGL(reduce_adamw_kernel<256>, grid, block, 0, stream, s0, s1, s2, nb0, nb0 + nb1, P, M, V, b, step, a); break;
  }
  return hipGetLastError();
}

}  // namespace rt
