// K3: data-parallel training of the 3-layer ETA MLP on gfx950 — fused forward/loss kernel,
// ReLU backward, and fused AdamW + MFMA-fragment re-pack.  (The reference has no training code at
// all: notebooks/.gitkeep; its feature schema is RO/Flaskr/ml.py:35-51.)
//
// One training step on a rank (routest_amd/train/fused.py::FusedMlp3Trainer):
//   1. eta_mlp3_train_fwd_kernel (this file): featurize + layer 1 + layer 2 + layer 3 + MSE
//      gradient + the whole input-gradient path dz2 -> dh1 = dz2 W2 -> dz1 = dh1 * relu'(z1) in
//      ONE launch.  Because dL/dz2 = dy * w3 * relu'(z2) needs only the ReLU mask, dz2 is
//      produced in-register the moment y (hence dy) is known, and it IS the B operand of the dgrad
//      MFMAs (accumulator layout == next-MFMA B layout, common.h); W2 is read a second time from
//      the same LDS image through the hardware-transposed ds_read_b64_tr_b16 as the A operand
//      W2^T; h1, still in registers, gives relu'(z1).  No library GEMM, no dh1 round trip.
//      Emits, bf16 row-major:
//        xf  [B,16]   the exact bf16 features the MFMA consumed, slot 14 := 1 (bias-grad column)
//        h1a [B,H+16] relu(z1) with column H := 1   (dW2 | db2 = dz2^T h1a)
//        h2a [B,H+16] relu(z2) with column H := 1   (dW3 | db3 = dy^T h2a)
//        dz2 [B,H], dz1 [B,H], dy [B,8] (col 0; pre-scaled by 2 / global_batch), per-row
//        squared errors.
//      The kernel never reads back what it stored (a load waits for every older store of the
//      wave: vmcnt counts both, in order), and nothing it needs per tile is hoisted out of the
//      tile loop (hoisted, it exceeds the VGPR budget and every spill reload after the stores
//      stalls the same way).
//   2. the three weight-gradient GEMMs (K = batch) on the split-K wgrad kernel (wgrad.hip) + one
//      deterministic slab reduction.
//   3. ONE flat fp32 gradient bucket -> one RCCL all-reduce over xGMI.
//   4. adamw_pack_kernel: AdamW on the flat fp32 master params, writing back the training blob the
//      next forward stages into LDS — no host work, no sync, so the whole step is capturable in a
//      HIP graph.
//
// Training blob (TrainLayout): [ w2img | w1p | b1p | b2p | w3p | tail ] where w2img holds W2
// row-major in 512-byte rows (natural unit order both ways) with 8-byte chunk k of row R at chunk
// k ^ w2swz(R).  That one image serves both operand reads conflict-free (bank rule,
// cdna_hip_programming.md §2 / MI355X_MICROARCH.md §LDS):
//   * layer 2, A = W2: lane (r, h) of tile (mt, ks) reads row 32mt + r, units 16ks + 4h .. +3 and
//     16ks + 8 + 4h .. +3 (the permuted k order of the h1 B fragments) with two ds_read_b64:
//     w2swz is a bijection of R mod 32, so a 32-lane half hits 64 distinct banks;
//   * dgrad, A = W2^T: ds_read_b64_tr_b16 over 4-row x 16-column blocks (rows 16ks + 4h + q and
//     16ks + 8 + 4h + q, columns 32mi + 16g .. +15): w2swz moves the 4 rows of a block to 4
//     different 8-chunk groups, so a 32-lane half touches 64 distinct banks.
// Natural column order is what makes relu'(z1) lane-local: dgrad accumulator register e of lane
// half h is unit 32mi + 8(e>>2) + 4h + (e&3), element e&7 of the lane's own h1 fragment.
// The rest of the blob is the inference layout (mlp3_tile.h): w1p, b1p, b2p, w3p, tail.
#include <cstdlib>

#include "lds_fill.h"
#include "mlp3_tile.h"
#include "ops.h"

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
  static constexpr size_t BLOB = W2B + W1B + 3 * VB + 16;
};

size_t eta_mlp3_train_blob_bytes(int H) { return (size_t)H * 512 + 44 * (size_t)H + 16; }

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
    float* __restrict__ w3slab, bf16x8* __restrict__ dz2t, bf16x8* __restrict__ dh1t,
    __bf16* __restrict__ dyb, float* __restrict__ sq_err, int* __restrict__ step_ctr) {
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
  const float b3 = reinterpret_cast<const float*>(w3p + H / 4)[0];

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
    const int4 rc = valid ? rec[row] : make_int4(0, 0, 0, 0);
    const bf16x8 xb = featurize_bf16(rc, h, np);
    if (valid)  // slots 14, 15 hold 1.0 (the b1 hi/lo inputs): dW1k[:,14] == db1
      *reinterpret_cast<bf16x8*>(xf + (size_t)row * 16 + 8 * h) = xb;

    // layer 1 (A fragments re-read from LDS per tile: no registers held across tiles)
    bf16x8 h1[KS];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      acc = mfma32(w1p[mt * 64 + lane], xb, acc);
      float a[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) a[e] = acc[e];
      relu_cvt_bf16x8(a, &h1[2 * mt]);
      relu_cvt_bf16x8(a + 8, &h1[2 * mt + 1]);
    }
    // (h1 is not stored: train_wgrad_kernel recomputes it from xf on the same MFMA)

    // layer 2 + layer 3 in TWO passes over the hidden tiles, relu(z2) never stored: pass 1 only
    // forms y (hence dy); pass 2 recomputes z2 per tile for the relu'(z2) mask and the dW3 | db3
    // partial.  The second 128 MFMAs per tile cost less than writing h2a (35.6 MB at 64k rows)
    // and reading it back in a split-K GEMM; keeping relu(z2) in registers instead (64 VGPRs next
    // to h1's 64) spilled.
    unsigned long long mask_lo = 0, mask_hi = 0;   // 16 relu'(z2) bits per hidden tile
    float ys = 0.f;
    float dy, diff;
    {
      // addresses as lane bases + immediates (a run-time or fully hoisted w2off() per fragment
      // costs VGPRs the compiler then spills — and a scratch reload after the activation stores
      // would wait for all of them, vmcnt being in order): chunk (2ks + h) ^ w2swz(r) only
      // depends on ks & 7, ks >> 3 adds 256 B
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
      auto layer2 = [&](int mt) {
        f32x16 acc = load_vec16(b2p, mt, h);
        lds_u8* pm = lrow + mt * 16384;
        // units 16ks + 4h + 0..3 and 16ks + 8 + 4h + 0..3: the permuted k order of h1
        auto frag = [&](int ks) {
          const int* xo = (ks >> 3) ? xk8[ks & 7] : xk[ks & 7];
          const s16x4 lo = *reinterpret_cast<const lds_s16x4*>(pm + xo[0]);
          const s16x4 hi = *reinterpret_cast<const lds_s16x4*>(pm + xo[1]);
          return join4(lo, hi);
        };
        bf16x8 ring[D];
#pragma unroll
        for (int d = 0; d < D; ++d) ring[d] = frag(d);
#pragma unroll
        for (int ks = 0; ks < KS; ks += D) {
          bf16x8 a[D];
#pragma unroll
          for (int d = 0; d < D; ++d) {
            a[d] = ring[d];
            if (ks + D + d < KS) ring[d] = frag(ks + D + d);
          }
#pragma unroll
          for (int d = 0; d < D; ++d) acc = mfma32(a[d], h1[ks + d], acc);
        }
        return acc;
      };
      // pass 1: y and the relu'(z2) bits (accumulator layout: units in registers, rows on lanes)
#pragma unroll 1
      for (int mt = 0; mt < MT; ++mt) {
        const f32x16 acc = layer2(mt);
        const f32x16 w3 = load_vec16(w3p, mt, h);
        unsigned mk = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          ys = __builtin_fmaf(relu_f(acc[e]), w3[e], ys);
          mk |= (acc[e] > 0.f ? 1u : 0u) << e;
        }
        if (mt < 4) mask_lo |= (unsigned long long)mk << (16 * mt);
        else mask_hi |= (unsigned long long)mk << (16 * (mt - 4));
      }
      ys += __shfl_xor(ys, 32);
      const float y = ys + b3;
      diff = valid ? (y - target[row]) : 0.f;
      dy = gscale * diff;
      // pass 2: the dW3 partial sum_r bf16(dy_r) bf16(relu(z2[r, c])) (the operands the split-K
      // GEMM over h2a used) on the TRANSPOSED tile: the same two operands with their MFMA roles
      // swapped (h1 as A, the W2 row fragment as B) give z2^T — hidden unit 32mt + r on the lanes,
      // the tile's rows 8(e>>2) + 4h + (e&3) in the registers — so the row sum is 16 in-lane FMAs
      // and ONE cross-half add per hidden tile instead of a 5-step lane reduce-scatter.  The rows'
      // dy reach the lanes through a 128-byte LDS broadcast; rows past B carry dy = 0.
      float* const dys = dyscr;                      // this wave's 32-float scratch
      if (h == 0) dys[r] = dy;
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
      const float* b2f = reinterpret_cast<const float*>(b2p);
      const int bpos = 2 * ((r >> 2) & 1) * 8 + 4 * (r >> 3) + (r & 3);   // b2 / w3 of unit 32mt + r
#pragma unroll 1
      for (int mt = 0; mt < MT; ++mt) {
        f32x16 acc;
        const float bias = b2f[mt * 32 + bpos];
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = bias;
        lds_u8* pm = lrow + mt * 16384;
        auto fragw = [&](int ks) {
          const int* xo = (ks >> 3) ? xk8[ks & 7] : xk[ks & 7];
          const s16x4 lo = *reinterpret_cast<const lds_s16x4*>(pm + xo[0]);
          const s16x4 hi = *reinterpret_cast<const lds_s16x4*>(pm + xo[1]);
          return join4(lo, hi);
        };
        bf16x8 ring[D];
#pragma unroll
        for (int d = 0; d < D; ++d) ring[d] = fragw(d);
#pragma unroll
        for (int ks = 0; ks < KS; ks += D) {
          bf16x8 a[D];
#pragma unroll
          for (int d = 0; d < D; ++d) {
            a[d] = ring[d];
            if (ks + D + d < KS) ring[d] = fragw(ks + D + d);
          }
#pragma unroll
          for (int d = 0; d < D; ++d) acc = mfma32(h1[ks + d], a[d], acc);
        }
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) t = __builtin_fmaf(dyv[e], (float)(__bf16)relu_f(acc[e]), t);
        t += __shfl_xor(t, 32);
        if (h == 0) {
          const int u = 32 * mt + r;                 // stored column: hperm(u) = u with bits 2, 3 swapped
          w3part[(u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1)] += t;
        }
      }
      // db3 = sum of dy over the rows (lanes of half 0 hold each row once)
      float d = h == 0 ? dy : 0.f;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) d += __shfl_xor(d, o);
      if (lv == 0) w3part[H] += d;
    }
    if (valid && h == 0) {  // dy as an [B,8] bf16 operand (cols 1..7 zero) for the wgrad kernel
      bf16x8 dv;
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[j] = (__bf16)0.f;
      dv[0] = (__bf16)dy;
      *reinterpret_cast<bf16x8*>(dyb + (size_t)row * 8) = dv;
    }
    // per-row squared error (no cross-lane reduction: its shuffle addresses were the values the
    // compiler spilled, and every reload after the activation stores waited for all of them)
    if (valid && h == 0) sq_err[row] = diff * diff;

    // dz2 = dy * w3 * relu'(z2): fragment 2mt + s element j is accumulator register 8s + j of
    // hidden tile mt, i.e. exactly the B-operand k order of the dgrad MFMAs below
    bf16x8 dz2f[KS];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const f32x16 w3 = load_vec16(w3p, mt, h);
      const unsigned mk = (unsigned)((mt < 4 ? mask_lo >> (16 * mt) : mask_hi >> (16 * (mt - 4))) & 0xffffu);
      // per output pair: two products, one v_cvt_pk_bf16_f32, and the pair's two mask bits
      // sign-extended (v_bfe_i32) into a 0xFFFF / 0xFFFF0000 mask
      typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
      typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
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
        dz2f[2 * mt + s] = __builtin_bit_cast(bf16x8, dw);
      }
    }
    // dz2^T for the weight-gradient kernel: each hidden tile transposed by TWO MFMAs against a
    // permuted identity (B[k][n] = 1 iff fragment k of this lane half holds unit n), which turns the
    // rows-on-lanes fragments into units-on-lanes / rows-in-registers — exact (every product is
    // x * 1) — and stored in the MFMA operand order: chunk (tile, K-step s, unit, lane half h)
    {
      bf16x8 eye0, eye1;
      const int n = lv & 31;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int u0 = (j & 3) + 8 * (j >> 2) + 4 * h;          // unit offset of k = 8h + j, K-step 0
        eye0[j] = (__bf16)(u0 == n ? 1.f : 0.f);
        eye1[j] = (__bf16)(u0 + 16 == n ? 1.f : 0.f);
      }
      f32x16 zero;
#pragma unroll
      for (int e = 0; e < 16; ++e) zero[e] = 0.f;
      typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
      typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f32x16 tt = mfma32(dz2f[2 * mt], eye0, zero);
        tt = mfma32(dz2f[2 * mt + 1], eye1, tt);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u32x4v ow;
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) {
            const f32x2 pr = {tt[8 * s2 + 2 * q2], tt[8 * s2 + 2 * q2 + 1]};
            ow[q2] = __builtin_bit_cast(unsigned, __builtin_convertvector(pr, bf16x2v));
          }
          dz2t[(((size_t)tile * 2 + s2) * H + 32 * mt + n) * 2 + h] = __builtin_bit_cast(bf16x8, ow);
        }
      }
    }

    // dgrad: dh1 = dz2 W2 on the TRANSPOSED tile — dz2 as the A operand (rows on the lanes) and
    // the W2^T fragment as B — so the accumulator holds input unit 32mi + (l&31) on the lane and the
    // tile's rows in the registers, in the MFMA k order.  That is the dW1 GEMM's A layout: stored
    // like dz2^T (one 16-byte chunk per K-step and lane half), it is read by train_wgrad_kernel
    // without any transpose; relu'(z1) is applied there, from the h1^T tile it recomputes anyway.
    {
      // transposed reads: rows 16ks + 8t + 4h + q, columns 32mi + 16(g&1) + 4p (8-byte chunk
      // 8mi + 4(g&1) + p) -> chunk ^ ((q << 3) | (4(ks&1) + 2t + h))
      // = 64 (mi ^ q) + 8 ((4(g&1) + p) ^ (4(ks&1) + 2t + h)): the lane part of the second term
      // takes four values (ks parity x t), so four lane bases + a per-mi offset + immediates
      // replace a full address computation per read
      const int g1 = (lv >> 4) & 1, p = lv & 3, q = (lv >> 2) & 3;
      const int lx = 4 * g1 + p;
      lds_u8* rb = img + (4 * h + q) * 512;
      lds_u8* bp[2][2];
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int t = 0; t < 2; ++t) bp[par][t] = rb + 4096 * t + 8 * (lx ^ (4 * par + 2 * t + h));
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int om = 64 * (mi ^ q);
        auto frag = [&](int ks) {
          lds_u8* r0 = bp[ks & 1][0] + om + 8192 * ks;
          lds_u8* r1 = bp[ks & 1][1] + om + 8192 * ks;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)r0);
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)r1);
          return join4(lo, hi);
        };
        f32x16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.f;
        bf16x8 ring[D];
#pragma unroll
        for (int d = 0; d < D; ++d) ring[d] = frag(d);
#pragma unroll
        for (int ks = 0; ks < KS; ks += D) {
          bf16x8 a[D];
#pragma unroll
          for (int d = 0; d < D; ++d) {
            a[d] = ring[d];
            if (ks + D + d < KS) ring[d] = frag(ks + D + d);
          }
#pragma unroll
          for (int d = 0; d < D; ++d) acc = mfma32(dz2f[ks + d], a[d], acc);
        }
        typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
        typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u32x4v ow;
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) {
            const f32x2 pr = {acc[8 * s2 + 2 * q2], acc[8 * s2 + 2 * q2 + 1]};
            ow[q2] = __builtin_bit_cast(unsigned, __builtin_convertvector(pr, bf16x2v));
          }
          dh1t[(((size_t)tile * 2 + s2) * H + 32 * mi + (lv & 31)) * 2 + h] = __builtin_bit_cast(bf16x8, ow);
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

// ---------------------------------------------------------------------------------------------
// Weight gradients dW2 | db2 = dz2^T [h1 | 1] and dW1 = (dh1 * relu'(z1))^T x, K = batch, with
// NO LDS and no barriers: one workgroup per k-slice, wave w owning output rows 32w .. 32w + 31 of
// both products and its accumulators (9 + 1 tiles of 32x32 at H = 256: 160 VGPRs) in registers for
// the whole slice.  Per 32-row tile a wave
//   * loads its dz2^T / dh1^T fragments — one 16-byte load per K-step, the forward stored them in
//     the MFMA operand order — and the tile's 32-byte feature rows;
//   * recomputes h1 = relu(W1k x) for every n-tile on the layer-1 MFMA with the operands swapped
//     (x as A, the forward's w1p fragment as B), which yields h1^T with the units on the lanes and
//     the rows in the registers: exactly the B operand of dW2 (K = rows), and, for n-tile w, the
//     relu'(z1) mask of dh1^T in its own layout;
//   * transposes x by one MFMA against an identity fragment for dW1's B operand;
//   * issues 2 MFMAs per output tile (K = 32 rows).
// The B operand [h1 | 1] never exists in memory (the old path stored h1a, 544 B/row, and read it
// back with dz2 through LDS-staged transposed reads).  Partial sums of slice s go to slab[s] in the
// bucket layout (hperm rows and columns, train/fused.py) and wgrad_reduce sums them in a fixed
// order.
template <int H>
__global__ __launch_bounds__(H / 32 * 64, 1) void train_wgrad_kernel(
    const __bf16* __restrict__ xf, int B, const unsigned char* __restrict__ blob,
    const bf16x8* __restrict__ dz2t, const bf16x8* __restrict__ dh1t, int tiles_per_slice,
    float* __restrict__ slab2, float* __restrict__ slab1) {
  using L = TrainLayout<H>;
  constexpr int MT = H / 32, LDG = H + 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, col = lane & 31, h = lane >> 5;
  const int ntiles = (B + 31) >> 5;
  const int t0 = blockIdx.x * tiles_per_slice;
  const int t1 = min(ntiles, t0 + tiles_per_slice);
  // the layer-1 fragments (the same for every wave) in LDS, not in 32 VGPRs per wave
  __shared__ bf16x8 s_w1[MT * 64];
  const bf16x8* w1p = reinterpret_cast<const bf16x8*>(blob + L::W2B);
  for (int i = threadIdx.x; i < MT * 64; i += blockDim.x) s_w1[i] = w1p[i];
  __syncthreads();
  bf16x8 eye;
#pragma unroll
  for (int j = 0; j < 8; ++j) eye[j] = (__bf16)(8 * h + j == col ? 1.f : 0.f);   // B (k = 8h + j, n = col)
  f32x16 acc2[MT], acc1;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    acc1[e] = 0.f;
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) acc2[nt][e] = 0.f;
  }
  float db2 = 0.f;                     // sum of this lane's dz2 values (unit 32w + col)
  f32x16 zero;
#pragma unroll
  for (int e = 0; e < 16; ++e) zero[e] = 0.f;
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
  // fragments of one 32-row tile: x (A of the layer-1 / identity MFMAs), dz2^T and dh1^T (A of
  // the two products, one 16-byte load per K-step); the next tile's are in flight while this one
  // computes (the loads are the only latency in the loop)
  struct Frags {
    bf16x8 x, a0, a1, g0, g1;
  };
  // buffer loads: 32-bit offsets against wave-uniform descriptors (no 64-bit address per load, which
  // left the kernel short of VGPRs), and the hardware range check zero-fills the rows past B
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)xf, 0, B * 32, 0x00020000);
  const int tb = ntiles * 32 * H * 2;                  // bytes of dz2t / dh1t
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)dz2t, 0, tb, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)dh1t, 0, tb, 0x00020000);
  auto load = [&](int tile) {
    Frags f;
    f.x = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rx, (tile * 32 + col) * 32 + 16 * h, 0, 0));
    const int c0 = ((tile * 2 * H + 32 * w + col) * 2 + h) * 16, c1 = c0 + H * 2 * 16;
    f.a0 = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, c0, 0, 0));
    f.a1 = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, c1, 0, 0));
    f.g0 = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rg, c0, 0, 0));
    f.g1 = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rg, c1, 0, 0));
    return f;
  };
  Frags cur;
  if (t0 < t1) cur = load(t0);
  for (int tile = t0; tile < t1; ++tile) {
    Frags nxt = cur;
    if (tile + 1 < t1) nxt = load(tile + 1);
    // db2 = sum over rows of dz2 (VALU on the A fragments; no MFMA tile for one column)
    {
      const u32x4v p0 = __builtin_bit_cast(u32x4v, cur.a0), p1 = __builtin_bit_cast(u32x4v, cur.a1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        db2 += __uint_as_float(p0[q] << 16) + __uint_as_float(p0[q] & 0xFFFF0000u);
        db2 += __uint_as_float(p1[q] << 16) + __uint_as_float(p1[q] & 0xFFFF0000u);
      }
    }
    bf16x8 g0 = cur.g0, g1 = cur.g1;
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) {
      const f32x16 hz = mfma32(cur.x, s_w1[nt * 64 + lane], zero);   // h1^T pre-activation, units 32nt + col
      acc2[nt] = mfma32(cur.a0, pack(hz, 0, true), acc2[nt]);
      acc2[nt] = mfma32(cur.a1, pack(hz, 1, true), acc2[nt]);
      if (nt == w) {                                    // relu'(z1) for this wave's dW1 rows
        u32x4v m0 = __builtin_bit_cast(u32x4v, g0), m1 = __builtin_bit_cast(u32x4v, g1);
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          const unsigned k0 = (hz[2 * q2] > 0.f ? 0xFFFFu : 0u) | (hz[2 * q2 + 1] > 0.f ? 0xFFFF0000u : 0u);
          const unsigned k1 = (hz[8 + 2 * q2] > 0.f ? 0xFFFFu : 0u) | (hz[8 + 2 * q2 + 1] > 0.f ? 0xFFFF0000u : 0u);
          m0[q2] &= k0;
          m1[q2] &= k1;
        }
        g0 = __builtin_bit_cast(bf16x8, m0);
        g1 = __builtin_bit_cast(bf16x8, m1);
      }
    }
    // x^T: D[row][f] with the feature on the lane and the rows in the registers
    const f32x16 xt = mfma32(cur.x, eye, zero);
    acc1 = mfma32(g0, pack(xt, 0, false), acc1);
    acc1 = mfma32(g1, pack(xt, 1, false), acc1);
    cur = nxt;
  }
  // D[m][n]: lane -> n = col, register e -> m = (e&3) + 8(e>>2) + 4h; rows / columns to the bucket's
  // hperm order (the stored unit order of every other gradient path)
  float* o2 = slab2 + (size_t)blockIdx.x * H * LDG;
  float* o1 = slab1 + (size_t)blockIdx.x * H * 16;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = 32 * w + (e & 3) + 8 * (e >> 2) + 4 * h;
    const int mr = hperm(m);
#pragma unroll
    for (int nt = 0; nt < MT; ++nt) o2[(size_t)mr * LDG + hperm(32 * nt + col)] = acc2[nt][e];
    if (col < 16) o1[(size_t)mr * 16 + col] = acc1[e];
  }
  // db2 column (and the zero columns H+1 .. H+15): both lane halves hold rows of unit 32w + col
  db2 += __shfl_xor(db2, 32);
  const int ur = hperm(32 * w + col);
  if (h == 0) o2[(size_t)ur * LDG + H] = db2;
  else
#pragma unroll
    for (int c = 1; c < 16; ++c) o2[(size_t)ur * LDG + H + c] = 0.f;
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

template <int H>
__global__ __launch_bounds__(256) void adamw_pack_kernel(float* __restrict__ P,
                                                         const float* __restrict__ G,
                                                         float* __restrict__ M, float* __restrict__ V,
                                                         unsigned char* __restrict__ blob,
                                                         const int* __restrict__ step, AdamWArgs a) {
  using L = TrainLayout<H>;
  constexpr int OFF_B1 = 12 * H, OFF_W2 = 13 * H, OFF_B2 = 13 * H + H * H, OFF_W3 = OFF_B2 + H,
                OFF_B3 = OFF_W3 + H, N = OFF_B3 + 1;
  constexpr int LDG = H + 16;
  const float* gW2a = G;
  const float* gW3a = G + H * LDG;
  const float* gW1a = gW3a + LDG;
  unsigned char* w2img = blob;
  __bf16* w1p = reinterpret_cast<__bf16*>(blob + L::W2B);
  float* b1p = reinterpret_cast<float*>(blob + L::W2B + L::W1B);
  float* b2p = b1p + H;
  float* w3p = b2p + H;
  float* tail = w3p + H;

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

// workgroups of the training forward (= rows of its dW3 slab): one per 8 row tiles, at most one
// per CU (the blob fills the LDS)
int train_fwd_grid(int B, int num_cus) {
  const int ntiles = (B + 31) / 32;
  const int g = (ntiles + TRAIN_TPB / 64 - 1) / (TRAIN_TPB / 64);
  return g < num_cus ? g : num_cus;
}

template <int H>
static hipError_t launch_train_fwd_h(const void* rec, const float* target, int B, const void* blob,
                                     const NormParams& np, float gscale, void* xf, float* w3slab, void* dz2t,
                                     void* dh1t, void* dyb, float* sq_err, int* step_ctr, int num_cus,
                                     hipStream_t stream) {
  using L = TrainLayout<H>;
  constexpr int TPB = TRAIN_TPB;
  // the blob + the waves' dW3 partials [TPB / 64][H + 16] f32 + their dy scratch [TPB / 64][32]
  constexpr size_t LDS = L::BLOB + (size_t)(TPB / 64) * (H + 16 + 32) * 4;
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
                     (__bf16*)xf, w3slab, (bf16x8*)dz2t, (bf16x8*)dh1t, (__bf16*)dyb, sq_err, step_ctr);
  return hipGetLastError();
}

hipError_t launch_eta_mlp3_train_fwd(const void* rec, const float* target, int B, const void* blob,
                                     int H, const NormParams& np, float gscale, void* xf,
                                     float* w3slab, void* dz2t, void* dh1t, void* dyb,
                                     float* sq_err, int* step_ctr, int num_cus,
                                     hipStream_t stream) {
  switch (H) {
    case 64: return launch_train_fwd_h<64>(rec, target, B, blob, np, gscale, xf, w3slab, dz2t, dh1t, dyb, sq_err, step_ctr, num_cus, stream);
    case 128: return launch_train_fwd_h<128>(rec, target, B, blob, np, gscale, xf, w3slab, dz2t, dh1t, dyb, sq_err, step_ctr, num_cus, stream);
    case 256: return launch_train_fwd_h<256>(rec, target, B, blob, np, gscale, xf, w3slab, dz2t, dh1t, dyb, sq_err, step_ctr, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

// k-slices of train_wgrad_kernel: one workgroup per CU at most (its waves hold ~170 VGPRs of
// accumulators and fragments), each slice a whole number of 32-row tiles
int train_wgrad_slices(int B, int num_cus) {
  static const int min_tiles = [] {
    const char* v = std::getenv("ROUTEST_TRAIN_WGRAD_TILES");
    const int t = v ? std::atoi(v) : 4;
    return t < 1 ? 1 : t;
  }();
  const int ntiles = (B + 31) / 32;
  int S = ntiles / min_tiles;          // >= min_tiles 32-row tiles per slice (the slab write amortised)
  if (S > num_cus) S = num_cus;
  return S < 1 ? 1 : S;
}

template <int H>
static hipError_t launch_train_wgrad_h(const void* xf, int B, const void* blob, const void* dz2t, const void* dh1t,
                                       float* slab2, float* slab1, int S, hipStream_t stream) {
  const int ntiles = (B + 31) / 32;
  const int tps = (ntiles + S - 1) / S;
  hipLaunchKernelGGL(train_wgrad_kernel<H>, dim3(S), dim3(H / 32 * 64), 0, stream, (const __bf16*)xf, B,
                     (const unsigned char*)blob, (const bf16x8*)dz2t, (const bf16x8*)dh1t, tps, slab2, slab1);
  return hipGetLastError();
}

hipError_t launch_train_wgrad(const void* xf, int B, const void* blob, int H, const void* dz2t, const void* dh1t,
                              float* slab2, float* slab1, int S, hipStream_t stream) {
  if (S < 1) return hipErrorInvalidValue;
  switch (H) {
    case 64: return launch_train_wgrad_h<64>(xf, B, blob, dz2t, dh1t, slab2, slab1, S, stream);
    case 128: return launch_train_wgrad_h<128>(xf, B, blob, dz2t, dh1t, slab2, slab1, S, stream);
    case 256: return launch_train_wgrad_h<256>(xf, B, blob, dz2t, dh1t, slab2, slab1, S, stream);
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

}  // namespace rt
