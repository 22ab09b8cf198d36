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
    __bf16* __restrict__ h1a, float* __restrict__ w3slab, __bf16* __restrict__ dz2,
    __bf16* __restrict__ dz1, __bf16* __restrict__ dyb, float* __restrict__ sq_err,
    int* __restrict__ step_ctr) {
  using L = TrainLayout<H>;
  constexpr int MT = H / 32, KS = H / 16, LDA = H + 16, D = KS < 4 ? KS : 4;
  // device-side optimizer step counter (read by adamw_pack_kernel later on the same stream), so a
  // captured HIP graph replays with correct bias corrections / LR schedule
  if (step_ctr != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *step_ctr += 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  lds_fill_block(smem, blob, (int)L::BLOB);
  const unsigned char* img = smem;
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
    __bf16* h1row = h1a + (size_t)row * LDA;
    if (valid) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<bf16x8*>(h1row + 16 * ks + 8 * h) = h1[ks];
      bf16x8 tailv;
#pragma unroll
      for (int j = 0; j < 8; ++j) tailv[j] = (__bf16)0.f;
      if (h == 0) tailv[0] = (__bf16)1.f;
      *reinterpret_cast<bf16x8*>(h1row + H + 8 * h) = tailv;
    }

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
      const unsigned char* lrow = img + r * 512;
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
        const unsigned char* pm = lrow + mt * 16384;
        // units 16ks + 4h + 0..3 and 16ks + 8 + 4h + 0..3: the permuted k order of h1
        auto frag = [&](int ks) {
          const int* xo = (ks >> 3) ? xk8[ks & 7] : xk[ks & 7];
          const s16x4 lo = *reinterpret_cast<const s16x4*>(pm + xo[0]);
          const s16x4 hi = *reinterpret_cast<const s16x4*>(pm + xo[1]);
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
      const float dyr = (float)(__bf16)dy;
      float* const dys = dyscr;                      // this wave's 32-float scratch
      if (h == 0) dys[r] = dyr;
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
      const int bpos = 2 * ((r >> 2) & 1) * 8 + 4 * (r >> 3) + (r & 3);   // b2 of unit 32mt + r
#pragma unroll 1
      for (int mt = 0; mt < MT; ++mt) {
        f32x16 acc;
        const float bias = b2f[mt * 32 + bpos];
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = bias;
        const unsigned char* pm = lrow + mt * 16384;
        auto fragw = [&](int ks) {
          const int* xo = (ks >> 3) ? xk8[ks & 7] : xk[ks & 7];
          const s16x4 lo = *reinterpret_cast<const s16x4*>(pm + xo[0]);
          const s16x4 hi = *reinterpret_cast<const s16x4*>(pm + xo[1]);
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
      // db3 = sum of bf16(dy) over the rows (lanes of half 0 hold each row once)
      float d = h == 0 ? dyr : 0.f;
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
    if (valid) {
      __bf16* drow = dz2 + (size_t)row * H;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<bf16x8*>(drow + 16 * ks + 8 * h) = dz2f[ks];
    }

    // dgrad: dh1^T tile mi = W2^T[32mi.., :] dz2^T, then dz1 = dh1 * relu'(z1).  Accumulator
    // register e is input unit 32mi + 8(e>>2) + 4h + (e&3): exactly element e&7 of this lane's own
    // h1 fragment 2mi + (e>>3), so relu'(z1) is a lane-local select on the packed bf16 output, and
    // dz1 lands at hperm positions 32mi + 16(e>>3) + 8h + (e&7) — two 16-byte stores like h1a.
    // The mi loop is unrolled so that h1 is indexed statically (kept in registers, never re-read
    // from memory: a load would wait for every older store of the wave).
    {
      __bf16* zrow = dz1 + (size_t)row * H;
      // transposed reads: rows 16ks + 8t + 4h + q, columns 32mi + 16(g&1) + 4p (8-byte chunk
      // 8mi + 4(g&1) + p) -> chunk ^ ((q << 3) | (4(ks&1) + 2t + h))
      // = 64 (mi ^ q) + 8 ((4(g&1) + p) ^ (4(ks&1) + 2t + h)): the lane part of the second term
      // takes four values (ks parity x t), so four lane bases + a per-mi offset + immediates
      // replace a full address computation per read
      const int g1 = (lv >> 4) & 1, p = lv & 3, q = (lv >> 2) & 3;
      const int lx = 4 * g1 + p;
      const unsigned char* rb = img + (4 * h + q) * 512;
      const unsigned char* bp[2][2];
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int t = 0; t < 2; ++t) bp[par][t] = rb + 4096 * t + 8 * (lx ^ (4 * par + 2 * t + h));
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) {
        const int om = 64 * (mi ^ q);
        auto frag = [&](int ks) {
          const unsigned char* r0 = bp[ks & 1][0] + om + 8192 * ks;
          const unsigned char* r1 = bp[ks & 1][1] + om + 8192 * ks;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<unsigned char*>(r0)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(const_cast<unsigned char*>(r1)));
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
          for (int d = 0; d < D; ++d) acc = mfma32(a[d], dz2f[ks + d], acc);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          // relu'(z1) from h1 as a packed mask: h1 halves are non-negative bf16 bit patterns
          // (0 .. 0x7F80), so x + 0x7FFF has bit 15 set iff x != 0 (iff z1 > 0) and no carry
          // crosses into the other half; an arithmetic >> 15 per half spreads it to 0xFFFF.
          // Per pair of outputs: one v_cvt_pk_bf16_f32, one add, one v_pk_ashrrev_i16, one and.
          typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
          typedef short s16x2v __attribute__((ext_vector_type(2)));
          typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
          const u32x4v hw = __builtin_bit_cast(u32x4v, h1[2 * mi + s]);
          u32x4v ow;
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) {
            const f32x2 pr = {acc[8 * s + 2 * q2], acc[8 * s + 2 * q2 + 1]};
            const unsigned cw = __builtin_bit_cast(unsigned, __builtin_convertvector(pr, bf16x2v));
            const s16x2v m = __builtin_bit_cast(s16x2v, hw[q2] + 0x7FFF7FFFu) >> (s16x2v){15, 15};
            ow[q2] = cw & __builtin_bit_cast(unsigned, m);
          }
          const bf16x8 ov = __builtin_bit_cast(bf16x8, ow);
          if (valid) *reinterpret_cast<bf16x8*>(zrow + 32 * mi + 16 * s + 8 * h) = ov;   // hperm order
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
                                     const NormParams& np, float gscale, void* xf, void* h1a,
                                     float* w3slab, void* dz2, void* dz1, void* dyb, float* sq_err,
                                     int* step_ctr, int num_cus, hipStream_t stream) {
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
    attr_set[dev & 63] = true;
  }
  const int grid = train_fwd_grid(B, num_cus);
  if (grid < 1) return hipSuccess;
  hipLaunchKernelGGL(eta_mlp3_train_fwd_kernel<H>, dim3(grid), dim3(TPB), LDS, stream,
                     (const int4*)rec, target, B, (const unsigned char*)blob, np, gscale,
                     (__bf16*)xf, (__bf16*)h1a, w3slab, (__bf16*)dz2, (__bf16*)dz1,
                     (__bf16*)dyb, sq_err, step_ctr);
  return hipGetLastError();
}

hipError_t launch_eta_mlp3_train_fwd(const void* rec, const float* target, int B, const void* blob,
                                     int H, const NormParams& np, float gscale, void* xf,
                                     void* h1a, float* w3slab, void* dz2, void* dz1, void* dyb,
                                     float* sq_err, int* step_ctr, int num_cus,
                                     hipStream_t stream) {
  switch (H) {
    case 64: return launch_train_fwd_h<64>(rec, target, B, blob, np, gscale, xf, h1a, w3slab, dz2, dz1, dyb, sq_err, step_ctr, num_cus, stream);
    case 128: return launch_train_fwd_h<128>(rec, target, B, blob, np, gscale, xf, h1a, w3slab, dz2, dz1, dyb, sq_err, step_ctr, num_cus, stream);
    case 256: return launch_train_fwd_h<256>(rec, target, B, blob, np, gscale, xf, h1a, w3slab, dz2, dz1, dyb, sq_err, step_ctr, num_cus, stream);
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
