// Wide ETA MLPs (H = 512, 1024): the layer-2 GEMM no longer fits LDS, so W2 streams from L2
// through double-buffered LDS tiles (the "L2-streamed" path; SURVEY C1 sizes the DP bucket for
// H = 1024; the reference artifact is a 2.44 MB model, RO/xgb_eta_model.pkl:1-3).
//
//   big_layer1_kernel  : records -> featurize -> layer 1 (MFMA 32x32x16, W1k fragments from L2)
//                        -> h1 bf16 [B, ld] in the hperm() unit order (16-byte stores); training
//                        also writes xf and the h1a ones-column.
//   gemm256_kernel     : the default for N % 256 == 0, K % 64 == 0 (see its comment below);
//   gemm_nt_kernel     : D = W^T-side GEMM  Z^T[n][m] = sum_k W[n][k] X[m][k]  (both operands
//                        row-major with K contiguous, bf16, fp32 accumulate), 128 x 128 tiles,
//                        4 waves of 64 x 64, K in 32-deep stages through LDS (16-byte row reads,
//                        XOR-swizzled chunks: conflict-free), batch on the lane so every epilogue
//                        reduction over hidden units stays in-lane:
//      EPI_Y    (inference): relu(z + b2) . w3 -> per-(row, 64-unit block) partial sums
//      EPI_H2Y  (training) : same + relu(z + b2) stored bf16 (hperm order) into h2a
//      EPI_STORE(dgrad)    : z stored bf16 (hperm order)
//   big_yreduce_kernel : y = sum of partials + b3 (inference) | + dy, dy operand, squared error
//                        (training)
//   big_dz2_kernel     : dz2 = dy * w3 * relu'(z2) from h2a (training)
//   big_dz2y_kernel    : training: big_yreduce + big_dz2 + the step counter in one launch
//
// Weight layouts (host: routest_amd/ops/mlp_big.py; training: adamw_pack_big_kernel):
//   w1p [H/32][64 lanes][8] bf16 (as mlp3_tile.h), w2k [H][H] bf16 row-major with K columns in
//   hperm order (w2k[n][c] = W2[n][hperm(c)]), w2t [H][H] bf16 row-major = W2^T with K (output
//   unit) columns in hperm order (training only), b2 / w3 f32 in natural order.
#include <atomic>
#include <cstdlib>

#include "common.h"
#include "ops.h"

namespace rt {

namespace {

__host__ __device__ __forceinline__ int hp(int u) { return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1); }

template <int RB>
struct BigRec;
template <>
struct BigRec<16> {
  static __device__ __forceinline__ bf16x8 feat(const void* p, int row, int h, const NormParams& np) {
    return featurize_bf16(reinterpret_cast<const int4*>(p)[row], h, np);
  }
};
template <>
struct BigRec<8> {
  static __device__ __forceinline__ bf16x8 feat(const void* p, int row, int h, const NormParams& np) {
    return featurize8_bf16(reinterpret_cast<const int2*>(p)[row], h, np);
  }
};
template <>
struct BigRec<6> {
  static __device__ __forceinline__ bf16x8 feat(const void* p, int row, int h, const NormParams& np) {
    const unsigned short* s = reinterpret_cast<const unsigned short*>(p) + 3 * (size_t)row;
    return featurize6_bf16((unsigned)s[0] | ((unsigned)s[1] << 16), s[2], h, np);
  }
};

// One wave per 32-row tile: lane (r, h) featurizes row r's half h, H/32 MFMAs, relu, bf16,
// stored as 16-byte chunks at hperm positions 16ks + 8h (= the MFMA B-fragment order).
template <int RB>
__global__ __launch_bounds__(256) void big_layer1_kernel(const void* __restrict__ rec, int B,
                                                         const bf16x8* __restrict__ w1p, int H,
                                                         NormParams np, __bf16* __restrict__ h1,
                                                         int ld, __bf16* __restrict__ xf,
                                                         unsigned* __restrict__ mbits) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int row = tile * 32 + r;
  if (tile * 32 >= B) return;                                   // whole wave leaves together
  const bool valid = row < B;
  bf16x8 xb;
  if (valid) {
    xb = BigRec<RB>::feat(rec, row, h, np);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) xb[j] = (__bf16)0.f;
  }
  if (xf != nullptr && valid) *reinterpret_cast<bf16x8*>(xf + (size_t)row * 16 + 8 * h) = xb;
  __bf16* out = h1 + (size_t)row * ld;
  for (int mt = 0; mt < H / 32; ++mt) {
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    acc = mfma32(w1p[mt * 64 + lane], xb, acc);
    float a[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = acc[e];
    bf16x8 v0, v1;
    relu_cvt_bf16x8(a, &v0);
    relu_cvt_bf16x8(a + 8, &v1);
    if (valid) {
      *reinterpret_cast<bf16x8*>(out + 32 * mt + 8 * h) = v0;
      *reinterpret_cast<bf16x8*>(out + 32 * mt + 16 + 8 * h) = v1;
    }
    if (mbits != nullptr) {             // relu'(z1) of positions 32mt .. 32mt + 31 as one word per row,
      unsigned bits = 0;                // from the stored bf16 values (the dgrad epilogue's mask)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bits |= ((float)v0[k] > 0.f ? 1u : 0u) << (8 * h + k);
        bits |= ((float)v1[k] > 0.f ? 1u : 0u) << (16 + 8 * h + k);
      }
      bits |= (unsigned)__shfl_xor((int)bits, 32);
      // tiled [row / 32][mt][row % 32]: the 32 rows of this tile store 128 contiguous bytes per mt
      if (valid && h == 0) mbits[((size_t)tile * (H / 32) + mt) * 32 + r] = bits;
    }
  }
  if (xf != nullptr && valid && ld > H) {                       // h1a ones-column (db2 input)
    bf16x8 t;
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = (__bf16)0.f;
    if (h == 0) t[0] = (__bf16)1.f;
    *reinterpret_cast<bf16x8*>(out + H + 8 * h) = t;
  }
}

constexpr int GT = 128;          // tile rows (units) and columns (batch rows)
constexpr int GK = 32;           // K per LDS stage
constexpr int EPI_Y = 0, EPI_H2Y = 1, EPI_STORE = 2, EPI_DW1 = 3;

// LDS tile: 128 rows x 64 bytes; 16-byte chunk c of row r at slot c ^ ((r >> 2) & 3) — the 16
// rows a ds_read_b128 lane group reads (lanes {0-3,12-15,20-27} etc.) hit 16 distinct slots.
__device__ __forceinline__ int toff(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); }

struct GemmArgs {
  const __bf16* W;   // [N][ldw]  MFMA A side (output units)
  const __bf16* X;   // [M][ldx]  MFMA B side (batch rows)
  int ldw, ldx, N, M, K;
  const float* b2;   // EPI_Y / EPI_H2Y: bias per unit (natural order)
  const float* w3;   //                 layer-3 weights per unit
  float* ypart;      //                 [M][N/64] partial dots
  __bf16* out;       // EPI_H2Y: h2a, EPI_STORE: output; [M][ldo], unit n at hperm position
  int ldo;
  int tiles_n;       // N / 128
  int st16;          // 256 x 256 epilogue: 16-byte row pieces (1) or 8-byte (0; ROUTEST_GEMM_ST16 A/B knob)
  // EPI_DW1 (256 x 256 loops only): relu' bit mask, words tiled [M / 32][N / 32][32 rows] (bit p % 32
  // of word p / 32 = hperm position p, written by big_layer1), features xf [M][16] and the dW1 slab
  // [M / 256 row tiles][N * 16] (position-major, 16 features)
  const unsigned* mbits = nullptr;
  const __bf16* xf = nullptr;
  float* slab1 = nullptr;
  long long slab1_ld = 0;
};

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char sm[2][2][GT * GK * 2];   // [stage][W|X]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // XCD-aware tile order: hardware round-robins consecutive workgroups over the 8 XCDs; remap
  // so that the tiles_n column blocks of one batch tile run on ONE XCD (its X tile stays in that
  // XCD's L2) — only when the grid divides evenly
  int bid = blockIdx.x;
  const int nb = gridDim.x;
  if ((nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);
  const int tn = bid % a.tiles_n, tm = bid / a.tiles_n;
  const int n0 = tn * GT, m0 = tm * GT;
  const int wn = w & 1, wm = w >> 1;        // wave: units [64wn, +64) x batch [64wm, +64)

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // global -> register staging: each thread moves 2 chunks of W and 2 of X per stage (rows of
  // X past M are clamped to row M-1: their products land in columns that are never stored)
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  i32x4 rw[2], rx[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u, r = c >> 2, ch = c & 3;
      rw[u] = *reinterpret_cast<const i32x4*>(a.W + (size_t)(n0 + r) * a.ldw + k0 + 8 * ch);
      const int mr = min(m0 + r, a.M - 1);
      rx[u] = *reinterpret_cast<const i32x4*>(a.X + (size_t)mr * a.ldx + k0 + 8 * ch);
    }
  };
  auto lstore = [&](int s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u, r = c >> 2, ch = c & 3;
      *reinterpret_cast<i32x4*>(&sm[s][0][toff(r, ch)]) = rw[u];
      *reinterpret_cast<i32x4*>(&sm[s][1][toff(r, ch)]) = rx[u];
    }
  };
  const int nk = a.K / GK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * GK);          // in flight under this stage's MFMAs
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 2 * ks + (lane >> 5);
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = *reinterpret_cast<const bf16x8*>(&sm[s][0][toff(64 * wn + 32 * i + (lane & 31), ch)]);
        fb[i] = *reinterpret_cast<const bf16x8*>(&sm[s][1][toff(64 * wm + 32 * i + (lane & 31), ch)]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
    if (kt + 1 < nk) {
      lstore(s ^ 1);                                   // the other buffer: consumed last stage
      __syncthreads();
    }
  }

  // epilogue: acc[i][j] = Z^T[units 64wn + 32i + (e&3) + 8(e>>2) + 4h][batch 64wm + 32j + (l&31)]
  const int h = lane >> 5, col = lane & 31;
  if constexpr (EPI == EPI_STORE) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + 64 * wm + 32 * j + col;
      if (m >= a.M) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ub = n0 + 64 * wn + 32 * i;
        // registers 0-7 are units ub + 4h + {0..3}, ub + 8 + 4h + {0..3}: hperm positions
        // ub + 8h + {0..7}; registers 8-15 the same +16
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (__bf16)acc[i][j][8 * s2 + q];
          *reinterpret_cast<bf16x8*>(a.out + (size_t)m * a.ldo + ub + 16 * s2 + 8 * h) = o;
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + 64 * wm + 32 * j + col;
      float ys = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ub = n0 + 64 * wn + 32 * i;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int e = 8 * s2 + q;
            const int u = ub + (e & 3) + 8 * (e >> 2) + 4 * h;
            const float v = relu_f(acc[i][j][e] + a.b2[u]);
            ys = __builtin_fmaf(v, a.w3[u], ys);
            o[q] = (__bf16)v;
          }
          if constexpr (EPI == EPI_H2Y) {
            if (m < a.M) *reinterpret_cast<bf16x8*>(a.out + (size_t)m * a.ldo + ub + 16 * s2 + 8 * h) = o;
          }
        }
      }
      ys += __shfl_xor(ys, 32);
      if (h == 0 && m < a.M) a.ypart[(size_t)m * (a.N / 64) + (n0 >> 6) + wn] = ys;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// gemm256_kernel: the same three products on 256 x 256 tiles (units x batch rows), 8 waves of
// 128 x 64 on mfma_f32_16x16x32_bf16 (32 accumulators of 4 = 128 VGPRs), K in 64-deep stages.
// Both operand tiles go global -> LDS with global_load_lds_dwordx4 (no VGPR staging, no ds_write
// pass): each wave-instruction writes 1 KB of the LDS image lane-linearly, so the XOR swizzle is
// applied to the per-lane GLOBAL address — row r's 16-byte chunk c lives at slot c ^ ((r >> 1) & 7)
// of its 128-byte LDS row, which makes each 16-lane group of a ds_read_b128 fragment read (16
// consecutive rows, one chunk) hit 16 distinct 16-byte bank groups.  Two stages (128 KB LDS, one
// workgroup per CU): the loads of stage k+1 are in flight under stage k's 64 MFMAs per wave.
// Workgroups are remapped XCD-aware (bijective for any grid) so the N/256 unit tiles of one
// batch-row block run on one XCD and share its X tile through that XCD's L2.  (A ring of four
// 32-deep stages with three in flight and all 12 fragment reads issued before the MFMAs measured
// SLOWER at the H = 1024 trainer's shape: 174 vs 161 us, profiles/gemm_probe_r4p.jsonl; so did reading
// both k-steps' fragments up front, 166 vs 161 us, r4ap.)
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int G2T = 256, G2K = 64;
constexpr int G2_STAGE = 2 * G2T * G2K * 2;          // A + B tile bytes per stage (64 KB)

// epilogue of both 256 x 256 K loops: acc[i][j] element e = Z^T[unit n0 + 128wu + 16i + 4g + e][row
// m0 + 64wr + 16j + fr] (g = lane >> 4); hperm swaps unit bits 2, 3: stored position 16i + 4 swap2(g) + e
// One row's pieces of fragments 2p and 2p + 1 as 16-byte stores (the 8-byte stores made the epilogue
// store-issue bound): lane l (g < 2, stored position 4gp) and lane l ^ 32 (position 4gp + 4) hold
// adjacent 8-byte pieces of both fragments; each swaps one piece with its partner, so the low lane
// stores fragment 2p's 16 bytes and the high lane fragment 2p + 1's.  Both lanes of a pair have the
// same row, so they are active together.
__device__ __forceinline__ void g256_store_pair(__bf16* row, int p, int gp, bool hi, bf16x4 o0, bf16x4 o1) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x2 send = __builtin_bit_cast(u32x2, hi ? o0 : o1);
  const u32x2 keep = __builtin_bit_cast(u32x2, hi ? o1 : o0);
  u32x2 recv;
  recv[0] = (unsigned)__shfl_xor((int)send[0], 32);
  recv[1] = (unsigned)__shfl_xor((int)send[1], 32);
  const u32x4 v = hi ? (u32x4){recv[0], recv[1], keep[0], keep[1]} : (u32x4){keep[0], keep[1], recv[0], recv[1]};
  *reinterpret_cast<u32x4*>(row + 16 * (2 * p + (hi ? 1 : 0)) + 4 * (hi ? gp - 1 : gp)) = v;
}

// EPI_DW1: the training dgrad dh1 = dz2 W2 consumed in place.  dh1 is needed only for dW1 =
// (dh1 * relu'(z1))^T [x | 1], so instead of storing it (128 MB at H = 1024, 64k rows) and re-reading it
// with the mask in a wgrad launch (61 us, profiles/train_h1024_64k_kernel_stats_r6h.csv), the tile
// rounds it to bf16 exactly as the store did, masks it with h1a, and multiplies it by the tile's 256
// feature rows on MFMA: one [256 positions][16] partial per row tile, summed by wgrad_reduce.
//   LDS (the K loop's buffers, free after a barrier): zt [256 positions][256 k] bf16 and xt [16][256 k]
//   bf16, 512-byte rows, 16-byte chunk ch of row r at slot ch ^ (r & 31) (the 16 rows one fragment
//   read touches land in 16 distinct slots).  k orders the tile's rows so a lane's 4 rows of one
//   position are adjacent: row 64wr + 16j + fr -> k = 64wr + 4fr + j (any order works: A and B agree).
constexpr int DW1_ZT = 256 * 512, DW1_LDS = DW1_ZT + 16 * 512;
__device__ __forceinline__ int dw1_off(int r, int k) { return r * 512 + ((((k >> 3) ^ (r & 31))) << 4) + ((k & 7) << 1); }

template <int EPI>
__device__ __forceinline__ void g256_epilogue(const GemmArgs& a, f32x4 (&acc)[8][4], int n0, int m0, int wu,
                                              int wr, int lane, unsigned char* lds = nullptr) {
  const int fr = lane & 15, g = lane >> 4, gp = ((g & 1) << 1) | (g >> 1);
  const bool hi = lane >= 32;
  const int ub = n0 + 128 * wu;
  if constexpr (EPI == EPI_DW1) {
    const int tid = threadIdx.x;
    // global loads first (they do not touch LDS): the tile's features and the relu' mask words
    // feature row t >> 1, features 8 (t & 1) .. + 7 (rows past M: zeros)
    const int xr = tid >> 1, xh = tid & 1;
    bf16x8 xv;
    if (m0 + xr < a.M) {
      xv = *reinterpret_cast<const bf16x8*>(a.xf + (size_t)(m0 + xr) * 16 + 8 * xh);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[q] = (__bf16)0.f;
    }
    // relu'(z1) of position 128wu + 16i + 4gp + e: word (ub >> 5) + i / 2 of row m, bit 16 (i & 1) +
    // 4gp + e; words tiled [m / 32][word][m % 32] (big_layer1): 16 lanes read 64 contiguous bytes
    const int wpr = a.N / 32;
    unsigned mk[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + 64 * wr + 16 * j + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        mk[j][q] = m < a.M ? a.mbits[((size_t)(m >> 5) * wpr + (ub >> 5) + q) * 32 + (m & 31)] : 0u;
    }
    __syncthreads();                                      // every wave is past its last K-loop read
    {
      const int k = 64 * (xr >> 6) + 4 * (xr & 15) + ((xr >> 4) & 3);
#pragma unroll
      for (int q = 0; q < 8; ++q) *reinterpret_cast<__bf16*>(lds + DW1_ZT + dw1_off(8 * xh + q, k)) = xv[q];
    }
    // dz1 = bf16(dh1) * relu'(z1), rows j = 0..3 of a position -> 4 adjacent k
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int bit = 16 * (i & 1) + 4 * gp + e;
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (mk[j][i >> 1] >> bit) & 1u ? (__bf16)acc[i][j][e] : (__bf16)0.f;
        const int pl = 128 * wu + 16 * i + 4 * gp + e;
        *reinterpret_cast<bf16x4*>(lds + dw1_off(pl, 64 * wr + 4 * fr)) = v;
      }
    }
    __syncthreads();
    // [256 positions][16] = zt (A: 16 positions x 32 k) x xt^T (B: 32 k x 16 features); wave w: position
    // blocks 2w, 2w + 1
    const int w = tid >> 6;
    float* orow = a.slab1 + (size_t)(m0 / 256) * a.slab1_ld + (size_t)n0 * 16;
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int pb = 16 * (2 * w + bb);
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int k = 32 * kk + 8 * g;
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(lds + dw1_off(pb + fr, k));
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(lds + DW1_ZT + dw1_off(fr, k));
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, d, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) orow[(pb + 4 * g + e) * 16 + fr] = d[e];
    }
  } else if constexpr (EPI == EPI_STORE) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + 64 * wr + 16 * j + fr;
      if (m >= a.M) continue;
      bf16x4 o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) o[i][e] = (__bf16)acc[i][j][e];
      if (a.st16) {
#pragma unroll
        for (int p = 0; p < 4; ++p) g256_store_pair(a.out + (size_t)m * a.ldo + ub, p, gp, hi, o[2 * p], o[2 * p + 1]);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<bf16x4*>(a.out + (size_t)m * a.ldo + ub + 16 * i + 4 * gp) = o[i];
      }
    }
  } else {
    f32x4 bv[8], wv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bv[i] = *reinterpret_cast<const f32x4*>(a.b2 + ub + 16 * i + 4 * g);
      wv[i] = *reinterpret_cast<const f32x4*>(a.w3 + ub + 16 * i + 4 * g);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + 64 * wr + 16 * j + fr;
      float ys[2] = {0.f, 0.f};
      bf16x4 o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = relu_f(acc[i][j][e] + bv[i][e]);
          ys[i >> 2] = __builtin_fmaf(v, wv[i][e], ys[i >> 2]);
          o[i][e] = (__bf16)v;
        }
      }
      if constexpr (EPI == EPI_H2Y) {
        if (m < a.M) {
          if (a.st16) {
#pragma unroll
            for (int p = 0; p < 4; ++p) g256_store_pair(a.out + (size_t)m * a.ldo + ub, p, gp, hi, o[2 * p], o[2 * p + 1]);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<bf16x4*>(a.out + (size_t)m * a.ldo + ub + 16 * i + 4 * gp) = o[i];
          }
        }
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        ys[hh] += __shfl_xor(ys[hh], 16);
        ys[hh] += __shfl_xor(ys[hh], 32);
      }
      if (g == 0 && m < a.M) {
        float* yp = a.ypart + (size_t)m * (a.N / 64) + (ub >> 6);
        yp[0] = ys[0];
        yp[1] = ys[1];
      }
    }
  }
}


template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm2[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int bid = blockIdx.x;
  {
    const int nb = gridDim.x, xcd = bid & 7, q = nb >> 3, r = nb & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tn = bid % a.tiles_n, tm = bid / a.tiles_n;
  const int n0 = tn * G2T, m0 = tm * G2T;
  const int wu = w & 1, wr = w >> 1;                 // units [128wu, +128) x rows [64wr, +64)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // staging: thread t moves chunk q*512 + t of each tile (q = 0..3): row q*64 + (t >> 3), LDS
  // slot t & 7, global chunk (t & 7) ^ ((t >> 4) & 7) — the same for every q
  const int srow = tid >> 3, schunk = (tid & 7) ^ ((tid >> 4) & 7);
  const __bf16* ga = a.W + (size_t)(n0 + srow) * a.ldw + 8 * schunk;
  const __bf16* gb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) gb[q] = a.X + (size_t)min(m0 + 64 * q + srow, a.M - 1) * a.ldx + 8 * schunk;
  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](int kt, int s) {
    unsigned char* st = sm2 + s * G2_STAGE;
    const int k0 = kt * G2K;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_global_load_lds((const void*)(ga + (size_t)(64 * q) * a.ldw + k0),
                                       (lds_void*)(st + (q * 8 + w) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gb[q] + k0),
                                       (lds_void*)(st + G2T * G2K * 2 + (q * 8 + w) * 1024), 16, 0, 0);
    }
  };

  // fragment offsets: row 16i + (lane & 15) of the wave's block, k chunk 4ks + (lane >> 4)
  const int fr = lane & 15, sw = (lane >> 1) & 7;
  const int offa = (128 * wu + fr) * 128, offb = G2T * G2K * 2 + (64 * wr + fr) * 128;
  const int nk = a.K / G2K;
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, s ^ 1);
    const unsigned char* st = sm2 + s * G2_STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int co = ((4 * ks + (lane >> 4)) ^ sw) << 4;
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(st + offa + i * 2048 + co);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(st + offb + j * 2048 + co);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stage k+1 landed
    __syncthreads();                                    // ... and stage k fully read
  }

  g256_epilogue<EPI>(a, acc, n0, m0, wu, wr, lane, sm2);
}

// ---------------------------------------------------------------------------------------------
// gemm256p_kernel: gemm256_kernel's tile, waves, MFMA and epilogue with the K loop as a PHASE
// pipeline (cdna_hip_programming.md §5, "The 256² 8-phase template").  gemm256_kernel drains its
// loads and barriers once per 64-deep K-tile with both waves of a SIMD parked at once (PMC r4as: a
// third of the wave cycles wait there).  Here:
//   * each K-tile runs as 4 phases, one per quadrant of the wave's 128 x 64 output (64 units x 32
//     rows, 16 MFMAs): P1 reads the B0 and A0 fragments, P2 B1, P3 A1, P4 none (B0 is still in
//     registers) — 24 ds_read_b128 per K-tile, as before;
//   * each LDS buffer is four 16 KB regions (A units half ih = rows 128wu + 64ih + 0..63 of both
//     unit halves, B rows half jh = rows 64wr + 32jh + 0..31 of all four row quarters), so phase
//     (ih, jh) reads exactly regions A_ih and B_jh; ONE region's global_load_lds (2 per thread) is
//     issued per phase: P1 B1(u+1), P2 A1(u+1), P3 A0(u+2), P4 B0(u+2) — each region restaged >= 2
//     phases after its last read, and K-tile u+1 retired by P4's counted vmcnt(4) (the youngest
//     two regions stay in flight across the raw barriers; never vmcnt(0) in the steady state);
//   * the two waves of a SIMD (w, w + 4) are in different groups and group 1 runs ONE barrier behind
//     group 0, so one group's MFMAs run while the other group reads its fragments and issues its
//     loads (s_setprio 1 around the MFMAs).
// Hazard bookkeeping (barrier indices, group 0 phase p: mid 2p, end 2p+1; group 1: 2p+1, 2p+2): a
// region last read in phase r is retired by both groups at barrier 2r+2, which group 0's phase r+2
// loads follow; a K-tile's data is retired by both groups' P4 waits before barrier 2p+1, which every
// read of the next K-tile follows.
constexpr int GP_REGION = 128 * 128;                 // bytes: 128 rows x 64 k bf16
constexpr int GP_BUF = 4 * GP_REGION;                 // A0 | A1 | B0 | B1

#define GP_BARRIER()                      \
  do {                                    \
    __builtin_amdgcn_sched_barrier(0);    \
    __builtin_amdgcn_s_barrier();         \
    __builtin_amdgcn_sched_barrier(0);    \
  } while (0)

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm256p_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm2[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int bid = blockIdx.x;
  {
    const int nb = gridDim.x, xcd = bid & 7, q = nb >> 3, r = nb & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tn = bid % a.tiles_n, tm = bid / a.tiles_n;
  const int n0 = tn * G2T, m0 = tm * G2T;
  const int wu = w >> 2, wr = w & 3;                 // group = wu; units [128wu, +128) x rows [64wr, +64)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // staging: wave w's instruction q of a region writes LDS rows 64q + 8w + (lane >> 3), 16-byte slot
  // lane & 7, from global chunk slot ^ ((row >> 1) & 7) (the read side's swizzle)
  const int srow = 8 * w + (lane >> 3);
  const int sch = (lane & 7) ^ ((srow >> 1) & 7);
  const __bf16* gA = a.W + (size_t)(n0 + srow) * a.ldw + 8 * sch;     // + (128q + 64ih) rows
  const __bf16* gB[2][2];
#pragma unroll
  for (int jh = 0; jh < 2; ++jh)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int row = m0 + 128 * q + 64 * (w >> 2) + 32 * jh + 8 * (w & 3) + (lane >> 3);
      gB[jh][q] = a.X + (size_t)min(row, a.M - 1) * a.ldx + 8 * sch;
    }
  typedef __attribute__((address_space(3))) void lds_void;
  // region reg (0 A0, 1 A1, 2 B0, 3 B1) of K-tile kt
  auto issue = [&](int kt, int reg) {
    unsigned char* dst = sm2 + (kt & 1) * GP_BUF + reg * GP_REGION + w * 1024;
    const int k0 = kt * G2K;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const __bf16* src = reg < 2 ? gA + (size_t)(128 * q + 64 * reg) * a.ldw + k0 : gB[reg - 2][q] + k0;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + q * 8192), 16, 0, 0);
    }
  };

  const int fr = lane & 15, sw = (lane >> 1) & 7;
  const int co[2] = {((lane >> 4) ^ sw) << 4, ((4 + (lane >> 4)) ^ sw) << 4};
  const int offA = (64 * wu + fr) * 128, offB = 2 * GP_REGION + (32 * wr + fr) * 128;
  bf16x8 fa[4][2], fb[2][2][2];                      // A half [i'][ks]; B halves [jh][j'][ks]
  auto readA = [&](const unsigned char* buf, int ih) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fa[i][ks] = *reinterpret_cast<const bf16x8*>(buf + ih * GP_REGION + offA + i * 2048 + co[ks]);
  };
  auto readB = [&](const unsigned char* buf, int jh) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        fb[jh][j][ks] = *reinterpret_cast<const bf16x8*>(buf + jh * GP_REGION + offB + j * 2048 + co[ks]);
  };
  auto quad = [&](int ih, int jh) {
    GP_BARRIER();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * ih + i][2 * jh + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[jh][j][ks], acc[4 * ih + i][2 * jh + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    GP_BARRIER();
  };

  const int nk = a.K / G2K;
  issue(0, 0);
  issue(0, 1);
  issue(0, 2);
  issue(0, 3);
  if (nk > 1) {
    issue(1, 0);
    issue(1, 2);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  GP_BARRIER();
  if (wu == 1) GP_BARRIER();                          // group 1: one barrier behind
  for (int u = 0; u < nk; ++u) {
    const unsigned char* buf = sm2 + (u & 1) * GP_BUF;
    // P1: B0 + A0; restage B1 of u + 1
    readB(buf, 0);
    readA(buf, 0);
    if (u + 1 < nk) issue(u + 1, 3);
    quad(0, 0);
    // P2: B1; restage A1 of u + 1
    readB(buf, 1);
    if (u + 1 < nk) issue(u + 1, 1);
    quad(0, 1);
    // P3: A1; restage A0 of u + 2
    readA(buf, 1);
    if (u + 2 < nk) issue(u + 2, 0);
    quad(1, 1);
    // P4: no reads; restage B0 of u + 2, then retire K-tile u + 1
    if (u + 2 < nk) {
      issue(u + 2, 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    quad(1, 0);
  }
  if (wu == 0) GP_BARRIER();                          // equal barrier counts on exit
  g256_epilogue<EPI>(a, acc, n0, m0, wu, wr, lane, sm2);
}
#undef GP_BARRIER

// ---------------------------------------------------------------------------------------------
// mlp_big_fused_kernel (inference): records -> featurize -> layer 1 -> layer 2 -> relu.w3 partials
// in ONE launch, so h1 never goes to HBM (at H = 1024 that is 2 KB per row written by a layer-1
// kernel and read back by the GEMM: 23 % of the unfused time).  Tiles and waves as gemm256_kernel
// (256 units x 256 rows, 8 waves of 128 x 64); only W2 is staged (global_load_lds, 2 x 32 KB).
// Each wave computes the B fragments of its own 64 rows per 64-deep K stage on MFMA:
//   h1^T block = W1k[16 units][16] . x^T[16][16 rows]   (mfma_f32_16x16x16bf16_1k, K = 16: the 12
//   features + hi/lo-split inputs + the two constant-1 slots that carry b1)
// lane (g = l >> 4, row l & 15) gets units 4g .. 4g+3 of the block; two blocks s = 0, 1 of a
// 32-unit chunk, relu'd and packed, are exactly one 16x16x32 B fragment when the chunk's K order
// is p = 8g + 4s + j  <->  unit 16s + 4g + j — the host packs W2's columns in that order (w2f).
// x^T stays in 8 VGPRs for the whole tile (featurized once); W1k fragments (w1q) sit in LDS.
struct FusedArgs {
  const void* rec;
  int B, H;
  const __bf16* w1q;   // [H/16][64 lanes][4]: W1k[16ub + (l & 15)][4(l >> 4) + j]
  const __bf16* w2f;   // [H][H] row-major, K columns in the chunk order above
  const float* b2;
  const float* w3;
  float* ypart;        // [B][H/64]
  int tiles_n;
  NormParams np;
};

typedef short s16x4v __attribute__((ext_vector_type(4)));

template <int RB, int NS>
__global__ __launch_bounds__(512, 1) void mlp_big_fused_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm3[];   // [NS x 32 KB W2 | w1q]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int bid = blockIdx.x;
  {
    const int nb = gridDim.x, xcd = bid & 7, q = nb >> 3, r = nb & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tn = bid % a.tiles_n, tm = bid / a.tiles_n;
  const int n0 = tn * G2T, m0 = tm * G2T;
  const int wu = w & 1, wr = w >> 1;
  const int g = lane >> 4, fr = lane & 15;
  constexpr int ABYTES = G2T * G2K * 2;              // one W2 stage
  unsigned char* w1s = sm3 + NS * ABYTES;

  // W2 stage 0 in flight first, then W1k fragments into LDS (plain 16-byte copies) and the
  // features of the wave's 64 rows (x^T fragments: features 4g .. 4g+3 of row 16jr + fr)
  const int srow = tid >> 3, schunk = (tid & 7) ^ ((tid >> 4) & 7);
  const __bf16* ga = a.w2f + (size_t)(n0 + srow) * a.H + 8 * schunk;
  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](int kt, int s) {
    unsigned char* st = sm3 + s * ABYTES;
    const int k0 = kt * G2K;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(ga + (size_t)(64 * q) * a.H + k0),
                                       (lds_void*)(st + (q * 8 + w) * 1024), 16, 0, 0);
  };
  {
    const int n16 = a.H * 16 * 2 / 16;               // w1q bytes / 16
    const int4* src = reinterpret_cast<const int4*>(a.w1q);
    int4* dst = reinterpret_cast<int4*>(w1s);
    for (int i = tid; i < n16; i += 512) dst[i] = src[i];
  }
  s16x4v xk[4];
#pragma unroll
  for (int jr = 0; jr < 4; ++jr) {
    const int row = min(m0 + 64 * wr + 16 * jr + fr, a.B - 1);
    const bf16x8 f8 = BigRec<RB>::feat(a.rec, row, g >> 1, a.np);
    const bf16x4 x4 = (g & 1) ? __builtin_shufflevector(f8, f8, 4, 5, 6, 7)
                              : __builtin_shufflevector(f8, f8, 0, 1, 2, 3);
    xk[jr] = __builtin_bit_cast(s16x4v, x4);
  }
  // the features are finished (and their record loads retired) BEFORE the first W2 DMA: a use
  // of an ordinary load's result below a global_load_lds makes the compiler drain every
  // outstanding DMA with vmcnt(0)
#pragma unroll
  for (int jr = 0; jr < 4; ++jr) asm volatile("" : "+v"(xk[jr]) :: "memory");
  const int nk = a.H / G2K;
  issue(0, 0);
  if constexpr (NS == 3) {
    // stage 1 stays in flight across the first barrier: counted vmcnt + raw s_barrier (a
    // __syncthreads() fence would drain every outstanding global_load_lds)
    if (nk > 1) {
      issue(1, 1);
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int sw = (lane >> 1) & 7;
  const int offa = (128 * wu + fr) * 128;
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt % NS;
    // the buffer refilled here was last read in iteration kt - 1, which every wave has left
    if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned char* st = sm3 + s * ABYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // layer 1 for units kt*64 + 32ks .. +31 (two 16-unit blocks) x the wave's 4 row blocks
      const int ub = kt * 4 + 2 * ks;
      const s16x4v w10 = *reinterpret_cast<const s16x4v*>(w1s + ((ub * 64 + lane) << 3));
      const s16x4v w11 = *reinterpret_cast<const s16x4v*>(w1s + (((ub + 1) * 64 + lane) << 3));
      bf16x8 fb[4];
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w10, xk[jr], z, 0, 0, 0);
        const f32x4 c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w11, xk[jr], z, 0, 0, 0);
        float t[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
        relu_cvt_bf16x8(t, &fb[jr]);
      }
      const int co = ((4 * ks + g) ^ sw) << 4;
      bf16x8 fa[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(st + offa + i * 2048 + co);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (NS == 3) {
      // stage kt + 1 landed (stage kt + 2, if issued, stays in flight), then everyone is past kt
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // epilogue (as gemm256_kernel EPI_Y): relu(z + b2) . w3 per (row, 64-unit block)
  const int ub0 = n0 + 128 * wu;
  f32x4 bv[8], wv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    bv[i] = *reinterpret_cast<const f32x4*>(a.b2 + ub0 + 16 * i + 4 * g);
    wv[i] = *reinterpret_cast<const f32x4*>(a.w3 + ub0 + 16 * i + 4 * g);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + 64 * wr + 16 * j + fr;
    float ys[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) ys[i >> 2] = __builtin_fmaf(relu_f(acc[i][j][e] + bv[i][e]), wv[i][e], ys[i >> 2]);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      ys[hh] += __shfl_xor(ys[hh], 16);
      ys[hh] += __shfl_xor(ys[hh], 32);
    }
    if (g == 0 && m < a.B) {
      float* yp = a.ypart + (size_t)m * (a.H / 64) + (ub0 >> 6);
      yp[0] = ys[0];
      yp[1] = ys[1];
    }
  }
}

// y = sum_j ypart[m][j] + b3 (fixed order: deterministic).  Training (target != null): dy, the
// bf16 dy operand [B,8] (col 0), squared error.
__global__ __launch_bounds__(256) void big_yreduce_kernel(const float* __restrict__ ypart, int nparts,
                                                          int B, float b3, const float* __restrict__ b3p,
                                                          float* __restrict__ y,
                                                          const float* __restrict__ target,
                                                          float gscale, float* __restrict__ dy,
                                                          __bf16* __restrict__ dyb,
                                                          float* __restrict__ sq_err) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B) return;
  const float* p = ypart + (size_t)m * nparts;
  float s = 0.f;
  for (int j = 0; j < nparts; ++j) s += p[j];
  const float yy = s + (b3p != nullptr ? *b3p : b3);     // training: b3 lives on the device
  if (y != nullptr) y[m] = yy;
  if (target != nullptr) {
    const float diff = yy - target[m];
    const float d = gscale * diff;
    dy[m] = d;
    sq_err[m] = diff * diff;
    bf16x8 dv;
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = (__bf16)0.f;
    dv[0] = (__bf16)d;
    *reinterpret_cast<bf16x8*>(dyb + (size_t)m * 8) = dv;
  }
}

// dz2[m][c] = dy[m] * w3[hperm(c)] * (h2a[m][c] > 0), 8 columns per thread (hperm order both).
__global__ __launch_bounds__(256) void big_dz2_kernel(const __bf16* __restrict__ h2a, int lda,
                                                      const float* __restrict__ dy,
                                                      const float* __restrict__ w3, int B, int H,
                                                      __bf16* __restrict__ dz2) {
  const long long i8 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = H / 8;
  if (i8 >= (long long)B * per) return;
  const long long m = i8 / per;
  const int c = (int)(i8 - m * per) * 8;
  const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h2a + m * lda + c);
  const float d = dy[m];
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (__bf16)(((float)hv[q] > 0.f) ? d * w3[hp(c + q)] : 0.f);
  *reinterpret_cast<bf16x8*>(dz2 + m * H + c) = o;
}

// Training: dy (+ its bf16 operand row, squared error) and dz2 for one row per wave, in one
// launch (was big_yreduce + big_dz2 + a step-counter increment): lanes < nparts fetch the row's
// relu.w3 partials, a butterfly sums them, and the wave then writes the row's H dz2 values
// (8 per lane per pass).  Block 0 advances the device step counter for adamw_pack_big.
__global__ __launch_bounds__(256) void big_dz2y_kernel(const float* __restrict__ ypart, int nparts,
                                                       int B, int H, const float* __restrict__ b3p,
                                                       const float* __restrict__ target, float gscale,
                                                       float* __restrict__ dy, __bf16* __restrict__ dyb,
                                                       float* __restrict__ sq_err,
                                                       const __bf16* __restrict__ h2a, int lda,
                                                       const float* __restrict__ w3,
                                                       __bf16* __restrict__ dz2, int* __restrict__ step_ctr) {
  if (step_ctr != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *step_ctr += 1;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= B) return;                                       // whole wave leaves together
  float s = lane < nparts ? ypart[(size_t)m * nparts + lane] : 0.f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  const float diff = s + b3p[0] - target[m];
  const float d = gscale * diff;
  if (lane == 0) {
    dy[m] = d;
    sq_err[m] = diff * diff;
    bf16x8 dv;
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = (__bf16)0.f;
    dv[0] = (__bf16)d;
    *reinterpret_cast<bf16x8*>(dyb + (size_t)m * 8) = dv;
  }
  for (int c = 8 * lane; c < H; c += 512) {
    const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h2a + (size_t)m * lda + c);
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (__bf16)(((float)hv[q] > 0.f) ? d * w3[hp(c + q)] : 0.f);
    *reinterpret_cast<bf16x8*>(dz2 + (size_t)m * H + c) = o;
  }
}

// The same step with dW3 | db3 folded in (was a separate wgrad launch that streamed h2a a second
// time): S workgroups of 16 waves, one split-K slice each, write slab[s][0 .. H+16) = sum over the
// slice's rows of dy * [relu(z2) | 1 | 0...] — the layout wgrad_reduce already sums.  A lane keeps its
// 8 (H = 512) or 16 (H = 1024) columns' w3 values and dW3 partials in registers for all its rows;
// rows go two at a time so each wave has two independent load chains in flight; the row loop never
// re-reads w3 (the round-2 kernel gathered w3[hperm(c)] per element, 8 loads per 16-byte output).
template <int KC>
__global__ __launch_bounds__(1024) void big_dz2y_w3_kernel(const float* __restrict__ ypart, int nparts, int B,
                                                           const float* __restrict__ b3p,
                                                           const float* __restrict__ target, float gscale,
                                                           float* __restrict__ dy, __bf16* __restrict__ dyb,
                                                           float* __restrict__ sq_err,
                                                           const __bf16* __restrict__ h2a, int lda,
                                                           const float* __restrict__ w3,
                                                           __bf16* __restrict__ dz2, int* __restrict__ step_ctr,
                                                           float* __restrict__ slab, long long slab_ld, int S) {
  constexpr int H = 512 * KC;
  __shared__ float red[16][H];
  __shared__ float dred[16];
  if (step_ctr != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *step_ctr += 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int s = blockIdx.x;
  const int r0 = (int)((long long)s * B / S), r1 = (int)((long long)(s + 1) * B / S);
  float w3r[KC][8], acc[KC][8];
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      w3r[k][q] = w3[hp(8 * lane + 512 * k + q)];
      acc[k][q] = 0.f;
    }
  const float b3 = b3p[0];
  float dsum = 0.f;
  auto row_dy = [&](int m) {
    float t = lane < nparts ? ypart[(size_t)m * nparts + lane] : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
    const float diff = t + b3 - target[m];
    const float d = gscale * diff;
    if (lane == 0) {
      dy[m] = d;
      sq_err[m] = diff * diff;
      bf16x8 dv;
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[j] = (__bf16)0.f;
      dv[0] = (__bf16)d;
      *reinterpret_cast<bf16x8*>(dyb + (size_t)m * 8) = dv;
    }
    return d;
  };
  auto row_out = [&](int m, float d, const bf16x8 (&hv)[KC]) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      bf16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float h = (float)hv[k][q];                 // relu(z2) >= 0
        o[q] = (__bf16)(h > 0.f ? d * w3r[k][q] : 0.f);
        acc[k][q] = __builtin_fmaf(d, h, acc[k][q]);
      }
      *reinterpret_cast<bf16x8*>(dz2 + (size_t)m * H + 8 * lane + 512 * k) = o;
    }
    dsum += d;
  };
  int m = r0 + wv;
  for (; m + 16 < r1; m += 32) {                         // rows m and m + 16 together
    bf16x8 ha[KC], hb[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      ha[k] = *reinterpret_cast<const bf16x8*>(h2a + (size_t)m * lda + 8 * lane + 512 * k);
      hb[k] = *reinterpret_cast<const bf16x8*>(h2a + (size_t)(m + 16) * lda + 8 * lane + 512 * k);
    }
    const float da = row_dy(m), db = row_dy(m + 16);
    row_out(m, da, ha);
    row_out(m + 16, db, hb);
  }
  if (m < r1) {
    bf16x8 ha[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
      ha[k] = *reinterpret_cast<const bf16x8*>(h2a + (size_t)m * lda + 8 * lane + 512 * k);
    row_out(m, row_dy(m), ha);
  }
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int q = 0; q < 8; ++q) red[wv][8 * lane + 512 * k + q] = acc[k][q];
  if (lane == 0) dred[wv] = dsum;
  __syncthreads();
  float* out = slab + (long long)s * slab_ld;
  for (int c = threadIdx.x; c < H; c += 1024) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][c];
    out[c] = t;
  }
  if (threadIdx.x < 16) {                                // db3 (the ones column), zero padding
    float t = 0.f;
    if (threadIdx.x == 0)
      for (int w = 0; w < 16; ++w) t += dred[w];
    out[H + threadIdx.x] = t;
  }
}

struct AdamWBigArgs {
  float lr, beta1, beta2, eps, wd;
  int warmup, total_steps;
  float min_lr_ratio;
  int update, H;
};

__device__ __forceinline__ float sched_lr_big(const AdamWBigArgs& a, int t) {
  float lr = a.lr;
  if (a.warmup > 0 && t < a.warmup) lr *= (float)t / (float)a.warmup;
  if (a.total_steps > 0 && t > a.warmup) {
    const float prog = fminf(1.f, (float)(t - a.warmup) / fmaxf(1.f, (float)(a.total_steps - a.warmup)));
    lr *= a.min_lr_ratio + (1.f - a.min_lr_ratio) * 0.5f * (1.f + cosf(3.14159265f * prog));
  }
  return lr;
}

// AdamW on the flat fp32 master params (W1[H][12] | b1 | W2[H][H] | b2 | w3 | b3) + re-pack of
// the wide trainer's operands: w1p fragments (b1 as bf16 hi/lo in k = 14, 15), w2k[o][hp(i)],
// w2t[i][hp(o)] (bf16), b2 / w3 / b3 f32.  Gradient bucket rows/columns are hperm positions
// (gW2a[hp(o)][hp(i)], gW3a[hp(o)], gW1a[hp(o)][16]): every activation is stored in that order.
__device__ __forceinline__ void adamw_big_elem(long long ep, float* __restrict__ P, const float* __restrict__ G,
                                               float* __restrict__ M, float* __restrict__ V,
                                               __bf16* __restrict__ w1p, __bf16* __restrict__ w2k,
                                               __bf16* __restrict__ w2t, float* __restrict__ b2,
                                               float* __restrict__ w3, float* __restrict__ b3,
                                               const int* __restrict__ step, const AdamWBigArgs& a) {
  const int H = a.H, LDG = H + 16;
  const long long OFF_B1 = 12LL * H, OFF_W2 = 13LL * H, OFF_B2 = OFF_W2 + (long long)H * H,
                  OFF_W3 = OFF_B2 + H, OFF_B3 = OFF_W3 + H, N = OFF_B3 + 1;
  const float* gW2a = G;
  const float* gW3a = G + (long long)H * LDG;
  const float* gW1a = gW3a + LDG;
  // the W2 block (H*H of the N parameters) is handled by adamw_w2_tile_kernel; this grid covers
  // the rest: index e' < OFF_W2 maps to itself, the others skip the W2 range
  const long long e = ep < OFF_W2 ? ep : ep + (long long)H * H;
  if (e >= N) return;
  float g;
  bool decay = false;
  int o = 0, i = 0;
  if (e < OFF_B1) {
    o = (int)(e / 12);
    i = (int)(e - 12LL * o);
    g = gW1a[hp(o) * 16 + i];
    if (i == 10) g += gW1a[hp(o) * 16 + 12];
    if (i == 11) g += gW1a[hp(o) * 16 + 13];
    decay = true;
  } else if (e < OFF_W2) {
    o = (int)(e - OFF_B1);
    g = gW1a[hp(o) * 16 + 14];
  } else if (e < OFF_B2) {
    const long long k = e - OFF_W2;
    o = (int)(k / H);
    i = (int)(k - (long long)o * H);
    g = gW2a[(long long)hp(o) * LDG + hp(i)];
    decay = true;
  } else if (e < OFF_W3) {
    o = (int)(e - OFF_B2);
    g = gW2a[(long long)hp(o) * LDG + H];
  } else if (e < OFF_B3) {
    o = (int)(e - OFF_W3);
    g = gW3a[hp(o)];
    decay = true;
  } else {
    g = gW3a[H];
  }
  float p = P[e];
  if (a.update) {
    const int t = *step > 0 ? *step : 1;
    const float lr = sched_lr_big(a, t);
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
  if (e < OFF_B1) {
    const int mt = o >> 5, rr = o & 31;
    auto put = [&](int kappa) { w1p[((size_t)(mt * 64 + rr + 32 * (kappa >> 3))) * 8 + (kappa & 7)] = (__bf16)p; };
    put(i);
    if (i == 10) put(12);
    if (i == 11) put(13);
  } else if (e < OFF_W2) {
    const int mt = o >> 5, rr = o & 31;
    const __bf16 hi = (__bf16)p;
    w1p[((size_t)(mt * 64 + rr + 32)) * 8 + 6] = hi;
    w1p[((size_t)(mt * 64 + rr + 32)) * 8 + 7] = (__bf16)(p - (float)hi);
  } else if (e < OFF_B2) {
    w2k[(size_t)o * H + hp(i)] = (__bf16)p;
    w2t[(size_t)i * H + hp(o)] = (__bf16)p;
  } else if (e < OFF_W3) {
    b2[o] = p;
  } else if (e < OFF_B3) {
    w3[o] = p;
  } else {
    b3[0] = p;
  }
}

// Wide AdamW + re-pack in ONE launch.  Blocks [0, (H/32)^2) take the W2 block in 32 x 32 tiles:
// P / M / V and the w2k rows are written coalesced as before, and the transposed copy w2t goes
// through an LDS tile so its rows are written coalesced too (one element per thread scattered
// 2-byte writes H*2 bytes apart).  The remaining blocks take the other 15H + 1 parameters one per
// thread (adamw_big_elem).
__global__ __launch_bounds__(256) void adamw_pack_big_kernel(float* __restrict__ P, const float* __restrict__ G,
                                                             float* __restrict__ M, float* __restrict__ V,
                                                             __bf16* __restrict__ w1p, __bf16* __restrict__ w2k,
                                                             __bf16* __restrict__ w2t, float* __restrict__ b2,
                                                             float* __restrict__ w3, float* __restrict__ b3,
                                                             const int* __restrict__ step, AdamWBigArgs a) {
  __shared__ __bf16 T[32][34];
  const int H = a.H, LDG = H + 16, tpr = H / 32, ntiles = tpr * tpr;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= ntiles) {
    const long long ep = (long long)(blockIdx.x - ntiles) * blockDim.x + tid;
    if (ep < 15LL * H + 1) adamw_big_elem(ep, P, G, M, V, w1p, w2k, w2t, b2, w3, b3, step, a);
    return;
  }
  const long long OFF_W2 = 13LL * H;
  const int o0 = (blockIdx.x / tpr) * 32, i0 = (blockIdx.x % tpr) * 32;
  const int t = *step > 0 ? *step : 1;
  const float lr = sched_lr_big(a, t);
  const float bc1 = 1.f - powf(a.beta1, (float)t);
  const float bc2 = 1.f - powf(a.beta2, (float)t);
#pragma unroll
  for (int idx = tid; idx < 1024; idx += 256) {
    const int oo = idx >> 5, ii = idx & 31, o = o0 + oo, i = i0 + ii;
    const long long e = OFF_W2 + (long long)o * H + i;
    float p = P[e];
    if (a.update) {
      const float g = G[(long long)hp(o) * LDG + hp(i)];
      p -= lr * a.wd * p;
      const float m = a.beta1 * M[e] + (1.f - a.beta1) * g;
      const float v = a.beta2 * V[e] + (1.f - a.beta2) * g * g;
      M[e] = m;
      V[e] = v;
      p -= lr * (m / bc1) / (sqrtf(v / bc2) + a.eps);
      P[e] = p;
    }
    const __bf16 pb = (__bf16)p;
    w2k[(size_t)o * H + hp(i)] = pb;
    T[ii][oo] = pb;
  }
  __syncthreads();
#pragma unroll
  for (int idx = tid; idx < 1024; idx += 256) {
    const int ii = idx >> 5, oo = idx & 31;
    w2t[(size_t)(i0 + ii) * H + o0 + hp(oo)] = T[ii][oo];
  }
}

}  // namespace

hipError_t launch_adamw_pack_big(float* P, const float* G, float* M, float* V, void* w1p, void* w2k,
                                 void* w2t, float* b2, float* w3, float* b3, const int* step, int H,
                                 float lr, float beta1, float beta2, float eps, float wd, int warmup,
                                 int total_steps, float min_lr_ratio, int update, hipStream_t stream) {
  AdamWBigArgs a{lr, beta1, beta2, eps, wd, warmup, total_steps, min_lr_ratio, update, H};
  if (H % 32) return hipErrorInvalidValue;
  const long long Nrest = 15LL * H + 1;                 // everything but the W2 block
  const unsigned nb = (unsigned)((H / 32) * (H / 32) + (Nrest + 255) / 256);
  hipLaunchKernelGGL(adamw_pack_big_kernel, dim3(nb), dim3(256), 0, stream,
                     P, G, M, V, (__bf16*)w1p, (__bf16*)w2k, (__bf16*)w2t, b2, w3, b3, step, a);
  return hipGetLastError();
}

hipError_t launch_big_layer1(const void* rec, int rec_bytes, int B, const void* w1p, int H,
                             const NormParams& np, void* h1, int ld, void* xf, hipStream_t stream,
                             unsigned* mbits) {
  if (B <= 0) return hipSuccess;
  if (H % 32 || ld % 8) return hipErrorInvalidValue;
  const int tiles = (B + 31) / 32;
  const dim3 grid((tiles + 3) / 4), block(256);
  switch (rec_bytes) {
    case 16: hipLaunchKernelGGL(big_layer1_kernel<16>, grid, block, 0, stream, rec, B, (const bf16x8*)w1p, H, np, (__bf16*)h1, ld, (__bf16*)xf, mbits); break;
    case 8: hipLaunchKernelGGL(big_layer1_kernel<8>, grid, block, 0, stream, rec, B, (const bf16x8*)w1p, H, np, (__bf16*)h1, ld, (__bf16*)xf, mbits); break;
    case 6: hipLaunchKernelGGL(big_layer1_kernel<6>, grid, block, 0, stream, rec, B, (const bf16x8*)w1p, H, np, (__bf16*)h1, ld, (__bf16*)xf, mbits); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// 256 (default where the shape allows) or 128: ROUTEST_GEMM_TILE A/B knob
static int gemm_tile() {
  static const int t = [] {
    const char* v = std::getenv("ROUTEST_GEMM_TILE");
    return (v && std::atoi(v) == 128) ? 128 : 256;
  }();
  return t;
}

// K loop of the 256 x 256 tile: 1 = phase pipeline (gemm256p_kernel), 0 = one drain per K-tile
// (gemm256_kernel); ROUTEST_GEMM_PIPE at start-up, gemm_pipe_mode(set) at run time (A/B tests)
static std::atomic<int> g_gemm_pipe{-1};
int gemm_pipe_mode(int set) {
  if (set >= 0) g_gemm_pipe.store(set ? 1 : 0);
  int v = g_gemm_pipe.load();
  if (v < 0) {
    const char* e = std::getenv("ROUTEST_GEMM_PIPE");
    v = (e == nullptr || std::atoi(e) != 0) ? 1 : 0;
    int expect = -1;
    if (!g_gemm_pipe.compare_exchange_strong(expect, v)) v = expect;
  }
  return v;
}
static bool gemm_pipe() { return gemm_pipe_mode(-1) == 1; }

template <int EPI>
static hipError_t launch_g256(const GemmArgs& a, dim3 grid, dim3 block, hipStream_t stream) {
  static bool attr[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  const int lds = 2 * G2_STAGE;
  static_assert(2 * G2_STAGE == 2 * GP_BUF, "both K loops use the same 128 KB of LDS");
  if (!attr[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm256_kernel<EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)gemm256p_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr[dev & 63] = true;
  }
  if (gemm_pipe()) hipLaunchKernelGGL(gemm256p_kernel<EPI>, grid, block, lds, stream, a);
  else hipLaunchKernelGGL(gemm256_kernel<EPI>, grid, block, lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_gemm_nt(int epi,const void* W, int ldw, const void* X, int ldx, int N, int M,
                          int K, const float* b2, const float* w3, float* ypart, void* out,
                          int ldo, hipStream_t stream) {
  if (M <= 0) return hipSuccess;
  if (N % GT || K % GK || ldw % 8 || ldx % 8 || (out != nullptr && ldo % 8)) return hipErrorInvalidValue;
  // the 256 x 256 epilogue stores 16-byte pieces of a row (out 16-byte aligned, ldo % 8 == 0)
  if (N % G2T == 0 && K % G2K == 0 && gemm_tile() == 256 && ((uintptr_t)out & 15) == 0) {
    static const int st16 = [] {
      const char* v = std::getenv("ROUTEST_GEMM_ST16");
      return (v != nullptr && std::atoi(v) == 0) ? 0 : 1;
    }();
    GemmArgs a{(const __bf16*)W, (const __bf16*)X, ldw, ldx, N, M, K, b2, w3, ypart, (__bf16*)out, ldo, N / G2T, st16};
    const dim3 grid((unsigned)((N / G2T) * ((M + G2T - 1) / G2T))), block(512);
    switch (epi) {
      case EPI_Y: return launch_g256<EPI_Y>(a, grid, block, stream);
      case EPI_H2Y: return launch_g256<EPI_H2Y>(a, grid, block, stream);
      case EPI_STORE: return launch_g256<EPI_STORE>(a, grid, block, stream);
      default: return hipErrorInvalidValue;
    }
  }
  GemmArgs a{(const __bf16*)W, (const __bf16*)X, ldw, ldx, N, M, K, b2, w3, ypart, (__bf16*)out, ldo, N / GT, 0};
  const dim3 grid((unsigned)((N / GT) * ((M + GT - 1) / GT))), block(256);
  switch (epi) {
    case EPI_Y: hipLaunchKernelGGL(gemm_nt_kernel<EPI_Y>, grid, block, 0, stream, a); break;
    case EPI_H2Y: hipLaunchKernelGGL(gemm_nt_kernel<EPI_H2Y>, grid, block, 0, stream, a); break;
    case EPI_STORE: hipLaunchKernelGGL(gemm_nt_kernel<EPI_STORE>, grid, block, 0, stream, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// dgrad with the dW1 epilogue (EPI_DW1): dh1 = dz2 W2 is never stored; slab1 row t receives the
// [N positions][16] dW1 partial of batch rows [256 t, 256 t + 256).  256 x 256 loops only.
hipError_t launch_gemm_dgrad_dw1(const void* W, int ldw, const void* X, int ldx, int N, int M, int K,
                                 const unsigned* mbits, const void* xf, float* slab1, long long slab1_ld,
                                 hipStream_t stream) {
  if (M <= 0) return hipSuccess;
  if (N % G2T || K % G2K || ldw % 8 || ldx % 8 || slab1_ld < 16LL * N || ((uintptr_t)mbits & 15) ||
      ((uintptr_t)xf & 15) || ((uintptr_t)slab1 & 3))
    return hipErrorInvalidValue;
  GemmArgs a{(const __bf16*)W, (const __bf16*)X, ldw, ldx, N, M, K, nullptr, nullptr, nullptr, nullptr, 0, N / G2T, 1};
  a.mbits = mbits;
  a.xf = (const __bf16*)xf;
  a.slab1 = slab1;
  a.slab1_ld = slab1_ld;
  static bool attr[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  static_assert(DW1_LDS >= 2 * G2_STAGE && DW1_LDS <= 160 * 1024, "the dW1 epilogue's LDS holds the K loop's");
  if (!attr[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm256_kernel<EPI_DW1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       DW1_LDS);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)gemm256p_kernel<EPI_DW1>, hipFuncAttributeMaxDynamicSharedMemorySize, DW1_LDS);
    if (e != hipSuccess) return e;
    attr[dev & 63] = true;
  }
  const dim3 grid((unsigned)((N / G2T) * ((M + G2T - 1) / G2T))), block(512);
  if (gemm_pipe()) hipLaunchKernelGGL(gemm256p_kernel<EPI_DW1>, grid, block, DW1_LDS, stream, a);
  else hipLaunchKernelGGL(gemm256_kernel<EPI_DW1>, grid, block, DW1_LDS, stream, a);
  return hipGetLastError();
}

// W2 stages in the fused kernel: 2 (default) or 3 (ROUTEST_BIG_STAGES=3: one stage kept in flight
// across each raw s_barrier with a counted vmcnt — measured 4-8 % SLOWER here,
// profiles/mlp_big_gemm256_r2.md: with 2 waves per SIMD the other wave already covers the DMA)
static int big_stages() {
  static const int n = [] {
    const char* v = std::getenv("ROUTEST_BIG_STAGES");
    return (v && std::atoi(v) == 3) ? 3 : 2;
  }();
  return n;
}

hipError_t launch_big_fused(const void* rec, int rec_bytes, int B, const void* w1q, const void* w2f,
                            int H, const NormParams& np, const float* b2, const float* w3,
                            float* ypart, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (H % G2T) return hipErrorInvalidValue;
  FusedArgs a{rec, B, H, (const __bf16*)w1q, (const __bf16*)w2f, b2, w3, ypart, H / G2T, np};
  const dim3 grid((unsigned)((H / G2T) * ((B + G2T - 1) / G2T))), block(512);
  const int ns = big_stages();
  const int lds = ns * G2T * G2K * 2 + H * 32;
  auto go = [&](auto kern) -> hipError_t {
    static bool attr[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (!attr[dev & 63]) {
      // sized once for the largest H (1024): 3 x 32 KB of W2 stages + 32 KB of W1k fragments
      const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               3 * G2T * G2K * 2 + 1024 * 32);
      if (e != hipSuccess) return e;
      attr[dev & 63] = true;
    }
    hipLaunchKernelGGL(kern, grid, block, lds, stream, a);
    return hipGetLastError();
  };
  switch (rec_bytes * 10 + ns) {
    case 163: return go(mlp_big_fused_kernel<16, 3>);
    case 83: return go(mlp_big_fused_kernel<8, 3>);
    case 63: return go(mlp_big_fused_kernel<6, 3>);
    case 162: return go(mlp_big_fused_kernel<16, 2>);
    case 82: return go(mlp_big_fused_kernel<8, 2>);
    case 62: return go(mlp_big_fused_kernel<6, 2>);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_big_yreduce(const float* ypart, int nparts, int B, float b3, const float* b3p,
                              float* y, const float* target, float gscale, float* dy, void* dyb,
                              float* sq_err, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(big_yreduce_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, ypart, nparts, B,
                     b3, b3p, y, target, gscale, dy, (__bf16*)dyb, sq_err);
  return hipGetLastError();
}

hipError_t launch_big_dz2y(const float* ypart, int nparts, int B, int H, const float* b3p,
                           const float* target, float gscale, float* dy, void* dyb, float* sq_err,
                           const void* h2a, int lda, const float* w3, void* dz2, int* step_ctr,
                           hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (H % 8 || nparts > 64 || lda % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(big_dz2y_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, ypart, nparts, B, H, b3p,
                     target, gscale, dy, (__bf16*)dyb, sq_err, (const __bf16*)h2a, lda, w3, (__bf16*)dz2,
                     step_ctr);
  return hipGetLastError();
}

hipError_t launch_big_dz2y_w3(const float* ypart, int nparts, int B, int H, const float* b3p,
                              const float* target, float gscale, float* dy, void* dyb, float* sq_err,
                              const void* h2a, int lda, const float* w3, void* dz2, int* step_ctr, float* slab,
                              long long slab_ld, int S, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if ((H != 512 && H != 1024) || nparts > 64 || lda % 8 || S < 1 || S > B || slab_ld < H + 16)
    return hipErrorInvalidValue;
#define RT_DZ2Y_W3(KCV)                                                                                        \
  hipLaunchKernelGGL(big_dz2y_w3_kernel<KCV>, dim3(S), dim3(1024), 0, stream, ypart, nparts, B, b3p, target, gscale, \
                     dy, (__bf16*)dyb, sq_err, (const __bf16*)h2a, lda, w3, (__bf16*)dz2, step_ctr, slab, slab_ld, S)
  if (H == 512) RT_DZ2Y_W3(1);
  else RT_DZ2Y_W3(2);
#undef RT_DZ2Y_W3
  return hipGetLastError();
}

hipError_t launch_big_dz2(const void* h2a, int lda, const float* dy, const float* w3, int B, int H,
                          void* dz2, hipStream_t stream) {
  const long long n = (long long)B * (H / 8);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(big_dz2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const __bf16*)h2a, lda, dy, w3, B, H, (__bf16*)dz2);
  return hipGetLastError();
}

}  // namespace rt
