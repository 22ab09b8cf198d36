// Weight-gradient GEMMs with K = batch:  C[m][n] = sum_k A[k][m] * Bm[k][n]   (bf16 in, fp32 out)
//
// hipBLASLt runs these tall-skinny reductions (K = 65536 rows, M = 256, N = 272) at ~40 TFLOP/s
// (measured: 236 us for dW2 in a 465 us training step, profiles/train_step_hipblaslt.csv), because
// they are really a streaming reduction over the batch.  This kernel is built for that shape:
//
//  * grid = (S k-slices, M/256 m-blocks, n-blocks of 32*NT columns); every workgroup streams ITS
//    slice of batch rows once, so all CUs pull bandwidth (a few large K-slices would leave the chip
//    idle).  With n-blocks, the nb workgroups of one slice share its A rows through L2 (same XCD
//    when S*mblocks % 8 == 0: their ids differ by multiples of it) and the slice can be nb x longer
//    for the same grid
//    — nb x fewer fp32 slabs to write and reduce.
//  * 32-row stages of A (256 cols) and Bm (32*NT cols) go through LDS with a row stride padded to
//    64 (mod 256) bytes, so each ds_read_b64_tr_b16 (hardware transpose: a lane receives 4
//    consecutive ROWS of its column) is bank-conflict-free; two such reads form the 8-deep k
//    fragment of mfma_f32_32x32x16_bf16 for both operands (k = batch row).
//  * next stage's global loads are issued into registers before the current stage's MFMAs and
//    written to LDS after the barrier (async-STAGE split, cdna_hip_programming.md T14).
//  * 8 waves per workgroup; wave w owns m-tile w (32 rows) x NT n-tiles of 32x32 accumulators
//    (<= 144 accumulator VGPRs: two waves per SIMD); the staged B tile is shared by all 8 waves.
//  * the fp32 partial of slice s is written to slab[s] in the caller's layout (the flat gradient
//    bucket); wgrad_reduce_kernel sums the S slabs in a fixed order — deterministic, no atomics.
#include <cstdlib>
#include <string>
#include <utility>

#include "common.h"
#include "ops.h"
#include "wgrad_reduce.h"

namespace rt {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int pad_stride_elems(int cols) {
  // bytes = 2*cols rounded up so that bytes % 256 == 64
  int b = 2 * cols;
  int r = b % 256;
  b += (r <= 64) ? (64 - r) : (256 - r + 64);
  return b / 2;
}

// 8-deep k fragment (rows kr..kr+3 and kr+4..kr+7 of column c0 + lane-in-group) via two
// hardware-transposed LDS reads.  g = lane >> 4 selects column half and k half.
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* base, int stride, int k0, int c0, int lane) {
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int row = k0 + 8 * (g >> 1) + q;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const lds_s16x4* a0 = (const lds_s16x4*)(base + row * stride + col);
  const lds_s16x4* a1 = (const lds_s16x4*)(base + (row + 4) * stride + col);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(a1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// keep each bf16 of `a` whose counterpart in `m` is > 0 (relu'(h) from the saved activation)
__device__ __forceinline__ int relu_mask_word(int a, int m) {
  const int lo = ((short)(m & 0xFFFF) > 0) ? 0x0000FFFF : 0;
  const int hi = ((short)((unsigned)m >> 16) > 0) ? (int)0xFFFF0000u : 0;
  return a & (lo | hi);
}

// MASK: A_eff = A * (mask > 0) applied while staging (mask has A's shape, leading dim ldm) — fuses
// the ReLU backward of the first layer into dW1 = dz1^T x, so dz1 is never materialised.
// MPERM: the mask's columns are in the trainer's hperm() unit order (h1a) while A's are natural
// (dh1): the 8 mask values of A columns m..m+7 (m % 8 == 0) are the two 8-byte runs at
// p0 = (m & ~15) + 4 * ((m >> 3) & 1) and p0 + 8.
// The body of one workgroup (k-slice bx, m-block by, n-block bz); the kernels below map their
// block ids onto it.
template <int NT, bool MASK, int KB, bool MPERM>
__device__ __forceinline__ void wgrad_body(const int bx, const int by, const int bz,
                                           const __bf16* __restrict__ A, int lda, int M, int Mout,
                                           const __bf16* __restrict__ Bm, int ldb, int N, int K,
                                           int kslice, float* __restrict__ slab, int ldo,
                                           long long slab_stride, const __bf16* __restrict__ mask,
                                           int ldm, int Nout) {
  constexpr int AW = 256, BW = 32 * NT;
  constexpr int ACH = AW / 8, BCH = BW / 8;           // 16-B chunks per staged row
  constexpr int TPB = 512;
  constexpr int APT = (KB * ACH + TPB - 1) / TPB;      // chunks per thread
  constexpr int BPT = (KB * BCH + TPB - 1) / TPB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int sa = pad_stride_elems(AW), sb = pad_stride_elems(BW);
  __bf16* sA = reinterpret_cast<__bf16*>(smem);
  __bf16* sB = sA + KB * sa;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m_base = by * AW;
  // n-block z: columns [n0, n0 + 32*NT) of Bm / the output (several workgroups per k-slice, so a
  // slice can cover more batch rows for the same grid: fewer fp32 slabs to write and reduce)
  const int n0 = bz * BW;
  Bm += n0;
  N -= n0;
  Nout -= n0;
  const int k_begin = bx * kslice;
  const int k_end = min(K, k_begin + kslice);

  f32x16 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[n][e] = 0.f;

  int4 ra[APT], rb[BPT];
  auto gload = [&](int kb) {
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const int c = tid + TPB * u;
      const int r = c / ACH, ch = c - r * ACH;
      const int k = kb + r, m = m_base + ch * 8;
      ra[u] = (c < KB * ACH && k < k_end && m < M)
                  ? *reinterpret_cast<const int4*>(A + (size_t)k * lda + m) : make_int4(0, 0, 0, 0);
      if constexpr (MASK) {
        if (c < KB * ACH && k < k_end && m < M) {
          int4 mk;
          if constexpr (MPERM) {
            const __bf16* mp = mask + (size_t)k * ldm + (m & ~15) + 4 * ((m >> 3) & 1);
            const int2 lo = *reinterpret_cast<const int2*>(mp);
            const int2 hi = *reinterpret_cast<const int2*>(mp + 8);
            mk = make_int4(lo.x, lo.y, hi.x, hi.y);
          } else {
            mk = *reinterpret_cast<const int4*>(mask + (size_t)k * ldm + m);
          }
          ra[u].x = relu_mask_word(ra[u].x, mk.x);
          ra[u].y = relu_mask_word(ra[u].y, mk.y);
          ra[u].z = relu_mask_word(ra[u].z, mk.z);
          ra[u].w = relu_mask_word(ra[u].w, mk.w);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int c = tid + TPB * u;
      const int r = c / BCH, ch = c - r * BCH;
      const int k = kb + r, n = ch * 8;
      rb[u] = (c < KB * BCH && k < k_end && n < N)
                  ? *reinterpret_cast<const int4*>(Bm + (size_t)k * ldb + n) : make_int4(0, 0, 0, 0);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const int c = tid + TPB * u;
      if (c < KB * ACH) {
        const int r = c / ACH, ch = c - r * ACH;
        *reinterpret_cast<int4*>(sA + r * sa + ch * 8) = ra[u];
      }
    }
#pragma unroll
    for (int u = 0; u < BPT; ++u) {
      const int c = tid + TPB * u;
      if (c < KB * BCH) {
        const int r = c / BCH, ch = c - r * BCH;
        *reinterpret_cast<int4*>(sB + r * sb + ch * 8) = rb[u];
      }
    }
  };

  const bool mt_live = m_base + 32 * w < M;
  if (k_begin < k_end) {
    gload(k_begin);
    for (int kb = k_begin; kb < k_end; kb += KB) {
      __syncthreads();  // previous stage fully consumed
      lstore();
      __syncthreads();
      if (kb + KB < k_end) gload(kb + KB);  // in flight under this stage's MFMAs
#pragma unroll
      for (int ks = 0; ks < KB / 16; ++ks) {
        if (mt_live) {
          const bf16x8 a = tr_frag(sA, sa, 16 * ks, 32 * w, lane);
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            const bf16x8 b = tr_frag(sB, sb, 16 * ks, 32 * n, lane);
            acc[n] = mfma32(a, b, acc[n]);
          }
        }
      }
    }
  }
  // partial of this k-slice -> slab[blockIdx.x]
  float* out = slab + (long long)bx * slab_stride + n0;
  const int h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int nn = 32 * n + col;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = m_base + 32 * w + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (m < Mout && nn < Nout) out[(size_t)m * ldo + nn] = acc[n][e];
    }
  }
}

template <int NT, bool MASK, int KB, bool MPERM = false>
__global__ __launch_bounds__(512, 2) void wgrad_kernel(const __bf16* __restrict__ A, int lda, int M,
                                                       int Mout, const __bf16* __restrict__ Bm,
                                                       int ldb, int N, int K, int kslice,
                                                       float* __restrict__ slab, int ldo,
                                                       long long slab_stride,
                                                       const __bf16* __restrict__ mask, int ldm,
                                                       int Nout) {
  wgrad_body<NT, MASK, KB, MPERM>(blockIdx.x, blockIdx.y, blockIdx.z, A, lda, M, Mout, Bm, ldb, N, K,
                                  kslice, slab, ldo, slab_stride, mask, ldm, Nout);
}

// Two independent weight-gradient GEMMs in ONE launch (the small trainer's dW2|db2 with NT0 n-tiles
// per workgroup, and dW1 with one): blocks [0, nb0) run segment 0 in the 3-D order of a plain launch
// (k-slice fastest, so a slice's n-blocks still land on one XCD), the rest segment 1.  The two
// grids (~240 + 256 workgroups) fit the 512 workgroup slots of the chip together, so dW1 streams
// its operands while dW2 runs instead of after it, and one dependent launch boundary goes away.
struct WgSeg {
  const __bf16* A;
  const __bf16* Bm;
  float* slab;
  long long slab_stride;
  int lda, M, Mout, ldb, N, K, kslice, ldo, Nout, S, mblocks;
};

template <int NT0, int KB>
__global__ __launch_bounds__(512, 2) void wgrad_dual_kernel(WgSeg s0, WgSeg s1, int nb0) {
  int b = (int)blockIdx.x;
  if (b < nb0) {
    const int x = b % s0.S, r = b / s0.S;
    wgrad_body<NT0, false, KB, false>(x, r % s0.mblocks, r / s0.mblocks, s0.A, s0.lda, s0.M, s0.Mout,
                                      s0.Bm, s0.ldb, s0.N, s0.K, s0.kslice, s0.slab, s0.ldo,
                                      s0.slab_stride, nullptr, 0, s0.Nout);
  } else {
    b -= nb0;
    const int x = b % s1.S, r = b / s1.S;
    wgrad_body<1, false, KB, false>(x, r % s1.mblocks, r / s1.mblocks, s1.A, s1.lda, s1.M, s1.Mout,
                                    s1.Bm, s1.ldb, s1.N, s1.K, s1.kslice, s1.slab, s1.ldo,
                                    s1.slab_stride, nullptr, 0, s1.Nout);
  }
}

// G[e] = sum_s slab[s][e] for e in [0, n) — deterministic (fixed summation tree, no atomics).
//
// 256 threads = 16 slab-lanes x 16 float4 columns: thread (sl, c) sums slabs sl, sl+16, ... of
// column c with 4 independent loads in flight, then the 16 partials are combined in LDS in a fixed
// order.  ~n/64 workgroups (1157 for the H=256 bucket) keep every CU streaming the 76 MB of slabs;
// the previous one-thread-per-column version ran 73 workgroups and 256 dependent loads per thread.
template <bool NTLOAD>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(RedSeg s0, RedSeg s1, RedSeg s2, int nb0,
                                                           int nb01) {
  const int bx = (int)blockIdx.x;
  const int seg = bx < nb0 ? 0 : (bx < nb01 ? 1 : 2);
  const RedSeg sg = seg == 0 ? s0 : (seg == 1 ? s1 : s2);
  float* __restrict__ G = sg.G;
  const int n = sg.n;
  const int blk = bx - (seg == 0 ? 0 : (seg == 1 ? nb0 : nb01));
  __shared__ RedPart part;
  const float4 r = red_sum<NTLOAD>(sg, blk, part);
  const int c = threadIdx.x & (RED_COLS - 1), sl = threadIdx.x / RED_COLS;
  const int e = (blk * RED_COLS + c) * 4;
  const bool vec = (sg.slab_stride % 4) == 0 && e + 4 <= n;
  if (sl == 0 && e < n) {
    if (sg.perm_h > 0) {
      int g0, step;
      native_to_bucket(e, sg.perm_h, g0, step);
      G[g0] = r.x;
      G[g0 + step] = r.y;
      G[g0 + 2 * step] = r.z;
      G[g0 + 3 * step] = r.w;
    } else if (vec) {
      *reinterpret_cast<float4*>(G + e) = r;
    } else {
      const float rr[4] = {r.x, r.y, r.z, r.w};
      for (int q = 0; q < 4 && e + q < n; ++q) G[e + q] = rr[q];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// wgrad256_kernel: the wide trainer's dW2 = dz2^T h1a (M = N = H units, K = batch rows) on 256 x 256
// OUTPUT-stationary tiles with split-K over the batch (wgrad_kernel<9> was 189 us at
// 3.4x its MFMA floor, the step's largest kernel).  The tile, waves and MFMA of gemm256_kernel
// (mlp_big.hip: 8 waves of 128 x 64 on mfma_f32_16x16x32_bf16, global_load_lds staging); both
// operands are K-MAJOR here (a batch row is a row of dz2 / h1a), so the fragments come from the
// row-major stage images through ds_read_b64_tr_b16 (T10: a 16-lane group reads 4 rows x 16 columns
// and each lane receives one column's 4 rows):
//  * both operands stream from HBM (unlike the forward GEMMs, whose weight tile sits in L2), so the
//    K loop is a RING of four 32-deep stages (32 KB each) with three in flight: one barrier per
//    stage, the loads of stage k + 3 issued right after it, counted vmcnt waits (2-stage 64-deep
//    double buffering measured 190 us: each stage's loads outlived the stage's MFMAs);
//  * stage image: 32 rows x 512 B per operand; row r's 16-byte chunk ch sits at slot
//    ch ^ (sw(r) << 1), sw(r) = (r & 3) | ((r >> 3 & 1) << 2) — the 8 rows one 32-lane half of a
//    transposed read touches (8g + q, 8g + 8 + q) hit 8 distinct 32-byte bank groups (bank of byte a:
//    (a / 4) % 64; a 512-byte row alone maps every row onto the same banks: 8-way);
//    global_load_lds writes lane-linearly, so each lane loads the GLOBAL chunk its slot holds;
//  * grid = S k-slices x tiles; the tiles of one slice run on one XCD (they share the slice's dz2
//    and h1a rows through that XCD's L2);
//  * the fp32 partial of slice s goes to slab[s] ([M][ldo]); wgrad_reduce sums the slices in a fixed
//    order (deterministic);
//  * db2 (the ones column of h1a, i.e. column sums of dz2) rides along: tile column tn sums rows
//    [32/tiles_n * tn, +32/tiles_n) of every stage of its A image (one ds_read_b128 per thread and
//    row group) into slab column db2_col + tn; the reduce folds those tiles_n columns into db2_col.
struct Wg256Args {
  const __bf16* A;
  const __bf16* B;
  float* slab;
  long long slab_stride;
  int lda, ldb, ldo, M, N, K, kslice, tiles_m, tiles_n, S, db2_col;
};
// KT rows per stage, a ring of NST stages (NST - 1 in flight): <32, 4> (default) keeps three 32-deep
// stages in flight, <64, 2> double-buffers 64-deep stages (ROUTEST_WGRAD256_CFG=64x2)
template <int KT>
struct W256Stage {
  static constexpr int TILE = KT * 512;         // one operand's stage image (bytes)
  static constexpr int STAGE = 2 * TILE;
  static constexpr int LOADS = 2 * (KT / 16);   // global_load_lds per thread per stage
};

__device__ __forceinline__ int w256_sw(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
// byte offset of columns col .. col + 3 (col % 4 == 0) of row r in a stage image
__device__ __forceinline__ int w256_off(int r, int col) {
  return r * 512 + (((col >> 3) ^ (w256_sw(r) << 1)) << 4) + (((col >> 2) & 1) << 3);
}
// the 16x16x32 operand fragment of columns c0 .. c0 + 15 and rows 0 .. 31: lane l gets column
// c0 + (l & 15), rows 8 (l >> 4) .. + 7 (two transposed reads of 4 rows)
__device__ __forceinline__ bf16x8 w256_frag(const unsigned char* img, int c0, int lane) {
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int r = 8 * g + q;
  const lds_s16x4* a0 = (const lds_s16x4*)(img + w256_off(r, c0 + 4 * p));
  const lds_s16x4* a1 = (const lds_s16x4*)(img + w256_off(r + 4, c0 + 4 * p));
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(a1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// 16-byte LDS-DMA (global_load_lds_dwordx4) in inline asm: hipcc's waitcnt bookkeeping does not see
// it, so the stage's fragment reads that follow (from ANOTHER buffer) are not preceded by a drain of
// the prefetch (with the builtin, hipcc emitted vmcnt(0) before them: it cannot tell the buffers
// apart) — the loop's counted s_waitcnt vmcnt(N) before each barrier is the only wait.  M0 (the
// destination base) is set and restored in the same statement (cdna_hip_programming.md, LDS-DMA recipe).
__device__ __forceinline__ void glds16_asm(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

template <int KT, int NST>
__global__ __launch_bounds__(512, 1) void wgrad256_kernel(Wg256Args a) {
  static_assert(KT % 16 == 0 && KT <= 64 && (NST & (NST - 1)) == 0 && NST >= 2, "stage shape");
  using SG = W256Stage<KT>;
  constexpr int W256_KT = KT, W256_NST = NST, W256_TILE = SG::TILE, W256_STAGE = SG::STAGE;
  constexpr int QN = KT / 16;                    // instructions per operand per wave and stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smw[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int T = a.tiles_m * a.tiles_n;
  int s, t;
  {
    const int bid = (int)blockIdx.x;
    if (a.S % 8 == 0) {                    // XCD x (= bid % 8) runs slices x, x + 8, ...
      const int loc = bid >> 3;
      s = (bid & 7) + 8 * (loc / T);
      t = loc % T;
    } else {
      s = bid / T;
      t = bid % T;
    }
  }
  const int tm = t / a.tiles_n, tn = t % a.tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const int k_begin = s * a.kslice;
  const int k_end = min(a.K, k_begin + a.kslice);
  const int nk = k_end > k_begin ? (k_end - k_begin) / W256_KT : 0;
  const int wu = w & 1, wr = w >> 1;       // units [128 wu, +128) x columns [64 wr, +64)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // staging: instruction q of wave w fills LDS rows 2 (8q + w) + (lane >> 5), slot lane & 31.  The
  // source pointers advance one stage per issue and stay live across the loop: a glds address held
  // in a temporary was reallocated to a ds_read destination right after, and the compiler then
  // drained the just-issued loads (vmcnt(0)) before the stage's fragment reads
  const __bf16* gA[QN];
  const __bf16* gB[QN];
#pragma unroll
  for (int q = 0; q < QN; ++q) {
    const int r = 2 * (8 * q + w) + (lane >> 5);
    const int ch = (lane & 31) ^ (w256_sw(r) << 1);
    gA[q] = a.A + (size_t)(k_begin + r) * a.lda + m0 + 8 * ch;
    gB[q] = a.B + (size_t)(k_begin + r) * a.ldb + n0 + 8 * ch;
  }
  const size_t stepA = (size_t)W256_KT * a.lda, stepB = (size_t)W256_KT * a.ldb;
  // the LDS byte address of the dynamic region (wave-uniform)
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned char*)smw);
  auto issue = [&](int kt) {                // stage kt (issued in order); SG::LOADS loads per thread
    const unsigned img = lds0 + (unsigned)((kt & (W256_NST - 1)) * W256_STAGE);
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      glds16_asm(gA[q], __builtin_amdgcn_readfirstlane(img + (8 * q + w) * 1024));
      glds16_asm(gB[q], __builtin_amdgcn_readfirstlane(img + W256_TILE + (8 * q + w) * 1024));
      gA[q] += stepA;
      gB[q] += stepB;
    }
  };

  // db2: this tile column's rows of each stage (rows_per = 32 / tiles_n), thread -> (row, 8 units)
  const bool db2 = a.db2_col >= 0 && (a.tiles_n == 1 || a.tiles_n == 2 || a.tiles_n == 4);
  const int rows_per = db2 ? W256_KT / a.tiles_n : 0;
  float dsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int drow = tid >> 5, dch = tid & 31;

  for (int kt = 0; kt < NST - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (up to NST - 2 younger stages may stay in flight), then every wave is past
    // stage kt - 1, whose buffer stage kt + NST - 1 refills
    const int younger = min(NST - 2, nk - 1 - kt);
    if constexpr (NST >= 4) {
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * SG::LOADS) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SG::LOADS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (NST == 3) {
      if (younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SG::LOADS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      (void)younger;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // a RAW barrier: __syncthreads()' fence would drain the loads still in flight (vmcnt(0));
    // every read of the buffer about to be refilled was consumed by this wave's MFMAs already
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + NST - 1 < nk) issue(kt + NST - 1);
    const int ks_n = KT / 32;
    const unsigned char* imgA = smw + (kt & (W256_NST - 1)) * W256_STAGE;
    const unsigned char* imgB = imgA + W256_TILE;
#pragma unroll
    for (int ks = 0; ks < ks_n; ++ks) {
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = w256_frag(imgA + 32 * ks * 512, 128 * wu + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = w256_frag(imgB + 32 * ks * 512, 64 * wr + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (db2) {
      for (int rr = 0; rr < rows_per; rr += 16) {
        if (rr + drow < rows_per) {
          const int r = rows_per * tn + rr + drow;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(imgA + r * 512 + ((dch ^ (w256_sw(r) << 1)) << 4));
#pragma unroll
          for (int e = 0; e < 8; ++e) dsum[e] += (float)v[e];
        }
      }
    }
  }

  // the slice's partial -> slab[s]: acc[i][j] element e = C[unit 128wu + 16i + 4g + e][col 64wr + 16j + fr]
  float* out = a.slab + (long long)s * a.slab_stride;
  const int fr = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* row = out + (size_t)(m0 + 128 * wu + 16 * i + 4 * g + e) * a.ldo + n0 + 64 * wr + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) row[16 * j] = acc[i][j][e];
    }
  if (db2) {
    // the 16 row slots of each unit: lanes l and l + 32 (rows 2w, 2w + 1), then the 8 waves via LDS
    __syncthreads();                                     // every wave is done with the stages
    float* red = reinterpret_cast<float*>(smw);          // [8 waves][256 units]
#pragma unroll
    for (int e = 0; e < 8; ++e) dsum[e] += __shfl_xor(dsum[e], 32);
    if (lane < 32)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[w * 256 + 8 * dch + e] = dsum[e];
    __syncthreads();
    if (tid < 256) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += red[q * 256 + tid];
      out[(size_t)(m0 + tid) * a.ldo + a.db2_col + tn] = v;
    }
  }
}

template <int KT, int NST>
static hipError_t launch_w256(const Wg256Args& a, hipStream_t stream) {
  constexpr int lds = NST * W256Stage<KT>::STAGE;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)wgrad256_kernel<KT, NST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((wgrad256_kernel<KT, NST>), dim3((unsigned)(a.S * a.tiles_m * a.tiles_n)), dim3(512), lds, stream,
                     a);
  return hipGetLastError();
}

hipError_t launch_wgrad256(const void* A, int lda, const void* B, int ldb, int M, int N, int K, int S, float* slab,
                           int ldo, long long slab_stride, int db2_col, hipStream_t stream) {
  // stage shape: ROUTEST_WGRAD256_CFG = 32x4 (default: 159 us against 173 us at H = 1024, 64k rows,
  // run r6g) | 64x2
  static const bool ring = [] {
    const char* v = std::getenv("ROUTEST_WGRAD256_CFG");
    return !(v && std::string(v) == "64x2");
  }();
  const int KT = ring ? 32 : 64;
  if (M % 256 || N % 256 || K % KT || lda % 8 || ldb % 8 || S < 1) return hipErrorInvalidValue;
  Wg256Args a{};
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.slab = slab;
  a.slab_stride = slab_stride;
  a.lda = lda;
  a.ldb = ldb;
  a.ldo = ldo;
  a.M = M;
  a.N = N;
  a.K = K;
  a.kslice = ((K + S - 1) / S + KT - 1) / KT * KT;
  a.tiles_m = M / 256;
  a.tiles_n = N / 256;
  a.S = S;
  a.db2_col = db2_col;
  if (db2_col >= 0 && (db2_col + a.tiles_n > ldo || (a.tiles_n != 1 && a.tiles_n != 2 && a.tiles_n != 4)))
    return hipErrorInvalidValue;
  return ring ? launch_w256<32, 4>(a, stream) : launch_w256<64, 2>(a, stream);
}

size_t wgrad_lds_bytes(int NT, int KB) {
  auto pad = [](int cols) {
    int b = 2 * cols, r = b % 256;
    b += (r <= 64) ? (64 - r) : (256 - r + 64);
    return b;
  };
  return (size_t)KB * pad(256) + (size_t)KB * pad(32 * NT);
}
size_t wgrad_lds_bytes(int NT) { return wgrad_lds_bytes(NT, 32); }

// rows staged per barrier: ROUTEST_WGRAD_KB = 32 | 64 (default: 2x the bytes in flight per CU,
// wgrad<3> 23.7 -> 20.9 us, profiles/superseded/train_wgrad_ab_r2.md) | 128
static int wgrad_kb() {
  static const int kb = [] {
    const char* v = std::getenv("ROUTEST_WGRAD_KB");
    const int k = v ? std::atoi(v) : 64;
    return (k == 64 || k == 128) ? k : 32;
  }();
  return kb;
}

template <int NT, bool MASK, int KB, bool MPERM = false>
static hipError_t launch_wgrad_kb(const void* A, int lda, int M, int Mout, const void* Bm, int ldb,
                                  int N, int K, int S, float* slab, int ldo, long long slab_stride,
                                  hipStream_t stream, const void* mask, int ldm, int Nout) {
  const int kslice = ((K + S - 1) / S + 31) / 32 * 32;
  const int mblocks = (M + 255) / 256;
  const int nblocks = (N + 32 * NT - 1) / (32 * NT);
  const size_t lds = wgrad_lds_bytes(NT, KB);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)wgrad_kernel<NT, MASK, KB, MPERM>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((wgrad_kernel<NT, MASK, KB, MPERM>), dim3(S, mblocks, nblocks), dim3(512), lds, stream,
                     (const __bf16*)A, lda, M, Mout, (const __bf16*)Bm, ldb, N, K, kslice, slab, ldo,
                     slab_stride, (const __bf16*)mask, ldm, Nout);
  return hipGetLastError();
}

template <int NT, bool MASK = false>
static hipError_t launch_wgrad_nt(const void* A, int lda, int M, int Mout, const void* Bm, int ldb,
                                  int N, int K, int S, float* slab, int ldo, long long slab_stride,
                                  hipStream_t stream, const void* mask = nullptr, int ldm = 0,
                                  int Nout = -1) {
  if (Nout < 0) Nout = N;
  switch (wgrad_kb()) {
    case 128: return launch_wgrad_kb<NT, MASK, 128>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, mask, ldm, Nout);
    case 64: return launch_wgrad_kb<NT, MASK, 64>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, mask, ldm, Nout);
    default: return launch_wgrad_kb<NT, MASK, 32>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, mask, ldm, Nout);
  }
}

hipError_t launch_wgrad(const void* A, int lda, int M, int Mout, const void* Bm, int ldb, int N,
                        int K, int S, float* slab, int ldo, long long slab_stride,
                        hipStream_t stream, const void* mask, int ldm, int Nout, bool mask_hperm,
                        int nsplit) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8) return hipErrorInvalidValue;
  if (Nout < 0 || Nout > N) Nout = N;
  if (nsplit < 1) nsplit = 1;
  const int NT = ((N + 31) / 32 + nsplit - 1) / nsplit;     // n-tiles per workgroup
  if (mask != nullptr) {
    if (ldm % 8 || NT != 1 || N > 32) return hipErrorInvalidValue;   // the dW1 shape (N = 16)
    if (mask_hperm) {
      if (M % 16) return hipErrorInvalidValue;
      return launch_wgrad_kb<1, true, 32, true>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride,
                                                stream, mask, ldm, Nout);
    }
    return launch_wgrad_nt<1, true>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, mask, ldm, Nout);
  }
  switch (NT) {
    case 1: return launch_wgrad_nt<1>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 2: return launch_wgrad_nt<2>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 3: return launch_wgrad_nt<3>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 4: return launch_wgrad_nt<4>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 5: return launch_wgrad_nt<5>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 6: return launch_wgrad_nt<6>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 7: return launch_wgrad_nt<7>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 8: return launch_wgrad_nt<8>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    case 9: return launch_wgrad_nt<9>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream, nullptr, 0, Nout);
    default: return hipErrorInvalidValue;
  }
}

template <int NT0, int KB>
static hipError_t launch_dual_kb(const WgSeg& s0, const WgSeg& s1, int nb0, int nb1, hipStream_t stream) {
  const size_t lds = wgrad_lds_bytes(NT0, KB);     // >= the NT = 1 segment's
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)wgrad_dual_kernel<NT0, KB>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((wgrad_dual_kernel<NT0, KB>), dim3(nb0 + nb1), dim3(512), lds, stream, s0, s1, nb0);
  return hipGetLastError();
}

hipError_t launch_wgrad_dual(const void* A0, int lda0, int M0, int Mout0, const void* B0, int ldb0,
                             int N0, int K, int S0, float* slab0, int ldo0, long long stride0, int Nout0,
                             int nsplit0, const void* A1, int lda1, int M1, int Mout1, const void* B1,
                             int ldb1, int N1, int S1, float* slab1, int ldo1, long long stride1,
                             int Nout1, hipStream_t stream) {
  if (M0 % 8 || N0 % 8 || lda0 % 8 || ldb0 % 8 || M1 % 8 || N1 % 8 || lda1 % 8 || ldb1 % 8 || N1 > 32 ||
      S0 < 1 || S1 < 1)
    return hipErrorInvalidValue;
  if (nsplit0 < 1) nsplit0 = 1;
  const int NT0 = ((N0 + 31) / 32 + nsplit0 - 1) / nsplit0;
  auto seg = [&](const void* A, int lda, int M, int Mout, const void* Bm, int ldb, int N, int S, float* slab,
                 int ldo, long long stride, int Nout, int NT) {
    WgSeg g{};
    g.A = (const __bf16*)A;
    g.Bm = (const __bf16*)Bm;
    g.slab = slab;
    g.slab_stride = stride;
    g.lda = lda; g.M = M; g.Mout = Mout; g.ldb = ldb; g.N = N; g.K = K; g.ldo = ldo;
    g.Nout = (Nout < 0 || Nout > N) ? N : Nout;
    g.kslice = ((K + S - 1) / S + 31) / 32 * 32;
    g.S = S;
    g.mblocks = (M + 255) / 256;
    return std::make_pair(g, S * g.mblocks * ((N + 32 * NT - 1) / (32 * NT)));
  };
  const auto p0 = seg(A0, lda0, M0, Mout0, B0, ldb0, N0, S0, slab0, ldo0, stride0, Nout0, NT0);
  const auto p1 = seg(A1, lda1, M1, Mout1, B1, ldb1, N1, S1, slab1, ldo1, stride1, Nout1, 1);
  const bool kb64 = wgrad_kb() != 32;
  switch (NT0) {
#define RT_DUAL(nt) case nt: return kb64 ? launch_dual_kb<nt, 64>(p0.first, p1.first, p0.second, p1.second, stream) \
                                         : launch_dual_kb<nt, 32>(p0.first, p1.first, p0.second, p1.second, stream);
    RT_DUAL(1) RT_DUAL(2) RT_DUAL(3) RT_DUAL(4) RT_DUAL(5) RT_DUAL(6) RT_DUAL(7) RT_DUAL(8) RT_DUAL(9)
#undef RT_DUAL
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_wgrad_reduce(const float* slab, int S, long long slab_stride, float* G, int n,
                               hipStream_t stream, const float* slab1, int S1,
                               long long slab_stride1, float* G1, int n1, const float* slab2, int S2,
                               long long slab_stride2, float* G2, int n2, int perm_h0, int fold_ld0,
                               int fold_col0) {
  if (perm_h0 > 0 && (perm_h0 % 64 || n != perm_h0 * (perm_h0 + 16))) return hipErrorInvalidValue;
  if (fold_ld0 > 0 && (fold_ld0 % 4 || fold_col0 % 4 || fold_col0 + 4 > fold_ld0 || perm_h0 > 0 || slab_stride % 4))
    return hipErrorInvalidValue;
  const RedSeg s0{slab, slab_stride, G, S, n, perm_h0, fold_ld0, fold_col0};
  const RedSeg s1{slab1, slab_stride1, G1, S1, slab1 ? n1 : 0, 0};
  const RedSeg s2{slab2, slab_stride2, G2, S2, slab2 ? n2 : 0, 0};
  const int nb0 = (n + 4 * RED_COLS - 1) / (4 * RED_COLS);
  const int nb1 = (s1.n + 4 * RED_COLS - 1) / (4 * RED_COLS);
  const int nb2 = (s2.n + 4 * RED_COLS - 1) / (4 * RED_COLS);
  if (nb0 + nb1 + nb2 == 0) return hipSuccess;
  // slab reads: plain loads (default: the slabs were written just before and partly sit in L2 / the
  // Infinity Cache; 64k-row step 75.1 -> 73.6 us, profiles/train_r4u.jsonl) or nontemporal
  // (ROUTEST_RED_NT=1)
  static const bool nt = [] {
    const char* v = std::getenv("ROUTEST_RED_NT");
    return v && std::atoi(v) == 1;
  }();
  if (nt) hipLaunchKernelGGL(wgrad_reduce_kernel<true>, dim3(nb0 + nb1 + nb2), dim3(256), 0, stream, s0, s1, s2, nb0, nb0 + nb1);
  else hipLaunchKernelGGL(wgrad_reduce_kernel<false>, dim3(nb0 + nb1 + nb2), dim3(256), 0, stream, s0, s1, s2, nb0, nb0 + nb1);
  return hipGetLastError();
}

}  // namespace rt
