// Weight-gradient GEMMs with K = batch:  C[m][n] = sum_k A[k][m] * Bm[k][n]   (bf16 in, fp32 out)
//
// hipBLASLt runs these tall-skinny reductions (K = 65536 rows, M = 256, N = 272) at ~40 TFLOP/s
// (measured: 236 us for dW2 in a 465 us training step, profiles/train_step_hipblaslt.csv), because
// they are really a streaming reduction over the batch.  This kernel is built for that shape:
//
//  * grid = (S k-slices, M/256 m-blocks); every workgroup streams ITS slice of batch rows exactly
//    once from HBM, so all CUs pull bandwidth (a few large K-slices would leave the chip idle).
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
#include "common.h"
#include "ops.h"

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

template <int NT>
__global__ __launch_bounds__(512, 2) void wgrad_kernel(const __bf16* __restrict__ A, int lda, int M,
                                                       int Mout, const __bf16* __restrict__ Bm,
                                                       int ldb, int N, int K, int kslice,
                                                       float* __restrict__ slab, int ldo,
                                                       long long slab_stride) {
  constexpr int KB = 32, AW = 256, BW = 32 * NT;
  constexpr int ACH = AW / 8, BCH = BW / 8;           // 16-B chunks per staged row
  constexpr int TPB = 512;
  constexpr int APT = (KB * ACH + TPB - 1) / TPB;      // chunks per thread
  constexpr int BPT = (KB * BCH + TPB - 1) / TPB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int sa = pad_stride_elems(AW), sb = pad_stride_elems(BW);
  __bf16* sA = reinterpret_cast<__bf16*>(smem);
  __bf16* sB = sA + KB * sa;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m_base = blockIdx.y * AW;
  const int k_begin = blockIdx.x * kslice;
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
  float* out = slab + (long long)blockIdx.x * slab_stride;
  const int h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int nn = 32 * n + col;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = m_base + 32 * w + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (m < Mout && nn < N) out[(size_t)m * ldo + nn] = acc[n][e];
    }
  }
}

// G[e] = sum_s slab[s][e] for e in [0, n), fixed order over s (deterministic).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, int S,
                                                           long long slab_stride,
                                                           float* __restrict__ G, int n) {
  const int i4 = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = i4 * 4;
  if (e >= n) return;
  if (e + 4 <= n && (slab_stride % 4) == 0) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) {
      const float4 v = *reinterpret_cast<const float4*>(slab + s * slab_stride + e);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    *reinterpret_cast<float4*>(G + e) = acc;
  } else {
    for (int q = e; q < min(n, e + 4); ++q) {
      float acc = 0.f;
      for (int s = 0; s < S; ++s) acc += slab[s * slab_stride + q];
      G[q] = acc;
    }
  }
}

size_t wgrad_lds_bytes(int NT) {
  auto pad = [](int cols) {
    int b = 2 * cols, r = b % 256;
    b += (r <= 64) ? (64 - r) : (256 - r + 64);
    return b;
  };
  return (size_t)32 * pad(256) + (size_t)32 * pad(32 * NT);
}

template <int NT>
static hipError_t launch_wgrad_nt(const void* A, int lda, int M, int Mout, const void* Bm, int ldb,
                                  int N, int K, int S, float* slab, int ldo, long long slab_stride,
                                  hipStream_t stream) {
  const int kslice = ((K + S - 1) / S + 31) / 32 * 32;
  const int mblocks = (M + 255) / 256;
  const size_t lds = wgrad_lds_bytes(NT);
  hipLaunchKernelGGL(wgrad_kernel<NT>, dim3(S, mblocks), dim3(512), lds, stream,
                     (const __bf16*)A, lda, M, Mout, (const __bf16*)Bm, ldb, N, K, kslice, slab, ldo,
                     slab_stride);
  return hipGetLastError();
}

hipError_t launch_wgrad(const void* A, int lda, int M, int Mout, const void* Bm, int ldb, int N,
                        int K, int S, float* slab, int ldo, long long slab_stride,
                        hipStream_t stream) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8) return hipErrorInvalidValue;
  const int NT = (N + 31) / 32;
  switch (NT) {
    case 1: return launch_wgrad_nt<1>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream);
    case 2: return launch_wgrad_nt<2>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream);
    case 3: return launch_wgrad_nt<3>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream);
    case 5: return launch_wgrad_nt<5>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream);
    case 9: return launch_wgrad_nt<9>(A, lda, M, Mout, Bm, ldb, N, K, S, slab, ldo, slab_stride, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_wgrad_reduce(const float* slab, int S, long long slab_stride, float* G, int n,
                               hipStream_t stream) {
  const int threads = (n + 3) / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, slab,
                     S, slab_stride, G, n);
  return hipGetLastError();
}

}  // namespace rt
