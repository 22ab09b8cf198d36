// K8 backward: training the 2-layer GCN route scorer on gfx950 (csrc/gcn.hip is the forward).
//
//   forward  H0 = Â X,  pre = H0 W1 + b1,  H1 = relu(pre),  Z = H1 W2,  E = Â Z + b2,
//            y = E . wo + bo,  delay = 0.5 + softplus(y),  L = mean_v (delay_v - t_v)^2
//   backward dy = 2 (delay - t) sigmoid(y) / N          (gcn_head_bwd_kernel, with dwo, dbo, L)
//            s  = Â dy                                   (Â is symmetric: Âᵀ dy = Â dy)
//            dZ = s ⊗ wo           -> rank one, so never materialised:
//            dW2 = (H1ᵀ s) ⊗ wo,   dH1 = s ⊗ c with c = W2 wo,
//            dW1 = c ⊙ (H0ᵀ (s ⊙ relu'(pre))),  db1 = c ⊙ Σ s relu'(pre),  db2 = (Σ dy) wo
//
// gcn_l1_bwd_kernel runs the whole layer-1 backward per 32-node wave tile in one pass: s for the
// tile's rows (CSR gather of dy), H0 re-aggregated into LDS (row-major for the pre-activation MFMA,
// and transposed), pre = H0 W1 on mfma_f32_32x32x16_bf16 with the hidden unit on the lane, then the
// weight-gradient GEMM H0ᵀ (s ⊙ relu'(pre)) with K = the tile's nodes, again on MFMA: the
// pre-activation accumulators ARE the B operand (each lane's 16 node rows, in register order; the
// A operand reads H0ᵀ at the same permuted node order), with s ⊙ relu' split into a bf16 hi/lo
// pair so the gradient keeps ~16 mantissa bits.  Per-wave partials are reduced in LDS per
// workgroup into a slab, and gcn_grad_reduce_kernel sums the slabs in a fixed order (bit-wise
// deterministic) into the flat gradient [W1 | b1 | W2 | b2 | wo | bo].
//
// Data parallel (routest_amd/models/gcn_train.py): every rank runs the cheap forward over all
// nodes, but the reductions over nodes (the whole backward) only over its own row range; the
// gradients are per-node sums, so one all-reduce of the 8,385-float bucket gives the full gradient.
#include <algorithm>

#include "lds_fill.h"
#include "common.h"
#include "ops.h"

namespace rt {

namespace {

constexpr int FIN = 32, FHID = 128, FZ = 32;
constexpr int SLAB1 = FIN * FHID + 2 * FHID;     // per workgroup: dW1 partial | g | db1 partial
constexpr int SLAB2 = FZ + 2;                    // per block of the head kernel: dwo | dbo | loss

__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// dy for every node; dwo / dbo / loss partials over the rows [r0, r1) only (4 lanes per node, 8
// features each, like gcn_spmm_score_kernel)
__global__ __launch_bounds__(256) void gcn_head_bwd_kernel(
    const __bf16* __restrict__ Z, const int* __restrict__ indptr, const int* __restrict__ indices,
    const float* __restrict__ values, const float* __restrict__ b2, const float* __restrict__ wo,
    const float* __restrict__ bo, const float* __restrict__ target, float inv_n2, int N, int r0, int r1,
    float* __restrict__ dy, float* __restrict__ slab2) {
  constexpr int G = FZ / 8;
  __shared__ float s_part[256][10];
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int v = gid / G;
  const int q = gid % G, c = q * 8;
  float e[8];
  float part = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = 0.f;
  if (v < N) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // (same accumulation order as the forward's gcn_spmm_score_kernel)
    for (int k = indptr[v]; k < indptr[v + 1]; ++k) {
      const float wv = values[k];
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(Z + (size_t)indices[k] * FZ + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += wv * (float)x[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      e[j] = acc[j] + b2[c + j];
      part += e[j] * wo[c + j];
    }
  }
  part += __shfl_xor(part, 1);
  part += __shfl_xor(part, 2);
  float d = 0.f, r = 0.f;
  if (v < N) {
    const float y = part + bo[0];
    const float delay = 0.5f + softplus_f(y);
    r = delay - target[v];
    d = r * inv_n2 / (1.f + expf(-y));          // 2 (delay - t) / N * sigmoid(y)
    if (q == 0) dy[v] = d;
  }
  const bool own = v >= r0 && v < r1;
#pragma unroll
  for (int j = 0; j < 8; ++j) s_part[threadIdx.x][j] = own ? e[j] * d : 0.f;
  s_part[threadIdx.x][8] = (own && q == 0) ? d : 0.f;
  s_part[threadIdx.x][9] = (own && q == 0) ? r * r : 0.f;
  __syncthreads();
  // fixed-order column sums: output f = dwo[f] (feature f lives in threads with q = f / 8), dbo, loss
  if (threadIdx.x < SLAB2) {
    const int f = threadIdx.x;
    float s = 0.f;
    if (f < FZ) {
      for (int t = f / 8; t < 256; t += G) s += s_part[t][f % 8];
    } else {
      for (int t = 0; t < 256; t += G) s += s_part[t][f == FZ ? 8 : 9];
    }
    slab2[(size_t)blockIdx.x * SLAB2 + f] = s;
  }
}

template <int RB>
__device__ __forceinline__ void csr_gather8(const __bf16* __restrict__ X, int F, int c,
                                            const int* __restrict__ indices,
                                            const float* __restrict__ values, int e0, int e1,
                                            float (&acc)[8]) {
  for (int eb = e0; eb < e1; eb += RB) {
    int u[RB];
    float wv[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const bool in = eb + j < e1;
      u[j] = in ? indices[eb + j] : 0;
      wv[j] = in ? values[eb + j] : 0.f;
    }
    bf16x8 x[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) x[j] = *reinterpret_cast<const bf16x8*>(X + (size_t)u[j] * F + c);
#pragma unroll
    for (int j = 0; j < RB; ++j)
      if (eb + j < e1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += wv[j] * (float)x[j][k];
      }
  }
}

typedef short i16x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gcn_l1_bwd_kernel(
    const __bf16* __restrict__ X, const int* __restrict__ indptr, const int* __restrict__ indices,
    const float* __restrict__ values, const bf16x8* __restrict__ w1frag, const float* __restrict__ b1,
    const float* __restrict__ dy, int r0, int r1, float* __restrict__ slab1) {
  constexpr int G = FIN / 8, RPP = 64 / G, NP = 32 / RPP, KS1 = FIN / 16, NT1 = FHID / 32;
  constexpr int LDA = FIN + 8;     // row-major H0 tile [32 rows][LDA]
  constexpr int LDT = 32 + 8;      // transposed H0 tile [32 features][LDT]
  __shared__ __attribute__((aligned(16))) bf16x8 s_w1[NT1 * KS1 * 64];
  __shared__ __attribute__((aligned(16))) __bf16 s_a[4][32 * LDA];
  __shared__ __attribute__((aligned(16))) __bf16 s_at[4][FIN * LDT];
  __shared__ float s_s[4][32];
  __shared__ float s_red[4][SLAB1 / 4];          // 4 passes of a quarter of the partials
  lds_fill_block(reinterpret_cast<unsigned char*>(s_w1), reinterpret_cast<const unsigned char*>(w1frag),
                 NT1 * KS1 * 64 * 16);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, col = lane & 31;
  __bf16* ta = s_a[w];
  __bf16* tt = s_at[w];
  float bias[NT1];
#pragma unroll
  for (int nt = 0; nt < NT1; ++nt) bias[nt] = b1[32 * nt + col];
  f32x16 dw[NT1];                // D[feature][hidden]: hidden 32nt + col on the lane
  float gp[NT1], dbp[NT1];
#pragma unroll
  for (int nt = 0; nt < NT1; ++nt) {
#pragma unroll
    for (int e = 0; e < 16; ++e) dw[nt][e] = 0.f;
    gp[nt] = dbp[nt] = 0.f;
  }
  const int ntiles = (r1 - r0 + 31) / 32;
  const int lb = (int)(blockIdx.x % 8u) * (int)(gridDim.x / 8u) + (int)(blockIdx.x / 8u);
  for (int t = lb * 4 + w; t < ntiles; t += gridDim.x * 4) {
    const int base = r0 + t * 32;
    // (0) s = Â dy for the tile's rows (lanes 0-31; rows past r1 contribute zero)
    if (lane < 32) {
      const int v = base + lane;
      float sv = 0.f;
      if (v < r1)
        for (int k = indptr[v]; k < indptr[v + 1]; ++k) sv += values[k] * dy[indices[k]];
      s_s[w][lane] = sv;
    }
    // (1) H0 = Â X for the tile, stored row-major and transposed
    {
      const int c = (lane % G) * 8;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int rr = p * RPP + lane / G;
        const int v = base + rr;
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
        if (v < r1) csr_gather8<8>(X, FIN, c, indices, values, indptr[v], indptr[v + 1], acc);
        const bf16x8 xb = to_bf16x8(acc);
        *reinterpret_cast<bf16x8*>(ta + rr * LDA + c) = xb;
#pragma unroll
        for (int j = 0; j < 8; ++j) tt[(c + j) * LDT + rr] = xb[j];
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // (2) pre-activation on MFMA (hidden unit on the lane, node rows in registers)
    f32x16 pre[NT1];
#pragma unroll
    for (int nt = 0; nt < NT1; ++nt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) pre[nt][e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(ta + col * LDA + 16 * ks + 8 * h);
        pre[nt] = mfma32(a, s_w1[(nt * KS1 + ks) * 64 + lane], pre[nt]);
      }
    }
    // the A operand of the weight-gradient GEMM: H0ᵀ[feature col][node rows in this lane's
    // register order]: k-block kb, slot j -> node (j & 3) + 8 (2 kb + (j >> 2)) + 4 h
    bf16x8 at[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const i16x4 lo = *reinterpret_cast<const i16x4*>(tt + col * LDT + 8 * (2 * kb) + 4 * h);
      const i16x4 hi = *reinterpret_cast<const i16x4*>(tt + col * LDT + 8 * (2 * kb + 1) + 4 * h);
      at[kb] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
    float sv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) sv[e] = s_s[w][(e & 3) + 8 * (e >> 2) + 4 * h];
    // (3) B operand = s ⊙ relu'(pre) (hi/lo bf16) straight from the accumulators; g and db1 partials
#pragma unroll
    for (int nt = 0; nt < NT1; ++nt) {
      float bv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float p = pre[nt][e] + bias[nt];
        const bool on = p > 0.f;
        bv[e] = on ? sv[e] : 0.f;
        gp[nt] += on ? p * sv[e] : 0.f;
        dbp[nt] += bv[e];
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        bf16x8 bhi, blo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = bv[8 * kb + j];
          bhi[j] = (__bf16)x;
          blo[j] = (__bf16)(x - (float)bhi[j]);
        }
        dw[nt] = mfma32(at[kb], bhi, dw[nt]);
        dw[nt] = mfma32(at[kb], blo, dw[nt]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();       // tiles free for the next aggregation
  }
  // (4) per-workgroup reduction of the 4 waves' partials (fixed order), one quarter at a time
  //     slab layout: dW1[k][i] (k = feature, i = hidden) | g[i] | db1[i]
  float* out = slab1 + (size_t)blockIdx.x * SLAB1;
  for (int qtr = 0; qtr < 4; ++qtr) {
    // quarter qtr holds dW1 rows k in [8 qtr, 8 qtr + 8) (1024 floats) + g / db1 entries [32 qtr, 32 qtr + 32)
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < NT1; ++nt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = (e & 3) + 8 * (e >> 2) + 4 * h;
        if ((k >> 3) == qtr) s_red[w][(k & 7) * FHID + 32 * nt + col] = dw[nt][e];
      }
    // g / db1: lanes h = 0 and 1 hold different node rows of the same hidden unit -> sum them
#pragma unroll
    for (int nt = 0; nt < NT1; ++nt) {
      const float g2 = gp[nt] + __shfl_xor(gp[nt], 32);
      const float d2 = dbp[nt] + __shfl_xor(dbp[nt], 32);
      if (nt == qtr && h == 0) {
        s_red[w][1024 + col] = g2;
        s_red[w][1024 + 32 + col] = d2;
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 1024 + 64; i += 256) {
      const float s = ((s_red[0][i] + s_red[1][i]) + s_red[2][i]) + s_red[3][i];
      if (i < 1024) out[(8 * qtr + i / FHID) * FHID + i % FHID] = s;
      else if (i < 1024 + 32) out[FIN * FHID + 32 * qtr + (i - 1024)] = s;
      else out[FIN * FHID + FHID + 32 * qtr + (i - 1024 - 32)] = s;
    }
  }
}

// flat gradient [W1 (32x128) | b1 | W2 (128x32) | b2 | wo | bo] + loss, slabs summed in a fixed order
__global__ __launch_bounds__(256) void gcn_grad_reduce_kernel(
    const float* __restrict__ slab1, int S1, const float* __restrict__ slab2, int S2,
    const float* __restrict__ W2, const float* __restrict__ wo, float* __restrict__ grad,
    float* __restrict__ loss) {
  constexpr int OW1 = 0, OB1 = OW1 + FIN * FHID, OW2 = OB1 + FHID, OB2 = OW2 + FHID * FZ, OWO = OB2 + FZ,
                OBO = OWO + FZ, NG = OBO + 1;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  auto cvec = [&](int hid) {   // c = W2 wo
    float c = 0.f;
    for (int j = 0; j < FZ; ++j) c += W2[hid * FZ + j] * wo[j];
    return c;
  };
  auto sum1 = [&](int off) {
    float s = 0.f;
    for (int b = 0; b < S1; ++b) s += slab1[(size_t)b * SLAB1 + off];
    return s;
  };
  auto sum2 = [&](int off) {
    float s = 0.f;
    for (int b = 0; b < S2; ++b) s += slab2[(size_t)b * SLAB2 + off];
    return s;
  };
  if (i < OB1) {
    grad[i] = cvec(i % FHID) * sum1(i);
  } else if (i < OW2) {
    const int hid = i - OB1;
    grad[i] = cvec(hid) * sum1(FIN * FHID + FHID + hid);
  } else if (i < OB2) {
    const int hid = (i - OW2) / FZ, j = (i - OW2) % FZ;
    grad[i] = sum1(FIN * FHID + hid) * wo[j];
  } else if (i < OWO) {
    grad[i] = sum2(FZ) * wo[i - OB2];
  } else if (i < OBO) {
    grad[i] = sum2(i - OWO);
  } else if (i == OBO) {
    grad[i] = sum2(FZ);
  } else if (i == NG) {
    loss[0] = sum2(FZ + 1);
  }
}

}  // namespace

int gcn_grad_numel() { return FIN * FHID + FHID + FHID * FZ + FZ + FZ + 1; }

hipError_t launch_gcn_train_bwd(const void* X, const void* Z, const int* indptr, const int* indices,
                                const float* values, const void* w1frag, const float* b1, const float* W2,
                                const float* b2, const float* wo, const float* bo, const float* target, int N,
                                int r0, int r1, float* dy, float* slab1, int slab1_rows, float* slab2,
                                float* grad, float* loss, int num_cus, hipStream_t stream) {
  if (N <= 0 || r0 < 0 || r1 > N || r0 > r1) return hipErrorInvalidValue;
  const int hb = (N * 4 + 255) / 256;
  hipLaunchKernelGGL(gcn_head_bwd_kernel, dim3(hb), dim3(256), 0, stream, (const __bf16*)Z, indptr, indices,
                     values, b2, wo, bo, target, 2.f / (float)N, N, r0, r1, dy, slab2);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int ntiles = (r1 - r0 + 31) / 32;
  int grid = std::min(slab1_rows, std::max(8, std::min(num_cus, (ntiles + 3) / 4)));
  grid = grid / 8 * 8;
  if (grid < 8 || grid > slab1_rows) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gcn_l1_bwd_kernel, dim3(grid), dim3(256), 0, stream, (const __bf16*)X, indptr, indices,
                     values, (const bf16x8*)w1frag, b1, dy, r0, r1, slab1);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int ng = gcn_grad_numel() + 1;
  hipLaunchKernelGGL(gcn_grad_reduce_kernel, dim3((ng + 255) / 256), dim3(256), 0, stream, slab1, grid, slab2, hb,
                     W2, wo, grad, loss);
  return hipGetLastError();
}

int gcn_train_slab2_rows(int N) { return (N * 4 + 255) / 256; }

}  // namespace rt
