// K8: 2-layer GCN road-graph route scorer on gfx950 (north-star config 4; no reference
// counterpart — the reference only calls remote routing engines, RO/Flaskr/utils.py:55,97,151).
//
//   H1    = relu( (Â X) W1 + b1 )          gcn_agg_gemm_kernel<FIN=32, FOUT=128, AGG=true>
//   Z     = H1 W2                          gcn_agg_gemm_kernel<128, 32, AGG=false>  (transform first:
//                                          aggregating 32 features is 4x cheaper than 128)
//   delay = 0.5 + softplus( (Â Z + b2) . wo + bo )   gcn_spmm_score_kernel (aggregation + head)
//   score(route) = sum_i delay(v_i) * |v_i v_{i+1}|   route_score_kernel (one wave per route)
//
// gcn_agg_gemm_kernel: each wave owns a 32-node tile.  Lanes are grouped FIN/8 per node (16 B of
// bf16 features each) and walk that node's CSR neighbour list with fp32 accumulation; the aggregated
// tile goes to the wave's private LDS tile (row-major, padded), which is directly the A operand
// (row = node, k = feature) of mfma_f32_32x32x16_bf16.  W is staged into LDS once per workgroup in
// B-fragment order (lane-linear 16-B reads).  The accumulator has the output feature on the lane,
// so the bias is a per-lane scalar and each result register is one node's 32 contiguous outputs.
#include "lds_fill.h"
#include "common.h"
#include "ops.h"

namespace rt {

// acc[0..8) += sum over CSR entries e0..e1 of values[e] * X[indices[e]][c .. c+8), in entry order
// (the same fp32 sums as a plain loop).  Entries go in batches of RB: all index/weight loads of a
// batch, then all RB feature-row loads, are in flight together — one memory round trip per level
// and batch instead of two dependent loads per edge (road-graph rows hold 3-9 entries).  Batch
// slots past e1 load row 0 (a valid address) and are masked out of the sum.
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

// The same for NP rows per lane at once (row p: entries e0[p]..e1[p], sums into acc[p]): batch b of
// every row is loaded together, so the NP rows share each round trip.
template <int RB, int NP>
__device__ __forceinline__ void csr_gather8_rows(const __bf16* __restrict__ X, int F, int c,
                                                 const int* __restrict__ indices,
                                                 const float* __restrict__ values,
                                                 const int (&e0)[NP], const int (&e1)[NP],
                                                 float (&acc)[NP][8]) {
  int nb = 0;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int n = (e1[p] - e0[p] + RB - 1) / RB;
    nb = n > nb ? n : nb;
  }
  for (int b = 0; b < nb; ++b) {
    int u[NP][RB];
    float wv[NP][RB];
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int e = e0[p] + b * RB + j;
        const bool in = e < e1[p];
        u[p][j] = in ? indices[e] : 0;
        wv[p][j] = in ? values[e] : 0.f;
      }
    bf16x8 x[NP][RB];
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < RB; ++j) x[p][j] = *reinterpret_cast<const bf16x8*>(X + (size_t)u[p][j] * F + c);
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < RB; ++j)
        if (e0[p] + b * RB + j < e1[p]) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[p][k] += wv[p][j] * (float)x[p][j][k];
        }
  }
}

template <int FIN, int FOUT, bool AGG, bool RELU>
__global__ __launch_bounds__(256) void gcn_agg_gemm_kernel(
    const __bf16* __restrict__ X, const int* __restrict__ indptr, const int* __restrict__ indices,
    const float* __restrict__ values, const bf16x8* __restrict__ wfrag, const float* __restrict__ bias,
    __bf16* __restrict__ Y, int row0, int row1) {
  constexpr int G = FIN / 8, RPP = 64 / G, KS = FIN / 16, NT = FOUT / 32;
  constexpr int LDT = FIN + 8;  // padded LDS row (bf16 elements): conflict-free ds_read_b128
  __shared__ __attribute__((aligned(16))) bf16x8 s_w[NT * KS * 64];
  __shared__ __attribute__((aligned(16))) __bf16 s_t[4][32 * LDT];
  lds_fill_block(reinterpret_cast<unsigned char*>(s_w), reinterpret_cast<const unsigned char*>(wfrag),
                 NT * KS * 64 * 16);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  __bf16* tile = s_t[w];
  const int n_rows = row1 - row0;
  const int ntiles = (n_rows + 31) / 32;
  // XCD-aware placement: workgroup b runs on XCD b % 8, so give each XCD one contiguous range of
  // node tiles (gridDim.x is a multiple of 8).  Neighbour rows of a road graph are nearby ids, so a
  // node's feature row is then re-read from the same XCD's L2 instead of from all eight.
  const int lb = (int)(blockIdx.x % 8u) * (int)(gridDim.x / 8u) + (int)(blockIdx.x / 8u);
  for (int t = lb * 4 + w; t < ntiles; t += gridDim.x * 4) {
    const int base = row0 + t * 32;
#pragma unroll
    for (int pass = 0; pass < 32 / RPP; ++pass) {
      const int rr = pass * RPP + lane / G;
      const int c = (lane % G) * 8;
      const int v = base + rr;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      if (v < row1) {
        if constexpr (AGG) {
          csr_gather8<8>(X, FIN, c, indices, values, indptr[v], indptr[v + 1], acc);
        } else {
          const bf16x8 x = *reinterpret_cast<const bf16x8*>(X + (size_t)v * FIN + c);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = (float)x[j];
        }
      }
      *reinterpret_cast<bf16x8*>(tile + rr * LDT + c) = to_bf16x8(acc);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // this wave's LDS writes complete (wave-private tile)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + (lane & 31) * LDT + 16 * ks + 8 * h);
        acc = mfma32(a, s_w[(nt * KS + ks) * 64 + lane], acc);
      }
      const int n = 32 * nt + (lane & 31);
      const float b = bias ? bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int v = base + (e & 3) + 8 * (e >> 2) + 4 * h;
        float o = acc[e] + b;
        if (RELU) o = relu_f(o);
        if (v < row1) Y[(size_t)v * FOUT + n] = (__bf16)o;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Fused layer 1 + layer-2 transform:  Z = relu((Â X) W1 + b1) W2  per 32-node wave tile.  H1 never
// leaves the wave's LDS tile: the unfused pair wrote H1 (N x 128 bf16 = 25.6 MB at 100k nodes) and
// read it back in a second launch.  H1 is rounded to bf16 in LDS exactly as the unfused path rounds
// it in HBM, and both GEMMs keep the unfused k order, so Z is bit-identical.  Z leaves through the
// LDS tile as 16-byte row chunks instead of one 2-byte store per accumulator register.
template <int FIN, int FHID, int FZ>
__global__ __launch_bounds__(256) void gcn_l1_fused_kernel(
    const __bf16* __restrict__ X, const int* __restrict__ indptr, const int* __restrict__ indices,
    const float* __restrict__ values, const bf16x8* __restrict__ w1frag, const float* __restrict__ b1,
    const bf16x8* __restrict__ w2frag, __bf16* __restrict__ Z, int row0, int row1) {
  constexpr int G = FIN / 8, RPP = 64 / G, KS1 = FIN / 16, NT1 = FHID / 32, KS2 = FHID / 16, NT2 = FZ / 32;
  constexpr int LDA = FIN + 8, LDH = FHID + 8, LDZ = FZ + 8;
  constexpr int TILE = 32 * (LDH > LDA ? LDH : LDA);
  __shared__ __attribute__((aligned(16))) bf16x8 s_w1[NT1 * KS1 * 64];
  __shared__ __attribute__((aligned(16))) bf16x8 s_w2[NT2 * KS2 * 64];
  __shared__ __attribute__((aligned(16))) __bf16 s_t[4][TILE];
  lds_fill_block(reinterpret_cast<unsigned char*>(s_w1), reinterpret_cast<const unsigned char*>(w1frag),
                 NT1 * KS1 * 64 * 16);
  lds_fill_block(reinterpret_cast<unsigned char*>(s_w2), reinterpret_cast<const unsigned char*>(w2frag),
                 NT2 * KS2 * 64 * 16);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  __bf16* tile = s_t[w];
  const int ntiles = (row1 - row0 + 31) / 32;
  float bias[NT1];
#pragma unroll
  for (int nt = 0; nt < NT1; ++nt) bias[nt] = b1[32 * nt + (lane & 31)];
  const int lb = (int)(blockIdx.x % 8u) * (int)(gridDim.x / 8u) + (int)(blockIdx.x / 8u);
  for (int t = lb * 4 + w; t < ntiles; t += gridDim.x * 4) {
    const int base = row0 + t * 32;
    // (1) aggregation Â X of the tile's 32 nodes -> A tile [32][LDA]: every lane gathers its rows of
    // all passes together (one round trip per CSR level for the whole tile)
    {
      constexpr int NP = 32 / RPP;
      const int c = (lane % G) * 8;
      int e0[NP], e1[NP];
      float acc[NP][8];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int v = base + p * RPP + lane / G;
        e0[p] = v < row1 ? indptr[v] : 0;
        e1[p] = v < row1 ? indptr[v + 1] : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[p][j] = 0.f;
      }
      csr_gather8_rows<8, NP>(X, FIN, c, indices, values, e0, e1, acc);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        *reinterpret_cast<bf16x8*>(tile + (p * RPP + lane / G) * LDA + c) = to_bf16x8(acc[p]);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // (2) layer 1 GEMM (+bias, ReLU): accumulators keep the hidden unit on the lane
    f32x16 h1[NT1];
#pragma unroll
    for (int nt = 0; nt < NT1; ++nt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) h1[nt][e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS1; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + (lane & 31) * LDA + 16 * ks + 8 * h);
        h1[nt] = mfma32(a, s_w1[(nt * KS1 + ks) * 64 + lane], h1[nt]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();          // A tile consumed: the region now holds H1 [32][LDH]
#pragma unroll
    for (int nt = 0; nt < NT1; ++nt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;
        tile[rr * LDH + 32 * nt + (lane & 31)] = (__bf16)relu_f(h1[nt][e] + bias[nt]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // (3) transform Z = H1 W2
    f32x16 z[NT2];
#pragma unroll
    for (int nt = 0; nt < NT2; ++nt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) z[nt][e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + (lane & 31) * LDH + 16 * ks + 8 * h);
        z[nt] = mfma32(a, s_w2[(nt * KS2 + ks) * 64 + lane], z[nt]);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();          // H1 consumed: the region now holds Z [32][LDZ]
#pragma unroll
    for (int nt = 0; nt < NT2; ++nt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;
        tile[rr * LDZ + 32 * nt + (lane & 31)] = (__bf16)z[nt][e];
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // (4) 16-byte row-chunk stores of the tile's Z rows
    constexpr int CPR = FZ / 8;               // 16-byte chunks per row
#pragma unroll
    for (int q = lane; q < 32 * CPR; q += 64) {
      const int rr = q / CPR, c8 = q % CPR;
      if (base + rr < row1)
        *reinterpret_cast<bf16x8*>(Z + (size_t)(base + rr) * FZ + 8 * c8) =
            *reinterpret_cast<const bf16x8*>(tile + rr * LDZ + 8 * c8);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();          // tile free for the next aggregation
  }
}

// delay[v] = 0.5 + softplus( sum_f (sum_u Â[v,u] Z[u,f] + b2[f]) * wo[f] + bo ),  F = 32 (4 lanes/row)
__global__ __launch_bounds__(256) void gcn_spmm_score_kernel(
    const __bf16* __restrict__ Z, const int* __restrict__ indptr, const int* __restrict__ indices,
    const float* __restrict__ values, const float* __restrict__ b2, const float* __restrict__ wo,
    float bo, float* __restrict__ delay, int row0, int row1) {
  constexpr int F = 32, G = F / 8;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int v = row0 + gid / G;
  const int c = (gid % G) * 8;
  float part = 0.f;
  if (v < row1) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    csr_gather8<8>(Z, F, c, indices, values, indptr[v], indptr[v + 1], acc);
#pragma unroll
    for (int j = 0; j < 8; ++j) part += (acc[j] + b2[c + j]) * wo[c + j];
  }
  part += __shfl_xor(part, 1);
  part += __shfl_xor(part, 2);
  if (v < row1 && (gid % G) == 0) {
    const float x = part + bo;
    const float sp = x > 20.f ? x : log1pf(expf(x));
    delay[v] = 0.5f + sp;
  }
}

// score[r] = sum_i delay[v_i] * haversine(v_i, v_{i+1}) over route r's node list (one wave / route).
// The kernel is bound by the texture path's gather rate (each wave-load of 64 random node ids
// touches up to 64 cache lines), not by latency: issuing 4 segments' loads ahead was slower.  So
// each node is gathered ONCE: lane l of a 64-node window loads node i = i0 + l (lat/lon as one
// 8-byte pair, its delay), and takes v_{i+1}'s position from lane l + 1 (ds_bpermute); windows
// advance by 63 nodes.  2 gathers per segment instead of 5 (lat, lon of both ends + delay).
// Node ids outside [0, N) contribute nothing.
__global__ __launch_bounds__(256) void route_score_kernel(const int* __restrict__ rptr,
                                                          const int* __restrict__ nodes,
                                                          const float2* __restrict__ latlon,
                                                          const float* __restrict__ delay,
                                                          float* __restrict__ score, int R, int N) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= R) return;
  const int p0 = rptr[r], p1 = rptr[r + 1];
  float s = 0.f;
  const float k = 0.017453292519943295f;
  for (int i0 = p0; i0 < p1 - 1; i0 += 63) {
    const int i = i0 + lane;
    const int a = i < p1 ? nodes[i] : -1;
    const bool ok = a >= 0 && a < N;
    const float2 ll = ok ? latlon[a] : make_float2(0.f, 0.f);
    const float dv = ok ? delay[a] : 0.f;
    const float lat2 = __shfl_down(ll.x, 1), lon2 = __shfl_down(ll.y, 1);
    const int b = __shfl_down(a, 1);
    if (lane < 63 && i + 1 < p1 && ok && b >= 0 && b < N) {
      const float la1 = ll.x * k, la2 = lat2 * k;
      const float dphi = la2 - la1, dl = (lon2 - ll.y) * k;
      const float s1 = __sinf(0.5f * dphi), s2 = __sinf(0.5f * dl);
      const float hv = s1 * s1 + __cosf(la1) * __cosf(la2) * s2 * s2;
      const float d = 2.f * 6371000.f * asinf(sqrtf(fminf(1.f, fmaxf(0.f, hv))));
      s += dv * d;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) score[r] = s;
}

hipError_t launch_gcn_agg_gemm(const void* X, const int* indptr, const int* indices,
                               const float* values, const void* wfrag, const float* bias, void* Y,
                               int fin, int fout, bool agg, bool relu, int row0, int row1,
                               int num_cus, hipStream_t stream) {
  const int ntiles = (row1 - row0 + 31) / 32;
  if (ntiles <= 0) return hipSuccess;
  int grid = (ntiles + 3) / 4;
  if (grid > num_cus * 4) grid = num_cus * 4;
  grid = (grid + 7) / 8 * 8;   // XCD remap in the kernel needs a multiple of 8 (extra WGs idle)
#define RT_GCN(FI, FO, AG, RL)                                                                   \
  if (fin == FI && fout == FO && agg == AG && relu == RL) {                                      \
    hipLaunchKernelGGL((gcn_agg_gemm_kernel<FI, FO, AG, RL>), dim3(grid), dim3(256), 0, stream,  \
                       (const __bf16*)X, indptr, indices, values, (const bf16x8*)wfrag, bias,    \
                       (__bf16*)Y, row0, row1);                                                  \
    return hipGetLastError();                                                                    \
  }
  RT_GCN(32, 128, true, true)
  RT_GCN(128, 32, false, false)
  RT_GCN(64, 64, true, true)
  RT_GCN(32, 32, true, true)
  RT_GCN(128, 128, true, true)
#undef RT_GCN
  return hipErrorInvalidValue;
}

hipError_t launch_gcn_l1_fused(const void* X, const int* indptr, const int* indices, const float* values,
                               const void* w1frag, const float* b1, const void* w2frag, void* Z, int fin,
                               int fhid, int fz, int row0, int row1, int num_cus, hipStream_t stream) {
  const int ntiles = (row1 - row0 + 31) / 32;
  if (ntiles <= 0) return hipSuccess;
  if (fin != 32 || fhid != 128 || fz != 32) return hipErrorInvalidValue;
  int grid = (ntiles + 3) / 4;
  if (grid > num_cus * 4) grid = num_cus * 4;
  grid = (grid + 7) / 8 * 8;
  hipLaunchKernelGGL((gcn_l1_fused_kernel<32, 128, 32>), dim3(grid), dim3(256), 0, stream, (const __bf16*)X,
                     indptr, indices, values, (const bf16x8*)w1frag, b1, (const bf16x8*)w2frag, (__bf16*)Z, row0,
                     row1);
  return hipGetLastError();
}

hipError_t launch_gcn_spmm_score(const void* Z, const int* indptr, const int* indices,
                                 const float* values, const float* b2, const float* wo, float bo,
                                 float* delay, int row0, int row1, hipStream_t stream) {
  const long long threads = (long long)(row1 - row0) * 4;
  if (threads <= 0) return hipSuccess;
  hipLaunchKernelGGL(gcn_spmm_score_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     stream, (const __bf16*)Z, indptr, indices, values, b2, wo, bo, delay, row0,
                     row1);
  return hipGetLastError();
}

hipError_t launch_route_score(const int* rptr, const int* nodes, const float* latlon,
                              const float* delay, float* score, int R, int N, hipStream_t stream) {
  if (R <= 0) return hipSuccess;
  hipLaunchKernelGGL(route_score_kernel, dim3((R + 3) / 4), dim3(256), 0, stream, rptr, nodes,
                     (const float2*)latlon, delay, score, R, N);
  return hipGetLastError();
}

}  // namespace rt
