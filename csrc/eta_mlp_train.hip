// K3: data-parallel training of the 3-layer ETA MLP on gfx950 — fused forward/loss kernel,
// ReLU backward, and fused AdamW + MFMA-fragment re-pack.  (The reference has no training code at
// all: notebooks/.gitkeep; its feature schema is RO/Flaskr/ml.py:35-51.)
//
// One training step on a rank (routest_amd/train/fused.py::FusedMlp3Trainer):
//   1. eta_mlp3_train_fwd_kernel (this file): featurize + layer 1 + layer 2 + layer 3 + MSE
//      gradient in ONE launch, same wave/tile structure and LDS-staged weight blob as inference.
//      Because dL/dz2 = dy * w3 * relu'(z2) needs only the ReLU mask, dz2 is produced in-register
//      the moment y (hence dy) is known — no second pass.  Emits, bf16 row-major:
//        xf  [B,16]   the exact bf16 features the MFMA consumed, slot 14 := 1 (bias-grad column)
//        h1a [B,H+16] relu(z1) with column H := 1   (dW2 | db2 = dz2^T h1a)
//        h2a [B,H+16] relu(z2) with column H := 1   (dW3 | db3 = dy^T h2a)
//        dz2 [B,H], dy [B,8] (col 0; pre-scaled by 2 / global_batch), per-tile squared errors.
//   2. dh1 = dz2 W2 on hipBLASLt (a plain [B,H]x[H,H] GEMM); the three weight-gradient GEMMs
//      (K = batch) on the split-K wgrad kernel (wgrad.hip) + one deterministic slab reduction.
//   3. relu_bwd_kernel: dz1 = dh1 * (h1 > 0).
//   4. ONE flat fp32 gradient bucket -> one RCCL all-reduce over xGMI.
//   5. adamw_pack_kernel: AdamW on the flat fp32 master params, writing back the bf16 fragment
//      blob the next forward stages into LDS (and a row-major bf16 W2 for step 2) — no host work,
//      no sync, so the whole step is capturable in a HIP graph.
#include "mlp3_tile.h"
#include "ops.h"

namespace rt {

// Stored hidden-unit order of the saved activations h1a / h2a / dz2 (and of the gradient bucket
// and w2bf built from them): element j of fragment ks on lane half h is hidden unit
// u = 16ks + 8(j>>2) + 4h + (j&3); storing it at column c = 16ks + 8h + j (= u with bits 2 and 3
// swapped, an involution) makes each lane's 8 values ONE contiguous 16-byte store instead of two
// 8-byte ones — the forward's activation writes went 42 -> 29 us at 65k rows.  adamw_pack_kernel
// reads the bucket through hperm() and train/fused.py::grads_from_bucket mirrors it.
__host__ __device__ __forceinline__ int hperm(int u) { return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1); }

template <int H>
__device__ __forceinline__ void store_act(__bf16* base_row, const bf16x8 (&a)[H / 16], int h) {
#pragma unroll
  for (int ks = 0; ks < H / 16; ++ks) *reinterpret_cast<bf16x8*>(base_row + 16 * ks + 8 * h) = a[ks];
}

// 8 waves per workgroup (2 per SIMD; <= 256 VGPRs incl. register-resident W1 fragments).
template <int H>
constexpr int train_tpb() { return 512; }

template <int H>
__global__ __launch_bounds__(512, 2) void eta_mlp3_train_fwd_kernel(
    const int4* __restrict__ rec, const float* __restrict__ target, int B,
    const unsigned char* __restrict__ blob, NormParams np, float gscale, __bf16* __restrict__ xf,
    __bf16* __restrict__ h1a, __bf16* __restrict__ h2a, __bf16* __restrict__ dz2,
    __bf16* __restrict__ dyb, float* __restrict__ loss_tiles, int* __restrict__ step_ctr) {
  constexpr int MT = H / 32, KS = H / 16, LDA = H + 16;
  // device-side optimizer step counter (read by adamw_pack_kernel later on the same stream), so a
  // captured HIP graph replays with correct bias corrections / LR schedule
  if (step_ctr != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *step_ctr += 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  stage_blob<H>(blob, smem);
  const Mlp3View<H> w(smem);
  const float b3 = w.tail[0];
  W1Frags<H> w1;
  w1.load(w, threadIdx.x & 63);

  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int r = lane & 31;
  const int wpb = blockDim.x >> 6;
  const int ntiles = (B + 31) >> 5;
  const int stride = gridDim.x * wpb;

  for (int tile = blockIdx.x * wpb + (threadIdx.x >> 6); tile < ntiles; tile += stride) {
    const int row = tile * 32 + r;
    const bool valid = row < B;
    const int4 rc = valid ? rec[row] : make_int4(0, 0, 0, 0);
    const bf16x8 xb = featurize_bf16(rc, h, np);
    if (valid)  // slots 14, 15 hold 1.0 (the b1 hi/lo inputs): dW1k[:,14] == db1
      *reinterpret_cast<bf16x8*>(xf + (size_t)row * 16 + 8 * h) = xb;

    bf16x8 h1[KS];
    mlp3_layer1<H>(w1, xb, h1);
    __bf16* h1row = h1a + (size_t)row * LDA;
    __bf16* h2row = h2a + (size_t)row * LDA;
    if (valid) {
      store_act<H>(h1row, h1, h);
      bf16x8 tailv;
#pragma unroll
      for (int j = 0; j < 8; ++j) tailv[j] = (__bf16)0.f;
      if (h == 0) tailv[0] = (__bf16)1.f;
      *reinterpret_cast<bf16x8*>(h1row + H + 8 * h) = tailv;
      *reinterpret_cast<bf16x8*>(h2row + H + 8 * h) = tailv;
    }

    // layer 2 + layer 3; relu(z2) goes straight to memory, only its mask stays in registers
    unsigned long long mask_lo = 0, mask_hi = 0;   // 16 mask bits per 32-row hidden tile
    float ys = 0.f;
    mlp3_layer2<H>(w, h1, lane, h, [&](int mt, const f32x16& acc) {
      const f32x16 w3 = load_vec16(w.w3p, mt, h);
      unsigned mk = 0;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 hv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = relu_f(acc[8 * s + j]);
          ys += v * w3[8 * s + j];
          hv[j] = (__bf16)v;
          mk |= (v > 0.f ? 1u : 0u) << (8 * s + j);
        }
        if (valid) {
          *reinterpret_cast<bf16x8*>(h2row + 16 * (2 * mt + s) + 8 * h) = hv;   // hperm order
        }
      }
      if (mt < 4) mask_lo |= (unsigned long long)mk << (16 * mt);
      else mask_hi |= (unsigned long long)mk << (16 * (mt - 4));
    });
    ys += __shfl_xor(ys, 32);
    const float y = ys + b3;
    const float diff = valid ? (y - target[row]) : 0.f;
    const float dy = gscale * diff;
    if (valid && h == 0) {  // dy as an [B,8] bf16 operand (cols 1..7 zero) for the wgrad kernel
      bf16x8 dv;
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[j] = (__bf16)0.f;
      dv[0] = (__bf16)dy;
      *reinterpret_cast<bf16x8*>(dyb + (size_t)row * 8) = dv;
    }
    // per-tile squared error (h = 0 half only), wave reduction
    float l = (h == 0) ? diff * diff : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) l += __shfl_xor(l, o);
    if (lane == 0) loss_tiles[tile] = l;

    // dz2 = dy * w3 * relu'(z2), in fragment order, stored row-major
    if (valid) {
      __bf16* drow = dz2 + (size_t)row * H;
#pragma unroll 1
      for (int mt = 0; mt < MT; ++mt) {
        const f32x16 w3 = load_vec16(w.w3p, mt, h);
        const unsigned mk = (unsigned)((mt < 4 ? mask_lo >> (16 * mt) : mask_hi >> (16 * (mt - 4))) & 0xffffu);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 d;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            d[j] = (__bf16)(((mk >> (8 * s + j)) & 1u) ? dy * w3[8 * s + j] : 0.f);
          *reinterpret_cast<bf16x8*>(drow + 16 * (2 * mt + s) + 8 * h) = d;     // hperm order
        }
      }
    }
  }
}

// dz1[b][o] = dh1[b][o] * (h1a[b][o] > 0), 8 bf16 per thread.
__global__ __launch_bounds__(256) void relu_bwd_kernel(const __bf16* __restrict__ dh1,
                                                       const __bf16* __restrict__ h1a, int lda,
                                                       __bf16* __restrict__ dz1, int B, int H) {
  const long long i8 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = H / 8;
  if (i8 >= (long long)B * per_row) return;
  const long long b = i8 / per_row;
  const int c = (int)(i8 - b * per_row) * 8;
  const bf16x8 g = *reinterpret_cast<const bf16x8*>(dh1 + b * H + c);
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(h1a + b * lda + c);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)a[j] > 0.f ? g[j] : (__bf16)0.f;
  *reinterpret_cast<bf16x8*>(dz1 + b * H + c) = o;
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
                                                         __bf16* __restrict__ w2bf,
                                                         const int* __restrict__ step, AdamWArgs a) {
  using L = Mlp3Layout<H>;
  constexpr int KS = H / 16;
  constexpr int OFF_B1 = 12 * H, OFF_W2 = 13 * H, OFF_B2 = 13 * H + H * H, OFF_W3 = OFF_B2 + H,
                OFF_B3 = OFF_W3 + H, N = OFF_B3 + 1;
  constexpr int LDG = H + 16;
  const float* gW2a = G;
  const float* gW3a = G + H * LDG;
  const float* gW1a = gW3a + LDG;
  __bf16* w2p = reinterpret_cast<__bf16*>(blob);
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
    const int po = hperm(o);
    g = gW1a[po * 16 + i];
    if (i == 10) g += gW1a[po * 16 + 12];
    if (i == 11) g += gW1a[po * 16 + 13];
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
    const int mt = o >> 5, rr = o & 31;
    const int ks = i >> 4, c = i & 15;
    const int hh = (c >> 2) & 1;
    const int j = 4 * (c >> 3) + (c & 3);
    const int ln = rr + 32 * hh;
    w2p[((size_t)((mt * KS + ks) * 64 + ln)) * 8 + j] = (__bf16)p;
    w2bf[(size_t)hperm(o) * H + hperm(i)] = (__bf16)p;   // rows/cols in the stored (hperm) order
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
static hipError_t launch_train_fwd_h(const void* rec, const float* target, int B, const void* blob,
                                     const NormParams& np, float gscale, void* xf, void* h1a,
                                     void* h2a, void* dz2, void* dyb, float* loss_tiles,
                                     int* step_ctr, int num_cus, hipStream_t stream) {
  using L = Mlp3Layout<H>;
  static bool attr_set[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!attr_set[dev & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)eta_mlp3_train_fwd_kernel<H>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::BLOB);
    if (e != hipSuccess) return e;
    attr_set[dev & 63] = true;
  }
  const int ntiles = (B + 31) / 32;
  constexpr int TPB = train_tpb<H>();
  int grid = (ntiles + TPB / 64 - 1) / (TPB / 64);
  if (grid > num_cus) grid = num_cus;
  if (grid < 1) return hipSuccess;
  hipLaunchKernelGGL(eta_mlp3_train_fwd_kernel<H>, dim3(grid), dim3(TPB), L::BLOB, stream,
                     (const int4*)rec, target, B, (const unsigned char*)blob, np, gscale,
                     (__bf16*)xf, (__bf16*)h1a, (__bf16*)h2a, (__bf16*)dz2, (__bf16*)dyb,
                     loss_tiles, step_ctr);
  return hipGetLastError();
}

hipError_t launch_eta_mlp3_train_fwd(const void* rec, const float* target, int B, const void* blob,
                                     int H, const NormParams& np, float gscale, void* xf,
                                     void* h1a, void* h2a, void* dz2, void* dyb,
                                     float* loss_tiles, int* step_ctr, int num_cus,
                                     hipStream_t stream) {
  switch (H) {
    case 64: return launch_train_fwd_h<64>(rec, target, B, blob, np, gscale, xf, h1a, h2a, dz2, dyb, loss_tiles, step_ctr, num_cus, stream);
    case 128: return launch_train_fwd_h<128>(rec, target, B, blob, np, gscale, xf, h1a, h2a, dz2, dyb, loss_tiles, step_ctr, num_cus, stream);
    case 256: return launch_train_fwd_h<256>(rec, target, B, blob, np, gscale, xf, h1a, h2a, dz2, dyb, loss_tiles, step_ctr, num_cus, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_relu_bwd(const void* dh1, const void* h1a, int lda, void* dz1, int B, int H,
                           hipStream_t stream) {
  const long long n = (long long)B * (H / 8);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const __bf16*)dh1, (const __bf16*)h1a, lda, (__bf16*)dz1, B, H);
  return hipGetLastError();
}

int mlp3_num_params(int H) { return H * H + 15 * H + 1; }
int mlp3_grad_bucket_floats(int H) { return H * (H + 16) + (H + 16) + 16 * H; }

hipError_t launch_adamw_pack(float* P, const float* G, float* M, float* V, void* blob, void* w2bf,
                             const int* step, int H, float lr, float beta1, float beta2, float eps,
                             float wd, int warmup, int total_steps, float min_lr_ratio, int update,
                             hipStream_t stream) {
  AdamWArgs a{lr, beta1, beta2, eps, wd, warmup, total_steps, min_lr_ratio, update};
  const int N = mlp3_num_params(H);
  const dim3 grid((N + 255) / 256), block(256);
  switch (H) {
    case 64: hipLaunchKernelGGL(adamw_pack_kernel<64>, grid, block, 0, stream, P, G, M, V, (unsigned char*)blob, (__bf16*)w2bf, step, a); break;
    case 128: hipLaunchKernelGGL(adamw_pack_kernel<128>, grid, block, 0, stream, P, G, M, V, (unsigned char*)blob, (__bf16*)w2bf, step, a); break;
    case 256: hipLaunchKernelGGL(adamw_pack_kernel<256>, grid, block, 0, stream, P, G, M, V, (unsigned char*)blob, (__bf16*)w2bf, step, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace rt
