// MFMA issue-rate probe for train_bwd_kernel's hidden-tile loop (csrc/eta_mlp_train.hip): s_memtime
// cycles per v_mfma_f32_32x32x16_bf16 on one wave per SIMD (4-wave workgroups, one per CU), for the
// accumulator placements that kernel mixes.  The backward's segment timing (ROUTEST_TRAIN_BWD_PROF)
// showed ~64-72 cycles per MFMA in that loop against the 32 of a bare back-to-back stream.
//   mode 0: 4 chains, accumulators in AGPRs (inline asm "+a")
//   mode 1: 4 chains, accumulators in VGPRs (inline asm "+v")
//   mode 2: 2 AGPR chains + 2 VGPR chains interleaved (the backward's dW2 / dgrad pattern)
//   mode 3: 4 chains through the builtin
//   mode 4: as mode 2, 8 AGPR tiles rotating (acc2[4][2]) — each tile 2 MFMAs per round
//   mode 5: as mode 4, plus 2 ds_read_b128 + 2 ds_read_b64_tr_b16 per 8 MFMAs, consumed at once
//   mode 6: as mode 4, plus the loop's db2 block: ~33 VALU under `(mt >> 1) == wave` (an exec-mask
//           branch: the wave index comes from threadIdx)
//   mode 7: as mode 6 with the wave index through readfirstlane (a scalar branch)
//   mode 8: as mode 6 with the block computed unconditionally and selected (no branch)
// Build (CPU side): hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_rate_probe.hip -o tools/probes/bin/mfma_rate_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ void ma(f32x16& acc, const bf16x8 a, const bf16x8 b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mv(f32x16& acc, const bf16x8 a, const bf16x8 b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void probe(int iters, unsigned long long* cyc, float* sink) {
  __shared__ __attribute__((aligned(16))) unsigned char img[64 * 1024];
  for (int i = threadIdx.x; i < 64 * 1024 / 4; i += 256) reinterpret_cast<int*>(img)[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  bf16x8 a, b, c, d;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.001f * (lane + j));
    b[j] = (__bf16)(0.002f * (lane - j));
    c[j] = (__bf16)(0.003f * (j + 1));
    d[j] = (__bf16)(-0.001f * (lane ^ j));
  }
  f32x16 x0 = {}, x1 = {}, x2 = {}, x3 = {};
  f32x16 t[4][2] = {};
  float dbs[2] = {0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int nmfma = 0;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 2; ++k) { ma(x0, a, b); ma(x1, a, c); ma(x2, d, b); ma(x3, d, c); }
      nmfma += 8;
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 2; ++k) { mv(x0, a, b); mv(x1, a, c); mv(x2, d, b); mv(x3, d, c); }
      nmfma += 8;
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int k = 0; k < 2; ++k) { ma(x0, a, b); ma(x1, a, c); mv(x2, d, b); mv(x3, d, c); }
      nmfma += 8;
    } else if constexpr (MODE == 3) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        x0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, c, x1, 0, 0, 0);
        x2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(d, b, x2, 0, 0, 0);
        x3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(d, c, x3, 0, 0, 0);
      }
      nmfma += 8;
    } else {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        bf16x8 la = a, lb = d;
        if constexpr (MODE == 5) {
          const unsigned base = (unsigned)((lane * 16 + mt * 2048 + it * 64) & 0xFFF0);
          bf16x8 r0 = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>((uintptr_t)base);
          bf16x8 r1 = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>((uintptr_t)(base ^ 1024));
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)((base ^ 2048) & 0xFFF8));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)((base ^ 4096) & 0xFFF8));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          la = r0 + __builtin_bit_cast(bf16x8, v);
          lb = r1;
        }
        ma(t[mt][0], la, b);
        ma(t[mt][1], la, c);
        mv(x2, lb, b);
        mv(x3, lb, c);
        ma(t[mt][0], a, c);
        ma(t[mt][1], a, b);
        mv(x2, d, c);
        mv(x3, d, b);
        if constexpr (MODE >= 6) {
          int wv = threadIdx.x >> 6;
          if constexpr (MODE == 7) wv = __builtin_amdgcn_readfirstlane(wv);
          typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
          const u32x4v q0 = __builtin_bit_cast(u32x4v, la), q1 = __builtin_bit_cast(u32x4v, lb);
          float sacc = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            sacc += __uint_as_float(q0[q] << 16) + __uint_as_float(q0[q] & 0xFFFF0000u);
            sacc += __uint_as_float(q1[q] << 16) + __uint_as_float(q1[q] & 0xFFFF0000u);
          }
          if constexpr (MODE == 8) {
            dbs[mt & 1] += ((mt >> 1) == (wv & 1)) ? sacc : 0.f;
          } else {
            if ((mt >> 1) == (wv & 1)) dbs[mt & 1] += sacc;
          }
        }
      }
      nmfma += 32;
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    s += x0[e] + x1[e] + x2[e] + x3[e];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) s += t[mt][0][e] + t[mt][1][e];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = s + dbs[0] + dbs[1];
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = (t1 - t0) * 1000ull / (unsigned long long)nmfma;
}

template <int MODE>
static void run(int iters) {
  const int blocks = 256;
  unsigned long long* d_cyc;
  float* d_sink;
  (void)hipMalloc(&d_cyc, blocks * 4 * sizeof(unsigned long long));
  (void)hipMalloc(&d_sink, blocks * 256 * sizeof(float));
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, iters, d_cyc, d_sink);
  hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, iters, d_cyc, d_sink);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("mode %d: launch failed\n", MODE);
    std::exit(1);
  }
  unsigned long long h[blocks * 4];
  (void)hipMemcpy(h, d_cyc, sizeof h, hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < blocks * 4; ++i) sum += (double)h[i];
  std::printf("{\"mode\": %d, \"cycles_per_mfma\": %.2f}\n", MODE, sum / (blocks * 4) / 1000.0);
  (void)hipFree(d_cyc);
  (void)hipFree(d_sink);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  run<0>(iters);
  run<1>(iters);
  run<2>(iters);
  run<3>(iters);
  run<4>(iters / 4);
  run<5>(iters / 4);
  run<6>(iters / 4);
  run<7>(iters / 4);
  run<8>(iters / 4);
  return 0;
}
