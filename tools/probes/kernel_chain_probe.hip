// Price of a kernel boundary on one stream (gfx950): N dependent launches of a kernel that does
// (almost) nothing, for several grid sizes.  Used to decide whether the CCH customization's ~12 us
// per level (csrc/cch.hip, ~960 levels per phase) is the boundary or the level's own work (run r5t:
// 2.6 us per boundary at 1-64 workgroups, 4.3 us at 8192 — the rest is the level's work).  (A
// work-queue persistent variant with per-level counters was tried in r5t and never finished within
// its limit; it is not kept.)
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/bin/kernel_chain_probe tools/probes/kernel_chain_probe.hip
//   tools/probes/bin/kernel_chain_probe [levels=200]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__global__ void touch_kernel(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1;
}

int main(int argc, char** argv) {
  const int levels = argc > 1 ? std::atoi(argv[1]) : 200;
  const int n = 1 << 22;
  int* p = nullptr;
  CK(hipMalloc(&p, n * sizeof(int)));
  CK(hipMemset(p, 0, n * sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int blocks : {1, 64, 1024, 8192}) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int l = 0; l < levels; ++l) hipLaunchKernelGGL(touch_kernel, dim3(blocks), dim3(256), 0, s, p, n);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep) {
        std::printf("{\"probe\": \"chain\", \"blocks\": %d, \"levels\": %d, \"us_per_kernel\": %.3f}\n", blocks, levels,
                    1e3 * ms / levels);
        std::fflush(stdout);
      }
    }
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
