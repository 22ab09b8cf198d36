// Price of a kernel boundary on one stream (gfx950): N dependent launches of a kernel that does
// (almost) nothing, for several grid sizes, and the same work as one persistent kernel whose
// workgroups pass N grid-wide "levels" through a device-scope counter (a work-queue wait: a
// workgroup waits only for levels every running workgroup has already taken, so it never needs
// the whole grid resident).  Used to decide whether the CCH customization's ~12 us per level
// (csrc/cch.hip, ~960 levels per phase) is the boundary or the level's own work.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/bin/kernel_chain_probe tools/probes/kernel_chain_probe.hip
//   tools/probes/bin/kernel_chain_probe [levels=1000]
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

// Persistent: `levels` levels of `per_level` items (one item = one wave's worth: 64 lanes add 1);
// a workgroup takes items in order from a global cursor and, before an item of level L, waits until
// every item of level L-1 is done.  Bounded wait (spin cap): on expiry the kernel sets *fail and
// every workgroup leaves, so a scheduling surprise can never hang the GPU.
__global__ void persistent_kernel(int* p, int n, int levels, int per_level, int* cursor, int* done, int* fail) {
  __shared__ int item;
  const int total = levels * per_level;
  while (true) {
    if (threadIdx.x == 0) item = atomicAdd(cursor, 1);
    __syncthreads();
    const int it = item;
    __syncthreads();
    if (it >= total) return;
    const int L = it / per_level;
    if (L > 0) {
      if (threadIdx.x == 0) {
        long spins = 0;
        while (__hip_atomic_load(done + L - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < per_level) {
          if (++spins > (1L << 26) || __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            atomicExch(fail, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
    const int i = (it % per_level) * 64 + (threadIdx.x & 63);
    if (threadIdx.x < 64 && i < n) __hip_atomic_fetch_add(p + i, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(done + L, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main(int argc, char** argv) {
  const int levels = argc > 1 ? std::atoi(argv[1]) : 1000;
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
      if (rep) std::printf("{\"probe\": \"chain\", \"blocks\": %d, \"levels\": %d, \"us_per_kernel\": %.3f}\n", blocks, levels,
                           1e3 * ms / levels);
    }
  }
  int *cursor = nullptr, *done = nullptr, *fail = nullptr;
  CK(hipMalloc(&cursor, sizeof(int)));
  CK(hipMalloc(&done, levels * sizeof(int)));
  CK(hipMalloc(&fail, sizeof(int)));
  for (int per_level : {1, 16, 128}) {
    for (int grid : {64, 256}) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemsetAsync(cursor, 0, sizeof(int), s));
        CK(hipMemsetAsync(done, 0, levels * sizeof(int), s));
        CK(hipMemsetAsync(fail, 0, sizeof(int), s));
        CK(hipEventRecord(a, s));
        hipLaunchKernelGGL(persistent_kernel, dim3(grid), dim3(256), 0, s, p, n, levels, per_level, cursor, done, fail);
        CK(hipGetLastError());
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        int f = 0;
        CK(hipMemcpy(&f, fail, sizeof(int), hipMemcpyDeviceToHost));
        if (rep)
          std::printf("{\"probe\": \"persistent\", \"grid\": %d, \"items_per_level\": %d, \"levels\": %d, \"us_per_level\": %.3f, \"failed\": %d}\n",
                      grid, per_level, levels, 1e3 * ms / levels, f);
      }
    }
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
