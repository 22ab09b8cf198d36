// Price of a kernel boundary on one stream (gfx950): N dependent launches of a kernel that does
// (almost) nothing, for several grid sizes.  Used to decide whether the CCH customization's ~12 us
// per level (csrc/cch.hip, ~960 levels per phase) is the boundary or the level's own work (run r5t:
// 2.6 us per boundary at 1-64 workgroups, 4.3 us at 8192 — the rest is the level's work).
//
// Work-queue persistent variant (round 6).  The r5t version (commit d7bf79b) "never finished within
// its limit", and so did a first round-6 rewrite with wall-clock-bounded waits (run r6k: killed at
// 90 s without printing a line).  Root cause, from the gfx950 ISA of both: the loop's exits
// (`if (item >= total) return;`, `if (*fail) return;`) tested per-lane VGPR values — the item read
// back from LDS, the flag from memory — so the compiler could not prove them uniform and structurized
// `while (true)` into a per-lane nested loop.  After the item's last barrier, lane 0 of wave 0 leaves
// the inner loop (it alone must bump done[L] and fetch the next item), and lanes 1-63 of wave 0, with
// the three other waves, re-enter the next iteration's barrier / read-item sequence, re-reading the
// STALE item; the wave keeps executing the inner loop until lanes 1-63 leave it, which needs a new
// item, which needs lane 0: a livelock in which no wait ever starts, so no wait bound can fire.
// Fix: the exit tests use __builtin_amdgcn_readfirstlane copies (SGPRs: one uniform loop) and break.
// Also: an agent-scope ACQUIRE poll is `global_load ... sc1` + `buffer_inv sc1` (an L2 invalidate per
// iteration) — mode 1 polls RELAXED and fences once after the flag is seen; mode 0 keeps the acquire
// poll for comparison; both bound every wait by wall clock (s_memrealtime, 100 MHz).
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

// Persistent: `levels` levels of `per_level` items (one item = 64 lanes adding 1); a workgroup takes
// items in order from a global cursor and, before an item of level L, waits until every item of level
// L - 1 is done.  Every wait is bounded by wall clock (max_ticks of the 100 MHz s_memrealtime
// counter): on expiry *fail is set and every workgroup leaves at its next check, so the grid always
// drains.  mode 0: acquire load per poll (the r5t pattern); mode 1: relaxed polls + one acquire fence.
__global__ void persistent_kernel(int* p, int n, int levels, int per_level, int* cursor, int* done, int* fail,
                                  int mode, long long max_ticks) {
  __shared__ int item;
  __shared__ int failed;
  const int total = levels * per_level;
  int prev = -1;                         // level of the item finished in the previous iteration
  while (true) {
    // lane 0's work of one iteration in ONE block, right before the iteration's first barrier: the
    // release of the previous item and the fetch of the next (a block of lane-0 code on each side of
    // the back edge lets the structurizer split the loop per lane; see the header comment)
    if (threadIdx.x == 0) {
      if (prev >= 0) __hip_atomic_fetch_add(done + prev, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      item = atomicAdd(cursor, 1);
    }
    __syncthreads();
    // wave-uniform (SGPR) copies: the loop's exits must not depend on a per-lane value
    const int it = __builtin_amdgcn_readfirstlane(item);
    __syncthreads();
    if (it >= total) break;
    const int L = it / per_level;
    if (L > 0) {
      if (threadIdx.x == 0) {
        int f = 0;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (true) {
          const int d = mode == 0 ? __hip_atomic_load(done + L - 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                  : __hip_atomic_load(done + L - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (d >= per_level) break;
          if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
              (long long)__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) {
            __hip_atomic_fetch_or(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            f = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (mode != 0) __atomic_thread_fence(__ATOMIC_ACQUIRE);      // once, after the flag is seen
        failed = f;
      }
      __syncthreads();
      const int f = __builtin_amdgcn_readfirstlane(failed);
      __syncthreads();
      if (f) break;
    }
    const int i = (it % per_level) * 64 + (threadIdx.x & 63);
    if (threadIdx.x < 64 && i < n) __hip_atomic_fetch_add(p + i, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    prev = L;
  }
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
  // work-queue persistent kernel, both poll modes; every wait bounded at 20 ms of wall clock
  int *cursor = nullptr, *done = nullptr, *fail = nullptr;
  CK(hipMalloc(&cursor, sizeof(int)));
  CK(hipMalloc(&done, levels * sizeof(int)));
  CK(hipMalloc(&fail, sizeof(int)));
  const long long max_ticks = 2000000;   // 20 ms at 100 MHz
  for (int mode : {1, 0}) {
    for (int per_level : {1, 16, 128}) {
      for (int grid : {64, 256}) {
        for (int rep = 0; rep < 2; ++rep) {
          CK(hipMemsetAsync(cursor, 0, sizeof(int), s));
          CK(hipMemsetAsync(done, 0, levels * sizeof(int), s));
          CK(hipMemsetAsync(fail, 0, sizeof(int), s));
          CK(hipEventRecord(a, s));
          hipLaunchKernelGGL(persistent_kernel, dim3(grid), dim3(256), 0, s, p, n, levels, per_level, cursor, done, fail,
                             mode, max_ticks);
          CK(hipGetLastError());
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, a, b));
          int f = 0;
          CK(hipMemcpy(&f, fail, sizeof(int), hipMemcpyDeviceToHost));
          if (rep) {
            std::printf("{\"probe\": \"persistent\", \"poll\": \"%s\", \"grid\": %d, \"items_per_level\": %d, "
                        "\"levels\": %d, \"us_per_level\": %.3f, \"timed_out\": %d}\n",
                        mode ? "relaxed+fence" : "acquire", grid, per_level, levels, 1e3 * ms / levels, f);
            std::fflush(stdout);
          }
        }
      }
    }
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
