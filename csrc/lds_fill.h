// LDS staging helper for gfx950 kernels (device code only: not included by the host bindings,
// whose translation unit is not compiled for gfx950).
#pragma once
#include <hip/hip_runtime.h>

namespace rt {

// Block-wide copy of `nbytes` (multiple of 16) from global memory into LDS with
// global_load_lds_dwordx4: every wave-instruction moves 1 KB (lane l's 16 bytes land at base +
// 16 l), all of a thread's loads are in flight at once, and ONE vmcnt(0) + barrier ends it — a
// plain "load; wait; ds_write" loop pays the full load latency once per 16 bytes per thread
// (18 round trips for the 139 KB training blob).  Caller: every thread of the block.
__device__ __forceinline__ void lds_fill_block(unsigned char* lds, const unsigned char* src, int nbytes) {
  typedef __attribute__((address_space(3))) void lds_void_t;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int nk = nbytes >> 10;                       // whole 1 KB pieces
  for (int c = w; c < nk; c += nw)
    __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)c * 1024 + 16 * lane),
                                     (lds_void_t*)(lds + c * 1024), 16, 0, 0);
  const int done = nk << 10;
  for (int i = done + 16 * (int)threadIdx.x; i < nbytes; i += 16 * (int)blockDim.x)
    *reinterpret_cast<int4*>(lds + i) = *reinterpret_cast<const int4*>(src + i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

}  // namespace rt
