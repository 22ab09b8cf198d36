// Persistent single-request scorer: the fused featurize + 3-layer MLP (K1+K2) kept RESIDENT on one
// CU and fed through a doorbell in pinned host memory, for the latency path of /api/predict_eta
// (SURVEY §7.5 hard part 2; §2.6 K2 "persistent-kernel option for small B").
//
// A normal launch per request costs a kernel dispatch, a cold weight fetch from L2 into the waves
// and a hipStreamSynchronize wake-up (~20 us of the 27 us native end-to-end p50,
// profiles/latency_breakdown_r1.json).  Here one 8-wave workgroup stages the 139 KiB weight blob
// into LDS ONCE and then loops:
//
//   wave 0 lane 0 polls mailbox.seq (system-scope loads of host memory, s_sleep between polls)
//   -> all 8 waves score the n <= cap records of the request (one 32-row MFMA tile per wave per
//      round, records read with system-scope loads, minutes written with system-scope stores
//      straight into the host's output slots)
//   -> next poll.
//
// Completion needs no flag and no release fence: the host fills the output slots with a
// signalling-NaN sentinel before ringing the doorbell and spins until no slot holds it (each
// 4-byte store is single-copy atomic; the kernel's results are never that bit pattern).
//
// Termination (every wave reaches it): mailbox.stop, `idle_ms` without a request, or `life_ms` of
// residency (checked between requests) — the kernel exits and the host relaunches it on the next
// request (pscore_run).  The lifetime bound matters because HIP multiplexes streams onto a few
// hardware queues (GPU_MAX_HW_QUEUES): a kernel that never ends would stall whatever else shares
// its queue.  The host parks the scorer (pscore_park) before its own large launches, bounds its
// wait, and falls back to a normal launch when the scorer does not answer.
#include <atomic>
#include <chrono>
#include <cstring>

#include "mlp3_tile.h"
#include "ops.h"

namespace rt {

struct alignas(64) ServeMailbox {
  unsigned seq;        // host -> GPU: doorbell (incremented per request batch)
  unsigned n;          // rows in this batch
  unsigned stop;       // host -> GPU: exit now
  unsigned pad[13];
};

constexpr unsigned kOutSentinel = 0x7fa5a5a5u;   // signalling NaN payload (never produced)
constexpr size_t kXchBytes = 4 * 4 * 64 * 16;     // single-tile mode: relu(z2) of 4 hidden tiles

__device__ __forceinline__ unsigned sys_load_u32(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int H>
__global__ __launch_bounds__(512, 1) void eta_mlp3_serve_kernel(ServeMailbox* mb, const int4* rec,
                                                                unsigned* out, int cap,
                                                                const unsigned char* __restrict__ blob,
                                                                NormParams np, unsigned last,
                                                                unsigned long long idle_ticks,
                                                                unsigned long long life_ticks) {
  constexpr int KS = H / 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ unsigned s_cmd[2];
  stage_blob<H>(blob, smem);
  const Mlp3View<H> w(smem);
  const float b3 = w.tail[0];
  W1Frags<H> w1;
  w1.load(w, threadIdx.x & 63);
  const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31, wave = threadIdx.x >> 6;
  const unsigned long long t_start = wall_clock64();

  while (true) {
    if (threadIdx.x == 0) {
      const unsigned long long t0 = wall_clock64();
      unsigned seq = last, n = 0;
      bool quit = false;
      while (true) {
        if (sys_load_u32(&mb->stop)) { quit = true; break; }
        seq = sys_load_u32(&mb->seq);
        if (seq != last) { n = sys_load_u32(&mb->n); break; }
        const unsigned long long now = wall_clock64();
        // idle, or resident for long enough: give the hardware queue back (only ever between
        // requests, so no doorbell is left half-served)
        if (now - t0 > idle_ticks || now - t_start > life_ticks) { quit = true; break; }
        __builtin_amdgcn_s_sleep(8);
      }
      s_cmd[0] = quit ? 1u : 0u;
      s_cmd[1] = quit ? 0u : (n > (unsigned)cap ? (unsigned)cap : n);
      last = seq;
    }
    __syncthreads();
    const bool quit = s_cmd[0] != 0;
    const int n = (int)s_cmd[1];
    __syncthreads();              // s_cmd is rewritten only after every wave has read it
    if (quit) break;
    const int ntiles = (n + 31) >> 5;
    if (ntiles == 1) {
      // one tile (n <= 32, the single-request case): split its layer 2 over the waves — wave w
      // computes hidden tile mt = w (16 MFMAs instead of 128 in one wave) — and let wave 0 run the
      // layer-3 dot over all tiles in the SAME order as the per-wave path, so the minutes are
      // bit-identical to the normal kernel.  relu(z2) of 4 tiles at a time goes through LDS
      // (16 KiB; the weight blob leaves ~21 KiB free).
      constexpr int MT = H / 32;
      const int row = r;
      int4 rc = make_int4(0, 0, 0, 0);
      if (row < n) {
        const unsigned long long* p = reinterpret_cast<const unsigned long long*>(rec + row);
        const unsigned long long lo = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long hi = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        rc = make_int4((int)lo, (int)(lo >> 32), (int)hi, (int)(hi >> 32));
      }
      f32x16 z;                                   // relu(z2) of hidden tile mt = wave
      if (wave < MT) {
        const bf16x8 xb = featurize_bf16(rc, h, np);
        bf16x8 h1[KS];
        mlp3_layer1<H>(w1, xb, h1);
        const bf16x8* wa = w.w2p + lane + wave * KS * 64;
        z = load_vec16(w.b2p, wave, h);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) z = mfma32(wa[ks * 64], h1[ks], z);
#pragma unroll
        for (int i = 0; i < 16; ++i) z[i] = relu_f(z[i]);
      }
      f32x4* xch = reinterpret_cast<f32x4*>(smem + Mlp3Layout<H>::BLOB);   // [4 tiles][4][64 lanes]
      f32x2 ys2 = {0.f, 0.f};
      for (int g0 = 0; g0 < MT; g0 += 4) {
        __syncthreads();
        if (wave >= g0 && wave < g0 + 4 && wave < MT) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 v = {z[4 * q], z[4 * q + 1], z[4 * q + 2], z[4 * q + 3]};
            xch[((wave - g0) * 4 + q) * 64 + lane] = v;
          }
        }
        __syncthreads();
        if (wave == 0) {
          for (int mt = g0; mt < g0 + 4 && mt < MT; ++mt) {
            const f32x16 w3 = load_vec16(w.w3p, mt, h);
            f32x16 a;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x4 v = xch[((mt - g0) * 4 + q) * 64 + lane];
              a[4 * q] = v[0];
              a[4 * q + 1] = v[1];
              a[4 * q + 2] = v[2];
              a[4 * q + 3] = v[3];
            }
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
              const f32x2 a2 = {a[i], a[i + 1]};
              const f32x2 w2 = {w3[i], w3[i + 1]};
              ys2 = __builtin_elementwise_fma(a2, w2, ys2);
            }
          }
        }
      }
      if (wave == 0) {
        float ys = ys2[0] + ys2[1];
        ys += __shfl_xor(ys, 32);
        if (h == 0 && row < n)
          __hip_atomic_store(out + row, __float_as_uint(ys + b3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      continue;
    }
    for (int tile = wave; tile < ntiles; tile += 8) {
      const int row = tile * 32 + r;
      int4 rc = make_int4(0, 0, 0, 0);
      if (row < n) {
        const unsigned long long* p = reinterpret_cast<const unsigned long long*>(rec + row);
        const unsigned long long lo = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long hi = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        rc = make_int4((int)lo, (int)(lo >> 32), (int)hi, (int)(hi >> 32));
      }
      const bf16x8 xb = featurize_bf16(rc, h, np);
      bf16x8 h1[KS];
      mlp3_layer1<H>(w1, xb, h1);
      f32x2 ys2 = {0.f, 0.f};
      mlp3_layer2<H, true>(w, h1, lane, h, [&](int mt, const f32x16& acc) {
        const f32x16 w3 = load_vec16(w.w3p, mt, h);
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 a2 = {relu_f(acc[i]), relu_f(acc[i + 1])};
          const f32x2 w2 = {w3[i], w3[i + 1]};
          ys2 = __builtin_elementwise_fma(a2, w2, ys2);
        }
      });
      float ys = ys2[0] + ys2[1];
      ys += __shfl_xor(ys, 32);
      if (h == 0 && row < n)
        __hip_atomic_store(out + row, __float_as_uint(ys + b3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Host side

struct PersistentScorer {
  int device = 0, H = 256, cap = 0;
  const void* blob = nullptr;
  NormParams np{};
  unsigned long long idle_ticks = 0, life_ticks = 0;
  hipStream_t stream{};
  ServeMailbox* mb = nullptr;   // pinned, coherent, mapped
  int4* rec = nullptr;
  unsigned* out = nullptr;
  ServeMailbox* d_mb = nullptr;
  int4* d_rec = nullptr;
  unsigned* d_out = nullptr;
  unsigned seq = 0;             // last doorbell value rung
  bool launched = false;
  bool broken = false;          // repeated timeouts: callers use the normal launch path
  int timeouts_in_row = 0;
  long long launches = 0, served = 0, fallbacks = 0;
};

template <int H>
static hipError_t launch_serve_h(PersistentScorer* s) {
  using L = Mlp3Layout<H>;
  static bool attr_set[64] = {};
  if (!attr_set[s->device & 63]) {
    hipError_t e = hipFuncSetAttribute((const void*)eta_mlp3_serve_kernel<H>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)(L::BLOB + kXchBytes));
    if (e != hipSuccess) return e;
    attr_set[s->device & 63] = true;
  }
  hipLaunchKernelGGL(eta_mlp3_serve_kernel<H>, dim3(1), dim3(512), L::BLOB + kXchBytes, s->stream, s->d_mb,
                     (const int4*)s->d_rec, s->d_out, s->cap, (const unsigned char*)s->blob, s->np,
                     s->seq, s->idle_ticks, s->life_ticks);
  return hipGetLastError();
}

static hipError_t pscore_launch(PersistentScorer* s) {
  hipError_t e = hipErrorInvalidValue;
  switch (s->H) {
    case 64: e = launch_serve_h<64>(s); break;
    case 128: e = launch_serve_h<128>(s); break;
    case 256: e = launch_serve_h<256>(s); break;
  }
  if (e == hipSuccess) {
    s->launched = true;
    ++s->launches;
  }
  return e;
}

PersistentScorer* pscore_create(int device, const void* blob, int H, const NormParams& np, int cap,
                                double idle_ms, double life_ms, hipError_t* err) {
  *err = hipSuccess;
  if ((H != 64 && H != 128 && H != 256) || cap <= 0) {
    *err = hipErrorInvalidValue;
    return nullptr;
  }
  auto* s = new PersistentScorer();
  s->device = device;
  s->H = H;
  s->cap = cap;
  s->blob = blob;
  s->np = np;
  int khz = 100000;                                       // wall_clock64() rate (100 MHz on gfx9)
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
    khz = 100000;
  s->idle_ticks = (unsigned long long)(idle_ms * (double)khz);
  s->life_ticks = (unsigned long long)(life_ms * (double)khz);
  const unsigned flags = hipHostMallocMapped | hipHostMallocCoherent;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipHostMalloc((void**)&s->mb, sizeof(ServeMailbox), flags);
  if (e == hipSuccess) e = hipHostMalloc((void**)&s->rec, (size_t)cap * sizeof(int4), flags);
  if (e == hipSuccess) e = hipHostMalloc((void**)&s->out, (size_t)cap * sizeof(unsigned), flags);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->d_mb, s->mb, 0);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->d_rec, s->rec, 0);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->d_out, s->out, 0);
  if (e != hipSuccess) {
    *err = e;
    pscore_destroy(s);
    return nullptr;
  }
  std::memset(s->mb, 0, sizeof(ServeMailbox));
  return s;
}

void* pscore_records(PersistentScorer* s) { return s->rec; }
const float* pscore_out(PersistentScorer* s) { return reinterpret_cast<const float*>(s->out); }
int pscore_cap(PersistentScorer* s) { return s->cap; }
bool pscore_broken(PersistentScorer* s) { return s->broken; }
void pscore_stats(PersistentScorer* s, long long* launches, long long* served, long long* fallbacks) {
  *launches = s->launches;
  *served = s->served;
  *fallbacks = s->fallbacks;
}

void pscore_park(PersistentScorer* s);

// Score records[0, n) (already written into pscore_records()).  Returns hipSuccess when every
// output slot is filled; hipErrorLaunchTimeOut if the scorer did not answer within timeout_ms (it is
// then parked — the caller re-scores with a normal launch).
hipError_t pscore_run(PersistentScorer* s, int n, double timeout_ms) {
  if (s->broken) return hipErrorNotReady;
  if (n <= 0) return hipSuccess;
  if (n > s->cap) return hipErrorInvalidValue;
  (void)hipSetDevice(s->device);
  volatile unsigned* out = s->out;
  for (int i = 0; i < n; ++i) out[i] = kOutSentinel;
  // (re)launch if the resident kernel exited (idle timeout) or was never started
  if (!s->launched || hipStreamQuery(s->stream) == hipSuccess) {
    hipError_t e = pscore_launch(s);
    if (e != hipSuccess) return e;
  }
  std::atomic_thread_fence(std::memory_order_release);
  __atomic_store_n(&s->mb->n, (unsigned)n, __ATOMIC_RELAXED);
  __atomic_store_n(&s->mb->seq, ++s->seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  int i = 0;
  unsigned spins = 0;
  while (true) {
    while (i < n && out[i] != kOutSentinel) ++i;
    if (i >= n) break;
    __builtin_ia32_pause();
    if ((++spins & 1023u) == 0) {
      const double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_ms) {
        // stop the kernel and wait until it is gone, so a late answer can never land in the
        // output slots of a later request; three timeouts in a row retire the scorer
        ++s->fallbacks;
        pscore_park(s);
        if (++s->timeouts_in_row >= 3) s->broken = true;
        return hipErrorLaunchTimeOut;
      }
      // the kernel idled out between our stream check and the doorbell: start it again (it
      // begins from the last answered doorbell, so it serves this request)
      if (hipStreamQuery(s->stream) == hipSuccess) {
        s->seq -= 1;
        hipError_t e = pscore_launch(s);
        s->seq += 1;
        if (e != hipSuccess) return e;
      }
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  ++s->served;
  s->timeouts_in_row = 0;
  return hipSuccess;
}

// Make the resident kernel exit and wait for it (it leaves at its next poll), e.g. before a large
// launch that may share its hardware queue.  The next pscore_run relaunches it.
void pscore_park(PersistentScorer* s) {
  if (s == nullptr || !s->launched) return;
  (void)hipSetDevice(s->device);
  __atomic_store_n(&s->mb->stop, 1u, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(s->stream);
  __atomic_store_n(&s->mb->stop, 0u, __ATOMIC_RELEASE);
  s->launched = false;
}

void pscore_destroy(PersistentScorer* s) {
  if (s == nullptr) return;
  if (s->mb != nullptr) {
    __atomic_store_n(&s->mb->stop, 1u, __ATOMIC_RELEASE);
    if (s->stream) (void)hipStreamSynchronize(s->stream);   // the kernel exits within one poll
  }
  if (s->stream) (void)hipStreamDestroy(s->stream);
  if (s->mb) (void)hipHostFree(s->mb);
  if (s->rec) (void)hipHostFree(s->rec);
  if (s->out) (void)hipHostFree(s->out);
  delete s;
}

}  // namespace rt
