// Shared device helpers for the routest_amd gfx950 (CDNA4) kernels.
//
// Layout convention used by every MLP kernel ("batch on the lane"):
//   an MFMA 32x32x16 accumulator tile X[32 hidden][32 batch] lives with the batch row on the lane
//   (col = lane & 31) and the hidden unit in the 16 registers
//   (row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)).
// A following MFMA that sums over the hidden index can therefore take X directly as its B operand
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"); the permuted k
// order this implies is absorbed by pre-permuting the weight fragments on the host
// (routest_amd/ops/eta_mlp.py::pack_mlp3).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace rt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Normalisation of the four numeric features (weekday, hour, distance_km, driver_age):
// f = x * scale + shift.  One-hots are used raw.
struct NormParams {
  float scale[4];
  float shift[4];
};

__device__ __forceinline__ f32x16 mfma32(const bf16x8 a, const bf16x8 b, const f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Packed request record (routest_amd/models/features.py::RECORD_DTYPE):
//   x = distance_m (f32 bits), y = driver_age (f32 bits), z = wall-clock seconds since
//   2020-01-01 (Wednesday), w = weather | traffic << 8.
// Returns the 8 features of lane-half h for the MFMA B operand (k = 8h + j):
//   h = 0: weather one-hot [0..3], traffic one-hot [4..7]
//   h = 1: weekday, hour, km_hi, age_hi, km_lo, age_lo, 1, 1
// km/age are split into a bf16 hi part and a bf16 residual so layer 1 sees ~16 mantissa bits of
// the continuous inputs; the host duplicates W1's km/age columns into k = 12, 13.  The two
// constant-1 inputs at k = 14, 15 carry b1 as a bf16 hi/lo pair, so layer 1 is a bare MFMA.
__device__ __forceinline__ void featurize_f32(const int4 rc, const int h, const NormParams& np,
                                              float f[8]) {
  if (h == 0) {
    const int w = rc.w & 0xff;
    const int t = (rc.w >> 8) & 0xff;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = (w == j) ? 1.f : 0.f;
      f[4 + j] = (t == j) ? 1.f : 0.f;
    }
  } else {
    const int secs = rc.z;
    // floor division for negative seconds (pre-2020 pickups)
    int days = secs / 86400;
    if (secs < 0 && days * 86400 != secs) days -= 1;
    const int sod = secs - days * 86400;
    int wd = (days + 2) % 7;
    if (wd < 0) wd += 7;
    const float hour = (float)(sod / 3600);
    const float km = __int_as_float(rc.x) / 1000.f;
    const float age = __int_as_float(rc.y);
    const float wdn = (float)wd * np.scale[0] + np.shift[0];
    const float hrn = hour * np.scale[1] + np.shift[1];
    const float kmn = km * np.scale[2] + np.shift[2];
    const float agn = age * np.scale[3] + np.shift[3];
    const float kmh = (float)(__bf16)kmn;
    const float agh = (float)(__bf16)agn;
    f[0] = wdn;
    f[1] = hrn;
    f[2] = kmh;
    f[3] = agh;
    f[4] = kmn - kmh;
    f[5] = agn - agh;
    f[6] = 1.f;
    f[7] = 1.f;
  }
}

// Compact 8-byte record (features.py::RECORD8_DTYPE): x = distance_m bits, y = fp16 age |
// weekday << 16 | hour << 19 | weather << 24 | traffic << 27.  Same lane-half feature split.
__device__ __forceinline__ void featurize8_f32(const int2 rc, const int h, const NormParams& np,
                                               float f[8]) {
  const unsigned pk = (unsigned)rc.y;
  if (h == 0) {
    const int w = (pk >> 24) & 7;
    const int t = (pk >> 27) & 7;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = (w == j) ? 1.f : 0.f;
      f[4 + j] = (t == j) ? 1.f : 0.f;
    }
  } else {
    const float wdn = (float)((pk >> 16) & 7) * np.scale[0] + np.shift[0];
    const float hrn = (float)((pk >> 19) & 31) * np.scale[1] + np.shift[1];
    const float kmn = (__int_as_float(rc.x) / 1000.f) * np.scale[2] + np.shift[2];
    const float agn = __half2float(__ushort_as_half((unsigned short)(pk & 0xffffu))) * np.scale[3] +
                      np.shift[3];
    const float kmh = (float)(__bf16)kmn;
    const float agh = (float)(__bf16)agn;
    f[0] = wdn;
    f[1] = hrn;
    f[2] = kmh;
    f[3] = agh;
    f[4] = kmn - kmh;
    f[5] = agn - agh;
    f[6] = 1.f;
    f[7] = 1.f;
  }
}

__device__ __forceinline__ bf16x8 to_bf16x8(const float f[8]) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)f[j];
  return v;
}

// Unnormalised R16 features (12 columns, reference order) of one record — the K1 standalone op.
__device__ __forceinline__ void featurize_raw12(const int4 rc, float f[12]) {
  const int w = rc.w & 0xff;
  const int t = (rc.w >> 8) & 0xff;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = (w == j) ? 1.f : 0.f;
    f[4 + j] = (t == j) ? 1.f : 0.f;
  }
  const int secs = rc.z;
  int days = secs / 86400;
  if (secs < 0 && days * 86400 != secs) days -= 1;
  const int sod = secs - days * 86400;
  int wd = (days + 2) % 7;
  if (wd < 0) wd += 7;
  f[8] = (float)wd;
  f[9] = (float)(sod / 3600);
  f[10] = __int_as_float(rc.x) / 1000.f;
  f[11] = __int_as_float(rc.y);
}

}  // namespace rt
