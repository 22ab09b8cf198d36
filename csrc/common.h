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

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

// ReLU as an integer max on the fp32 bit pattern: negative floats (sign bit set) are negative
// int32s, so max(bits, 0) is relu in ONE v_max_i32.  fmaxf(x, 0.f) costs two v_max_f32 on gfx950
// (IEEE mode inserts a NaN-quieting self-max before every use), which made the MLP epilogues
// VALU-bound.
__device__ __forceinline__ float relu_f(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}

// 8 fp32 -> relu -> bf16x8: convert pairs (v_cvt_pk_bf16_f32), then ReLU on the packed bf16 bit
// patterns with v_pk_max_i16 (round-to-nearest preserves the sign, and -0 -> +0), i.e. 1
// instruction per value instead of 2.5.  Bit-identical to (__bf16)fmaxf(x, 0).
__device__ __forceinline__ void relu_cvt_bf16x8(const float* v, void* dst) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  i16x2* d = reinterpret_cast<i16x2*>(dst);
  const i16x2 z = {0, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 p = {v[2 * q], v[2 * q + 1]};
    const bf16x2 t = __builtin_convertvector(p, bf16x2);
    d[q] = __builtin_elementwise_max(__builtin_bit_cast(i16x2, t), z);
  }
}

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
    const float km = __int_as_float(rc.x) * 1e-3f;   // not '/': an IEEE divide is ~10 VALU ops
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

// 8-byte wire record (features.py::RECORD8_DTYPE): x = distance_m bits, y = fp16 age | hours << 16 |
// weather << 26 | traffic << 29, where `hours` counts wall-clock hours from 00:00 of the batch's
// base Monday.  The featurisation of the time happens here: weekday = (hours / 24) % 7 and hour =
// hours % 24, as multiply-shifts that are exact over the 10-bit range (hours < 1024, days < 43;
// checked exhaustively in tests/test_runtime_cpu.py).
__device__ __forceinline__ void wire8_time(const unsigned pk, float& wd, float& hr) {
  const unsigned hrs = (pk >> 16) & 1023u;
  const unsigned day = (hrs * 2731u) >> 16;                 // hrs / 24
  const unsigned wdi = day - ((day * 9363u) >> 16) * 7u;    // day % 7
  wd = (float)wdi;
  hr = (float)(hrs - day * 24u);
}

__device__ __forceinline__ void featurize8_f32(const int2 rc, const int h, const NormParams& np,
                                               float f[8]) {
  const unsigned pk = (unsigned)rc.y;
  if (h == 0) {
    const int w = (pk >> 26) & 7;
    const int t = (pk >> 29) & 7;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = (w == j) ? 1.f : 0.f;
      f[4 + j] = (t == j) ? 1.f : 0.f;
    }
  } else {
    float wd, hr;
    wire8_time(pk, wd, hr);
    const float wdn = wd * np.scale[0] + np.shift[0];
    const float hrn = hr * np.scale[1] + np.shift[1];
    const float kmn = (__int_as_float(rc.x) * 1e-3f) * np.scale[2] + np.shift[2];
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

// One-hot pair (weather, traffic) straight as bf16 B-fragment bits for lane half h = 0:
// bf16(1.0) = 0x3F80 in slot c of each 4-wide group; an unknown category (c >= 4) gives all
// zeros, like the reference's dummies of an unseen value (RO/Flaskr/ml.py:35-48).
__device__ __forceinline__ bf16x8 onehot_pair_bf16(unsigned w, unsigned t) {
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  u64x2 v;
  v[0] = w < 4u ? (0x3F80ull << (16u * w)) : 0ull;
  v[1] = t < 4u ? (0x3F80ull << (16u * t)) : 0ull;
  return __builtin_bit_cast(bf16x8, v);
}

// Branch-free B fragment of lane half h, bit-identical to to_bf16x8(featurize*_f32(..., h, ...)):
// both halves compute both feature groups and select (a divergent branch runs the two halves'
// paths one after the other anyway), and the one-hot group costs a few VALU ops instead of ~20.
__device__ __forceinline__ bf16x8 featurize_bf16(const int4 rc, const int h, const NormParams& np) {
  float f[8];
  featurize_f32(rc, 1, np, f);
  const bf16x8 nb = to_bf16x8(f);
  const bf16x8 oh = onehot_pair_bf16((unsigned)rc.w & 0xffu, ((unsigned)rc.w >> 8) & 0xffu);
  return h == 0 ? oh : nb;
}
__device__ __forceinline__ bf16x8 featurize8_bf16(const int2 rc, const int h, const NormParams& np) {
  float f[8];
  featurize8_f32(rc, 1, np, f);
  const bf16x8 nb = to_bf16x8(f);
  const unsigned pk = (unsigned)rc.y;
  const bf16x8 oh = onehot_pair_bf16((pk >> 26) & 7u, (pk >> 29) & 7u);
  return h == 0 ? oh : nb;
}

// 6-byte records (features.py RECORD6): one 48-bit word, lo = bits 0-31, hi = bits 32-47.
// Same fragment as featurize8_bf16 (distance -> km exactly as q * 0.125 m * 1e-3).
__device__ __forceinline__ bf16x8 featurize6_bf16(const unsigned lo, const unsigned hi, const int h,
                                                  const NormParams& np) {
  const float wdn = (float)((hi >> 2) & 7u) * np.scale[0] + np.shift[0];
  const float hrn = (float)((hi >> 5) & 31u) * np.scale[1] + np.shift[1];
  const float kmn = ((float)(lo & 0x7ffffffu) * (0.125f * 1e-3f)) * np.scale[2] + np.shift[2];
  const float agn = (float)((lo >> 27) | ((hi & 3u) << 5)) * np.scale[3] + np.shift[3];
  const float kmh = (float)(__bf16)kmn;
  const float agh = (float)(__bf16)agn;
  const float f[8] = {wdn, hrn, kmh, agh, kmn - kmh, agn - agh, 1.f, 1.f};
  const bf16x8 nb = to_bf16x8(f);
  const bf16x8 oh = onehot_pair_bf16((hi >> 10) & 7u, (hi >> 13) & 7u);
  return h == 0 ? oh : nb;
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
