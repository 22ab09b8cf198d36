// Alternative routes per leg, shared by the Python app (routing/alternatives.py, through _rt) and the
// native route service (csrc/route_service.hip), so both pick byte-identical candidates:
//
//  * via_nodes: for a leg s -> t, nodes w inside the s-t bounding box widened by the stretch whose
//    great-circle detour d(s,w) + d(w,t) lies in [1.03, stretch] x d(s,t) (Abraham et al.'s via-node
//    alternatives), taken in the order of a splitmix64 hash of (s, t, w) — reproducible per leg with
//    no RNG state;
//  * candidate_score: the GCN scorer's value of one candidate path from its node delay factors —
//    kind "observed" (models/gcn_observed.py): edge-cost seconds + predicted hidden seconds
//    sum_i (delay(v_i) - 0.5) |v_i v_{i+1}| / V_REF; kind "edge" (round 3): the delay-weighted
//    length sum_i delay(v_i) |v_i v_{i+1}|.  Lower is better; segment lengths on the float32
//    coordinates the GCN kernels use, summed in path order.
// The reference routes each trip along the single ORS answer (RO/Flaskr/utils.py:147-165).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

#include "route_core.h"

namespace ralt {

constexpr double V_REF = 20.0;     // models/gcn_train.py V_REF
constexpr int MAX_K = 8;

inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

inline std::vector<int> via_nodes(const double* lat, const double* lon, int N, int s, int t, int n,
                                  double stretch = 1.35) {
  std::vector<int> out;
  if (n <= 0 || s < 0 || t < 0 || s >= N || t >= N) return out;
  const double d_st = rtr::haversine_m(lat[s], lon[s], lat[t], lon[t]);
  if (!(d_st >= 1.0)) return out;
  const double lat0 = std::min(lat[s], lat[t]), lat1 = std::max(lat[s], lat[t]);
  const double lon0 = std::min(lon[s], lon[t]), lon1 = std::max(lon[s], lon[t]);
  const double pad = 0.5 * (stretch - 1.0) * ((lat1 - lat0) + (lon1 - lon0)) + 1e-3;
  const double hi = stretch * d_st, lo = 1.03 * d_st;
  const uint64_t key = mix64(((uint64_t)(uint32_t)s << 32) | (uint32_t)t);
  std::vector<std::pair<uint64_t, int>> ok;
  for (int w = 0; w < N; ++w) {
    if (lat[w] < lat0 - pad || lat[w] > lat1 + pad || lon[w] < lon0 - pad || lon[w] > lon1 + pad) continue;
    const double det = rtr::haversine_m(lat[s], lon[s], lat[w], lon[w]) + rtr::haversine_m(lat[w], lon[w], lat[t], lon[t]);
    if (det <= hi && det >= lo) ok.emplace_back(mix64(key ^ (uint64_t)(uint32_t)w), w);
  }
  const size_t k = std::min(ok.size(), (size_t)n);
  std::partial_sort(ok.begin(), ok.begin() + k, ok.end());
  out.reserve(k);
  for (size_t i = 0; i < k; ++i) out.push_back(ok[i].second);
  return out;
}

enum ScoreKind { OBSERVED = 0, EDGE = 1 };

// one candidate's score (see header); seconds = its edge-cost seconds (unused for EDGE)
inline double candidate_score(const double* lat, const double* lon, const double* delay, const int32_t* p, size_t n,
                              double seconds, int kind) {
  double acc = 0.0;
  for (size_t i = 0; i + 1 < n; ++i) {
    const double d = rtr::haversine_m((double)(float)lat[p[i]], (double)(float)lon[p[i]], (double)(float)lat[p[i + 1]],
                                      (double)(float)lon[p[i + 1]]);
    acc += kind == OBSERVED ? (delay[p[i]] - 0.5) * d / V_REF : delay[p[i]] * d;
  }
  return kind == OBSERVED ? seconds + acc : acc;
}

// index of the least score (non-finite = +inf; first on ties), -1 when empty
inline int argmin_score(const std::vector<double>& v) {
  int best = -1;
  double bv = 0.0;
  for (size_t i = 0; i < v.size(); ++i) {
    const double x = std::isfinite(v[i]) ? v[i] : INFINITY;
    if (best < 0 || x < bv) {
      best = (int)i;
      bv = x;
    }
  }
  return best;
}

}  // namespace ralt
