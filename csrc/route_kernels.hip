// K5 + K6: batched multi-stop route construction for many concurrent requests (gfx950).
//
// Replaces, per request, the remote ORS matrix call (RO/Flaskr/utils.py:93-109) and the pure
// Python greedy loop (utils.py:111-139), which the reference runs one request at a time.
//
// K5 haversine_matrix_kernel: D[r][i][j] = 2R asin(sqrt(hav)) * circuity, fp64 (the greedy
//    feasibility tests compare sums of distances against maximum_distance, so we keep the
//    reference's float64 semantics).  One thread per (r, i, j).
//
// K6 greedy_cvrp_kernel: ONE WAVEFRONT PER REQUEST.  Reference semantics (see
//    routest_amd/routing/greedy.py): candidates are scanned once per trip in the (stable) order of
//    their distance from the depot; a candidate is accepted iff load + demand <= cap and
//    trip_dist + d[cur][i] + d[i][0] <= max_dist.  Sequential in the reference; here each
//    acceptance is one parallel step: the 64 lanes test the candidates after the current scan
//    position, a 64-bit ballot finds the FIRST feasible one in scan order (exactly the one the
//    sequential scan would accept next, since everything before it was rejected under the same
//    state), the state advances, repeat.  O(accepted stops) wave-steps instead of O(N) serial
//    iterations.  A trip that accepts nothing means the remaining stops are infeasible on their
//    own: status = 1 (the reference loops forever there — Appendix B #3).
//    Order ranks are computed by counting (stable sort), the scan order and visited flags live in
//    LDS.
#include "common.h"
#include "ops.h"

namespace rt {

__global__ __launch_bounds__(256) void haversine_matrix_kernel(const double* __restrict__ lat,
                                                               const double* __restrict__ lon,
                                                               const int* __restrict__ npts, int R,
                                                               int NM, double circuity,
                                                               double* __restrict__ D) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)R * NM * NM;
  if (tid >= total) return;
  const int r = (int)(tid / ((long long)NM * NM));
  const int rem = (int)(tid - (long long)r * NM * NM);
  const int i = rem / NM;
  const int j = rem - i * NM;
  const int n = npts[r];
  double d = 0.0;
  if (i < n && j < n && i != j) {
    const double k = 3.14159265358979323846 / 180.0;
    const double p1 = lat[r * NM + i] * k, p2 = lat[r * NM + j] * k;
    const double dphi = p2 - p1;
    const double dl = lon[r * NM + j] * k - lon[r * NM + i] * k;
    const double s1 = sin(dphi * 0.5), s2 = sin(dl * 0.5);
    double a = s1 * s1 + cos(p1) * cos(p2) * s2 * s2;
    a = a < 0.0 ? 0.0 : (a > 1.0 ? 1.0 : a);
    d = 2.0 * 6371000.0 * asin(sqrt(a)) * circuity;
  }
  D[tid] = d;
}

// LDS per request (one wave): order[NMAX] (int), visited[NMAX] (uchar).
template <int NMAX>
__global__ __launch_bounds__(256) void greedy_cvrp_kernel(
    const double* __restrict__ D, const int* __restrict__ npts, const double* __restrict__ demand,
    const double* __restrict__ cap, const double* __restrict__ maxd, int R, int NM,
    int* __restrict__ visit, int* __restrict__ trip_of, int* __restrict__ ntrips,
    int* __restrict__ status) {
  __shared__ int s_order[4][NMAX];
  __shared__ unsigned char s_vis[4][NMAX];
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + w;
  if (r >= R) return;  // wave-uniform exit: no block barrier is used below
  const int n = npts[r];            // points incl. depot at index 0
  const int ns = n - 1;             // stops
  const double* d = D + (size_t)r * NM * NM;
  const double* dem = demand + (size_t)r * NM;
  int* vout = visit + (size_t)r * NM;
  int* tout = trip_of + (size_t)r * NM;
  const double C = cap[r], MD = maxd[r];

  // stable rank of stop i (1..ns) by d[0][i]
  for (int i = 1 + lane; i <= ns; i += 64) {
    const double key = d[i];
    int rank = 0;
    for (int j = 1; j <= ns; ++j) {
      const double kj = d[j];
      rank += (kj < key) || (kj == key && j < i);
    }
    s_order[w][rank] = i;
    s_vis[w][i] = 0;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes visible to the wave
  __builtin_amdgcn_wave_barrier();

  int placed = 0, trips = 0, st = 0;
  while (placed < ns) {
    double load = 0.0, tdist = 0.0;
    int cur = 0, pos = 0, accepted = 0;
    while (pos < ns) {
      // find the first feasible candidate at scan position >= pos
      int found = -1;
      for (int base = pos; base < ns && found < 0; base += 64) {
        const int q = base + lane;
        bool ok = false;
        if (q < ns) {
          const int i = s_order[w][q];
          if (!s_vis[w][i]) {
            const double di = d[(size_t)cur * NM + i] + d[(size_t)i * NM];
            ok = (load + dem[i]) <= C && (tdist + di) <= MD;
          }
        }
        const unsigned long long m = __ballot(ok);
        if (m) found = base + __builtin_ctzll(m);
      }
      if (found < 0) break;
      const int i = s_order[w][found];
      load += dem[i];
      tdist += d[(size_t)cur * NM + i];
      cur = i;
      if (lane == 0) {
        s_vis[w][i] = 1;
        vout[placed] = i;
        tout[placed] = trips;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      ++placed;
      ++accepted;
      pos = found + 1;
    }
    if (accepted == 0) {  // remaining stops infeasible on their own: reference would hang
      st = 1;
      break;
    }
    ++trips;
  }
  if (lane == 0) {
    ntrips[r] = trips;
    status[r] = st;
    for (int k = placed; k < NM; ++k) {
      vout[k] = -1;
      tout[k] = -1;
    }
  }
}

hipError_t launch_haversine_matrix(const double* lat, const double* lon, const int* npts, int R,
                                   int NM, double circuity, double* D, hipStream_t stream) {
  const long long total = (long long)R * NM * NM;
  if (total == 0) return hipSuccess;
  const int grid = (int)((total + 255) / 256);
  hipLaunchKernelGGL(haversine_matrix_kernel, dim3(grid), dim3(256), 0, stream, lat, lon, npts, R,
                     NM, circuity, D);
  return hipGetLastError();
}

hipError_t launch_greedy_cvrp(const double* D, const int* npts, const double* demand,
                              const double* cap, const double* maxd, int R, int NM, int* visit,
                              int* trip_of, int* ntrips, int* status, hipStream_t stream) {
  if (R == 0) return hipSuccess;
  const int grid = (R + 3) / 4;
  if (NM <= 64) {
    hipLaunchKernelGGL(greedy_cvrp_kernel<64>, dim3(grid), dim3(256), 0, stream, D, npts, demand,
                       cap, maxd, R, NM, visit, trip_of, ntrips, status);
  } else if (NM <= 1024) {
    hipLaunchKernelGGL(greedy_cvrp_kernel<1024>, dim3(grid), dim3(256), 0, stream, D, npts,
                       demand, cap, maxd, R, NM, visit, trip_of, ntrips, status);
  } else if (NM <= 4096) {
    hipLaunchKernelGGL(greedy_cvrp_kernel<4096>, dim3(grid), dim3(256), 0, stream, D, npts,
                       demand, cap, maxd, R, NM, visit, trip_of, ntrips, status);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace rt
