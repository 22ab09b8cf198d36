// Host-side launcher declarations for every routest_amd HIP kernel (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace rt {

struct NormParams;

// ---- ETA MLP (K1 featurize + K2 forward) : eta_mlp_fwd.hip ----
size_t eta_mlp3_blob_bytes(int H);
// variant: -1 auto, 0 weights from global/L2, 1 weights staged in LDS (persistent grid)
hipError_t launch_eta_mlp3_fwd(const void* rec, float* out, int B, const void* blob, int H,
                               const NormParams& np, float b3, int variant, int num_cus,
                               hipStream_t stream);
hipError_t launch_eta_featurize(const void* rec, float* out, int B, hipStream_t stream);

// ---- batched routing (K5 distance matrix + K6 greedy CVRP) : route_kernels.hip ----
hipError_t launch_haversine_matrix(const double* lat, const double* lon, const int* npts, int R,
                                   int NM, double circuity, double* D, hipStream_t stream);
hipError_t launch_greedy_cvrp(const double* D, const int* npts, const double* demand,
                              const double* cap, const double* maxd, int R, int NM, int* visit,
                              int* trip_of, int* ntrips, int* status, hipStream_t stream);

}  // namespace rt
