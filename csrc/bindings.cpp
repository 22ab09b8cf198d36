// PyTorch bindings for the routest_amd gfx950 kernels (module routest_amd._C).
//
// Every op takes device tensors, launches on the caller's current HIP stream (so torch streams,
// CUDA-graph capture and multi-GPU device guards all compose), allocates outputs through the torch
// caching allocator and never synchronises.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include <vector>

#include "ops.h"
#include "common.h"

namespace {

#define RT_CHECK_HIP(expr)                                                             \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    TORCH_CHECK(_e == hipSuccess, "HIP error in ", #expr, ": ", hipGetErrorString(_e)); \
  } while (0)

int num_cus(int dev) {
  static int cache[64] = {0};
  if (cache[dev & 63] == 0) {
    int v = 0;
    RT_CHECK_HIP(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev));
    cache[dev & 63] = v;
  }
  return cache[dev & 63];
}

hipStream_t cur_stream(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check_dev(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

torch::Tensor eta_mlp3_forward(torch::Tensor records, torch::Tensor blob, int64_t H,
                               std::vector<double> norm, double b3, int64_t variant) {
  check_dev(records, "records");
  check_dev(blob, "blob");
  TORCH_CHECK(records.scalar_type() == torch::kInt32 && records.dim() == 2 && records.size(1) == 4,
              "records must be int32 [B,4] (16-byte EtaRecord rows)");
  TORCH_CHECK(blob.scalar_type() == torch::kUInt8, "blob must be uint8");
  TORCH_CHECK((size_t)blob.numel() == rt::eta_mlp3_blob_bytes((int)H),
              "blob has ", blob.numel(), " bytes, expected ", rt::eta_mlp3_blob_bytes((int)H),
              " for H=", H);
  TORCH_CHECK(norm.size() == 8, "norm must hold 4 scales + 4 shifts");
  TORCH_CHECK(records.device() == blob.device(), "records/blob on different devices");
  TORCH_CHECK(records.size(0) < (1LL << 31) - 64, "batch too large");
  const c10::DeviceGuard guard(records.device());
  const int B = (int)records.size(0);
  auto out = torch::empty({B}, records.options().dtype(torch::kFloat32));
  rt::NormParams np;
  for (int i = 0; i < 4; ++i) {
    np.scale[i] = (float)norm[i];
    np.shift[i] = (float)norm[4 + i];
  }
  RT_CHECK_HIP(rt::launch_eta_mlp3_fwd(records.data_ptr(), out.data_ptr<float>(), B,
                                       blob.data_ptr(), (int)H, np, (float)b3, (int)variant,
                                       num_cus(records.device().index()), cur_stream(records)));
  return out;
}

torch::Tensor eta_featurize(torch::Tensor records) {
  check_dev(records, "records");
  TORCH_CHECK(records.scalar_type() == torch::kInt32 && records.dim() == 2 && records.size(1) == 4,
              "records must be int32 [B,4]");
  const c10::DeviceGuard guard(records.device());
  const int B = (int)records.size(0);
  auto out = torch::empty({B, 12}, records.options().dtype(torch::kFloat32));
  RT_CHECK_HIP(rt::launch_eta_featurize(records.data_ptr(), out.data_ptr<float>(), B,
                                        cur_stream(records)));
  return out;
}

torch::Tensor route_haversine_matrix(torch::Tensor lat, torch::Tensor lon, torch::Tensor npts,
                                     double circuity) {
  check_dev(lat, "lat");
  check_dev(lon, "lon");
  check_dev(npts, "npts");
  TORCH_CHECK(lat.scalar_type() == torch::kFloat64 && lat.dim() == 2, "lat must be f64 [R,NM]");
  TORCH_CHECK(lon.sizes() == lat.sizes() && lon.scalar_type() == torch::kFloat64, "lon mismatch");
  TORCH_CHECK(npts.scalar_type() == torch::kInt32 && npts.numel() == lat.size(0), "npts mismatch");
  const c10::DeviceGuard guard(lat.device());
  const int R = (int)lat.size(0), NM = (int)lat.size(1);
  auto D = torch::empty({R, NM, NM}, lat.options());
  RT_CHECK_HIP(rt::launch_haversine_matrix(lat.data_ptr<double>(), lon.data_ptr<double>(),
                                           npts.data_ptr<int>(), R, NM, circuity,
                                           D.data_ptr<double>(), cur_stream(lat)));
  return D;
}

std::vector<torch::Tensor> route_greedy_cvrp(torch::Tensor D, torch::Tensor npts,
                                             torch::Tensor demand, torch::Tensor cap,
                                             torch::Tensor maxd) {
  for (auto* t : {&D, &npts, &demand, &cap, &maxd}) check_dev(*t, "route tensor");
  TORCH_CHECK(D.scalar_type() == torch::kFloat64 && D.dim() == 3 && D.size(1) == D.size(2),
              "D must be f64 [R,NM,NM]");
  const int R = (int)D.size(0), NM = (int)D.size(1);
  TORCH_CHECK(NM <= 4096, "at most 4095 stops per request");
  TORCH_CHECK(npts.scalar_type() == torch::kInt32 && npts.numel() == R, "npts must be i32 [R]");
  TORCH_CHECK(demand.scalar_type() == torch::kFloat64 && demand.numel() == (int64_t)R * NM,
              "demand must be f64 [R,NM]");
  TORCH_CHECK(cap.scalar_type() == torch::kFloat64 && cap.numel() == R, "cap must be f64 [R]");
  TORCH_CHECK(maxd.scalar_type() == torch::kFloat64 && maxd.numel() == R, "maxd must be f64 [R]");
  const c10::DeviceGuard guard(D.device());
  auto iopt = D.options().dtype(torch::kInt32);
  auto visit = torch::empty({R, NM}, iopt);
  auto trip_of = torch::empty({R, NM}, iopt);
  auto ntrips = torch::empty({R}, iopt);
  auto status = torch::empty({R}, iopt);
  RT_CHECK_HIP(rt::launch_greedy_cvrp(D.data_ptr<double>(), npts.data_ptr<int>(),
                                      demand.data_ptr<double>(), cap.data_ptr<double>(),
                                      maxd.data_ptr<double>(), R, NM, visit.data_ptr<int>(),
                                      trip_of.data_ptr<int>(), ntrips.data_ptr<int>(),
                                      status.data_ptr<int>(), cur_stream(D)));
  return {visit, trip_of, ntrips, status};
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "routest_amd native gfx950 kernels";
  m.def("eta_mlp3_forward", &eta_mlp3_forward, "fused featurize + 3-layer MLP forward (bf16 MFMA)");
  m.def("eta_featurize", &eta_featurize, "K1: packed records -> R16 features [B,12] fp32");
  m.def("eta_mlp3_blob_bytes", [](int64_t H) { return (int64_t)rt::eta_mlp3_blob_bytes((int)H); });
  m.def("route_haversine_matrix", &route_haversine_matrix, "K5: batched haversine matrices (f64)");
  m.def("route_greedy_cvrp", &route_greedy_cvrp, "K6: batched greedy multi-trip CVRP");
  m.attr("ARCH") = "gfx950";
}
