// ETA models the native front end serves (csrc/native_server.hip) and the route service's use_ml_eta
// path: every family the Python EtaService serves (routest_amd/serve/eta_service.py), so a wide or
// tree model no longer sends the main port back to uvicorn.
//
//   mlp3    H = 64/128/256: the fused featurize + MLP kernel (K1+K2, csrc/eta_mlp_fwd.hip)
//   wide    H = 512/1024:  the fused wide kernel + partial-sum reduce (csrc/mlp_big.hip)
//   forest  tree ensembles (XGBoost JSON / sklearn HGB -> K4, csrc/forest.hip)
//
// A model object owns device copies of its weights (so a hot swap can free the old ones once the
// last round using them has finished: shared_ptr) and a host fp32 copy for the CPU fallback
// (cpu_predict: the numpy-equivalent fp32 forward, used when every GPU is quarantined).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "runtime/rt_core.h"

namespace rt {

// per-caller device workspace (grows on demand)
struct ModelWs {
  void* p = nullptr;
  size_t bytes = 0;
  int device = -1;
  ~ModelWs();
  hipError_t need(int dev, size_t b);
};

struct NativeModel {
  enum Kind { MLP3 = 0, WIDE = 1, FOREST = 2 };
  int kind = MLP3;
  int device = 0;
  int H = 0;
  uint64_t epoch = 0;
  virtual ~NativeModel() = default;
  // minutes for B records at device-visible `rec` (16-byte EtaRecord, or 8-byte wire records when
  // takes_wire8()) into device-visible `out`, on stream s (asynchronous)
  virtual hipError_t predict(const void* rec, int rec_bytes, float* out, int B, hipStream_t s, ModelWs& ws) const = 0;
  virtual bool takes_wire8() const { return true; }
  // the 32x32 fused kernel's blob (resident scorer) or nullptr
  virtual const void* mlp3_blob() const { return nullptr; }
  virtual const NormParams* mlp3_norm() const { return nullptr; }
  // CPU fallback on 16-byte records (false: this model has none)
  virtual bool cpu_predict(const rtc::EtaRecord* rec, float* out, int B) const = 0;
  virtual std::string describe() const = 0;
};

// Host fp32 weights of an MLP (EtaMLP state: l1/l2/l3 + x/y normalisation), for the CPU forward.
struct MlpHost {
  int H = 0;
  std::vector<float> w1, b1, w2, b2, w3, x_mean, x_std;   // w1 [H,12], w2 [H,H], w3 [H]
  float b3 = 0.f, y_mean = 0.f, y_std = 1.f;
};

struct ForestHost {
  std::vector<float> values;
  std::vector<uint32_t> info;
  std::vector<int32_t> roots;
  float base = 0.f;
  bool le = false;
  int fmap[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
};

// Constructors copy device tensors (given as device pointers on `device`) into owned allocations.
std::shared_ptr<NativeModel> make_mlp3_model(int device, const void* blob, size_t blob_bytes, int H,
                                             const NormParams& np, int variant, int num_cus, MlpHost host,
                                             std::string& err);
std::shared_ptr<NativeModel> make_wide_model(int device, int H, const void* w1q, size_t w1q_bytes, const void* w2f,
                                             size_t w2f_bytes, const float* b2, const float* w3, float b3,
                                             const NormParams& np, MlpHost host, std::string& err);
std::shared_ptr<NativeModel> make_forest_model(int device, ForestHost host, std::string& err);

// fp32 MLP forward on one record (numpy-equivalent order of operations)
float mlp_cpu_forward(const MlpHost& m, const rtc::EtaRecord& r);

}  // namespace rt
