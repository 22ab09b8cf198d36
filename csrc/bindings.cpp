// PyTorch bindings for the routest_amd gfx950 kernels (module routest_amd._C).
//
// Every op takes device tensors, launches on the caller's current HIP stream (so torch streams,
// CUDA-graph capture and multi-GPU device guards all compose), allocates outputs through the torch
// caching allocator and never synchronises.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "ops.h"
#include "common.h"
#include "native_model.h"
#include "route_service.h"

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

// Record wire format from the tensor: int32 [B,4] = 16-byte, int32 [B,2] = 8-byte compact,
// int16 [B,3] = 6-byte bulk records (routest_amd/models/features.py).
static int record_bytes(const torch::Tensor& r) {
  if (r.dim() == 2 && r.scalar_type() == torch::kInt32 && (r.size(1) == 4 || r.size(1) == 2))
    return (int)r.size(1) * 4;
  if (r.dim() == 2 && r.scalar_type() == torch::kInt16 && r.size(1) == 3) return 6;
  TORCH_CHECK(false, "records must be int32 [B,4] (16-byte), int32 [B,2] (8-byte) or int16 [B,3] "
              "(6-byte) records");
  return 0;
}

// variant >= 16 selects the 16x16-MFMA kernel (blob16 layout): 16 -> 2, 17 -> 4, 18 -> 1 batch
// halves per wave-tile (8 waves per CU), 19 -> 2 halves with 12 waves per CU; anything else the
// 32x32 kernel (blob layout)
static int fwd16_halves(int64_t variant) {
  return variant == 16 ? 2 : variant == 17 ? 4 : variant == 18 ? 1 : variant == 19 ? 3
       : variant == 20 ? 5 : variant == 21 ? 6 : variant == 22 ? 7 : variant == 23 ? 8 : 0;
}
static size_t fwd_blob_bytes(int64_t variant, int64_t H) {
  return fwd16_halves(variant) ? rt::eta_mlp3_blob16_bytes((int)H) : rt::eta_mlp3_blob_bytes((int)H);
}
static hipError_t launch_fwd_any(const void* rec, float* out, int B, const void* blob, int64_t H,
                                 const rt::NormParams& np, int64_t variant, int cus, hipStream_t st,
                                 int rb) {
  if (const int nh = fwd16_halves(variant))
    return rt::launch_eta_mlp3_fwd16(rec, out, B, blob, (int)H, np, nh, cus, st, rb);
  return rt::launch_eta_mlp3_fwd(rec, out, B, blob, (int)H, np, (int)variant, cus, st, rb);
}

torch::Tensor eta_mlp3_forward(torch::Tensor records, torch::Tensor blob, int64_t H,
                               std::vector<double> norm, int64_t variant) {
  check_dev(records, "records");
  check_dev(blob, "blob");
  const int rb = record_bytes(records);
  TORCH_CHECK(blob.scalar_type() == torch::kUInt8, "blob must be uint8");
  TORCH_CHECK((size_t)blob.numel() == fwd_blob_bytes(variant, H),
              "blob has ", blob.numel(), " bytes, expected ", fwd_blob_bytes(variant, H),
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
  RT_CHECK_HIP(launch_fwd_any(records.data_ptr(), out.data_ptr<float>(), B, blob.data_ptr(), H, np,
                              variant, num_cus(records.device().index()), cur_stream(records), rb));
  return out;
}

// Pinned host buffer of `nbytes` on a 2 MiB-aligned anonymous mapping, optionally advised onto
// transparent huge pages, faulted in and registered with HIP (mapped, portable).  torch sees it as a
// pinned uint8 CPU tensor.  On 2 MiB pages the copy engine's reads and the kernel's zero-copy writes
// walk 512x fewer page-table entries than on hipHostMalloc's 4 KiB pages.
torch::Tensor pinned_host_empty(int64_t nbytes, bool huge) {
  TORCH_CHECK(nbytes > 0, "nbytes must be positive");
  const size_t align = size_t(2) << 20;
  const size_t len = ((size_t)nbytes + align - 1) / align * align;
  void* base = mmap(nullptr, len + align, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  TORCH_CHECK(base != MAP_FAILED, "mmap of ", len + align, " bytes failed");
  char* p = (char*)(((uintptr_t)base + align - 1) & ~(uintptr_t)(align - 1));
  if (huge) madvise(p, len, MADV_HUGEPAGE);
  std::memset(p, 0, len);
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess) {
    munmap(base, len + align);
    TORCH_CHECK(false, "hipHostRegister failed: ", hipGetErrorString(e));
  }
  auto del = [p, base, len, align](void*) {
    (void)hipHostUnregister(p);
    munmap(base, len + align);
  };
  return torch::from_blob(p, {nbytes}, del, torch::TensorOptions().dtype(torch::kUInt8));
}

// Zero-copy variant: records and/or out may be PINNED HOST tensors, which the kernel reads/writes
// directly over PCIe through their device-mapped addresses (no staging buffers).  Mixed placements
// are allowed: HBM records (brought in by the copy engine) + zero-copy minutes out is the "hybrid"
// serving pipeline of bench.py.
static void* kernel_ptr(const torch::Tensor& t, const char* name) {
  if (t.is_cuda()) {
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    return t.data_ptr();
  }
  TORCH_CHECK(t.is_pinned() && t.is_contiguous(), name, " must be a contiguous pinned host tensor or on the GPU");
  void* d = nullptr;
  RT_CHECK_HIP(hipHostGetDevicePointer(&d, t.data_ptr(), 0));
  return d;
}

void eta_mlp3_forward_hostio(torch::Tensor records, torch::Tensor out, torch::Tensor blob, int64_t H,
                             std::vector<double> norm, int64_t variant) {
  const int rb = record_bytes(records);
  TORCH_CHECK(out.scalar_type() == torch::kFloat32 && out.numel() == records.size(0), "out must be f32 [B]");
  check_dev(blob, "blob");
  TORCH_CHECK((size_t)blob.numel() == fwd_blob_bytes(variant, H), "bad blob");
  TORCH_CHECK(norm.size() == 8, "norm must hold 4 scales + 4 shifts");
  for (const torch::Tensor* t : {&records, &out})
    TORCH_CHECK(!t->is_cuda() || t->device() == blob.device(), "GPU operands must be on the blob's device");
  const c10::DeviceGuard guard(blob.device());
  void* drec = kernel_ptr(records, "records");
  void* dout = kernel_ptr(out, "out");
  rt::NormParams np;
  for (int i = 0; i < 4; ++i) {
    np.scale[i] = (float)norm[i];
    np.shift[i] = (float)norm[4 + i];
  }
  RT_CHECK_HIP(launch_fwd_any(drec, (float*)dout, (int)records.size(0), blob.data_ptr(), H, np,
                              variant, num_cus(blob.device().index()), cur_stream(blob), rb));
}

// ---------------------------------------------------------------- wide MLPs (mlp_big.hip)
void check_bf16(const torch::Tensor& t, const char* name, int64_t rows, int64_t cols);

static rt::NormParams norm_params(const std::vector<double>& norm) {
  TORCH_CHECK(norm.size() == 8, "norm must hold 4 scales + 4 shifts");
  rt::NormParams np;
  for (int i = 0; i < 4; ++i) {
    np.scale[i] = (float)norm[i];
    np.shift[i] = (float)norm[4 + i];
  }
  return np;
}

// records may be pinned host memory (zero-copy) or on the GPU; h1 (and xf) on the GPU.
// wide-MLP inference in one launch: records -> layer 1 -> layer 2 -> relu.w3 partials (mlp_big.hip)
void big_fused(torch::Tensor records, torch::Tensor w1q, torch::Tensor w2f, torch::Tensor b2,
               torch::Tensor w3, int64_t H, std::vector<double> norm, torch::Tensor ypart) {
  const int rb = record_bytes(records);
  for (auto* t : {&w1q, &w2f, &b2, &w3, &ypart}) check_dev(*t, "big_fused operand");
  TORCH_CHECK(H % 256 == 0, "big_fused needs H % 256 == 0");
  TORCH_CHECK(w1q.scalar_type() == torch::kBFloat16 && w1q.numel() == H * 16, "w1q must be bf16 [H*16]");
  TORCH_CHECK(w2f.scalar_type() == torch::kBFloat16 && w2f.numel() == H * H, "w2f must be bf16 [H, H]");
  TORCH_CHECK(b2.scalar_type() == torch::kFloat32 && b2.numel() == H && w3.scalar_type() == torch::kFloat32 &&
                  w3.numel() == H, "b2 / w3 must be f32 [H]");
  TORCH_CHECK(ypart.scalar_type() == torch::kFloat32 && ypart.numel() >= records.size(0) * (H / 64),
              "ypart must be f32 [B, H/64]");
  TORCH_CHECK(!records.is_cuda() || records.device() == w2f.device(), "records on the weights' device");
  TORCH_CHECK(records.size(0) < (1LL << 31) - 256, "batch too large");
  const c10::DeviceGuard guard(w2f.device());
  RT_CHECK_HIP(rt::launch_big_fused(kernel_ptr(records, "records"), rb, (int)records.size(0), w1q.data_ptr(), w2f.data_ptr(),
                                    (int)H, norm_params(norm), b2.data_ptr<float>(), w3.data_ptr<float>(),
                                    ypart.data_ptr<float>(), cur_stream(w2f)));
}

void big_layer1(torch::Tensor records, torch::Tensor w1p, int64_t H, std::vector<double> norm,
                torch::Tensor h1, c10::optional<torch::Tensor> xf, c10::optional<torch::Tensor> mbits) {
  const int rb = record_bytes(records);
  const int64_t B = records.size(0);
  check_dev(w1p, "w1p");
  check_dev(h1, "h1");
  TORCH_CHECK(H % 32 == 0 && H >= 32, "H must be a multiple of 32");
  TORCH_CHECK(w1p.scalar_type() == torch::kBFloat16 && w1p.numel() == H * 16, "w1p bf16 [H*16]");
  TORCH_CHECK(h1.scalar_type() == torch::kBFloat16 && h1.dim() == 2 && h1.size(0) >= B && h1.size(1) >= H &&
              h1.size(1) % 8 == 0, "h1 must be bf16 [>=B, >=H] (ld % 8 == 0)");
  void* xfp = nullptr;
  if (xf.has_value() && xf->defined()) {
    check_bf16(*xf, "xf", B, 16);
    xfp = xf->data_ptr();
  }
  unsigned* mb = nullptr;
  if (mbits.has_value() && mbits->defined()) {
    check_dev(*mbits, "mbits");
    TORCH_CHECK(mbits->scalar_type() == torch::kInt32 && mbits->dim() == 2 && mbits->is_contiguous() &&
                    mbits->size(0) >= (B + 31) / 32 * 32 && mbits->size(1) == H / 32,
                "mbits int32 [>= ceil(B/32)*32, H/32] (tiled [row/32][word][row%32])");
    mb = reinterpret_cast<unsigned*>(mbits->data_ptr<int>());
  }
  TORCH_CHECK(B < (1LL << 31) - 64, "batch too large");
  const c10::DeviceGuard guard(h1.device());
  RT_CHECK_HIP(rt::launch_big_layer1(kernel_ptr(records, "records"), rb, (int)B, w1p.data_ptr(), (int)H,
                                     norm_params(norm), h1.data_ptr(), (int)h1.size(1), xfp, cur_stream(h1), mb));
}

// dh1 = dz2 W2 (W = w2t [N][K], X = dz2 [M][K]) consumed by its epilogue: slab1[t] = the dW1 partial
// (dh1 * relu'(z1))^T xf of batch rows [256 t, 256 t + 256), [N positions][16]
void gemm_dgrad_dw1(torch::Tensor W, torch::Tensor X, int64_t N, int64_t M, int64_t K, torch::Tensor mbits,
                    torch::Tensor xf, torch::Tensor slab1) {
  for (auto* t : {&W, &X, &xf}) {
    check_dev(*t, "operand");
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->dim() == 2 && t->is_contiguous(), "bf16 2-D contiguous");
  }
  TORCH_CHECK(W.size(0) >= N && W.size(1) >= K && X.size(0) >= M && X.size(1) >= K, "operand shapes");
  TORCH_CHECK(N % 256 == 0 && K % 64 == 0, "N % 256 == 0 and K % 64 == 0 required");
  check_dev(mbits, "mbits");
  TORCH_CHECK(mbits.scalar_type() == torch::kInt32 && mbits.dim() == 2 && mbits.is_contiguous() &&
                  mbits.size(0) >= (M + 31) / 32 * 32 && mbits.size(1) == N / 32,
              "mbits int32 [>= ceil(M/32)*32, N/32] (big_layer1's tiled relu bit mask)");
  TORCH_CHECK(xf.size(0) >= M && xf.size(1) == 16, "xf bf16 [>=M, 16]");
  check_dev(slab1, "slab1");
  TORCH_CHECK(slab1.scalar_type() == torch::kFloat32 && slab1.dim() == 2 && slab1.is_contiguous() &&
                  slab1.size(0) >= (M + 255) / 256 && slab1.size(1) >= 16 * N,
              "slab1 f32 [>= ceil(M/256), >= 16 N]");
  TORCH_CHECK(M < (1LL << 31) - 256, "M too large");
  const c10::DeviceGuard guard(W.device());
  RT_CHECK_HIP(rt::launch_gemm_dgrad_dw1(W.data_ptr(), (int)W.size(1), X.data_ptr(), (int)X.size(1), (int)N, (int)M,
                                         (int)K, reinterpret_cast<const unsigned*>(mbits.data_ptr<int>()), xf.data_ptr(),
                                         slab1.data_ptr<float>(), (long long)slab1.size(1), cur_stream(W)));
}

// epi 0: ypart = relu(W X^T + b2) . w3 per 64-unit block; 1: + h2 stored into out; 2: out = W X^T
void gemm_nt(int64_t epi, torch::Tensor W, torch::Tensor X, int64_t N, int64_t M, int64_t K,
             c10::optional<torch::Tensor> b2, c10::optional<torch::Tensor> w3,
             c10::optional<torch::Tensor> ypart, c10::optional<torch::Tensor> out) {
  check_dev(W, "W");
  check_dev(X, "X");
  TORCH_CHECK(W.scalar_type() == torch::kBFloat16 && X.scalar_type() == torch::kBFloat16, "bf16 W/X");
  TORCH_CHECK(W.dim() == 2 && X.dim() == 2 && W.size(0) >= N && W.size(1) >= K && X.size(0) >= M &&
              X.size(1) >= K, "operand shapes");
  TORCH_CHECK(N % 128 == 0 && K % 32 == 0, "N % 128 == 0 and K % 32 == 0 required");
  TORCH_CHECK(epi >= 0 && epi <= 2, "epi in 0..2");
  const float* b2p = nullptr;
  const float* w3p = nullptr;
  float* yp = nullptr;
  void* op = nullptr;
  int ldo = 0;
  if (epi <= 1) {
    TORCH_CHECK(b2.has_value() && w3.has_value() && ypart.has_value(), "b2, w3, ypart required");
    for (auto* t : {&*b2, &*w3}) {
      check_dev(*t, "vec");
      TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->numel() >= N, "b2/w3 f32 [N]");
    }
    check_dev(*ypart, "ypart");
    TORCH_CHECK(ypart->scalar_type() == torch::kFloat32 && ypart->numel() >= M * (N / 64), "ypart f32 [M, N/64]");
    b2p = b2->data_ptr<float>();
    w3p = w3->data_ptr<float>();
    yp = ypart->data_ptr<float>();
  }
  if (epi >= 1) {
    TORCH_CHECK(out.has_value(), "out required");
    check_dev(*out, "out");
    TORCH_CHECK(out->scalar_type() == torch::kBFloat16 && out->dim() == 2 && out->size(0) >= M &&
                out->size(1) >= N && out->size(1) % 8 == 0, "out bf16 [>=M, >=N]");
    op = out->data_ptr();
    ldo = (int)out->size(1);
  }
  TORCH_CHECK(M < (1LL << 31) - 256, "M too large");
  const c10::DeviceGuard guard(W.device());
  RT_CHECK_HIP(rt::launch_gemm_nt((int)epi, W.data_ptr(), (int)W.size(1), X.data_ptr(), (int)X.size(1),
                                  (int)N, (int)M, (int)K, b2p, w3p, yp, op, ldo, cur_stream(W)));
}

// y (f32 [B], GPU or pinned host) = sum of ypart rows + b3; training outputs optional
void big_yreduce(torch::Tensor ypart, int64_t nparts, double b3, c10::optional<torch::Tensor> y,
                 c10::optional<torch::Tensor> target, double gscale, c10::optional<torch::Tensor> dy,
                 c10::optional<torch::Tensor> dyb, c10::optional<torch::Tensor> sq_err,
                 c10::optional<torch::Tensor> b3_dev) {
  check_dev(ypart, "ypart");
  TORCH_CHECK(ypart.scalar_type() == torch::kFloat32 && nparts > 0 && ypart.numel() % nparts == 0, "ypart");
  const int64_t B = ypart.numel() / nparts;
  float* yp = nullptr;
  if (y.has_value() && y->defined()) {
    TORCH_CHECK(y->scalar_type() == torch::kFloat32 && y->numel() >= B, "y f32 [B]");
    yp = (float*)kernel_ptr(*y, "y");
  }
  const float* tp = nullptr;
  float* dyp = nullptr;
  void* dybp = nullptr;
  float* sqp = nullptr;
  if (target.has_value() && target->defined()) {
    TORCH_CHECK(dy.has_value() && dyb.has_value() && sq_err.has_value(), "training outputs required");
    check_dev(*target, "target");
    check_dev(*dy, "dy");
    check_dev(*sq_err, "sq_err");
    TORCH_CHECK(target->numel() >= B && dy->numel() >= B && sq_err->numel() >= B, "training vectors [B]");
    check_bf16(*dyb, "dyb", B, 8);
    tp = target->data_ptr<float>();
    dyp = dy->data_ptr<float>();
    dybp = dyb->data_ptr();
    sqp = sq_err->data_ptr<float>();
  }
  const float* b3p = nullptr;
  if (b3_dev.has_value() && b3_dev->defined()) {
    check_dev(*b3_dev, "b3");
    TORCH_CHECK(b3_dev->scalar_type() == torch::kFloat32 && b3_dev->numel() >= 1, "b3 f32 [1]");
    b3p = b3_dev->data_ptr<float>();
  }
  const c10::DeviceGuard guard(ypart.device());
  RT_CHECK_HIP(rt::launch_big_yreduce(ypart.data_ptr<float>(), (int)nparts, (int)B, (float)b3, b3p, yp, tp,
                                      (float)gscale, dyp, dybp, sqp, cur_stream(ypart)));
}

void adamw_pack_big(torch::Tensor P, torch::Tensor G, torch::Tensor M, torch::Tensor V,
                    torch::Tensor w1p, torch::Tensor w2k, torch::Tensor w2t, torch::Tensor b2,
                    torch::Tensor w3, torch::Tensor b3, torch::Tensor step, int64_t H, double lr,
                    double beta1, double beta2, double eps, double wd, int64_t warmup,
                    int64_t total_steps, double min_lr_ratio, bool update) {
  const int64_t N = H * H + 15 * H + 1;
  for (auto* t : {&P, &M, &V}) {
    check_dev(*t, "adam state");
    TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->numel() == N, "P/M/V f32 [", N, "]");
  }
  check_dev(G, "G");
  TORCH_CHECK(G.scalar_type() == torch::kFloat32 && G.numel() == rt::mlp3_grad_bucket_floats((int)H), "G bucket");
  check_bf16(w1p, "w1p", H, 16);
  check_bf16(w2k, "w2k", H, H);
  check_bf16(w2t, "w2t", H, H);
  for (auto* t : {&b2, &w3, &b3}) {
    check_dev(*t, "vec");
    TORCH_CHECK(t->scalar_type() == torch::kFloat32, "f32 vectors");
  }
  TORCH_CHECK(b2.numel() == H && w3.numel() == H && b3.numel() >= 1, "b2/w3 [H], b3 [1]");
  check_dev(step, "step");
  const c10::DeviceGuard guard(P.device());
  RT_CHECK_HIP(rt::launch_adamw_pack_big(P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(),
                                         V.data_ptr<float>(), w1p.data_ptr(), w2k.data_ptr(), w2t.data_ptr(),
                                         b2.data_ptr<float>(), w3.data_ptr<float>(), b3.data_ptr<float>(),
                                         step.data_ptr<int>(), (int)H, (float)lr, (float)beta1, (float)beta2,
                                         (float)eps, (float)wd, (int)warmup, (int)total_steps,
                                         (float)min_lr_ratio, update ? 1 : 0, cur_stream(P)));
}

// wide trainer: dy / dyb / sq_err from the relu.w3 partials + dz2 from h2a + step counter (one launch)
void big_dz2y(torch::Tensor ypart, int64_t nparts, torch::Tensor b3_dev, torch::Tensor target, double gscale,
              torch::Tensor dy, torch::Tensor dyb, torch::Tensor sq_err, torch::Tensor h2a,
              torch::Tensor w3, int64_t H, torch::Tensor dz2, torch::Tensor step_ctr,
              c10::optional<torch::Tensor> slab) {
  for (auto* t : {&ypart, &b3_dev, &target, &dy, &sq_err, &h2a, &w3, &step_ctr}) check_dev(*t, "big_dz2y operand");
  const int64_t B = dz2.size(0);
  check_bf16(dz2, "dz2", B, H);
  check_bf16(dyb, "dyb", B, 8);
  TORCH_CHECK(ypart.scalar_type() == torch::kFloat32 && nparts > 0 && nparts <= 64 &&
                  ypart.numel() >= B * nparts, "ypart f32 [B, nparts <= 64]");
  TORCH_CHECK(target.numel() >= B && dy.numel() >= B && sq_err.numel() >= B && w3.numel() >= H &&
                  b3_dev.numel() >= 1, "training vectors");
  TORCH_CHECK(h2a.scalar_type() == torch::kBFloat16 && h2a.dim() == 2 && h2a.size(0) >= B &&
                  h2a.size(1) >= H && H % 8 == 0, "h2a bf16 [B, >=H]");
  TORCH_CHECK(step_ctr.scalar_type() == torch::kInt32, "step_ctr i32");
  const c10::DeviceGuard guard(h2a.device());
  if (slab.has_value() && slab->defined()) {
    // dW3 | db3 partials folded in: slab[s][0 .. H+16) for s < S, summed by wgrad_reduce
    check_dev(*slab, "slab");
    TORCH_CHECK(slab->scalar_type() == torch::kFloat32 && slab->dim() == 2 && slab->is_contiguous() &&
                    slab->size(1) >= H + 16 && slab->size(0) >= 1 && slab->size(0) <= B,
                "slab f32 [S <= B, >= H + 16]");
    TORCH_CHECK(H == 512 || H == 1024, "fused dW3 path: H = 512 or 1024");
    RT_CHECK_HIP(rt::launch_big_dz2y_w3(ypart.data_ptr<float>(), (int)nparts, (int)B, (int)H, b3_dev.data_ptr<float>(),
                                        target.data_ptr<float>(), (float)gscale, dy.data_ptr<float>(), dyb.data_ptr(),
                                        sq_err.data_ptr<float>(), h2a.data_ptr(), (int)h2a.size(1),
                                        w3.data_ptr<float>(), dz2.data_ptr(), step_ctr.data_ptr<int>(),
                                        slab->data_ptr<float>(), (long long)slab->size(1), (int)slab->size(0),
                                        cur_stream(h2a)));
    return;
  }
  RT_CHECK_HIP(rt::launch_big_dz2y(ypart.data_ptr<float>(), (int)nparts, (int)B, (int)H, b3_dev.data_ptr<float>(),
                                   target.data_ptr<float>(), (float)gscale, dy.data_ptr<float>(), dyb.data_ptr(),
                                   sq_err.data_ptr<float>(), h2a.data_ptr(), (int)h2a.size(1),
                                   w3.data_ptr<float>(), dz2.data_ptr(), step_ctr.data_ptr<int>(),
                                   cur_stream(h2a)));
}

void big_dz2(torch::Tensor h2a, torch::Tensor dy, torch::Tensor w3, int64_t H, torch::Tensor dz2) {
  check_dev(h2a, "h2a");
  check_dev(dy, "dy");
  check_dev(w3, "w3");
  const int64_t B = dz2.size(0);
  check_bf16(dz2, "dz2", B, H);
  TORCH_CHECK(h2a.scalar_type() == torch::kBFloat16 && h2a.dim() == 2 && h2a.size(0) >= B &&
              h2a.size(1) >= H && H % 8 == 0, "h2a bf16 [B, >=H]");
  TORCH_CHECK(dy.numel() >= B && w3.numel() >= H, "dy [B], w3 [H]");
  const c10::DeviceGuard guard(h2a.device());
  RT_CHECK_HIP(rt::launch_big_dz2(h2a.data_ptr(), (int)h2a.size(1), dy.data_ptr<float>(),
                                  w3.data_ptr<float>(), (int)B, (int)H, dz2.data_ptr(), cur_stream(h2a)));
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

rt::NormParams norm_from(const std::vector<double>& norm) {
  TORCH_CHECK(norm.size() == 8, "norm must hold 4 scales + 4 shifts");
  rt::NormParams np;
  for (int i = 0; i < 4; ++i) {
    np.scale[i] = (float)norm[i];
    np.shift[i] = (float)norm[4 + i];
  }
  return np;
}

void check_bf16(const torch::Tensor& t, const char* name, int64_t rows, int64_t cols) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.numel() == rows * cols, name, " must have ", rows, "x", cols, " elements");
}

// Writes every output in place (static buffers: the step is HIP-graph capturable).
void eta_mlp3_train_fwd(torch::Tensor records, torch::Tensor target, torch::Tensor blob, int64_t H,
                        std::vector<double> norm, double gscale, torch::Tensor xf, torch::Tensor w3slab,
                        torch::Tensor dz2r, torch::Tensor sq_err, torch::Tensor step_ctr) {
  check_dev(records, "records");
  check_dev(target, "target");
  check_dev(blob, "blob");
  TORCH_CHECK(records.scalar_type() == torch::kInt32 && records.dim() == 2 && records.size(1) == 4,
              "records must be int32 [B,4]");
  const int64_t B = records.size(0);
  TORCH_CHECK(target.scalar_type() == torch::kFloat32 && target.numel() == B, "target must be f32 [B]");
  TORCH_CHECK(H == 64 || H == 128 || H == 256, "fused trainer: H in (64, 128, 256)");
  TORCH_CHECK(blob.scalar_type() == torch::kUInt8 &&
              (size_t)blob.numel() == rt::eta_mlp3_train_blob_bytes((int)H), "bad training blob");
  const int64_t tiles = (B + 31) / 32;
  check_bf16(xf, "xf", tiles * 32, 16);
  check_dev(w3slab, "w3slab");
  const int grid = rt::train_fwd_grid((int)B, num_cus(records.device().index()));
  TORCH_CHECK(w3slab.scalar_type() == torch::kFloat32 && w3slab.is_contiguous() && w3slab.dim() == 2 &&
                  w3slab.size(0) == grid && w3slab.size(1) == H + 16,
              "w3slab must be f32 [train_fwd_grid(B), H + 16] = [", grid, ", ", H + 16, "]");
  check_dev(dz2r, "dz2r");
  TORCH_CHECK(dz2r.scalar_type() == torch::kBFloat16 && dz2r.is_contiguous() && dz2r.numel() == tiles * 32 * H,
              "dz2r must be bf16 with ceil(B/32) * 32 * H elements");
  check_dev(sq_err, "sq_err");
  TORCH_CHECK(sq_err.scalar_type() == torch::kFloat32 && sq_err.numel() >= B, "sq_err must be f32 [B]");
  check_dev(step_ctr, "step_ctr");
  TORCH_CHECK(step_ctr.scalar_type() == torch::kInt32 && step_ctr.numel() >= 1, "step_ctr i32");
  const c10::DeviceGuard guard(records.device());
  RT_CHECK_HIP(rt::launch_eta_mlp3_train_fwd(
      records.data_ptr(), target.data_ptr<float>(), (int)B, blob.data_ptr(), (int)H,
      norm_from(norm), (float)gscale, xf.data_ptr(), w3slab.data_ptr<float>(), dz2r.data_ptr(),
      sq_err.data_ptr<float>(), step_ctr.data_ptr<int>(), num_cus(records.device().index()),
      cur_stream(records)));
}

// dgrad + relu'(z1) + dW2|db2 and dW1 partial sums per k-slice from the forward's dz2 fragments
// (train_bwd_kernel)
void train_bwd(torch::Tensor xf, int64_t B, torch::Tensor blob, int64_t H, torch::Tensor dz2r,
               torch::Tensor slab2, torch::Tensor slab1) {
  for (auto* t : {&xf, &blob, &dz2r, &slab2, &slab1}) check_dev(*t, "train_bwd tensor");
  TORCH_CHECK(H == 64 || H == 128 || H == 256, "H in (64, 128, 256)");
  const int64_t tiles = (B + 31) / 32;
  check_bf16(xf, "xf", tiles * 32, 16);
  TORCH_CHECK(dz2r.numel() == tiles * 32 * H && dz2r.scalar_type() == torch::kBFloat16 && dz2r.is_contiguous(),
              "dz2r shape");
  TORCH_CHECK(blob.scalar_type() == torch::kUInt8 && (size_t)blob.numel() == rt::eta_mlp3_train_blob_bytes((int)H),
              "bad training blob");
  const int64_t S = slab2.size(0);
  TORCH_CHECK(slab2.scalar_type() == torch::kFloat32 && slab2.dim() == 2 && slab2.size(1) == H * (H + 16) &&
                  slab1.scalar_type() == torch::kFloat32 && slab1.dim() == 2 && slab1.size(0) == S &&
                  slab1.size(1) == H * 16 && S >= 1 && S <= tiles,
              "slab2 f32 [S, H*(H+16)], slab1 f32 [S, H*16], 1 <= S <= ceil(B/32)");
  const c10::DeviceGuard guard(xf.device());
  RT_CHECK_HIP(rt::launch_train_bwd(xf.data_ptr(), (int)B, blob.data_ptr(), (int)H, dz2r.data_ptr(),
                                    slab2.data_ptr<float>(), slab1.data_ptr<float>(), (int)S, cur_stream(xf)));
}

void adamw_pack(torch::Tensor P, torch::Tensor G, torch::Tensor M, torch::Tensor V,
                torch::Tensor blob, torch::Tensor step, int64_t H, double lr,
                double beta1, double beta2, double eps, double wd, int64_t warmup,
                int64_t total_steps, double min_lr_ratio, bool update) {
  const int64_t N = rt::mlp3_num_params((int)H);
  for (auto* t : {&P, &M, &V}) {
    check_dev(*t, "adam state");
    TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->numel() == N, "P/M/V must be f32 [", N, "]");
  }
  check_dev(G, "G");
  TORCH_CHECK(G.scalar_type() == torch::kFloat32 && G.numel() == rt::mlp3_grad_bucket_floats((int)H),
              "G must be the flat f32 gradient bucket");
  TORCH_CHECK(H == 64 || H == 128 || H == 256, "fused trainer: H in (64, 128, 256)");
  check_dev(blob, "blob");
  TORCH_CHECK(blob.scalar_type() == torch::kUInt8 &&
              (size_t)blob.numel() == rt::eta_mlp3_train_blob_bytes((int)H), "bad training blob");
  check_dev(step, "step");
  const c10::DeviceGuard guard(P.device());
  RT_CHECK_HIP(rt::launch_adamw_pack(P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(),
                                     V.data_ptr<float>(), blob.data_ptr(),
                                     step.data_ptr<int>(), (int)H, (float)lr, (float)beta1,
                                     (float)beta2, (float)eps, (float)wd, (int)warmup,
                                     (int)total_steps, (float)min_lr_ratio, update ? 1 : 0,
                                     cur_stream(P)));
}

// wgrad_reduce(slab2 -> G[:H*ldg] register-native, slab -> G[H*ldg+ldg:], w3slab -> G[H*ldg:H*ldg+ldg])
// followed by adamw_pack(update=True), fused (one rank: no gradient communication in between)
void reduce_adamw(torch::Tensor slab2, torch::Tensor slab1, torch::Tensor w3slab, torch::Tensor P,
                  torch::Tensor G, torch::Tensor M, torch::Tensor V, torch::Tensor blob, torch::Tensor step,
                  int64_t H, double lr, double beta1, double beta2, double eps, double wd, int64_t warmup,
                  int64_t total_steps, double min_lr_ratio) {
  TORCH_CHECK(H == 64 || H == 128 || H == 256, "fused trainer: H in (64, 128, 256)");
  const int64_t N = rt::mlp3_num_params((int)H), ldg = H + 16;
  for (auto* t : {&P, &M, &V}) {
    check_dev(*t, "adam state");
    TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->numel() == N, "P/M/V must be f32 [", N, "]");
  }
  check_dev(G, "G");
  TORCH_CHECK(G.scalar_type() == torch::kFloat32 && G.numel() == rt::mlp3_grad_bucket_floats((int)H),
              "G must be the flat f32 gradient bucket");
  auto chk = [&](const torch::Tensor& sl, int64_t w, const char* what) {
    check_dev(sl, what);
    TORCH_CHECK(sl.scalar_type() == torch::kFloat32 && sl.dim() == 2 && sl.is_contiguous() &&
                    sl.size(0) >= 1 && sl.size(1) == w && sl.device() == G.device(),
                what, ": f32 [S, ", w, "] on G's device");
  };
  chk(slab2, H * ldg, "slab2");
  chk(slab1, 16 * H, "slab1");
  chk(w3slab, ldg, "w3slab");
  check_dev(blob, "blob");
  TORCH_CHECK(blob.scalar_type() == torch::kUInt8 &&
              (size_t)blob.numel() == rt::eta_mlp3_train_blob_bytes((int)H), "bad training blob");
  check_dev(step, "step");
  TORCH_CHECK(step.scalar_type() == torch::kInt32 && step.numel() >= 1, "step: int32");
  const c10::DeviceGuard guard(P.device());
  RT_CHECK_HIP(rt::launch_reduce_adamw(
      slab2.data_ptr<float>(), (int)slab2.size(0), (long long)slab2.size(1), slab1.data_ptr<float>(),
      (int)slab1.size(0), (long long)slab1.size(1), w3slab.data_ptr<float>(), (int)w3slab.size(0),
      (long long)w3slab.size(1), G.data_ptr<float>(), P.data_ptr<float>(), M.data_ptr<float>(),
      V.data_ptr<float>(), blob.data_ptr(), step.data_ptr<int>(), (int)H, (float)lr, (float)beta1,
      (float)beta2, (float)eps, (float)wd, (int)warmup, (int)total_steps, (float)min_lr_ratio,
      cur_stream(P)));
}

// slab: f32 [S, stride]; the partial of k-slice s is written at slab[s, offset + m*ldo + n].
void wgrad(torch::Tensor A, int64_t M, int64_t Mout, torch::Tensor Bm, int64_t N, torch::Tensor slab,
           int64_t offset, int64_t ldo, c10::optional<torch::Tensor> mask, int64_t nout,
           bool mask_hperm, int64_t nsplit) {
  check_dev(A, "A");
  if (nout < 0 || nout > N) nout = N;
  const void* mptr = nullptr;
  int ldm = 0;
  if (mask.has_value() && mask->defined()) {
    check_dev(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == torch::kBFloat16 && mask->dim() == 2 && mask->size(0) == A.size(0) &&
                    mask->size(1) >= M && mask->size(1) % 8 == 0, "mask must be bf16 [K, >=M] (ld % 8 == 0)");
    TORCH_CHECK((N + 31) / 32 == 1, "masked wgrad supports N <= 32");
    mptr = mask->data_ptr();
    ldm = (int)mask->size(1);
  }
  // Bm may be a column block of a wider row-major matrix (the wide trainer's N-blocked dW2)
  TORCH_CHECK(Bm.is_cuda() && Bm.dim() == 2 && Bm.stride(1) == 1 && Bm.stride(0) % 8 == 0 &&
                  (reinterpret_cast<uintptr_t>(Bm.data_ptr()) & 15) == 0,
              "Bm must be a row-major (column-sliced allowed) GPU tensor, 16-byte aligned");
  check_dev(slab, "slab");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && Bm.scalar_type() == torch::kBFloat16, "bf16 A/Bm");
  TORCH_CHECK(A.dim() == 2 && Bm.dim() == 2 && A.size(0) == Bm.size(0), "A/Bm must be [K, *]");
  TORCH_CHECK(M <= A.size(1) && N <= Bm.size(1) && Mout <= M, "M/N exceed operand widths");
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0 && A.size(1) % 8 == 0,
              "M, N and leading dims must be multiples of 8");
  const int NT = (int)(((N + 31) / 32 + std::max<int64_t>(nsplit, 1) - 1) / std::max<int64_t>(nsplit, 1));
  TORCH_CHECK(NT >= 1 && NT <= 9, "unsupported N=", N, " with nsplit=", nsplit,
              " (at most 288 columns per n-block)");
  TORCH_CHECK(slab.scalar_type() == torch::kFloat32 && slab.dim() == 2, "slab must be f32 [S, stride]");
  TORCH_CHECK(nsplit >= 1 && (nsplit == 1 || !mptr), "nsplit >= 1 (1 with a mask)");
  TORCH_CHECK(offset + (Mout - 1) * ldo + nout <= slab.size(1), "slab region out of range");
  const c10::DeviceGuard guard(A.device());
  RT_CHECK_HIP(rt::launch_wgrad(A.data_ptr(), (int)A.size(1), (int)M, (int)Mout, Bm.data_ptr(),
                                (int)Bm.stride(0), (int)N, (int)A.size(0), (int)slab.size(0),
                                slab.data_ptr<float>() + offset, (int)ldo, (long long)slab.size(1),
                                cur_stream(A), mptr, ldm, (int)nout, mask_hperm, (int)nsplit));
}

// dW2|db2 (segment 0, nsplit0 n-blocks per k-slice) and dW1 (segment 1, N <= 32) in ONE launch:
// each segment's fp32 partials go to row s of its own slab (whole rows, offset 0)
void wgrad_dual(torch::Tensor A0, int64_t M0, torch::Tensor B0, int64_t N0, torch::Tensor slab0, int64_t ldo0,
                int64_t nsplit0, torch::Tensor A1, int64_t M1, torch::Tensor B1, int64_t N1, torch::Tensor slab1,
                int64_t ldo1) {
  auto chk = [](const torch::Tensor& A, int64_t M, const torch::Tensor& Bm, int64_t N, const torch::Tensor& slab,
                int64_t ldo) {
    check_dev(A, "A");
    check_dev(Bm, "Bm");
    check_dev(slab, "slab");
    TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && Bm.scalar_type() == torch::kBFloat16, "bf16 A/Bm");
    TORCH_CHECK(A.dim() == 2 && Bm.dim() == 2 && A.size(0) == Bm.size(0) && A.is_contiguous() &&
                    Bm.is_contiguous(), "A/Bm must be contiguous [K, *]");
    TORCH_CHECK(M <= A.size(1) && N <= Bm.size(1) && M % 8 == 0 && N % 8 == 0 && A.size(1) % 8 == 0 &&
                    Bm.size(1) % 8 == 0, "M/N: multiples of 8 within the operand widths");
    TORCH_CHECK(slab.scalar_type() == torch::kFloat32 && slab.dim() == 2 && slab.is_contiguous() &&
                    (M - 1) * ldo + N <= slab.size(1), "slab must be f32 [S, >= (M-1)*ldo+N]");
  };
  chk(A0, M0, B0, N0, slab0, ldo0);
  chk(A1, M1, B1, N1, slab1, ldo1);
  TORCH_CHECK(A0.size(0) == A1.size(0), "both segments reduce over the same batch");
  TORCH_CHECK(N1 <= 32, "segment 1 takes N <= 32");
  TORCH_CHECK(A0.device() == A1.device() && slab0.device() == A0.device() && slab1.device() == A0.device(),
              "one device");
  const int nsp = (int)std::max<int64_t>(nsplit0, 1);
  const int NT0 = (int)((N0 + 31) / 32 + nsp - 1) / nsp;
  TORCH_CHECK(NT0 >= 1 && NT0 <= 9, "at most 288 columns per n-block");
  const c10::DeviceGuard guard(A0.device());
  RT_CHECK_HIP(rt::launch_wgrad_dual(A0.data_ptr(), (int)A0.size(1), (int)M0, (int)M0, B0.data_ptr(),
                                     (int)B0.size(1), (int)N0, (int)A0.size(0), (int)slab0.size(0),
                                     slab0.data_ptr<float>(), (int)ldo0, (long long)slab0.size(1), (int)N0, nsp,
                                     A1.data_ptr(), (int)A1.size(1), (int)M1, (int)M1, B1.data_ptr(),
                                     (int)B1.size(1), (int)N1, (int)slab1.size(0), slab1.data_ptr<float>(),
                                     (int)ldo1, (long long)slab1.size(1), (int)N1, cur_stream(A0)));
}

// dW2|db2 of the wide trainer on 256 x 256 output tiles (wgrad.hip wgrad256_kernel): A [K, >= M], B [K, >= N]
// bf16 row-major, slab f32 [S, >= M * ldo]; db2_col >= 0 also writes the column sums of A per tile column
void wgrad256(torch::Tensor A, torch::Tensor B, int64_t M, int64_t N, torch::Tensor slab, int64_t ldo, int64_t db2_col) {
  check_dev(A, "A");
  check_dev(B, "B");
  check_dev(slab, "slab");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "bf16 A/B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0) && A.is_contiguous() && B.is_contiguous(),
              "A/B must be contiguous [K, *]");
  TORCH_CHECK(M % 256 == 0 && N % 256 == 0 && M <= A.size(1) && N <= B.size(1) && A.size(0) % 64 == 0 &&
                  A.size(1) % 8 == 0 && B.size(1) % 8 == 0,
              "wgrad256: M, N multiples of 256 within the operands, K a multiple of 64");
  TORCH_CHECK(slab.scalar_type() == torch::kFloat32 && slab.dim() == 2 && slab.is_contiguous() &&
                  (M - 1) * ldo + std::max<int64_t>(N, db2_col >= 0 ? db2_col + N / 256 : 0) <= slab.size(1) &&
                  ldo >= N,
              "slab must be f32 [S, >= M * ldo]");
  TORCH_CHECK(db2_col < 0 || (db2_col >= N && db2_col + N / 256 <= ldo), "db2 columns must lie beside the output");
  const c10::DeviceGuard guard(A.device());
  RT_CHECK_HIP(rt::launch_wgrad256(A.data_ptr(), (int)A.size(1), B.data_ptr(), (int)B.size(1), (int)M, (int)N,
                                   (int)A.size(0), (int)slab.size(0), slab.data_ptr<float>(), (int)ldo,
                                   (long long)slab.size(1), (int)db2_col, cur_stream(A)));
}

void wgrad_reduce(torch::Tensor slab, torch::Tensor G, c10::optional<torch::Tensor> slab1,
                  c10::optional<torch::Tensor> G1, c10::optional<torch::Tensor> slab2,
                  c10::optional<torch::Tensor> G2, int64_t perm_h, int64_t fold_ld, int64_t fold_col) {
  auto chk = [&](const torch::Tensor& sl, const torch::Tensor& g) {
    check_dev(sl, "slab");
    check_dev(g, "G");
    TORCH_CHECK(sl.scalar_type() == torch::kFloat32 && g.scalar_type() == torch::kFloat32, "f32");
    TORCH_CHECK(sl.dim() == 2 && sl.size(1) >= g.numel() && sl.is_contiguous() && g.is_contiguous(),
                "slab/G shape");
    TORCH_CHECK(sl.device() == G.device() && g.device() == G.device(), "one device");
  };
  chk(slab, G);
  const bool two = slab1.has_value() && slab1->defined();
  TORCH_CHECK(two == (G1.has_value() && G1->defined()), "slab1 and G1 go together");
  const bool three = slab2.has_value() && slab2->defined();
  TORCH_CHECK(three == (G2.has_value() && G2->defined()), "slab2 and G2 go together");
  if (two) chk(*slab1, *G1);
  if (three) chk(*slab2, *G2);
  const c10::DeviceGuard guard(G.device());
  RT_CHECK_HIP(rt::launch_wgrad_reduce(
      slab.data_ptr<float>(), (int)slab.size(0), (long long)slab.size(1), G.data_ptr<float>(),
      (int)G.numel(), cur_stream(G), two ? slab1->data_ptr<float>() : nullptr,
      two ? (int)slab1->size(0) : 0, two ? (long long)slab1->size(1) : 0,
      two ? G1->data_ptr<float>() : nullptr, two ? (int)G1->numel() : 0,
      three ? slab2->data_ptr<float>() : nullptr, three ? (int)slab2->size(0) : 0,
      three ? (long long)slab2->size(1) : 0, three ? G2->data_ptr<float>() : nullptr,
      three ? (int)G2->numel() : 0, (int)perm_h, (int)fold_ld, (int)fold_col));
}

void check_csr(const torch::Tensor& indptr, const torch::Tensor& indices, const torch::Tensor& values) {
  for (auto* t : {&indptr, &indices, &values}) check_dev(*t, "csr");
  TORCH_CHECK(indptr.scalar_type() == torch::kInt32 && indices.scalar_type() == torch::kInt32 &&
              values.scalar_type() == torch::kFloat32, "CSR must be int32/int32/f32");
  TORCH_CHECK(indices.numel() == values.numel(), "indices/values length");
}

void gcn_agg_gemm(torch::Tensor X, torch::Tensor indptr, torch::Tensor indices, torch::Tensor values,
                  torch::Tensor wfrag, c10::optional<torch::Tensor> bias, torch::Tensor Y, int64_t fin,
                  int64_t fout, bool agg, bool relu, int64_t row0, int64_t row1) {
  check_dev(X, "X");
  check_dev(wfrag, "wfrag");
  check_dev(Y, "Y");
  check_csr(indptr, indices, values);
  TORCH_CHECK(X.scalar_type() == torch::kBFloat16 && X.dim() == 2 && X.size(1) == fin, "X bf16 [N,fin]");
  TORCH_CHECK(Y.scalar_type() == torch::kBFloat16 && Y.dim() == 2 && Y.size(1) == fout &&
              Y.size(0) >= row1, "Y bf16 [N,fout]");
  TORCH_CHECK(wfrag.scalar_type() == torch::kBFloat16 && wfrag.numel() == fin * fout, "wfrag");
  TORCH_CHECK(0 <= row0 && row0 <= row1 && row1 <= X.size(0) && indptr.numel() >= row1 + 1, "rows");
  const float* bptr = nullptr;
  if (bias.has_value()) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == fout, "bias f32 [fout]");
    bptr = bias->data_ptr<float>();
  }
  const c10::DeviceGuard guard(X.device());
  RT_CHECK_HIP(rt::launch_gcn_agg_gemm(X.data_ptr(), indptr.data_ptr<int>(), indices.data_ptr<int>(),
                                       values.data_ptr<float>(), wfrag.data_ptr(), bptr, Y.data_ptr(),
                                       (int)fin, (int)fout, agg, relu, (int)row0, (int)row1,
                                       num_cus(X.device().index()), cur_stream(X)));
}

void gcn_l1_fused(torch::Tensor X, torch::Tensor indptr, torch::Tensor indices, torch::Tensor values,
                  torch::Tensor w1frag, torch::Tensor b1, torch::Tensor w2frag, torch::Tensor Z, int64_t row0,
                  int64_t row1) {
  check_dev(X, "X");
  check_dev(w1frag, "w1frag");
  check_dev(w2frag, "w2frag");
  check_dev(b1, "b1");
  check_dev(Z, "Z");
  check_csr(indptr, indices, values);
  const int64_t fin = X.size(1), fhid = b1.numel(), fz = Z.size(1);
  TORCH_CHECK(X.scalar_type() == torch::kBFloat16 && X.dim() == 2, "X bf16 [N,fin]");
  TORCH_CHECK(Z.scalar_type() == torch::kBFloat16 && Z.dim() == 2 && Z.size(0) >= row1, "Z bf16 [N,fz]");
  TORCH_CHECK(fin == 32 && fhid == 128 && fz == 32, "fused layer 1 is built for 32 -> 128 -> 32");
  TORCH_CHECK(w1frag.numel() == fin * fhid && w2frag.numel() == fhid * fz, "weight fragments");
  TORCH_CHECK(b1.scalar_type() == torch::kFloat32, "b1 f32");
  TORCH_CHECK(0 <= row0 && row0 <= row1 && row1 <= X.size(0) && indptr.numel() >= row1 + 1, "rows");
  const c10::DeviceGuard guard(X.device());
  RT_CHECK_HIP(rt::launch_gcn_l1_fused(X.data_ptr(), indptr.data_ptr<int>(), indices.data_ptr<int>(),
                                       values.data_ptr<float>(), w1frag.data_ptr(), b1.data_ptr<float>(),
                                       w2frag.data_ptr(), Z.data_ptr(), (int)fin, (int)fhid, (int)fz, (int)row0,
                                       (int)row1, num_cus(X.device().index()), cur_stream(X)));
}

void gcn_spmm_score(torch::Tensor Z, torch::Tensor indptr, torch::Tensor indices, torch::Tensor values,
                    torch::Tensor b2, torch::Tensor wo, double bo, torch::Tensor delay, int64_t row0,
                    int64_t row1) {
  check_dev(Z, "Z");
  check_csr(indptr, indices, values);
  TORCH_CHECK(Z.scalar_type() == torch::kBFloat16 && Z.dim() == 2 && Z.size(1) == 32, "Z bf16 [N,32]");
  TORCH_CHECK(b2.numel() == 32 && wo.numel() == 32, "b2/wo [32]");
  TORCH_CHECK(delay.scalar_type() == torch::kFloat32 && delay.numel() >= row1, "delay f32 [N]");
  const c10::DeviceGuard guard(Z.device());
  RT_CHECK_HIP(rt::launch_gcn_spmm_score(Z.data_ptr(), indptr.data_ptr<int>(), indices.data_ptr<int>(),
                                         values.data_ptr<float>(), b2.data_ptr<float>(),
                                         wo.data_ptr<float>(), (float)bo, delay.data_ptr<float>(),
                                         (int)row0, (int)row1, cur_stream(Z)));
}

// latlon: f32 [N, 2] (degrees), delay: f32 [>= N]; node ids outside [0, N) add nothing
torch::Tensor route_score(torch::Tensor rptr, torch::Tensor nodes, torch::Tensor latlon, torch::Tensor delay) {
  for (auto* t : {&rptr, &nodes, &latlon, &delay}) check_dev(*t, "route_score input");
  TORCH_CHECK(rptr.scalar_type() == torch::kInt32 && nodes.scalar_type() == torch::kInt32 &&
                  rptr.is_contiguous() && nodes.is_contiguous(), "i32 routes");
  TORCH_CHECK(latlon.scalar_type() == torch::kFloat32 && latlon.dim() == 2 && latlon.size(1) == 2 &&
                  latlon.is_contiguous(), "latlon must be f32 [N, 2]");
  TORCH_CHECK(delay.scalar_type() == torch::kFloat32 && delay.numel() >= latlon.size(0), "delay f32 [>= N]");
  const c10::DeviceGuard guard(rptr.device());
  const int R = (int)rptr.numel() - 1;
  auto score = torch::empty({R}, delay.options());
  RT_CHECK_HIP(rt::launch_route_score(rptr.data_ptr<int>(), nodes.data_ptr<int>(), latlon.data_ptr<float>(),
                                      delay.data_ptr<float>(), score.data_ptr<float>(), R,
                                      (int)latlon.size(0), cur_stream(rptr)));
  return score;
}

// One tier's workspace from (tab int64 [S, 2 << (tbits-1) ... i.e. 2 * TS], heap int64 [S, cap],
// touched int32 [S, TS / 2]) — routing/graph.py AstarTier.  None -> tier off.
static bool ws_from(const py::object& o, rt::AstarWs& ws, const torch::Device& dev) {
  if (o.is_none()) return false;
  auto t = o.cast<std::tuple<torch::Tensor, torch::Tensor, torch::Tensor>>();
  torch::Tensor tab = std::get<0>(t), heap = std::get<1>(t), touched = std::get<2>(t);
  for (auto* x : {&tab, &heap, &touched}) check_dev(*x, "astar workspace");
  TORCH_CHECK(tab.device() == dev && heap.device() == dev && touched.device() == dev, "workspace on another GPU");
  TORCH_CHECK(tab.scalar_type() == torch::kInt64 && tab.dim() == 2 && heap.scalar_type() == torch::kInt64 &&
                  heap.dim() == 2 && touched.scalar_type() == torch::kInt32 && touched.dim() == 2,
              "workspace dtypes: tab int64 [S, 2*TS], heap int64 [S, cap], touched int32 [S, TS/2]");
  const int64_t TS = tab.size(1) / 2;
  TORCH_CHECK(TS >= 64 && (TS & (TS - 1)) == 0 && tab.size(1) == 2 * TS, "table size must be a power of two");
  TORCH_CHECK(heap.size(0) == tab.size(0) && touched.size(0) == tab.size(0) && touched.size(1) == TS / 2,
              "workspace rows");
  ws.tab = tab.data_ptr();
  ws.heap = heap.data_ptr();
  ws.touched = touched.data_ptr<int>();
  ws.slots = (int)tab.size(0);
  ws.cap = (int)heap.size(1);
  int tb = 0;
  while ((int64_t(1) << tb) < TS) ++tb;
  ws.tbits = tb;
  return true;
}

// The tiered batched A* (csrc/astar.hip astar_search).  Returns [lane queries, wave queries,
// escalated queries, lane ms, wave ms, big ms, retried queries, retry ms].
std::vector<double> astar_search(torch::Tensor indptr, torch::Tensor indices, torch::Tensor cost, torch::Tensor lat,
                                 torch::Tensor lon, double inv_vmax, c10::optional<torch::Tensor> landmarks,
                                 torch::Tensor src, torch::Tensor dst, py::object lane, py::object wave,
                                 py::object big, torch::Tensor out_cost, torch::Tensor out_len,
                                 torch::Tensor out_status, torch::Tensor out_path,
                                 c10::optional<torch::Tensor> out_iters, torch::Tensor scratch, int64_t max_iters,
                                 int64_t lane_pops, int64_t wave_only_below, double delta,
                                 c10::optional<torch::Tensor> arena, c10::optional<torch::Tensor> arena_ctr,
                                 double lane_max_m, int64_t wave_nw, int64_t retry_nw) {
  for (auto* t : {&indptr, &indices, &cost, &lat, &lon, &src, &dst, &out_cost, &out_len, &out_status, &out_path,
                  &scratch})
    check_dev(*t, "astar tensor");
  const int64_t N = lat.numel();
  TORCH_CHECK(indptr.numel() == N + 1 && cost.numel() == indices.numel() && lon.numel() == N, "graph shapes");
  TORCH_CHECK(indptr.scalar_type() == torch::kInt32 && indices.scalar_type() == torch::kInt32 &&
                  cost.scalar_type() == torch::kFloat32 && lat.scalar_type() == torch::kFloat32 &&
                  lon.scalar_type() == torch::kFloat32 && src.scalar_type() == torch::kInt32 &&
                  dst.scalar_type() == torch::kInt32,
              "graph dtypes");
  const int64_t Q = src.numel();
  TORCH_CHECK(dst.numel() == Q && out_cost.numel() == Q && out_len.numel() == Q && out_status.numel() == Q &&
                  out_path.dim() == 2 && out_path.size(0) == Q && out_status.scalar_type() == torch::kInt32 &&
                  out_len.scalar_type() == torch::kInt32 && out_path.scalar_type() == torch::kInt32 &&
                  out_cost.scalar_type() == torch::kFloat32,
              "outputs [Q]");
  TORCH_CHECK(scratch.scalar_type() == torch::kInt32 && scratch.numel() >= Q + 1, "scratch int32 [Q + 1]");
  rt::AstarGraphDev g;
  g.indptr = indptr.data_ptr<int>();
  g.indices = indices.data_ptr<int>();
  g.cost = cost.data_ptr<float>();
  g.lat = lat.data_ptr<float>();
  g.lon = lon.data_ptr<float>();
  g.N = (int)N;
  g.inv_vmax = (float)inv_vmax;
  if (landmarks.has_value() && landmarks->defined()) {
    check_dev(*landmarks, "landmarks");
    TORCH_CHECK(landmarks->scalar_type() == torch::kFloat32 && landmarks->dim() == 2 && landmarks->size(0) == N &&
                    (landmarks->size(1) == 16 || landmarks->size(1) == 32 || landmarks->size(1) == 64),
                "landmarks must be f32 [N, 2K] with K in {8, 16, 32}");
    g.lm = landmarks->data_ptr<float>();
    g.K = (int)landmarks->size(1) / 2;
  }
  rt::AstarOut o;
  o.cost = out_cost.data_ptr<float>();
  o.len = out_len.data_ptr<int>();
  o.status = out_status.data_ptr<int>();
  o.path = out_path.data_ptr<int>();
  o.max_path = (int)out_path.size(1);
  if (out_iters.has_value() && out_iters->defined()) {
    check_dev(*out_iters, "out_iters");
    TORCH_CHECK(out_iters->scalar_type() == torch::kInt32 && out_iters->numel() == Q, "out_iters int32 [Q]");
    o.iters = out_iters->data_ptr<int>();
  }
  rt::AstarWs wl, ww, wb;
  const bool hl = ws_from(lane, wl, lat.device()), hw = ws_from(wave, ww, lat.device()),
             hb = ws_from(big, wb, lat.device());
  TORCH_CHECK(hl || hw, "need a lane or a wave tier");
  TORCH_CHECK((!hl || rt::astar_ws_ok(wl, false)) && (!hw || rt::astar_ws_ok(ww, true)) &&
                  (!hb || rt::astar_ws_ok(wb, true)),
              "A* workspace too small (wave tiers need cap >= 128, cap % 8 == 0)");
  rt::AstarPlan pl;
  pl.max_iters = (int)max_iters;
  pl.lane_pops = (int)lane_pops;
  pl.wave_only_below = (int)wave_only_below;
  pl.delta = (float)delta;
  pl.lane_max_m = (float)lane_max_m;
  pl.wave_nw = (int)wave_nw;
  pl.retry_nw = (int)retry_nw;
  TORCH_CHECK(wave_nw == 0 || wave_nw == 1 || wave_nw == 2 || wave_nw == 4 || wave_nw == 8, "wave_nw in {0,1,2,4,8}");
  TORCH_CHECK(retry_nw == 0 || retry_nw == 1 || retry_nw == 2 || retry_nw == 4 || retry_nw == 8, "retry_nw in {0,1,2,4,8}");
  rt::AstarRunStats st;
  rt::AstarArenaBuf ab;
  if (arena.has_value() && arena->defined()) {
    TORCH_CHECK(arena_ctr.has_value() && arena_ctr->defined(), "arena needs its counter");
    check_dev(*arena, "arena");
    check_dev(*arena_ctr, "arena_ctr");
    TORCH_CHECK(arena->scalar_type() == torch::kInt64 && arena->is_contiguous() && arena->numel() % 2 == 0 &&
                    arena_ctr->scalar_type() == torch::kInt64 && arena_ctr->numel() >= 1,
                "arena int64 [2n] (all-ones), counter int64 [1]");
    ab.base = arena->data_ptr();
    ab.entries = (unsigned long long)(arena->numel() / 2);
    ab.ctr = (unsigned long long*)arena_ctr->data_ptr();
  }
  const c10::DeviceGuard guard(lat.device());
  RT_CHECK_HIP(rt::astar_search(g, src.data_ptr<int>(), dst.data_ptr<int>(), (int)Q, hl ? &wl : nullptr,
                                hw ? &ww : nullptr, hb ? &wb : nullptr, o, pl, scratch.data_ptr<int>(),
                                cur_stream(lat), &st, ab.base ? &ab : nullptr));
  return {(double)st.lane, (double)st.wave, (double)st.escalated, st.lane_ms, st.wave_ms, st.big_ms,
          (double)st.retried, st.retry_ms};
}

torch::Tensor forest_predict(torch::Tensor records, torch::Tensor values, torch::Tensor info,
                             torch::Tensor roots, double base, bool le, std::vector<int64_t> fmap) {
  for (auto* t : {&records, &values, &info, &roots}) check_dev(*t, "forest tensor");
  TORCH_CHECK(records.scalar_type() == torch::kInt32 && records.dim() == 2 && records.size(1) == 4,
              "records must be int32 [B,4]");
  TORCH_CHECK(values.scalar_type() == torch::kFloat32 && info.scalar_type() == torch::kInt32 &&
              values.numel() == info.numel() && roots.scalar_type() == torch::kInt32, "forest arrays");
  TORCH_CHECK(fmap.size() == 12, "fmap must have 12 entries");
  const c10::DeviceGuard guard(records.device());
  const int B = (int)records.size(0);
  auto out = torch::empty({B}, values.options());
  int fm[12];
  for (int j = 0; j < 12; ++j) fm[j] = (int)fmap[j];
  RT_CHECK_HIP(rt::launch_forest(records.data_ptr(), values.data_ptr<float>(),
                                 (const unsigned*)info.data_ptr<int>(), roots.data_ptr<int>(),
                                 out.data_ptr<float>(), B, (int)roots.numel(), (int)values.numel(),
                                 (float)base, le ? 1 : 0, fm, cur_stream(records)));
  return out;
}

// ---------------------------------------------------------------- resident scorer (persistent_serve.hip)
std::mutex g_ps_mu;
std::vector<rt::PersistentScorer*> g_ps;

rt::PersistentScorer* ps_get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_ps_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_ps.size() && g_ps[h] != nullptr, "bad resident scorer handle");
  return g_ps[h];
}

int64_t pscore_create(torch::Tensor blob, int64_t H, std::vector<double> norm, int64_t cap, double idle_ms,
                      double life_ms) {
  check_dev(blob, "blob");
  TORCH_CHECK((size_t)blob.numel() == rt::eta_mlp3_blob_bytes((int)H), "bad blob");
  TORCH_CHECK(norm.size() == 8, "norm must hold 4 scales + 4 shifts");
  rt::NormParams np;
  for (int i = 0; i < 4; ++i) {
    np.scale[i] = (float)norm[i];
    np.shift[i] = (float)norm[4 + i];
  }
  hipError_t e = hipSuccess;
  rt::PersistentScorer* p = rt::pscore_create((int)blob.device().index(), blob.data_ptr(), (int)H, np, (int)cap,
                                              idle_ms, life_ms, &e);
  TORCH_CHECK(p != nullptr, "resident scorer: ", hipGetErrorString(e));
  std::lock_guard<std::mutex> lk(g_ps_mu);
  g_ps.push_back(p);
  return (int64_t)g_ps.size() - 1;
}

// rec: CPU int32 [n,4] (16-byte records), out: CPU f32 [n].  False when the scorer did not answer
// (the caller then scores with a normal launch).  Not thread-safe per handle (callers hold a lock).
bool pscore_score(int64_t h, torch::Tensor rec, torch::Tensor out) {
  rt::PersistentScorer* p = ps_get(h);
  TORCH_CHECK(!rec.is_cuda() && rec.is_contiguous() && rec.scalar_type() == torch::kInt32 && rec.dim() == 2 &&
                  rec.size(1) == 4, "rec must be contiguous CPU int32 [n,4]");
  TORCH_CHECK(!out.is_cuda() && out.is_contiguous() && out.scalar_type() == torch::kFloat32 &&
                  out.numel() == rec.size(0), "out must be contiguous CPU f32 [n]");
  const int n = (int)rec.size(0);
  if (n > rt::pscore_cap(p) || rt::pscore_broken(p)) return false;
  hipError_t e;
  {
    py::gil_scoped_release nogil;
    std::memcpy(rt::pscore_records(p), rec.data_ptr(), (size_t)n * 16);
    e = rt::pscore_run(p, n, 200.0);
    if (e == hipSuccess) std::memcpy(out.data_ptr(), rt::pscore_out(p), (size_t)n * 4);
  }
  return e == hipSuccess;
}

// ---------------------------------------------------------------- GCN scorer training (gcn_train.hip)
// One backward pass of the scorer over the rows [r0, r1) (all nodes' dy): writes the flat fp32
// gradient [W1 | b1 | W2 | b2 | wo | bo] and the squared-error sum of those rows.
void gcn_train_bwd(torch::Tensor X, torch::Tensor Z, torch::Tensor indptr, torch::Tensor indices,
                   torch::Tensor values, torch::Tensor w1frag, torch::Tensor b1, torch::Tensor W2,
                   torch::Tensor b2, torch::Tensor wo, torch::Tensor bo, torch::Tensor target, int64_t r0,
                   int64_t r1, torch::Tensor dy, torch::Tensor slab1, torch::Tensor slab2, torch::Tensor grad,
                   torch::Tensor loss) {
  for (auto* t : {&X, &Z, &indptr, &indices, &values, &w1frag, &b1, &W2, &b2, &wo, &bo, &target, &dy, &slab1,
                  &slab2, &grad, &loss})
    check_dev(*t, "gcn_train_bwd tensor");
  const int64_t N = X.size(0);
  TORCH_CHECK(X.scalar_type() == torch::kBFloat16 && X.dim() == 2 && X.size(1) == 32, "X bf16 [N,32]");
  TORCH_CHECK(Z.scalar_type() == torch::kBFloat16 && Z.dim() == 2 && Z.size(0) >= N && Z.size(1) == 32, "Z bf16 [N,32]");
  TORCH_CHECK(indptr.numel() == N + 1 && indices.numel() == values.numel(), "CSR shapes");
  TORCH_CHECK(w1frag.scalar_type() == torch::kBFloat16 && w1frag.numel() == 32 * 128, "w1frag bf16 [32*128]");
  TORCH_CHECK(b1.numel() == 128 && W2.numel() == 128 * 32 && b2.numel() == 32 && wo.numel() == 32 && bo.numel() == 1,
              "parameter shapes");
  for (auto* t : {&b1, &W2, &b2, &wo, &bo, &target, &dy, &slab1, &slab2, &grad, &loss})
    TORCH_CHECK(t->scalar_type() == torch::kFloat32, "fp32 operands");
  TORCH_CHECK(target.numel() == N && dy.numel() >= N, "target / dy [N]");
  TORCH_CHECK(0 <= r0 && r0 <= r1 && r1 <= N, "row range");
  TORCH_CHECK(slab1.dim() == 2 && slab1.size(1) == 32 * 128 + 256 && slab1.size(0) >= 8, "slab1 [>=8, 4352]");
  TORCH_CHECK(slab2.dim() == 2 && slab2.size(1) == 34 && slab2.size(0) >= rt::gcn_train_slab2_rows((int)N),
              "slab2 [rows, 34]");
  TORCH_CHECK(grad.numel() == rt::gcn_grad_numel() && loss.numel() >= 1, "grad [8385], loss [1]");
  const c10::DeviceGuard guard(X.device());
  RT_CHECK_HIP(rt::launch_gcn_train_bwd(X.data_ptr(), Z.data_ptr(), indptr.data_ptr<int>(), indices.data_ptr<int>(),
                                        values.data_ptr<float>(), w1frag.data_ptr(), b1.data_ptr<float>(),
                                        W2.data_ptr<float>(), b2.data_ptr<float>(), wo.data_ptr<float>(),
                                        bo.data_ptr<float>(), target.data_ptr<float>(), (int)N, (int)r0, (int)r1,
                                        dy.data_ptr<float>(), slab1.data_ptr<float>(), (int)slab1.size(0),
                                        slab2.data_ptr<float>(), grad.data_ptr<float>(), loss.data_ptr<float>(),
                                        num_cus(X.device().index()), cur_stream(X)));
}

// ---------------------------------------------------------------- native predict server
// One route service config per GPU from a Python dict (routest_amd/serve/native_server.py
// route_config): scalars, host arrays (CPU tensors) and device tensors the caller keeps alive.
static rt::RouteServiceCfg route_cfg_from(const py::dict& d, int device) {
  rt::RouteServiceCfg c;
  auto has = [&](const char* k) { return d.contains(k) && !d[k].is_none(); };
  auto tptr = [&](const char* k, bool cuda) -> void* {
    if (!has(k)) return nullptr;
    torch::Tensor t = d[k].cast<torch::Tensor>();
    TORCH_CHECK(t.is_contiguous(), "route config tensor ", k, " must be contiguous");
    TORCH_CHECK(t.is_cuda() == cuda, "route config tensor ", k, cuda ? " must be on the GPU" : " must be on the CPU");
    if (cuda) TORCH_CHECK(t.device().index() == device, "route config tensor ", k, " on the wrong GPU");
    return t.data_ptr();
  };
  c.device = device;
  c.provider = d["provider"].cast<std::string>() == "graph" ? 1 : 0;
  if (has("circuity")) c.circuity = d["circuity"].cast<double>();
  if (has("step_m")) c.step_m = d["step_m"].cast<double>();
  if (has("engine")) c.engine = d["engine"].cast<std::string>();
  if (has("compat200")) c.compat200 = d["compat200"].cast<bool>();
  if (has("batch_max")) c.batch_max = d["batch_max"].cast<int>();
  if (has("timeout_us")) c.timeout_us = d["timeout_us"].cast<double>();
  if (has("chunk_threads")) c.chunk_threads = d["chunk_threads"].cast<int>();
  if (has("sqlite_path")) c.sqlite_path = d["sqlite_path"].cast<std::string>();
  if (c.provider == 1 && has("cch_ptr")) {
    // road graph through the CCH router (routing/cch.py RoadRouter.gpu on this device)
    c.cch = reinterpret_cast<rt::CchGpu*>((uintptr_t)d["cch_ptr"].cast<uint64_t>());
    TORCH_CHECK(c.cch != nullptr && c.cch->device() == device, "route config: CCH router on the wrong GPU");
    c.cch_contexts = has("cch_contexts") ? d["cch_contexts"].cast<bool>() : true;
    if (has("cch_fixed_key")) c.cch_fixed_key = d["cch_fixed_key"].cast<uint64_t>();
    c.glat = (const double*)tptr("glat", false);
    c.glon = (const double*)tptr("glon", false);
    c.h_indptr = (const int*)tptr("h_indptr", false);
    c.h_indices = (const int*)tptr("h_indices", false);
    c.h_length = (const float*)tptr("h_length", false);
    c.h_edge_name = (const int32_t*)tptr("h_edge_name", false);
    if (has("names")) c.names = d["names"].cast<std::vector<std::string>>();
    c.N = d["N"].cast<int>();
    c.snap_c = d["snap_c"].cast<double>();
    c.max_path = d["max_path"].cast<int>();
    TORCH_CHECK(c.glat && c.glon && c.h_indptr && c.h_indices && c.h_length && c.N == c.cch->topo().N &&
                    c.max_path > 0,
                "CCH route config incomplete");
  } else if (c.provider == 1) {
    c.glat = (const double*)tptr("glat", false);
    c.glon = (const double*)tptr("glon", false);
    c.h_indptr = (const int*)tptr("h_indptr", false);
    c.h_indices = (const int*)tptr("h_indices", false);
    c.h_cost = (const float*)tptr("h_cost", false);
    c.indptr = (const int*)tptr("indptr", true);
    c.indices = (const int*)tptr("indices", true);
    c.cost = (const float*)tptr("cost", true);
    c.lat32 = (const float*)tptr("lat32", true);
    c.lon32 = (const float*)tptr("lon32", true);
    c.lm = (const float*)tptr("lm", true);
    const torch::Device dev(torch::kCUDA, device);
    ws_from(d.contains("lane_ws") ? py::object(d["lane_ws"]) : py::object(py::none()), c.lane_ws, dev);
    ws_from(d.contains("wave_ws") ? py::object(d["wave_ws"]) : py::object(py::none()), c.wave_ws, dev);
    ws_from(d.contains("big_ws") ? py::object(d["big_ws"]) : py::object(py::none()), c.big_ws, dev);
    if (has("arena")) {
      torch::Tensor ar = d["arena"].cast<torch::Tensor>(), ctr = d["arena_ctr"].cast<torch::Tensor>();
      TORCH_CHECK(ar.is_cuda() && ar.device().index() == device && ar.scalar_type() == torch::kInt64 &&
                      ctr.is_cuda() && ctr.scalar_type() == torch::kInt64, "route config arena");
      c.arena.base = ar.data_ptr();
      c.arena.entries = (unsigned long long)(ar.numel() / 2);
      c.arena.ctr = (unsigned long long*)ctr.data_ptr();
    }
    c.N = d["N"].cast<int>();
    c.K = has("K") ? d["K"].cast<int>() : 0;
    c.snap_c = d["snap_c"].cast<double>();
    c.max_path = d["max_path"].cast<int>();
    c.max_iters = d["max_iters"].cast<int>();
    c.lane_pops = d["lane_pops"].cast<int>();
    if (has("wave_only_below")) c.wave_only_below = d["wave_only_below"].cast<int>();
    c.inv_vmax = d["inv_vmax"].cast<float>();
    c.wave_delta = d["wave_delta"].cast<float>();
    if (has("lane_max_m")) c.lane_max_m = d["lane_max_m"].cast<float>();
    TORCH_CHECK(c.glat && c.glon && c.indptr && c.indices && c.cost && c.lat32 && c.lon32 &&
                    (c.lane_ws.slots > 0 || c.wave_ws.slots > 0) && c.N > 0 && c.max_path > 0,
                "graph route config incomplete");
    TORCH_CHECK(c.lm == nullptr || c.K == 8 || c.K == 16 || c.K == 32, "landmarks K must be 8, 16 or 32");
    TORCH_CHECK((c.lane_ws.slots == 0 || rt::astar_ws_ok(c.lane_ws, false)) &&
                    (c.wave_ws.slots == 0 || rt::astar_ws_ok(c.wave_ws, true)) &&
                    (c.big_ws.slots == 0 || rt::astar_ws_ok(c.big_ws, true)),
                "A* workspace too small");
  }
  return c;
}

// One native model (csrc/native_model.h) on `device` from a Python spec (serve/native_server.py
// native_model_spec): {"kind": "mlp3" | "wide" | "forest", ...device tensors / params..., "host":
// {fp32 CPU copies for the CPU fallback}}.  The native side copies the device tensors.
static std::vector<float> host_f32(const py::dict& h, const char* k) {
  torch::Tensor t = h[k].cast<torch::Tensor>().to(torch::kCPU).to(torch::kFloat32).contiguous();
  return std::vector<float>(t.data_ptr<float>(), t.data_ptr<float>() + t.numel());
}
static rt::MlpHost mlp_host_from(const py::dict& d) {
  rt::MlpHost m;
  if (!d.contains("host") || d["host"].is_none()) return m;
  py::dict h = d["host"].cast<py::dict>();
  m.w1 = host_f32(h, "w1");
  m.b1 = host_f32(h, "b1");
  m.w2 = host_f32(h, "w2");
  m.b2 = host_f32(h, "b2");
  m.w3 = host_f32(h, "w3");
  m.b3 = h["b3"].cast<float>();
  m.x_mean = host_f32(h, "x_mean");
  m.x_std = host_f32(h, "x_std");
  m.y_mean = h["y_mean"].cast<float>();
  m.y_std = h["y_std"].cast<float>();
  m.H = (int)m.b1.size();
  TORCH_CHECK(m.w1.size() == (size_t)m.H * 12 && m.w2.size() == (size_t)m.H * m.H && m.b2.size() == (size_t)m.H &&
                  m.w3.size() == (size_t)m.H && m.x_mean.size() == 12 && m.x_std.size() == 12,
              "model host weights shapes");
  return m;
}
static rt::NormParams norm_from(const py::dict& d) {
  std::vector<double> norm = d["norm"].cast<std::vector<double>>();
  TORCH_CHECK(norm.size() == 8, "norm must hold 4 scales + 4 shifts");
  rt::NormParams np;
  for (int i = 0; i < 4; ++i) {
    np.scale[i] = (float)norm[i];
    np.shift[i] = (float)norm[4 + i];
  }
  return np;
}
static std::shared_ptr<const rt::NativeModel> model_from(const py::dict& d, int device) {
  const std::string kind = d["kind"].cast<std::string>();
  if (kind == "none") return nullptr;        // predictions relayed to the app (unsupported family)
  std::string err;
  std::shared_ptr<rt::NativeModel> m;
  auto dev_t = [&](const char* k) {
    torch::Tensor t = d[k].cast<torch::Tensor>();
    TORCH_CHECK(t.is_cuda() && t.device().index() == device && t.is_contiguous(), "model tensor ", k,
                " must be contiguous on GPU ", device);
    return t;
  };
  const c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, device));
  if (kind == "mlp3") {
    torch::Tensor blob = dev_t("blob");
    const int H = d["H"].cast<int>();
    TORCH_CHECK(blob.scalar_type() == torch::kUInt8 && (size_t)blob.numel() == rt::eta_mlp3_blob_bytes(H), "mlp3 blob");
    m = rt::make_mlp3_model(device, blob.data_ptr(), (size_t)blob.numel(), H, norm_from(d),
                            d.contains("variant") ? d["variant"].cast<int>() : -1, num_cus(device), mlp_host_from(d),
                            err);
  } else if (kind == "wide") {
    torch::Tensor w1q = dev_t("w1q"), w2f = dev_t("w2f"), b2 = dev_t("b2"), w3 = dev_t("w3");
    const int H = d["H"].cast<int>();
    TORCH_CHECK(b2.scalar_type() == torch::kFloat32 && w3.scalar_type() == torch::kFloat32 && b2.numel() == H &&
                    w3.numel() == H, "wide b2/w3 f32 [H]");
    m = rt::make_wide_model(device, H, w1q.data_ptr(), (size_t)w1q.nbytes(), w2f.data_ptr(), (size_t)w2f.nbytes(),
                            b2.data_ptr<float>(), w3.data_ptr<float>(), d["b3"].cast<float>(), norm_from(d),
                            mlp_host_from(d), err);
  } else if (kind == "forest") {
    rt::ForestHost f;
    torch::Tensor v = d["values"].cast<torch::Tensor>().to(torch::kCPU).contiguous();
    torch::Tensor in = d["info"].cast<torch::Tensor>().to(torch::kCPU).contiguous();
    torch::Tensor r = d["roots"].cast<torch::Tensor>().to(torch::kCPU).contiguous();
    TORCH_CHECK(v.scalar_type() == torch::kFloat32 && in.scalar_type() == torch::kInt32 &&
                    r.scalar_type() == torch::kInt32, "forest arrays f32 / int32 / int32");
    f.values.assign(v.data_ptr<float>(), v.data_ptr<float>() + v.numel());
    f.info.assign((const uint32_t*)in.data_ptr<int>(), (const uint32_t*)in.data_ptr<int>() + in.numel());
    f.roots.assign(r.data_ptr<int>(), r.data_ptr<int>() + r.numel());
    f.base = d["base"].cast<float>();
    f.le = d["le"].cast<bool>();
    std::vector<int> fm = d["fmap"].cast<std::vector<int>>();
    TORCH_CHECK(fm.size() == 12, "fmap: 12 entries");
    for (int j = 0; j < 12; ++j) f.fmap[j] = fm[j];
    m = rt::make_forest_model(device, std::move(f), err);
  } else {
    TORCH_CHECK(false, "unknown native model kind ", kind);
  }
  TORCH_CHECK(m != nullptr, "native model: ", err);
  return m;
}

int64_t native_server_start(int64_t port, int64_t threads, std::vector<int64_t> devices, py::list models,
                            int64_t max_batch, std::vector<std::string> cors, bool cors_vercel, bool bind_any,
                            int64_t upstream_port, py::list routes, std::string history_db) {
  TORCH_CHECK(!devices.empty() && models.size() == devices.size(), "one model spec per GPU slot");
  TORCH_CHECK(max_batch >= 1 && max_batch <= (1 << 24), "max_batch out of range");
  TORCH_CHECK(routes.empty() || routes.size() == devices.size(), "one route config per GPU (or none)");
  std::vector<int> devs;
  std::vector<std::shared_ptr<const rt::NativeModel>> ms;
  for (size_t g = 0; g < devices.size(); ++g) {
    devs.push_back((int)devices[g]);
    ms.push_back(model_from(models[g].cast<py::dict>(), (int)devices[g]));
  }
  std::vector<rt::RouteServiceCfg> rcfg;
  for (size_t g = 0; g < routes.size(); ++g) rcfg.push_back(route_cfg_from(routes[g].cast<py::dict>(), devs[g]));
  std::string err;
  const int64_t h = rt::native_server_start((int)port, (int)threads, devs, ms, (int)max_batch, cors, cors_vercel,
                                            bind_any, (int)upstream_port, rcfg, history_db, err);
  TORCH_CHECK(h >= 0, "native server: ", err);
  return h;
}

int64_t native_server_set_models(int64_t h, std::vector<int64_t> devices, py::list models) {
  TORCH_CHECK(models.size() == devices.size(), "one model spec per GPU slot");
  std::vector<std::shared_ptr<const rt::NativeModel>> ms;
  for (size_t g = 0; g < devices.size(); ++g) ms.push_back(model_from(models[g].cast<py::dict>(), (int)devices[g]));
  std::string err;
  int64_t ep;
  {
    py::gil_scoped_release nogil;
    ep = rt::native_server_set_models(h, ms, err);
  }
  TORCH_CHECK(ep >= 0, "native server: ", err);
  return ep;
}

py::dict native_server_health(int64_t h) {
  uint64_t epoch = 0;
  auto rows = rt::native_server_health(h, epoch);
  py::list slots;
  for (auto& r : rows) {
    py::dict d;
    d["device"] = std::stoi(r[0]);
    d["quarantined"] = r[1] == "1";
    d["consecutive_failures"] = std::stoll(r[2]);
    d["failures"] = std::stoll(r[3]);
    d["rounds"] = std::stoll(r[4]);
    d["quarantines"] = std::stoll(r[5]);
    d["fault_injected"] = r[6] == "1";
    d["model"] = r[7];
    d["deadline_timeouts"] = std::stoll(r[8]);
    d["hang_injected"] = r[9] == "1";
    slots.append(d);
  }
  py::dict out;
  out["model_epoch"] = epoch;
  out["slots"] = slots;
  return out;
}

// ---------------------------------------------------------------- native collectives (comm.hip)
py::bytes comm_unique_id() {
  char id[128];
  TORCH_CHECK(rt::comm_unique_id(id) == 0, "ncclGetUniqueId failed");
  return py::bytes(id, 128);
}

int64_t comm_create(py::bytes uid, int64_t rank, int64_t world, int64_t device, int64_t oneshot_bytes,
                    bool use_rccl) {
  std::string u = uid;
  TORCH_CHECK(!use_rccl || u.size() == 128, "unique id must be 128 bytes");
  u.resize(128);
  std::string err;
  int64_t h;
  {
    py::gil_scoped_release nogil;   // ncclCommInitRank blocks until every rank joined
    h = rt::comm_create(u.data(), (int)rank, (int)world, (int)device, (size_t)oneshot_bytes, use_rccl, err);
  }
  TORCH_CHECK(h >= 0, "comm_create: ", err);
  return h;
}

py::bytes comm_ipc_handles(int64_t h) {
  std::string out(rt::comm_ipc_handle_bytes(), '\0');
  const int r = rt::comm_ipc_handles(h, out.data());
  TORCH_CHECK(r == 0, "hipIpcGetMemHandle failed (", r, ")");
  return py::bytes(out);
}

void comm_open_peers(int64_t h, std::vector<py::bytes> handles) {
  std::vector<std::string> hs(handles.begin(), handles.end());
  std::string err;
  TORCH_CHECK(rt::comm_open_peers(h, hs, err) == 0, "comm_open_peers: ", err);
}

void comm_all_reduce(int64_t h, torch::Tensor t, int64_t algo) {
  check_dev(t, "all_reduce tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, "all_reduce: float32 buckets only");
  const c10::DeviceGuard guard(t.device());
  std::string err;
  const hipError_t e = rt::comm_all_reduce_f32(h, t.data_ptr<float>(), (size_t)t.numel(), (int)algo, cur_stream(t), err);
  TORCH_CHECK(e == hipSuccess, "comm_all_reduce: ", err.empty() ? hipGetErrorString(e) : err);
}

// one-shot all-gather (op 0) / broadcast (op 2) over the IPC-mapped peer buffers; any dtype
void comm_oneshot(int64_t h, int64_t op, torch::Tensor in, torch::Tensor out, int64_t root) {
  check_dev(in, "input");
  check_dev(out, "output");
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "one-shot: contiguous tensors only");
  TORCH_CHECK(in.scalar_type() == out.scalar_type(), "dtype mismatch");
  const c10::DeviceGuard guard(in.device());
  std::string err;
  const size_t bytes = (size_t)in.numel() * in.element_size();
  const int world = rt::comm_world(h);
  TORCH_CHECK(world >= 1, "bad comm handle");
  hipError_t e;
  if (op == 0) {
    TORCH_CHECK(out.numel() == in.numel() * world, "all_gather: out must hold world x input");
    e = rt::comm_all_gather_oneshot(h, in.data_ptr(), out.data_ptr(), bytes, cur_stream(in), err);
  } else {
    TORCH_CHECK(in.data_ptr() == out.data_ptr(), "one-shot broadcast is in place");
    e = rt::comm_broadcast_oneshot(h, in.data_ptr(), bytes, (int)root, cur_stream(in), err);
  }
  TORCH_CHECK(e == hipSuccess, "comm_oneshot: ", err.empty() ? hipGetErrorString(e) : err);
}

int dtype_code(const torch::Tensor& t) {
  if (t.scalar_type() == torch::kFloat32) return 0;
  if (t.scalar_type() == torch::kBFloat16) return 1;
  if (t.scalar_type() == torch::kInt32) return 2;
  TORCH_CHECK(false, "collective dtype must be float32, bfloat16 or int32");
  return -1;
}

void comm_collective(int64_t h, int64_t op, torch::Tensor in, torch::Tensor out, int64_t root) {
  check_dev(in, "input");
  check_dev(out, "output");
  TORCH_CHECK(in.scalar_type() == out.scalar_type(), "dtype mismatch");
  const c10::DeviceGuard guard(in.device());
  std::string err;
  // counts are per-rank for all_gather / reduce_scatter (nccl convention)
  const size_t count = op == 0 ? (size_t)in.numel() : (op == 1 ? (size_t)out.numel() : (size_t)in.numel());
  TORCH_CHECK(rt::comm_nccl_call(h, (int)op, in.data_ptr(), out.data_ptr(), count, dtype_code(in), (int)root,
                                 cur_stream(in), err) == 0, "RCCL collective: ", err);
}

// LDS-staged tree ensemble: nodes2 int32 [M,2] = (value bits, info), chunks int32 [C+1,2]
torch::Tensor forest_predict_lds(torch::Tensor records, torch::Tensor nodes2, torch::Tensor roots,
                                 torch::Tensor chunks, double base, bool le, std::vector<int64_t> fmap) {
  for (auto* t : {&records, &nodes2, &roots, &chunks}) check_dev(*t, "forest tensor");
  TORCH_CHECK(records.scalar_type() == torch::kInt32 && records.dim() == 2 && records.size(1) == 4,
              "records must be int32 [B,4]");
  TORCH_CHECK(nodes2.scalar_type() == torch::kInt32 && nodes2.dim() == 2 && nodes2.size(1) == 2, "nodes2 int32 [M,2]");
  TORCH_CHECK(chunks.scalar_type() == torch::kInt32 && chunks.dim() == 2 && chunks.size(1) == 2 &&
              chunks.size(0) >= 2, "chunks int32 [C+1,2]");
  TORCH_CHECK(roots.scalar_type() == torch::kInt32, "roots int32");
  TORCH_CHECK(fmap.size() == 12, "fmap must have 12 entries");
  const c10::DeviceGuard guard(records.device());
  const int B = (int)records.size(0);
  auto out = torch::empty({B}, records.options().dtype(torch::kFloat32));
  int fm[12];
  for (int j = 0; j < 12; ++j) fm[j] = (int)fmap[j];
  RT_CHECK_HIP(rt::launch_forest_lds(records.data_ptr(), nodes2.data_ptr(), roots.data_ptr<int>(),
                                     chunks.data_ptr<int>(), (int)chunks.size(0) - 1, out.data_ptr<float>(), B,
                                     (int)roots.numel(), (int)nodes2.size(0), (float)base, le ? 1 : 0, fm,
                                     num_cus(records.device().index()), cur_stream(records)));
  return out;
}

}  // namespace

void bind_cch_gpu(py::module& m);   // cch_bindings.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "routest_amd native gfx950 kernels";
  bind_cch_gpu(m);
  m.def("eta_mlp3_forward", &eta_mlp3_forward, "fused featurize + 3-layer MLP forward (bf16 MFMA)");
  m.def("eta_mlp3_forward_hostio", &eta_mlp3_forward_hostio,
        "zero-copy: fused kernel reads records / writes minutes in pinned host memory");
  m.def("pinned_host_empty", &pinned_host_empty, "registered pinned host buffer (optionally THP-backed)",
        py::arg("nbytes"), py::arg("huge") = true);
  m.def("eta_featurize", &eta_featurize,"K1: packed records -> R16 features [B,12] fp32");
  m.def("eta_mlp3_blob_bytes", [](int64_t H) { return (int64_t)rt::eta_mlp3_blob_bytes((int)H); });
  m.def("eta_mlp3_blob16_bytes", [](int64_t H) { return (int64_t)rt::eta_mlp3_blob16_bytes((int)H); });
  m.def("route_haversine_matrix", &route_haversine_matrix, "K5: batched haversine matrices (f64)");
  m.def("route_greedy_cvrp", &route_greedy_cvrp, "K6: batched greedy multi-trip CVRP");
  m.def("big_layer1", &big_layer1, "wide MLP: featurize + layer 1 -> h1 (hperm order)",
        py::arg("records"), py::arg("w1p"), py::arg("H"), py::arg("norm"), py::arg("h1"),
        py::arg("xf") = py::none(), py::arg("mbits") = py::none());
  m.def("big_fused", &big_fused, "wide MLP inference: featurize + layer 1 + layer 2 + relu.w3 partials, one launch");
  m.def("gemm_dgrad_dw1", &gemm_dgrad_dw1, "training dgrad with the dW1 partials in its epilogue (dh1 not stored)");
  m.def("gemm_nt", &gemm_nt, "wide MLP layer GEMM Z^T = W X^T with fused epilogues (0 y-partials, 1 +h2, 2 store)",
        py::arg("epi"), py::arg("W"), py::arg("X"), py::arg("N"), py::arg("M"), py::arg("K"),
        py::arg("b2") = py::none(), py::arg("w3") = py::none(), py::arg("ypart") = py::none(),
        py::arg("out") = py::none());
  m.def("gemm_pipe", [](int64_t set) { return (int64_t)rt::gemm_pipe_mode((int)set); },
        "wide GEMM K loop: 1 phase pipeline, 0 one drain per K-tile; set < 0 only reads", py::arg("set") = -1);
  m.def("big_yreduce", &big_yreduce, "y = sum of partials + b3 (+ dy, dy operand, squared error)",
        py::arg("ypart"), py::arg("nparts"), py::arg("b3"), py::arg("y") = py::none(),
        py::arg("target") = py::none(), py::arg("gscale") = 0.0, py::arg("dy") = py::none(),
        py::arg("dyb") = py::none(), py::arg("sq_err") = py::none(), py::arg("b3_dev") = py::none());
  m.def("adamw_pack_big", &adamw_pack_big, "wide trainer: AdamW + re-pack of w1p / w2k / w2t / b2 / w3 / b3");
  m.def("big_dz2y", &big_dz2y,
        "wide trainer: dy, dyb, squared error, dz2 and the step counter in one launch (+ dW3|db3 slab rows)",
        py::arg("ypart"), py::arg("nparts"), py::arg("b3"), py::arg("target"), py::arg("gscale"), py::arg("dy"),
        py::arg("dyb"), py::arg("sq_err"), py::arg("h2a"), py::arg("w3"), py::arg("H"), py::arg("dz2"),
        py::arg("step_ctr"), py::arg("slab") = py::none());
  m.def("big_dz2", &big_dz2, "dz2 = dy * w3 * relu'(z2) from h2a (hperm order)");
  m.def("eta_mlp3_train_fwd", &eta_mlp3_train_fwd, "K3: fused featurize+MLP forward (one pass over layer 2) + MSE grad + dW3 partial -> dz2 fragments");
  m.def("train_bwd", &train_bwd, "K3: dgrad + relu'(z1) + dW2|db2 and dW1 split-K partials in one kernel (train_bwd_kernel)");
  m.def("train_wgrad_slices", [](int64_t B, int64_t device, int64_t H) {
    return (int64_t)rt::train_wgrad_slices((int)B, num_cus((int)device), (int)H);
  }, py::arg("B"), py::arg("device"), py::arg("H") = 256);
  m.def("adamw_pack", &adamw_pack, "fused AdamW on flat fp32 params + training-blob re-pack");
  m.def("reduce_adamw", &reduce_adamw, "one-rank fused slab reduction + AdamW + blob re-pack");
  m.def("eta_mlp3_train_blob_bytes", [](int64_t H) { return (int64_t)rt::eta_mlp3_train_blob_bytes((int)H); });
  m.def("mlp3_num_params", [](int64_t H) { return (int64_t)rt::mlp3_num_params((int)H); });
  m.def("mlp3_grad_bucket_floats", [](int64_t H) { return (int64_t)rt::mlp3_grad_bucket_floats((int)H); });
  m.def("wgrad", &wgrad, "split-K weight-gradient GEMM (K = batch) into fp32 slabs",
        py::arg("A"), py::arg("M"), py::arg("Mout"), py::arg("Bm"), py::arg("N"), py::arg("slab"),
        py::arg("offset"), py::arg("ldo"), py::arg("mask") = py::none(), py::arg("nout") = -1, py::arg("mask_hperm") = false,
        py::arg("nsplit") = 1);
  m.def("wgrad_dual", &wgrad_dual, "two split-K weight-gradient GEMMs (dW2|db2 and dW1) in one launch");
  m.def("wgrad_reduce", &wgrad_reduce, "deterministic sum of wgrad slabs (optionally a second and third region)",
        py::arg("slab"), py::arg("G"), py::arg("slab1") = py::none(), py::arg("G1") = py::none(),
        py::arg("slab2") = py::none(), py::arg("G2") = py::none(), py::arg("perm_h") = 0, py::arg("fold_ld") = 0,
        py::arg("fold_col") = 0);
  m.def("wgrad256", &wgrad256, "dW2-shaped weight gradient on 256x256 output tiles, split-K over the slab's rows",
        py::arg("A"), py::arg("B"), py::arg("M"), py::arg("N"), py::arg("slab"), py::arg("ldo"), py::arg("db2_col") = -1);
  m.def("train_fwd_grid", [](int64_t B, int64_t dev) { return (int64_t)rt::train_fwd_grid((int)B, num_cus((int)dev)); },
        "workgroups of the training forward = rows of its dW3 slab");
  m.def("num_cus", [](int64_t dev) { return (int64_t)num_cus((int)dev); });
  m.def("gcn_agg_gemm", &gcn_agg_gemm, "K8: fused CSR aggregation + MFMA GEMM + bias/ReLU");
  m.def("gcn_l1_fused", &gcn_l1_fused, "K8: fused aggregation + W1 GEMM + ReLU + W2 transform (H1 stays in LDS)");
  m.def("gcn_spmm_score", &gcn_spmm_score, "K8: layer-2 aggregation + delay head");
  m.def("route_score", &route_score, "K8: per-route delay-weighted length");
  m.def("astar_search", &astar_search, "K9: tiered batched A* (lane -> wave -> big tier) with learned edge costs",
        py::arg("indptr"), py::arg("indices"), py::arg("cost"), py::arg("lat"), py::arg("lon"), py::arg("inv_vmax"),
        py::arg("landmarks"), py::arg("src"), py::arg("dst"), py::arg("lane"), py::arg("wave"), py::arg("big"),
        py::arg("out_cost"), py::arg("out_len"), py::arg("out_status"), py::arg("out_path"), py::arg("out_iters"),
        py::arg("scratch"), py::arg("max_iters"), py::arg("lane_pops"), py::arg("wave_only_below"),
        py::arg("delta"), py::arg("arena") = py::none(), py::arg("arena_ctr") = py::none(),
        py::arg("lane_max_m") = -1.0, py::arg("wave_nw") = 0, py::arg("retry_nw") = 0);
  m.def("forest_predict", &forest_predict, "K4: fused featurize + tree-ensemble inference");
  m.def("forest_predict_lds", &forest_predict_lds, "K4: LDS-staged tree chunks, 2 walks per thread");
  m.def("pscore_create", &pscore_create, "resident single-request scorer kernel on the blob's GPU");
  m.def("pscore_score", &pscore_score, "score n <= cap records on the resident scorer (False: not answered)");
  m.def("pscore_park", [](int64_t h) {
    rt::PersistentScorer* p = ps_get(h);
    py::gil_scoped_release nogil;
    rt::pscore_park(p);
  });
  m.def("pscore_stats", [](int64_t h) {
    long long l, s, f;
    rt::pscore_stats(ps_get(h), &l, &s, &f);
    return std::vector<int64_t>{l, s, f};
  });
  m.def("pscore_destroy", [](int64_t h) {
    rt::PersistentScorer* p = nullptr;
    {
      std::lock_guard<std::mutex> lk(g_ps_mu);
      if (h < 0 || h >= (int64_t)g_ps.size()) return;
      p = g_ps[h];
      g_ps[h] = nullptr;
    }
    py::gil_scoped_release nogil;
    rt::pscore_destroy(p);
  });
  m.def("gcn_train_bwd", &gcn_train_bwd, "GCN scorer backward over a row range -> flat gradient + loss");
  m.def("gcn_grad_numel", []() { return (int64_t)rt::gcn_grad_numel(); });
  m.def("gcn_train_slab2_rows", [](int64_t n) { return (int64_t)rt::gcn_train_slab2_rows((int)n); });
  m.def("native_server_start", &native_server_start, "native HTTP front end (predictions, routes, relay)",
        py::arg("port"), py::arg("threads"), py::arg("devices"), py::arg("models"), py::arg("max_batch"),
        py::arg("cors"), py::arg("cors_vercel"), py::arg("bind_any"), py::arg("upstream_port") = 0,
        py::arg("routes") = py::list(), py::arg("history_db") = "");
  m.def("native_server_set_models", &native_server_set_models,
        "hot-swap the served models (one spec per GPU slot); returns the new epoch");
  m.def("native_server_set_fault", [](int64_t h, int64_t slot, bool on) {
    return rt::native_server_set_fault(h, (int)slot, on);
  });
  m.def("native_server_set_hang", [](int64_t h, int64_t slot, bool on) {
    return rt::native_server_set_hang(h, (int)slot, on);
  }, "latency-watchdog fault hook: launches on the slot first wait on a host flag");
  m.def("native_server_set_scorer", [](int64_t h, std::vector<double> delay, int64_t kind, std::string engine) {
    return rt::native_server_set_scorer(h, std::move(delay), (int)kind, engine);
  }, "publish the GCN scorer's node delays for native \"alternatives\" requests");
  m.def("native_server_health", &native_server_health, "per-GPU-slot health, models and the model epoch");
  m.def("native_server_stop", [](int64_t h) {
    py::gil_scoped_release nogil;
    rt::native_server_stop(h);
  });
  m.def("native_server_stats", [](int64_t h) {
    const auto v = rt::native_server_stats(h);
    return std::vector<int64_t>(v.begin(), v.end());
  });
  m.def("comm_unique_id", &comm_unique_id, "RCCL unique id (128 bytes) for comm_create");
  m.def("comm_create", &comm_create, "own RCCL communicator + one-shot IPC buffers");
  m.def("comm_ipc_handles", &comm_ipc_handles, "IPC handles of this rank's one-shot buffers");
  m.def("comm_open_peers", &comm_open_peers, "map every peer's one-shot buffers (xGMI)");
  m.def("comm_all_reduce", &comm_all_reduce, "in-place SUM all-reduce on the current stream (0=rccl, 1=oneshot)");
  m.def("comm_collective", &comm_collective, "RCCL all_gather(0)/reduce_scatter(1)/broadcast(2)/all_reduce(3)");
  m.def("comm_oneshot", &comm_oneshot, "one-shot IPC all_gather(0)/broadcast(2) on the current stream");
  m.def("comm_error", [](int64_t h) { return (int64_t)rt::comm_error(h); });
  m.def("comm_destroy", [](int64_t h) { rt::comm_destroy(h); });
  m.def("rccl_version", []() { return (int64_t)rt::comm_rccl_version(); });
  m.attr("ARCH") = "gfx950";
}
