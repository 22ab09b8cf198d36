// torch bindings of the GPU customizable contraction hierarchy (csrc/cch.hip): routest_amd._C.CchGpu.
// routing/cch.py wraps it (context cache, CPU fallback); the native route service
// (csrc/route_service.hip) takes the same object through `ptr()`.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <chrono>
#include <memory>
#include <mutex>
#include <unordered_map>

#include "cch_gpu.h"
#include "ops.h"

namespace py = pybind11;

namespace {

#define CCH_CHECK_HIP(expr)                                                            \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    TORCH_CHECK(_e == hipSuccess, "HIP error in ", #expr, ": ", hipGetErrorString(_e)); \
  } while (0)

hipStream_t stream_of(int dev) { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(dev).stream(); }

template <class T>
const T* host_ptr(const torch::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(!t.is_cuda() && t.is_contiguous() && t.numel() == n, name, ": contiguous CPU tensor of ", n);
  return t.data_ptr<T>();
}

class PyCchGpu {
 public:
  PyCchGpu(torch::Tensor indptr, torch::Tensor indices, torch::Tensor lat, torch::Tensor lon, torch::Tensor length,
           torch::Tensor road_class, torch::Tensor base_traffic, int64_t device) {
    TORCH_CHECK(indptr.scalar_type() == torch::kInt32 && indices.scalar_type() == torch::kInt32 &&
                    lat.scalar_type() == torch::kFloat64 && lon.scalar_type() == torch::kFloat64 &&
                    length.scalar_type() == torch::kFloat32 && road_class.scalar_type() == torch::kUInt8 &&
                    base_traffic.scalar_type() == torch::kUInt8,
                "CchGpu: indptr/indices int32, lat/lon float64, length float32, road_class/base_traffic uint8");
    const int64_t N = lat.numel();
    const int32_t* ip = host_ptr<int32_t>(indptr, N + 1, "indptr");
    const int64_t E = ip[N];
    const int32_t* ix = host_ptr<int32_t>(indices, E, "indices");
    for (int64_t e = 0; e < E; ++e) TORCH_CHECK(ix[e] >= 0 && ix[e] < N, "edge target out of range");
    for (int64_t v = 0; v < N; ++v) TORCH_CHECK(ip[v] <= ip[v + 1], "indptr not monotone");
    auto t0 = std::chrono::steady_clock::now();
    rcch::Topology T;
    {
      py::gil_scoped_release nogil;
      T = rcch::build_topology((int)N, ip, ix, host_ptr<double>(lat, N, "lat"), host_ptr<double>(lon, N, "lon"));
    }
    build_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    dev_ = (int)device;
    g_ = std::make_unique<rt::CchGpu>(std::move(T), host_ptr<float>(length, E, "length"),
                                      host_ptr<uint8_t>(road_class, E, "road_class"),
                                      host_ptr<uint8_t>(base_traffic, E, "base_traffic"), dev_);
    sc_ = std::make_unique<rt::CchScratch>();
  }

  void set_eta(torch::Tensor blob, int64_t H, std::vector<double> norm, int64_t variant) {
    TORCH_CHECK(blob.is_cuda() && blob.device().index() == dev_ && blob.scalar_type() == torch::kUInt8,
                "blob: uint8 on the router's GPU");
    TORCH_CHECK((size_t)blob.numel() == rt::eta_mlp3_blob_bytes((int)H), "blob size for H=", H);
    TORCH_CHECK(norm.size() == 8, "norm: 4 scales + 4 shifts");
    rt::NormParams np;
    for (int i = 0; i < 4; ++i) {
      np.scale[i] = (float)norm[i];
      np.shift[i] = (float)norm[4 + i];
    }
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_);
    blob_ = blob;
    g_->set_eta(blob_.data_ptr(), (int)H, np, (int)variant, cus);
  }

  py::dict stats() const {
    const rcch::Topology& T = g_->topo();
    py::dict d;
    d["nodes"] = T.N;
    d["arcs"] = T.M;
    d["edges"] = T.E;
    d["max_depth"] = T.max_depth;
    d["max_height"] = T.max_height;
    d["top_separator"] = T.separator_top;
    d["build_ms"] = build_ms_;
    d["cached_metrics"] = g_->cached();
    d["triangle_table"] = g_->has_triangle_table();
    d["triangles"] = g_->triangles();
    d["basic_tasks"] = g_->basic_tasks();
    d["basic_tail_levels"] = g_->basic_tail_levels();
    d["perfect_tail_levels"] = g_->perfect_tail_levels();
    d["perfect_tasks"] = g_->perfect_tasks();
    d["supernodal"] = g_->supernodal();
    d["sup_fronts"] = g_->sup_fronts();
    d["sup_nodes"] = g_->sup_nodes();
    d["sup_levels"] = g_->sup_levels();
    d["sup_blocks"] = g_->sup_blocks();
    d["sparse_heights"] = g_->sparse_heights();
    d["sparse_depths"] = g_->sparse_depths();
    d["cache_capacity"] = g_->capacity();
    d["cache_gb"] = g_->cache_gb();
    d["metric_bytes"] = g_->metric_bytes();
    const auto a = g_->async_stats();
    d["async_queued"] = a.queued;
    d["async_built"] = a.built;
    d["async_failed"] = a.failed;
    d["async_pending"] = a.pending;
    d["async_build_ms"] = a.build_ms;
    d["async_alloc_ms"] = a.alloc_ms;
    d["async_hostcopy_ms"] = a.hostcopy_ms;
    d["builder_max_wg"] = g_->builder_pacing();
    d["async_paced"] = a.paced;
    return d;
  }

  // queue a context's build on the router's background builder (returns at once)
  void request_build(int64_t weather, int64_t congestion, int64_t weekhour, double age, bool urgent) {
    TORCH_CHECK(g_->has_eta(), "CchGpu: set_eta first");
    rt::CchContext c;
    c.weather = (int)weather;
    c.congestion = (int)congestion;
    c.weekhour = (int)weekhour;
    c.driver_age = (float)age;
    g_->request_build(c, urgent);
  }
  bool is_cached(int64_t key) {
    std::shared_ptr<rt::CchMetricDev> m;
    return g_->cached_metric((uint64_t)key, m);
  }
  void set_cache_gb(double gb) { g_->set_cache_gb(gb); }
  void set_builder_pacing(int n, bool always) { g_->set_builder_pacing(n, always); }

  py::dict info(const rt::CchMetricDev& m, bool fresh) const {
    py::dict d;
    d["key"] = m.key;
    d["fresh"] = fresh;
    d["cost_ms"] = m.cost_ms;
    d["customize_ms"] = m.customize_ms;
    d["basic_ms"] = m.basic_ms;
    d["perfect_ms"] = m.perfect_ms;
    d["prune_ms"] = m.prune_ms;
    d["kept_f"] = m.kept_f;
    d["kept_b"] = m.kept_b;
    return d;
  }

  // metric of a routing context (built on first use, then cached on the GPU).  pin: also hold it
  // outside the LRU until unpin(key) — a caller that customizes several contexts and then queries
  // them (a flush with more contexts than the cache holds) cannot lose one to eviction in between
  py::dict metric_for(int64_t weather, int64_t congestion, int64_t weekhour, double age, bool pin) {
    TORCH_CHECK(g_->has_eta(), "CchGpu: set_eta first");
    rt::CchContext c;
    c.weather = (int)weather;
    c.congestion = (int)congestion;
    c.weekhour = (int)weekhour;
    c.driver_age = (float)age;
    const c10::DeviceGuard guard(c10::Device(c10::DeviceType::CUDA, dev_));
    std::shared_ptr<rt::CchMetricDev> m;
    bool fresh = false;
    hipError_t e;
    {
      py::gil_scoped_release nogil;
      e = g_->metric_for(c, stream_of(dev_), m, &fresh);
    }
    CCH_CHECK_HIP(e);
    if (pin) pin_ptr(m);
    return info(*m, fresh);
  }

  void unpin(int64_t key) {
    std::lock_guard<std::mutex> lk(pin_mu_);
    auto it = pins_.find((uint64_t)key);
    if (it != pins_.end() && --it->second.second <= 0) pins_.erase(it);
  }
  int64_t pinned() {
    std::lock_guard<std::mutex> lk(pin_mu_);
    return (int64_t)pins_.size();
  }

  py::dict metric_from_costs(int64_t key, torch::Tensor cost) {
    TORCH_CHECK(cost.is_cuda() && cost.device().index() == dev_ && cost.scalar_type() == torch::kFloat32 &&
                    cost.is_contiguous() && cost.numel() == g_->topo().E,
                "cost: float32 [E] on the router's GPU");
    // weights are ordered by their float bits (cch.h pack_w, atomicMin on the bits): NaN, negative
    // costs and -0.0 would sort above every real weight and drop the edge — reject / normalise
    TORCH_CHECK(torch::isfinite(cost).all().item<bool>() && (cost >= 0).all().item<bool>(),
                "edge costs must be finite and >= 0");
    cost = cost.add(0.0);                       // -0.0 -> +0.0
    const c10::DeviceGuard guard(cost.device());
    std::shared_ptr<rt::CchMetricDev> m;
    hipError_t e;
    {
      py::gil_scoped_release nogil;
      e = g_->metric_from_costs((uint64_t)key, cost.data_ptr<float>(), stream_of(dev_), m);
    }
    CCH_CHECK_HIP(e);
    return info(*m, true);
  }

  // device copies of a cached metric's arrays (tests: two customization paths must agree bit for bit)
  py::dict metric_dump(int64_t key) {
    auto m = get(key);
    const int64_t M = g_->topo().M, N = g_->topo().N;
    const auto opt = torch::TensorOptions().device(torch::kCUDA, dev_);
    const c10::DeviceGuard guard(opt.device());
    py::dict d;
    auto put = [&](const char* name, const void* src, int64_t n, torch::ScalarType t) {
      auto out = torch::empty({n}, opt.dtype(t));
      if (n > 0)
        CCH_CHECK_HIP(hipMemcpyAsync(out.data_ptr(), src, n * out.element_size(), hipMemcpyDeviceToDevice, stream_of(dev_)));
      d[name] = out;
    };
    put("sub_up", m->sub_up, 2 * M, torch::kInt32);
    put("sub_dn", m->sub_dn, 2 * M, torch::kInt32);
    put("len_up", m->len_up, M, torch::kFloat32);
    put("len_dn", m->len_dn, M, torch::kFloat32);
    put("cnt_up", m->cnt_up, M, torch::kInt32);
    put("cnt_dn", m->cnt_dn, M, torch::kInt32);
    put("f_ptr", m->f_ptr, N + 1, torch::kInt32);
    put("b_ptr", m->b_ptr, N + 1, torch::kInt32);
    put("f_rec", m->f_rec, 4 * m->kept_f, torch::kInt32);
    put("b_rec", m->b_rec, 4 * m->kept_b, torch::kInt32);
    return d;
  }

  torch::Tensor costs(int64_t key) {
    auto m = get(key);
    auto out = torch::empty({(int64_t)g_->topo().E},
                            torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, dev_));
    const c10::DeviceGuard guard(out.device());
    CCH_CHECK_HIP(hipMemcpyAsync(out.data_ptr<float>(), m->cost, g_->topo().E * 4, hipMemcpyDeviceToDevice,
                                 stream_of(dev_)));
    return out;
  }

  // (sec, metres, status, len, path) for node-id pairs (CUDA int32 tensors)
  py::tuple route(int64_t key, torch::Tensor src, torch::Tensor dst, int64_t max_path, bool want_path) {
    auto m = get(key);
    TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.device().index() == dev_ && dst.device().index() == dev_ &&
                    src.scalar_type() == torch::kInt32 && dst.scalar_type() == torch::kInt32 &&
                    src.is_contiguous() && dst.is_contiguous() && src.numel() == dst.numel(),
                "src/dst: int32 [Q] on the router's GPU");
    const int64_t Q = src.numel();
    const int N = g_->topo().N;
    if (Q > 0) {
      const auto mn = torch::minimum(src.min(), dst.min()).item<int>();
      const auto mx = torch::maximum(src.max(), dst.max()).item<int>();
      TORCH_CHECK(mn >= 0 && mx < N, "node id out of range");
    }
    auto o32 = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, dev_);
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, dev_);
    auto sec = torch::empty({Q}, of), met = torch::empty({Q}, of);
    auto st = torch::empty({Q}, o32), len = torch::zeros({Q}, o32);
    auto path = want_path ? torch::empty({Q, max_path}, o32) : torch::empty({0, max_path}, o32);
    rt::CchRouteOut o;
    o.sec = sec.data_ptr<float>();
    o.metres = met.data_ptr<float>();
    o.status = st.data_ptr<int>();
    o.len = len.data_ptr<int>();
    o.path = want_path ? path.data_ptr<int>() : nullptr;
    o.max_path = (int)max_path;
    const c10::DeviceGuard guard(src.device());
    std::lock_guard<std::mutex> lk(mu_);
    CCH_CHECK_HIP(g_->route(*m, src.data_ptr<int>(), dst.data_ptr<int>(), (int)Q, o, *sc_, stream_of(dev_)));
    return py::make_tuple(sec, met, st, len, path);
  }

  // per-request matrices: pts int32 [R, NM] node ids, npts int32 [R] -> (sec, metres) [R, NM, NM]
  py::tuple matrix(int64_t key, torch::Tensor pts, torch::Tensor npts) {
    auto m = get(key);
    TORCH_CHECK(pts.is_cuda() && npts.is_cuda() && pts.dim() == 2 && pts.scalar_type() == torch::kInt32 &&
                    npts.scalar_type() == torch::kInt32 && npts.numel() == pts.size(0) && pts.is_contiguous(),
                "pts int32 [R, NM], npts int32 [R] on the router's GPU");
    const int R = (int)pts.size(0), NM = (int)pts.size(1);
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, dev_);
    auto sec = torch::empty({R, NM, NM}, of), met = torch::empty({R, NM, NM}, of);
    const c10::DeviceGuard guard(pts.device());
    std::lock_guard<std::mutex> lk(mu_);
    CCH_CHECK_HIP(g_->matrix(*m, pts.data_ptr<int>(), npts.data_ptr<int>(), R, NM, sec.data_ptr<float>(),
                             met.data_ptr<float>(), nullptr, *sc_, stream_of(dev_)));
    return py::make_tuple(sec, met);
  }

  // matrix() that also returns the tag of its chains (kept for legs_from_matrix until the next call)
  py::tuple matrix_keep(int64_t key, torch::Tensor pts, torch::Tensor npts) {
    auto sm = matrix(key, pts, npts);
    std::lock_guard<std::mutex> lk(mu_);
    return py::make_tuple(sm[0], sm[1], (uint64_t)sc_->chain_tag);
  }

  // legs (r, i, j) between points of the matrix_keep() call `tag` (pts as given to it): its chains
  // are reused, so only the meet + unpack launches run -> (sec, metres, status, len, path)
  py::tuple legs_from_matrix(int64_t key, uint64_t tag, torch::Tensor pts, torch::Tensor r, torch::Tensor i,
                             torch::Tensor j, int64_t max_path, bool want_path) {
    auto m = get(key);
    for (const torch::Tensor* t : {&pts, &r, &i, &j})
      TORCH_CHECK(t->is_cuda() && t->device().index() == dev_ && t->scalar_type() == torch::kInt32 && t->is_contiguous(),
                  "pts / r / i / j: int32 on the router's GPU");
    TORCH_CHECK(pts.dim() == 2 && r.numel() == i.numel() && r.numel() == j.numel(), "pts [R, NM]; r, i, j [Q]");
    const int64_t Q = r.numel();
    const int R = (int)pts.size(0), NM = (int)pts.size(1);
    if (Q > 0) {
      TORCH_CHECK(r.min().item<int>() >= 0 && r.max().item<int>() < R, "leg request index out of range");
      TORCH_CHECK(torch::minimum(i.min(), j.min()).item<int>() >= 0 && torch::maximum(i.max(), j.max()).item<int>() < NM,
                  "leg point index out of range");
    }
    auto o32 = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, dev_);
    auto of = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, dev_);
    auto sec = torch::empty({Q}, of), met = torch::empty({Q}, of);
    auto st = torch::empty({Q}, o32), len = torch::zeros({Q}, o32);
    auto path = want_path ? torch::empty({Q, max_path}, o32) : torch::empty({0, max_path}, o32);
    rt::CchRouteOut o;
    o.sec = sec.data_ptr<float>();
    o.metres = met.data_ptr<float>();
    o.status = st.data_ptr<int>();
    o.len = len.data_ptr<int>();
    o.path = want_path ? path.data_ptr<int>() : nullptr;
    o.max_path = (int)max_path;
    const c10::DeviceGuard guard(pts.device());
    auto src = Q > 0 ? pts.index({r.to(torch::kLong), i.to(torch::kLong)}).contiguous() : torch::empty({0}, o32);
    std::lock_guard<std::mutex> lk(mu_);
    TORCH_CHECK(tag != 0 && tag == sc_->chain_tag && sc_->chain_nm == NM && sc_->chain_r == R,
                "legs_from_matrix: the matrix chains of this tag are gone (another call ran since)");
    CCH_CHECK_HIP(g_->legs_from_matrix(*m, src.data_ptr<int>(), r.data_ptr<int>(), i.data_ptr<int>(), j.data_ptr<int>(),
                                       (int)Q, tag, o, *sc_, stream_of(dev_)));
    return py::make_tuple(sec, met, st, len, path);
  }

  void set_capacity(int64_t n) { g_->set_capacity((int)n); }
  uintptr_t ptr() const { return reinterpret_cast<uintptr_t>(g_.get()); }
  py::dict topology_arrays() const {
    const rcch::Topology& T = g_->topo();
    py::dict d;
    auto i32 = [](const std::vector<int32_t>& v) {
      auto t = torch::empty({(int64_t)v.size()}, torch::kInt32);
      if (!v.empty()) std::memcpy(t.data_ptr<int32_t>(), v.data(), v.size() * 4);
      return t;
    };
    d["rank"] = i32(T.rank);
    d["parent"] = i32(T.parent);
    d["depth"] = i32(T.depth);
    d["up_head"] = i32(T.up_head);
    return d;
  }

 private:
  void pin_ptr(const std::shared_ptr<rt::CchMetricDev>& m) {
    std::lock_guard<std::mutex> lk(pin_mu_);
    auto& p = pins_[m->key];
    p.first = m;
    ++p.second;
  }

  std::shared_ptr<rt::CchMetricDev> get(int64_t key) {
    std::shared_ptr<rt::CchMetricDev> m;
    if (g_->cached_metric((uint64_t)key, m)) return m;
    {
      std::lock_guard<std::mutex> lk(pin_mu_);
      auto it = pins_.find((uint64_t)key);
      if (it != pins_.end()) return it->second.first;
    }
    TORCH_CHECK(false, "CchGpu: no cached metric for key ", key, " (evicted or never built)");
    return m;
  }

  std::mutex pin_mu_;
  std::unordered_map<uint64_t, std::pair<std::shared_ptr<rt::CchMetricDev>, int>> pins_;

  std::unique_ptr<rt::CchGpu> g_;
  std::unique_ptr<rt::CchScratch> sc_;
  std::mutex mu_;
  torch::Tensor blob_;
  int dev_ = 0;
  double build_ms_ = 0.0;
};

}  // namespace

void bind_cch_gpu(py::module& m) {
  py::class_<PyCchGpu>(m, "CchGpu")
      .def(py::init<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
                    torch::Tensor, int64_t>(),
           py::arg("indptr"), py::arg("indices"), py::arg("lat"), py::arg("lon"), py::arg("length"),
           py::arg("road_class"), py::arg("base_traffic"), py::arg("device"))
      .def("set_eta", &PyCchGpu::set_eta, py::arg("blob"), py::arg("H"), py::arg("norm"), py::arg("variant") = -1)
      .def("stats", &PyCchGpu::stats)
      .def("metric_for", &PyCchGpu::metric_for, py::arg("weather"), py::arg("congestion"), py::arg("weekhour"),
           py::arg("driver_age") = 35.0, py::arg("pin") = false)
      .def("unpin", &PyCchGpu::unpin, py::arg("key"))
      .def("pinned", &PyCchGpu::pinned)
      .def("metric_from_costs", &PyCchGpu::metric_from_costs, py::arg("key"), py::arg("cost"))
      .def("costs", &PyCchGpu::costs, py::arg("key"))
      .def("metric_dump", &PyCchGpu::metric_dump, py::arg("key"))
      .def("route", &PyCchGpu::route, py::arg("key"), py::arg("src"), py::arg("dst"), py::arg("max_path") = 4096,
           py::arg("want_path") = true)
      .def("matrix", &PyCchGpu::matrix, py::arg("key"), py::arg("pts"), py::arg("npts"))
      .def("matrix_keep", &PyCchGpu::matrix_keep, py::arg("key"), py::arg("pts"), py::arg("npts"))
      .def("legs_from_matrix", &PyCchGpu::legs_from_matrix, py::arg("key"), py::arg("tag"), py::arg("pts"), py::arg("r"),
           py::arg("i"), py::arg("j"), py::arg("max_path") = 4096, py::arg("want_path") = true)
      .def("set_capacity", &PyCchGpu::set_capacity)
      .def("set_cache_gb", &PyCchGpu::set_cache_gb, py::arg("gb"))
      .def("set_builder_pacing", &PyCchGpu::set_builder_pacing, py::arg("max_workgroups"), py::arg("always") = false)
      .def("request_build", &PyCchGpu::request_build, py::arg("weather"), py::arg("congestion"), py::arg("weekhour"),
           py::arg("driver_age") = 35.0, py::arg("urgent") = true)
      .def("is_cached", &PyCchGpu::is_cached, py::arg("key"))
      .def("ptr", &PyCchGpu::ptr)
      .def("topology_arrays", &PyCchGpu::topology_arrays);
}
