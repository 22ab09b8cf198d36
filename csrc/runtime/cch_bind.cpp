// routest_amd._rt bindings of the host CCH (csrc/runtime/cch.h): the CPU reference the GPU router
// (csrc/cch.hip) is tested against bit for bit, the GPU-less deployment path, and the same-box
// multi-thread CPU baseline (bench/cch_cpu_baseline.py).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <cmath>
#include <vector>
#include <memory>

#include "cch.h"

namespace py = pybind11;

namespace {

template <class T>
using arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

template <class T>
py::array_t<T> to_np(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

struct PyMetric {
  std::shared_ptr<rcch::Metric> m;
  double ms = 0.0;
};

class PyCCH {
 public:
  PyCCH(arr<int32_t> indptr, arr<int32_t> indices, arr<double> lat, arr<double> lon, unsigned threads)
      : pool_(threads) {
    const int N = (int)lat.shape(0);
    if (indptr.shape(0) != N + 1 || lon.shape(0) != N) throw std::invalid_argument("graph shapes");
    const int32_t* ip = indptr.data();
    for (int v = 0; v < N; ++v)
      if (ip[v] > ip[v + 1]) throw std::invalid_argument("indptr not monotone");
    if (ip[N] != indices.shape(0)) throw std::invalid_argument("indices length");
    const int32_t* ix = indices.data();
    for (py::ssize_t e = 0; e < indices.shape(0); ++e)
      if (ix[e] < 0 || ix[e] >= N) throw std::out_of_range("edge target out of range");
    auto t0 = std::chrono::steady_clock::now();
    {
      py::gil_scoped_release nogil;
      T_ = rcch::build_topology(N, ip, ix, lat.data(), lon.data());
    }
    build_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }

  py::dict stats() const {
    py::dict d;
    d["nodes"] = T_.N;
    d["arcs"] = T_.M;
    d["edges"] = T_.E;
    d["max_depth"] = T_.max_depth;
    d["max_height"] = T_.max_height;
    d["top_separator"] = T_.separator_top;
    d["build_ms"] = build_ms_;
    d["threads"] = pool_.size();
    int64_t tri = 0;
    for (int r = 0; r < T_.N; ++r) {
      const int64_t k = T_.up_ptr[r + 1] - T_.up_ptr[r];
      tri += k * (k - 1) / 2;
    }
    d["triangles"] = tri;
    return d;
  }

  py::dict arrays() const {
    py::dict d;
    d["rank"] = to_np(T_.rank);
    d["node"] = to_np(T_.node);
    d["up_ptr"] = to_np(T_.up_ptr);
    d["up_head"] = to_np(T_.up_head);
    d["arc_lo"] = to_np(T_.arc_lo);
    d["parent"] = to_np(T_.parent);
    d["depth"] = to_np(T_.depth);
    d["height"] = to_np(T_.height);
    d["edge_arc"] = to_np(T_.edge_arc);
    d["edge_dir"] = to_np(T_.edge_dir);
    return d;
  }

  PyMetric customize(arr<float> cost, arr<float> length) {
    if (cost.shape(0) != T_.E || length.shape(0) != T_.E) throw std::invalid_argument("cost/length per edge");
    // weights are ordered by their float bits (cch.h pack_w): a NaN, a negative cost or -0.0 (sign
    // bit set) would sort above every real weight and silently drop the edge — reject / normalise
    std::vector<float> c(cost.data(), cost.data() + T_.E);
    for (float& x : c) {
      if (!std::isfinite(x) || x < 0.f) throw std::invalid_argument("edge costs must be finite and >= 0");
      x += 0.f;                                 // -0.0 -> +0.0
    }
    PyMetric pm;
    pm.m = std::make_shared<rcch::Metric>();
    auto t0 = std::chrono::steady_clock::now();
    {
      py::gil_scoped_release nogil;
      rcch::customize(T_, c.data(), length.data(), *pm.m, pool_);
    }
    pm.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return pm;
  }

  // (sec f32[Q], metres f32[Q], status i32[Q], paths: list of int32 arrays or None)
  py::tuple query(const PyMetric& pm, arr<int32_t> src, arr<int32_t> dst, bool want_path, int64_t max_path) {
    const py::ssize_t Q = src.shape(0);
    if (dst.shape(0) != Q) throw std::invalid_argument("src/dst length");
    for (py::ssize_t i = 0; i < Q; ++i)
      if (src.data()[i] < 0 || src.data()[i] >= T_.N || dst.data()[i] < 0 || dst.data()[i] >= T_.N)
        throw std::out_of_range("query node out of range");
    std::vector<rcch::P2P> res(Q);
    const int32_t* s = src.data();
    const int32_t* t = dst.data();
    {
      py::gil_scoped_release nogil;
      std::vector<rcch::ChainScratch> cs(pool_.size() + 1);
      std::atomic<int> slot{0};
      thread_local int my = -1;
      (void)my;
      pool_.run((size_t)Q, [&](size_t i) {
        thread_local rcch::ChainScratch local;
        rcch::query(T_, *pm.m, s[i], t[i], local, res[i], want_path, (size_t)max_path);
      }, 16);
    }
    py::array_t<float> sec(Q), met(Q);
    py::array_t<int32_t> st(Q);
    py::list paths;
    for (py::ssize_t i = 0; i < Q; ++i) {
      sec.mutable_data()[i] = res[i].status == 0 ? res[i].sec : -1.f;
      met.mutable_data()[i] = res[i].status == 0 ? res[i].metres : -1.f;
      st.mutable_data()[i] = res[i].status;
      if (want_path) paths.append(to_np(res[i].path));
    }
    return py::make_tuple(sec, met, st, want_path ? py::object(paths) : py::object(py::none()));
  }

  // timing-only batch (the CPU baseline): queries without paths or with paths, returns wall ms
  double bench(const PyMetric& pm, arr<int32_t> src, arr<int32_t> dst, bool want_path) {
    const py::ssize_t Q = src.shape(0);
    const int32_t* s = src.data();
    const int32_t* t = dst.data();
    auto t0 = std::chrono::steady_clock::now();
    {
      py::gil_scoped_release nogil;
      pool_.run((size_t)Q, [&](size_t i) {
        thread_local rcch::ChainScratch local;
        thread_local rcch::P2P r;
        rcch::query(T_, *pm.m, s[i], t[i], local, r, want_path);
      }, 16);
    }
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }

  py::dict metric_arrays(const PyMetric& pm) const {
    const rcch::Metric& m = *pm.m;
    py::dict d;
    std::vector<float> wu(T_.M), wd(T_.M);
    std::vector<uint32_t> pu(T_.M), pd(T_.M);
    for (int64_t a = 0; a < T_.M; ++a) {
      wu[a] = rcch::w_of(m.up[a]);
      wd[a] = rcch::w_of(m.dn[a]);
      pu[a] = (uint32_t)m.up[a];
      pd[a] = (uint32_t)m.dn[a];
    }
    d["w_up"] = to_np(wu);
    d["w_dn"] = to_np(wd);
    d["pay_up"] = to_np(pu);
    d["pay_dn"] = to_np(pd);
    d["sub_up"] = to_np(m.sub_up);
    d["sub_dn"] = to_np(m.sub_dn);
    d["len_up"] = to_np(m.len_up);
    d["len_dn"] = to_np(m.len_dn);
    d["p_up"] = to_np(m.pup);
    d["p_dn"] = to_np(m.pdn);
    d["kept_f"] = m.kept_f;
    d["kept_b"] = m.kept_b;
    d["customize_ms"] = pm.ms;
    return d;
  }

 private:
  rcch::Pool pool_;
  rcch::Topology T_;
  double build_ms_ = 0.0;
};

}  // namespace

void bind_cch(py::module& m) {
  py::class_<PyMetric>(m, "CchMetric").def_readonly("customize_ms", &PyMetric::ms);
  py::class_<PyCCH>(m, "CCH")
      .def(py::init<arr<int32_t>, arr<int32_t>, arr<double>, arr<double>, unsigned>(), py::arg("indptr"),
           py::arg("indices"), py::arg("lat"), py::arg("lon"), py::arg("threads") = 0)
      .def("stats", &PyCCH::stats)
      .def("arrays", &PyCCH::arrays)
      .def("customize", &PyCCH::customize, py::arg("cost"), py::arg("length"))
      .def("query", &PyCCH::query, py::arg("metric"), py::arg("src"), py::arg("dst"), py::arg("want_path") = true,
           py::arg("max_path") = 1 << 20)
      .def("bench", &PyCCH::bench, py::arg("metric"), py::arg("src"), py::arg("dst"), py::arg("want_path") = false)
      .def("metric_arrays", &PyCCH::metric_arrays);
}
