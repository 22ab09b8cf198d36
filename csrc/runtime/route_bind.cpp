// routest_amd._rt bindings of the native route assembler (csrc/runtime/route_core.h).
//
//  * haversine_m / path_length_m / NodeGrid: the libm-dependent values of the Python providers
//    (routing/providers.py, routing/graph.py, data/graph.py) come from these, so the Python path
//    and the native front end (csrc/native_server.hip) produce identical bits.
//  * route_optimize_cpu: the whole haversine-provider request on the CPU in C++ (parse, matrix,
//    R21 greedy, directions, assembly) -> (status, body) or None (fallback to Python) — the CPU
//    reference the GPU service is tested against, and a fast path for GPU-less deployments.
//  * route_assemble_graph: graph-provider assembly from given trips + searched legs (tests).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <map>
#include <memory>
#include <mutex>

#include "alternatives.h"
#include "history_db.h"
#include "route_core.h"
#include "route_record.h"

namespace py = pybind11;

namespace {

using rtr::Value;

double py_haversine(double lat1, double lon1, double lat2, double lon2) {
  return rtr::haversine_m(lat1, lon1, lat2, lon2);
}

double py_path_length(py::array_t<double, py::array::c_style | py::array::forcecast> lat,
                      py::array_t<double, py::array::c_style | py::array::forcecast> lon,
                      py::array_t<int32_t, py::array::c_style | py::array::forcecast> path) {
  const int64_t n = lat.shape(0);
  const int32_t* p = path.data();
  for (py::ssize_t i = 0; i < path.shape(0); ++i)
    if (p[i] < 0 || p[i] >= n) throw std::out_of_range("path node out of range");
  return rtr::path_length_m(lat.data(), lon.data(), p, (size_t)path.shape(0));
}

py::array_t<double> py_haversine_matrix(py::array_t<double, py::array::c_style | py::array::forcecast> lat,
                                        py::array_t<double, py::array::c_style | py::array::forcecast> lon,
                                        double circuity) {
  const py::ssize_t n = lat.shape(0);
  py::array_t<double> D({n, n});
  double* d = D.mutable_data();
  const double* la = lat.data();
  const double* lo = lon.data();
  for (py::ssize_t i = 0; i < n; ++i)
    for (py::ssize_t j = 0; j < n; ++j)
      d[i * n + j] = i == j ? 0.0 : rtr::haversine_m(la[i], lo[i], la[j], lo[j]) * circuity;
  return D;
}

class PyNodeGrid {
 public:
  PyNodeGrid(py::array_t<double, py::array::c_style | py::array::forcecast> lat,
             py::array_t<double, py::array::c_style | py::array::forcecast> lon, double c)
      : c_(c) {
    if (lat.shape(0) != lon.shape(0) || lat.shape(0) == 0) throw std::invalid_argument("lat/lon mismatch");
    g_.build(lat.data(), lon.data(), (size_t)lat.shape(0), c);
  }
  py::array_t<int32_t> nearest(py::array_t<double, py::array::c_style | py::array::forcecast> lats,
                               py::array_t<double, py::array::c_style | py::array::forcecast> lons) const {
    const py::ssize_t n = lats.shape(0);
    py::array_t<int32_t> out(n);
    int32_t* o = out.mutable_data();
    const double* la = lats.data();
    const double* lo = lons.data();
    {
      py::gil_scoped_release nogil;
      for (py::ssize_t i = 0; i < n; ++i) o[i] = g_.nearest(la[i], lo[i], c_);
    }
    return out;
  }

 private:
  rtr::NodeGrid g_;
  double c_;
};

// Maneuvers of graph legs (route_core.h leg_steps) for the Python GraphProvider: the graph's
// arrays are held once; per call the leg's node path, seconds and the context's edge costs.
class PyGraphSteps {
 public:
  PyGraphSteps(py::array_t<int32_t, py::array::c_style | py::array::forcecast> indptr,
               py::array_t<int32_t, py::array::c_style | py::array::forcecast> indices,
               py::array_t<float, py::array::c_style | py::array::forcecast> length,
               py::array_t<double, py::array::c_style | py::array::forcecast> lat,
               py::array_t<double, py::array::c_style | py::array::forcecast> lon, py::object edge_name,
               std::vector<std::string> names)
      : indptr_(indptr), indices_(indices), length_(length), lat_(lat), lon_(lon), names_(std::move(names)) {
    const py::ssize_t N = lat.shape(0), E = indices.shape(0);
    if (indptr.shape(0) != N + 1 || lon.shape(0) != N || length.shape(0) != E || indptr.data()[N] != E)
      throw std::invalid_argument("graph shapes");
    if (!edge_name.is_none()) {
      name_ = edge_name.cast<py::array_t<int32_t, py::array::c_style | py::array::forcecast>>();
      if (name_.shape(0) != E) throw std::invalid_argument("edge_name per edge");
    }
  }
  // the graph host view with the given per-edge costs (kept alive by the caller)
  rtr::GraphHost host(const py::array_t<float, py::array::c_style | py::array::forcecast>& cost) const {
    if (cost.shape(0) != indices_.shape(0)) throw std::invalid_argument("cost per edge");
    rtr::GraphHost g;
    g.indptr = indptr_.data();
    g.indices = indices_.data();
    g.length = length_.data();
    g.cost = cost.data();
    g.edge_name = name_.size() ? name_.data() : nullptr;
    g.names = &names_;
    return g;
  }
  // the compact route records' view of this graph (built on first use: CoordCache, headings,
  // fingerprint); shared with a HistoryDb
  std::shared_ptr<const rrec::RecordGraph> record_graph() const {
    std::lock_guard<std::mutex> lk(rg_mu_);
    if (!rg_) {
      auto g = std::make_shared<rrec::RecordGraph>();
      g->build((int)lat_.shape(0), lat_.data(), lon_.data(), indptr_.data(), indices_.data(), length_.data(),
               name_.size() ? name_.data() : nullptr, &names_);
      rg_ = g;
    }
    return rg_;
  }
  // (legs JSON, geometry JSON) of a record the native route service persisted (store.py)
  py::tuple decode_record(py::bytes rec) const {
    const std::string b = rec;
    auto g = record_graph();
    std::string seg, geo, err;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = rrec::decode(*g, b.data(), b.size(), seg, geo, &err);
    }
    if (!ok) throw std::invalid_argument(err);
    return py::make_tuple(seg, geo);
  }
  std::string fingerprint() const { return std::to_string(record_graph()->fp); }
  py::list steps(py::array_t<int32_t, py::array::c_style | py::array::forcecast> path, double sec,
                 py::array_t<float, py::array::c_style | py::array::forcecast> cost, double speed_scale,
                 long long start, long long end) const {
    const py::ssize_t N = lat_.shape(0);
    if (cost.shape(0) != indices_.shape(0)) throw std::invalid_argument("cost per edge");
    for (py::ssize_t i = 0; i < path.shape(0); ++i)
      if (path.data()[i] < 0 || path.data()[i] >= N) throw std::out_of_range("path node");
    rtr::GraphHost g;
    g.indptr = indptr_.data();
    g.indices = indices_.data();
    g.length = length_.data();
    g.cost = cost.data();
    g.edge_name = name_.size() ? name_.data() : nullptr;
    g.names = &names_;
    rtr::Leg L;
    L.sec = sec;
    L.path = path.data();
    L.len = (int)path.shape(0);
    std::vector<rtr::Step> st;
    rtr::leg_steps(g, lat_.data(), lon_.data(), L, speed_scale, start, end, st);
    py::list out;
    for (const auto& x : st)
      out.append(py::make_tuple(x.dist, x.dur, x.type, x.instruction(), x.name_str(), x.wp0, x.wp1));
    return out;
  }

 private:
  py::array_t<int32_t, py::array::c_style | py::array::forcecast> indptr_, indices_;
  py::array_t<float, py::array::c_style | py::array::forcecast> length_;
  py::array_t<double, py::array::c_style | py::array::forcecast> lat_, lon_;
  py::array_t<int32_t, py::array::c_style | py::array::forcecast> name_;
  std::vector<std::string> names_;
  mutable std::mutex rg_mu_;
  mutable std::shared_ptr<const rrec::RecordGraph> rg_;
};

py::bytes to_bytes(const std::string& s) { return py::bytes(s); }

// The native history reader (history_db.h) for CPU tests: (status, body) or None (-> the app).
class PyHistoryDb {
 public:
  explicit PyHistoryDb(const std::string& path, py::object graph) {
    std::string err;
    if (!db_.open(path, err)) throw std::runtime_error("HistoryDb: " + err);
    if (!graph.is_none()) db_.set_graph(graph.cast<const PyGraphSteps&>().record_graph());
  }
  py::object wrap(const rth::Reply& r) {
    if (r.fallback) return py::none();
    return py::make_tuple(r.status, to_bytes(r.body));
  }
  py::object history(py::object limit) {
    if (limit.is_none()) return wrap(db_.history(nullptr));
    const std::string l = limit.cast<std::string>();
    return wrap(db_.history(l.c_str()));
  }
  py::object detail(const std::string& id) { return wrap(db_.detail(id)); }
  py::object del(const std::string& id) { return wrap(db_.del(id)); }
  py::object locations() { return wrap(db_.locations()); }

 private:
  rth::HistoryDb db_;
};

// Finish an assembled request as the FastAPI handler answers it (no ETA, no persistence).
std::pair<int, std::string> finish_plain(const rtr::Assembled& a, bool request_route_compat, bool is_request_route) {
  if (!a.error.empty()) {
    const int st = (is_request_route && request_route_compat) ? 200 : 400;
    return {st, rtr::error_body(a.error)};
  }
  return {200, a.body + "}}"};
}

py::object route_optimize_cpu(py::bytes body, bool json_ok, const std::string& engine, double circuity,
                              double step_m, bool is_request_route, bool compat200) {
  const std::string b = body;
  Value root;
  bool parsed = false;
  if (json_ok && !b.empty()) {
    try {
      root = rtj::Parser(b.data(), b.size()).parse();
      parsed = true;
    } catch (const std::exception&) {
    }
  }
  if (is_request_route && (!json_ok || (!parsed && !b.empty()))) return py::none();   // 415 / 400: Python
  Value empty;
  empty.kind = Value::Obj;
  const Value* rootp = parsed ? &root : (is_request_route ? nullptr : &empty);
  if (!is_request_route && parsed && root.kind != Value::Obj) rootp = &empty;   // silent: non-dict -> {}
  rtr::RouteReq r = rtr::parse_route_request(rootp);
  if (r.fallback || r.alt_k > 0) return py::none();     // alternatives: graph provider + scorer only
  rtr::Plan plan;
  if (r.error.empty() && r.dst.size() > 1) {
    const int n1 = (int)r.dst.size() + 1;
    std::vector<double> lat(n1), lon(n1), dem(n1, 0.0), D((size_t)n1 * n1, 0.0);
    lat[0] = r.src.lat;
    lon[0] = r.src.lon;
    for (int i = 1; i < n1; ++i) {
      lat[i] = r.dst[i - 1].lat;
      lon[i] = r.dst[i - 1].lon;
      dem[i] = r.dst[i - 1].demand;
    }
    for (int i = 0; i < n1; ++i)
      for (int j = 0; j < n1; ++j)
        D[(size_t)i * n1 + j] = i == j ? 0.0 : rtr::haversine_m(lat[i], lon[i], lat[j], lon[j]) * circuity;
    plan.infeasible = !rtr::greedy_trips(D, n1, dem, r.cap, r.maxd, plan.trips, plan.infeasible_stops);
  }
  std::vector<std::vector<std::pair<double, double>>> calls;
  rtr::directions_calls(r, plan, calls);
  std::vector<rtr::Dir> dirs(calls.size());
  for (size_t k = 0; k < calls.size(); ++k)
    rtr::haversine_directions(calls[k], r.profile, circuity, step_m, dirs[k]);
  rtr::Assembled a;
  if (!rtr::assemble(r, plan, dirs, engine, a)) return py::none();
  auto res = finish_plain(a, compat200, is_request_route);
  return py::make_tuple(res.first, to_bytes(res.second));
}

// Graph-provider assembly with given trips and searched legs: `trips` per request as index lists
// (None for point-to-point), `legs` {(s, t): (seconds, [nodes]) | (seconds, metres, [nodes])}
// (missing / empty = not found); with `steps` (GraphSteps) + `cost` the segments carry maneuvers.
py::object route_assemble_graph(py::bytes body, const std::string& engine,
                                py::array_t<double, py::array::c_style | py::array::forcecast> glat,
                                py::array_t<double, py::array::c_style | py::array::forcecast> glon,
                                py::array_t<int32_t, py::array::c_style | py::array::forcecast> nodes_of_calls,
                                py::object trips_obj, py::dict legs_obj, py::object steps_obj, py::object cost_obj,
                                bool with_record) {
  const std::string b = body;
  Value root = rtj::Parser(b.data(), b.size()).parse();
  rtr::RouteReq r = rtr::parse_route_request(&root);
  if (r.fallback) return py::none();
  rtr::Plan plan;
  if (!trips_obj.is_none()) plan.trips = trips_obj.cast<std::vector<std::vector<int>>>();
  std::vector<std::vector<std::pair<double, double>>> calls;
  rtr::directions_calls(r, plan, calls);
  // legs table
  std::map<std::pair<int, int>, std::pair<rtr::Leg, std::vector<int32_t>>> table;
  for (auto kv : legs_obj) {
    auto key = kv.first.cast<std::pair<int, int>>();
    py::tuple val = kv.second.cast<py::tuple>();
    auto& e = table[key];
    e.first.sec = val[0].cast<double>();
    if (val.size() == 3) {
      e.first.metres = val[1].cast<double>();
      e.second = val[2].cast<std::vector<int32_t>>();
    } else {
      e.second = val[1].cast<std::vector<int32_t>>();
    }
    e.first.len = (int)e.second.size();
    e.first.path = e.second.data();
  }
  rtr::GraphHost gh;
  const rtr::GraphHost* ghp = nullptr;
  py::array_t<float, py::array::c_style | py::array::forcecast> cost;
  std::shared_ptr<const rrec::RecordGraph> rg;
  if (!steps_obj.is_none()) {
    const PyGraphSteps& st = steps_obj.cast<const PyGraphSteps&>();
    if (with_record) rg = st.record_graph();
    if (!cost_obj.is_none()) {
      cost = cost_obj.cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
      gh = st.host(cost);
      ghp = &gh;
    }
  }
  // (the compact record, as the route service writes it: route_record.h)
  rrec::Writer rw;
  bool rec_ok = rg != nullptr;
  if (rec_ok) rrec::begin(rw, *rg, ghp != nullptr, r.profile, calls.size());
  const int32_t* nodes = nodes_of_calls.data();
  std::vector<rtr::Dir> dirs(calls.size());
  size_t off = 0;
  rtr::Leg missing;
  for (size_t k = 0; k < calls.size(); ++k) {
    std::vector<const rtr::Leg*> legs;
    for (size_t i = 0; i + 1 < calls[k].size(); ++i) {
      auto it = table.find({nodes[off + i], nodes[off + i + 1]});
      legs.push_back(it == table.end() ? &missing : &it->second.first);
    }
    std::vector<uint64_t> durs;
    std::vector<uint32_t> per_leg;
    rtr::StepDurs sd;
    sd.out = &durs;
    sd.per_leg = &per_leg;
    const std::string e = rtr::graph_directions(calls[k], nodes + off, legs, r.profile, glat.data(), glon.data(), dirs[k],
                                                ghp, rec_ok && ghp ? &sd : nullptr);
    off += calls[k].size();
    if (!e.empty()) {
      r.error = e;
      rec_ok = false;
      break;
    }
    if (rec_ok) rec_ok = !sd.bad && rrec::add_call(rw, *rg, ghp, calls[k], legs, durs, per_leg);
  }
  rtr::Assembled a;
  if (!rtr::assemble(r, plan, dirs, engine, a)) return py::none();
  auto res = finish_plain(a, true, false);
  if (!with_record) return py::make_tuple(res.first, to_bytes(res.second));
  // (status, body, record bytes or None, the row's legs text, the row's geometry text)
  std::string geo = "{\"type\":\"LineString\",\"coordinates\":" + a.coords + "}";
  return py::make_tuple(res.first, to_bytes(res.second), rec_ok && a.ok ? py::object(to_bytes(rw.b)) : py::object(py::none()),
                        a.segments, geo);
}

using F64 = py::array_t<double, py::array::c_style | py::array::forcecast>;
using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;

std::vector<int> py_via_nodes(F64 lat, F64 lon, int s, int t, int n, double stretch) {
  if (lat.shape(0) != lon.shape(0)) throw std::invalid_argument("lat/lon length mismatch");
  py::gil_scoped_release nogil;
  return ralt::via_nodes(lat.data(), lon.data(), (int)lat.shape(0), s, t, n, stretch);
}

std::vector<double> py_alt_scores(F64 lat, F64 lon, F64 delay, std::vector<I32> paths, std::vector<double> seconds,
                                  int kind) {
  const int64_t N = lat.shape(0);
  if (lon.shape(0) != N || delay.shape(0) != N) throw std::invalid_argument("lat/lon/delay length mismatch");
  if (seconds.size() != paths.size()) throw std::invalid_argument("one seconds value per path");
  std::vector<double> out(paths.size());
  for (size_t i = 0; i < paths.size(); ++i) {
    const int32_t* p = paths[i].data();
    const size_t n = (size_t)paths[i].shape(0);
    for (size_t k = 0; k < n; ++k)
      if (p[k] < 0 || p[k] >= N) throw std::out_of_range("path node out of range");
    out[i] = ralt::candidate_score(lat.data(), lon.data(), delay.data(), p, n, seconds[i], kind);
  }
  return out;
}

}  // namespace

void bind_route(py::module& m) {
  m.def("via_nodes", &py_via_nodes, py::arg("lat"), py::arg("lon"), py::arg("s"), py::arg("t"), py::arg("n"),
        py::arg("stretch") = 1.35);
  m.def("alt_scores", &py_alt_scores, py::arg("lat"), py::arg("lon"), py::arg("delay"), py::arg("paths"),
        py::arg("seconds"), py::arg("kind"));
  m.def("haversine_m", &py_haversine);
  m.def("path_length_m", &py_path_length);
  m.def("haversine_matrix", &py_haversine_matrix);
  py::class_<PyNodeGrid>(m, "NodeGrid")
      .def(py::init<py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>, double>())
      .def("nearest", &PyNodeGrid::nearest);
  m.def("route_optimize_cpu", &route_optimize_cpu, py::arg("body"), py::arg("json_ok") = true,
        py::arg("engine") = "backend:mi355x", py::arg("circuity") = 1.3, py::arg("step_m") = 150.0,
        py::arg("is_request_route") = false, py::arg("compat200") = true);
  m.def("route_assemble_graph", &route_assemble_graph, py::arg("body"), py::arg("engine"), py::arg("glat"),
        py::arg("glon"), py::arg("nodes"), py::arg("trips"), py::arg("legs"), py::arg("steps") = py::none(),
        py::arg("cost") = py::none(), py::arg("with_record") = false);
  m.def("py_round", &rtr::py_round);
  m.def("json_float", [](double v) {     // the native JSON writer's float (tests: == json.dumps)
    std::string o;
    rtr::put_float(o, v);
    return o;
  });
  py::class_<PyHistoryDb>(m, "HistoryDb")
      .def(py::init<const std::string&, py::object>(), py::arg("path"), py::arg("graph") = py::none())
      .def("history", &PyHistoryDb::history, py::arg("limit") = py::none())
      .def("detail", &PyHistoryDb::detail)
      .def("delete", &PyHistoryDb::del)
      .def("locations", &PyHistoryDb::locations);
  py::class_<PyGraphSteps>(m, "GraphSteps")
      .def(py::init<py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<float, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>, py::object,
                    std::vector<std::string>>(),
           py::arg("indptr"), py::arg("indices"), py::arg("length"), py::arg("lat"), py::arg("lon"),
           py::arg("edge_name") = py::none(), py::arg("names") = std::vector<std::string>())
      .def("steps", &PyGraphSteps::steps, py::arg("path"), py::arg("sec"), py::arg("cost"), py::arg("speed_scale"),
           py::arg("start"), py::arg("end"))
      .def("decode_record", &PyGraphSteps::decode_record, py::arg("record"))
      .def("fingerprint", &PyGraphSteps::fingerprint);
  m.def("bearing_word", [](double a, double b, double c, double d) { return std::string(rtr::bearing_word(a, b, c, d)); });
}
