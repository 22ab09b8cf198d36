// routest_amd._rt — CPU-side native runtime (pybind11, no GPU dependency).
//
//  * pack_predict_batch / format_predict_batch: the batched /predict wire path in C++: raw JSON body
//    -> 16-byte EtaRecords (+ pickup timestamps) and minutes -> response JSON, with the reference's
//    field semantics (RO/Flaskr/routes.py:365-383, RO/Flaskr/ml.py:23-58): defaults Sunny/Low/30,
//    `float(x or default)` truthiness, unknown categories -> all-zero one-hot, completion time =
//    pickup + timedelta(minutes) with CPython's microsecond rounding and isoformat() layout.
//  * iso_parse: datetime.fromisoformat (3.12 semantics for the common forms).
//  * greedy_trips: R21 semantics (scan order = distance from the depot, single pass per trip) with
//    the infeasible-stop guard — CPU fallback for the K6 kernel.
//  * astar_batch: multi-threaded A* / Dijkstra on a CSR graph — CPU fallback for the K9 kernel.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <queue>
#include <stdexcept>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "rt_core.h"
#include "http_client.h"

namespace py = pybind11;

using namespace rtc;

// body -> (records uint8 [N,16], pickup_secs int64 [N], pickup_us int32 [N], tz int32 [N, 2]
//          (has_tz, offset_s), errors list[str], is_batch)
py::tuple pack_predict_batch(py::bytes body, int64_t now_secs, int32_t now_us) {
  std::string b = body;
  Stamp now;
  now.secs = now_secs;
  now.us = now_us;
  // Fast path for big top-level arrays: split items with one scan, then parse + pack them in
  // parallel (each item is an independent JSON value).  Anything else takes the DOM path.
  std::vector<std::pair<size_t, size_t>> spans;
  bool split = false;
  {
    py::gil_scoped_release nogil;
    if (b.size() > (64u << 10)) split = split_top_array(b.data(), b.size(), spans);
  }
  if (split) {
    const size_t n = spans.size();
    py::array_t<uint8_t> rec({(py::ssize_t)n, (py::ssize_t)16});
    py::array_t<int64_t> secs(n);
    py::array_t<int32_t> us(n);
    py::array_t<int32_t> tz({(py::ssize_t)n, (py::ssize_t)2});
    std::vector<std::string> errs(n);
    std::atomic<bool> bad{false};
    std::string bad_msg;
    std::mutex bad_mu;
    {
      auto R = rec.mutable_unchecked<2>();
      auto S = secs.mutable_unchecked<1>();
      auto U = us.mutable_unchecked<1>();
      auto T = tz.mutable_unchecked<2>();
      py::gil_scoped_release nogil;
      parallel_chunks(n, 1024, 16, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi && !bad.load(std::memory_order_relaxed); ++i) {
          EtaRecord r{};
          Stamp st;
          try {
            rtj::Value v = rtj::Parser(b.data() + spans[i].first, spans[i].second - spans[i].first).parse();
            errs[i] = pack_item(v, now, r, st);
          } catch (const std::exception& e) {
            std::lock_guard<std::mutex> lk(bad_mu);
            if (!bad.exchange(true)) bad_msg = e.what();
            return;
          }
          std::memcpy(&R(i, 0), &r, 16);
          S(i) = st.secs;
          U(i) = st.us;
          T(i, 0) = st.has_tz ? 1 : 0;
          T(i, 1) = st.tz_sec;
        }
      });
    }
    if (bad) throw std::runtime_error(bad_msg);
    return py::make_tuple(rec, secs, us, tz, errs, true);
  }
  rtj::Value root;
  {
    py::gil_scoped_release nogil;
    root = rtj::Parser(b.data(), b.size()).parse();
  }
  const std::vector<rtj::Value>* items = nullptr;
  std::vector<rtj::Value> single;
  bool is_batch = true;
  if (root.kind == rtj::Value::Arr) {
    items = &root.arr;
  } else if (root.kind == rtj::Value::Obj && root.get("items") && root.get("items")->kind == rtj::Value::Arr) {
    items = &root.get("items")->arr;
  } else {
    is_batch = false;
    single.push_back(root.kind == rtj::Value::Obj ? root : rtj::Value{});
    if (root.kind != rtj::Value::Obj) single[0].kind = rtj::Value::Obj;  // silent -> {}
    items = &single;
  }
  const size_t n = items->size();
  py::array_t<uint8_t> rec({(py::ssize_t)n, (py::ssize_t)16});
  py::array_t<int64_t> secs(n);
  py::array_t<int32_t> us(n);
  py::array_t<int32_t> tz({(py::ssize_t)n, (py::ssize_t)2});
  std::vector<std::string> errs(n);
  {
    auto R = rec.mutable_unchecked<2>();
    auto S = secs.mutable_unchecked<1>();
    auto U = us.mutable_unchecked<1>();
    auto T = tz.mutable_unchecked<2>();
    py::gil_scoped_release nogil;
    parallel_chunks(n, 2048, 16, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        EtaRecord r{};
        Stamp st;
        errs[i] = pack_item((*items)[i], now, r, st);
        std::memcpy(&R(i, 0), &r, 16);
        S(i) = st.secs;
        U(i) = st.us;
        T(i, 0) = st.has_tz ? 1 : 0;
        T(i, 1) = st.tz_sec;
      }
    });
  }
  return py::make_tuple(rec, secs, us, tz, errs, is_batch);
}

// uint8 [N,16] EtaRecords -> uint8 [N,8] wire8 records, or None if the batch is not exactly
// representable (the native front end's guard, rt_core.h pack_wire8).
py::object pack_wire8_py(py::array_t<uint8_t, py::array::c_style> rec) {
  if (rec.ndim() != 2 || rec.shape(1) != 16) throw std::invalid_argument("records must be uint8 [N,16]");
  const size_t n = (size_t)rec.shape(0);
  py::array_t<uint8_t> out({(py::ssize_t)n, (py::ssize_t)8});
  bool ok;
  {
    py::gil_scoped_release nogil;
    ok = pack_wire8(reinterpret_cast<const EtaRecord*>(rec.data()), n,
                    reinterpret_cast<Wire8*>(out.mutable_data()));
  }
  if (!ok) return py::none();
  return std::move(out);
}

// minutes + stamps -> the reference's response JSON (batch: {"predictions": [...]}).
py::bytes format_predict_batch(py::array_t<float, py::array::c_style | py::array::forcecast> minutes,
                               py::array_t<int64_t> secs, py::array_t<int32_t> us,
                               py::array_t<int32_t> tz, std::vector<std::string> errs,
                               bool is_batch) {
  auto M = minutes.unchecked<1>();
  auto S = secs.unchecked<1>();
  auto U = us.unchecked<1>();
  auto T = tz.unchecked<2>();
  const size_t n = (size_t)M.shape(0);
  std::string o;
  {
    py::gil_scoped_release nogil;
    o.reserve(n * 96 + 32);
    if (is_batch) o += "{\"predictions\":[";
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>(std::min(hw, 16u), n / 2048);
    if (nt <= 1) {
      for (size_t i = 0; i < n; ++i) {
        if (i) o += ',';
        format_one(o, (double)M(i), S(i), U(i), T(i, 0) != 0, T(i, 1), errs[i]);
      }
    } else {
      std::vector<std::string> parts(nt);
      const size_t per = (n + nt - 1) / nt;
      parallel_chunks(nt, 1, 16, [&](size_t klo, size_t khi) {
        for (size_t k = klo; k < khi; ++k) {
          std::string& part = parts[k];
          const size_t lo = k * per, hi = std::min(n, lo + per);
          part.reserve((hi - lo) * 96);
          for (size_t i = lo; i < hi; ++i) {
            if (i) part += ',';
            format_one(part, (double)M(i), S(i), U(i), T(i, 0) != 0, T(i, 1), errs[i]);
          }
        }
      });
      for (auto& part : parts) o += part;
    }
    if (is_batch) o += "]}";
  }
  return py::bytes(o);
}

py::object iso_parse(const std::string& s) {
  Stamp st;
  if (!parse_iso(s, st)) return py::none();
  return py::make_tuple(st.secs, st.us, st.has_tz, st.tz_sec);
}

std::string iso_add_minutes(int64_t secs, int32_t us, bool has_tz, int32_t tz_sec, double minutes) {
  Stamp tzs;
  tzs.has_tz = has_tz;
  tzs.tz_sec = tz_sec;
  int64_t tot_us = (int64_t)us + timedelta_minutes_us(minutes);
  int64_t s = secs + (tot_us >= 0 ? tot_us / 1000000 : -((-tot_us + 999999) / 1000000));
  return isoformat(s, tot_us - (s - secs) * 1000000, tzs);
}

std::string py_float_repr(double v) {
  std::string o;
  append_pyfloat(o, v);
  return o;
}

// ------------------------------------------------------------------ R21 greedy (CPU fallback)
py::object greedy_trips(py::array_t<double, py::array::c_style | py::array::forcecast> D,
                        std::vector<double> demand, double cap, double maxd) {
  auto d = D.unchecked<2>();
  const int n = (int)d.shape(0) - 1;
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i + 1;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return d(0, a) < d(0, b); });
  std::vector<char> vis(n + 1, 0);
  int remaining = n;
  std::vector<std::vector<int>> trips;
  while (remaining) {
    std::vector<int> trip{0};
    double load = 0, td = 0;
    int cur = 0;
    for (int idx : order) {
      if (vis[idx]) continue;
      const double dem = demand[idx];
      if (load + dem <= cap && td + (d(cur, idx) + d(idx, 0)) <= maxd) {
        trip.push_back(idx);
        load += dem;
        td += d(cur, idx);
        cur = idx;
      }
    }
    if (trip.size() == 1) {
      std::vector<int> rest;
      for (int idx : order)
        if (!vis[idx]) rest.push_back(idx - 1);
      return py::make_tuple(py::none(), rest);
    }
    for (size_t k = 1; k < trip.size(); ++k) vis[trip[k]] = 1;
    remaining -= (int)trip.size() - 1;
    trip.push_back(0);
    trips.push_back(std::move(trip));
  }
  return py::make_tuple(trips, py::none());
}

// ------------------------------------------------------------------ A* (CPU fallback)
py::tuple astar_batch(py::array_t<int32_t> indptr, py::array_t<int32_t> indices,
                      py::array_t<float> cost, py::array_t<float> lat, py::array_t<float> lon,
                      py::array_t<int32_t> src, py::array_t<int32_t> dst, double inv_vmax,
                      int threads) {
  auto ip = indptr.unchecked<1>();
  auto ix = indices.unchecked<1>();
  auto c = cost.unchecked<1>();
  auto la = lat.unchecked<1>();
  auto lo = lon.unchecked<1>();
  auto S = src.unchecked<1>();
  auto T = dst.unchecked<1>();
  const int N = (int)la.shape(0);
  const int Q = (int)S.shape(0);
  py::array_t<float> out(Q);
  auto O = out.mutable_unchecked<1>();
  std::vector<std::vector<int>> paths(Q);
  {
    py::gil_scoped_release nogil;
    std::atomic<int> next{0};
    auto worker = [&]() {
      std::vector<float> g(N, INFINITY);
      std::vector<int> par(N, -1);
      std::vector<char> closed(N, 0);
      std::vector<int> touched;
      const double k = M_PI / 180.0;
      while (true) {
        const int q = next.fetch_add(1);
        if (q >= Q) break;
        const int s = S(q), t = T(q);
        const double tl = la(t) * k, tn = lo(t) * k, ct = std::cos(tl);
        auto h = [&](int v) {
          const double l1 = la(v) * k;
          const double s1 = std::sin(0.5 * (tl - l1)), s2 = std::sin(0.5 * (tn - lo(v) * k));
          const double hv = s1 * s1 + std::cos(l1) * ct * s2 * s2;
          return 0.999 * 2 * 6371000.0 * std::asin(std::sqrt(std::min(1.0, std::max(0.0, hv)))) * inv_vmax;
        };
        using E = std::pair<double, int>;
        std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
        g[s] = 0;
        touched.push_back(s);
        pq.push({h(s), s});
        bool found = false;
        while (!pq.empty()) {
          const int v = pq.top().second;
          pq.pop();
          if (closed[v]) continue;
          closed[v] = 1;
          if (v == t) { found = true; break; }
          for (int e = ip(v); e < ip(v + 1); ++e) {
            const int u = ix(e);
            if (closed[u]) continue;
            const float ng = g[v] + c(e);
            if (ng < g[u]) {
              if (std::isinf(g[u])) touched.push_back(u);
              g[u] = ng;
              par[u] = v;
              pq.push({ng + h(u), u});
            }
          }
        }
        O(q) = found ? g[t] : -1.f;
        if (found) {
          for (int v = t; v != -1; v = (v == s ? -1 : par[v])) paths[q].push_back(v);
          std::reverse(paths[q].begin(), paths[q].end());
        }
        for (int v : touched) {
          g[v] = INFINITY;
          par[v] = -1;
          closed[v] = 0;
        }
        touched.clear();
      }
    };
    std::vector<std::thread> pool;
    const int nt = std::max(1, std::min(threads, Q));
    for (int i = 0; i < nt; ++i) pool.emplace_back(worker);
    for (auto& th : pool) th.join();
  }
  return py::make_tuple(out, paths);
}

// Native closed-loop HTTP client (bench.py p50, load sweeps): returns the sorted latencies (us) and
// counters; the GIL is released while the sockets run.
py::dict py_http_load(int port, int connections, double seconds, const std::string& path, const std::string& body,
                   int threads, long long max_requests, int warmup) {
  rtc::LoadResult r;
  {
    py::gil_scoped_release nogil;
    r = rtc::http_load(port, connections, seconds, path, body, threads, max_requests, warmup);
  }
  py::dict d;
  d["seconds"] = r.seconds;
  d["requests"] = r.requests;
  d["errors"] = r.errors;
  d["latencies_us"] = py::array_t<float>(r.lat_us.size(), r.lat_us.data());
  return d;
}

void bind_route(py::module& m);   // route_bind.cpp
void bind_cch(py::module& m);     // cch_bind.cpp

// The same over many different requests (path, body), cycled — e.g. 1k distinct route requests.
py::dict py_http_load_multi(int port, int connections, double seconds, const std::vector<std::string>& paths,
                            const std::vector<std::string>& bodies, int threads, long long max_requests,
                            int warmup) {
  if (paths.size() != bodies.size() || paths.empty()) throw std::invalid_argument("paths/bodies mismatch");
  std::vector<std::string> reqs;
  for (size_t i = 0; i < paths.size(); ++i) reqs.push_back(rtc::post_request(paths[i], bodies[i]));
  rtc::LoadResult r;
  {
    py::gil_scoped_release nogil;
    r = rtc::http_load_multi(port, connections, seconds, reqs, threads, max_requests, warmup);
  }
  py::dict d;
  d["seconds"] = r.seconds;
  d["requests"] = r.requests;
  d["errors"] = r.errors;
  d["bytes"] = r.bytes;
  d["latencies_us"] = py::array_t<float>(r.lat_us.size(), r.lat_us.data());
  return d;
}

// Mixed raw requests (any method) with per-kind status tallies — tools/app_soak.py --stack.
py::dict py_http_load_mixed(int port, int connections, double seconds, const std::vector<py::bytes>& raw,
                            const std::vector<int>& kinds, int nkinds, int threads) {
  if (raw.size() != kinds.size() || raw.empty()) throw std::invalid_argument("raw/kinds mismatch");
  std::vector<std::string> reqs;
  for (const auto& b : raw) reqs.push_back(std::string(b));
  rtc::LoadResult r;
  {
    py::gil_scoped_release nogil;
    r = rtc::http_load_mixed(port, connections, seconds, reqs, kinds, nkinds, threads);
  }
  py::dict d;
  d["seconds"] = r.seconds;
  d["requests"] = r.requests;
  d["errors"] = r.errors;
  d["bytes"] = r.bytes;
  d["latencies_us"] = py::array_t<float>(r.lat_us.size(), r.lat_us.data());
  py::list by;
  for (const auto& v : r.status_by_kind) {
    py::dict k;
    for (const auto& pc : v) k[py::int_(pc.first)] = pc.second;
    by.append(k);
  }
  d["status_by_kind"] = by;
  py::list pk;
  for (const auto& q : r.p50_p99_by_kind) pk.append(py::make_tuple(q.first, q.second));
  d["p50_p99_us_by_kind"] = pk;
  return d;
}

PYBIND11_MODULE(_rt, m) {
  m.doc() = "routest_amd CPU native runtime";
  bind_route(m);
  bind_cch(m);
  m.def("http_load", &py_http_load, py::arg("port"), py::arg("connections") = 1, py::arg("seconds") = 2.0,
        py::arg("path") = "/api/predict_eta", py::arg("body") = "", py::arg("threads") = 1,
        py::arg("max_requests") = 0, py::arg("warmup") = 0);
  m.def("http_load_multi", &py_http_load_multi, py::arg("port"), py::arg("connections"), py::arg("seconds"),
        py::arg("paths"), py::arg("bodies"), py::arg("threads") = 4, py::arg("max_requests") = 0,
        py::arg("warmup") = 0);
  m.def("http_load_mixed", &py_http_load_mixed, py::arg("port"), py::arg("connections"), py::arg("seconds"),
        py::arg("raw"), py::arg("kinds"), py::arg("nkinds"), py::arg("threads") = 4);
  m.def("pack_predict_batch", &pack_predict_batch, py::arg("body"), py::arg("now_secs"), py::arg("now_us"));
  m.def("format_predict_batch", &format_predict_batch);
  m.def("pack_wire8", &pack_wire8_py);
  m.def("iso_parse", &iso_parse);
  m.def("iso_add_minutes", &iso_add_minutes);
  m.def("py_float_repr", &py_float_repr);
  m.def("greedy_trips", &greedy_trips);
  m.def("astar_batch", &astar_batch, py::arg("indptr"), py::arg("indices"), py::arg("cost"),
        py::arg("lat"), py::arg("lon"), py::arg("src"), py::arg("dst"), py::arg("inv_vmax"),
        py::arg("threads") = 8);
  m.attr("EPOCH2020_DAYS") = EPOCH2020_DAYS;
}
