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
#include <thread>
#include <vector>

#include "json_lite.h"

namespace py = pybind11;

namespace {

// ------------------------------------------------------------------ civil calendar
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}
void civil_from_days(int64_t z, int64_t& y, unsigned& m, unsigned& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = (unsigned)(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = (int64_t)yoe + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp + (mp < 10 ? 3 : -9);
  y += m <= 2;
}
const int64_t EPOCH2020_DAYS = days_from_civil(2020, 1, 1);

struct Stamp {          // naive wall-clock fields + optional UTC offset (as written)
  int64_t secs = 0;     // wall-clock seconds since 1970-01-01 (tz ignored)
  int32_t us = 0;
  bool has_tz = false;
  int32_t tz_sec = 0;   // offset in seconds
  int32_t tz_us = 0;
};

bool digits(const std::string& s, size_t p, size_t n, int& out) {
  if (p + n > s.size()) return false;
  int v = 0;
  for (size_t i = 0; i < n; ++i) {
    char c = s[p + i];
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
  }
  out = v;
  return true;
}

// datetime.fromisoformat for YYYY-MM-DD[(T| )HH[:MM[:SS[.f{1,9}]]]][Z|±HH[:MM[:SS[.ffffff]]]]
bool parse_iso(const std::string& s, Stamp& st) {
  int Y, M, D, h = 0, mi = 0, se = 0, us = 0;
  if (!digits(s, 0, 4, Y) || s.size() < 10 || s[4] != '-' || !digits(s, 5, 2, M) || s[7] != '-' ||
      !digits(s, 8, 2, D))
    return false;
  if (M < 1 || M > 12 || D < 1) return false;
  static const int mdays[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  if (D > mdays[M - 1] + (M == 2 && leap)) return false;
  size_t p = 10;
  if (p < s.size()) {
    if (s[p] != 'T' && s[p] != ' ') return false;
    ++p;
    if (!digits(s, p, 2, h)) return false;
    p += 2;
    if (p < s.size() && s[p] == ':') {
      if (!digits(s, p + 1, 2, mi)) return false;
      p += 3;
      if (p < s.size() && s[p] == ':') {
        if (!digits(s, p + 1, 2, se)) return false;
        p += 3;
        if (p < s.size() && (s[p] == '.' || s[p] == ',')) {
          ++p;
          size_t q = p;
          while (q < s.size() && s[q] >= '0' && s[q] <= '9') ++q;
          const size_t nd = q - p;
          if (nd == 0 || nd > 9) return false;
          std::string frac = s.substr(p, std::min<size_t>(6, nd));
          while (frac.size() < 6) frac += '0';
          us = std::stoi(frac);
          p = q;
        }
      }
    }
    if (h > 23 || mi > 59 || se > 59) return false;
    if (p < s.size()) {
      char c = s[p];
      if (c == 'Z' || c == 'z') {
        st.has_tz = true;
        ++p;
      } else if (c == '+' || c == '-') {
        const int sign = c == '-' ? -1 : 1;
        int th, tm = 0, ts = 0, tus = 0;
        if (!digits(s, p + 1, 2, th)) return false;
        size_t r = p + 3;
        if (r < s.size() && s[r] == ':') {
          if (!digits(s, r + 1, 2, tm)) return false;
          r += 3;
          if (r < s.size() && s[r] == ':') {
            if (!digits(s, r + 1, 2, ts)) return false;
            r += 3;
          }
        } else if (r + 2 <= s.size() && digits(s, r, 2, tm)) {
          r += 2;
        }
        if (th > 23 || tm > 59 || ts > 59) return false;
        st.has_tz = true;
        st.tz_sec = sign * (th * 3600 + tm * 60 + ts);
        st.tz_us = sign * tus;
        p = r;
      } else {
        return false;
      }
      if (p != s.size()) return false;
    }
  }
  st.secs = days_from_civil(Y, (unsigned)M, (unsigned)D) * 86400 + h * 3600 + mi * 60 + se;
  st.us = us;
  return true;
}

// CPython timedelta(minutes=x) microseconds (Modules/_datetimemodule.c accum + round_half_even)
int64_t timedelta_minutes_us(double x) {
  const double us_per_min = 60000000.0;
  double ip;
  double frac = std::modf(x, &ip);
  int64_t total = (int64_t)ip * 60000000LL;
  double leftover = 0.0;
  if (frac != 0.0) {
    double d = us_per_min * frac;
    double ip2;
    double f2 = std::modf(d, &ip2);
    total += (int64_t)ip2;
    leftover = f2;
  }
  // CPython: round(leftover); exact halves go to even on the TOTAL (not on leftover alone)
  double whole = std::round(leftover);
  if (std::fabs(whole - leftover) == 0.5) {
    const int odd = (int)(total & 1);
    whole = 2.0 * std::round((leftover + odd) * 0.5) - odd;
  }
  return total + (int64_t)whole;
}

void append_2(std::string& o, int v) {
  o += (char)('0' + v / 10);
  o += (char)('0' + v % 10);
}

// datetime.isoformat() of (secs, us) [+ offset]
std::string isoformat(int64_t secs, int64_t us, const Stamp& tz) {
  int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
  int64_t sod = secs - days * 86400;
  int64_t y;
  unsigned m, d;
  civil_from_days(days, y, m, d);
  std::string o;
  o.reserve(40);
  char yb[8];
  std::snprintf(yb, sizeof yb, "%04lld", (long long)y);
  o += yb;
  o += '-';
  append_2(o, (int)m);
  o += '-';
  append_2(o, (int)d);
  o += 'T';
  append_2(o, (int)(sod / 3600));
  o += ':';
  append_2(o, (int)(sod / 60 % 60));
  o += ':';
  append_2(o, (int)(sod % 60));
  if (us) {
    char ub[8];
    std::snprintf(ub, sizeof ub, ".%06lld", (long long)us);
    o += ub;
  }
  if (tz.has_tz) {
    int off = tz.tz_sec;
    o += off < 0 ? '-' : '+';
    off = std::abs(off);
    append_2(o, off / 3600);
    o += ':';
    append_2(o, off / 60 % 60);
    if (off % 60) {
      o += ':';
      append_2(o, off % 60);
    }
  }
  return o;
}

// Python repr(float)
void append_pyfloat(std::string& o, double v) {
  if (std::isnan(v)) { o += "NaN"; return; }
  if (std::isinf(v)) { o += v > 0 ? "Infinity" : "-Infinity"; return; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  std::string sci(buf, r.ptr);
  // sci = [-]d[.ddd]e[+-]XX
  size_t epos = sci.find('e');
  int exp = std::stoi(sci.substr(epos + 1));
  std::string mant = sci.substr(0, epos);
  bool neg = mant[0] == '-';
  if (neg) mant = mant.substr(1);
  std::string digs;
  for (char c : mant)
    if (c != '.') digs += c;
  std::string out;
  if (exp >= -4 && exp < 16) {
    if (exp >= 0) {
      if ((int)digs.size() <= exp + 1) {
        out = digs + std::string(exp + 1 - digs.size(), '0') + ".0";
      } else {
        out = digs.substr(0, exp + 1) + "." + digs.substr(exp + 1);
      }
    } else {
      out = "0." + std::string(-exp - 1, '0') + digs;
    }
  } else {
    out = digs.substr(0, 1);
    if (digs.size() > 1) out += "." + digs.substr(1);
    char eb[8];
    std::snprintf(eb, sizeof eb, "e%c%02d", exp < 0 ? '-' : '+', std::abs(exp));
    out += eb;
  }
  if (neg) o += '-';
  o += out;
}

bool num_of(const rtj::Value* v, double& out) {
  if (!v) return false;
  if (v->kind == rtj::Value::Num) { out = v->num; return true; }
  if (v->kind == rtj::Value::Bool) { out = v->b ? 1.0 : 0.0; return true; }
  if (v->kind == rtj::Value::Str) {  // float("12.5") semantics
    const char* s = v->str.c_str();
    char* e = nullptr;
    out = std::strtod(s, &e);
    while (e && *e == ' ') ++e;
    return e && *e == 0 && e != s;
  }
  return false;
}

int code_of(const rtj::Value* v, const char* const names[4], const char* deflt) {
  std::string s = deflt;
  if (v) {
    if (v->kind != rtj::Value::Str) return 255;
    s = v->str;
  }
  for (int i = 0; i < 4; ++i)
    if (s == names[i]) return i;
  return 255;
}

const char* const WEATHERS[4] = {"Cloudy", "Stormy", "Sunny", "Windy"};
const char* const TRAFFICS[4] = {"High", "Jam", "Low", "Medium"};

#pragma pack(push, 1)
struct EtaRecord {
  float distance_m;
  float driver_age;
  int32_t wallclock_s;
  uint8_t weather, traffic;
  uint16_t pad;
};
#pragma pack(pop)
static_assert(sizeof(EtaRecord) == 16, "record layout");

// One /predict item -> record (+stamp) or error text.
std::string pack_item(const rtj::Value& it, const Stamp& now, EtaRecord& r, Stamp& st) {
  if (it.kind != rtj::Value::Obj) return "item must be a JSON object";
  double dist = 0.0;
  const rtj::Value* summ = it.get("summary");
  if (summ && summ->truthy()) {
    if (summ->kind != rtj::Value::Obj) return "summary must be an object";
    const rtj::Value* dv = summ->get("distance");
    if (dv && dv->truthy() && !num_of(dv, dist)) return "invalid summary.distance";
  }
  double age = 30.0;                      // float(body.get("driver_age", 30)) then `or 30.0`
  const rtj::Value* av = it.get("driver_age");
  if (av) {
    if (!num_of(av, age)) return "invalid driver_age";
    if (age == 0.0) age = 30.0;
  }
  const rtj::Value* pv = it.get("pickup_time");
  if (pv && pv->truthy() && pv->kind == rtj::Value::Str) {
    if (!parse_iso(pv->str, st)) return "Invalid isoformat string: '" + pv->str + "'";
  } else {
    st = now;                             // missing / falsy / non-string -> now() (ml.py:28-33)
  }
  r.distance_m = (float)dist;
  r.driver_age = (float)age;
  const int64_t rel = st.secs - EPOCH2020_DAYS * 86400;
  if (rel < INT32_MIN || rel > INT32_MAX) return "pickup_time out of range";
  r.wallclock_s = (int32_t)rel;
  r.weather = (uint8_t)code_of(it.get("weather"), WEATHERS, "Sunny");
  r.traffic = (uint8_t)code_of(it.get("traffic"), TRAFFICS, "Low");
  r.pad = 0;
  return "";
}

}  // namespace

// body -> (records uint8 [N,16], pickup_secs int64 [N], pickup_us int32 [N], tz int32 [N, 2]
//          (has_tz, offset_s), errors list[str], is_batch)
py::tuple pack_predict_batch(py::bytes body, int64_t now_secs, int32_t now_us) {
  std::string b = body;
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
  Stamp now;
  now.secs = now_secs;
  now.us = now_us;
  {
    auto R = rec.mutable_unchecked<2>();
    auto S = secs.mutable_unchecked<1>();
    auto U = us.mutable_unchecked<1>();
    auto T = tz.mutable_unchecked<2>();
    py::gil_scoped_release nogil;
    for (size_t i = 0; i < n; ++i) {
      EtaRecord r{};
      Stamp st;
      errs[i] = pack_item((*items)[i], now, r, st);
      std::memcpy(&R(i, 0), &r, 16);
      S(i) = st.secs;
      U(i) = st.us;
      T(i, 0) = st.has_tz ? 1 : 0;
      T(i, 1) = st.tz_sec;
    }
  }
  return py::make_tuple(rec, secs, us, tz, errs, is_batch);
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
    for (size_t i = 0; i < n; ++i) {
      if (i) o += ',';
      if (!errs[i].empty()) {
        o += "{\"error\":\"";
        for (char c : errs[i]) {
          if (c == '"' || c == '\\') o += '\\';
          if ((unsigned char)c >= 0x20) o += c;
        }
        o += "\"}";
        continue;
      }
      const double m = (double)M(i);
      Stamp tzs;
      tzs.has_tz = T(i, 0) != 0;
      tzs.tz_sec = T(i, 1);
      int64_t tot_us = (int64_t)U(i) + timedelta_minutes_us(m);
      int64_t s = S(i) + (tot_us >= 0 ? tot_us / 1000000 : -((-tot_us + 999999) / 1000000));
      int64_t u = tot_us - (s - S(i)) * 1000000;
      o += "{\"eta_minutes_ml\":";
      append_pyfloat(o, m);
      o += ",\"eta_completion_time_ml\":\"";
      o += isoformat(s, u, tzs);
      o += "\"}";
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

PYBIND11_MODULE(_rt, m) {
  m.doc() = "routest_amd CPU native runtime";
  m.def("pack_predict_batch", &pack_predict_batch, py::arg("body"), py::arg("now_secs"), py::arg("now_us"));
  m.def("format_predict_batch", &format_predict_batch);
  m.def("iso_parse", &iso_parse);
  m.def("iso_add_minutes", &iso_add_minutes);
  m.def("py_float_repr", &py_float_repr);
  m.def("greedy_trips", &greedy_trips);
  m.def("astar_batch", &astar_batch, py::arg("indptr"), py::arg("indices"), py::arg("cost"),
        py::arg("lat"), py::arg("lon"), py::arg("src"), py::arg("dst"), py::arg("inv_vmax"),
        py::arg("threads") = 8);
  m.attr("EPOCH2020_DAYS") = EPOCH2020_DAYS;
}
