// Host-only self-test + fuzz harness for the native runtime core (rt_core.h, json_lite.h) and the
// route service's host code (route_core.h: route-request parsing, Python-exact float fast paths;
// alternatives.h: via-node candidates and scores; history_db.h: the native history reads over a
// fuzzed database and fuzzed limits / ids).
// Built with -fsanitize=address,undefined by `tools/build_ext.py --sanitize` or the CMake `asan`
// preset (the reference has no race detection / sanitizers at all), and run by
// tests/test_sanitize_cpu.py.  Exit code 0 = all invariants held and no sanitizer report.
//
//   rt_selftest [iterations] [seed]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "alternatives.h"
#include "history_db.h"
#include "route_core.h"
#include "rt_core.h"

using namespace rtc;

static int g_fail = 0;
#define CHECK(c, ...)                                      \
  do {                                                     \
    if (!(c)) {                                            \
      std::fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      ++g_fail;                                            \
    }                                                      \
  } while (0)

static const char* SEEDS[] = {
    R"({"summary":{"distance":12345},"pickup_time":"2025-08-25T08:30:00","driver_age":34,"weather":"Sunny","traffic":"Medium"})",
    R"([{"summary":{"distance":1000.5}},{"summary":{"distance":"2500"},"traffic":"Jam","pickup_time":"2024-02-29 23:59:59.999999+05:30"}])",
    R"({"items":[{"summary":null,"driver_age":0,"weather":"Hail"},{"pickup_time":"2025-01-01T00:00:00Z"}]})",
    R"({"summary":{"distance":1e308},"driver_age":"abc","pickup_time":"not-a-date"})",
    R"([1, "x", null, true, {"a":[1,2,{"b":NaN}],"c":Infinity,"d":-Infinity,"e":"é\"\\"}])",
};

static void fuzz_json(std::mt19937_64& rng, int iters) {
  const Stamp now{1756110600, 123456, false, 0, 0};
  for (int it = 0; it < iters; ++it) {
    std::string s = SEEDS[rng() % (sizeof SEEDS / sizeof *SEEDS)];
    const int muts = (int)(rng() % 6);
    for (int k = 0; k < muts && !s.empty(); ++k) {
      const size_t p = rng() % s.size();
      switch (rng() % 4) {
        case 0: s[p] = (char)(rng() & 0xFF); break;                       // flip a byte
        case 1: s.erase(p, 1 + rng() % 8); break;                          // delete a run
        case 2: s.insert(p, s.substr(rng() % s.size(), 1 + rng() % 16)); break;  // duplicate
        default: s.resize(p); break;                                       // truncate
      }
    }
    rtj::Value root;
    bool full_ok = true;
    try {
      root = rtj::Parser(s.data(), s.size()).parse();
    } catch (...) {
      full_ok = false;  // malformed JSON is rejected, never read out of bounds
    }
    // the parallel item splitter must agree with the full parser whenever it accepts a body
    std::vector<std::pair<size_t, size_t>> spans;
    if (split_top_array(s.data(), s.size(), spans)) {
      bool items_ok = true;
      for (auto& sp : spans) {
        try {
          rtj::Parser(s.data() + sp.first, sp.second - sp.first).parse();
        } catch (...) {
          items_ok = false;
        }
      }
      CHECK(items_ok == full_ok, "splitter/parser disagree on validity: %s", s.c_str());
      if (items_ok && full_ok)
        CHECK(root.kind == rtj::Value::Arr && root.arr.size() == spans.size(), "item count %zu vs %zu",
              root.arr.size(), spans.size());
    }
    if (!full_ok) continue;
    std::vector<const rtj::Value*> items;
    if (root.kind == rtj::Value::Arr)
      for (auto& v : root.arr) items.push_back(&v);
    else
      items.push_back(&root);
    std::string out;
    for (const rtj::Value* v : items) {
      EtaRecord r{};
      Stamp st;
      std::string err = pack_item(*v, now, r, st);
      if (err.empty()) {
        CHECK(r.weather <= 3 || r.weather == 255, "weather code %d", r.weather);
        CHECK(r.traffic <= 3 || r.traffic == 255, "traffic code %d", r.traffic);
      }
      static const double MINS[] = {17.25, 0.0, -3.5, 1e30, NAN, INFINITY, 1234567.891};
      format_one(out, MINS[rng() % 7], st.secs, st.us, st.has_tz, st.tz_sec, err);
    }
  }
}

static void fuzz_iso(std::mt19937_64& rng, int iters) {
  static const char alpha[] = "0123456789-:T .Z+z,";
  for (int it = 0; it < iters; ++it) {
    std::string s;
    const int n = (int)(rng() % 40);
    for (int k = 0; k < n; ++k) s += alpha[rng() % (sizeof alpha - 1)];
    Stamp st;
    if (parse_iso(s, st)) {
      // a parsed stamp re-formats to a string that parses to the same instant
      std::string f = isoformat(st.secs, st.us, st);
      Stamp st2;
      CHECK(parse_iso(f, st2) && st2.secs == st.secs && st2.us == st.us && st2.tz_sec == st.tz_sec,
            "iso round trip '%s' -> '%s'", s.c_str(), f.c_str());
    }
  }
  // calendar round trip over 600 years
  for (int64_t d = -80000; d < 140000; d += 17) {
    int64_t y;
    unsigned m, dd;
    civil_from_days(d, y, m, dd);
    CHECK(days_from_civil(y, m, dd) == d, "civil round trip %lld", (long long)d);
  }
}

static void fuzz_float(std::mt19937_64& rng, int iters) {
  for (int it = 0; it < iters; ++it) {
    double v;
    switch (rng() % 3) {
      case 0: { uint64_t b = rng(); std::memcpy(&v, &b, 8); break; }         // any bit pattern
      case 1: v = std::ldexp((double)(rng() % 100000), (int)(rng() % 80) - 40); break;
      default: v = (double)(float)((rng() % 200000) / 997.0); break;           // float32 minutes
    }
    std::string o;
    append_pyfloat(o, v);
    if (std::isfinite(v)) {
      CHECK(std::strtod(o.c_str(), nullptr) == v, "repr round trip %.17g -> %s", v, o.c_str());
    }
    const int64_t us = timedelta_minutes_us(std::isfinite(v) && std::fabs(v) < 1e9 ? v : 1.5);
    (void)us;
  }
  CHECK(timedelta_minutes_us(0.5) == 30000000, "timedelta 0.5 min");
  CHECK(timedelta_minutes_us(1.0 / 60000000.0 * 2.5) == 2, "half-even rounding");
}

// route_core.h: py_round(x, 1)'s fast path, put_float's integer-tenths path and put_coord's
// six-decimal path must give the bits / text of their slow (CPython-equivalent) references, and
// parse_route_request must survive any mutated request body.
// route_core.h CoordCache: a route's coordinates copied from the per-node strings equal the
// formatted ones, byte for byte (nodes near 0, negative, with trailing zeros, repr-form values)
static void fuzz_coord_cache(std::mt19937_64& rng, int iters) {
  const size_t N = 512;
  std::vector<double> lat(N), lon(N);
  std::uniform_real_distribution<double> U(-180.0, 180.0);
  for (size_t n = 0; n < N; ++n) {
    switch (n % 5) {
      case 0: lat[n] = U(rng) / 2; lon[n] = U(rng); break;
      case 1: lat[n] = std::round(U(rng) * 1e3) / 1e3; lon[n] = std::round(U(rng) * 10) / 10; break;
      case 2: lat[n] = U(rng) * 1e-6; lon[n] = -U(rng) * 1e-5; break;
      case 3: lat[n] = 14.5 + U(rng) * 1e-4; lon[n] = 121.0 + U(rng) * 1e-4; break;
      default: lat[n] = 0.0; lon[n] = -0.0; break;
    }
  }
  rtr::CoordCache cc;
  cc.build(lat.data(), lon.data(), N);
  for (int it = 0; it < iters; ++it) {
    std::vector<double> xy;
    std::vector<uint8_t> raw;
    std::vector<int32_t> node;
    const int len = 1 + (int)(rng() % 40);
    for (int i = 0; i < len; ++i) {
      if (rng() % 4 == 0) {
        xy.push_back(U(rng));
        xy.push_back(U(rng) / 2);
        raw.push_back(1);
        node.push_back(-1);
      } else {
        const int n = (int)(rng() % N);
        xy.push_back(rtr::np_round6(lon[n]));
        xy.push_back(rtr::np_round6(lat[n]));
        raw.push_back(0);
        node.push_back(n);
      }
    }
    std::string a, b;
    rtr::put_coords(a, xy, raw);
    rtr::put_coords(b, xy, raw, &node, &cc);
    CHECK(a == b, "coord cache: %s vs %s", a.c_str(), b.c_str());
  }
}

static void fuzz_route(std::mt19937_64& rng, int iters) {
  for (int it = 0; it < iters; ++it) {
    double x;
    switch (rng() % 4) {
      case 0: x = ((double)(int64_t)(rng() % 2000000000) - 1e9) / 997.0; break;
      case 1: x = ((double)(int64_t)(rng() % 20000001) - 1e7 + 0.5) / 10.0; break;     // midpoints
      case 2: x = std::nextafter(((double)(rng() % 100000) + 0.05), rng() & 1 ? 1e9 : -1e9); break;
      default: { uint64_t b = rng(); std::memcpy(&x, &b, 8); break; }
    }
    if (!std::isfinite(x)) continue;
    char b[64];
    std::snprintf(b, sizeof b, "%.1f", x);
    const double slow = std::strtod(b, nullptr);
    const double fast = rtr::py_round(x, 1);
    CHECK(std::memcmp(&slow, &fast, 8) == 0 || (slow == 0.0 && fast == 0.0 && std::signbit(slow) == std::signbit(fast)),
          "py_round(%.17g, 1): fast %.17g, slow %.17g", x, fast, slow);
    std::string a1, a2;
    rtr::put_float(a1, fast);
    rtc::append_pyfloat(a2, fast);
    CHECK(a1 == a2, "put_float(%.17g): %s vs repr %s", fast, a1.c_str(), a2.c_str());
    const double c = rtr::np_round6(x / 1000.0);
    std::string c1, c2;
    rtr::put_coord(c1, c);
    rtc::append_pyfloat(c2, c);
    CHECK(c1 == c2, "put_coord(%.17g): %s vs repr %s", c, c1.c_str(), c2.c_str());
  }
  static const char* RSEEDS[] = {
      R"({"source_point":{"lat":14.55,"lon":121.02},"destination_points":[{"lat":14.56,"lon":121.03,"payload":2},{"lat":14.57,"lon":121.0}],"vehicle_capacity":5,"maximum_distance":90000,"use_ml_eta":true,"context":{"weather":"Stormy","traffic":"High"},"alternatives":3})",
      R"({"source_point":{"lat":"14.5","lon":121},"destination_points":[],"vehicle_type":"motorcycle","driver_details":{"driver_age":"41"},"meta":{"origin_id":7,"destination_ids":[1,2]}})",
      R"({"source_point":null,"destination_points":[{"lat":1e308,"lon":-1e308}],"vehicle_capacity":-1,"alternatives":1e30})",
  };
  for (int it = 0; it < iters; ++it) {
    std::string s = RSEEDS[rng() % (sizeof RSEEDS / sizeof *RSEEDS)];
    const int muts = (int)(rng() % 5);
    for (int k = 0; k < muts && !s.empty(); ++k) {
      const size_t p = rng() % s.size();
      switch (rng() % 3) {
        case 0: s[p] = (char)(rng() & 0xFF); break;
        case 1: s.erase(p, 1 + rng() % 6); break;
        default: s.insert(p, s.substr(rng() % s.size(), 1 + rng() % 12)); break;
      }
    }
    try {
      rtj::Value root = rtj::Parser(s.data(), s.size()).parse();
      const rtr::RouteReq r = rtr::parse_route_request(&root);
      CHECK(r.error.empty() || r.dst.empty() || true, "unreachable");
    } catch (...) {
    }
  }
}

// alternatives.h: via nodes stay in range, unique, within the detour band, and reproducible; the
// argmin treats non-finite scores as +inf
static void fuzz_alternatives(std::mt19937_64& rng, int iters) {
  for (int it = 0; it < iters / 50; ++it) {
    const int N = 1 + (int)(rng() % 2000);
    std::vector<double> lat(N), lon(N);
    for (int i = 0; i < N; ++i) {
      lat[i] = 14.5 + (double)(rng() % 100000) * 1e-6 * (rng() % 5 == 0 ? 0.0 : 1.0);
      lon[i] = 121.0 + (double)(rng() % 100000) * 1e-6;
    }
    const int s = (int)(rng() % (N + 4)) - 2, t = (int)(rng() % (N + 4)) - 2, n = (int)(rng() % 12) - 1;
    const double stretch = 1.0 + (double)(rng() % 1000) / 1000.0;
    const std::vector<int> v = ralt::via_nodes(lat.data(), lon.data(), N, s, t, n, stretch);
    CHECK((int)v.size() <= std::max(n, 0), "via_nodes: %zu > n %d", v.size(), n);
    std::vector<int> seen(v);
    std::sort(seen.begin(), seen.end());
    CHECK(std::unique(seen.begin(), seen.end()) == seen.end(), "via_nodes: duplicate candidate");
    for (int w : v) {
      CHECK(w >= 0 && w < N, "via_nodes: %d out of [0, %d)", w, N);
      if (w < 0 || w >= N) break;
      const double d_st = rtr::haversine_m(lat[s], lon[s], lat[t], lon[t]);
      const double det = rtr::haversine_m(lat[s], lon[s], lat[w], lon[w]) + rtr::haversine_m(lat[w], lon[w], lat[t], lon[t]);
      CHECK(det <= stretch * d_st && det >= 1.03 * d_st, "via_nodes: detour %.3f outside band of %.3f", det, d_st);
    }
    CHECK(v == ralt::via_nodes(lat.data(), lon.data(), N, s, t, n, stretch), "via_nodes: not reproducible");
    std::vector<double> sc(rng() % 9);
    for (double& x : sc) {
      const int k = (int)(rng() % 4);
      x = k == 0 ? NAN : k == 1 ? INFINITY : (double)(rng() % 1000);
    }
    const int b = ralt::argmin_score(sc);
    CHECK(sc.empty() ? b == -1 : (b >= 0 && b < (int)sc.size()), "argmin_score: %d of %zu", b, sc.size());
  }
}

// history_db.h over an in-memory database with the store's schema (routest_amd/store/store.py
// SCHEMA): rows with fuzzed texts (any bytes, non-JSON stops), then list / detail / delete /
// locations with fuzzed limit strings and ids — every reply a valid status, nothing read out of
// bounds.  Skipped when libsqlite3 cannot be loaded.
static void fuzz_history(std::mt19937_64& rng, int iters) {
  rtsql::Api sql;
  std::string err;
  if (!sql.load(err)) {
    std::printf("fuzz_history: skipped (%s)\n", err.c_str());
    return;
  }
  const std::string uri = "file:rt_selftest_hist?mode=memory&cache=shared";
  void* db = nullptr;
  if (sql.open_v2(uri.c_str(), &db, rtsql::OPEN_READWRITE | rtsql::OPEN_CREATE | rtsql::OPEN_URI, nullptr) != rtsql::OK) {
    std::printf("fuzz_history: skipped (open)\n");
    return;
  }
  const char* ddl =
      "CREATE TABLE locations (id TEXT PRIMARY KEY, name TEXT NOT NULL, latitude REAL NOT NULL, longitude REAL NOT NULL, created_at TEXT);"
      "CREATE TABLE route_requests (id TEXT PRIMARY KEY, origin_id TEXT, stops TEXT NOT NULL, request_time TEXT NOT NULL,"
      " status TEXT NOT NULL DEFAULT 'pending', engine TEXT, vehicle_id TEXT, driver_age REAL);"
      "CREATE TABLE route_results (id TEXT PRIMARY KEY, request_id TEXT NOT NULL REFERENCES route_requests(id) ON DELETE CASCADE,"
      " optimized_order TEXT, total_distance REAL, total_duration REAL, legs TEXT, geometry TEXT, eta_minutes_ml REAL,"
      " eta_completion_time_ml TEXT, created_at TEXT);";
  CHECK(sql.exec(db, ddl, nullptr, nullptr, nullptr) == rtsql::OK, "history schema");
  void *ins_req = nullptr, *ins_res = nullptr, *ins_loc = nullptr;
  sql.prepare_v2(db, "INSERT INTO route_requests(id,origin_id,stops,request_time,status,engine,vehicle_id,driver_age) VALUES(?,?,?,?,?,?,?,?)", -1, &ins_req, nullptr);
  sql.prepare_v2(db, "INSERT INTO route_results(id,request_id,optimized_order,total_distance,total_duration,legs,geometry,eta_minutes_ml,eta_completion_time_ml,created_at) VALUES(?,?,?,?,?,?,?,?,?,?)", -1, &ins_res, nullptr);
  sql.prepare_v2(db, "INSERT INTO locations(id,name,latitude,longitude,created_at) VALUES(?,?,?,?,?)", -1, &ins_loc, nullptr);
  auto junk = [&](size_t maxlen) {
    static const char* frags[] = {"{\"destination_ids\":[1,2],\"destination_points\":[[14.5,121.0]]}", "[0,2,1]", "null",
                                  "{\"type\":\"LineString\",\"coordinates\":[]}", "2026-10-17T00:00:00", "\"\\u00e9\"", "{"};
    std::string t = rng() % 2 ? frags[rng() % 7] : "";
    const size_t n = rng() % maxlen;
    for (size_t i = 0; i < n; ++i) t += (char)(rng() & 0xFF);
    return t;
  };
  std::vector<std::string> ids;
  for (int i = 0; i < 60; ++i) {
    const std::string rid = "req-" + std::to_string(i), stops = junk(40), tm = junk(24), st = junk(8), eng = junk(8);
    sql.reset(ins_req);
    sql.clear_bindings(ins_req);
    sql.bind_text(ins_req, 1, rid.data(), (int)rid.size(), rtsql::TRANSIENT);
    if (rng() % 2) sql.bind_null(ins_req, 2); else sql.bind_int64(ins_req, 2, (long long)(rng() % 100));
    sql.bind_text(ins_req, 3, stops.data(), (int)stops.size(), rtsql::TRANSIENT);
    sql.bind_text(ins_req, 4, tm.data(), (int)tm.size(), rtsql::TRANSIENT);
    sql.bind_text(ins_req, 5, st.data(), (int)st.size(), rtsql::TRANSIENT);
    sql.bind_text(ins_req, 6, eng.data(), (int)eng.size(), rtsql::TRANSIENT);
    sql.bind_null(ins_req, 7);
    if (rng() % 3) sql.bind_double(ins_req, 8, (double)(rng() % 90)); else sql.bind_null(ins_req, 8);
    CHECK(sql.step(ins_req) == rtsql::DONE, "insert request");
    ids.push_back(rid);
    if (rng() % 4) {
      const std::string xid = "res-" + std::to_string(i), order = junk(16), legs = junk(64), geom = junk(64), iso = junk(24);
      sql.reset(ins_res);
      sql.clear_bindings(ins_res);
      sql.bind_text(ins_res, 1, xid.data(), (int)xid.size(), rtsql::TRANSIENT);
      sql.bind_text(ins_res, 2, rid.data(), (int)rid.size(), rtsql::TRANSIENT);
      sql.bind_text(ins_res, 3, order.data(), (int)order.size(), rtsql::TRANSIENT);
      sql.bind_double(ins_res, 4, (double)(rng() % 100000) / 7.0);
      if (rng() % 5) sql.bind_double(ins_res, 5, (double)(rng() % 100000) / 3.0); else sql.bind_null(ins_res, 5);
      sql.bind_text(ins_res, 6, legs.data(), (int)legs.size(), rtsql::TRANSIENT);
      sql.bind_text(ins_res, 7, geom.data(), (int)geom.size(), rtsql::TRANSIENT);
      if (rng() % 2) sql.bind_double(ins_res, 8, (double)(rng() % 1000) / 9.0); else sql.bind_null(ins_res, 8);
      sql.bind_text(ins_res, 9, iso.data(), (int)iso.size(), rtsql::TRANSIENT);
      sql.bind_text(ins_res, 10, iso.data(), (int)iso.size(), rtsql::TRANSIENT);
      CHECK(sql.step(ins_res) == rtsql::DONE, "insert result");
    }
    if (i % 6 == 0) {
      const std::string lid = "loc-" + std::to_string(i), name = junk(12);
      sql.reset(ins_loc);
      sql.clear_bindings(ins_loc);
      sql.bind_text(ins_loc, 1, lid.data(), (int)lid.size(), rtsql::TRANSIENT);
      sql.bind_text(ins_loc, 2, name.data(), (int)name.size(), rtsql::TRANSIENT);
      sql.bind_double(ins_loc, 3, 14.5);
      sql.bind_double(ins_loc, 4, 121.0);
      sql.bind_null(ins_loc, 5);
      CHECK(sql.step(ins_loc) == rtsql::DONE, "insert location");
    }
  }
  for (void* st : {ins_req, ins_res, ins_loc}) sql.finalize(st);
  rth::HistoryDb h;
  CHECK(h.open(uri, err), "history open: %s", err.c_str());
  auto valid = [](const rth::Reply& r) { return r.fallback || (r.status >= 200 && r.status < 600); };
  static const char* LIMITS[] = {"", "0", "-2", "3", "20", "100000", "abc", "2.5", "1_0", " 7", "99999999999999999999999", "+4"};
  for (int it = 0; it < iters / 100; ++it) {
    switch (rng() % 5) {
      case 0: {
        const bool absent = rng() % 6 == 0;
        std::string lim = LIMITS[rng() % (sizeof LIMITS / sizeof *LIMITS)];
        if (rng() % 4 == 0) lim = junk(10);
        CHECK(valid(h.history(absent ? nullptr : lim.c_str())), "history(%s)", lim.c_str());
        break;
      }
      case 1: CHECK(valid(h.detail(rng() % 2 ? ids[rng() % ids.size()] : junk(50))), "detail"); break;
      case 2: CHECK(valid(h.del(rng() % 3 ? ids[rng() % ids.size()] : junk(50))), "delete"); break;
      default: CHECK(valid(h.locations()), "locations"); break;
    }
  }
  h.close();
  sql.close(db);
}

// The batched /predict path splits a big array with split_top_array and packs / formats items on
// parallel_chunks threads (rt.cpp); replay that shape here so TSan sees the real sharing pattern.
static void threaded_pack_format(int n_items) {
  std::string body = "[";
  for (int i = 0; i < n_items; ++i) {
    if (i) body += ',';
    body += "{\"summary\":{\"distance\":" + std::to_string(1000 + i) +
            "},\"pickup_time\":\"2025-08-25T08:30:00+02:00\",\"traffic\":\"High\"}";
  }
  body += "]";
  std::vector<std::pair<size_t, size_t>> spans;
  CHECK(split_top_array(body.data(), body.size(), spans) && (int)spans.size() == n_items, "split");
  const Stamp now{1756110600, 0, false, 0, 0};
  std::vector<EtaRecord> recs(spans.size());
  std::vector<Stamp> st(spans.size());
  std::vector<std::string> errs(spans.size());
  parallel_chunks(spans.size(), 64, 8, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      rtj::Value v = rtj::Parser(body.data() + spans[i].first, spans[i].second - spans[i].first).parse();
      errs[i] = pack_item(v, now, recs[i], st[i]);
    }
  });
  std::vector<std::string> parts(8);
  const size_t per = (spans.size() + 7) / 8;
  parallel_chunks(8, 1, 8, [&](size_t klo, size_t khi) {
    for (size_t k = klo; k < khi; ++k)
      for (size_t i = k * per; i < std::min(spans.size(), (k + 1) * per); ++i)
        format_one(parts[k], 12.5 + (double)i, st[i].secs, st[i].us, st[i].has_tz, st[i].tz_sec, errs[i]);
  });
  size_t ok = 0;
  for (auto& e : errs) ok += e.empty();
  CHECK(ok == spans.size(), "threaded pack errors");
  CHECK(recs[n_items - 1].distance_m == (float)(1000 + n_items - 1), "threaded pack record");
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
  std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1234);
  fuzz_json(rng, iters);
  fuzz_iso(rng, iters);
  fuzz_float(rng, iters);
  fuzz_route(rng, iters);
  fuzz_coord_cache(rng, iters);
  fuzz_alternatives(rng, iters);
  fuzz_history(rng, iters);
  threaded_pack_format(20000);
  std::printf("rt_selftest: %d iterations, %d failures\n", iters, g_fail);
  return g_fail ? 1 : 0;
}
