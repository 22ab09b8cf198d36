// Pure C++ core of the routest_amd._rt runtime (no Python): ISO-8601 parsing, CPython-exact
// timedelta rounding / isoformat / float repr, /predict item -> 16-byte EtaRecord packing and
// response formatting.  Kept header-only and free of pybind11 so the same code is linked into the
// extension (rt.cpp) and into the ASan/UBSan fuzz harness (rt_selftest.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <charconv>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "json_lite.h"

namespace rtc {

// ------------------------------------------------------------------ civil calendar
inline int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}
inline void civil_from_days(int64_t z, int64_t& y, unsigned& m, unsigned& d) {
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
inline const int64_t EPOCH2020_DAYS = days_from_civil(2020, 1, 1);

struct Stamp {          // naive wall-clock fields + optional UTC offset (as written)
  int64_t secs = 0;     // wall-clock seconds since 1970-01-01 (tz ignored)
  int32_t us = 0;
  bool has_tz = false;
  int32_t tz_sec = 0;   // offset in seconds
  int32_t tz_us = 0;
};

inline bool digits(const std::string& s, size_t p, size_t n, int& out) {
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
inline bool parse_iso(const std::string& s, Stamp& st) {
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
inline int64_t timedelta_minutes_us(double x) {
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

inline void append_2(std::string& o, int v) {
  o += (char)('0' + v / 10);
  o += (char)('0' + v % 10);
}

// datetime.isoformat() of (secs, us) [+ offset]
inline void append_isoformat(std::string& o, int64_t secs, int64_t us, const Stamp& tz) {
  int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
  int64_t sod = secs - days * 86400;
  int64_t y;
  unsigned m, d;
  civil_from_days(days, y, m, d);
  char b[48];
  int k = 0;
  if (y < 0 || y > 9999) {
    k = std::snprintf(b, sizeof b, "%04lld", (long long)y);
  } else {
    b[k++] = (char)('0' + y / 1000);
    b[k++] = (char)('0' + y / 100 % 10);
    b[k++] = (char)('0' + y / 10 % 10);
    b[k++] = (char)('0' + y % 10);
  }
  auto two = [&](int v) { b[k++] = (char)('0' + v / 10); b[k++] = (char)('0' + v % 10); };
  b[k++] = '-'; two((int)m); b[k++] = '-'; two((int)d); b[k++] = 'T';
  two((int)(sod / 3600)); b[k++] = ':'; two((int)(sod / 60 % 60)); b[k++] = ':'; two((int)(sod % 60));
  if (us) {
    b[k++] = '.';
    int64_t u = us;
    for (int div = 100000; div; div /= 10) { b[k++] = (char)('0' + u / div % 10); }
  }
  if (tz.has_tz) {
    int off = tz.tz_sec;
    b[k++] = off < 0 ? '-' : '+';
    off = std::abs(off);
    two(off / 3600); b[k++] = ':'; two(off / 60 % 60);
    if (off % 60) { b[k++] = ':'; two(off % 60); }
  }
  o.append(b, k);
}

// datetime.isoformat() of (secs, us) [+ offset]
inline std::string isoformat(int64_t secs, int64_t us, const Stamp& tz) {
  std::string o;
  append_isoformat(o, secs, us, tz);
  return o;
}

// Python repr(float): shortest round-trip digits (to_chars), laid out with CPython's rule — fixed
// notation when -4 <= exponent < 16, else d[.ddd]e[+-]XX.  Char buffers only (no allocation).
inline void append_pyfloat(std::string& o, double v) {
  if (std::isnan(v)) { o += "NaN"; return; }
  if (std::isinf(v)) { o += v > 0 ? "Infinity" : "-Infinity"; return; }
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  const char* p = buf;
  const char* end = r.ptr;
  const char* epos = p;
  while (epos < end && *epos != 'e') ++epos;
  int exp = 0;
  std::from_chars(epos + 1 + (epos[1] == '+'), end, exp);
  if (*p == '-') { o += '-'; ++p; }
  char digs[32];
  int nd = 0;
  for (const char* q = p; q < epos; ++q)
    if (*q != '.') digs[nd++] = *q;
  char out[64];
  int k = 0;
  if (exp >= -4 && exp < 16) {
    if (exp >= 0) {
      if (nd <= exp + 1) {
        for (int i = 0; i < nd; ++i) out[k++] = digs[i];
        for (int i = nd; i < exp + 1; ++i) out[k++] = '0';
        out[k++] = '.';
        out[k++] = '0';
      } else {
        for (int i = 0; i < exp + 1; ++i) out[k++] = digs[i];
        out[k++] = '.';
        for (int i = exp + 1; i < nd; ++i) out[k++] = digs[i];
      }
    } else {
      out[k++] = '0';
      out[k++] = '.';
      for (int i = 0; i < -exp - 1; ++i) out[k++] = '0';
      for (int i = 0; i < nd; ++i) out[k++] = digs[i];
    }
  } else {
    out[k++] = digs[0];
    if (nd > 1) {
      out[k++] = '.';
      for (int i = 1; i < nd; ++i) out[k++] = digs[i];
    }
    out[k++] = 'e';
    out[k++] = exp < 0 ? '-' : '+';
    const int ae = exp < 0 ? -exp : exp;
    if (ae >= 100) out[k++] = (char)('0' + ae / 100);
    out[k++] = (char)('0' + ae / 10 % 10);
    out[k++] = (char)('0' + ae % 10);
  }
  o.append(out, k);
}

inline bool num_of(const rtj::Value* v, double& out) {
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

inline int code_of(const rtj::Value* v, const char* const names[4], const char* deflt) {
  std::string s = deflt;
  if (v) {
    if (v->kind != rtj::Value::Str) return 255;
    s = v->str;
  }
  for (int i = 0; i < 4; ++i)
    if (s == names[i]) return i;
  return 255;
}

inline const char* const WEATHERS[4] = {"Cloudy", "Stormy", "Sunny", "Windy"};
inline const char* const TRAFFICS[4] = {"High", "Jam", "Low", "Medium"};

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

// 8-byte wire record (routest_amd/models/features.py RECORD8_DTYPE, csrc/common.h featurize8_f32):
// distance_m (f32) | fp16(age) | hours since the batch's base Monday << 16 | weather << 26 |
// traffic << 29.  Used for every batch it represents exactly (halves the PCIe bytes per request).
#pragma pack(push, 1)
struct Wire8 {
  float distance_m;
  uint32_t packed;
};
#pragma pack(pop)
static_assert(sizeof(Wire8) == 8, "wire8 layout");

// f32 -> fp16 bits, only if the value is exactly representable (no rounding anywhere).
inline bool f16_exact(float v, uint16_t& h) {
  uint32_t b;
  std::memcpy(&b, &v, 4);
  const uint16_t sign = (uint16_t)((b >> 16) & 0x8000u);
  const int exp = (int)((b >> 23) & 0xffu);
  const uint32_t man = b & 0x7fffffu;
  if (exp == 0 && man == 0) { h = sign; return true; }
  if (exp == 0 || exp == 255) return false;             // f32 subnormal / inf / nan
  const int e = exp - 127;
  if (e > 15) return false;
  if (e >= -14) {                                        // normal half
    if (man & 0x1fffu) return false;
    h = (uint16_t)(sign | (uint16_t)((e + 15) << 10) | (uint16_t)(man >> 13));
    return true;
  }
  const int s = -(e + 1);                                // subnormal half: m = full >> s
  if (s > 24) return false;
  const uint32_t full = man | 0x800000u;
  if (full & ((1u << s) - 1u)) return false;
  h = (uint16_t)(sign | (uint16_t)(full >> s));
  return true;
}

inline int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// Pack n 16-byte records as wire8 into `out`; false (out untouched beyond n) if any record is not
// exactly representable.  The base is 00:00 of the Monday on or before the earliest pickup (the
// records' epoch 2020-01-01 is a Wednesday: day d has weekday (d + 2) % 7).
inline bool pack_wire8(const EtaRecord* r, size_t n, Wire8* out) {
  if (n == 0) return true;
  int64_t hmin = INT64_MAX;
  for (size_t i = 0; i < n; ++i) hmin = std::min(hmin, floor_div(r[i].wallclock_s, 3600));
  const int64_t d0 = floor_div(hmin, 24);
  const int64_t base = (d0 - ((d0 + 2) % 7 + 7) % 7) * 24;
  for (size_t i = 0; i < n; ++i) {
    uint16_t a;
    if (!f16_exact(r[i].driver_age, a)) return false;
    const int64_t hrs = floor_div(r[i].wallclock_s, 3600) - base;
    if (hrs < 0 || hrs >= 1024) return false;
    const uint32_t w = r[i].weather > 3 ? 7u : r[i].weather;
    const uint32_t t = r[i].traffic > 3 ? 7u : r[i].traffic;
    out[i].distance_m = r[i].distance_m;
    out[i].packed = (uint32_t)a | ((uint32_t)hrs << 16) | (w << 26) | (t << 29);
  }
  return true;
}

// One /predict item -> record (+stamp) or error text.
inline std::string pack_item(const rtj::Value& it, const Stamp& now, EtaRecord& r, Stamp& st) {
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

// One prediction -> the reference's response object (appended to o).
inline void format_one(std::string& o, double m, int64_t secs, int32_t us, bool has_tz, int32_t tz_sec,
                       const std::string& err) {
  if (!err.empty()) {
    o += "{\"error\":\"";
    for (char c : err) {
      if (c == '"' || c == '\\') o += '\\';
      if ((unsigned char)c >= 0x20) o += c;
    }
    o += "\"}";
    return;
  }
  // timedelta(minutes=m) raises for NaN/inf/overflow in Python (the reference then answers 503);
  // never let a diverged model reach the int64 casts below (UB).
  if (!std::isfinite(m) || std::fabs(m) > 1.4e9) {
    o += "{\"error\":\"prediction out of range\"}";
    return;
  }
  Stamp tzs;
  tzs.has_tz = has_tz;
  tzs.tz_sec = tz_sec;
  const int64_t tot_us = (int64_t)us + timedelta_minutes_us(m);
  const int64_t s = secs + (tot_us >= 0 ? tot_us / 1000000 : -((-tot_us + 999999) / 1000000));
  const int64_t u = tot_us - (s - secs) * 1000000;
  o += "{\"eta_minutes_ml\":";
  append_pyfloat(o, m);
  o += ",\"eta_completion_time_ml\":\"";
  append_isoformat(o, s, u, tzs);
  o += "\"}";
}


// Split a top-level JSON array into item spans with one string-aware pass (no DOM), so items can
// be parsed in parallel.  Returns false on anything unusual; callers then run the full parser,
// which produces the proper error.
inline bool split_top_array(const char* s, size_t n, std::vector<std::pair<size_t, size_t>>& spans) {
  size_t p = 0;
  auto ws = [&]() { while (p < n && (s[p] == ' ' || s[p] == '\n' || s[p] == '\r' || s[p] == '\t')) ++p; };
  ws();
  if (p >= n || s[p] != '[') return false;
  ++p;
  ws();
  if (p < n && s[p] == ']') {
    ++p;
    ws();
    return p == n;
  }
  size_t start = p;
  int depth = 0;
  bool in_str = false;
  for (; p < n; ++p) {
    const char c = s[p];
    if (in_str) {
      if (c == '\\') ++p;
      else if (c == '"') in_str = false;
      continue;
    }
    if (c == '"') in_str = true;
    else if (c == '{' || c == '[') ++depth;
    else if (c == '}' || c == ']') {
      if (depth == 0) {             // the closing bracket of the top-level array
        if (c != ']') return false;
        spans.emplace_back(start, p);
        ++p;
        ws();
        return p == n;
      }
      --depth;
    } else if (c == ',' && depth == 0) {
      spans.emplace_back(start, p);
      start = p + 1;
    }
  }
  return false;
}

// A process-wide pool of worker threads (ROUTEST_CPU_POOL, default min(cores, 16)) for
// parallel_chunks: the route service calls it several times per flush (snapping, plan unpacking,
// assembly, row texts), and a fresh std::thread per chunk per call cost ~20 us each — thousands of
// thread creations per second competing for the CPU with the SQLite writer.  Leaked on purpose: its
// workers are detached and wait on it until the process ends.
class WorkPool {
 public:
  static WorkPool& get() {
    static WorkPool* p = new WorkPool();
    return *p;
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  WorkPool() {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const char* v = std::getenv("ROUTEST_CPU_POOL");
    const unsigned n = v ? (unsigned)std::max(1, std::atoi(v)) : std::min(hw, 16u);
    for (unsigned i = 0; i < n; ++i) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    while (true) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

// Run fn(begin, end) over [0, n) in up to `max_threads` chunks (serial below `min_per_thread`):
// the pool's workers and the caller take chunks from a shared counter, the caller returns when all
// are done.  The caller always works too, so a call made from a pool worker (or in a forked child
// whose pool has no workers) still finishes; a helper that starts late finds no chunk left and
// never touches fn.
template <class F>
inline void parallel_chunks(size_t n, size_t min_per_thread, unsigned max_threads, F fn) {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  size_t t = std::min<size_t>({(size_t)std::min(hw, max_threads), n / std::max<size_t>(1, min_per_thread)});
  if (t <= 1) {
    fn((size_t)0, n);
    return;
  }
  const size_t per = (n + t - 1) / t;
  const size_t chunks = (n + per - 1) / per;
  struct State {
    std::atomic<size_t> next{0}, done{0};
    std::mutex m;
    std::condition_variable cv;
    std::exception_ptr err;               // the first chunk's exception (rethrown by the caller)
  };
  auto st = std::make_shared<State>();
  F* fp = &fn;
  // a chunk that throws still counts as done (its exception kept), so the caller never unwinds its
  // frame — fn and what it captures — while a pool worker may still be calling (*fp)
  auto work = [st, fp, chunks, per, n]() {
    size_t k;
    while ((k = st->next.fetch_add(1)) < chunks) {
      try {
        (*fp)(k * per, std::min(n, (k + 1) * per));
      } catch (...) {
        std::lock_guard<std::mutex> lk(st->m);
        if (!st->err) st->err = std::current_exception();
      }
      if (st->done.fetch_add(1) + 1 == chunks) {
        std::lock_guard<std::mutex> lk(st->m);
        st->cv.notify_all();
      }
    }
  };
  for (size_t k = 1; k < chunks; ++k) WorkPool::get().submit(work);
  work();
  std::unique_lock<std::mutex> lk(st->m);
  st->cv.wait(lk, [&] { return st->done.load() == chunks; });
  if (st->err) std::rethrow_exception(st->err);
}

}  // namespace rtc
