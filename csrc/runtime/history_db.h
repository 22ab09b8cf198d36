// Native history / locations reads over the store's SQLite database: the long-tail routes the
// native front end used to relay to the single Python process (verdict r3 item 8).  Bodies are
// byte-identical to the FastAPI handlers (routest_amd/api/app.py history / history_detail /
// delete_history / locations over routest_amd/store/store.py SQLiteStore; reference
// RO/Flaskr/routes.py:185-279,386-406 and the Next/Laravel /api/locations): the same queries, the
// stored JSON columns parsed and re-emitted like json.loads + json.dumps, SQLite REAL -> Python
// float repr, INTEGER -> int, NULL -> null.  Anything unusual (a malformed stored row, an odd limit
// string, an SQL error) returns `fallback` so the Python app answers with its own error semantics.
#pragma once
#include <fcntl.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "json_lite.h"
#include "route_core.h"
#include "route_record.h"
#include "sqlite_lite.h"

namespace rth {

struct Reply {
  bool fallback = false;
  int status = 200;
  std::string body;
};

class HistoryDb {
 public:
  ~HistoryDb() { close(); }

  bool open(const std::string& path, std::string& err) {
    if (!sql_.load(err)) return false;
    if (sql_.open_v2(path.c_str(), &db_, rtsql::OPEN_READWRITE | rtsql::OPEN_URI | rtsql::OPEN_NOMUTEX, nullptr) !=
        rtsql::OK) {
      err = "open failed";
      close();
      return false;
    }
    // runs on a reactor thread: a lock held elsewhere (the app, the route persister's group commit,
    // a checkpoint) makes the call fall back to the app after ~2 ms instead of waiting up to ~20 s
    sql_.wait_briefly(db_);
    sql_.exec(db_, "PRAGMA foreign_keys=ON", nullptr, nullptr, nullptr);
    blob_path_ = path + ".blobs";
    return true;
  }
  void close() {
    for (void* st : {st_list_, st_first_, st_req_, st_res_, st_del_, st_loc_})
      if (st) sql_.finalize(st);
    st_list_ = st_first_ = st_req_ = st_res_ = st_del_ = st_loc_ = nullptr;
    if (db_) sql_.close(db_);
    db_ = nullptr;
    if (blob_fd_ >= 0) ::close(blob_fd_);
    blob_fd_ = -1;
  }
  bool ok() const { return db_ != nullptr; }
  // the road graph compact route records are rebuilt against (route_record.h); unset: such rows
  // are relayed to the app
  void set_graph(std::shared_ptr<const rrec::RecordGraph> g) { rg_ = std::move(g); }

  // Every call resets its statements on the way out: a statement left on a ROW keeps the
  // connection's read transaction (its WAL snapshot) open, and later reads would not see rows the
  // route service or the app wrote or deleted since.
  struct ResetAll {
    HistoryDb* h;
    ~ResetAll() {
      for (void* st : {h->st_list_, h->st_first_, h->st_req_, h->st_res_, h->st_del_, h->st_loc_})
        if (st) h->sql_.reset(st);
    }
  };

  // GET /api/history?limit=<raw>; raw = nullptr when absent
  Reply history(const char* raw_limit) {
    ResetAll guard{this};
    Reply r;
    int lim = 20;
    if (raw_limit != nullptr && !parse_limit(raw_limit, lim)) return fb();
    lim = lim < 1 ? 1 : (lim > 100 ? 100 : lim);
    if (!prep(st_list_, "SELECT id,origin_id,stops,request_time,engine,vehicle_id FROM route_requests"
                        " ORDER BY request_time DESC, rowid DESC LIMIT ?") ||
        !prep(st_first_, "SELECT total_distance,total_duration,optimized_order,eta_minutes_ml,eta_completion_time_ml"
                         " FROM route_results WHERE request_id=? ORDER BY rowid LIMIT 1"))
      return fb();
    sql_.reset(st_list_);
    sql_.bind_int64(st_list_, 1, lim);
    std::string o = "{\"items\":[";
    int n = 0, rc;
    while ((rc = sql_.step(st_list_)) == rtsql::ROW) {
      // stops -> dest_count (json.loads, then .get("destination_ids") or [])
      size_t dest = 0;
      if (sql_.column_type(st_list_, 2) != rtsql::T_NULL) {
        const std::string js = text(st_list_, 2);
        if (!js.empty()) {
          rtj::Value v;
          if (!parse(js, v)) return fb();
          if (v.truthy()) {
            if (v.kind != rtj::Value::Obj) return fb();
            const rtj::Value* d = v.get("destination_ids");
            if (d && d->truthy()) {
              if (d->kind == rtj::Value::Arr) dest = d->arr.size();
              else if (d->kind == rtj::Value::Obj) dest = d->obj.size();
              else if (d->kind == rtj::Value::Str) return fb();   // len(str): not mirrored
              else return fb();
            }
          }
        }
      }
      if (n++) o += ',';
      o += "{\"request_id\":";
      if (!put_col(o, st_list_, 0)) return fb();
      o += ",\"created_at\":";
      if (!put_col(o, st_list_, 3)) return fb();
      o += ",\"origin_id\":";
      if (!put_col(o, st_list_, 1)) return fb();
      o += ",\"dest_count\":";
      rtr::put_int(o, (long long)dest);
      // first result row
      const std::string id = text(st_list_, 0);
      sql_.reset(st_first_);
      sql_.bind_text(st_first_, 1, id.data(), (int)id.size(), rtsql::TRANSIENT);
      const int rr = sql_.step(st_first_);
      if (rr != rtsql::ROW && rr != rtsql::DONE) return fb();
      const bool have = rr == rtsql::ROW;
      o += ",\"total_distance\":";
      if (have ? !put_col(o, st_first_, 0) : (o += "null", false)) return fb();
      o += ",\"total_duration\":";
      if (have ? !put_col(o, st_first_, 1) : (o += "null", false)) return fb();
      bool optimized = false;
      if (have && sql_.column_type(st_first_, 2) != rtsql::T_NULL) {
        const std::string js = text(st_first_, 2);
        if (!js.empty()) {
          rtj::Value v;
          if (!parse(js, v)) return fb();
          optimized = v.truthy();
        }
      }
      o += optimized ? ",\"optimized\":true" : ",\"optimized\":false";
      o += ",\"engine\":";
      if (!put_or_default(o, st_list_, 4, "default")) return fb();
      o += ",\"vehicle_id\":";
      if (!put_col(o, st_list_, 5)) return fb();
      o += ",\"eta_minutes_ml\":";
      if (have ? !put_col(o, st_first_, 3) : (o += "null", false)) return fb();
      o += ",\"eta_completion_time_ml\":";
      if (have ? !put_col(o, st_first_, 4) : (o += "null", false)) return fb();
      o += '}';
    }
    if (rc != rtsql::DONE) return fb();
    o += "]}";
    r.body = std::move(o);
    return r;
  }

  // GET /api/history/<id>
  Reply detail(const std::string& id) {
    ResetAll guard{this};
    Reply r;
    if (!prep(st_req_, "SELECT id,origin_id,stops,status,request_time,engine,vehicle_id,driver_age FROM"
                       " route_requests WHERE id=?") ||
        !prep(st_res_, "SELECT id,optimized_order,total_distance,total_duration,eta_minutes_ml,eta_completion_time_ml,"
                       "created_at,legs,geometry FROM route_results WHERE request_id=? ORDER BY rowid LIMIT 1"))
      return fb();
    sql_.reset(st_req_);
    sql_.bind_text(st_req_, 1, id.data(), (int)id.size(), rtsql::TRANSIENT);
    const int rc = sql_.step(st_req_);
    if (rc == rtsql::DONE) {
      r.status = 404;
      r.body = "{\"error\":\"not found\"}";
      return r;
    }
    if (rc != rtsql::ROW) return fb();
    std::string o = "{\"request\":{\"id\":";
    if (!put_col(o, st_req_, 0)) return fb();
    o += ",\"origin_id\":";
    if (!put_col(o, st_req_, 1)) return fb();
    o += ",\"stops\":";
    if (!put_json_col(o, st_req_, 2, "{}", true)) return fb();
    o += ",\"status\":";
    if (!put_col(o, st_req_, 3)) return fb();
    o += ",\"request_time\":";
    if (!put_col(o, st_req_, 4)) return fb();
    o += ",\"engine\":";
    if (!put_or_default(o, st_req_, 5, "default")) return fb();
    o += ",\"vehicle_id\":";
    if (!put_col(o, st_req_, 6)) return fb();
    o += ",\"driver_age\":";
    if (!put_col(o, st_req_, 7)) return fb();
    o += "},\"result\":";
    sql_.reset(st_res_);
    sql_.bind_text(st_res_, 1, id.data(), (int)id.size(), rtsql::TRANSIENT);
    const int r2 = sql_.step(st_res_);
    if (r2 == rtsql::DONE) {
      o += "null";
    } else if (r2 == rtsql::ROW) {
      o += "{\"id\":";
      if (!put_col(o, st_res_, 0)) return fb();
      o += ",\"optimized_order\":";
      if (!put_json_col(o, st_res_, 1, "[]", false)) return fb();
      static const char* const rest[] = {"total_distance", "total_duration", "eta_minutes_ml",
                                         "eta_completion_time_ml", "created_at"};
      for (int k = 0; k < 5; ++k) {
        o += ",\"";
        o += rest[k];
        o += "\":";
        if (!put_col(o, st_res_, 2 + k)) return fb();
      }
      if (sql_.column_type(st_res_, 7) == rtsql::T_BLOB) {
        // a compact route record: legs and geometry rebuilt by the route service's own formatter,
        // then through the same json.loads / json.dumps mirror as a text row
        const void* b = sql_.column_blob(st_res_, 7);
        const int nb = sql_.column_bytes(st_res_, 7);
        std::string seg, geo;
        if (!rg_ || b == nullptr || !rrec::decode(*rg_, b, (size_t)nb, seg, geo)) return fb();
        o += ",\"legs\":";
        if (!put_json_text(o, seg)) return fb();
        o += ",\"geometry\":";
        if (!put_json_text(o, geo)) return fb();
      } else {
        o += ",\"legs\":";
        if (!put_json_col(o, st_res_, 7, "[]", false)) return fb();
        o += ",\"geometry\":";
        if (!put_json_col(o, st_res_, 8, "null", false)) return fb();
      }
      o += '}';
    } else {
      return fb();
    }
    o += '}';
    r.body = std::move(o);
    return r;
  }

  // DELETE /api/history/<id> -> 204 (reference semantics: 204 whether or not it existed)
  Reply del(const std::string& id) {
    ResetAll guard{this};
    Reply r;
    if (!prep(st_del_, "DELETE FROM route_requests WHERE id=?")) return fb();
    sql_.reset(st_del_);
    sql_.bind_text(st_del_, 1, id.data(), (int)id.size(), rtsql::TRANSIENT);
    if (sql_.step(st_del_) != rtsql::DONE) return fb();
    r.status = 204;
    return r;
  }

  // GET /api/locations
  Reply locations() {
    ResetAll guard{this};
    Reply r;
    if (!prep(st_loc_, "SELECT * FROM locations ORDER BY created_at, rowid")) return fb();
    sql_.reset(st_loc_);
    const int nc = sql_.column_count(st_loc_);
    std::string o = "[";
    int n = 0, rc;
    while ((rc = sql_.step(st_loc_)) == rtsql::ROW) {
      if (n++) o += ',';
      o += '{';
      for (int c = 0; c < nc; ++c) {
        if (c) o += ',';
        rtr::put_str(o, std::string(sql_.column_name(st_loc_, c)));
        o += ':';
        if (!put_col(o, st_loc_, c)) return fb();
      }
      o += '}';
    }
    if (rc != rtsql::DONE) return fb();
    o += ']';
    r.body = std::move(o);
    return r;
  }

 private:
  rtsql::Api sql_;
  void* db_ = nullptr;
  // large route texts written by the native route service live in <db>.blobs; a column holds
  // "\x01blob:<offset>:<length>" (store/store.py BLOB_REF) — resolved here to the same bytes the app
  // reads
  std::string blob_path_;
  int blob_fd_ = -1;
  std::shared_ptr<const rrec::RecordGraph> rg_;
  bool resolve(std::string& s) {
    static const char kRef[] = "\001blob:";
    if (s.compare(0, sizeof(kRef) - 1, kRef) != 0) return true;
    char* end = nullptr;
    const long long off = std::strtoll(s.c_str() + sizeof(kRef) - 1, &end, 10);
    if (end == nullptr || *end != ':') return false;
    const long long n = std::strtoll(end + 1, nullptr, 10);
    if (off < 0 || n < 0 || n > (1ll << 31)) return false;
    if (blob_fd_ < 0) blob_fd_ = ::open(blob_path_.c_str(), O_RDONLY | O_CLOEXEC);
    if (blob_fd_ < 0) return false;
    std::string out((size_t)n, '\0');
    size_t got = 0;
    while (got < (size_t)n) {
      const ssize_t r = ::pread(blob_fd_, &out[got], (size_t)n - got, (off_t)(off + (long long)got));
      if (r <= 0) return false;
      got += (size_t)r;
    }
    s.swap(out);
    return true;
  }
  void *st_list_ = nullptr, *st_first_ = nullptr, *st_req_ = nullptr, *st_res_ = nullptr, *st_del_ = nullptr,
       *st_loc_ = nullptr;

  static Reply fb() {
    Reply r;
    r.fallback = true;
    return r;
  }
  bool prep(void*& st, const char* q) {
    if (st) return true;
    if (!db_) return false;
    return sql_.prepare_v2(db_, q, -1, &st, nullptr) == rtsql::OK;
  }
  std::string text(void* st, int c) {
    const unsigned char* t = sql_.column_text(st, c);
    const int n = sql_.column_bytes(st, c);
    return t ? std::string((const char*)t, (size_t)n) : std::string();
  }
  static bool parse(const std::string& s, rtj::Value& v) {
    try {
      v = rtj::Parser(s.data(), s.size()).parse();
      return true;
    } catch (const std::exception&) {
      return false;
    }
  }
  // a column as Python's sqlite3 returns it, then json.dumps
  bool put_col(std::string& o, void* st, int c) {
    switch (sql_.column_type(st, c)) {
      case rtsql::T_NULL: o += "null"; return true;
      case rtsql::T_INTEGER: rtr::put_int(o, sql_.column_int64(st, c)); return true;
      case rtsql::T_FLOAT: {
        const double d = sql_.column_double(st, c);
        if (!std::isfinite(d)) return false;
        rtr::put_float(o, d);
        return true;
      }
      case rtsql::T_TEXT: rtr::put_str(o, text(st, c)); return true;
      default: return false;     // blobs: not mirrored
    }
  }
  // `x or "default"` for a text column
  bool put_or_default(std::string& o, void* st, int c, const char* dflt) {
    const int t = sql_.column_type(st, c);
    if (t == rtsql::T_NULL || (t == rtsql::T_TEXT && sql_.column_bytes(st, c) == 0)) {
      rtr::put_str(o, std::string(dflt));
      return true;
    }
    if (t == rtsql::T_INTEGER && sql_.column_int64(st, c) == 0) {
      rtr::put_str(o, std::string(dflt));
      return true;
    }
    if (t == rtsql::T_FLOAT && sql_.column_double(st, c) == 0.0) {
      rtr::put_str(o, std::string(dflt));
      return true;
    }
    return put_col(o, st, c);
  }
  // json.loads(col) if col else <dflt>; with `falsy_default` the parsed value's falsiness also
  // gives the default (store.py: `req.get("stops") or {}`)
  bool put_json_col(std::string& o, void* st, int c, const char* dflt, bool falsy_default) {
    const int t = sql_.column_type(st, c);
    if (t == rtsql::T_NULL || (t == rtsql::T_TEXT && sql_.column_bytes(st, c) == 0)) {
      o += dflt;
      return true;
    }
    if (t != rtsql::T_TEXT) return false;
    rtj::Value v;
    std::string s = text(st, c);
    if (!resolve(s) || !parse(s, v)) return false;
    if (falsy_default && !v.truthy()) {
      o += dflt;
      return true;
    }
    return rtr::put_value(o, v);
  }
  bool put_json_text(std::string& o, const std::string& s) {
    rtj::Value v;
    if (!parse(s, v)) return false;
    return rtr::put_value(o, v);
  }
  // Python int(str): optional surrounding whitespace, sign, digits (underscore forms -> fallback)
  static bool parse_limit(const char* s, int& out) {
    std::string t = s;
    const char* ws = " \t\n\r\x0b\x0c";
    const size_t b = t.find_first_not_of(ws);
    if (b == std::string::npos) { out = 20; return true; }            // int("") -> ValueError -> 20
    t = t.substr(b, t.find_last_not_of(ws) - b + 1);
    size_t i = 0;
    bool neg = false;
    if (t[i] == '+' || t[i] == '-') { neg = t[i] == '-'; ++i; }
    if (i >= t.size()) { out = 20; return true; }
    long long v = 0;
    for (; i < t.size(); ++i) {
      const char ch = t[i];
      if (ch == '_') return false;
      if (ch < '0' || ch > '9') { out = 20; return true; }              // ValueError -> 20
      v = v * 10 + (ch - '0');
      if (v > 1000000) v = 1000000;
    }
    out = (int)(neg ? -v : v);
    return true;
  }
};

}  // namespace rth
