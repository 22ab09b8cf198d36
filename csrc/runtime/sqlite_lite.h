// Minimal run-time binding of the system SQLite library (libsqlite3.so.0, the same library Python's
// sqlite3 module uses; the image ships no sqlite3.h).  The native route service writes the
// reference's two persistence rows (RO/Flaskr/routes.py:134-182; routest_amd/store/store.py
// SQLiteStore) into the same database file the Python store reads, in WAL mode with a short-sleep
// busy handler so the connections interleave safely.
#pragma once
#include <dlfcn.h>

#include <chrono>
#include <cstdint>
#include <string>
#include <thread>

namespace rtsql {

struct Api {
  void* h = nullptr;
  int (*open_v2)(const char*, void**, int, const char*) = nullptr;
  int (*close)(void*) = nullptr;
  int (*busy_timeout)(void*, int) = nullptr;
  int (*exec)(void*, const char*, void*, void*, char**) = nullptr;
  int (*prepare_v2)(void*, const char*, int, void**, const char**) = nullptr;
  int (*bind_text)(void*, int, const char*, int, void (*)(void*)) = nullptr;
  int (*bind_double)(void*, int, double) = nullptr;
  int (*bind_int64)(void*, int, long long) = nullptr;
  int (*bind_null)(void*, int) = nullptr;
  int (*bind_blob)(void*, int, const void*, int, void (*)(void*)) = nullptr;
  int (*step)(void*) = nullptr;
  int (*reset)(void*) = nullptr;
  int (*clear_bindings)(void*) = nullptr;
  int (*finalize)(void*) = nullptr;
  const char* (*errmsg)(void*) = nullptr;
  void (*free_)(void*) = nullptr;
  int (*column_count)(void*) = nullptr;
  int (*column_type)(void*, int) = nullptr;
  double (*column_double)(void*, int) = nullptr;
  long long (*column_int64)(void*, int) = nullptr;
  const unsigned char* (*column_text)(void*, int) = nullptr;
  const void* (*column_blob)(void*, int) = nullptr;
  int (*column_bytes)(void*, int) = nullptr;
  const char* (*column_name)(void*, int) = nullptr;
  int (*changes)(void*) = nullptr;
  int (*wal_checkpoint_v2)(void*, const char*, int, int*, int*) = nullptr;
  int (*busy_handler)(void*, int (*)(void*, int), void*) = nullptr;

  bool load(std::string& err) {
    if (h) return true;
    h = dlopen("libsqlite3.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libsqlite3.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) { err = "libsqlite3 not found"; return false; }
    bool ok = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      ok = ok && fn != nullptr;
    };
    sym(open_v2, "sqlite3_open_v2");
    sym(close, "sqlite3_close");
    sym(busy_timeout, "sqlite3_busy_timeout");
    sym(exec, "sqlite3_exec");
    sym(prepare_v2, "sqlite3_prepare_v2");
    sym(bind_text, "sqlite3_bind_text");
    sym(bind_double, "sqlite3_bind_double");
    sym(bind_int64, "sqlite3_bind_int64");
    sym(bind_null, "sqlite3_bind_null");
    sym(bind_blob, "sqlite3_bind_blob");
    sym(step, "sqlite3_step");
    sym(reset, "sqlite3_reset");
    sym(clear_bindings, "sqlite3_clear_bindings");
    sym(finalize, "sqlite3_finalize");
    sym(errmsg, "sqlite3_errmsg");
    sym(free_, "sqlite3_free");
    sym(column_count, "sqlite3_column_count");
    sym(column_type, "sqlite3_column_type");
    sym(column_double, "sqlite3_column_double");
    sym(column_int64, "sqlite3_column_int64");
    sym(column_text, "sqlite3_column_text");
    sym(column_blob, "sqlite3_column_blob");
    sym(column_bytes, "sqlite3_column_bytes");
    sym(column_name, "sqlite3_column_name");
    sym(changes, "sqlite3_changes");
    sym(wal_checkpoint_v2, "sqlite3_wal_checkpoint_v2");
    sym(busy_handler, "sqlite3_busy_handler");
    if (!ok) err = "libsqlite3: missing symbols";
    return ok;
  }

  // Waits for a lock another connection holds in short sleeps (50 us, then 200 us, then 1 ms; ~20 s
  // in all) — sqlite3_busy_timeout's back-off sleeps 1, 2, 5, 10 ... 100 ms, so a native DELETE
  // that met the route persister's group commit (a millisecond) waited tens of milliseconds.
  static int short_sleeps(void*, int n) {
    if (n >= 20000) return 0;
    std::this_thread::sleep_for(std::chrono::microseconds(n < 20 ? 50 : (n < 200 ? 200 : 1000)));
    return 1;
  }
  void wait_on_locks(void* db) { busy_handler(db, &Api::short_sleeps, nullptr); }
  // For a connection used on an event-loop thread (the native front end's reactors): at most ~2 ms
  // of 50 us sleeps, then SQLITE_BUSY — the caller relays the request to the app instead of
  // stalling every connection of its reactor behind a writer's lock.
  static int brief_sleeps(void*, int n) {
    if (n >= 40) return 0;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
    return 1;
  }
  void wait_briefly(void* db) { busy_handler(db, &Api::brief_sleeps, nullptr); }
};

constexpr int OK = 0, ROW = 100, DONE = 101;
constexpr int T_INTEGER = 1, T_FLOAT = 2, T_TEXT = 3, T_BLOB = 4, T_NULL = 5;
constexpr int OPEN_READWRITE = 0x2, OPEN_CREATE = 0x4, OPEN_URI = 0x40, OPEN_NOMUTEX = 0x8000;
constexpr int CHECKPOINT_PASSIVE = 0;
inline void (*const TRANSIENT)(void*) = reinterpret_cast<void (*)(void*)>(-1);
inline void (*const STATIC)(void*) = nullptr;      // the caller keeps the bytes alive until step/reset

}  // namespace rtsql
