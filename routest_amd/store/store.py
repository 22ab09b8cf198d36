"""Persistence for route requests/results + locations (R11-R14, L01-L03).

Reference: Supabase PostgREST calls in ``RO/Flaskr/routes.py:134-182`` (insert),
``:185-231`` (history list), ``:234-279`` (detail), ``:386-406`` (delete); schema in
``LV/database/migrations/2025_08_12_14{4039,4349,4521}_*.php`` plus the columns the Flask adapter
writes that the migrations lack: ``route_requests.{engine, vehicle_id,
driver_age}``, ``route_results.{geometry, eta_minutes_ml, eta_completion_time_ml}``.

* :class:`SQLiteStore` (default, ``ROUTEST_STORE=sqlite:///path`` or ``:memory:``): all written
  columns exist, ``origin_id`` is nullable and not FK-checked (the dashboard sends
  ``origin_id: null`` for "My Current Location", which the reference's NOT NULL FK silently
  rejects — Appendix B #5), results cascade-delete with their request.
* :class:`PostgRESTStore`: the reference's exact REST calls for a Supabase deployment.

A road-graph route persisted by the native route service does not store its formatted legs and
geometry (~30-100 KB of GeoJSON per route): ``legs`` holds a compact route record (a BLOB starting
``RECORD_MAGIC``: waypoints, per-hop adjacency slots, per-step durations; ~1-3 KB,
csrc/runtime/route_record.h) and ``geometry`` is NULL.  Readers — this class through the graph
provider's ``_rt.GraphSteps.decode_record`` (:meth:`SQLiteStore.set_record_graph`) and the native
history reader (csrc/runtime/history_db.h) — rebuild the texts with the route service's own
formatter, byte-identical to what it answered.  Rows of earlier rounds may instead hold a reference
(``BLOB_REF`` + ``offset:length``) into the append-only side file ``<db>.blobs``; both readers still
resolve those.
"""
from __future__ import annotations

import atexit
import datetime as dt
import json
import os
import sqlite3
import tempfile
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

from ..data.synth import seed_locations
from ..utils.faults import maybe_fail

SCHEMA = """
CREATE TABLE IF NOT EXISTS locations (
    id TEXT PRIMARY KEY,
    name TEXT NOT NULL,
    latitude REAL NOT NULL,
    longitude REAL NOT NULL,
    created_at TEXT
);
CREATE TABLE IF NOT EXISTS route_requests (
    id TEXT PRIMARY KEY,
    origin_id TEXT,
    stops TEXT NOT NULL,
    request_time TEXT NOT NULL,
    status TEXT NOT NULL DEFAULT 'pending',
    engine TEXT,
    vehicle_id TEXT,
    driver_age REAL
);
CREATE INDEX IF NOT EXISTS route_requests_time ON route_requests(request_time);
CREATE TABLE IF NOT EXISTS route_results (
    id TEXT PRIMARY KEY,
    request_id TEXT NOT NULL REFERENCES route_requests(id) ON DELETE CASCADE,
    optimized_order TEXT,
    total_distance REAL,
    total_duration REAL,
    legs TEXT,
    geometry TEXT,
    eta_minutes_ml REAL,
    eta_completion_time_ml TEXT,
    created_at TEXT
);
CREATE INDEX IF NOT EXISTS route_results_req ON route_results(request_id);
"""


class StoreUnavailable(RuntimeError):
    pass


#: prefix of a column value stored in the side file (never the first byte of JSON text); rows of
#: rounds before the compact records still carry it
BLOB_REF = "\x01blob:"
#: first bytes of a compact route record (csrc/runtime/route_record.h), stored as a BLOB in `legs`
RECORD_MAGIC = b"\x02RR1"


_EPHEMERAL: List[str] = []


def _remove_db(path: str) -> None:
    for suffix in ("", "-wal", "-shm", ".blobs"):
        try:
            os.remove(path + suffix)
        except OSError:
            pass


@atexit.register
def _cleanup_ephemeral() -> None:  # pragma: no cover - exit path
    for p in _EPHEMERAL:
        _remove_db(p)


def _now_iso() -> str:
    return dt.datetime.now(dt.timezone.utc).isoformat()


def build_rows(payload: Dict[str, Any], feature: Dict[str, Any]):
    """The two rows the reference writes (routes.py:138-176)."""
    meta = payload.get("meta") or {}
    driver = payload.get("driver_details") or {}
    engine = "ml" if payload.get("use_ml_eta") else "default"
    stops = {"destination_ids": meta.get("destination_ids") or [],
             "destination_points": payload.get("destination_points") or []}
    req_row = {"origin_id": meta.get("origin_id"), "stops": stops, "status": "completed",
               "engine": engine, "vehicle_id": driver.get("driver_name"),
               "driver_age": driver.get("driver_age")}
    props = (feature or {}).get("properties", {}) or {}
    summary = props.get("summary", {}) or {}
    res_row = {"total_distance": float(summary.get("distance") or 0),
               "total_duration": float(summary.get("duration") or 0),
               "optimized_order": props.get("optimized_order") or [],
               "legs": props.get("segments", []) or [],
               "geometry": (feature or {}).get("geometry") or None,
               "eta_minutes_ml": props.get("eta_minutes_ml"),
               "eta_completion_time_ml": props.get("eta_completion_time_ml")}
    return req_row, res_row


def _history_item(req: Dict[str, Any], first: Dict[str, Any]) -> Dict[str, Any]:
    """routes.py:211-229 flattening."""
    stops = req.get("stops") or {}
    dest_ids = stops.get("destination_ids") or []
    return {
        "request_id": req["id"],
        "created_at": req.get("request_time"),
        "origin_id": req.get("origin_id"),
        "dest_count": len(dest_ids),
        "total_distance": first.get("total_distance"),
        "total_duration": first.get("total_duration"),
        "optimized": bool(first.get("optimized_order") or []),
        "engine": req.get("engine") or "default",
        "vehicle_id": req.get("vehicle_id"),
        "eta_minutes_ml": first.get("eta_minutes_ml"),
        "eta_completion_time_ml": first.get("eta_completion_time_ml"),
    }


class SQLiteStore:
    blocking = False       # local SQLite: a row insert is ~0.3 ms, cheaper inline than a thread hop
    kind = "sqlite"

    def __init__(self, path: str = ":memory:", seed: bool = True):
        # ":memory:" (the default, nothing survives a restart) is backed by a private temporary
        # file deleted at exit, so the native route service (csrc/route_service.hip) can write the
        # same database through its own connection; WAL + a busy timeout interleave the two
        self.ephemeral = path == ":memory:"
        if self.ephemeral:
            fd, path = tempfile.mkstemp(prefix="routest-store-", suffix=".db")
            os.close(fd)
            _EPHEMERAL.append(path)
        self.path = path
        self.blob_path = path + ".blobs"
        self._blob_fd: Optional[int] = None
        self._record_graph: Any = None
        self._lock = threading.Lock()
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None, timeout=10.0)
        self._db.row_factory = sqlite3.Row
        self._db.execute("PRAGMA foreign_keys=ON")
        # 16 KB pages (only takes effect on a new database file): a persisted route is ~30-100 KB of
        # GeoJSON geometry + segments, i.e. ~10-25 overflow pages and WAL frames at the 4 KB
        # default; larger pages cost more again in statement journals (measured: 4 KB 124 us/row,
        # 16 KB 88, 64 KB 101-113 for a 33 KB route in one transaction; route_service.hip)
        self._db.execute("PRAGMA page_size=16384")
        self._db.execute("PRAGMA journal_mode=WAL")
        # WAL + NORMAL for a file store: commits append to the WAL without an fsync (synced at
        # checkpoints); the temporary default store needs no durability at all
        self._db.execute("PRAGMA synchronous=OFF" if self.ephemeral else "PRAGMA synchronous=NORMAL")
        self._db.executescript(SCHEMA)
        if seed:
            self.seed_locations()

    @property
    def sqlite_uri(self) -> str:
        """Database file for other connections (the native route service)."""
        return os.path.abspath(self.path)

    def close(self) -> None:
        with self._lock:
            try:
                self._db.close()
            except Exception:  # pragma: no cover
                pass
            if self._blob_fd is not None:
                os.close(self._blob_fd)
                self._blob_fd = None
        if self.ephemeral:
            _remove_db(self.path)

    # ---- locations (L03, F10, L04) ----
    def seed_locations(self) -> None:
        with self._lock:
            for loc in seed_locations():
                self._db.execute("INSERT OR IGNORE INTO locations(id,name,latitude,longitude,created_at)"
                                 " VALUES(?,?,?,?,?)", (loc["id"], loc["name"], loc["latitude"],
                                                        loc["longitude"], "2025-08-12T14:40:39+00:00"))

    def locations(self) -> List[Dict[str, Any]]:
        with self._lock:
            rows = self._db.execute("SELECT * FROM locations ORDER BY created_at, rowid").fetchall()
        return [dict(r) for r in rows]

    # ---- health ----
    def ping(self) -> Dict[str, Any]:
        t0 = time.time()
        try:
            maybe_fail("store_fail")
            with self._lock:
                self._db.execute("SELECT id FROM route_requests LIMIT 1").fetchall()
            return {"status": "ok", "latency_ms": int((time.time() - t0) * 1000), "kind": self.kind}
        except Exception as e:
            return {"status": "error", "latency_ms": int((time.time() - t0) * 1000),
                    "error": str(e)[:200], "kind": self.kind}

    # ---- writes (R14) ----
    def persist_request_and_result(self, payload: Dict[str, Any], feature: Dict[str, Any]) -> str:
        maybe_fail("store_fail")
        req, res = build_rows(payload, feature)
        rid = str(uuid.uuid4())
        now = _now_iso()
        with self._lock:
            self._db.execute("BEGIN")
            try:
                self._db.execute(
                    "INSERT INTO route_requests(id,origin_id,stops,request_time,status,engine,vehicle_id,"
                    "driver_age) VALUES(?,?,?,?,?,?,?,?)",
                    (rid, req["origin_id"], json.dumps(req["stops"]), now, req["status"], req["engine"],
                     req["vehicle_id"], req["driver_age"]))
                self._db.execute(
                    "INSERT INTO route_results(id,request_id,optimized_order,total_distance,"
                    "total_duration,legs,geometry,eta_minutes_ml,eta_completion_time_ml,created_at)"
                    " VALUES(?,?,?,?,?,?,?,?,?,?)",
                    (str(uuid.uuid4()), rid, json.dumps(res["optimized_order"]),
                     round(res["total_distance"], 2), round(res["total_duration"], 2),
                     json.dumps(res["legs"]),
                     json.dumps(res["geometry"]) if res["geometry"] is not None else None,
                     res["eta_minutes_ml"], res["eta_completion_time_ml"], now))
                self._db.execute("COMMIT")
            except Exception:
                self._db.execute("ROLLBACK")
                raise
        return rid

    @staticmethod
    def _req_dict(r: sqlite3.Row) -> Dict[str, Any]:
        d = dict(r)
        d["stops"] = json.loads(d["stops"]) if d.get("stops") else {}
        return d

    def _text(self, v: Any) -> Any:
        """A column value, with a side-file reference (``BLOB_REF`` + ``offset:length``) resolved."""
        if not isinstance(v, str) or not v.startswith(BLOB_REF):
            return v
        off, n = (int(x) for x in v[len(BLOB_REF):].split(":"))
        if self._blob_fd is None:
            self._blob_fd = os.open(self.blob_path, os.O_RDONLY)
        b = os.pread(self._blob_fd, n, off)
        if len(b) != n:
            raise StoreUnavailable(f"route side file {self.blob_path} is short at {off}+{n}")
        return b.decode("utf-8")

    def set_record_graph(self, steps: Any) -> None:
        """The road graph (``_rt.GraphSteps`` of the GraphProvider) that compact route records are
        rebuilt against (csrc/runtime/route_record.h)."""
        self._record_graph = steps

    def _decode_record(self, rec: bytes):
        g = self._record_graph
        if g is None:
            raise StoreUnavailable("a compact route record needs the road graph it was routed on "
                                   "(serve with the same graph provider)")
        try:
            return g.decode_record(rec)
        except ValueError as e:
            raise StoreUnavailable(f"route record: {e}") from None

    def _res_dict(self, r: sqlite3.Row, full: bool) -> Dict[str, Any]:
        d = dict(r)
        d["optimized_order"] = json.loads(d["optimized_order"]) if d.get("optimized_order") else []
        legs = d.pop("legs", None)
        geom = d.pop("geometry", None)
        d.pop("request_id", None)
        if full and isinstance(legs, (bytes, bytearray, memoryview)) and bytes(legs[:4]) == RECORD_MAGIC:
            # a compact record of the native route service: legs and geometry rebuilt by its formatter
            legs, geom = self._decode_record(bytes(legs))
        elif full:
            legs, geom = self._text(legs), self._text(geom)
        if full:
            d["legs"] = json.loads(legs) if legs else []
            d["geometry"] = json.loads(geom) if geom else None
        return d

    # ---- reads (R11, R12) ----
    def history(self, limit: int) -> List[Dict[str, Any]]:
        maybe_fail("store_fail")
        with self._lock:
            reqs = self._db.execute("SELECT * FROM route_requests ORDER BY request_time DESC, rowid DESC"
                                    " LIMIT ?", (int(limit),)).fetchall()
            items = []
            for r in reqs:
                res = self._db.execute(
                    "SELECT id,total_distance,total_duration,optimized_order,created_at,eta_minutes_ml,"
                    "eta_completion_time_ml,request_id,NULL AS legs,NULL AS geometry FROM route_results"
                    " WHERE request_id=? ORDER BY rowid LIMIT 1", (r["id"],)).fetchone()
                items.append(_history_item(self._req_dict(r), self._res_dict(res, False) if res else {}))
        return items

    def history_detail(self, req_id: str) -> Optional[Dict[str, Any]]:
        maybe_fail("store_fail")
        with self._lock:
            r = self._db.execute("SELECT * FROM route_requests WHERE id=?", (req_id,)).fetchone()
            if r is None:
                return None
            res = self._db.execute("SELECT * FROM route_results WHERE request_id=? ORDER BY rowid LIMIT 1",
                                   (req_id,)).fetchone()
        req = self._req_dict(r)
        return {
            "request": {"id": req["id"], "origin_id": req.get("origin_id"), "stops": req.get("stops") or {},
                        "status": req.get("status"), "request_time": req.get("request_time"),
                        "engine": req.get("engine") or "default", "vehicle_id": req.get("vehicle_id"),
                        "driver_age": req.get("driver_age")},
            "result": self._res_dict(res, True) if res else None,
        }

    def delete(self, req_id: str) -> bool:
        maybe_fail("store_fail")
        with self._lock:
            cur = self._db.execute("DELETE FROM route_requests WHERE id=?", (req_id,))
        return cur.rowcount > 0


class PostgRESTStore:
    blocking = True        # remote HTTPS
    """The reference's Supabase calls (routes.py:14-23,156,177,203,240,333,394)."""

    kind = "postgrest"

    def __init__(self, url: str, service_key: str, session: Any = None):
        import requests
        self.rest = f"{url}/rest/v1"
        self.key = service_key
        self.http = session or requests.Session()
        self.headers = {"apikey": service_key, "Authorization": f"Bearer {service_key}",
                        "Content-Type": "application/json", "Prefer": "return=representation"}

    def ping(self) -> Dict[str, Any]:
        t0 = time.time()
        try:
            r = self.http.get(f"{self.rest}/route_requests", headers=self.headers,
                              params={"select": "id", "limit": "1"}, timeout=3)
            return {"status": "ok" if 200 <= r.status_code < 300 else "degraded",
                    "latency_ms": int((time.time() - t0) * 1000), "code": r.status_code, "kind": self.kind}
        except Exception as e:
            return {"status": "error", "latency_ms": int((time.time() - t0) * 1000), "error": str(e)[:200],
                    "kind": self.kind}

    def persist_request_and_result(self, payload: Dict[str, Any], feature: Dict[str, Any]) -> str:
        req, res = build_rows(payload, feature)
        r = self.http.post(f"{self.rest}/route_requests", headers=self.headers, json=req, timeout=20)
        r.raise_for_status()
        rid = r.json()[0]["id"]
        res = dict(res, request_id=rid)
        r2 = self.http.post(f"{self.rest}/route_results", headers=self.headers, json=res, timeout=20)
        r2.raise_for_status()
        return rid

    def history(self, limit: int) -> List[Dict[str, Any]]:
        import requests
        params = {"select": ("id,request_time,origin_id,stops,engine,vehicle_id,driver_age,"
                             "route_results(id,total_distance,total_duration,optimized_order,created_at,"
                             "eta_minutes_ml,eta_completion_time_ml)"),
                  "order": "request_time.desc", "limit": str(limit)}
        try:
            r = self.http.get(f"{self.rest}/route_requests", headers=self.headers, params=params, timeout=20)
            r.raise_for_status()
            rows = r.json()
        except requests.RequestException as e:
            status = getattr(e.response, "status_code", "n/a")
            text = getattr(e.response, "text", str(e))
            raise StoreUnavailable(f"supabase fetch failed (status {status}): {text}")
        out = []
        for rr in rows:
            res = rr.get("route_results") or []
            out.append(_history_item(rr, res[0] if res else {}))
        return out

    def history_detail(self, req_id: str) -> Optional[Dict[str, Any]]:
        import requests
        params = {"select": ("id,origin_id,stops,status,request_time,engine,vehicle_id,driver_age,"
                             "route_results(id,total_distance,total_duration,optimized_order,legs,created_at,"
                             "eta_minutes_ml,eta_completion_time_ml,geometry)"),
                  "id": f"eq.{req_id}", "limit": "1"}
        try:
            r = self.http.get(f"{self.rest}/route_requests", headers=self.headers, params=params, timeout=20)
            r.raise_for_status()
            rows = r.json()
        except requests.RequestException as e:
            status = getattr(e.response, "status_code", "n/a")
            text = getattr(e.response, "text", str(e))
            raise StoreUnavailable(f"supabase fetch failed (status {status}): {text}")
        if not rows:
            return None
        req = rows[0]
        results = req.get("route_results") or []
        return {"request": {"id": req["id"], "origin_id": req.get("origin_id"), "stops": req.get("stops") or {},
                            "status": req.get("status"), "request_time": req.get("request_time"),
                            "engine": req.get("engine") or "default", "vehicle_id": req.get("vehicle_id"),
                            "driver_age": req.get("driver_age")},
                "result": results[0] if results else None}

    def delete(self, req_id: str) -> bool:
        import requests
        headers = dict(self.headers)
        headers.pop("Prefer", None)
        try:
            r = self.http.delete(f"{self.rest}/route_requests", headers=headers,
                                 params={"id": f"eq.{req_id}"}, timeout=10)
        except requests.RequestException as e:
            status = getattr(e.response, "status_code", "n/a")
            text = getattr(e.response, "text", str(e))
            raise StoreUnavailable(f"supabase delete failed (status {status}): {text}")
        if r.status_code not in (200, 204):
            raise StoreUnavailable(f"delete failed: {r.status_code} {r.text}")
        return True

    def locations(self) -> List[Dict[str, Any]]:
        r = self.http.get(f"{self.rest}/locations", headers=self.headers,
                          params={"select": "*", "order": "created_at"}, timeout=10)
        r.raise_for_status()
        return r.json()


def open_store(url: str, supabase_url: Optional[str] = None, supabase_key: Optional[str] = None):
    """``sqlite:///path`` | ``sqlite:///:memory:`` | ``postgrest`` | ``none``."""
    if url == "none":
        return None
    if url == "postgrest":
        if not (supabase_url and supabase_key):
            return None
        return PostgRESTStore(supabase_url, supabase_key)
    if url.startswith("sqlite:///"):
        return SQLiteStore(url[len("sqlite:///"):] or ":memory:")
    raise ValueError(f"unknown store url {url!r}")
