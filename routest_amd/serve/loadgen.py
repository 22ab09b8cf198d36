"""Closed-loop HTTP load against the serving stack's main port (native client, csrc/runtime/http_client.h).

Shared by ``bench.py`` (the ``route_optimizer.http`` variant and the main-port p50) and
``bench/route_http_bench.py``: multi-stop ``/api/optimize_route`` bodies, and one load run reported
as req/s, latency percentiles, response bytes/s and the route service's per-flush stage times.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Sequence

import numpy as np


def route_payloads(lat: np.ndarray, lon: np.ndarray, n: int, seed: int = 1) -> List[Dict[str, Any]]:
    """``n`` requests with a depot and 2-10 stops drawn from the given coordinates."""
    rng = np.random.default_rng(seed)
    reqs = []
    for i in range(n):
        idx = rng.integers(0, len(lat), int(rng.integers(3, 12)))
        reqs.append({"source_point": {"lat": float(lat[idx[0]]), "lon": float(lon[idx[0]])},
                     "destination_points": [{"lat": float(lat[j]), "lon": float(lon[j]), "payload": 1}
                                            for j in idx[1:]],
                     "driver_details": {"driver_name": f"v{i}", "vehicle_type": "car",
                                        "vehicle_capacity": 4, "maximum_distance": 1e7}})
    return reqs


def f02_payloads(lat: np.ndarray, lon: np.ndarray, n: int, seed: int = 2, location_ids: Sequence[str] = (),
                 radius_km: float = 8.0) -> List[Dict[str, Any]]:
    """``n`` requests exactly as the dashboard sends them (``FE/app/ui/page.jsx:1578-1617``):
    ``use_ml_eta``, ``context`` {Sunny, Medium} (no pickup_time: routed at "now"), ``meta`` with the
    seed locations' ids (``origin_id`` null for "My Current Location" one time in five), capacity
    9999, ``maximum_distance`` 100 km, 1-10 stops (``MAX_STOPS``) within ``radius_km`` of the depot."""
    rng = np.random.default_rng(seed)
    ids = list(location_ids)
    reqs = []
    for i in range(n):
        d = int(rng.integers(0, len(lat)))
        k = int(rng.integers(1, 11))
        r = radius_km * np.sqrt(rng.random(k))
        th = rng.random(k) * 2 * np.pi
        slat = lat[d] + r * np.cos(th) / 111.195
        slon = lon[d] + r * np.sin(th) / (111.195 * np.cos(np.radians(lat[d])))
        meta = {"origin_id": (ids[0] if ids and i % 5 else None),
                "destination_ids": [ids[1 + (i + j) % (len(ids) - 1)] for j in range(k)] if len(ids) > 1 else [],
                "vehicle_id": f"VAN-{i % 40:02d}"}
        reqs.append({"source_point": {"lat": float(lat[d]), "lon": float(lon[d])},
                     "destination_points": [{"lat": float(a), "lon": float(b), "payload": 1} for a, b in zip(slat, slon)],
                     "driver_details": {"driver_name": f"Driver {i % 40}", "vehicle_type": "car",
                                        "vehicle_capacity": 9999, "maximum_distance": 100000,
                                        "driver_age": int(20 + i % 45)},
                     "meta": meta, "use_ml_eta": True, "context": {"weather": "Sunny", "traffic": "Medium"}})
    return reqs


def _pct(lat_us: Sequence[float], q: float):
    if not len(lat_us):
        return None
    return float(lat_us[min(len(lat_us) - 1, max(0, int(len(lat_us) * q) - (1 if q >= 0.99 else 0)))]) / 1e3


def native_route_load(stack, reqs: Sequence[Dict[str, Any]], concurrency: int, seconds: float,
                      client_threads: int = 8, path: str = "/api/optimize_route") -> Dict[str, Any]:
    """Drive ``stack`` (serve/frontend.py ServingStack) with ``concurrency`` keep-alive connections
    cycling the request bodies for ``seconds``; returns throughput, latency and stage breakdown."""
    from ..ops import _ext
    rt = _ext.runtime(required=True)
    bodies = [json.dumps(r) for r in reqs]
    paths = [path] * len(bodies)
    rt.http_load_multi(stack.port, min(64, concurrency), 2.0, paths, bodies, client_threads)   # warm-up
    f0 = stack.front.stats()
    r = rt.http_load_multi(stack.port, concurrency, seconds, paths, bodies, client_threads, 0, 1)
    f1 = stack.front.stats()
    lat_us = r["latencies_us"]
    flushes = max(1, f1["route_flushes"] - f0["route_flushes"])
    return {"concurrency": concurrency, "seconds": r["seconds"], "requests": int(r["requests"]),
            "req_per_s": r["requests"] / r["seconds"], "errors": int(r["errors"]),
            "p50_ms": _pct(lat_us, 0.5), "p99_ms": _pct(lat_us, 0.99),
            "response_MB_per_s": r["bytes"] / r["seconds"] / 1e6,
            "flushes": f1["route_flushes"] - f0["route_flushes"],
            "legs_searched": f1["route_legs"] - f0["route_legs"],
            "legs_on_host": f1["route_host_legs"] - f0["route_host_legs"],
            "legs_reusing_matrix_chains": f1.get("route_legs_reused", 0) - f0.get("route_legs_reused", 0),
            "contexts_customized": f1.get("route_contexts_built", 0) - f0.get("route_contexts_built", 0),
            "legs_escalated": f1.get("route_astar_escalated", 0) - f0.get("route_astar_escalated", 0),
            "fallbacks_to_python": f1["route_service_fallbacks"] - f0["route_service_fallbacks"],
            "rows_persisted": f1["route_persisted"] - f0["route_persisted"],
            "record_bytes_per_row": ((f1.get("route_record_bytes", 0) - f0.get("route_record_bytes", 0)) /
                                     max(1, f1.get("route_records", 0) - f0.get("route_records", 0))),
            "jobs_waited_for_context": f1.get("route_ctx_deferred", 0) - f0.get("route_ctx_deferred", 0),
            "stage_ms_per_flush": {k[9:]: (f1[k] - f0[k]) / 1e3 / flushes for k in f1 if k.startswith("route_us_")},
            "client": "native closed-loop (csrc/runtime/http_client.h)",
            "path": f"HTTP/1.1 loopback POST {path} -> native front end (main port) -> route service "
                    "(CCH road matrices per routing context + K6 + CCH legs with paths + C++ GeoJSON with "
                    "maneuvers) -> response bytes"}
