#!/usr/bin/env python3
"""Mixed-traffic soak of the whole FastAPI app in-process (ASGI): concurrent clients hit
/api/predict_eta, /predict (batched), /api/optimize_route (ML ETA on, persisted to SQLite),
/route, /api/history, /api/history/<id>, DELETE, /api/health and /metrics for ``--seconds``, on
the GPU services when a GPU is visible (micro-batched ETA kernel, cross-request route batcher with
the road-graph provider and batched A*).  Every response is checked against its endpoint's
contract; exits non-zero on any unexpected status, malformed body or exception.

    python tools/app_soak.py --seconds 30 --clients 64

``--stack``: the same mix over real sockets against the serving stack's main port — the native
front end (predictions and routes answered natively, the rest relayed to the FastAPI app) —
driven by the native mixed-traffic client (csrc/runtime/http_client.h http_load_mixed) with
``--clients`` keep-alive connections.  Every response's status is checked against its endpoint's
contract; a sample of each endpoint's bodies is then validated in Python.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--graph-nodes", type=int, default=20000)
    ap.add_argument("--stack", action="store_true", help="real sockets against the native front end")
    ap.add_argument("--front-threads", type=int, default=8)
    a = ap.parse_args()
    import httpx
    import numpy as np
    import torch

    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider, edge_costs
    from routest_amd.serve.eta_service import EtaService, default_model
    from routest_amd.store.store import SQLiteStore

    gpu = torch.cuda.is_available()
    dev = torch.device("cuda:0") if gpu else None
    model = default_model(seed=0, hidden=256, steps=100)
    g = synth_road_graph(a.graph_nodes, seed=7)
    cost = edge_costs(g, model, device=dev)
    prov = GraphProvider(g, cost, device=dev)
    s = load_settings(env={}, dotenv_path=None, devices=[0] if gpu else [], device="cuda:0" if gpu else "cpu",
                      route_batch="auto" if gpu else "0", route_gpu_min_stops=1, warm_scorer=False)
    tmp = tempfile.mkdtemp()
    store = SQLiteStore(os.path.join(tmp, "soak.db"))
    eta = EtaService(model, devices=[0]) if gpu else EtaService(model, device="cpu")
    sv = build_services(s, eta=eta, provider=prov, store=store)
    app = create_app(sv)
    rng = random.Random(1)
    lat, lon = g.lat, g.lon

    def route_req(k):
        idx = [rng.randrange(len(lat)) for _ in range(k + 1)]
        return {"source_point": {"lat": float(lat[idx[0]]), "lon": float(lon[idx[0]])},
                "destination_points": [{"lat": float(lat[i]), "lon": float(lon[i]), "payload": 1} for i in idx[1:]],
                "driver_details": {"driver_name": f"d{rng.randrange(1000)}", "vehicle_type": "car",
                                   "vehicle_capacity": 9999, "maximum_distance": 1e7, "driver_age": 30},
                "use_ml_eta": True, "context": {"weather": "Rainy", "traffic": "High"}}

    def eta_req():
        return {"summary": {"distance": rng.uniform(500, 40000)}, "pickup_time": "2026-10-15T08:30:00",
                "driver_age": rng.randint(18, 70), "weather": rng.choice(["Sunny", "Rainy", "Foggy", "Stormy"]),
                "traffic": rng.choice(["Low", "Medium", "High"])}

    if a.stack:
        return stack_soak(a, sv, app, model, route_req, eta_req, rng)

    stats = {"requests": 0, "errors": [], "by_ep": {}}
    ids = []

    def bad(ep, msg):
        if len(stats["errors"]) < 20:
            stats["errors"].append(f"{ep}: {msg}")

    async def client(c: httpx.AsyncClient, deadline: float):
        while time.perf_counter() < deadline:
            op = rng.random()
            try:
                if op < 0.35:
                    ep = "predict_eta"
                    r = await c.post("/api/predict_eta", json=eta_req())
                    ok = r.status_code == 200 and "eta_minutes_ml" in r.json()
                elif op < 0.45:
                    ep = "predict_batch"
                    r = await c.post("/predict", json={"items": [eta_req() for _ in range(rng.randint(1, 64))]})
                    ok = r.status_code == 200
                elif op < 0.70:
                    ep = "optimize_route"
                    r = await c.post("/api/optimize_route", json=route_req(rng.randint(1, 6)))
                    body = r.json()
                    ok = r.status_code in (200, 400) and (("error" in body) == (r.status_code == 400))
                    if r.status_code == 200 and body.get("properties", {}).get("request_id"):
                        ids.append(body["properties"]["request_id"])
                elif op < 0.80:
                    ep = "route"
                    r = await c.post("/route", json=route_req(1))
                    ok = r.status_code in (200, 400)
                elif op < 0.88:
                    ep = "history"
                    r = await c.get("/api/history")
                    ok = r.status_code == 200 and isinstance(r.json(), (list, dict))
                elif op < 0.93 and ids:
                    ep = "history_id"
                    r = await c.get(f"/api/history/{rng.choice(ids)}")
                    ok = r.status_code in (200, 404)
                elif op < 0.95 and ids:
                    ep = "delete"
                    r = await c.delete(f"/api/history/{ids.pop()}")
                    ok = r.status_code in (200, 204, 404)
                elif op < 0.98:
                    ep = "health"
                    r = await c.get("/api/health")
                    ok = r.status_code == 200 and "status" in r.json()
                else:
                    ep = "metrics"
                    r = await c.get("/metrics")
                    ok = r.status_code == 200
            except Exception as e:  # noqa: BLE001
                ep, ok, r = "exception", False, None
                bad(ep, repr(e)[:200])
            stats["requests"] += 1
            stats["by_ep"][ep] = stats["by_ep"].get(ep, 0) + 1
            if not ok and r is not None:
                bad(ep, f"status {r.status_code} body {r.text[:200]}")

    async def run():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://soak",
                                     timeout=60) as c:
            deadline = time.perf_counter() + a.seconds
            await asyncio.gather(*[client(c, deadline) for _ in range(a.clients)])

    t0 = time.perf_counter()
    rb = sv.route_batcher
    try:
        asyncio.run(run())
    finally:
        sv.close()
    el = time.perf_counter() - t0
    out = {"gpu": gpu, "seconds": round(el, 1), "clients": a.clients, "requests": stats["requests"],
           "req_per_s": round(stats["requests"] / el, 1), "by_endpoint": stats["by_ep"],
           "errors": stats["errors"], "route_flushes": sum(rb.flushes) if rb is not None else None}
    print(json.dumps(out), flush=True)
    return 0 if not stats["errors"] else 1


KINDS = ["predict_eta", "predict_batch", "optimize_route", "route", "history", "history_id", "delete",
         "health", "metrics"]
ALLOWED = {0: {200}, 1: {200}, 2: {200, 400}, 3: {200, 400}, 4: {200}, 5: {200, 404}, 6: {204, 404},
           7: {200}, 8: {200}}


def _raw(method: str, path: str, body=None) -> bytes:
    b = b"" if body is None else json.dumps(body).encode()
    h = f"{method} {path} HTTP/1.1\r\nHost: soak\r\n"
    if body is not None:
        h += f"Content-Type: application/json\r\nContent-Length: {len(b)}\r\n"
    return (h + "\r\n").encode() + b


def stack_soak(a, sv, app, model, route_req, eta_req, rng) -> int:
    import http.client
    from routest_amd.ops import _ext
    from routest_amd.serve.frontend import ServingStack
    rt = _ext.runtime(required=True)
    out = {"mode": "stack (native front end on the main port + FastAPI app behind it)", "clients": a.clients}
    with ServingStack(sv, app, model, [0], threads=a.front_threads) as st:
        c = http.client.HTTPConnection("127.0.0.1", st.port, timeout=60)

        def call(method, path, body=None):
            c.request(method, path, body=None if body is None else json.dumps(body),
                      headers={"Content-Type": "application/json"} if body is not None else {})
            r = c.getresponse()
            return r.status, r.read()
        ids = []
        for _ in range(300):                  # persisted natively, read back through the relay
            code, body = call("POST", "/api/optimize_route", route_req(rng.randint(1, 6)))
            if code == 200:
                ids.append(json.loads(body)["properties"]["request_id"])
        raw, kinds = [], []
        for i in range(20000):
            op = rng.random()
            if op < 0.35:
                k, r = 0, _raw("POST", "/api/predict_eta", eta_req())
            elif op < 0.45:
                k, r = 1, _raw("POST", "/predict", {"items": [eta_req() for _ in range(rng.randint(1, 64))]})
            elif op < 0.70:
                k, r = 2, _raw("POST", "/api/optimize_route", route_req(rng.randint(1, 6)))
            elif op < 0.80:
                k, r = 3, _raw("POST", "/route", route_req(1))
            elif op < 0.88:
                k, r = 4, _raw("GET", "/api/history")
            elif op < 0.93:
                k, r = 5, _raw("GET", f"/api/history/{rng.choice(ids)}")
            elif op < 0.95:
                k, r = 6, _raw("DELETE", f"/api/history/{ids[i % len(ids)]}")
            elif op < 0.98:
                k, r = 7, _raw("GET", "/api/health")
            else:
                k, r = 8, _raw("GET", "/metrics")
            raw.append(r)
            kinds.append(k)
        rt.http_load_mixed(st.port, 16, 2.0, raw[:2000], kinds[:2000], len(KINDS), 4)     # warm-up
        f0 = st.front.stats()
        res = rt.http_load_mixed(st.port, a.clients, a.seconds, raw, kinds, len(KINDS), 8)
        f1 = st.front.stats()
        bad = {}
        by = {}
        for k, counts in enumerate(res["status_by_kind"]):
            by[KINDS[k]] = {str(code): n for code, n in sorted(counts.items())}
            wrong = {code: n for code, n in counts.items() if code not in ALLOWED[k]}
            if wrong:
                bad[KINDS[k]] = wrong
        # body contracts on a sample of every endpoint, through the same port
        sample_errors = []
        for _ in range(20):
            checks = [
                ("POST", "/api/predict_eta", eta_req(), lambda s, b: s == 200 and "eta_minutes_ml" in b),
                ("POST", "/predict", {"items": [eta_req(), eta_req()]}, lambda s, b: s == 200 and len(b["predictions"]) == 2),
                ("POST", "/api/optimize_route", route_req(3),
                 lambda s, b: (s == 200 and b["type"] == "Feature" and "eta_minutes_ml" in b["properties"]
                               and b["properties"].get("saved") is True) or (s == 400 and "error" in b)),
                ("GET", "/api/history", None, lambda s, b: s == 200 and isinstance(b.get("items"), list)),
                ("GET", "/api/health", None, lambda s, b: s == 200 and "status" in b),
            ]
            for method, path, body, ok in checks:
                code, raw_b = call(method, path, body)
                try:
                    good = ok(code, json.loads(raw_b))
                except Exception:  # noqa: BLE001
                    good = False
                if not good and len(sample_errors) < 10:
                    sample_errors.append(f"{path}: {code} {raw_b[:200]!r}")
        lat = res["latencies_us"]
        out.update({"seconds": round(res["seconds"], 1), "requests": int(res["requests"]),
                    "req_per_s": round(res["requests"] / res["seconds"], 1), "transport_errors": int(res["errors"]),
                    "p50_ms": float(lat[len(lat) // 2]) / 1e3, "p99_ms": float(lat[int(len(lat) * 0.99) - 1]) / 1e3,
                    "status_by_endpoint": by,
                    "p50_p99_ms_by_endpoint": {KINDS[k]: [round(q[0] / 1e3, 2), round(q[1] / 1e3, 2)]
                                               for k, q in enumerate(res["p50_p99_us_by_kind"])},
                    "contract_errors": bad, "body_sample_errors": sample_errors,
                    "native_route_jobs": f1["route_jobs"] - f0["route_jobs"], "relayed": f1["relayed"] - f0["relayed"],
                    "history_native": f1["history_native"] - f0["history_native"],
                    "cached": f1["cached"] - f0["cached"],
                    "route_flushes": f1["route_flushes"] - f0["route_flushes"],
                    "route_stage_ms_per_flush": {k[9:]: round((f1[k] - f0[k]) / 1e3 / max(1, f1["route_flushes"] - f0["route_flushes"]), 3)
                                                 for k in f1 if k.startswith("route_us_")},
                    "route_persisted": f1["route_persisted"] - f0["route_persisted"]})
    sv.close()
    print(json.dumps(out), flush=True)
    return 0 if not bad and not sample_errors and not res["errors"] else 1


if __name__ == "__main__":
    sys.exit(main())
