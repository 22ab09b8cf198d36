"""HTTP API: the reference's 11 Flask routes under ``/api`` (``RO/Flaskr/routes.py``) + SSE mount
(``RO/Flaskr/__init__.py:28``), re-implemented on FastAPI/ASGI, plus the north-star aliases
``POST /predict`` (single or batched) and ``POST /route``, ``/metrics`` and admin endpoints.

Wire compatibility notes:
* ``/api/request_route`` returns **200** with an ``{"error": ...}`` body (quirk #1, behind
  ``compat_request_route_200``); ``/api/optimize_route`` returns 400 on errors.
* ``/api/predict_eta`` returns 503 ``{"error": "model unavailable"}`` without a model.
* ``/api/health`` is always HTTP 200 with keys ``backend, checks{engine,redis,supabase}, db, osrm,
  redis, tiles, status, version`` (+ ``gpu``, ``model``).
* ``/api/history`` without a store returns 503 like the detail route (fix #6; ``compat_history_500``
  restores the reference's 500).
* The SSE stream speaks Flask-SSE's wire format on ``/api/realtime_feed?channel=``.
"""
from __future__ import annotations

import asyncio
import datetime as dt
import json
import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from fastapi import FastAPI, Request
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import (HTMLResponse, JSONResponse, PlainTextResponse, Response,
                               StreamingResponse)
from starlette.concurrency import run_in_threadpool

from ..config import Settings, get_settings
from ..realtime.broker import MemoryBroker, Simulator, format_sse_data, make_broker
from ..routing.optimizer import optimize_many, optimize_route
from ..routing.providers import HaversineProvider, ORSProvider
from ..serve.eta_service import EtaService
from ..store.store import StoreUnavailable, open_store
from ..utils.logging import get_logger
from ..utils.metrics import REGISTRY

log = get_logger("api")


@dataclass
class Services:
    settings: Settings
    eta: EtaService
    provider: Any
    store: Any
    broker: MemoryBroker
    simulator: Simulator
    route_device: Optional[Any] = None
    route_batcher: Optional[Any] = None
    started: float = field(default_factory=time.time)
    scorer: Optional[Any] = None
    native: Optional[Any] = None        # the native front end owning the main port (serve/frontend.py)
    _scorer_lock: Any = field(default_factory=lambda: __import__("threading").Lock())

    def get_scorer(self):
        """Candidate-route scorer (GCN on the road graph), built on first use: the provider's graph
        when ``ROUTEST_PROVIDER=graph``, else a synthetic ``ROUTEST_GRAPH_NODES``-node graph.  It is
        trained for ``ROUTEST_SCORER_TRAIN_STEPS`` (HIP backward on a GPU):

        * ``ROUTEST_SCORER_TARGET=observed`` (default): on ``ROUTEST_SCORER_TRIPS`` observed trips of
          the seeded synthetic trip world (models/gcn_observed.py TripWorld: the edge-cost model's
          seconds plus hidden hot-spot / signal delays — offline there is no real trip log), so it
          predicts what the edge costs do not know;
        * ``edge``: the round-3 target, node delays from the learned edge times (gcn_train.py)."""
        with self._scorer_lock:
            if self.scorer is None:
                from ..routing.scorer import RouteScorer
                g = getattr(self.provider, "g", None)
                prov_graph = g is not None
                if g is None:
                    from ..data.graph import synth_road_graph
                    g = synth_road_graph(self.settings.graph_nodes)
                model, info = None, None
                kind = "edge"
                steps = int(self.settings.scorer_train_steps)
                if steps > 0:
                    cost = self._scorer_costs(g, prov_graph)
                    if self.settings.scorer_target == "observed":
                        from ..models.gcn_observed import TripWorld, train_observed
                        search = self._world_search(g, cost, prov_graph)
                        obs = TripWorld(g, cost, seed=3).observe(int(self.settings.scorer_trips), search, seed=1)
                        model, info = train_observed(g, obs, steps=steps, lr=1e-2, device=self.route_device,
                                                     log_every=steps)
                        kind = "observed"
                    else:
                        from ..models.gcn_train import train
                        model, info = train(g, cost, steps=steps, lr=5e-3, device=self.route_device, log_every=steps)
                self.scorer = RouteScorer(g, model=model, device=self.route_device, kind=kind)
                self.scorer.training = info
                hook = getattr(self, "on_scorer", None)
                if hook is not None:
                    try:
                        hook(self.scorer)
                    except Exception as e:  # noqa: BLE001
                        log.warning("scorer hook failed: %r", e)
            return self.scorer

    def _scorer_costs(self, g, prov_graph: bool):
        """Edge seconds the scorer's world starts from: the provider's fixed costs, its default
        context's costs (context-aware CCH provider), or the ETA model's over a synthetic graph."""
        import numpy as np
        if prov_graph:
            if getattr(self.provider, "cost", None) is not None:
                return np.asarray(self.provider.cost, dtype=np.float32)
            if hasattr(self.provider, "metric_key"):
                return self.provider.edge_seconds(self.provider.metric_key(None))
        from ..models.mlp3 import EtaMLP
        from ..routing.graph import edge_costs
        m = getattr(self.eta, "model", None)
        if isinstance(m, EtaMLP):
            return edge_costs(g, m, device=self.route_device)
        from ..data.graph import CLASS_SPEED_KMH
        return (g.length_m / (CLASS_SPEED_KMH[g.road_class] / 3.6)).astype("float32")

    def _world_search(self, g, cost, prov_graph: bool):
        """(src, dst) -> [(seconds, path)] exact on ``cost`` (the CCH router of that metric)."""
        from ..routing.cch import RoadRouter
        if prov_graph and hasattr(self.provider, "router"):
            r = self.provider.router()
        else:
            r = RoadRouter(g, device=self.route_device)
        key = r.metric_from_costs(1 << 43, cost)

        def search(src, dst):
            sec, _, st, paths = r.route(src, dst, key)
            return [(float(sec[i]), paths[i].tolist()) if st[i] == 0 else (float("nan"), []) for i in range(len(src))]
        return search

    def graph_search(self):
        """(src, dst) -> [(seconds, node path)] on the provider's graph: the route batcher's batched
        A* workspace on the GPU (under its lock), else host Dijkstra."""
        rb, dev = self.route_batcher, self.route_device
        if rb is not None and dev is not None:
            astar, lock = rb._astar_for(dev)

            def search(src, dst):
                with lock:
                    return astar.paths(src, dst)
            return search
        return lambda src, dst: self.provider._shortest(list(zip(src, dst)))

    def warm_scorer_async(self) -> None:
        """Build the scorer (graph + GCN + first node-delay pass) on a background thread at
        startup, so the first /api/score_routes does not pay for it."""
        import threading

        def _warm():
            try:
                sc = self.get_scorer()
                if hasattr(sc, "warm"):
                    sc.warm()
            except Exception as e:  # pragma: no cover - the request path retries on demand
                log.warning("scorer warm-up failed: %r", e)
        threading.Thread(target=_warm, name="scorer-warmup", daemon=True).start()

    def close(self) -> None:
        if self.route_batcher is not None:
            self.route_batcher.close()
            self.route_batcher = None
        self.eta.close()


def _gpu_devices(s: Settings) -> List[Any]:
    try:
        import torch
        if s.device == "cpu" or not torch.cuda.is_available():
            return []
        return [torch.device("cuda", i) for i in (s.devices or range(torch.cuda.device_count()))]
    except Exception:
        return []


def build_services(settings: Optional[Settings] = None, eta: Optional[EtaService] = None,
                   provider: Any = None, store: Any = "default") -> Services:
    s = settings or get_settings()
    if eta is None:
        model_path = s.default_model_dir or s.eta_model_path
        import os
        eta = EtaService(model_path=model_path, device=s.device, devices=s.devices,
                         batch_max=s.batch_max, timeout_us=s.batch_timeout_us,
                         allow_pickle=os.environ.get("ROUTEST_ALLOW_PICKLE") == "1")
    gpus = _gpu_devices(s)
    route_device = gpus[0] if gpus else None
    if provider is None:
        if s.provider == "ors" and s.ors_api_key:
            provider = ORSProvider(s.ors_api_key)
        elif s.provider == "graph":
            from ..routing.graph import GraphProvider
            if s.graph_path:
                provider = GraphProvider.from_path(s.graph_path, device=route_device)
            else:
                provider = GraphProvider.synthetic(num_nodes=s.graph_nodes, device=route_device)
        else:
            provider = HaversineProvider()
    if store == "default":
        store = open_store(s.store_url, s.supabase_url, s.supabase_service_key)
    # compact route records (native route service) are rebuilt against the provider's road graph
    steps = getattr(provider, "_steps", None)
    if steps is not None and hasattr(store, "set_record_graph"):
        store.set_record_graph(steps)
    broker = make_broker(s.broker, s.redis_url)
    sim = Simulator(broker, s.sim_tick_min_s, s.sim_tick_max_s, s.max_simulations, s.sse_delta)
    # cross-request optimizer batching (routing/route_batcher.py): one worker per GPU
    batcher = None
    batchable = getattr(provider, "name", "") in ("haversine", "graph")
    if batchable and (s.route_batch in ("1", "true", "on") or (s.route_batch == "auto" and gpus)):
        from ..routing.route_batcher import RouteBatcher
        batcher = RouteBatcher(provider, s.engine_name, gpus or [None], batch_max=s.route_batch_max,
                               timeout_us=s.route_batch_timeout_us)
    return Services(s, eta, provider, store, broker, sim, route_device, route_batcher=batcher)


class _MetricsASGI:
    """Pure-ASGI timing middleware (cheaper than BaseHTTPMiddleware)."""

    def __init__(self, app):
        self.app = app

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        t0 = time.perf_counter()
        status = {"code": 500}

        async def _send(msg):
            if msg["type"] == "http.response.start":
                status["code"] = msg["status"]
            await send(msg)
        try:
            await self.app(scope, receive, _send)
        finally:
            path = scope.get("path", "")
            if not path.startswith("/api/realtime_feed"):
                REGISTRY.latency.observe(time.perf_counter() - t0)
            REGISTRY.requests.inc(route=path if path.count("/") <= 2 else path.rsplit("/", 1)[0],
                                  status=str(status["code"]))


class _FastPredictASGI:
    """Pure-ASGI fast path for single-item ``POST /api/predict_eta`` and ``POST /predict``,
    dispatched by :class:`RoutestApp` ahead of Starlette's whole middleware stack.

    The request body goes straight to the native packer (``_rt.pack_predict_batch``: C++ JSON ->
    16-byte record with the reference's field semantics), the record to the micro-batcher, and the
    minutes back through the native formatter — no FastAPI routing, Request object, ``json.loads``
    or ``JSONResponse`` rendering on the hot path.  Anything that is not a clean single prediction
    (pack error, batch body, model unavailable, no native runtime) is replayed unchanged into the
    FastAPI handler, which owns the error semantics (RO/Flaskr/routes.py:365-383)."""

    PATHS = (b"/api/predict_eta", b"/predict")

    def __init__(self, app, sv, rt_native):
        self.app, self.sv, self.rt = app, sv, rt_native

    def matches(self, scope) -> bool:
        if scope["type"] != "http" or scope["method"] != "POST" or self.rt is None:
            return False
        if scope.get("raw_path", scope["path"].encode()) not in self.PATHS:
            return False
        for k, _ in scope.get("headers", ()):
            if k == b"origin":          # cross-origin: let CORSMiddleware add its headers
                return False
        return True

    async def __call__(self, scope, receive, send):
        t0 = time.perf_counter()
        chunks = []
        more = True
        while more:
            msg = await receive()
            if msg["type"] != "http.request":
                return await self.app(scope, _replay(b"".join(chunks), msg), send)
            chunks.append(msg.get("body", b""))
            more = msg.get("more_body", False)
        raw = b"".join(chunks)
        out = await self._try(scope, raw)
        if out is None:
            return await self.app(scope, _replay(raw), send)
        await send({"type": "http.response.start", "status": 200,
                    "headers": [(b"content-type", b"application/json"),
                                (b"content-length", str(len(out)).encode())]})
        await send({"type": "http.response.body", "body": out})
        REGISTRY.latency.observe(time.perf_counter() - t0)
        REGISTRY.requests.inc(route=scope["path"], status="200")

    async def _try(self, scope, raw: bytes):
        ctype = b""
        for k, v in scope.get("headers", ()):
            if k == b"content-type":
                ctype = v
        if b"json" not in ctype.lower():
            raw = b"{}"                 # Flask get_json(silent=True) -> None -> {} (both routes)
        eta = self.sv.eta
        if eta.batcher is None or not eta.available:
            return None
        now = dt.datetime.now()
        now_secs = int((now - dt.datetime(1970, 1, 1)).total_seconds() // 1)
        try:
            rec_u8, secs, us, tz, errs, is_batch = self.rt.pack_predict_batch(raw, now_secs, now.microsecond)
        except Exception:
            return None                 # malformed JSON: the handler applies silent semantics
        if is_batch or errs[0]:
            return None
        from ..models.features import RECORD_DTYPE
        rec = rec_u8.view(RECORD_DTYPE).reshape(-1)[0].item()
        try:
            minutes = await eta.batcher.submit(rec)
        except Exception:
            return None
        import numpy as np
        REGISTRY.preds.inc()
        return self.rt.format_predict_batch(np.array([minutes], dtype=np.float32), secs, us, tz, errs, False)


class RoutestApp(FastAPI):
    """FastAPI app whose ASGI entry first offers the request to the native single-predict fast
    path (``fast``); everything else takes the normal middleware + router stack."""

    fast: Optional[_FastPredictASGI] = None

    async def __call__(self, scope, receive, send):
        f = self.fast
        if f is not None and f.matches(scope):
            return await f(scope, receive, send)
        return await super().__call__(scope, receive, send)


def _replay(body: bytes, tail=None):
    sent = [False]

    async def receive():
        if not sent[0]:
            sent[0] = True
            return {"type": "http.request", "body": body, "more_body": False}
        if tail is not None:
            return tail
        return {"type": "http.disconnect"}
    return receive


async def _call(obj, fn, *args):
    """Run ``fn`` inline when its owner is local CPU work (``obj.blocking`` False), otherwise in the
    thread pool: a thread hop costs more than the sub-millisecond haversine optimizer or SQLite
    insert it would wrap, while remote / GPU-synchronising calls must not block the event loop."""
    if getattr(obj, "blocking", True):
        return await run_in_threadpool(fn, *args)
    return fn(*args)


async def _json_body(request: Request, silent: bool):
    """Flask ``get_json()`` semantics: non-silent -> 415 on non-JSON content type, 400 on bad JSON;
    silent -> None on either."""
    ctype = request.headers.get("content-type", "")
    raw = await request.body()
    if "json" not in ctype.lower():
        if silent:
            return None
        return JSONResponse({"error": "Unsupported Media Type: expected application/json"}, 415)
    try:
        return json.loads(raw) if raw else None
    except ValueError:
        if silent:
            return None
        return JSONResponse({"error": "Bad Request: failed to decode JSON object"}, 400)


def create_app(services: Optional[Services] = None, settings: Optional[Settings] = None) -> FastAPI:
    sv = services or build_services(settings)
    s = sv.settings

    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(_app):
        if s.warm_scorer and sv.route_device is not None:
            sv.warm_scorer_async()
        yield
        await sv.simulator.shutdown()
        sv.close()

    app = RoutestApp(title="routest_amd", version="1.0", lifespan=lifespan)
    app.state.services = sv
    rt_fast = None
    if s.fast_predict:
        try:
            from ..ops import _ext
            rt_fast = _ext.runtime(required=False)
        except Exception:  # pragma: no cover
            rt_fast = None
    app.add_middleware(CORSMiddleware, allow_origins=s.cors_origins,
                       allow_origin_regex=s.cors_origin_regex, allow_credentials=True,
                       allow_methods=["*"], allow_headers=["*"])
    app.add_middleware(_MetricsASGI)
    if rt_fast is not None:
        # fall-through requests re-enter the full stack (middleware + router) with the body replayed
        app.fast = _FastPredictASGI(super(RoutestApp, app).__call__, sv, rt_fast)

    # ------------------------------------------------------------------ routing
    async def _optimize_one(payload):
        """One request through the cross-request GPU batcher when enabled, else inline.  With the
        road-graph provider every request is batched (one A* launch per flush: 9x the per-request
        req/s); haversine requests below ``route_gpu_min_stops`` destinations stay inline (their
        10x10 greedy is cheaper than a queue hop: 1.26k vs 0.97k req/s, profiles/superseded/route_http_r2.jsonl)."""
        if sv.route_batcher is not None:
            dests = payload.get("destination_points") if isinstance(payload, dict) else None
            if (getattr(sv.provider, "name", "") == "graph" or
                    (isinstance(dests, list) and len(dests) >= s.route_gpu_min_stops)):
                return await sv.route_batcher.submit(payload)
        return await _call(sv.provider, optimize_route, payload, sv.provider, s.engine_name)

    async def _route(payload):
        """One optimizer answer: ranked alternatives when the request asks for them (graph
        provider, routing/alternatives.py), else the batched / inline optimizer."""
        alt = payload.get("alternatives") if isinstance(payload, dict) else None
        if alt and not isinstance(alt, bool) and isinstance(alt, (int, float)) and alt >= 2:
            from ..routing.alternatives import optimize_with_alternatives
            scorer = await run_in_threadpool(sv.get_scorer)
            # road providers route the candidates themselves (provider.legs); others need a search
            search = None if hasattr(sv.provider, "legs") else sv.graph_search()
            return await run_in_threadpool(optimize_with_alternatives, payload, sv.provider, scorer,
                                           search, s.engine_name, int(alt))
        return await _optimize_one(payload)

    @app.post("/api/request_route")
    async def request_route(request: Request):
        data = await _json_body(request, silent=False)
        if isinstance(data, Response):
            return data
        result = await _route(data)
        if not result:
            return JSONResponse({"error": "no response acquired from the optimizer."}, 400)
        if isinstance(result, dict) and result.get("error") and not s.compat_request_route_200:
            return JSONResponse(result, 400)
        return JSONResponse(result, 200)

    async def _optimize(request: Request):
        payload = await _json_body(request, silent=True) or {}
        if not isinstance(payload, dict):
            payload = {}
        result = await _route(payload)
        if isinstance(result, dict) and result.get("error"):
            return JSONResponse(result, 400)
        if payload.get("use_ml_eta"):
            props = result.setdefault("properties", {}) or {}
            summary = props.get("summary", {}) or {}
            try:
                distance_m = float(summary.get("distance") or 0)
                ctx = payload.get("context") or {}
                driver_age = float((payload.get("driver_details") or {}).get("driver_age", 30))
                eta_min, eta_iso = await sv.eta.apredict(
                    weather=ctx.get("weather", "Sunny"), traffic=ctx.get("traffic", "Low"),
                    distance_m=distance_m, pickup_time=dt.datetime.now(), driver_age=driver_age)
            except (TypeError, ValueError):
                eta_min, eta_iso = None, None
            if eta_min is not None:
                props["eta_minutes_ml"] = eta_min
                props["eta_completion_time_ml"] = eta_iso
        if sv.store is not None:
            try:
                rid = await _call(sv.store, sv.store.persist_request_and_result, payload, result)
                if rid:
                    result.setdefault("properties", {})["request_id"] = rid
                    result["properties"]["saved"] = True
            except Exception as e:  # best-effort persistence (routes.py:119-125)
                log.warning("Persist failed: %r", e)
        return JSONResponse(result, 200)

    app.post("/api/optimize_route")(_optimize)
    app.post("/route")(_optimize)

    @app.post("/api/optimize_routes_batch")
    async def optimize_batch(request: Request):
        """Many independent requests in one call: K5+K6 batched on the GPU."""
        body = await _json_body(request, silent=True)
        reqs = body.get("requests") if isinstance(body, dict) else body
        if not isinstance(reqs, list):
            return JSONResponse({"error": "expected a JSON array of route requests"}, 400)
        if sv.route_batcher is not None:
            res = await run_in_threadpool(sv.route_batcher.run_batch, reqs, sv.route_device)
        else:
            res = await run_in_threadpool(optimize_many, reqs, sv.provider, s.engine_name, sv.route_device)
        return JSONResponse({"results": res}, 200)

    @app.post("/api/score_routes")
    async def score_routes(request: Request):
        """Rank candidate routes with the GCN road-graph scorer (HIP kernels on the GPU).
        Body: {"routes": [[[lon, lat], ...] | {"coordinates": ...} | {"nodes": [...]} , ...]}."""
        body = await _json_body(request, silent=False)
        if isinstance(body, Response):
            return body
        routes = body.get("routes") if isinstance(body, dict) else body
        if not isinstance(routes, list) or not routes:
            return JSONResponse({"error": "expected {'routes': [route, ...]}"}, 400)
        scorer = await run_in_threadpool(sv.get_scorer)
        try:
            res = await _call(scorer, scorer.score, routes)
        except (ValueError, TypeError) as e:
            return JSONResponse({"error": f"invalid route: {e}"}, 400)
        return JSONResponse(res, 200)

    # ------------------------------------------------------------------ ETA
    async def _predict_one(body: Dict[str, Any]):
        summary = body.get("summary") or {}
        pickup = body.get("pickup_time") or dt.datetime.now().isoformat()
        try:
            driver_age = float(body.get("driver_age", 30))
            distance_m = float(summary.get("distance") or 0) if isinstance(summary, dict) else 0.0
            if isinstance(pickup, str):
                from ..utils.timeutil import parse_iso
                parse_iso(pickup)
        except (TypeError, ValueError) as e:
            return None, None, f"invalid input: {e}"
        if not sv.eta.available:
            return None, None, None
        m, iso = await sv.eta.apredict(weather=body.get("weather", "Sunny"),
                                       traffic=body.get("traffic", "Low"), distance_m=distance_m,
                                       pickup_time=pickup, driver_age=driver_age)
        return m, iso, None

    @app.post("/api/predict_eta")
    async def predict_eta(request: Request):
        body = await _json_body(request, silent=True) or {}
        if not isinstance(body, dict):
            body = {}
        m, iso, err = await _predict_one(body)
        if err:
            return JSONResponse({"error": err}, 400)
        if m is None:
            return JSONResponse({"error": "model unavailable"}, 503)
        REGISTRY.preds.inc()
        return JSONResponse({"eta_minutes_ml": m, "eta_completion_time_ml": iso}, 200)

    rt_native = None
    try:
        from ..ops import _ext
        rt_native = _ext.runtime(required=False)
    except Exception:  # pragma: no cover
        rt_native = None

    async def _predict_native(raw: bytes):
        """Batched /predict fully in native code: C++ JSON -> records, ONE fused kernel launch for
        the whole array, C++ response formatting (routest_amd._rt)."""
        now = dt.datetime.now()
        now_secs = int((now - dt.datetime(1970, 1, 1)).total_seconds() // 1)
        try:
            rec_u8, secs, us, tz, errs, is_batch = rt_native.pack_predict_batch(raw, now_secs, now.microsecond)
        except Exception as e:
            return JSONResponse({"error": str(e)}, 400)
        if not sv.eta.available:
            return JSONResponse({"error": "model unavailable"}, 503)
        import numpy as np
        from ..models.features import RECORD_DTYPE
        rec = rec_u8.view(RECORD_DTYPE).reshape(-1)
        ok = np.array([not e for e in errs], dtype=bool)
        minutes = np.zeros(len(errs), dtype=np.float32)
        if ok.any():
            minutes[ok] = await run_in_threadpool(sv.eta.predict_records, rec[ok])
        REGISTRY.preds.inc(int(ok.sum()))
        out = rt_native.format_predict_batch(minutes, secs, us, tz, errs, is_batch)
        return Response(out, media_type="application/json")

    @app.post("/predict")
    async def predict(request: Request):
        raw = await request.body()
        head = raw.lstrip()[:1]
        if rt_native is not None and head == b"[" and "json" in request.headers.get("content-type", ""):
            return await _predict_native(raw)
        body = await _json_body(request, silent=True)
        items = body if isinstance(body, list) else (body.get("items") if isinstance(body, dict) and
                                                     isinstance(body.get("items"), list) else None)
        if items is None:
            return await predict_eta(request)
        res = await asyncio.gather(*[_predict_one(b if isinstance(b, dict) else {}) for b in items])
        if any(m is None and err is None for m, _, err in res):
            return JSONResponse({"error": "model unavailable"}, 503)
        REGISTRY.preds.inc(len(items))
        return JSONResponse({"predictions": [
            {"error": err} if err else {"eta_minutes_ml": m, "eta_completion_time_ml": iso}
            for m, iso, err in res]}, 200)

    @app.post("/api/admin/reload_model")
    async def reload_model(request: Request):
        body = await _json_body(request, silent=True) or {}
        path = body.get("path") if isinstance(body, dict) else None
        ok = await run_in_threadpool(sv.eta.reload, path)
        return JSONResponse({"ok": ok, "model": sv.eta.describe()}, 200 if ok else 503)

    # ------------------------------------------------------------------ realtime
    @app.post("/api/confirm_route")
    async def confirm_route(request: Request):
        data = await _json_body(request, silent=False)
        if isinstance(data, Response):
            return data
        if not isinstance(data, dict) or not sv.simulator.start(data):
            if isinstance(data, dict):
                return JSONResponse({"error": "too many active simulations"}, 503)
        return JSONResponse({"status": "route simulation initialized."}, 200)

    @app.post("/api/update_tracker")
    async def update_tracker(request: Request):
        data = await _json_body(request, silent=False)
        if isinstance(data, Response):
            return data
        if not data:
            return JSONResponse({"error": "no data provided in the publish request."}, 400)
        try:
            msg = format_sse_data(data)
        except (KeyError, TypeError, ValueError) as e:
            return JSONResponse({"error": f"invalid tracker payload: {e!r}"}, 400)
        sv.broker.publish(msg, channel=f"{data.get('route_id')}")
        return JSONResponse({"status": "published"}, 200)

    @app.get("/api/realtime_feed")
    async def realtime_feed(request: Request, channel: str = "sse"):
        q = sv.broker.subscribe(channel)

        async def gen():
            try:
                yield ": connected\n\n"
                while True:
                    try:
                        msg = await asyncio.wait_for(q.get(), timeout=15.0)
                        yield msg
                    except asyncio.TimeoutError:
                        yield ": keep-alive\n\n"
                    if await request.is_disconnected():
                        break
            finally:
                sv.broker.unsubscribe(channel, q)
        return StreamingResponse(gen(), media_type="text/event-stream",
                                 headers={"Cache-Control": "no-cache", "X-Accel-Buffering": "no"})

    # ------------------------------------------------------------------ misc
    @app.get("/api/ping")
    async def ping():
        return JSONResponse({"ok": True, "service": "route-optimizer"}, 200)

    @app.get("/api/health")
    async def health():
        from .health import health_payload
        return JSONResponse(await run_in_threadpool(health_payload, sv), 200)

    @app.get("/api/locations")
    async def locations():
        if sv.store is not None and hasattr(sv.store, "locations"):
            try:
                return JSONResponse(await _call(sv.store, sv.store.locations), 200)
            except Exception as e:
                return JSONResponse({"error": str(e)}, 500)
        from ..data.synth import seed_locations
        return JSONResponse(seed_locations(), 200)

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(REGISTRY.render(), media_type="text/plain; version=0.0.4")

    # ------------------------------------------------------------------ history
    def _no_store() -> JSONResponse:
        if s.compat_history_500:
            return JSONResponse({"error": "supabase fetch failed (status n/a): not configured"}, 500)
        return JSONResponse({"error": "history disabled: SUPABASE not configured"}, 503)

    @app.get("/api/history")
    async def history(limit: str = "20"):
        try:
            lim = int(limit)
        except ValueError:
            lim = 20
        lim = max(1, min(lim, 100))
        if sv.store is None:
            return _no_store()
        try:
            items = await _call(sv.store, sv.store.history, lim)
        except Exception as e:
            return JSONResponse({"error": f"history fetch failed: {e}"}, 500)
        return JSONResponse({"items": items}, 200)

    @app.get("/api/history/{req_id}")
    async def history_detail(req_id: str):
        if sv.store is None:
            return JSONResponse({"error": "history disabled: SUPABASE not configured"}, 503)
        try:
            d = await _call(sv.store, sv.store.history_detail, req_id)
        except Exception as e:
            return JSONResponse({"error": f"history fetch failed: {e}"}, 500)
        if d is None:
            return JSONResponse({"error": "not found"}, 404)
        return JSONResponse(d, 200)

    @app.delete("/api/history/{req_id}")
    async def delete_history(req_id: str):
        if sv.store is None:
            return JSONResponse({"error": "history disabled: SUPABASE not configured"}, 503)
        try:
            await _call(sv.store, sv.store.delete, req_id)
        except StoreUnavailable as e:
            return JSONResponse({"error": str(e)}, 500)
        except Exception as e:
            return JSONResponse({"error": f"delete failed: {e}"}, 500)
        return Response(status_code=204)

    # ------------------------------------------------------------------ built-in dashboard (F01-F09)
    ui_cache: Dict[str, str] = {}

    def _dashboard() -> HTMLResponse:
        if "html" not in ui_cache:
            with open(os.path.join(os.path.dirname(__file__), "static", "dashboard.html"), encoding="utf-8") as f:
                ui_cache["html"] = f.read()
        return HTMLResponse(ui_cache["html"])

    @app.get("/ui", include_in_schema=False)
    @app.get("/ui/", include_in_schema=False)
    @app.get("/ui/history", include_in_schema=False)
    @app.get("/ui/health", include_in_schema=False)
    async def ui_page():
        return _dashboard()

    @app.get("/ui/history/{req_id}", include_in_schema=False)
    async def ui_history_detail(req_id: str):
        return _dashboard()

    return app
