"""Assemble the serving stack: the native front end on the main port, the FastAPI app behind it.

    client ──HTTP──> native front end (C++ reactors, csrc/native_server.hip)  :5000
                       ├─ /api/predict_eta, /predict ........ fused K1+K2 kernel
                       ├─ /api/optimize_route, /route,
                       │  /api/request_route ................ native route service per GPU
                       │                                       (CCH road matrices + K6 + CCH legs
                       │                                        + C++ GeoJSON with maneuvers)
                       ├─ /api/history[/<id>] (GET, DELETE),
                       │  /api/locations .................... the store's SQLite file, natively
                       └─ everything else, and requests the native paths do not mirror
                                                 ──relay──> FastAPI app (uvicorn)  127.0.0.1:<private>

The reference serves all of it from one Flask process (``RO/app.py:8``, gunicorn in
``RO/requirements.txt:10``).  Here the request paths that carry the traffic never enter Python,
and the Python app keeps the long tail (history, health, SSE, admin, scorer) with identical
semantics — byte-identical bodies on the shared routes (tests/test_frontend_gpu.py).
"""
from __future__ import annotations

import threading
import time
from typing import Any, List, Optional, Sequence

from ..utils.logging import get_logger

log = get_logger("frontend")


class AppServer:
    """uvicorn serving ``app`` on 127.0.0.1:``port`` from a background thread (the relay target)."""

    def __init__(self, app, port: int = 0, host: str = "127.0.0.1", log_level: str = "warning"):
        import uvicorn
        from .native_server import free_port
        self.port = port or free_port()
        self.server = uvicorn.Server(uvicorn.Config(app, host=host, port=self.port, log_level=log_level,
                                                    access_log=False, lifespan="on"))
        self.thread = threading.Thread(target=self.server.run, name="uvicorn-app", daemon=True)
        self.thread.start()
        t0 = time.time()
        while not self.server.started:
            if not self.thread.is_alive() or time.time() - t0 > 60:
                raise RuntimeError("the FastAPI app server did not start")
            time.sleep(0.01)

    def close(self) -> None:
        self.server.should_exit = True
        self.thread.join(timeout=15)


def native_route_reason(sv) -> Optional[str]:
    """None if the native route service can answer this app's route requests, else why not."""
    name = getattr(sv.provider, "name", "")
    if name not in ("haversine", "graph"):
        return f"provider {name!r} (remote calls) stays in Python"
    st = sv.store
    if st is not None and getattr(st, "kind", "") != "sqlite":
        return f"store {getattr(st, 'kind', type(st).__name__)!r} is written by the Python app only"
    if name == "graph" and getattr(sv.provider, "device", None) is None:
        return "road-graph provider without a GPU"
    return None


def route_pipelines_for(sv) -> int:
    """Native route services per GPU: ``settings.route_pipelines`` if set, else 2 when the route
    service persists every answer itself (SQLite store) and 1 otherwise.

    Measured on one MI355X (profiles/route_pipelines_r6ax.md): with persistence, a flush holds its
    GPU thread ~4 ms and then ~4 ms of assembly + group commit, so a second service per GPU keeps the
    GPU fed — the dashboard's request went 51.8k -> 85.0k req/s, p99 22.3 -> 15.1 ms.  Without a
    store the route path is bound by response bytes (~7.5 GB/s of GeoJSON over loopback): a second
    service added 6 % throughput but moved p99 from 14 to 34 ms, so it stays at one."""
    k = int(getattr(sv.settings, "route_pipelines", 0) or 0)
    if k > 0:
        return k
    st = sv.store
    return 2 if st is not None and getattr(st, "kind", "") == "sqlite" else 1


def route_configs(sv, devices: Sequence[int], batch_max: int = 1024, timeout_us: int = 500,
                  chunk_threads: int = 16) -> List[dict]:
    """One native route service config per slot (serve/native_server.py route_config).

    ``chunk_threads``: host fan-out per parallel_chunks call of each service.  Halving it with two
    services per GPU cut the no-store p99 from 34 to 24 ms but did not help the persisted path
    (profiles/route_pipelines_r6ax.md, run r6bb), so it stays at 16."""
    import torch
    from .native_server import route_config
    s = sv.settings
    out = []
    for d in devices:
        astar = None
        if getattr(sv.provider, "name", "") == "graph" and getattr(sv.provider, "engine", "astar") == "astar":
            from ..routing.graph import BatchedAstar
            astar = BatchedAstar(sv.provider.g, sv.provider.cost, torch.device("cuda", d),
                                 slots=int(getattr(s, "route_astar_slots", 8192)))
        out.append(route_config(sv.provider, d, engine=s.engine_name, compat200=s.compat_request_route_200,
                                batch_max=batch_max, timeout_us=timeout_us, store=sv.store, astar=astar,
                                chunk_threads=chunk_threads))
    return out


def start_front_end(sv, model, devices: Sequence[int], port: int = 0, upstream_port: int = 0,
                    threads: int = 8, bind_any: bool = False, routes: bool = True,
                    batch_max: Optional[int] = None, timeout_us: Optional[int] = None,
                    cors_origins: Optional[Sequence[str]] = None):
    """Start the native front end for ``sv``'s app (relaying to ``upstream_port``)."""
    from .native_server import NativePredictServer
    s = sv.settings
    cfgs: List[dict] = []
    if routes:
        why = native_route_reason(sv)
        if why is None:
            # route_pipelines > 1: that many slots (route service + scorer) per GPU; the reactors
            # spread over the slots, so the GPU stages of one flush overlap the host stages
            # (assembly, persistence) of another on the same GPU.  Slots go round by round over the
            # GPUs ([0, 1, .., 0, 1, ..]): a failover goes to slot + 1 first
            # (csrc/native_server.hip), which is then another GPU, not the hung one's sibling
            k = route_pipelines_for(sv)
            devices = [d for _ in range(k) for d in devices]
            cfgs = route_configs(sv, devices, batch_max or s.route_batch_max,
                                 timeout_us if timeout_us is not None else s.route_batch_timeout_us)
        else:
            log.info("route requests relayed to the Python app: %s", why)
    # history / locations read natively from the SQLite store (the app still owns writes it makes)
    from ..utils.faults import active_faults
    hist = ""
    st = sv.store
    if st is not None and getattr(st, "kind", "") == "sqlite" and "store_fail" not in active_faults():
        hist = st.sqlite_uri
    srv = NativePredictServer(model, device=list(devices), port=port, threads=max(threads, len(devices)),
                              cors_origins=cors_origins if cors_origins is not None else s.cors_origins,
                              bind_any=bind_any, upstream_port=upstream_port, routes=cfgs, history_db=hist)
    return srv


class ServingStack:
    """FastAPI app on a private port + the native front end on ``port`` (tests, benches, serve)."""

    def __init__(self, sv, app, model, devices: Sequence[int], port: int = 0, threads: int = 8,
                 bind_any: bool = False, routes: bool = True, **kw: Any):
        self.app_server = AppServer(app)
        try:
            self.front = start_front_end(sv, model, devices, port=port, upstream_port=self.app_server.port,
                                         threads=threads, bind_any=bind_any, routes=routes, **kw)
        except BaseException:
            self.app_server.close()
            raise
        self.port = self.front.port
        # the app reports the native front end's state in /api/health, and a model (re)load in the
        # app (/api/admin/reload_model) is hot-swapped into the native front end
        self.sv = sv
        sv.native = self.front
        self._hook = self._swap
        sv.eta.on_activate.append(self._hook)
        # the GCN scorer, once trained, serves "alternatives" requests natively too
        if self.front.routes:
            sv.on_scorer = self.front.set_scorer
            if getattr(sv, "scorer", None) is not None:
                self.front.set_scorer(sv.scorer)

    def _swap(self, model) -> None:
        from .native_server import native_supported
        self.front.set_model(model if native_supported(model) else None)

    def close(self) -> None:
        try:
            self.sv.eta.on_activate.remove(self._hook)
        except ValueError:
            pass
        self.sv.native = None
        if getattr(self.sv, "on_scorer", None) == self.front.set_scorer:
            self.sv.on_scorer = None
        self.front.close()
        self.app_server.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
