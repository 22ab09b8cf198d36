"""Native HTTP front end (``csrc/native_server.hip``): the service's main port.

* ``POST /api/predict_eta`` and ``POST /predict`` are answered by C++ reactor threads — native
  JSON packing, one zero-copy fused-kernel launch per wake-up (natural batching across
  connections), CPython-exact response formatting.
* ``POST /api/optimize_route``, ``/route`` and ``/api/request_route`` go to one native route service
  per GPU (``csrc/route_service.hip``: cross-request batching, K5 + K6, the batched A*, C++ GeoJSON
  assembly byte-identical to the FastAPI handler, ``use_ml_eta`` on the fused MLP kernel, SQLite
  persistence into the Python store's database).
* Everything else — and any request whose semantics the native path does not mirror — is relayed
  to the FastAPI app listening on a private loopback port (``upstream_port``); a streamed answer
  (the SSE feed) turns its connection into a byte tunnel.

No Python runs on the native request paths.  ``python -m routest_amd serve`` puts this front end
on the main port (5000) with uvicorn behind it; the reference serves every route through Flask
(``RO/Flaskr/routes.py``), and single-request latency is host-stack bound.
"""
from __future__ import annotations

import socket
from typing import Dict, List, Optional, Sequence

import torch

from ..ops._ext import native
from ..ops.eta_mlp import EtaMlpKernel


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mlp_host(model) -> dict:
    """fp32 CPU copy of an EtaMLP for the native CPU fallback forward (csrc/native_model.h)."""
    m = model.float().cpu()
    return {"w1": m.l1.weight.detach().contiguous(), "b1": m.l1.bias.detach().contiguous(),
            "w2": m.l2.weight.detach().contiguous(), "b2": m.l2.bias.detach().contiguous(),
            "w3": m.l3.weight.detach().reshape(-1).contiguous(), "b3": float(m.l3.bias.detach()[0]),
            "x_mean": m.x_mean.detach().contiguous(), "x_std": m.x_std.detach().contiguous(),
            "y_mean": float(m.y_mean), "y_std": float(m.y_std)}


def native_supported(model) -> bool:
    """Model families the native front end serves: EtaMLP (H 64-1024) and tree ensembles."""
    from ..models.forest import ForestModel
    from ..models.mlp3 import EtaMLP
    return (isinstance(model, EtaMLP) and model.hidden in (64, 128, 256, 512, 1024)) or isinstance(model, ForestModel)


def native_model_spec(model, device: int, variant: int = -1) -> dict:
    """The native model spec of ``model`` on GPU ``device`` (bindings.cpp model_from): the fused
    K1+K2 blob for H <= 256, the wide kernel's packed weights for H = 512 / 1024, the packed trees
    of a forest; MLPs also carry an fp32 host copy for the CPU fallback."""
    from ..models.forest import ForestModel
    from ..models.mlp3 import EtaMLP
    dev = torch.device("cuda", device)
    if isinstance(model, EtaMLP) and model.hidden in (64, 128, 256):
        k = EtaMlpKernel(model, dev, variant=variant)
        return {"kind": "mlp3", "blob": k.packed.blob, "H": k.hidden, "norm": list(k.packed.norm),
                "variant": int(variant), "host": _mlp_host(model)}
    if isinstance(model, EtaMLP) and model.hidden in (512, 1024):
        from ..ops.mlp_big import PackedBig
        p = PackedBig(model.float().cpu(), dev)
        return {"kind": "wide", "H": p.hidden, "w1q": p.w1q, "w2f": p.w2f, "b2": p.b2, "w3": p.w3, "b3": p.b3,
                "norm": list(p.norm), "host": _mlp_host(model)}
    if isinstance(model, ForestModel):
        import numpy as np
        model.validate()
        return {"kind": "forest", "values": torch.from_numpy(np.ascontiguousarray(model.values)),
                "info": torch.from_numpy(np.ascontiguousarray(model.info.view(np.int32))),
                "roots": torch.from_numpy(np.ascontiguousarray(model.roots)), "base": float(model.base_score),
                "le": bool(model.le), "fmap": [int(x) for x in model.feature_map]}
    raise ValueError(f"the native front end does not serve {type(model).__name__} models")


class NativePredictServer:
    """``device``: one GPU index or a list — reactor threads are spread round-robin over the GPUs
    (each GPU slot gets its own model copy; use ``threads >= len(devices)``).

    Lifecycle (verdict r3 item 4): :meth:`set_model` hot-swaps the served model on
    every GPU slot (rounds in flight finish on the old weights; the resident scorers restart), a
    GPU slot whose launches keep failing is quarantined and its reactors' rounds run on the other
    GPUs — or on the model's fp32 CPU forward when none is left — and :meth:`health` reports it.
    ``history_db``: the store's SQLite file — GET/DELETE /api/history[/<id>] and GET /api/locations
    are then answered natively from it (csrc/runtime/history_db.h, byte-identical to the app).
    ``ROUTEST_FAULT=gpu_fail[@slot]`` (or :meth:`set_fault`) injects launch failures."""

    def __init__(self, model, device=0, port: int = 0, threads: int = 2, max_batch: int = 1 << 18,
                 cors_origins: Sequence[str] = ("http://localhost:3000", "http://127.0.0.1:3000"),
                 cors_vercel: bool = True, bind_any: bool = False, variant: int = -1,
                 upstream_port: int = 0, routes: Optional[List[dict]] = None, history_db: str = ""):
        self.C = native(required=True)
        self.devices = [device] if isinstance(device, int) else list(device)
        self.routes = list(routes or [])      # keeps the route configs' tensors alive
        self.variant = variant
        threads = max(threads, len(self.devices))
        self.port = port or free_port()
        specs = [native_model_spec(model, d, variant) for d in self.devices]
        self.model_epoch = 1
        self.h: Optional[int] = self.C.native_server_start(
            self.port, threads, self.devices, specs, max_batch, list(cors_origins), cors_vercel, bind_any,
            int(upstream_port), self.routes, history_db)
        self.history_db = history_db

    def set_model(self, model) -> int:
        """Hot swap on every GPU slot; returns the new model epoch.  ``None`` (a model family the
        native path does not serve): predictions are relayed to the app from then on."""
        specs = [native_model_spec(model, d, self.variant) if model is not None else {"kind": "none"}
                 for d in self.devices]
        self.model_epoch = int(self.C.native_server_set_models(self.h, self.devices, specs))
        return self.model_epoch

    def set_fault(self, slot: int, on: bool = True, kind: str = "fail") -> bool:
        """Fault injection on a GPU slot: ``fail`` — its launches fail without running; ``hang`` —
        its launches (predictions and route flushes) first run a kernel that waits on a host flag,
        so they miss the latency watchdog's deadline (``ROUTEST_GPU_DEADLINE_MS`` /
        ``ROUTEST_ROUTE_DEADLINE_MS``) until the fault is cleared."""
        if kind == "hang":
            return bool(self.C.native_server_set_hang(self.h, slot, on))
        return bool(self.C.native_server_set_fault(self.h, slot, on))

    def set_scorer(self, scorer) -> bool:
        """Publish the GCN scorer (routing/scorer.py RouteScorer) to the route services: requests with
        ``"alternatives"`` are then answered natively (csrc/route_service.hip); ``None`` withdraws it."""
        if self.h is None:
            return False
        if scorer is None:
            return bool(self.C.native_server_set_scorer(self.h, [], 0, ""))
        import numpy as np
        from ..routing.alternatives import KINDS
        delay = np.ascontiguousarray(scorer.node_delays(), dtype=np.float64)
        return bool(self.C.native_server_set_scorer(self.h, delay.tolist(), KINDS[getattr(scorer, "kind", "edge")],
                                                    str(getattr(scorer, "engine", "gcn"))))

    def health(self) -> Dict:
        if self.h is None:
            return {}
        h = dict(self.C.native_server_health(self.h))
        st = self.stats()
        h["stats"] = {k: st.get(k) for k in ("requests", "predictions", "launches", "errors", "resident",
                                             "fallbacks", "failovers", "cpu_rounds", "route_jobs",
                                             "route_flushes", "route_service_fallbacks", "route_legs",
                                             "route_contexts_built", "route_failed_over", "timeouts")}
        h["degraded"] = any(s["quarantined"] for s in h["slots"])
        return h

    def stats(self) -> Dict[str, int]:
        if self.h is None:
            return {}
        v = self.C.native_server_stats(self.h)
        # resident: rounds scored by the persistent kernel (csrc/persistent_serve.hip);
        # fallbacks: rounds it did not answer in time, re-scored by a normal launch;
        # wire8: launches that read 8-byte wire records (features.py RECORD8) instead of 16-byte;
        # route_*: the native route service (jobs, flushes, jobs handed to Python, unique legs
        # searched, legs finished on the host, rows persisted); relayed: requests sent to the app
        names = ("requests", "predictions", "launches", "errors", "resident", "fallbacks", "wire8",
                 "route_requests", "route_fallbacks", "relayed", "route_jobs", "route_flushes",
                 "route_service_fallbacks", "route_legs", "route_host_legs", "route_persisted",
                 # accumulated stage times of the route service (us)
                 "route_us_parse", "route_us_trips", "route_us_snap", "route_us_astar", "route_us_copyout",
                 "route_us_assemble", "route_us_eta", "route_us_persist",
                 # A* searches that overflowed a wave-tier table and were rerun in the big tier
                 "route_astar_escalated",
                 # CCH: routing contexts customized by the services, and their total build time (us)
                 "route_contexts_built", "route_us_context",
                 # multi-stop legs that reused their matrix chains (no second sweep)
                 "route_legs_reused",
                 # rounds re-run on another GPU slot (failover) / on the CPU forward (no GPU left)
                 "failovers", "cpu_rounds",
                 # history / locations requests answered from the store's database natively
                 "history_native",
                 # GET /api/health and /metrics answered from the front end's micro-cache
                 "cached",
                 # CCH contexts off the flush's critical path: jobs that waited for their context's
                 # background build, their total wait (us), next-week-hour contexts prefetched
                 "route_ctx_deferred", "route_us_ctx_wait", "route_ctx_prefetched",
                 # latency watchdog: route jobs handed to another GPU's route service after a
                 # flush missed its deadline; prediction rounds abandoned at the deadline
                 "route_failed_over", "timeouts",
                 # persisted graph routes stored as compact route records, and their bytes
                 "route_records", "route_record_bytes",
                 # the route services' GPU threads: collecting flushes, waiting for assembly (us)
                 "route_us_collect", "route_us_handoff")
        return dict(zip(names, v))

    def close(self) -> None:
        if self.h is not None:
            self.C.native_server_stop(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def route_config(provider, device, *, engine: str = "backend:mi355x", compat200: bool = True,
                 batch_max: int = 1024, timeout_us: int = 500, store=None, astar=None,
                 chunk_threads: int = 16) -> dict:
    """The native route service's configuration for one GPU (``csrc/route_service.h``).

    ``provider``: the app's HaversineProvider or GraphProvider.  A GraphProvider on the CCH engine
    hands over its router for ``device`` (the same ``_C.CchGpu`` object the app routes with, so both
    share the customized contexts and answer byte-identically); on the legacy A* engine ``astar`` is
    a :class:`~routest_amd.routing.graph.BatchedAstar` on ``device`` whose device tensors the service
    searches with (the caller keeps it alive).
    ``store``: the app's store — an :class:`SQLiteStore` is written natively (same database file);
    any other store kind is not mirrored, so route requests are then relayed to the Python app
    (the caller passes no route configs)."""
    name = getattr(provider, "name", "")
    cfg = {"provider": "graph" if name == "graph" else "haversine", "engine": engine,
           "compat200": bool(compat200), "batch_max": int(batch_max), "timeout_us": float(timeout_us),
           "chunk_threads": max(1, int(chunk_threads)),
           "circuity": float(getattr(provider, "circuity", 1.3)), "step_m": float(getattr(provider, "step_m", 150.0)),
           "sqlite_path": getattr(store, "sqlite_uri", "") if store is not None else ""}
    if name == "graph" and getattr(provider, "engine", "astar") != "astar":
        import numpy as np
        g = provider.g
        dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        router = provider.router(dev)
        if router.gpu is None:
            raise ValueError("the native route service needs the GPU router")
        cfg.update({
            "router": "cch", "cch_ptr": int(router.gpu.ptr()), "cch_contexts": bool(provider.uses_context),
            "cch_fixed_key": int(provider.FIXED_KEY),
            "glat": torch.from_numpy(np.ascontiguousarray(g.lat, dtype=np.float64)),
            "glon": torch.from_numpy(np.ascontiguousarray(g.lon, dtype=np.float64)),
            "h_indptr": torch.from_numpy(np.ascontiguousarray(g.indptr, dtype=np.int32)),
            "h_indices": torch.from_numpy(np.ascontiguousarray(g.indices, dtype=np.int32)),
            "h_length": torch.from_numpy(np.ascontiguousarray(g.length_m, dtype=np.float32)),
            "h_edge_name": (torch.from_numpy(np.ascontiguousarray(g.edge_name, dtype=np.int32))
                            if g.edge_name is not None else None),
            "names": list(g.names or []),
            "N": int(g.num_nodes), "snap_c": float(g.SNAP_C), "max_path": int(router.max_path),
            "_router": router})
        return cfg
    if name == "graph":
        import numpy as np
        a = astar
        if a is None or a.perm is not None:
            raise ValueError("graph routes need a BatchedAstar without node reordering")
        g = a.g
        cfg.update({
            "glat": torch.from_numpy(np.ascontiguousarray(g.lat, dtype=np.float64)),
            "glon": torch.from_numpy(np.ascontiguousarray(g.lon, dtype=np.float64)),
            "h_indptr": torch.from_numpy(np.ascontiguousarray(g.indptr, dtype=np.int32)),
            "h_indices": torch.from_numpy(np.ascontiguousarray(g.indices, dtype=np.int32)),
            "h_cost": a.cost.detach().cpu().contiguous(),
            "indptr": a.indptr, "indices": a.indices, "cost": a.cost, "lat32": a.lat, "lon32": a.lon,
            "lm": a.lm, "K": (a.lm.shape[1] // 2) if a.lm is not None else 0,
            "lane_ws": a.lane_tier.ws(), "wave_ws": a.wave_tier.ws() if a.wave_tier else None,
            "big_ws": a.big_tier.ws() if a.big_tier else None,
            "arena": a.arena, "arena_ctr": a.arena_ctr if a.arena is not None else None,
            "N": int(g.num_nodes), "snap_c": float(g.SNAP_C),
            "max_path": int(a.max_path), "max_iters": int(a.max_iters), "lane_pops": int(a.lane_pops),
            "wave_only_below": int(a.wave_only_below),
            "inv_vmax": float(a.inv_vmax), "wave_delta": float(a.wave_delta),
            "lane_max_m": float(a.lane_max_m),
            "_astar": a})
    return cfg


NativeFrontEnd = NativePredictServer
