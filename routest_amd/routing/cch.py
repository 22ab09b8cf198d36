"""Context-aware road routing on a customizable contraction hierarchy (CCH).

The reference routes every trip through the remote OpenRouteService (directions per trip and a
distance matrix per request, ``RO/Flaskr/utils.py:55-62,97-105,151-156``) and reads the request's
``context.weather`` / ``context.traffic`` only for its ETA (``Flaskr/routes.py:102-104``).  Here the
road times themselves depend on the context: each (weather, city-wide traffic level, week-hour)
gets edge costs from the ETA MLP (``routing/graph.py`` edge model) and its own customization of one
metric-independent hierarchy, cached on the GPU ("precomputed per (graph, context) and
cached").

* :class:`RouteContext` — the context of one request (the dashboard sends ``weather: "Sunny",
  traffic: "Medium"``; defaults ``Sunny`` / ``Low`` like the reference's ETA; week-hour of
  ``context.pickup_time`` when it is an ISO string, else of now, local time).
* :class:`RoadRouter` — legs and many-to-many matrices under a context.  GPU: ``_C.CchGpu``
  (csrc/cch.hip: costs, customization and queries all on the device, LRU of customized contexts in
  HBM).  CPU: ``_rt.CCH`` (csrc/runtime/cch.h, the bit-identical reference, multi-threaded).

Legs come back as (seconds, metres, status, node path); a matrix entry is the metre length of the
time-shortest road path, which is exactly what a trip over those legs reports — so the greedy's
``maximum_distance`` (R21) is checked on the distances the response will carry.
"""
from __future__ import annotations

import datetime as dt
import threading
from collections import OrderedDict
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..data.graph import RoadGraph
from ..models.features import weather_code
from ..utils.timeutil import parse_iso

#: city-wide traffic level of a request -> congestion shift of every edge's level (graph.py
#: edge_traffic); a missing or unknown level is the reference's default, "Low"
CONGESTION = {"Low": 0, "Medium": 1, "High": 2, "Jam": 3}


@dataclass(frozen=True)
class RouteContext:
    weather: int = 2          # features.py weather code (Sunny); 255 = unknown (zero one-hot)
    congestion: int = 0       # 0..3
    weekhour: int = 9         # Monday 00:00 = 0
    driver_age: float = 35.0  # the edge-cost model's fixed driver (a route does not depend on who drives)

    @property
    def key(self) -> int:
        return (self.weather & 0xFF) | ((self.congestion & 0xFF) << 8) | ((self.weekhour & 0xFFFF) << 16)

    @classmethod
    def from_request(cls, data: Any, now: Optional[dt.datetime] = None) -> "RouteContext":
        ctx = data.get("context") if isinstance(data, dict) else None
        if not isinstance(ctx, dict):
            ctx = {}
        w = ctx.get("weather", "Sunny")
        t = ctx.get("traffic", "Low")
        pickup = None
        pt = ctx.get("pickup_time")
        if isinstance(pt, str):
            try:
                pickup = parse_iso(pt)
            except (ValueError, TypeError):
                pickup = None
        if pickup is None:
            pickup = now or dt.datetime.now()
        return cls(weather=weather_code(w) if isinstance(w, str) else 255,
                   congestion=CONGESTION.get(t, 0) if isinstance(t, str) else 0,
                   weekhour=pickup.weekday() * 24 + pickup.hour)


def base_traffic(g: RoadGraph) -> np.ndarray:
    """Per-edge traffic level before the context's congestion shift (graph.py edge_traffic at
    congestion 1, i.e. shift 0)."""
    from .graph import edge_traffic
    return edge_traffic(g, congestion=1).astype(np.uint8)


def context_costs_cpu(g: RoadGraph, eta_model, ctx: RouteContext) -> np.ndarray:
    """Edge seconds of a context on the CPU (fp32 torch model; the GPU path computes them with the
    bf16 kernel in csrc/cch.hip)."""
    from .graph import edge_costs
    pickup = dt.datetime(2025, 8, 25) + dt.timedelta(hours=ctx.weekhour)
    weather = {0: "Cloudy", 1: "Stormy", 2: "Sunny", 3: "Windy"}.get(ctx.weather, "Unknown")
    return edge_costs(g, eta_model, None, weather=weather, congestion=ctx.congestion, pickup=pickup,
                      driver_age=ctx.driver_age)


class RoadRouter:
    """Legs and matrices under a routing context (GPU CCH, or the CPU reference)."""

    def __init__(self, g: RoadGraph, eta_model=None, device=None, capacity: Optional[int] = None,
                 max_path: int = 4096, threads: int = 0, cache_gb: Optional[float] = None):
        from ..ops import _ext
        self.g = g
        self.dev = torch.device(device) if device is not None else torch.device("cpu")
        self.max_path = int(max_path)
        if eta_model is None:
            from ..serve.eta_service import default_model
            eta_model = default_model(hidden=64, steps=100)
        self.eta_model = eta_model
        self._lock = threading.Lock()
        self._length = np.ascontiguousarray(g.length_m, dtype=np.float32)
        if self.dev.type == "cuda":
            C = _ext.native(required=True)
            from ..ops.eta_mlp import EtaMlpKernel
            self._kern = EtaMlpKernel(eta_model, self.dev)
            self.gpu = C.CchGpu(torch.from_numpy(np.ascontiguousarray(g.indptr, dtype=np.int32)),
                                torch.from_numpy(np.ascontiguousarray(g.indices, dtype=np.int32)),
                                torch.from_numpy(np.ascontiguousarray(g.lat, dtype=np.float64)),
                                torch.from_numpy(np.ascontiguousarray(g.lon, dtype=np.float64)),
                                torch.from_numpy(self._length),
                                torch.from_numpy(np.ascontiguousarray(g.road_class, dtype=np.uint8)),
                                torch.from_numpy(base_traffic(g)), self.dev.index or 0)
            self.gpu.set_eta(self._kern.packed.blob, self._kern.hidden, list(self._kern.packed.norm), -1)
            # LRU of customized contexts: a fixed count if given, else as many as fit the HBM budget
            # (ROUTEST_CCH_CACHE_GB, default 48 GB of the 288; csrc/cch.hip insert_cached)
            if capacity is not None:
                self.gpu.set_capacity(int(capacity))
            elif cache_gb is not None:
                self.gpu.set_cache_gb(float(cache_gb))
            self.cpu = None
        else:
            rt = _ext.runtime(required=True)
            self.gpu = None
            self.cpu = rt.CCH(np.ascontiguousarray(g.indptr, dtype=np.int32),
                              np.ascontiguousarray(g.indices, dtype=np.int32),
                              np.ascontiguousarray(g.lat, dtype=np.float64),
                              np.ascontiguousarray(g.lon, dtype=np.float64), threads)
            self._cpu_metrics: "OrderedDict[int, Any]" = OrderedDict()
            self._cpu_costs: Dict[int, np.ndarray] = {}
            self._cpu_pins: Dict[int, int] = {}
            self.capacity = 32 if capacity is None else int(capacity)
        self.last_metric: Dict[str, Any] = {}

    # ---- metrics ----
    def stats(self) -> Dict[str, Any]:
        return dict(self.gpu.stats() if self.gpu is not None else self.cpu.stats())

    def metric(self, ctx: RouteContext, pin: bool = False) -> int:
        """Make sure the context's metric is customized (and cached); returns its key.  ``pin``:
        also hold it outside the LRU until :meth:`unpin` (see :meth:`pinned`)."""
        if self.gpu is not None:
            self.last_metric = dict(self.gpu.metric_for(ctx.weather, ctx.congestion, ctx.weekhour,
                                                        ctx.driver_age, pin))
            return ctx.key
        with self._lock:
            if ctx.key in self._cpu_metrics:
                self._cpu_metrics.move_to_end(ctx.key)
                self.last_metric = {"key": ctx.key, "fresh": False}
            else:
                cost = context_costs_cpu(self.g, self.eta_model, ctx)
                m = self.cpu.customize(cost, self._length)
                self._cpu_metrics[ctx.key] = m
                self._cpu_costs[ctx.key] = cost
                self.last_metric = {"key": ctx.key, "fresh": True, "customize_ms": m.customize_ms}
            if pin:
                self._cpu_pins[ctx.key] = self._cpu_pins.get(ctx.key, 0) + 1
            self._evict_cpu()
            return ctx.key

    def _evict_cpu(self) -> None:
        """LRU beyond ``capacity``, never a pinned metric (caller holds the lock)."""
        while len(self._cpu_metrics) > self.capacity:
            k = next((k for k in self._cpu_metrics if k not in self._cpu_pins), None)
            if k is None:
                return
            del self._cpu_metrics[k]
            self._cpu_costs.pop(k, None)

    def prefetch(self, ctx: RouteContext, urgent: bool = False) -> bool:
        """Queue the context's customization on the GPU router's background builder (returns at
        once; False on the CPU router, which has none)."""
        if self.gpu is None:
            return False
        self.gpu.request_build(ctx.weather, ctx.congestion, ctx.weekhour, ctx.driver_age, urgent)
        return True

    def is_cached(self, ctx_or_key) -> bool:
        key = ctx_or_key.key if isinstance(ctx_or_key, RouteContext) else int(ctx_or_key)
        if self.gpu is not None:
            return bool(self.gpu.is_cached(key))
        with self._lock:
            return key in self._cpu_metrics

    def unpin(self, key: int) -> None:
        if self.gpu is not None:
            self.gpu.unpin(int(key))
            return
        with self._lock:
            n = self._cpu_pins.get(int(key), 0) - 1
            if n > 0:
                self._cpu_pins[int(key)] = n
            else:
                self._cpu_pins.pop(int(key), None)
                self._evict_cpu()

    @contextmanager
    def pinned(self, ctx_or_key):
        """``with router.pinned(ctx) as key:`` — the context's metric (customized if needed) stays
        usable for the whole block, however many other contexts are built meanwhile (a flush with
        more contexts than the cache holds, or concurrent callers on the same router)."""
        if isinstance(ctx_or_key, RouteContext):
            key = self.metric(ctx_or_key, pin=True)
            try:
                yield key
            finally:
                self.unpin(key)
        else:
            yield int(ctx_or_key)

    def metric_from_costs(self, key: int, cost: np.ndarray) -> int:
        """A metric from given edge costs (tests / benches), cached under ``key``."""
        cost = np.ascontiguousarray(cost, dtype=np.float32)
        if self.gpu is not None:
            self.last_metric = dict(self.gpu.metric_from_costs(int(key), torch.from_numpy(cost).to(self.dev)))
            return int(key)
        with self._lock:
            self._cpu_metrics[int(key)] = self.cpu.customize(cost, self._length)
            self._cpu_costs[int(key)] = cost
            return int(key)

    def costs(self, ctx_or_key) -> np.ndarray:
        key = ctx_or_key.key if isinstance(ctx_or_key, RouteContext) else int(ctx_or_key)
        if self.gpu is not None:
            return self.gpu.costs(key).cpu().numpy()
        return self._cpu_costs[key]

    # ---- queries ----
    def route(self, src: Sequence[int], dst: Sequence[int], ctx_or_key, want_path: bool = True):
        """(sec [Q], metres [Q], status [Q], paths: list of node-id arrays) — status 0 found,
        1 unreachable, 4 longer than max_path."""
        with self.pinned(ctx_or_key) as key:
            return self._route(src, dst, key, want_path)

    def _route(self, src, dst, key: int, want_path: bool):
        s = np.ascontiguousarray(src, dtype=np.int32)
        t = np.ascontiguousarray(dst, dtype=np.int32)
        if self.gpu is not None:
            sec, met, st, ln, path = self.gpu.route(key, torch.from_numpy(s).to(self.dev),
                                                    torch.from_numpy(t).to(self.dev), self.max_path, want_path)
            sec, met, st = sec.cpu().numpy(), met.cpu().numpy(), st.cpu().numpy()
            paths = None
            if want_path:
                ln, path = ln.cpu().numpy(), path.cpu().numpy()
                paths = [path[i, :ln[i]].copy() if st[i] == 0 else np.zeros(0, np.int32) for i in range(len(s))]
            return sec, met, st, paths
        sec, met, st, paths = self.cpu.query(self._cpu_metrics[key], s, t, want_path, self.max_path)
        return np.asarray(sec), np.asarray(met), np.asarray(st), paths

    def matrix(self, nodes: Sequence[int], ctx_or_key) -> Tuple[np.ndarray, np.ndarray]:
        """(seconds, metres) [n, n] between the given nodes (the diagonal is 0; unreachable = inf)."""
        with self.pinned(ctx_or_key) as key:
            return self._matrix(nodes, key)

    def _matrix(self, nodes, key: int):
        n = len(nodes)
        if self.gpu is not None:
            pts = torch.tensor(np.asarray(nodes, dtype=np.int32)[None, :], device=self.dev)
            npts = torch.tensor([n], dtype=torch.int32, device=self.dev)
            sec, met = self.gpu.matrix(key, pts, npts)
            return sec[0].cpu().numpy(), met[0].cpu().numpy()
        ii, jj = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
        nd = np.asarray(nodes, dtype=np.int32)
        sec, met, st, _ = self.cpu.query(self._cpu_metrics[key], nd[ii.ravel()], nd[jj.ravel()], False, self.max_path)
        sec = np.where(st == 0, sec, np.inf).reshape(n, n).astype(np.float32)
        met = np.where(st == 0, met, np.inf).reshape(n, n).astype(np.float32)
        np.fill_diagonal(sec, 0.0)
        np.fill_diagonal(met, 0.0)
        return sec, met

    def matrices(self, node_lists: Sequence[Sequence[int]], ctx_or_key) -> List[Tuple[np.ndarray, np.ndarray]]:
        """Many requests' matrices at once (ONE sweep + meet launch on the GPU)."""
        with self.pinned(ctx_or_key) as key:
            if self.gpu is None or not node_lists:
                return [self._matrix(n, key) for n in node_lists]
            return self._matrices(node_lists, key)

    def _matrices(self, node_lists, key: int):
        NM = max(len(n) for n in node_lists)
        pts = np.zeros((len(node_lists), NM), dtype=np.int32)
        npts = np.zeros(len(node_lists), dtype=np.int32)
        for r, n in enumerate(node_lists):
            pts[r, :len(n)] = n
            npts[r] = len(n)
        sec, met = self.gpu.matrix(key, torch.from_numpy(pts).to(self.dev), torch.from_numpy(npts).to(self.dev))
        sec, met = sec.cpu().numpy(), met.cpu().numpy()
        return [(sec[r, :len(n), :len(n)], met[r, :len(n), :len(n)]) for r, n in enumerate(node_lists)]
