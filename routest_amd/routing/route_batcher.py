"""Cross-request micro-batching for ``/api/optimize_route``, ``/route`` and ``/api/request_route``.

The reference optimises one request at a time: an ORS matrix call, a Python greedy loop, then one
ORS directions call per trip (``RO/Flaskr/utils.py:85-193``, ``RO/Flaskr/routes.py:89-127``).
Here concurrent requests queue up and one worker per GPU flushes them together
(``batch_max`` requests or ``timeout_us`` after the first arrival):

1. every multi-stop request of the flush goes through ONE K5 launch (all haversine matrices) and
   ONE K6 launch (all greedy multi-trip constructions, a wavefront per request) —
   :func:`routing.batched.batched_trips`;
2. with the road-graph provider, every leg of every trip (and every point-to-point request) of
   the flush is snapped to graph nodes in one KD-tree query and searched by ONE batched A* launch
   (K9, :class:`routing.graph.BatchedAstar` on the worker's own GPU); duplicate legs are searched
   once;
3. the GeoJSON Features are assembled on the host by the same code as the per-request path
   (:func:`routing.optimizer.optimize_route` with the precomputed trips and a provider view that
   answers ``directions`` from the precomputed legs), so responses are identical to it.  The
   assembly runs back on the caller's thread (the event loop for HTTP requests): the worker thread
   only runs the short GPU phases, so it does not fight the request handlers for the GIL.

Several GPUs: one worker thread per device pulling from the same queue (no
collective); each worker's launches and host syncs touch only its own device, so flushes on
different GPUs overlap.  A leg the search does not find is an explicit error response.
"""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import queue
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ..utils.logging import get_logger
from ..utils.metrics import REGISTRY
from ..utils.queues import get_until
from .batched import batched_trips
from .greedy import InfeasibleStops
from .optimizer import optimize_route
from .providers import ProviderError

log = get_logger("route_batcher")


def _valid_points(r: Any) -> bool:
    return (isinstance(r, dict) and isinstance(r.get("destination_points"), list)
            and len(r["destination_points"]) > 0 and isinstance(r.get("source_point"), dict)
            and "lat" in r["source_point"] and "lon" in r["source_point"]
            and all(isinstance(p, dict) and "lat" in p and "lon" in p for p in r["destination_points"]))


class _LegView:
    """Provider view for the host-side assembly of one flush: ``directions`` answers from the legs
    searched in the batch's launches (keyed by the metric they were routed on) and the host copies
    of those metrics' edge costs taken while they were pinned; everything else delegates to the
    real provider.  Nothing here customizes or looks up a GPU metric, so assembly cannot stall on
    (or fail by) a context evicted since the plan."""

    def __init__(self, base, legs: Dict[tuple, tuple], device=None,
                 host_costs: Optional[Dict[int, np.ndarray]] = None):
        self.base = base
        self.legs = legs
        self.name = base.name
        self.uses_context = getattr(base, "uses_context", False)
        self.device = device
        self.host_costs = host_costs or {}

    def matrix(self, points, profile, **kw):
        return self.base.matrix(points, profile, **kw)

    def _key(self, ctx) -> Optional[int]:
        if not hasattr(self.base, "metric_key"):
            return None
        if self.uses_context:
            from .cch import RouteContext
            return (ctx or RouteContext()).key
        return self.base.metric_key(None, self.device)

    def directions(self, coords, profile, ctx=None):
        nodes, pairs = self.base.leg_pairs(coords)
        key = self._key(ctx)
        # keyed by (metric, s, t); plain (s, t) keys (routing/alternatives.py) hold fixed-metric legs
        legs = [self.legs[(key, p[0], p[1])] if (key, p[0], p[1]) in self.legs else self.legs[p] for p in pairs]
        if key is None:
            return self.base.feature_from_legs(coords, nodes, legs, profile)
        return self.base.feature_from_legs(coords, nodes, legs, profile, key=key, device=self.device,
                                           ecost=self.host_costs.get(key))


class RouteBatcher:
    def __init__(self, provider, engine: str = "backend:mi355x", devices: Sequence[Any] = (None,),
                 batch_max: int = 1024, timeout_us: int = 500, astar_slots: int = 8192):
        self.provider = provider
        self.engine = engine
        self.devices = list(devices) or [None]
        self.batch_max = batch_max
        self.timeout_s = timeout_us / 1e6
        self.astar_slots = astar_slots
        self._astar: Dict[Any, Any] = {}
        self._astar_lock = threading.Lock()
        self._streams: Dict[str, Any] = {}
        self._stream_lock = threading.Lock()
        self.q: "queue.SimpleQueue[Optional[tuple]]" = queue.SimpleQueue()
        self.flushes = [0] * len(self.devices)
        self.threads = [threading.Thread(target=self._worker, args=(d, i), name=f"route-batch-{i}",
                                         daemon=True) for i, d in enumerate(self.devices)]
        for t in self.threads:
            t.start()

    # ------------------------------------------------------------------ batch function
    def _stream_for(self, device):
        import torch
        with self._stream_lock:
            key = str(device)
            st = self._streams.get(key)
            if st is None:
                with torch.cuda.device(device):
                    st = self._streams[key] = torch.cuda.Stream(device)
            return st

    def _astar_for(self, device):
        """The device's A* workspace and the lock that serialises its searches (two workers on one
        device would otherwise run on the same per-slot state rows at once)."""
        from .graph import BatchedAstar
        key = str(device)
        with self._astar_lock:
            a = self._astar.get(key)
            if a is None:
                a = (BatchedAstar(self.provider.g, self.provider.cost, device, slots=self.astar_slots),
                     threading.Lock())
                self._astar[key] = a
            return a

    def _contexts(self, payloads: List[Any]) -> List[Any]:
        """Each request's routing context, resolved ONCE per flush (one ``now`` for requests
        without a pickup time); carried to assembly with the plan."""
        if not getattr(self.provider, "uses_context", False):
            return [None] * len(payloads)
        import datetime as dt
        from .cch import RouteContext
        now = dt.datetime.now()
        return [RouteContext.from_request(p, now=now) if _valid_points(p) else None for p in payloads]

    def _graph_plan(self, payloads: List[Any], device, ctxs: List[Any]) -> tuple:
        """Road-graph flush: per routing context, ONE many-to-many launch for every multi-stop
        request's road-metre matrix, ONE greedy launch (K6) over those matrices, then every trip leg
        (and point-to-point request) in ONE leg launch.  Each context group runs start to finish
        under a pin of its metric, and its edge costs are copied to the host then, so a flush with
        more contexts than the metric cache holds never loses one in between.  Returns (trips by
        request, legs dict, host edge costs by metric key)."""
        prov = self.provider
        trips: Dict[int, Any] = {}
        legs: Dict[tuple, tuple] = {}
        host_costs: Dict[int, np.ndarray] = {}
        valid = [k for k, r in enumerate(payloads) if _valid_points(r)]
        if not valid:
            return trips, legs, host_costs
        groups: Dict[Any, List[int]] = {}
        first: Dict[Any, Any] = {}
        for k in valid:
            gk = ctxs[k].key if ctxs[k] is not None else None
            groups.setdefault(gk, []).append(k)
            first.setdefault(gk, ctxs[k])
        for gk, ks in groups.items():
            with prov.pinned_metric(first[gk], device) as key:
                self._plan_group(payloads, ks, key, device, trips, legs)
                if getattr(prov, "_steps", None) is not None:
                    host_costs[key] = prov.edge_seconds(key, device)
        return trips, legs, host_costs

    def _plan_group(self, payloads, ks, key, device, trips, legs) -> None:
        prov = self.provider
        pts = {k: [payloads[k]["source_point"]] + list(payloads[k]["destination_points"]) for k in ks}
        flat = np.array([[p["lon"], p["lat"]] for k in ks for p in pts[k]], dtype=np.float64)
        nodes_all = prov.g.nearest_nodes(flat[:, 1], flat[:, 0])
        nodes: Dict[int, np.ndarray] = {}
        o = 0
        for k in ks:
            nodes[k] = nodes_all[o:o + len(pts[k])]
            o += len(pts[k])
        multi = [k for k in ks if len(pts[k]) > 2]
        if multi:
            mats = prov.router(device).matrices([nodes[k].tolist() for k in multi], key)
            nm = max(len(pts[k]) for k in multi)
            D = np.zeros((len(multi), nm, nm))
            for i, (k, (_, met)) in enumerate(zip(multi, mats)):
                n = len(pts[k])
                D[i, :n, :n] = met
            res = batched_trips([payloads[k] for k in multi], device=device, D=D)
            trips.update(zip(multi, res))
        pairs = set()
        for k in ks:
            if len(pts[k]) == 2:
                seqs = [[0, 1]]
            elif isinstance(trips.get(k), list):
                seqs = trips[k]
            else:
                continue
            for seq in seqs:
                n = nodes[k][seq]
                pairs.update((int(n[i]), int(n[i + 1])) for i in range(len(n) - 1))
        pairs = sorted(pairs)
        if pairs:
            res, _ = prov.legs(pairs, key=key, device=device)
            legs.update({(key, s, t): r for (s, t), r in zip(pairs, res)})

    def _graph_legs(self, payloads: List[Any], trips: Dict[int, Any], device) -> Dict[tuple, tuple]:
        """Legacy A* engine: every leg of the flush -> {(key, s, t): (seconds, node path)} from ONE
        batched search on the provider's fixed costs."""
        prov = self.provider
        coord_lists: List[List[List[float]]] = []
        for k, r in enumerate(payloads):
            if not _valid_points(r):
                continue
            pts = [r["source_point"]] + list(r["destination_points"])
            if len(pts) == 2:
                coord_lists.append([[pts[0]["lon"], pts[0]["lat"]], [pts[1]["lon"], pts[1]["lat"]]])
            elif isinstance(trips.get(k), list):
                for trip in trips[k]:
                    coord_lists.append([[pts[i]["lon"], pts[i]["lat"]] for i in trip])
        if not coord_lists:
            return {}
        flat = np.array([c for cl in coord_lists for c in cl], dtype=np.float64)
        nodes = prov.g.nearest_nodes(flat[:, 1], flat[:, 0])
        pairs = set()
        o = 0
        for cl in coord_lists:
            n = nodes[o:o + len(cl)]
            pairs.update((int(n[i]), int(n[i + 1])) for i in range(len(cl) - 1))
            o += len(cl)
        pairs = sorted(pairs)
        if device is not None and getattr(device, "type", str(device)).startswith("cuda"):
            astar, lock = self._astar_for(device)
            with lock:
                res = astar.paths([p[0] for p in pairs], [p[1] for p in pairs])
        else:
            res = prov._shortest_astar(pairs) if hasattr(prov, "_shortest_astar") else prov._shortest(pairs)
        key = prov.FIXED_KEY if hasattr(prov, "FIXED_KEY") else None
        return {(key, s, t): r for (s, t), r in zip(pairs, res)}

    def plan_batch(self, payloads: Sequence[Any], device=None) -> List[tuple]:
        """The GPU phases of a flush: per request ``(trips or InfeasibleStops or None, view, ctx)``."""
        payloads = list(payloads)
        name = getattr(self.provider, "name", "")
        trips: Dict[int, Any] = {}
        view = self.provider
        if name == "graph" and getattr(self.provider, "engine", "astar") != "astar":
            ctxs = self._contexts(payloads)
            try:
                trips, legs, hc = self._graph_plan(payloads, device, ctxs)
            except ProviderError as e:
                return [(e, None, None) for _ in payloads]
            view = _LegView(self.provider, legs, device, hc)
            return [(trips.get(k), view, ctxs[k]) for k in range(len(payloads))]
        multi = [k for k, r in enumerate(payloads) if _valid_points(r) and len(r["destination_points"]) > 1]
        if multi and name in ("haversine", "graph"):
            res = batched_trips([payloads[k] for k in multi], circuity=self.provider.circuity,
                                device=device)
            trips = dict(zip(multi, res))
        if name == "graph":
            try:
                view = _LegView(self.provider, self._graph_legs(payloads, trips, device), device)
            except ProviderError as e:
                return [(e, None, None) for _ in payloads]
        return [(trips.get(k), view, None) for k in range(len(payloads))]

    def assemble(self, payload: Any, plan: tuple) -> Dict[str, Any]:
        """Host side of one request: GeoJSON Feature (or error) from its planned trips/legs, under
        the routing context it was planned with."""
        t, view, ctx = plan
        if isinstance(t, (InfeasibleStops, ProviderError)):
            return {"error": str(t)}
        return optimize_route(payload, view, self.engine, trips=t, ctx=ctx)

    def run_batch(self, payloads: Sequence[Any], device=None) -> List[Dict[str, Any]]:
        """Optimise a list of request payloads together (plan + assembly; also callable directly,
        e.g. ``/api/optimize_routes_batch``)."""
        payloads = list(payloads)
        return [self.assemble(p, pl) for p, pl in zip(payloads, self.plan_batch(payloads, device))]

    # ------------------------------------------------------------------ queue side
    def submit_nowait(self, payload: Any, loop: Optional[asyncio.AbstractEventLoop] = None):
        fut = loop.create_future() if loop is not None else cf.Future()
        self.q.put((payload, fut, loop, time.perf_counter()))
        return fut

    async def submit(self, payload: Any) -> Dict[str, Any]:
        plan = await self.submit_nowait(payload, asyncio.get_running_loop())
        return self.assemble(payload, plan)

    def optimize_sync(self, payload: Any, timeout: float = 60.0) -> Dict[str, Any]:
        return self.assemble(payload, self.submit_nowait(payload).result(timeout))

    @staticmethod
    def _resolve(fut, loop, value=None, exc: Optional[BaseException] = None) -> None:
        def _set():
            if fut.done():
                return
            if exc is not None:
                fut.set_exception(exc)
            else:
                fut.set_result(value)
        if loop is not None:
            try:
                loop.call_soon_threadsafe(_set)
            except RuntimeError:
                pass
        else:
            _set()

    def _collect(self, first) -> list:
        batch = [first]
        deadline = first[3] + self.timeout_s
        while len(batch) < self.batch_max:
            try:
                it = get_until(self.q, deadline)         # (not q.get(timeout=...): see utils/queues.py)
            except queue.Empty:
                break
            batch.append(it)
            if it is None:
                break
        return batch

    def _worker(self, device, idx: int) -> None:
        import torch
        # the flushes run on a NON-blocking stream, so their launches and copies never queue behind
        # the legacy null stream's implicit wait for every blocking stream on the device (a kernel
        # hung on one — the watchdog rehearsal's fault streams are blocking — stalled every request
        # relayed here for the hang's whole duration).  ONE stream per device, shared by the
        # device's workers: their searches share per-device workspaces, and the lock around them is
        # released when the host calls return, so the GPU work must stay ordered on one stream
        stream = None
        if device is not None and getattr(device, "type", "") == "cuda":
            stream = self._stream_for(device)
        while True:
            first = self.q.get()
            if first is None:
                self.q.put(None)
                return
            batch = self._collect(first)
            stop = batch[-1] is None
            if stop:
                batch.pop()
            t0 = time.perf_counter()
            try:
                if stream is not None:
                    with torch.cuda.device(device), torch.cuda.stream(stream):
                        res = self.plan_batch([b[0] for b in batch], device)
                else:
                    res = self.plan_batch([b[0] for b in batch], device)
                for (_, fut, loop, _), r in zip(batch, res):
                    self._resolve(fut, loop, r)
            except BaseException as e:  # noqa: BLE001 - fail the flush's requests, keep serving
                log.error("route flush of %d failed on %s: %r", len(batch), device, e)
                for _, fut, loop, _ in batch:
                    self._resolve(fut, loop, exc=e)
            self.flushes[idx] += 1
            REGISTRY.route_batch.observe(len(batch))
            REGISTRY.route_flush_time.observe(time.perf_counter() - t0)
            if stop:
                self.q.put(None)
                return

    def close(self) -> None:
        self.q.put(None)
        for t in self.threads:
            t.join(timeout=10)
