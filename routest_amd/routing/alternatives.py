"""Candidate routes ranked by the trained GCN scorer (``"alternatives": k`` on /api/optimize_route).

The reference routes every trip along the single ORS answer (``RO/Flaskr/utils.py:147-165``).  With
the road-graph provider and ``alternatives = k`` (2..8) in the request, the trips are planned as
usual (road-metre matrix + R21 greedy, under the request's routing context), and every leg of them
gets up to k candidates — the time-shortest path under the context's edge costs plus k - 1 via-node
detours (csrc/runtime/alternatives.h via_nodes: nodes w with d(s, w) + d(w, t) within
[1.03, 1.35] x d(s, t), in a per-leg hash order, so answers are reproducible) — all routed in ONE
batched CCH call.  The GCN scorer picks one per leg:

* ``kind == "observed"`` (default, models/gcn_observed.py): trained on observed trips, it predicts
  the hidden seconds the edge costs do not know; the pick minimises edge-cost seconds + predicted
  hidden seconds;
* ``kind == "edge"`` (round 3, models/gcn_train.py): the pick minimises the delay-weighted length.

Both scores come from the same C++ helper the native route service uses (``_rt.alt_scores``), so
the native front end answers these requests byte-identically (csrc/route_service.hip).  The
response is the usual Feature plus ``properties.alternatives``: per leg the candidates' scores,
their edge-cost seconds and the chosen index.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .providers import ProviderError, haversine_m

MAX_K = 8
KINDS = {"observed": 0, "edge": 1}


def _rt():
    from ..ops import _ext
    return _ext.runtime(required=False)


def _mix64(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def via_nodes(g, s: int, t: int, n: int, stretch: float = 1.35) -> List[int]:
    """Via candidates of leg s -> t (see module docstring); the C++ helper when built."""
    rt = _rt()
    if rt is not None and hasattr(rt, "via_nodes"):
        return list(rt.via_nodes(g.lat, g.lon, int(s), int(t), int(n), float(stretch)))
    d_st = float(haversine_m(g.lat[s], g.lon[s], g.lat[t], g.lon[t]))
    if not d_st >= 1.0 or n <= 0:
        return []
    lat0, lat1 = sorted((g.lat[s], g.lat[t]))
    lon0, lon1 = sorted((g.lon[s], g.lon[t]))
    pad = 0.5 * (stretch - 1.0) * ((lat1 - lat0) + (lon1 - lon0)) + 1e-3
    near = np.nonzero((g.lat >= lat0 - pad) & (g.lat <= lat1 + pad) & (g.lon >= lon0 - pad) & (g.lon <= lon1 + pad))[0]
    det = (haversine_m(g.lat[s], g.lon[s], g.lat[near], g.lon[near]) +
           haversine_m(g.lat[near], g.lon[near], g.lat[t], g.lon[t]))
    ok = near[(det <= stretch * d_st) & (det >= 1.03 * d_st)].astype(np.uint64)
    with np.errstate(over="ignore"):
        key = _mix64(np.array([(int(s) << 32) | int(t)], dtype=np.uint64))[0]
        h = _mix64(key ^ ok)
    order = np.lexsort((ok, h))[:n]
    return [int(w) for w in ok[order]]


def candidate_scores(g, delay: np.ndarray, paths: Sequence[Sequence[int]], seconds: Sequence[float],
                     kind: str) -> List[float]:
    rt = _rt()
    k = KINDS[kind]
    if rt is not None and hasattr(rt, "alt_scores"):
        return list(rt.alt_scores(g.lat, g.lon, np.ascontiguousarray(delay, dtype=np.float64),
                                  [np.asarray(p, dtype=np.int32) for p in paths], [float(x) for x in seconds], k))
    lat = g.lat.astype(np.float32).astype(np.float64)
    lon = g.lon.astype(np.float32).astype(np.float64)
    out = []
    for p, sec in zip(paths, seconds):
        acc = 0.0
        for a, b in zip(p[:-1], p[1:]):
            d = float(haversine_m(lat[a], lon[a], lat[b], lon[b]))
            acc += (delay[a] - 0.5) * d / 20.0 if k == 0 else delay[a] * d
        out.append(float(sec) + acc if k == 0 else acc)
    return out


def _argmin(v: Sequence[float]) -> int:
    a = np.asarray(v, dtype=np.float64)
    return int(np.argmin(np.where(np.isfinite(a), a, np.inf)))


class AlternativeLegs:
    """``choose(pairs, k)`` -> ({(s, t): (seconds, metres, path)} of the chosen candidates, per-pair
    info).  ``search(pairs)`` -> [(seconds, metres, path)] per (s, t) (nan, nan, [] when none)."""

    def __init__(self, g, scorer, search):
        self.g = g
        self.scorer = scorer
        self.search = search

    def choose(self, pairs: Sequence[Tuple[int, int]], k: int):
        k = max(1, min(int(k), MAX_K))
        q: List[Tuple[int, int]] = []
        plan = []
        for s, t in pairs:
            vias = via_nodes(self.g, s, t, k - 1)
            plan.append(vias)
            q.append((s, t))
            for w in vias:
                q += [(s, w), (w, t)]
        res = self.search(q) if q else []
        delay = self.scorer.node_delays()
        kind = getattr(self.scorer, "kind", "edge")
        chosen: Dict[Tuple[int, int], Tuple[float, float, List[int]]] = {}
        info: Dict[Tuple[int, int], Dict[str, Any]] = {}
        i = 0
        for (s, t), vias in zip(pairs, plan):
            cands = []
            sec, met, p = res[i]
            i += 1
            if p:
                cands.append((float(sec), float(met), list(p)))
            for _ in vias:
                (c1, m1, p1), (c2, m2, p2) = res[i], res[i + 1]
                i += 2
                if p1 and p2:
                    cands.append((float(c1) + float(c2), float(m1) + float(m2), list(p1) + list(p2[1:])))
            if not cands:
                chosen[(s, t)] = (float("nan"), float("nan"), [])
                info[(s, t)] = {"candidates": 0}
                continue
            sc = candidate_scores(self.g, delay, [c[2] for c in cands], [c[0] for c in cands], kind)
            j = _argmin(sc)
            chosen[(s, t)] = cands[j]
            info[(s, t)] = {"candidates": len(cands), "chosen": j, "scores": [float(x) for x in sc],
                            "seconds": [float(c[0]) for c in cands]}
        return chosen, info


def optimize_with_alternatives(payload: Dict[str, Any], provider, scorer, search=None, engine: str = "backend:mi355x",
                               k: int = 4) -> Dict[str, Any]:
    """optimize_route with every leg chosen among k scored candidates (graph provider only)."""
    from .greedy import InfeasibleStops, greedy_trips
    from .optimizer import _float, _vehicle_type, optimize_route
    from .providers import profile_for
    from .route_batcher import _LegView, _valid_points
    if getattr(provider, "name", "") != "graph":
        return {"error": "alternatives need the road-graph provider (ROUTEST_PROVIDER=graph)"}
    if not _valid_points(payload):
        return optimize_route(payload, provider, engine)
    ctx = None
    if getattr(provider, "uses_context", False):
        from .cch import RouteContext
        ctx = RouteContext.from_request(payload)      # resolved once: planning and assembly agree
    if hasattr(provider, "pinned_metric"):
        with provider.pinned_metric(ctx) as key:      # the metric stays usable for the whole request
            return _alternatives_on(payload, provider, scorer, search, engine, k, ctx, key)
    return _alternatives_on(payload, provider, scorer, search, engine, k, ctx, None)


def _alternatives_on(payload, provider, scorer, search, engine, k, ctx, key):
    from .greedy import InfeasibleStops, greedy_trips
    from .optimizer import _float, _vehicle_type, optimize_route
    from .providers import profile_for
    from .route_batcher import _LegView
    driver = payload.get("driver_details") or {}
    profile = profile_for(_vehicle_type(driver))
    pts = [payload["source_point"]] + list(payload["destination_points"])
    trips = None
    if len(pts) > 2:
        D = provider.matrix(pts, profile, **({"ctx": ctx} if ctx is not None else {}))
        cap = _float(driver.get("vehicle_capacity", 9e12), 9e12)
        max_dist = _float(driver.get("maximum_distance", 9e12), 9e12)
        demand = [0.0] + [_float(p.get("payload", 0), 0.0) for p in payload["destination_points"]]
        try:
            trips = greedy_trips(np.asarray(D, dtype=np.float64).tolist(), demand, cap, max_dist)
        except InfeasibleStops as e:
            return {"error": str(e)}
    calls = [pts] if trips is None else [[pts[i] for i in tr] for tr in trips]
    pairs, seen = [], set()
    for c in calls:
        nodes = provider.g.nearest_nodes([p["lat"] for p in c], [p["lon"] for p in c])
        for a, b in zip(nodes[:-1], nodes[1:]):
            pk = (int(a), int(b))
            if pk not in seen:
                seen.add(pk)
                pairs.append(pk)
    if hasattr(provider, "legs"):
        def run(q):
            return provider.legs(q, key=key)[0] if q else []
    else:                                   # legacy (seconds, path) search
        def run(q):
            out = search([a for a, _ in q], [b for _, b in q])
            return [(c, float("nan"), p) for c, p in out]
    chosen, info = AlternativeLegs(provider.g, scorer, run).choose(pairs, k)
    hc = ({key: provider.edge_seconds(key)} if key is not None and getattr(provider, "_steps", None) is not None
          else None)
    view = _LegView(provider, {(key, s, t): v for (s, t), v in chosen.items()} if key is not None else chosen,
                    host_costs=hc)
    try:
        res = optimize_route(payload, view, engine, trips=trips, ctx=ctx)
    except ProviderError as e:
        return {"error": str(e)}
    if "error" not in res:
        res.setdefault("properties", {})["alternatives"] = {
            "k": max(1, min(int(k), MAX_K)), "scorer": getattr(scorer, "engine", "gcn"),
            "legs": [dict(from_node=s, to_node=t, **info[(s, t)]) for s, t in pairs]}
    return res
