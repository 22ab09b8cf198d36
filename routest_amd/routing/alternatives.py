"""Candidate routes ranked by the trained GCN scorer (``"alternatives": k`` on /api/optimize_route).

The reference routes every trip along the single ORS answer (``RO/Flaskr/utils.py:147-165``).  With
the road-graph provider and ``alternatives = k`` (2..8) in the request, every leg of the optimized
trips gets k candidates — the shortest path under the learned edge times plus k - 1 via-node detours
(nodes w with d(s, w) + d(w, t) <= 1.35 d(s, t), seeded per leg so answers are reproducible) — all
searched in ONE batched A* launch, scored by the GCN candidate-route scorer (trained on the same
edge times, ``models/gcn_train.py``), and the best-scored candidate becomes the leg.  The response
is the usual Feature plus ``properties.alternatives``: per leg the candidates' scores, their A*
seconds and the chosen index.  (Requests carrying ``alternatives`` are answered by the Python app;
the native front end relays them.)
"""
from __future__ import annotations

import zlib
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .providers import ProviderError, haversine_m

MAX_K = 8


def via_nodes(g, s: int, t: int, n: int, stretch: float = 1.35, pool: int = 2048) -> List[int]:
    rng = np.random.default_rng(zlib.crc32(f"{s}:{t}".encode()))
    d_st = float(haversine_m(g.lat[s], g.lon[s], g.lat[t], g.lon[t]))
    if d_st < 1.0 or n <= 0:
        return []
    # sample around the s-t segment: the ellipse's bounding box, widened by the stretch
    lat0, lat1 = sorted((g.lat[s], g.lat[t]))
    lon0, lon1 = sorted((g.lon[s], g.lon[t]))
    pad = 0.5 * (stretch - 1.0) * (abs(lat1 - lat0) + abs(lon1 - lon0)) + 1e-3
    near = np.nonzero((g.lat >= lat0 - pad) & (g.lat <= lat1 + pad) & (g.lon >= lon0 - pad) & (g.lon <= lon1 + pad))[0]
    if len(near) == 0:
        return []
    cand = near[rng.integers(0, len(near), min(pool, 4 * len(near)))]
    det = (haversine_m(g.lat[s], g.lon[s], g.lat[cand], g.lon[cand]) +
           haversine_m(g.lat[cand], g.lon[cand], g.lat[t], g.lon[t]))
    ok = np.unique(cand[(det <= stretch * d_st) & (det >= 1.03 * d_st)])
    if len(ok) == 0:
        return []
    return [int(w) for w in rng.choice(ok, min(n, len(ok)), replace=False)]


class AlternativeLegs:
    """``choose(pairs, k)`` -> ({(s, t): (seconds, path)} of the chosen candidates, per-pair info)."""

    def __init__(self, g, scorer, search):
        self.g = g
        self.scorer = scorer
        self.search = search            # (src list, dst list) -> [(seconds, path)]

    def choose(self, pairs: Sequence[Tuple[int, int]], k: int):
        k = max(1, min(int(k), MAX_K))
        src, dst, plan = [], [], []
        for s, t in pairs:
            vias = via_nodes(self.g, s, t, k - 1)
            plan.append(vias)
            src.append(s); dst.append(t)
            for w in vias:
                src += [s, w]; dst += [w, t]
        res = self.search(src, dst)
        chosen: Dict[Tuple[int, int], Tuple[float, List[int]]] = {}
        info: Dict[Tuple[int, int], Dict[str, Any]] = {}
        cands_all, i = [], 0
        for (s, t), vias in zip(pairs, plan):
            cands = [(res[i][0], list(res[i][1]))]
            i += 1
            for _ in vias:
                (c1, p1), (c2, p2) = res[i], res[i + 1]
                i += 2
                if p1 and p2:
                    cands.append((float(c1) + float(c2), list(p1) + list(p2[1:])))
            cands = [c for c in cands if c[1]]
            cands_all.append(cands)
        flat = [c[1] for cands in cands_all for c in cands]
        scores = self.scorer.score([{"nodes": p} for p in flat])["scores"] if flat else []
        o = 0
        for (s, t), cands in zip(pairs, cands_all):
            sc = scores[o:o + len(cands)]
            o += len(cands)
            if not cands:
                chosen[(s, t)] = (float("nan"), [])
                info[(s, t)] = {"candidates": 0}
                continue
            j = int(np.argmin(sc))
            chosen[(s, t)] = cands[j]
            info[(s, t)] = {"candidates": len(cands), "chosen": j, "scores": [float(x) for x in sc],
                            "seconds": [float(c[0]) for c in cands]}
        return chosen, info


def optimize_with_alternatives(payload: Dict[str, Any], provider, scorer, search, engine: str,
                               k: int) -> Dict[str, Any]:
    """optimize_route with every leg chosen among k scored candidates (graph provider only)."""
    from .optimizer import optimize_route
    from .route_batcher import _LegView, _valid_points
    from .batched import batched_trips
    if getattr(provider, "name", "") != "graph":
        return {"error": "alternatives need the road-graph provider (ROUTEST_PROVIDER=graph)"}
    if not _valid_points(payload):
        return optimize_route(payload, provider, engine)
    pts = [payload["source_point"]] + list(payload["destination_points"])
    trips = None
    if len(pts) > 2:
        t = batched_trips([payload], circuity=provider.circuity)[0]
        if not isinstance(t, list):
            return {"error": str(t)}
        trips = t
    calls = [pts] if trips is None else [[pts[i] for i in tr] for tr in trips]
    pairs, seen = [], set()
    for c in calls:
        nodes = provider.g.nearest_nodes([p["lat"] for p in c], [p["lon"] for p in c])
        for a, b in zip(nodes[:-1], nodes[1:]):
            key = (int(a), int(b))
            if key not in seen:
                seen.add(key)
                pairs.append(key)
    chosen, info = AlternativeLegs(provider.g, scorer, search).choose(pairs, k)
    try:
        res = optimize_route(payload, _LegView(provider, chosen), engine, trips=trips)
    except ProviderError as e:
        return {"error": str(e)}
    if "error" not in res:
        res.setdefault("properties", {})["alternatives"] = {
            "k": max(1, min(int(k), MAX_K)), "scorer": getattr(scorer, "engine", "gcn"),
            "legs": [dict(from_node=s, to_node=t, **info[(s, t)]) for s, t in pairs]}
    return res
