"""Candidate-route scorer service (north star: "the candidate-route scorer ... hand-written CDNA4 HIP
kernels"; config 4's GCN, ``models/gcn.py``).

Given candidate routes for the same trip (GeoJSON LineString coordinates, or road-graph node ids),
every point is snapped to the road graph, and each route gets the GCN's delay-weighted length
``sum_i delay(v_i) * |v_i v_i+1|`` (lower is better).  Node delays depend only on the graph and
the model, so they are computed once (``gcn_agg_gemm`` x2 + ``gcn_spmm_score`` on the GPU, or the
fp32 torch reference on CPU) and cached; a scoring call is one ``route_score`` launch for all
candidates.  Exposed as ``POST /api/score_routes``.  The reference has no route scorer (its
"optimization" is the greedy R21 order plus remote ORS directions).
"""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ..data.graph import RoadGraph
from ..models.gcn import GcnScorer, score_routes_ref


class RouteScorer:
    blocking = True      # GPU synchronisation / graph snapping: handlers run it in the thread pool

    def __init__(self, g: RoadGraph, model: Optional[GcnScorer] = None, device: Optional[Any] = None,
                 kind: str = "edge"):
        self.g = g
        # "observed": trained on observed trips (predicted hidden seconds, models/gcn_observed.py);
        # "edge": the round-3 delay-weighted length (routing/alternatives.py picks accordingly)
        self.kind = kind
        self.model = model or GcnScorer(seed=0)
        self.device = torch.device(device) if device is not None else None
        self._hip = None
        self._delay_cpu: Optional[np.ndarray] = None
        self._lock = threading.Lock()
        if self.device is not None and self.device.type == "cuda":
            from ..models.gcn import GcnScorerHip
            self._hip = GcnScorerHip(self.model, g, self.device)
            self._hip.node_delays()
        self.engine = "gcn-hip" if self._hip is not None else "gcn-cpu"
        self.training: Optional[Dict[str, Any]] = None     # set when trained (models/gcn_train.py)

    @classmethod
    def synthetic(cls, num_nodes: int = 100_000, device=None) -> "RouteScorer":
        from ..data.graph import synth_road_graph
        return cls(synth_road_graph(num_nodes), device=device)

    # ------------------------------------------------------------------ inputs
    def to_nodes(self, route: Any) -> List[int]:
        """[[lon, lat], ...] | {"coordinates": [...]} | {"geometry": {"coordinates": [...]}} |
        {"nodes": [...]} -> snapped node ids (consecutive duplicates removed)."""
        if isinstance(route, dict):
            if "nodes" in route:
                nodes = [int(v) for v in route["nodes"]]
                if any(v < 0 or v >= self.g.num_nodes for v in nodes):
                    raise ValueError("node id out of range")
                return nodes
            route = route.get("coordinates") or (route.get("geometry") or {}).get("coordinates")
        if not isinstance(route, list) or not route:
            raise ValueError("route must be a non-empty coordinate list or {'nodes': [...]}")
        pts = np.asarray(route, dtype=np.float64)
        if pts.ndim != 2 or pts.shape[1] < 2 or not np.isfinite(pts[:, :2]).all():
            raise ValueError("coordinates must be [[lon, lat], ...]")
        ids = self.g.nearest_nodes(pts[:, 1], pts[:, 0])
        keep = np.ones(len(ids), dtype=bool)
        keep[1:] = ids[1:] != ids[:-1]
        return ids[keep].astype(int).tolist()

    def warm(self) -> None:
        """Startup warm-up: KD-tree for coordinate snapping + node delays (GPU: done in __init__)."""
        self.g.nearest_nodes([float(self.g.lat[0])], [float(self.g.lon[0])])
        self.node_delays()

    # ------------------------------------------------------------------ scoring
    def node_delays(self) -> np.ndarray:
        if self._hip is not None:
            return self._hip.delay[:self.g.num_nodes].cpu().numpy()
        with self._lock:
            if self._delay_cpu is None:
                with torch.no_grad():
                    A = GcnScorer.adjacency(self.g)
                    X = torch.from_numpy(self.g.features)
                    self._delay_cpu = self.model(A, X).float().numpy()
            return self._delay_cpu

    def score(self, routes: Sequence[Any]) -> Dict[str, Any]:
        node_lists = [self.to_nodes(r) for r in routes]
        if self._hip is not None:
            from ..models.gcn import routes_to_csr
            rptr, nodes = routes_to_csr(node_lists)
            d = self.device
            with self._lock:
                s = self._hip.score_routes(torch.from_numpy(rptr).to(d), torch.from_numpy(nodes).to(d))
                scores = s.double().cpu().numpy()
        else:
            scores = score_routes_ref(self.g, self.node_delays(), node_lists)
        best = int(np.argmin(scores)) if len(scores) else None
        out = {"scores": [float(x) for x in scores], "best": best, "engine": self.engine,
               "trained": self.training is not None, "nodes_per_route": [len(n) for n in node_lists]}
        if self.kind == "observed":
            # predicted hidden seconds per route (the part of its time the edge costs do not know)
            from .alternatives import candidate_scores
            out["kind"] = "observed"
            out["hidden_seconds"] = [float(x) for x in candidate_scores(self.g, self.node_delays(), node_lists,
                                                                         [0.0] * len(node_lists), "observed")]
        return out
