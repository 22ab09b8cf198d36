"""The GCN candidate-route scorer trained on OBSERVED trips (verdict r3 item 5).

The round-3 scorer regressed node delays onto the same edge costs the router already minimises, so
its ranking could at best reproduce the router's (``gcn_train.py`` node_delay_targets).  Here it
learns what the edge-cost model does not know, from trip observations:

* **World** (:class:`TripWorld`, synthetic and seeded — there is no real trip log offline): the true
  time of a route is the edge-cost model's seconds (what the CCH router minimises) plus *hidden*
  delays the edge-cost MLP never sees — incident / congestion hot spots (Gaussian bumps of extra
  pace, s/m, over a few km²) and signalised intersections (degree >= 4 with mixed road classes) —
  plus 3 % observation noise.  Hidden pace h(v) applies to the segment leaving node v:
  ``true(P) = sum_e cost(e) + sum_i h(v_i) |v_i v_{i+1}|``.
* **Observations**: trips between random node pairs, driven along the time-shortest path or (half
  of them) through a random via node, each observed once with its total time — the shape of what
  ``/api/update_tracker`` receives (RO/Flaskr/routes.py tracker: route + duration per trip).
* **Model**: the GCN's node output is a delay factor ``delay(v) = 0.5 + softplus(.)``; the route's
  predicted hidden seconds are ``sum_i (delay(v_i) - 0.5) |v_i v_{i+1}| / V_REF``.  The loss is the
  mean squared error between that and each observed trip's residual (observed - edge-cost seconds):
  a path-aggregated regression, no per-node labels.  On a GPU the backward is the HIP trainer of
  ``gcn_train.py`` (:class:`GcnTrainerHip`): the path loss' gradient w.r.t. every node's delay is
  scattered on the device and handed to ``gcn_train_bwd`` as the equivalent per-node target
  (``t = delay - N/2 * dL/ddelay``, the kernel's MSE gradient is ``2 (delay - t) / N``), so the
  MFMA weight-gradient GEMM and the fused AdamW are reused unchanged; data parallel by node rows
  exactly as there (every rank sees all trips, backward over its rows, one all-reduce).
* **Choice** (:func:`choose`): among a leg's candidates (time-shortest path + via-node detours), the
  one with the least ``edge-cost seconds + predicted hidden seconds``.

:func:`evaluate` compares, on held-out trips, the true time of the route picked by: the router alone
(time-shortest under the edge costs), the random-init scorer, the round-3 edge-cost scorer
(argmin of its delay-weighted length), the observed-trip scorer, and an oracle.
"""
from __future__ import annotations

import math
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..data.graph import RoadGraph
from .gcn import GcnScorer
from .gcn_train import V_REF, GcnTrainerHip, candidate_routes, via_alternatives

Search = Callable[[Sequence[int], Sequence[int]], List[Tuple[float, List[int]]]]


def _km_xy(g: RoadGraph) -> Tuple[np.ndarray, np.ndarray]:
    lat0, lon0 = float(g.lat.mean()), float(g.lon.mean())
    x = (g.lon - lon0) * 111.32 * math.cos(math.radians(lat0))
    y = (g.lat - lat0) * 110.57
    return x, y


def segment_lengths(g: RoadGraph, nodes: np.ndarray, rptr: np.ndarray) -> np.ndarray:
    """Metres from each path node to the next one of the same path (0 at each path's end), on the
    float32 coordinates the scorer kernels use (models/gcn.py score_routes_ref)."""
    from ..routing.providers import haversine_m
    lat = g.lat.astype(np.float32).astype(np.float64)
    lon = g.lon.astype(np.float32).astype(np.float64)
    d = np.zeros(len(nodes), dtype=np.float64)
    if len(nodes) > 1:
        d[:-1] = haversine_m(lat[nodes[:-1]], lon[nodes[:-1]], lat[nodes[1:]], lon[nodes[1:]])
    ends = rptr[1:] - 1
    d[ends[ends >= 0]] = 0.0
    return d


def paths_csr(paths: Sequence[Sequence[int]]) -> Tuple[np.ndarray, np.ndarray]:
    rptr = np.zeros(len(paths) + 1, dtype=np.int64)
    rptr[1:] = np.cumsum([len(p) for p in paths])
    nodes = np.concatenate([np.asarray(p, dtype=np.int64) for p in paths]) if paths else np.zeros(0, np.int64)
    return rptr, nodes


class TripWorld:
    """Synthetic ground truth: edge-cost seconds + hidden node pace (see module docstring)."""

    def __init__(self, g: RoadGraph, cost: np.ndarray, seed: int = 0, hot_per_100km2: float = 6.0,
                 hot_amp: Tuple[float, float] = (0.05, 0.12), hot_sigma_km: Tuple[float, float] = (0.6, 1.4),
                 signal_pace: float = 0.04, noise: float = 0.03):
        self.g = g
        self.cost = np.asarray(cost, dtype=np.float64)
        self.noise = noise
        rng = np.random.default_rng(seed)
        x, y = _km_xy(g)
        area = max(1.0, float((x.max() - x.min()) * (y.max() - y.min())))
        n_hot = max(3, int(round(area / 100.0 * hot_per_100km2)))
        cx = rng.uniform(x.min(), x.max(), n_hot)
        cy = rng.uniform(y.min(), y.max(), n_hot)
        amp = rng.uniform(*hot_amp, n_hot)
        sig = rng.uniform(*hot_sigma_km, n_hot)
        h = np.zeros(g.num_nodes)
        for k in range(n_hot):
            h += amp[k] * np.exp(-((x - cx[k]) ** 2 + (y - cy[k]) ** 2) / (2 * sig[k] ** 2))
        deg = np.diff(g.indptr)
        src = np.repeat(np.arange(g.num_nodes), deg)
        mix = np.zeros((g.num_nodes, 4))
        np.add.at(mix, (src, np.minimum(g.road_class, 3)), 1.0)
        signal = (deg >= 4) & ((mix > 0).sum(1) >= 2)
        h += signal_pace * signal
        self.hidden = h                       # s/m on the segment leaving the node
        self.hotspots = n_hot
        self.signals = int(signal.sum())
        self._src = src

    def edge_seconds(self, paths: Sequence[Sequence[int]]) -> np.ndarray:
        """Edge-cost seconds along node paths (consecutive nodes must be adjacent)."""
        g = self.g
        out = np.zeros(len(paths))
        for i, p in enumerate(paths):
            p = np.asarray(p, dtype=np.int64)
            if len(p) < 2:
                continue
            tot = 0.0
            for a, b in zip(p[:-1], p[1:]):
                lo, hi = g.indptr[a], g.indptr[a + 1]
                j = lo + int(np.searchsorted(g.indices[lo:hi], b))
                if j >= hi or g.indices[j] != b:
                    raise ValueError(f"path step {a}->{b} is not an edge")
                tot += self.cost[j]
            out[i] = tot
        return out

    def hidden_seconds(self, paths: Sequence[Sequence[int]]) -> np.ndarray:
        rptr, nodes = paths_csr(paths)
        d = segment_lengths(self.g, nodes, rptr)
        seg = np.repeat(np.arange(len(paths)), np.diff(rptr))
        return np.bincount(seg, weights=self.hidden[nodes] * d, minlength=len(paths)) if len(nodes) else np.zeros(len(paths))

    def true_seconds(self, paths: Sequence[Sequence[int]], known: Optional[np.ndarray] = None) -> np.ndarray:
        known = self.edge_seconds(paths) if known is None else np.asarray(known, dtype=np.float64)
        return known + self.hidden_seconds(paths)

    def observe(self, n: int, search: Search, seed: int = 1, min_km: float = 1.5, max_km: float = 15.0,
                via_share: float = 0.5) -> "Observations":
        """n observed trips: (path, observed seconds, edge-cost seconds)."""
        from ..data.graph import synth_route_queries
        from ..routing.providers import haversine_m
        g = self.g
        rng = np.random.default_rng(seed)
        s, t = synth_route_queries(g, n, seed=seed, min_km=min_km, max_km=max_km)
        via = rng.random(n) < via_share
        w = rng.integers(0, g.num_nodes, n)
        # a via node near the s-t corridor: resample a few times, keep the best detour ratio <= 1.5
        for _ in range(6):
            d_st = haversine_m(g.lat[s], g.lon[s], g.lat[t], g.lon[t])
            det = haversine_m(g.lat[s], g.lon[s], g.lat[w], g.lon[w]) + haversine_m(g.lat[w], g.lon[w], g.lat[t], g.lon[t])
            bad = via & (det > 1.5 * d_st)
            if not bad.any():
                break
            w[bad] = rng.integers(0, g.num_nodes, int(bad.sum()))
        src, dst, kind = [], [], []
        for i in range(n):
            if via[i] and w[i] != s[i] and w[i] != t[i]:
                src += [int(s[i]), int(w[i])]
                dst += [int(w[i]), int(t[i])]
                kind.append(2)
            else:
                src.append(int(s[i]))
                dst.append(int(t[i]))
                kind.append(1)
        res = search(src, dst)
        paths, known = [], []
        o = 0
        for k in kind:
            if k == 1:
                sec, p = res[o]
                o += 1
            else:
                (c1, p1), (c2, p2) = res[o], res[o + 1]
                o += 2
                sec, p = (c1 + c2, list(p1) + list(p2[1:])) if p1 and p2 else (float("nan"), [])
            if p and len(p) > 1 and np.isfinite(sec):
                paths.append(list(map(int, p)))
                known.append(float(sec))
        known = np.asarray(known)
        true = self.true_seconds(paths, known)
        obs = true * (1.0 + self.noise * rng.standard_normal(len(true)))
        return Observations(self.g, paths, obs, known)


class Observations:
    """Observed trips as device-ready CSR: node ids, per-node segment metres, trip ids, residuals."""

    def __init__(self, g: RoadGraph, paths: List[List[int]], observed: np.ndarray, known: np.ndarray):
        self.paths = paths
        self.observed = np.asarray(observed, dtype=np.float64)
        self.known = np.asarray(known, dtype=np.float64)
        self.residual = self.observed - self.known
        self.rptr, self.nodes = paths_csr(paths)
        self.dseg = segment_lengths(g, self.nodes, self.rptr)
        self.trip = np.repeat(np.arange(len(paths)), np.diff(self.rptr))

    def __len__(self) -> int:
        return len(self.paths)

    def tensors(self, device) -> Dict[str, torch.Tensor]:
        d = torch.device(device) if device is not None else torch.device("cpu")
        return {"nodes": torch.from_numpy(self.nodes).to(d), "trip": torch.from_numpy(self.trip).to(d),
                "dseg": torch.from_numpy(self.dseg.astype(np.float32)).to(d),
                "residual": torch.from_numpy(self.residual.astype(np.float32)).to(d)}


def predicted_hidden(delay: torch.Tensor, T: Dict[str, torch.Tensor], n_trips: int) -> torch.Tensor:
    """Per trip: sum_i (delay(v_i) - 0.5) |v_i v_{i+1}| / V_REF."""
    contrib = (delay[T["nodes"]] - 0.5) * T["dseg"] / V_REF
    return torch.zeros(n_trips, dtype=contrib.dtype, device=contrib.device).index_add_(0, T["trip"], contrib)


class ObservedTrainerTorch:
    """fp32 autograd reference (CPU tests, gradient checks)."""

    def __init__(self, model: GcnScorer, g: RoadGraph, obs: Observations, lr: float = 3e-3):
        self.m = model
        self.A = GcnScorer.adjacency(g)
        self.X = torch.from_numpy(g.features)
        self.T = obs.tensors(None)
        self.n = len(obs)
        self.opt = torch.optim.AdamW(self.m.parameters(), lr=lr, weight_decay=0.0)

    def loss(self) -> torch.Tensor:
        pred = predicted_hidden(self.m(self.A, self.X), self.T, self.n)
        return ((pred - self.T["residual"]) ** 2).mean()

    def step(self) -> float:
        self.opt.zero_grad()
        l = self.loss()
        l.backward()
        self.opt.step()
        return float(l.detach())


class ObservedTrainerHip(GcnTrainerHip):
    """The HIP trainer (forward kernels, MFMA backward, fused AdamW) on the path-aggregated loss."""

    def __init__(self, model: GcnScorer, g: RoadGraph, obs: Observations, device, lr: float = 3e-3, **dp: Any):
        super().__init__(model, g, np.zeros(g.num_nodes, dtype=np.float32), device, lr=lr, **dp)
        self.T = obs.tensors(self.dev)
        self.n = len(obs)
        self.delay = torch.zeros(self.N, dtype=torch.float32, device=self.dev)
        self.path_loss = torch.zeros((), dtype=torch.float32, device=self.dev)

    def node_delays(self) -> torch.Tensor:
        self._frags()
        self.C.gcn_l1_fused(self.X, self.indptr, self.indices, self.values, self.w1frag, self.v["b1"],
                            self.w2frag, self.Z, 0, self.N)
        self.C.gcn_spmm_score(self.Z, self.indptr, self.indices, self.values, self.v["b2"], self.v["wo"],
                              float(self.v["bo"].item()), self.delay, 0, self.N)
        return self.delay

    def grad(self) -> torch.Tensor:
        delay = self.node_delays()
        err = predicted_hidden(delay, self.T, self.n) - self.T["residual"]
        self.path_loss = (err * err).mean()
        # dL/ddelay(v) = sum over trip nodes of 2 err / n * dseg / V_REF
        gd = torch.zeros(self.N, dtype=torch.float32, device=self.dev).index_add_(
            0, self.T["nodes"], (2.0 / self.n) * err[self.T["trip"]] * self.T["dseg"] / V_REF)
        self.target.copy_(delay - 0.5 * self.N * gd)
        r0, r1 = self.rows
        self.C.gcn_train_bwd(self.X, self.Z, self.indptr, self.indices, self.values, self.w1frag, self.v["b1"],
                             self.v["W2"], self.v["b2"], self.v["wo"], self.v["bo"], self.target, r0, r1,
                             self.dy, self.slab1, self.slab2, self.P.grad, self.loss_last)
        return self.P.grad

    def mse(self) -> float:
        return float(self.path_loss.item())


def train_observed(g: RoadGraph, obs: Observations, steps: int = 400, lr: float = 5e-3, device=None, seed: int = 0,
                   log_every: int = 0, **dp: Any) -> Tuple[GcnScorer, Dict[str, Any]]:
    model = GcnScorer(seed=seed)
    hist = []
    if device is not None and torch.device(device).type == "cuda":
        tr = ObservedTrainerHip(model, g, obs, device, lr=lr, **dp)
        for i in range(steps):
            tr.step()
            if log_every and (i % log_every == 0 or i == steps - 1):
                hist.append({"step": i, "path_mse": tr.mse()})
        model = tr.to_model()
    else:
        tr = ObservedTrainerTorch(model, g, obs, lr=lr)
        for i in range(steps):
            l = tr.step()
            if log_every and (i % log_every == 0 or i == steps - 1):
                hist.append({"step": i, "path_mse": l})
    r = obs.residual
    return model, {"target": "observed trips", "trips": len(obs), "history": hist,
                   "residual_mean_s": float(r.mean()), "residual_std_s": float(r.std())}


def node_delays(model: GcnScorer, g: RoadGraph, device=None) -> np.ndarray:
    if device is not None and torch.device(device).type == "cuda":
        from .gcn import GcnScorerHip
        return GcnScorerHip(model, g, torch.device(device)).node_delays().cpu().numpy().astype(np.float64)
    with torch.no_grad():
        return model(GcnScorer.adjacency(g), torch.from_numpy(g.features)).double().numpy()


def hidden_from_delays(g: RoadGraph, delay: np.ndarray, paths: Sequence[Sequence[int]]) -> np.ndarray:
    """Predicted hidden seconds of node paths from node delay factors."""
    rptr, nodes = paths_csr(paths)
    d = segment_lengths(g, nodes, rptr)
    seg = np.repeat(np.arange(len(paths)), np.diff(rptr))
    return np.bincount(seg, weights=(delay[nodes] - 0.5) * d / V_REF, minlength=len(paths)) if len(nodes) else np.zeros(len(paths))


def choose(seconds: Sequence[float], hidden_pred: Sequence[float]) -> int:
    """The candidate with the least edge-cost seconds + predicted hidden seconds."""
    tot = np.asarray(seconds, dtype=np.float64) + np.asarray(hidden_pred, dtype=np.float64)
    tot = np.where(np.isfinite(tot), tot, np.inf)
    return int(np.argmin(tot))


def evaluate(world: TripWorld, search: Search, delays: Dict[str, np.ndarray], n_trips: int = 2000, k: int = 6,
             seed: int = 7, edge_scorer_delay: Optional[np.ndarray] = None) -> Dict[str, Any]:
    """Held-out trips with k candidates each; mean TRUE seconds of each policy's pick.

    ``delays``: name -> node delay factors of observed-trip scorers (picked by seconds + hidden);
    ``edge_scorer_delay``: the round-3 edge-cost scorer (picked by argmin delay-weighted length)."""
    from .gcn import score_routes_ref
    g = world.g
    trips = via_alternatives(g, n_trips, k=k, seed=seed, min_km=3.0, max_km=15.0)
    routes, secs = candidate_routes(trips, search)
    picks: Dict[str, List[float]] = {"router_shortest": [], "oracle": []}
    for name in delays:
        picks[name] = []
    if edge_scorer_delay is not None:
        picks["edge_cost_scorer"] = []
    changed = {name: 0 for name in delays}
    for rr, ss in zip(routes, secs):
        ok = [i for i, p in enumerate(rr) if p and len(p) > 1 and np.isfinite(ss[i])]
        if len(ok) < 2:
            continue
        paths = [rr[i] for i in ok]
        known = np.asarray([ss[i] for i in ok])
        true = world.true_seconds(paths, known)
        base = int(np.argmin(known))
        picks["router_shortest"].append(true[base])
        picks["oracle"].append(true.min())
        for name, dl in delays.items():
            j = choose(known, hidden_from_delays(g, dl, paths))
            picks[name].append(true[j])
            changed[name] += int(j != base)
        if edge_scorer_delay is not None:
            j = int(np.argmin(score_routes_ref(g, edge_scorer_delay, paths)))
            picks["edge_cost_scorer"].append(true[j])
    base = float(np.mean(picks["router_shortest"]))
    out: Dict[str, Any] = {"trips": len(picks["router_shortest"]), "k": k,
                           "mean_true_s": {n: round(float(np.mean(v)), 2) for n, v in picks.items()},
                           "gain_vs_router_pct": {n: round(100.0 * (base - float(np.mean(v))) / base, 2)
                                                  for n, v in picks.items()},
                           "picks_changed": changed}
    return out
