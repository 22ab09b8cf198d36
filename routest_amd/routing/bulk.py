"""Config 5 step: R concurrent multi-stop requests on one device, end to end on the GPU.

Per step, for all R requests of this rank (each: depot + 2..10 stops snapped to road-graph nodes),
with the CCH router (default, ``router=`` a :class:`routing.cch.RoadRouter`):

  road-metre matrices of every request (CCH chain sweeps + meets, one launch set)
  + K6 greedy multi-trip CVRP over them                    (one launch, all requests)
  -> every trip leg as one CCH query with its path unpacked  (sweep + meet + unpack launches)
  -> edge times from the ETA MLP for the step's routing context (customized once, cached)

or, with ``engine="astar"`` (round 3): K5 haversine matrices + K6, then every leg in the tiered
batched A* (K9).

The legs are derived on the device from K6's visit order; only the (src, dst) node lists cross to
the host once for the A* launch.  Used by ``bench/route_bench.py`` and the ``route_optimizer`` key of
``bench.py`` (requests sharded over ranks, no collective: SURVEY §2.7 C6 / §2.8 P2).  Replaces the
reference's per-request remote ORS matrix + greedy loop + per-trip directions
(``/root/reference/backend/route_optimizer_twx2/Flaskr/utils.py:85-193``).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..ops import _ext
from .batched import pack_requests
from .graph import BatchedAstar


class BulkRouteStep:
    def __init__(self, g, cost: np.ndarray, device, requests: int, seed: int = 100,
                 max_slots: int = 98304, astar: Optional[BatchedAstar] = None,
                 radius_km: Optional[float] = None, router=None, key: Optional[int] = None,
                 engine: str = "cch"):
        self.C = _ext.native(required=True)
        self.dev = d = torch.device(device)
        rng = np.random.default_rng(seed)
        reqs, snapped = [], []
        # radius_km: every request's depot and stops lie within that distance of a random centre
        # (a delivery area, snapped to the nearest road nodes); None: uniform over the whole graph
        local = None
        if radius_km:
            ns = rng.integers(2, 11, requests)
            c = rng.integers(0, g.num_nodes, requests)
            tot = int((ns + 1).sum())
            rc = np.repeat(c, ns + 1)
            r = radius_km * np.sqrt(rng.random(tot))
            th = rng.random(tot) * 2 * np.pi
            plat = g.lat[rc] + r * np.cos(th) / 111.195
            plon = g.lon[rc] + r * np.sin(th) / (111.195 * np.cos(np.radians(g.lat[rc])))
            local = np.split(np.asarray(g.nearest_nodes(plat, plon), dtype=np.int64), np.cumsum(ns + 1)[:-1])
        for k in range(requests):
            if local is not None:
                nodes = local[k]
                n = len(nodes) - 1
            else:
                n = int(rng.integers(2, 11))
                nodes = rng.integers(0, g.num_nodes, n + 1)
            reqs.append({"source_point": {"lat": float(g.lat[nodes[0]]), "lon": float(g.lon[nodes[0]])},
                         "destination_points": [{"lat": float(g.lat[v]), "lon": float(g.lon[v]),
                                                 "payload": int(rng.integers(1, 4))} for v in nodes[1:]],
                         "driver_details": {"vehicle_capacity": 8, "maximum_distance": 150_000}})
            snapped.append(nodes.astype(np.int32))
        lat, lon, dem, npts, cap, maxd = pack_requests(reqs)
        T = lambda x, dt=torch.float64: torch.as_tensor(x, dtype=dt).to(d)  # noqa: E731
        self.lat, self.lon, self.dem = T(lat), T(lon), T(dem)
        self.npts, self.cap, self.maxd = T(npts, torch.int32), T(cap), T(maxd)
        snap = np.full((requests, lat.shape[1]), -1, dtype=np.int32)
        for k, s in enumerate(snapped):
            snap[k, :len(s)] = s
        self.snap = torch.from_numpy(snap).to(d)
        self.requests = requests
        # every leg of a step in ONE lane-tier launch (~80k concurrent searches on one GPU) and the
        # searches left after the pop budget in one or a few wave-tier launches, so each CU keeps
        # several waves of searches in flight (sparse per-search tables: ~33 GB of HBM3E in all)
        legs_est = int(sum(len(s) for s in snapped) * 1.4) + 1024
        slots = min(legs_est, max_slots)
        # every search the lane tier leaves (with the length split: ~65k+ of 80k here) in ONE wave-tier
        # launch with 2^14-entry starting tables (fewer growth steps): 163 -> 142 ms per 10k-request
        # step on the 100k-node graph (profiles/superseded/route_tiering_ab_r3q.jsonl); 98304 slots instead of
        # 65536 once the long legs skip the lane tier: 124.2 -> 119.6 ms (route_wave_slots_ab_r3aj.jsonl).
        # Workspace: lane tier ~8 GB, wave tier ~39 GB, big tier ~4 GB, growth arena 16 GB (of 288 GB)
        self.engine = engine
        self.router = self.key = self.astar = None
        if engine == "cch":
            from .cch import RoadRouter
            self.router = router or RoadRouter(g, device=d)
            self.key = key if key is not None else self.router.metric_from_costs(1 << 41, cost)
            return
        ws = int(os.environ.get("ROUTEST_BULK_WAVE_SLOTS", "98304"))
        tb = int(os.environ.get("ROUTEST_BULK_WAVE_TBITS", "14"))
        self.astar = astar or BatchedAstar(g, cost, d, slots=slots, wave_slots=min(slots, ws), arena_gb=16,
                                           wave_tbits=tb)

    reuse_chains = os.environ.get("ROUTEST_BULK_REUSE_CHAINS", "1") != "0"

    def legs(self, with_index: bool = False):
        """Matrices (CCH road metres, or K5 haversine) + K6 for every request, then the trip legs as
        (src, dst) node tensors on the device (``with_index``: also the legs' (request, from point,
        to point) indices and the tag of the matrix chains they can reuse)."""
        C = self.C
        tag = 0
        if self.engine == "cch":
            _, met, tag = self.router.gpu.matrix_keep(self.key, self.snap, self.npts)
            D = met.double()
        else:
            D = C.route_haversine_matrix(self.lat, self.lon, self.npts, 1.3)
        visit, trip_of, ntrips, status = C.route_greedy_cvrp(D, self.npts, self.dem, self.cap, self.maxd)
        snap = self.snap
        valid = visit >= 0
        prev_same = torch.zeros_like(valid)
        prev_same[:, 1:] = valid[:, 1:] & (trip_of[:, 1:] == trip_of[:, :-1])
        next_same = torch.zeros_like(valid)
        next_same[:, :-1] = valid[:, :-1] & (trip_of[:, :-1] == trip_of[:, 1:])
        vnode = torch.gather(snap, 1, visit.clamp_min(0).long())
        depot = snap[:, :1].expand_as(vnode)
        prev_node = torch.where(prev_same, torch.roll(vnode, 1, 1), depot)
        last = valid & ~next_same
        src = torch.cat([prev_node[valid], vnode[last]])
        dst = torch.cat([vnode[valid], depot[last]])
        if not with_index:
            return src, dst, status
        vis = visit.clamp_min(0)
        prev_i = torch.where(prev_same, torch.roll(vis, 1, 1), torch.zeros_like(vis))
        rows = torch.arange(vis.shape[0], device=vis.device, dtype=vis.dtype)[:, None].expand_as(vis)
        ri = torch.cat([rows[valid], rows[last]]).int().contiguous()
        ii = torch.cat([prev_i[valid], vis[last]]).int().contiguous()
        jj = torch.cat([vis[valid], torch.zeros_like(vis[last])]).int().contiguous()
        return src, dst, status, (ri, ii, jj, tag)

    def step(self):
        """One whole step; returns (legs, per-leg cost [s], per-leg status, per-request K6 status).
        CCH: the legs run between points whose chains the matrix stage already swept, so they reuse
        them (meet + unpack only; ROUTEST_BULK_REUSE_CHAINS=0 sweeps them again)."""
        if self.engine == "cch":
            src, dst, status, (ri, ii, jj, tag) = self.legs(with_index=True)
            if self.reuse_chains:
                sec, _, st, _, _ = self.router.gpu.legs_from_matrix(self.key, tag, self.snap, ri, ii, jj,
                                                                    self.router.max_path, True)
            else:
                sec, _, st, _, _ = self.router.gpu.route(self.key, src.int().contiguous(), dst.int().contiguous(),
                                                         self.router.max_path, True)
            return int(src.numel()), sec, st, status
        src, dst, status = self.legs()
        c, _, st, _ = self.astar.run(src.cpu().numpy(), dst.cpu().numpy())
        return int(src.numel()), c, st, status
