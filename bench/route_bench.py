#!/usr/bin/env python3
"""Config 5: batched multi-stop route optimizer with A* over MLP edge costs — R concurrent
requests sharded over the node's GPUs (no collective: SURVEY §2.8 P2).

Per step on every rank, for its R/world requests (each: depot + 2..10 stops on the road graph):
  K5 haversine matrices + K6 greedy multi-trip CVRP (one launch each, all requests)
  -> every trip leg (consecutive stops incl. depot returns) as one A* query (K9, one launch)
  -> per-request duration (sum of leg costs from the learned edge times).
Stops are snapped to graph nodes once at request-parse time (outside the timed loop)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=10_000, help="total concurrent requests")
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU; without torchrun this script launches them itself")
    a = ap.parse_args()
    from routest_amd.parallel.launch import ensure_ranks, share_gpu
    ensure_ranks(a.gpus, __file__)
    import numpy as np
    import torch
    import torch.distributed as dist
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.ops import _ext
    from routest_amd.parallel.dp import allreduce_scalars, barrier, init_distributed
    from routest_amd.routing.batched import pack_requests
    from routest_amd.routing.graph import BatchedAstar, edge_costs
    from routest_amd.serve.eta_service import default_model

    di = init_distributed()
    dev = di.device
    C = _ext.native()
    g = synth_road_graph(a.nodes, seed=0)
    torch.manual_seed(0)
    cost = edge_costs(g, default_model(hidden=256, steps=200), device=dev)
    rng = np.random.default_rng(100 + di.rank)
    R = a.requests // di.world
    reqs, snapped = [], []
    for _ in range(R):
        n = int(rng.integers(2, 11))
        nodes = rng.integers(0, g.num_nodes, n + 1)
        reqs.append({"source_point": {"lat": float(g.lat[nodes[0]]), "lon": float(g.lon[nodes[0]])},
                     "destination_points": [{"lat": float(g.lat[v]), "lon": float(g.lon[v]),
                                             "payload": int(rng.integers(1, 4))} for v in nodes[1:]],
                     "driver_details": {"vehicle_capacity": 8, "maximum_distance": 150_000}})
        snapped.append(nodes.astype(np.int32))
    lat, lon, dem, npts, cap, maxd = pack_requests(reqs)
    T = lambda x, dt=torch.float64: torch.as_tensor(x, dtype=dt).to(dev)  # noqa: E731
    lat_t, lon_t, dem_t, npts_t, cap_t, maxd_t = T(lat), T(lon), T(dem), T(npts, torch.int32), T(cap), T(maxd)
    NM = lat.shape[1]
    snap = np.full((R, NM), -1, dtype=np.int32)
    for k, s in enumerate(snapped):
        snap[k, :len(s)] = s
    snap_t = torch.from_numpy(snap).to(dev)
    # every leg of a step in ONE launch: ~80k concurrent searches (dense per-slot state ~95 GB —
    # sized for 288 GB of HBM3E) so each CU keeps ~5 waves of latency-bound searches in flight
    legs_est = int(sum(len(s) for s in snapped) * 1.4) + 1024
    astar = BatchedAstar(g, cost, dev, slots=min(legs_est, 98304), cap=65536)

    def step():
        D = C.route_haversine_matrix(lat_t, lon_t, npts_t, 1.3)
        visit, trip_of, ntrips, status = C.route_greedy_cvrp(D, npts_t, dem_t, cap_t, maxd_t)
        # legs: depot -> first stop, stop -> stop within a trip, last stop -> depot  (device-side)
        valid = visit >= 0
        prev_same = torch.zeros_like(valid)
        prev_same[:, 1:] = valid[:, 1:] & (trip_of[:, 1:] == trip_of[:, :-1])
        next_same = torch.zeros_like(valid)
        next_same[:, :-1] = valid[:, :-1] & (trip_of[:, :-1] == trip_of[:, 1:])
        vnode = torch.gather(snap_t, 1, visit.clamp_min(0).long())
        prev_node = torch.where(prev_same, torch.roll(vnode, 1, 1), snap_t[:, :1].expand_as(vnode))
        src = torch.cat([prev_node[valid], vnode[valid & ~next_same]])
        dst = torch.cat([vnode[valid], snap_t[:, :1].expand_as(vnode)[valid & ~next_same]])
        c, n, st, _ = astar.run(src.cpu().numpy(), dst.cpu().numpy())
        return int(src.numel()), c, st

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    barrier(dev)
    t0 = time.perf_counter()
    legs = 0
    for _ in range(a.steps):
        nl, c, st = step()
        legs += nl
    torch.cuda.synchronize()
    barrier(dev)
    el = allreduce_scalars([time.perf_counter() - t0], dev, op="max")[0]
    tot_legs = allreduce_scalars([legs], dev)[0]
    ok = float((st == 0).float().mean())
    status_hist = torch.bincount(st.long().cpu(), minlength=5).tolist()
    if di.is_main:
        print(json.dumps({"metric": "batched multi-stop optimizer (greedy CVRP + A* w/ MLP edge costs)",
                          "n_gpus": di.world, "requests_per_step": a.requests, "nodes": g.num_nodes,
                          "ms_per_step": el / a.steps * 1e3, "requests_per_s": a.requests * a.steps / el,
                          "astar_legs_per_s": tot_legs / el, "legs_per_step": tot_legs / a.steps,
                          "astar_found_frac": ok, "astar_status_hist": status_hist}), flush=True)
    if di.world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
