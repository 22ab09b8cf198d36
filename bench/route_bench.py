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
    import torch
    import torch.distributed as dist
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.parallel.dp import allreduce_scalars, barrier, init_distributed
    from routest_amd.routing.bulk import BulkRouteStep
    from routest_amd.routing.graph import edge_costs
    from routest_amd.serve.eta_service import default_model

    di = init_distributed()
    dev = di.device
    g = synth_road_graph(a.nodes, seed=0)
    torch.manual_seed(0)
    cost = edge_costs(g, default_model(hidden=256, steps=200), device=dev)
    R = a.requests // di.world
    bulk = BulkRouteStep(g, cost, dev, R, seed=100 + di.rank)

    def step():
        nl, c, st, _ = bulk.step()
        return nl, c, st

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
