#!/usr/bin/env python3
"""GCN candidate-route scorer training (models/gcn_train.py, csrc/gcn_train.hip) on one GPU.

Trains the 2-layer GCN on per-node delay targets derived from the learned edge times of a synthetic
road graph, then ranks held-out candidate routes (shortest path + via-node detours from the batched
A*) and reports the Spearman correlation of scores vs true seconds — trained and random-init — plus
the training step time of the HIP forward/backward (+ fused torch AdamW)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--lr", type=float, default=5e-3)
    ap.add_argument("--trips", type=int, default=300)
    a = ap.parse_args()
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.models.gcn import GcnScorer, GcnScorerHip
    from routest_amd.models.gcn_train import (GcnTrainerHip, candidate_routes, evaluate_ranking,
                                              node_delay_targets, score_with_delays, via_alternatives)
    from routest_amd.routing.graph import BatchedAstar, edge_costs
    from routest_amd.serve.eta_service import default_model
    dev = torch.device("cuda", 0)
    g = synth_road_graph(a.nodes, seed=4)
    cost = edge_costs(g, default_model(hidden=64, steps=80), device=dev)
    t = node_delay_targets(g, cost)
    tr = GcnTrainerHip(GcnScorer(seed=0), g, t, dev, lr=a.lr)
    for _ in range(3):
        tr.grad()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        tr.grad()
    torch.cuda.synchronize()
    grad_ms = (time.perf_counter() - t0) / 20 * 1e3
    tr = GcnTrainerHip(GcnScorer(seed=0), g, t, dev, lr=a.lr)
    mse0 = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.step()
        if i == 0:
            mse0 = tr.mse()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / a.steps * 1e3
    mse1 = tr.mse()
    model = tr.to_model()
    astar = BatchedAstar(g, cost, dev, slots=4096)
    trips = via_alternatives(g, a.trips, k=4, seed=99)
    routes, secs = candidate_routes(trips, astar.paths)

    def delays(m):
        return GcnScorerHip(m, g, dev).node_delays().cpu().numpy()
    trained = evaluate_ranking(routes, secs, score_with_delays(g, delays(model), routes))
    floor = evaluate_ranking(routes, secs, score_with_delays(g, delays(GcnScorer(seed=0)), routes))
    oracle = evaluate_ranking(routes, secs, score_with_delays(g, t, routes))
    print(json.dumps({"metric": "GCN scorer training (HIP fwd/bwd + fused AdamW)", "nodes": g.num_nodes,
                      "steps": a.steps, "ms_per_step": round(step_ms, 3), "ms_fwd_bwd": round(grad_ms, 3),
                      "nodes_per_s": round(g.num_nodes / step_ms * 1e3), "mse_first": mse0, "mse_last": mse1,
                      "held_out_trips": trained["trips"], "trained": trained, "random_init": floor,
                      "oracle_targets": oracle}), flush=True)


if __name__ == "__main__":
    main()
