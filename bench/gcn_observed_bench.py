"""GCN scorer trained on observed trips (routest_amd/models/gcn_observed.py, verdict r3 item 5).

Synthetic world on a --nodes road graph: edge costs from the ETA MLP (what the CCH router
minimises) + hidden hot spots / signal delays; --trips observed trips train the scorer (HIP trainer
on a GPU, autograd on CPU); held-out trips with k candidates compare the TRUE time of the route
picked by the router alone, the random-init scorer, the round-3 edge-cost scorer, the observed-trip
scorer, and an oracle.  One JSON line.

    python bench/gcn_observed_bench.py --nodes 100000 --trips 50000 --steps 400
"""
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
    ap.add_argument("--trips", type=int, default=50_000)
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--eval-trips", type=int, default=2000)
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--edge-steps", type=int, default=300)
    ap.add_argument("--hot-density", type=float, default=3.0, help="hot spots per 100 km2")
    ap.add_argument("--hot-amp", type=float, nargs=2, default=[0.15, 0.35], help="extra pace s/m at a hot spot centre")
    ap.add_argument("--signal", type=float, default=0.02, help="extra pace s/m leaving a signalised node")
    a = ap.parse_args()
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.models.gcn import GcnScorer
    from routest_amd.models.gcn_observed import TripWorld, node_delays, train_observed, evaluate
    from routest_amd.models.gcn_train import train as train_edge
    from routest_amd.routing.cch import RoadRouter
    from routest_amd.routing.graph import edge_costs
    from routest_amd.serve.eta_service import default_model
    dev = None if a.cpu or not torch.cuda.is_available() else torch.device("cuda:0")
    t0 = time.time()
    g = synth_road_graph(a.nodes, seed=11)
    cost = edge_costs(g, default_model(hidden=64, steps=50), device=dev)
    router = RoadRouter(g, device=dev)
    key = router.metric_from_costs(1 << 42, cost)

    def search(src, dst):
        sec, _, st, paths = router.route(src, dst, key)
        return [(float(sec[i]), paths[i].tolist()) if st[i] == 0 else (float("nan"), []) for i in range(len(src))]

    world = TripWorld(g, cost, seed=3, hot_per_100km2=a.hot_density, hot_amp=tuple(a.hot_amp), signal_pace=a.signal)
    t1 = time.time()
    obs = world.observe(a.trips, search, seed=1)
    t_obs = time.time() - t1
    t1 = time.time()
    model, info = train_observed(g, obs, steps=a.steps, lr=a.lr, device=dev, log_every=max(1, a.steps // 8))
    if dev is not None:
        torch.cuda.synchronize()
    t_train = time.time() - t1
    edge_model, _ = train_edge(g, cost, steps=a.edge_steps, lr=5e-3, device=dev)
    delays = {"random_init_scorer": node_delays(GcnScorer(seed=0), g, dev),
              "observed_trip_scorer": node_delays(model, g, dev)}
    ev = evaluate(world, search, delays, n_trips=a.eval_trips, k=a.k, seed=7,
                  edge_scorer_delay=node_delays(edge_model, g, dev))
    hid = world.hidden_seconds(obs.paths)
    out = {"metric": "held-out true trip time of the picked route (GCN scorer trained on observed trips)",
           "device": str(dev) if dev is not None else "cpu", "nodes": g.num_nodes, "observed_trips": len(obs),
           "hidden_share_of_true_time": round(float(hid.sum() / (obs.known.sum() + hid.sum())), 3),
           "world": {"hotspots": world.hotspots, "signal_nodes": world.signals, "hot_per_100km2": a.hot_density,
                     "hot_amp_s_per_m": a.hot_amp, "signal_s_per_m": a.signal},
           "train_steps": a.steps, "train_s": round(t_train, 2), "observe_s": round(t_obs, 2),
           "path_mse_first_last": [info["history"][0]["path_mse"], info["history"][-1]["path_mse"]],
           "residual_var": round(float(np.var(obs.residual)), 2), **ev, "wall_s": round(time.time() - t0, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
