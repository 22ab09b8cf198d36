#!/usr/bin/env python3
"""Small A* run for profilers (rocprofv3 --kernel-trace / --pmc): the 100k-node graph, --legs random
1-25 km legs searched --repeat times.  With legs >= 32768 the lane tier runs first (astar_kernel)
and the rest finish in the wave tier (astar_wave_kernel); fewer legs run the wave tier only."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from routest_amd.data.graph import synth_road_graph, synth_route_queries  # noqa: E402
from routest_amd.routing.graph import BatchedAstar, edge_costs  # noqa: E402
from routest_amd.serve.eta_service import default_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--legs", type=int, default=40_000)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    g = synth_road_graph(a.nodes, seed=0)
    cost = edge_costs(g, default_model(hidden=64, steps=50), device="cuda:0")
    S, T = synth_route_queries(g, a.legs, seed=5, min_km=1, max_km=25)
    astar = BatchedAstar(g, cost, "cuda:0", slots=min(a.legs, 65536), wave_slots=min(a.legs, 32768))
    astar.run(S[:512], T[:512])
    torch.cuda.synchronize()
    for _ in range(a.repeat):
        t0 = time.perf_counter()
        c, n, st, _ = astar.run(S, T)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"legs": a.legs, "ms": round(el * 1e3, 2), "legs_per_s": round(a.legs / el),
                          "tiers": astar.last_stats, "status": np.bincount(st.cpu().numpy(), minlength=5).tolist()}),
              flush=True)


if __name__ == "__main__":
    main()
