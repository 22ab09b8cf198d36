#!/usr/bin/env python3
"""A* diagnostics (1 GPU): 80k random 1-25 km legs on the 100k-node graph, with and without the
spatial (source-sorted, XCD-aware) launch order; status histogram and wall time per launch."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from routest_amd.data.graph import synth_road_graph, synth_route_queries  # noqa: E402
from routest_amd.routing.graph import BatchedAstar, edge_costs  # noqa: E402
from routest_amd.serve.eta_service import default_model  # noqa: E402

g = synth_road_graph(100_000)
cost = edge_costs(g, default_model(hidden=64, steps=60), "cuda:0")
S, T = synth_route_queries(g, 80000, seed=5, min_km=1, max_km=25)
a = BatchedAstar(g, cost, "cuda:0", slots=80000, wave_slots=32768, arena_gb=16)
for sort in (False, True, False, True):
    a.run(S[:1000], T[:1000], sort=sort)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c, n, st, _ = a.run(S, T, sort=sort)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"sort={sort}: {el * 1e3:.1f} ms ({len(S) / el:.0f} legs/s), status {np.bincount(st.cpu().numpy(), minlength=5).tolist()}",
          flush=True)
