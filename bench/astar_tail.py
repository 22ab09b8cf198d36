#!/usr/bin/env python3
"""A* tail analysis on route-bench-shaped legs (uniform random stops over the 100k-node graph):
pops per query percentiles and launch time for 16 vs 32 ALT landmarks."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from routest_amd.data.graph import synth_road_graph  # noqa: E402
from routest_amd.routing.graph import BatchedAstar, edge_costs  # noqa: E402
from routest_amd.serve.eta_service import default_model  # noqa: E402

g = synth_road_graph(100_000, seed=0)
torch.manual_seed(0)
cost = edge_costs(g, default_model(hidden=256, steps=200), device="cuda:0")
rng = np.random.default_rng(100)
S = rng.integers(0, g.num_nodes, 80000).astype(np.int32)
T = rng.integers(0, g.num_nodes, 80000).astype(np.int32)
for K, meth in ((32, "farthest"),):
    a = BatchedAstar(g, cost, "cuda:0", slots=80000, wave_slots=32768, arena_gb=16, landmarks=K, landmark_method=meth)
    a.run(S[:1000], T[:1000])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c, n, st, _ = a.run(S, T)
    print("tiers", a.last_stats, "workspace GB", round(a.workspace_bytes / 2**30, 2), flush=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    it = a.last_iters.cpu().numpy()
    pct = np.percentile(it, [50, 90, 99, 99.9, 100]).astype(int).tolist()
    print(f"K={K} {meth}: {el * 1e3:.1f} ms, pops p50/p90/p99/p99.9/max = {pct}, status {np.bincount(st.cpu().numpy(), minlength=5).tolist()}",
          flush=True)
    del a
    torch.cuda.empty_cache()
