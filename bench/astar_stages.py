#!/usr/bin/env python3
"""Two-stage A* timing breakdown on the 80k route-bench legs: lane stage (pop budget) vs wave stage
(one wave per remaining query), tail size, and the wave stage at different chunk sizes."""
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
a = BatchedAstar(g, cost, "cuda:0", slots=80000, cap=65536)
a.run(S[:2000], T[:2000])
torch.cuda.synchronize()
d = a.dev
s, t = torch.as_tensor(S).to(d), torch.as_tensor(T).to(d)
Q = len(S)
oc = torch.empty(Q, dtype=torch.float32, device=d)
ol = torch.empty(Q, dtype=torch.int32, device=d)
os_ = torch.empty(Q, dtype=torch.int32, device=d)
op = torch.empty((Q, a.max_path), dtype=torch.int32, device=d)
it = torch.empty(Q, dtype=torch.int32, device=d)
BUDGETS = [int(x) for x in os.environ.get("BUDGETS", "1,1000,2000").split(",")]
CHUNKS = [int(x) for x in os.environ.get("CHUNKS", "16384,32768,65536").split(",")]
for budget in BUDGETS:
    t0 = time.perf_counter()
    a.C.astar(a.indptr, a.indices, a.cost, a.lat, a.lon, s, t, a.state, a.heap, a.touched, oc, ol, os_, op,
              0, budget, a.inv_vmax, a.lm, it)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tail = (os_ == 3).nonzero().flatten().to(torch.int32)
    if a.hcache is None or a.hcache.shape[0] < max(CHUNKS):
        a.hcache = None
        torch.cuda.empty_cache()
        a.hcache = torch.full((max(CHUNKS), g.num_nodes), float("nan"), dtype=torch.float32, device=d)
    for chunk in CHUNKS:
        # re-run only the tail chunk-wise (costs identical, exact)
        t2 = time.perf_counter()
        for i0 in range(0, tail.numel(), chunk):
            a.C.astar(a.indptr, a.indices, a.cost, a.lat, a.lon, s, t, a.state, a.heap, a.touched, oc, ol, os_, op,
                      0, a.max_iters, a.inv_vmax, a.lm, it, tail[i0:i0 + chunk].contiguous(), a.wave_delta, a.hcache)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        ex = it[tail.long()].cpu().numpy()
        print(f"budget {budget}: lane stage {1e3 * (t1 - t0):.1f} ms, tail {tail.numel()} queries, wave stage "
              f"(chunk {chunk}) {1e3 * (t3 - t2):.1f} ms, expansions p50/p99/max "
              f"{np.percentile(ex, [50, 99, 100]).astype(int).tolist()}, total {int(ex.sum())}", flush=True)
        # restore tail status for the next chunk-size trial
        os_[tail.long()] = 3
