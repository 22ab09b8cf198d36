#!/usr/bin/env python3
"""A/B of the tiered A* workspace knobs on the route bench's leg mix (80k random 1-25 km legs on
the 100k-node graph): initial wave-table size (growth), f-band list capacity, wave slots per launch,
lane pop budget.  One process, one graph and landmark set; prints one JSON line per configuration."""
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

CONFIGS = [
    # name, env overrides, ctor kwargs
    ("default", {}, {}),
    ("tables_2^16_no_growth", {"ROUTEST_ASTAR_WAVE_TBITS": "16"}, {}),
    ("lists_64k", {}, {"cap": 65536}),
    ("wave_slots_65536", {}, {"wave_slots": 65536}),
    ("lane_pops_1000", {"ROUTEST_ASTAR_LANE_POPS": "1000"}, {}),
    ("wave_only_65536", {"ROUTEST_ASTAR_WAVE_ONLY_BELOW": "1000000"}, {"wave_slots": 65536}),
]


def main():
    g = synth_road_graph(100_000, seed=0)
    torch.manual_seed(0)
    cost = edge_costs(g, default_model(hidden=256, steps=200), device="cuda:0")
    S, T = synth_route_queries(g, 80000, seed=5, min_km=1, max_km=25)
    only = set(sys.argv[1:])
    lm = None
    for name, env, kw in CONFIGS:
        if only and name not in only:
            continue
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            a = BatchedAstar(g, cost, "cuda:0", slots=80000, **{"wave_slots": 32768, "arena_gb": 16, **kw})
            if lm is None:
                lm = a.lm
            a.run(S[:2000], T[:2000])
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                c, n, st, _ = a.run(S, T)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ms = 1e3 * float(np.median(ts))
            print(json.dumps({"config": name, "ms": round(ms, 1), "legs_per_s": round(len(S) / ms * 1e3),
                              "tiers": a.last_stats, "status": np.bincount(st.cpu().numpy(), minlength=5).tolist(),
                              "workspace_GB": round(a.workspace_bytes / 2**30, 2)}), flush=True)
            del a
            torch.cuda.empty_cache()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main()
