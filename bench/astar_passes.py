#!/usr/bin/env python3
"""Wave-tier diagnostics: mean expansions vs mean f-band passes per search (= the mean number of
near nodes a pass hands the wave's 64 lanes) on the route bench's legs, every search in the wave
tier.  Run twice: plain, and with ROUTEST_ASTAR_COUNT_PASSES=1 (out_iters then holds passes)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from routest_amd.data.graph import synth_road_graph  # noqa: E402
from routest_amd.routing.bulk import BulkRouteStep  # noqa: E402
from routest_amd.routing.graph import BatchedAstar, edge_costs  # noqa: E402
from routest_amd.serve.eta_service import default_model  # noqa: E402


def main():
    g = synth_road_graph(100_000, seed=0)
    torch.manual_seed(0)
    cost = edge_costs(g, default_model(hidden=256, steps=200), device="cuda:0")
    step = BulkRouteStep(g, cost, "cuda:0", 10000)
    src, dst, _ = step.legs()
    a = step.astar
    a.wave_only_below = 10 ** 9                   # every search in the wave tier
    c, n, st, _ = a.run(src.cpu().numpy(), dst.cpu().numpy())
    it = a.last_iters.cpu().numpy().astype(np.float64)
    print(json.dumps({"count_passes": os.environ.get("ROUTEST_ASTAR_COUNT_PASSES", "0"), "legs": int(len(it)),
                      "mean": float(it.mean()), "p50": float(np.median(it)), "p90": float(np.percentile(it, 90)),
                      "p99": float(np.percentile(it, 99)), "max": float(it.max())}), flush=True)


if __name__ == "__main__":
    main()
