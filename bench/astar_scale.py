#!/usr/bin/env python3
"""Road routing at scale: a synthetic road graph of --nodes nodes (default 1M) serving --requests
concurrent multi-stop requests (2-10 stops each; matrices + K6 trips; every trip leg routed with its
path) in ONE step on one GPU.  ``--engine cch`` (default): CCH road-metre matrices + CCH legs
(csrc/cch.hip; the customization for the step's metric is timed separately, it is cached per
context); ``--engine astar``: round 3's K5 haversine matrices + the sparse-state A* (csrc/astar.hip).

Reports the search workspace (all three tiers) and the peak device memory, wall time per step, legs
and requests per second, the tier split (lane / wave / big) and host fallbacks, and checks a sample
of legs against scipy Dijkstra (exact costs).  --radius-km R puts each request's stops within R km of
a random centre (a delivery area); 0 spreads them over the whole map (legs across the city).

    python bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from routest_amd.data.graph import synth_road_graph  # noqa: E402
from routest_amd.routing.bulk import BulkRouteStep  # noqa: E402
from routest_amd.routing.graph import BatchedAstar, edge_costs  # noqa: E402
from routest_amd.serve.eta_service import default_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--requests", type=int, default=10_000)
    ap.add_argument("--radius-km", type=float, default=8.0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--slots", type=int, default=65536)
    ap.add_argument("--wave-slots", type=int, default=32768)
    ap.add_argument("--arena-gb", type=float, default=16.0)
    ap.add_argument("--check", type=int, default=12)
    ap.add_argument("--engine", default="cch", choices=["cch", "astar"])
    args = ap.parse_args()
    if args.engine == "cch":
        return main_cch(args)
    d = torch.device("cuda", 0)
    t0 = time.time()
    g = synth_road_graph(args.nodes, seed=0)
    cost = edge_costs(g, default_model(hidden=64, steps=50), device=d)
    print(f"graph {g.num_nodes} nodes / {len(g.indices)} edges in {time.time() - t0:.1f} s", flush=True)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(d)
    t0 = time.time()
    astar = BatchedAstar(g, cost, d, slots=args.slots, wave_slots=args.wave_slots, arena_gb=args.arena_gb)
    print(f"A* ready in {time.time() - t0:.1f} s (landmarks included)", flush=True)
    step = BulkRouteStep(g, cost, d, args.requests, astar=astar, radius_km=args.radius_km or None)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(d)
    t1 = time.perf_counter()
    legs, c, st, _ = step.step()                       # warm-up
    torch.cuda.synchronize()
    print(f"warm-up step: {legs} legs in {time.perf_counter() - t1:.2f} s, tiers {astar.last_stats}", flush=True)
    times, tiers = [], []
    for _ in range(args.steps):
        t1 = time.perf_counter()
        legs, c, st, _ = step.step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t1)
        tiers.append(dict(astar.last_stats, fallbacks=astar.last_fallbacks))
        print(f"step: {times[-1] * 1e3:.1f} ms, tiers {tiers[-1]}", flush=True)
    peak = torch.cuda.max_memory_allocated(d)
    stc = np.bincount(st.cpu().numpy(), minlength=5).tolist()
    # exactness on a sample of legs (scipy Dijkstra per source)
    src, dst, _ = step.legs()
    src, dst = src.cpu().numpy(), dst.cpu().numpy()
    rng = np.random.default_rng(0)
    pick = rng.choice(len(src), min(args.check, len(src)), replace=False)
    from routest_amd.routing.graph import dijkstra_ref
    ref = dijkstra_ref(g, cost, src[pick], dst[pick])
    got = c.cpu().numpy()[pick]
    ok = bool(np.allclose(got, ref, rtol=1e-4, atol=1e-3))
    ms = 1e3 * float(np.median(times))
    out = {"metric": "multi-stop requests in one step (sparse A* workspace)", "nodes": g.num_nodes,
           "edges": int(len(g.indices)), "requests": args.requests, "radius_km": args.radius_km, "legs": legs,
           "ms_per_step": round(ms, 2), "req_per_s": round(args.requests / ms * 1e3, 1),
           "legs_per_s": round(legs / ms * 1e3, 1), "status": stc, "tiers": tiers[-1],
           "workspace_GB": round(astar.workspace_bytes / 2**30, 2),
           "tiers_GB": {k: round(t.nbytes / 2**30, 2) for k, t in (("lane", astar.lane_tier), ("wave", astar.wave_tier),
                                                                   ("big", astar.big_tier)) if t is not None},
           "peak_device_GB_above_graph": round((peak - base) / 2**30, 2),
           "sample_exact_vs_dijkstra": ok, "sample": len(pick)}
    print(json.dumps(out), flush=True)


def main_cch(args):
    from routest_amd.routing.cch import RoadRouter
    from routest_amd.routing.graph import dijkstra_ref
    d = torch.device("cuda", 0)
    t0 = time.time()
    g = synth_road_graph(args.nodes, seed=0)
    cost = edge_costs(g, default_model(hidden=64, steps=50), device=d)
    print(f"graph {g.num_nodes} nodes / {len(g.indices)} edges in {time.time() - t0:.1f} s", flush=True)
    t0 = time.time()
    # city-wide legs on a 1M-node grid run to several thousand road nodes
    router = RoadRouter(g, device=d, max_path=16384)
    topo_s = time.time() - t0
    print(f"CCH topology in {topo_s:.1f} s: {router.stats()}", flush=True)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(d)
    t0 = time.perf_counter()
    key = router.metric_from_costs(1 << 41, cost)
    torch.cuda.synchronize()
    cust_ms = (time.perf_counter() - t0) * 1e3
    print(f"customization {cust_ms:.1f} ms: {router.last_metric}", flush=True)
    step = BulkRouteStep(g, cost, d, args.requests, radius_km=args.radius_km or None, router=router, key=key)
    torch.cuda.reset_peak_memory_stats(d)
    t1 = time.perf_counter()
    legs, c, st, _ = step.step()                       # warm-up
    torch.cuda.synchronize()
    print(f"warm-up step: {legs} legs in {time.perf_counter() - t1:.3f} s", flush=True)
    times = []
    for _ in range(args.steps):
        t1 = time.perf_counter()
        legs, c, st, _ = step.step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t1)
        print(f"step: {times[-1] * 1e3:.1f} ms", flush=True)
    # matrix-only share of the step
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    step.legs()
    torch.cuda.synchronize()
    mat_ms = (time.perf_counter() - t1) * 1e3
    peak = torch.cuda.max_memory_allocated(d)
    stc = np.bincount(st.cpu().numpy(), minlength=5).tolist()
    src, dst, _ = step.legs()
    src, dst = src.cpu().numpy(), dst.cpu().numpy()
    rng = np.random.default_rng(0)
    pick = rng.choice(len(src), min(args.check, len(src)), replace=False)
    ref = dijkstra_ref(g, cost, src[pick], dst[pick])
    got = c.cpu().numpy()[pick]
    ok = bool(np.allclose(got, ref, rtol=1e-4, atol=1e-3))
    ms = 1e3 * float(np.median(times))
    out = {"metric": "multi-stop requests in one step (CCH matrices + legs with paths)", "engine": "cch",
           "nodes": g.num_nodes, "edges": int(len(g.indices)), "requests": args.requests,
           "radius_km": args.radius_km, "legs": legs, "ms_per_step": round(ms, 2),
           "matrix_plus_greedy_ms": round(mat_ms, 2), "req_per_s": round(args.requests / ms * 1e3, 1),
           "legs_per_s": round(legs / ms * 1e3, 1), "status": stc, "topology_build_s": round(topo_s, 2),
           "customize_ms": round(cust_ms, 1), "cch": router.stats(),
           "peak_device_GB_above_graph": round((peak - base) / 2**30, 2),
           "sample_exact_vs_dijkstra": ok, "sample": len(pick)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
