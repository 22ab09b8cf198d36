#!/usr/bin/env python3
"""Config 4: 2-layer GCN route scorer over a 100k-node synthetic road graph, 1 -> 8 GPUs.

    python bench/gcn_bench.py [--mode replicate|partition]
    torchrun --nproc-per-node 8 bench/gcn_bench.py --mode partition

A step = all node delays (2 GCN layers over the whole graph, strong scaling in partition mode)
+ scoring R candidate routes (sharded over ranks).  Reports routes/s and ms per step."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--routes", type=int, default=10_000)
    ap.add_argument("--mode", default="partition")
    ap.add_argument("--comm", default="device", choices=["device", "dist"],
                    help="partition gathers: native DeviceComm (one-shot IPC / RCCL on the stream) "
                         "or torch.distributed")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU; without torchrun this script launches them itself")
    a = ap.parse_args()
    from routest_amd.parallel.launch import ensure_ranks, share_gpu
    ensure_ranks(a.gpus, __file__)
    import numpy as np
    import torch
    import torch.distributed as dist
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.models.gcn import GcnScorer, GcnScorerHip, routes_to_csr
    from routest_amd.parallel.dp import allreduce_scalars, barrier, init_distributed

    di = init_distributed()
    dev = di.device
    g = synth_road_graph(a.nodes, seed=0)
    m = GcnScorer(seed=0)
    comm = None
    if a.mode == "partition" and di.world > 1 and a.comm == "device":
        from routest_amd.parallel.comm import DeviceComm
        comm = DeviceComm(dev, use_rccl=not share_gpu(), oneshot_bytes=32 << 20)
    hip = GcnScorerHip(m, g, dev, mode=a.mode, rank=di.rank, world=di.world, comm=comm)
    rng = np.random.default_rng(di.rank)
    routes = []
    for _ in range(a.routes // di.world):
        v = int(rng.integers(0, g.num_nodes))
        path = [v]
        for _ in range(int(rng.integers(50, 300))):
            nb = g.indices[g.indptr[v]:g.indptr[v + 1]]
            v = int(nb[rng.integers(0, len(nb))])
            path.append(v)
        routes.append(path)
    ptr, nodes = routes_to_csr(routes)
    ptr_t, nodes_t = torch.from_numpy(ptr).to(dev), torch.from_numpy(nodes).to(dev)

    def step():
        hip.node_delays()
        return hip.score_routes(ptr_t, nodes_t)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    barrier(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    barrier(dev)
    el = allreduce_scalars([time.perf_counter() - t0], dev, op="max")[0]
    if di.is_main:
        print(json.dumps({"metric": "GCN route scorer", "n_gpus": di.world, "mode": a.mode, "comm": a.comm if comm is not None else "none",
                          "shared_gpu": share_gpu() and di.world > 1, "nodes": g.num_nodes,
                          "edges": g.num_edges, "routes_per_step": a.routes, "ms_per_step": el / a.steps * 1e3,
                          "routes_per_s": a.routes * a.steps / el,
                          "node_updates_per_s": g.num_nodes * a.steps / el}), flush=True)
    if di.world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
