"""Per-context CCH customization time on the GPU (csrc/cch.hip CchGpu::customize): ETA-model edge
costs + basic + perfect customization + pruning for ``--contexts`` fresh routing contexts on a
synthetic city of ``--nodes`` nodes.  One JSON line per context, then a summary line.

Used for the customization work of round 5 (verdict r4 item 3: <= 15 ms per context on the
100k-node graph, <= 250 ms on the 1M-node city) and, under ``rocprofv3 --pmc``, for the hardware
counters of ``basic_level_kernel`` / ``perfect_level_kernel``."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--contexts", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--check", action="store_true", help="compare the last metric with the CPU reference")
    a = ap.parse_args()
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.cch import RoadRouter, RouteContext
    from routest_amd.serve.eta_service import default_model
    dev = torch.device("cuda:0")
    t0 = time.time()
    g = synth_road_graph(a.nodes, seed=a.seed)
    m = default_model(hidden=64, steps=50)
    router = RoadRouter(g, m, device=dev)
    st = router.stats()
    print(json.dumps({"stage": "setup", "s": round(time.time() - t0, 2), **st}), flush=True)
    walls, gpu = [], []
    for i in range(a.contexts):
        ctx = RouteContext(weather=i % 4, congestion=(i // 4) % 4, weekhour=(7 + 5 * i) % 168)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        router.metric(ctx)
        w = (time.perf_counter() - t1) * 1e3
        info = dict(router.last_metric)
        walls.append(w)
        gpu.append(info.get("customize_ms") or 0.0)
        print(json.dumps({"stage": "context", "i": i, "wall_ms": round(w, 3), **info}), flush=True)
    rest = walls[1:] or walls
    out = {"stage": "summary", "nodes": g.num_nodes, "arcs": st["arcs"], "contexts": a.contexts,
           "wall_ms_min": round(min(rest), 3), "wall_ms_mean": round(sum(rest) / len(rest), 3),
           "customize_ms_min": round(min(gpu[1:] or gpu), 3)}
    if a.check:
        import threading
        import numpy as np
        done = threading.Event()

        def beat():          # the CPU reference takes minutes on the 1M city: keep the log alive
            while not done.wait(30):
                print(json.dumps({"stage": "check_running", "s": round(time.time() - t0, 1)}), flush=True)
        threading.Thread(target=beat, daemon=True).start()
        from routest_amd import _rt
        c = _rt.CCH(g.indptr, g.indices, g.lat, g.lon, 16)
        cost = router.costs(ctx)
        mc = c.customize(cost, g.length_m)
        rng = np.random.default_rng(1)
        src = rng.integers(0, g.num_nodes, 4000).astype(np.int32)
        dst = rng.integers(0, g.num_nodes, 4000).astype(np.int32)
        s_gpu, m_gpu, st_gpu, _ = router.route(src, dst, ctx.key, want_path=False)
        s_cpu, m_cpu, st_cpu, _ = c.query(mc, src, dst, False, 4096)
        out["bit_identical_vs_cpu"] = bool(np.array_equal(np.asarray(s_gpu), np.asarray(s_cpu)) and
                                           np.array_equal(np.asarray(m_gpu), np.asarray(m_cpu)) and
                                           np.array_equal(np.asarray(st_gpu), np.asarray(st_cpu)))
        done.set()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
