#!/usr/bin/env python3
"""Config 3 benchmark: data-parallel ETA-MLP training samples/s (weak scaling, one rank per GPU).

    python bench/train_bench.py                        # 1 GPU
    torchrun --nproc-per-node 8 bench/train_bench.py   # 8 GPUs, RCCL all-reduce over xGMI

Modes: ``fused`` (HIP kernels only, eager launches), ``graph`` (the whole fused step incl. the RCCL
all-reduce captured in one HIP graph), ``autograd`` (PyTorch eager bf16-autocast baseline with the
same flat-bucket all-reduce).  Each mode: W warmup steps, then K timed steps between barriers.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Pinned:
    """DeviceComm with a fixed algorithm (for A/B sweeps)."""

    def __init__(self, comm, algo):
        self.comm, self.algo = comm, algo

    def all_reduce(self, t):
        return self.comm.all_reduce(t, self.algo)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536, help="per-GPU batch")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--modes", default="fused,graph,autograd")
    ap.add_argument("--trace", default="", help="write a Chrome trace of 3 extra steps per mode (prefix)")
    ap.add_argument("--comm", default="torch", choices=["torch", "rccl", "oneshot", "auto"],
                    help="gradient all-reduce for the fused modes: ProcessGroup, or native (csrc/comm.hip)")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU; without torchrun this script launches them itself")
    a = ap.parse_args()
    from routest_amd.parallel.launch import ensure_ranks, share_gpu
    ensure_ranks(a.gpus, __file__)
    import torch
    import torch.distributed as dist
    from routest_amd.data.synth import synth_records, synth_trips
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.ops.eta_mlp import featurize_torch, records_to_tensor
    from routest_amd.parallel.dp import FlatGrads, allreduce_scalars, barrier, init_distributed
    from routest_amd.train.fused import FusedMlp3Trainer

    di = init_distributed()
    dev = di.device
    torch.manual_seed(0)
    xs, ys = synth_trips(65536, 12345)
    B = a.batch
    rec, y = synth_records(B, 100 + di.rank)
    rt = records_to_tensor(rec).to(dev)
    comm = None
    if a.comm != "torch" and di.world > 1:
        from routest_amd.parallel.comm import DeviceComm
        comm = DeviceComm(dev, use_rccl=not share_gpu())
        comm_algo = a.comm
    results = {}
    for mode in a.modes.split(","):
        m = EtaMLP(a.hidden)
        m.fit_normalization(xs, ys)
        yn = ((torch.from_numpy(y) - m.y_mean) / m.y_std).float().to(dev)
        if mode in ("fused", "graph"):
            tr = FusedMlp3Trainer(m, dev, B, B * di.world, lr=1e-3, allreduce=di.world > 1, comm=comm)
            if comm is not None and comm_algo != "auto":
                tr.comm = _Pinned(comm, comm_algo)
            step = lambda: tr.step(rt, yn)  # noqa: E731
            if mode == "graph":
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for _ in range(3):
                        tr.step(rt, yn)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                barrier(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    tr.step(rt, yn)
                step = g.replay
        else:
            m = m.to(dev)
            fg = FlatGrads(list(m.parameters()))
            opt = torch.optim.AdamW(m.parameters(), lr=1e-3, fused=True)

            def step():
                fg.zero()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    pred = m.forward_normalized(featurize_torch(rt))
                loss = torch.nn.functional.mse_loss(pred.float(), yn)
                loss.backward()
                fg.allreduce_avg()
                opt.step()
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        barrier(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        barrier(dev)
        torch.cuda.synchronize()
        el = allreduce_scalars([time.perf_counter() - t0], dev, op="max")[0]
        if a.trace and di.is_main:           # outside the timed region
            from routest_amd.utils.profiling import chrome_trace
            with chrome_trace(f"{a.trace}_{mode}.json"):
                for _ in range(3):
                    step()
        results[mode] = {"ms_per_step": el / a.steps * 1e3,
                         "samples_per_s": B * di.world * a.steps / el}
    if di.is_main:
        print(json.dumps({"metric": "ETA MLP DP training samples/s", "n_gpus": di.world,
                          "shared_gpu": share_gpu() and di.world > 1,
                          "batch_per_gpu": B, "hidden": a.hidden, "results": results}), flush=True)
    if di.world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
