#!/usr/bin/env python3
"""RCCL all-reduce / all-gather latency and bus bandwidth vs message size over xGMI.

    torchrun --standalone --nproc-per-node 8 bench/rccl_bench.py

Bus bandwidth follows the nccl-tests convention: all_reduce busbw = algbw * 2 (n-1)/n,
all_gather busbw = algbw * (n-1)/n.  The ETA-MLP gradient bucket (74,000 fp32 at H=256 = 296 KB)
is marked: it sits deep in the latency regime, which is why training issues exactly one
collective per step.  With >1 rank the native paths of ``csrc/comm.hip`` are measured too: our own
RCCL communicator called from C++ and the one-shot xGMI peer-read all-reduce.  Sweep RCCL knobs from the environment (NCCL_ALGO, NCCL_PROTO,
NCCL_MIN_NCHANNELS) — they are read by RCCL at init."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch
    import torch.distributed as dist
    from routest_amd.parallel.dp import init_distributed

    di = init_distributed()
    dev = di.device
    n = di.world
    sizes = [4 << 10, 64 << 10, 296_000, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20]
    native = None
    if n > 1:
        from routest_amd.parallel.comm import DeviceComm
        native = DeviceComm(dev, oneshot_bytes=8 << 20)
    rows = []
    for nbytes in sizes:
        ops = ["all_reduce", "all_gather"]
        if native is not None:
            ops.append("all_reduce_native_rccl")
            if native.oneshot and nbytes <= (8 << 20):
                ops.append("all_reduce_oneshot")
        for op in ops:
            numel = nbytes // 4
            if op == "all_gather":
                numel = max(1, numel // max(1, n))
                x = torch.ones(numel, device=dev)
                out = torch.empty(numel * n, device=dev)
                fn = lambda: dist.all_gather_into_tensor(out, x) if n > 1 else out[:numel].copy_(x)  # noqa
            elif op == "all_reduce_native_rccl":
                x = torch.ones(numel, device=dev)
                fn = lambda: native.all_reduce(x, "rccl")  # noqa
            elif op == "all_reduce_oneshot":
                x = torch.ones((numel + 3) // 4 * 4, device=dev)
                fn = lambda: native.all_reduce(x, "oneshot")  # noqa
            else:
                x = torch.ones(numel, device=dev)
                fn = lambda: dist.all_reduce(x) if n > 1 else x.mul_(1.0)  # noqa
            iters = 50 if nbytes <= (4 << 20) else 10
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            algbw = nbytes / dt / 1e9
            factor = (2 * (n - 1) / n) if op.startswith("all_reduce") else ((n - 1) / n)
            rows.append({"op": op, "bytes": nbytes, "us": dt * 1e6, "algbw_GBps": algbw,
                         "busbw_GBps": algbw * factor if n > 1 else None,
                         "note": "ETA-MLP grad bucket" if nbytes == 296_000 else ""})
    if di.is_main:
        print(json.dumps({"metric": "RCCL collectives", "n_gpus": n, "env": {k: os.environ.get(k) for k in
                          ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS")}, "rows": rows}), flush=True)
    if native is not None:
        native.check()
        native.close()
    if n > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
