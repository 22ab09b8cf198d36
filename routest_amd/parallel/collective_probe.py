"""Short collective sweep over the live process group: latency and bus bandwidth of
RCCL all-reduce / all-gather at the message sizes this framework issues, plus the native one-shot
xGMI all-reduce of ``csrc/comm.hip`` where it applies.

``bench.py`` runs it after its timed region whenever it has >1 rank on separate GPUs, so every
multi-GPU run of the headline also records what the links delivered (extra JSON key
``collectives``); ``bench/rccl_bench.py`` is the long form with environment knob sweeps.

Bus bandwidth follows the nccl-tests convention: all_reduce busbw = algbw * 2(n-1)/n,
all_gather busbw = algbw * (n-1)/n.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

# the H = 256 gradient bucket (74,000 fp32), the H = 1024 bucket (~4.3 MB), the GCN all-gather
# (25.6 MB at 100k nodes x 128 bf16) and two bandwidth-regime sizes
DEFAULT_SIZES = (296_000, 4_300_000, 25_600_000, 64 << 20, 256 << 20)


def _time(fn, iters: int, warm: int = 3, device: Optional[torch.device] = None) -> float:
    cuda = device is None or device.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    for _ in range(warm):
        fn()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    sync()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float64, device=torch.cuda.current_device() if cuda else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sweep(device: torch.device, sizes: Sequence[int] = DEFAULT_SIZES,
          native: Optional[object] = None, checkpoint: Optional[Callable[[], None]] = None) -> List[Dict]:
    """All ranks call this together with the same arguments; every decision below depends on
    those arguments only (never on local timing), so no rank can leave the others waiting in a
    collective.  Returns the same rows on every rank (times are the max over ranks).
    ``checkpoint`` (bench.py's SectionGuard) runs before each size's collectives, so a rank that
    failed is noticed by its peers before they enter the next all-reduce it will never reach."""
    n = dist.get_world_size()
    rows: List[Dict] = []
    for nbytes in sizes:
        if checkpoint is not None:
            checkpoint()
        iters = 20 if nbytes <= (4 << 20) else 5
        numel = (nbytes // 4 + 3) // 4 * 4
        x = torch.ones(numel, device=device)
        cases = [("all_reduce", lambda: dist.all_reduce(x), 2 * (n - 1) / n)]
        per = max(1, numel // n)
        xs = torch.ones(per, device=device)
        out = torch.empty(per * n, device=device)
        cases.append(("all_gather", lambda: dist.all_gather_into_tensor(out, xs), (n - 1) / n))
        if native is not None and getattr(native, "oneshot", False) and nbytes <= getattr(native, "oneshot_bytes", 0):
            cases.append(("all_reduce_oneshot", lambda: native.all_reduce(x, "oneshot"), 2 * (n - 1) / n))
        for op, fn, factor in cases:
            dt = _time(fn, iters, device=device)
            moved = nbytes if op != "all_gather" else per * n * 4
            algbw = moved / dt / 1e9
            rows.append({"op": op, "bytes": moved, "us": round(dt * 1e6, 2),
                         "algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * factor, 2)})
        del x, xs, out
    return rows
