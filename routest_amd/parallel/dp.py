"""Data parallelism over RCCL (xGMI) — or Gloo on CPU for tests.

One process per GPU (``torchrun --nproc-per-node N``), rank i pinned to GPU ``LOCAL_RANK``.
Backend ``"nccl"`` *is* RCCL on ROCm.  The ETA MLP's whole gradient is one flat fp32 bucket
(H=256: 69,904 floats = 280 KB), far inside the latency regime of an xGMI ring, so each step issues
exactly ONE ``all_reduce`` on it (C1) — DDP-style 25 MB bucketing would only add launches.  For
much larger models :func:`bucket_slices` splits a flat buffer into a few buckets so reductions can
be issued while later gradients are still being produced.

Also: initial-weight broadcast (C2), scalar metric all-reduce (C3), barrier (C5), and the env
knobs for failure handling (``TORCH_NCCL_ASYNC_ERROR_HANDLING``, collective timeout).
"""
from __future__ import annotations

import datetime as dt
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..utils.faults import maybe_fail


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: Optional[str] = None, timeout_s: float = 300.0) -> DistInfo:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).  No-op for 1 rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # 1-GPU rehearsal (parallel/launch.py): every rank on GPU 0, gloo rendezvous
    share = os.environ.get("ROUTEST_BENCH_SHARE_GPU") == "1"
    use_gpu = torch.cuda.is_available() and (backend != "gloo" or share)
    device = torch.device("cuda", 0 if share else local) if use_gpu else torch.device("cpu")
    if share:
        backend = "gloo"
    if use_gpu:
        torch.cuda.set_device(device)
    if world <= 1:
        return DistInfo(0, 1, 0, "none", device)
    be = backend or ("nccl" if use_gpu else "gloo")
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        kw = {"backend": be, "timeout": dt.timedelta(seconds=timeout_s)}
        if be == "nccl":
            kw["device_id"] = device
        restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0)
        if restart > 0 and "MASTER_PORT" in os.environ:
            # a `torchrun --max-restarts` relaunch with a static rendezvous re-uses the agent's store:
            # the previous attempt's connection keys are still in it (a rank can read a dead peer's
            # address and fail connectFullMesh), so every attempt gets its own key prefix
            agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                                 is_master=(not agent and rank == 0),
                                 timeout=dt.timedelta(seconds=timeout_s), multi_tenant=not agent)
            kw.update(store=dist.PrefixStore(f"routest/attempt_{restart}", base), rank=rank,
                      world_size=world)
        dist.init_process_group(**kw)
    return DistInfo(dist.get_rank(), dist.get_world_size(), local, be, device)


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def allreduce_flat(buf: torch.Tensor, average: bool = False, group=None) -> torch.Tensor:
    """ONE collective on a contiguous flat bucket (in place)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return buf
    maybe_fail("rccl_timeout")
    if average:
        if buf.is_cuda:
            dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group)
        else:  # gloo has no AVG
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
            buf.div_(dist.get_world_size(group))
    else:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def broadcast_flat(buf: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(buf, src=src, group=group)
    return buf


def _gloo() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo"


def allreduce_scalars(vals: Sequence[float], device: torch.device, op: str = "sum") -> List[float]:
    t = torch.tensor(list(vals), dtype=torch.float64, device="cpu" if _gloo() else device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                               "min": dist.ReduceOp.MIN}[op])
    return t.tolist()


def barrier(device: Optional[torch.device] = None) -> None:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and device.type == "cuda" and not _gloo():
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def bucket_slices(numel: int, bucket_bytes: int = 64 << 20, elem_bytes: int = 4) -> List[Tuple[int, int]]:
    """Split a flat buffer into buckets of at most ``bucket_bytes`` (default 64 MB: with 288 GB HBM
    per GPU memory is never the constraint; buckets exist only to overlap with backward)."""
    per = max(1, bucket_bytes // elem_bytes)
    return [(s, min(numel, s + per)) for s in range(0, numel, per)]


class FlatGrads:
    """Make every parameter's ``.grad`` a view into ONE flat buffer (autograd / CPU path), so the
    reduction is a single collective on contiguous memory."""

    def __init__(self, params: Sequence[torch.nn.Parameter]):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.buf = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.buf[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero(self) -> None:
        self.buf.zero_()

    def allreduce_avg(self) -> None:
        allreduce_flat(self.buf, average=True)
