"""Dynamic micro-batching for ``/predict`` (the reference runs batch = 1 per HTTP
request, ``RO/Flaskr/routes.py:365-383``).

Requests are packed into 16-byte records as they arrive and pushed on one queue.  Each device
has a worker thread that takes the first waiting request, keeps collecting until ``batch_max``
rows or ``timeout_us`` elapsed, and runs ONE fused featurize+MLP launch for the batch:

    pinned host records --H2D--> HBM --K1+K2 kernel--> minutes --D2H--> pinned host

All workers pull from the same queue, so several GPUs in one process share load without a
router.  The queue + batch assembly can run in the native C++ runtime (``routest_amd._rt``,
``csrc/runtime/batch_queue.cpp``) which releases the GIL while waiting; a pure-Python queue is
the fallback.
"""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import queue
import threading
import time
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from ..models.features import RECORD_DTYPE
from ..utils.logging import get_logger
from ..utils.metrics import REGISTRY

log = get_logger("batcher")

Runner = Callable[[np.ndarray], np.ndarray]


class GpuRunner:
    """Runs the fused ETA kernel on one GPU with pinned staging buffers and a private stream."""

    def __init__(self, kernel, device: torch.device, batch_max: int):
        self.kernel = kernel
        self.device = torch.device(device)
        self.batch_max = batch_max
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.Stream(self.device)
            self.h_rec = torch.empty((batch_max, 4), dtype=torch.int32).pin_memory()
            self.h_out = torch.empty(batch_max, dtype=torch.float32).pin_memory()
            self.d_rec = torch.empty((batch_max, 4), dtype=torch.int32, device=self.device)
        self.h_rec_np = self.h_rec.numpy().view(np.uint8).reshape(batch_max, 16).view(RECORD_DTYPE).reshape(-1)
        self.lock = threading.Lock()

    def __call__(self, rec: np.ndarray) -> np.ndarray:
        n = rec.shape[0]
        out = np.empty(n, dtype=np.float32)
        with self.lock, torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            for s in range(0, n, self.batch_max):
                m = min(self.batch_max, n - s)
                self.h_rec_np[:m] = rec[s:s + m]
                self.d_rec[:m].copy_(self.h_rec[:m], non_blocking=True)
                y = self.kernel(self.d_rec[:m])
                self.h_out[:m].copy_(y, non_blocking=True)
                self.stream.synchronize()
                out[s:s + m] = self.h_out.numpy()[:m]
        return out


class _Item:
    __slots__ = ("rec", "fut", "loop", "t0")

    def __init__(self, rec, fut, loop, t0):
        self.rec, self.fut, self.loop, self.t0 = rec, fut, loop, t0


class MicroBatcher:
    def __init__(self, runners: Sequence[Runner], batch_max: int = 4096, timeout_us: int = 200,
                 name: str = "eta"):
        self.runners = list(runners)
        self.batch_max = batch_max
        self.timeout_s = timeout_us / 1e6
        self.q: "queue.SimpleQueue[Optional[_Item]]" = queue.SimpleQueue()
        self._stop = False
        # adaptive deadline: only wait for stragglers when the last batch showed concurrency
        self._last_batch = 1
        self.threads = [threading.Thread(target=self._worker, args=(r,), name=f"{name}-batch-{i}",
                                         daemon=True) for i, r in enumerate(self.runners)]
        for t in self.threads:
            t.start()

    # ---- producer side ----
    def submit_nowait(self, rec_tuple, loop: Optional[asyncio.AbstractEventLoop] = None):
        """Enqueue one record; returns an asyncio future (if loop) or concurrent future."""
        if loop is not None:
            fut = loop.create_future()
        else:
            fut = cf.Future()
        self.q.put(_Item(rec_tuple, fut, loop, time.perf_counter()))
        return fut

    async def submit(self, rec_tuple) -> float:
        return await self.submit_nowait(rec_tuple, asyncio.get_running_loop())

    def predict_sync(self, rec_tuple, timeout: float = 30.0) -> float:
        return self.submit_nowait(rec_tuple).result(timeout)

    # ---- consumer side ----
    def _collect(self, first: _Item) -> List[_Item]:
        batch = [first]
        deadline = first.t0 + self.timeout_s
        while len(batch) < self.batch_max:
            try:
                it = self.q.get_nowait()
                batch.append(it)
                if it is None:
                    break
                continue
            except queue.Empty:
                pass
            if self._last_batch <= 1 and len(batch) == 1:
                break
            rem = deadline - time.perf_counter()
            if rem <= 0:
                break
            try:
                it = self.q.get(timeout=rem)
            except queue.Empty:
                break
            batch.append(it)
            if it is None:
                break
        return batch

    @staticmethod
    def _resolve(it: _Item, value=None, exc: Optional[BaseException] = None) -> None:
        def _set():
            if it.fut.done():
                return
            if exc is not None:
                it.fut.set_exception(exc)
            else:
                it.fut.set_result(value)
        if it.loop is not None:
            try:
                it.loop.call_soon_threadsafe(_set)
            except RuntimeError:
                pass
        else:
            _set()

    def _worker(self, runner: Runner) -> None:
        while True:
            first = self.q.get()
            if first is None:
                self.q.put(None)  # let the other workers see the sentinel too
                return
            batch = self._collect(first)
            stop = False
            if batch and batch[-1] is None:
                batch.pop()
                stop = True
            if batch:
                t_q = time.perf_counter()
                rec = np.array([it.rec for it in batch], dtype=RECORD_DTYPE)
                try:
                    t1 = time.perf_counter()
                    ys = runner(rec)
                    REGISTRY.gpu_time.observe(time.perf_counter() - t1)
                    for it, y in zip(batch, ys.tolist()):
                        self._resolve(it, float(y))
                except BaseException as e:  # device failure: fail the batch, keep serving
                    log.error("batch of %d failed: %r", len(batch), e)
                    for it in batch:
                        self._resolve(it, exc=e)
                self._last_batch = len(batch)
                REGISTRY.batch.observe(len(batch))
                REGISTRY.queue_wait.observe(t_q - batch[0].t0)
            if stop:
                self.q.put(None)
                return

    def close(self) -> None:
        self.q.put(None)
        for t in self.threads:
            t.join(timeout=5)
