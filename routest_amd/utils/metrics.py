"""Tiny thread-safe metrics registry rendered in Prometheus text format at ``/metrics``.

The reference has no metrics at all (``print()`` only).  We track request counts,
latency quantiles (p50/p99 via a bounded reservoir), batch-size histograms and GPU timings.
"""
from __future__ import annotations

import bisect
import threading
from collections import deque
from typing import Deque, Dict, List, Optional, Sequence, Tuple


class Counter:
    def __init__(self, name: str, help_: str):
        self.name, self.help = name, help_
        self._v: Dict[Tuple[Tuple[str, str], ...], float] = {}
        self._lock = threading.Lock()

    def inc(self, n: float = 1.0, **labels: str) -> None:
        key = tuple(sorted(labels.items()))
        with self._lock:
            self._v[key] = self._v.get(key, 0.0) + n

    def value(self, **labels: str) -> float:
        with self._lock:
            return self._v.get(tuple(sorted(labels.items())), 0.0)

    def render(self) -> List[str]:
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} counter"]
        with self._lock:
            for k, v in sorted(self._v.items()):
                lab = ",".join(f'{a}="{b}"' for a, b in k)
                out.append(f"{self.name}{{{lab}}} {v}" if lab else f"{self.name} {v}")
        return out


class Histogram:
    def __init__(self, name: str, help_: str, buckets: Sequence[float], reservoir: int = 4096):
        self.name, self.help = name, help_
        self.buckets = list(buckets)
        self._counts = [0] * (len(self.buckets) + 1)
        self._sum = 0.0
        self._n = 0
        self._recent: Deque[float] = deque(maxlen=reservoir)
        self._lock = threading.Lock()

    def observe(self, v: float) -> None:
        with self._lock:
            self._counts[bisect.bisect_left(self.buckets, v)] += 1
            self._sum += v
            self._n += 1
            self._recent.append(v)

    def quantile(self, q: float) -> Optional[float]:
        with self._lock:
            xs = sorted(self._recent)
        if not xs:
            return None
        i = min(len(xs) - 1, max(0, int(round(q * (len(xs) - 1)))))
        return xs[i]

    @property
    def count(self) -> int:
        return self._n

    def render(self) -> List[str]:
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} histogram"]
        with self._lock:
            acc = 0
            for b, c in zip(self.buckets, self._counts):
                acc += c
                out.append(f'{self.name}_bucket{{le="{b}"}} {acc}')
            acc += self._counts[-1]
            out.append(f'{self.name}_bucket{{le="+Inf"}} {acc}')
            out.append(f"{self.name}_sum {self._sum}")
            out.append(f"{self.name}_count {self._n}")
        for q in (0.5, 0.99):
            v = self.quantile(q)
            if v is not None:
                out.append(f'{self.name}_quantile{{q="{q}"}} {v}')
        return out


class Registry:
    def __init__(self) -> None:
        self.requests = Counter("routest_requests_total", "HTTP requests by route and status")
        self.preds = Counter("routest_eta_predictions_total", "ETA predictions served")
        self.latency = Histogram("routest_request_latency_seconds", "request latency",
                                 [1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 0.1, 1.0])
        self.batch = Histogram("routest_batch_size", "micro-batch sizes",
                               [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 4096, 16384, 65536])
        self.queue_wait = Histogram("routest_batch_queue_wait_seconds", "time in batch queue",
                                    [1e-5, 5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 5e-3, 1e-2])
        self.gpu_time = Histogram("routest_batch_device_seconds", "device time per batch",
                                  [1e-5, 2.5e-5, 5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 5e-3])

        self.device_failures = Counter("routest_device_failures_total", "batches that raised on a device")
        self.slow_batches = Counter("routest_slow_batches_total", "batches slower than the watchdog limit")
        self.route_batch = Histogram("routest_route_batch_size", "route requests per optimizer flush",
                                     [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 4096])
        self.route_flush_time = Histogram("routest_route_flush_seconds", "optimizer flush time (K5+K6+K9 + assembly)",
                                          [1e-4, 5e-4, 1e-3, 5e-3, 1e-2, 5e-2, 0.1, 0.5, 1.0])
        self.sse_dropped = Counter("routest_sse_dropped_total", "SSE messages dropped for slow subscribers")

    def render(self) -> str:
        lines: List[str] = []
        for m in (self.requests, self.preds, self.latency, self.batch, self.queue_wait, self.gpu_time,
                  self.device_failures, self.slow_batches, self.route_batch, self.route_flush_time,
                  self.sse_dropped):
            lines.extend(m.render())
        lines.extend(_device_gauges())
        return "\n".join(lines) + "\n"


def _device_gauges() -> List[str]:
    """HBM used/total per visible GPU (gauges; empty without a GPU)."""
    try:
        import torch
        if not torch.cuda.is_available():
            return []
        out = ["# HELP routest_gpu_hbm_bytes HBM per device", "# TYPE routest_gpu_hbm_bytes gauge"]
        for i in range(torch.cuda.device_count()):
            free, total = torch.cuda.mem_get_info(i)
            out.append(f'routest_gpu_hbm_bytes{{device="{i}",kind="used"}} {total - free}')
            out.append(f'routest_gpu_hbm_bytes{{device="{i}",kind="total"}} {total}')
        return out
    except Exception:  # pragma: no cover - metrics must never fail a scrape
        return []


REGISTRY = Registry()
