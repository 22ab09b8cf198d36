"""Tracing / profiling helpers (the reference has none beyond health-probe latencies).

* :func:`chrome_trace` — ``torch.profiler`` with CPU + HIP activities around a block, exported as a
  Chrome trace (``chrome://tracing`` / Perfetto).  On ROCm the "CUDA" activity is HIP (roctracer).
* :class:`HipTimer` — hipEvent-based device timer for a stream region (no host sync until read).
* :func:`apply_debug_env` — kernel-serialising debug modes (``AMD_SERIALIZE_KERNEL=3``,
  ``HIP_LAUNCH_BLOCKING=1``), enabled by ``ROUTEST_DEBUG_SYNC=1``; must run before HIP initialises.

Kernel-level numbers come from rocprofv3 (``bench/profile_eta.sh``, ``bench/profile_kernels.sh``).
"""
from __future__ import annotations

import contextlib
import os
from typing import Iterator, Optional


def apply_debug_env(environ=os.environ) -> bool:
    """Serialise every kernel launch and make launch errors synchronous (debugging only)."""
    if environ.get("ROUTEST_DEBUG_SYNC", "") not in ("1", "true", "yes"):
        return False
    environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
    environ.setdefault("AMD_SERIALIZE_COPY", "3")
    environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
    return True


@contextlib.contextmanager
def chrome_trace(path: Optional[str], record_shapes: bool = False) -> Iterator[None]:
    """Profile the enclosed block and write a Chrome trace to ``path`` (no-op when path is falsy)."""
    if not path:
        yield
        return
    import torch
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts, record_shapes=record_shapes) as prof:
        yield
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    prof.export_chrome_trace(path)


class HipTimer:
    """``with HipTimer() as t: ...`` then ``t.ms`` (synchronises on read)."""

    def __init__(self, stream=None):
        import torch
        self.stream = stream
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e1 = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.e0.record(self.stream)
        return self

    def __exit__(self, *exc):
        self.e1.record(self.stream)
        return False

    @property
    def ms(self) -> float:
        self.e1.synchronize()
        return self.e0.elapsed_time(self.e1)
