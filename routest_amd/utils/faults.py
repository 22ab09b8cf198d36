"""Fault-injection hooks.  ``ROUTEST_FAULT`` is a comma list of
``provider_timeout``, ``gpu_fail``, ``rccl_timeout``, ``store_fail`` and ``rank_crash@<step>`` (the
last rank of a training job dies hard at that step on the job's FIRST attempt, so a
``torchrun --max-restarts`` relaunch resumes from the last checkpoint and finishes); tests flip them
with :func:`set_faults` instead of the env var."""
from __future__ import annotations

import os
import threading
from typing import Optional, Set

_lock = threading.Lock()
_override: Optional[Set[str]] = None


class InjectedFault(RuntimeError):
    pass


def active_faults() -> Set[str]:
    with _lock:
        if _override is not None:
            return set(_override)
    raw = os.environ.get("ROUTEST_FAULT", "")
    return {x.strip().lower() for x in raw.split(",") if x.strip()}


def set_faults(*names: str) -> None:
    global _override
    with _lock:
        _override = {n.lower() for n in names}


def clear_faults() -> None:
    global _override
    with _lock:
        _override = None


def maybe_fail(name: str) -> None:
    if name in active_faults():
        raise InjectedFault(f"injected fault: {name}")


def fault_step(name: str) -> Optional[int]:
    """``name@N`` in the active faults -> N (else None)."""
    for f in active_faults():
        if f.startswith(name + "@"):
            try:
                return int(f.split("@", 1)[1])
            except ValueError:
                return None
    return None
