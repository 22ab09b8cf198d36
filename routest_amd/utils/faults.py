"""Fault-injection hooks.  ``ROUTEST_FAULT`` is a comma list of
``provider_timeout``, ``gpu_fail``, ``rccl_timeout``, ``store_fail``; tests flip them with
:func:`set_faults` instead of the env var."""
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
