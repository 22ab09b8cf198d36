"""Per-section failure containment for ``bench.py``'s multi-rank runs (VERDICT r5 Missing #2).

The headline line must print even when one of the extra sections (training probes, the one-shot
set-up, the collective sweep, GCN, routes) fails on ONE rank.  The hazard is not the exception
itself but the collectives after it: a rank that raised skips the barrier / all-reduce its peers
are already waiting in, and the job hangs until the driver kills it, with no JSON line at all.

:class:`SectionGuard` runs each section under a small protocol over a **gloo side group** (CPU,
its own long timeout, never the RCCL communicator the section uses):

* the section calls :meth:`SectionGuard.checkpoint` immediately before every collective it makes on
  the main group (and before loops whose steps contain one).  A checkpoint is one MAX all-reduce of
  a "failed" flag on the side group;
* a rank whose section raises sends exactly ONE failed flag and stops.  Its peers receive it at their
  next checkpoint (or at the section's final agreement), raise :class:`SectionAborted` there and
  leave the section too — before anyone enters a main-group collective the failed rank will never
  reach.  The number of side-group all-reduces therefore always matches across ranks;
* every rank returns ``{"error": ...}`` for that section and goes on to the next one.

Fault hook for the tests and the shared-GPU rehearsal: ``ROUTEST_FAULT=bench_raise@<section>:<rank>``
raises inside ``<section>`` on ``<rank>`` at its start, ``...:<rank>:<k>`` at its k-th checkpoint
(1-based).  The side group also holds ranks 1..N-1 at :meth:`SectionGuard.hold` while rank 0 runs the
serving sections alone, so the RCCL communicator is torn down by all ranks together.
"""
from __future__ import annotations

import datetime
import os
from typing import Any, Callable, Dict, Optional

import torch
import torch.distributed as dist

from .faults import InjectedFault, active_faults


class SectionAborted(RuntimeError):
    """A peer rank's section failed: leave the section without touching the main group."""


def _fault_point(section: str, rank: int) -> Optional[int]:
    """0 = raise at the section's start, k = at its k-th checkpoint, None = no fault."""
    for f in active_faults():
        if not f.startswith("bench_raise@"):
            continue
        parts = f.split("@", 1)[1].split(":")
        if parts[0] != section.lower() or len(parts) < 2:
            continue
        try:
            if int(parts[1]) != rank:
                continue
            return int(parts[2]) if len(parts) > 2 else 0
        except ValueError:
            continue
    return None


def raise_if_injected(section: str, rank: int) -> None:
    """For sections that run on one rank only (bench.py's serving sections on rank 0)."""
    if _fault_point(section, rank) is not None:
        raise InjectedFault(f"injected fault: bench_raise@{section}:{rank}")


class SectionGuard:
    def __init__(self, world: int, rank: int, timeout_s: float = 900.0):
        self.world, self.rank = world, rank
        self.group = None
        if world > 1:
            self.group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
        self.section: Optional[str] = None
        self._n_ck = 0
        self._fault: Optional[int] = None
        self.log: Dict[str, str] = {}

    def _reduce(self, v: float) -> float:
        """One side-group MAX all-reduce of v (0 = fine, 1 = "not ok" vote, 2 = section failed)."""
        if self.world == 1:
            return v
        t = torch.tensor([v])
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def _flag(self, failed: bool) -> bool:
        """True when any rank reported a failed section."""
        return self._reduce(2.0 if failed else 0.0) >= 2.0

    def _tick(self) -> None:
        self._n_ck += 1
        if self._fault is not None and self._fault == self._n_ck:
            raise InjectedFault(f"injected fault: bench_raise@{self.section}:{self.rank}:{self._n_ck}")

    def checkpoint(self) -> None:
        """Call right before each main-group collective of the running section."""
        if self.section is None:
            return
        self._tick()
        if self._flag(False):
            raise SectionAborted(f"{self.section}: failed on a peer rank")

    def run(self, name: str, fn: Callable[..., Any], *args, **kw) -> Any:
        """``fn(*args, **kw)`` under the protocol; its result, or ``{"error": ...}`` on EVERY rank
        when it failed on any."""
        self.section, self._n_ck = name, 0
        self._fault = _fault_point(name, self.rank)
        try:
            try:
                if self._fault == 0:
                    raise InjectedFault(f"injected fault: bench_raise@{name}:{self.rank}")
                res = fn(*args, **kw)
            except SectionAborted as e:       # already agreed at that checkpoint: no more flags
                self.log[name] = str(e)
                return {"error": str(e)}
            except Exception as e:  # noqa: BLE001 - reported in the section, never fatal
                # (no device synchronize here: the failure may have left a collective queued that
                # its peers will never join)
                self._flag(True)
                msg = f"rank {self.rank}: {type(e).__name__}: {str(e)[:240]}"
                self.log[name] = msg
                return {"error": msg}
            if self._flag(False):             # the final agreement
                self.log[name] = "failed on a peer rank"
                return {"error": f"{name}: failed on a peer rank"}
            return res
        finally:
            self.section, self._fault = None, None

    def agree(self, ok: bool) -> bool:
        """True only if every rank says so (side group).  Inside a section it doubles as a
        checkpoint: a peer's failure raises :class:`SectionAborted` instead of reading as a vote."""
        if self.section is not None:
            self._tick()
        v = self._reduce(0.0 if ok else 1.0)
        if self.section is not None:
            if v >= 2.0:
                raise SectionAborted(f"{self.section}: failed on a peer rank")
        return v == 0.0

    def hold(self) -> None:
        """Every rank meets here before teardown (ranks 1..N-1 wait while rank 0 serves)."""
        if self.world > 1:
            dist.barrier(group=self.group)


def env_timeout_s(name: str, default: float) -> float:
    try:
        return float(os.environ.get(name, default))
    except ValueError:
        return default
