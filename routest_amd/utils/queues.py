"""Queue helpers for the micro-batchers (serve/batcher.py, routing/route_batcher.py).

Both batchers have several consumer threads (one per GPU) on ONE ``queue.SimpleQueue`` and collect a
batch until a deadline.  CPython 3.10's timed ``SimpleQueue.get(timeout=...)`` is unsafe with more
than one consumer: when a put wakes a waiting consumer but another consumer takes the item first,
the woken one re-waits with its remaining timeout recomputed — and once that is negative the re-wait
has no timeout at all, so the consumer sleeps (holding the requests it already collected) until the
next put, which under a finished burst never comes.  Reproduced with two fake runners on CPU
(tests/test_batcher_cpu.py: items lost within ~10 rounds of 6000 concurrent requests).
:func:`get_until` polls instead: non-blocking gets with short sleeps, never past the deadline.
"""
from __future__ import annotations

import queue
import time

_POLL_S = 50e-6


def get_until(q: "queue.SimpleQueue", deadline: float):
    """Next item, or ``queue.Empty`` once ``time.perf_counter()`` passes ``deadline``."""
    while True:
        try:
            return q.get_nowait()
        except queue.Empty:
            pass
        rem = deadline - time.perf_counter()
        if rem <= 0:
            raise queue.Empty
        time.sleep(rem if rem < _POLL_S else _POLL_S)
