"""Time helpers shared by the ETA feature path and the SSE formatter.

The reference parses ``pickup_time`` with ``datetime.fromisoformat`` on Python 3.12
(``RO/Flaskr/ml.py:28-33``, ``RO/Flaskr/utils.py:255``; ``RO/runtime.txt:1``).  Python 3.10's
``fromisoformat`` rejects a trailing ``Z`` and non-3/6-digit fractions, so we parse
tolerantly.  Features use the *wall-clock fields as written* (``dt.weekday()``, ``dt.hour``), never
a timezone conversion, exactly like the reference.
"""
from __future__ import annotations

import calendar
import datetime as dt
import re
from typing import Any

_FRAC_RE = re.compile(r"(\.\d+)")

#: Kernel epoch: wall-clock seconds are stored relative to this naive instant (int32 range covers
#: 1952..2088).  2020-01-01 was a Wednesday (weekday()==2).
KERNEL_EPOCH = dt.datetime(2020, 1, 1)
KERNEL_EPOCH_WEEKDAY = 2
_KERNEL_EPOCH_TS = calendar.timegm(KERNEL_EPOCH.timetuple())


def parse_iso(s: str) -> dt.datetime:
    """``fromisoformat`` with 3.12-like leniency (``Z`` suffix, 1-9 digit fractions, space sep)."""
    t = s.strip()
    if t.endswith(("Z", "z")):
        t = t[:-1] + "+00:00"
    m = _FRAC_RE.search(t)
    if m:
        frac = m.group(1)[1:]
        frac = (frac + "000000")[:6]
        t = t[: m.start()] + "." + frac + t[m.end():]
    return dt.datetime.fromisoformat(t)


def coerce_pickup(pickup_time: Any) -> dt.datetime:
    """Reference semantics (ml.py:28-33): ISO str -> parsed; datetime -> itself; else now()."""
    if isinstance(pickup_time, str):
        return parse_iso(pickup_time)
    if isinstance(pickup_time, dt.datetime):
        return pickup_time
    return dt.datetime.now()


def wallclock_seconds(d: dt.datetime) -> int:
    """Seconds of the *wall-clock* fields since KERNEL_EPOCH (tz ignored, like weekday()/hour)."""
    return calendar.timegm(d.replace(tzinfo=None).timetuple()) - _KERNEL_EPOCH_TS


def weekday_hour_from_seconds(secs: int):
    """Inverse used by the kernels: weekday (Mon=0) and hour from KERNEL_EPOCH-relative seconds."""
    days = secs // 86400
    sod = secs - days * 86400
    return (days + KERNEL_EPOCH_WEEKDAY) % 7, sod // 3600
