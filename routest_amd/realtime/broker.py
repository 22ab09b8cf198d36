"""Live tracking: SSE pub/sub broker, payload formatter and drive simulator (R06-R08, R24-R26).

Reference: Flask-SSE publishes through Redis ``PUBLISH`` and streams with ``SUBSCRIBE``
(``RO/Flaskr/__init__.py:8,25,28``, ``routes.py:86``); the simulator thread POSTs every tick back
to its own ``/api/update_tracker`` over loopback HTTP with retries (``utils.py:206-251``).

Here the broker is in-process (asyncio queues, thread-safe ``publish``), so a simulator tick is a
direct publish — no loopback HTTP, no Redis needed.  A Redis broker is used instead when
``ROUTEST_BROKER=redis`` and the ``redis`` module is importable (not in this image).
The wire format is Flask-SSE's: ``data:<json>\\n\\n`` (default ``message`` event), which the
dashboard's ``EventSource.onmessage`` consumes (``FE/app/ui/page.jsx:598-650``).
"""
from __future__ import annotations

import asyncio
import datetime as dt
import json
import random
import threading
from typing import Any, Dict, List, Optional, Set, Tuple

from ..utils.logging import get_logger
from ..utils.timeutil import parse_iso

log = get_logger("realtime")


def format_sse_data(data: Dict[str, Any]) -> Dict[str, Any]:
    """R26 (utils.py:253-267)."""
    pickup = parse_iso(data["pickup_time"])
    completion = pickup + dt.timedelta(seconds=float(data["duration"]))
    return {
        "destinations": data["destinations"],
        "remaining_routes": data["route"],
        "overall_duration": data["duration"],
        "overall_travel_distance": data["distance"],
        "overall_estimated_completion_time": completion.isoformat(),
        "total_trips": data.get("trips", 1),
        "assigned_driver": data["driver_name"],
        "transport_mode": data["vehicle_type"],
        "start_time": data["pickup_time"],
    }


def sse_message(data: Any, type_: Optional[str] = None, id_: Optional[str] = None) -> str:
    lines = []
    if type_:
        lines.append(f"event:{type_}")
    if id_:
        lines.append(f"id:{id_}")
    for ln in json.dumps(data).splitlines() or [""]:
        lines.append(f"data:{ln}")
    return "\n".join(lines) + "\n\n"


class MemoryBroker:
    kind = "memory"

    def __init__(self, max_queue: int = 1024):
        self._subs: Dict[str, Set[Tuple[asyncio.AbstractEventLoop, asyncio.Queue]]] = {}
        self._lock = threading.Lock()
        self.max_queue = max_queue
        self.published = 0

    def publish(self, data: Any, channel: str = "sse", type_: Optional[str] = None) -> int:
        msg = sse_message(data, type_)
        with self._lock:
            subs = list(self._subs.get(str(channel), ()))
            self.published += 1
        for loop, q in subs:
            def _put(q=q, msg=msg):
                if q.qsize() < self.max_queue:
                    q.put_nowait(msg)
            try:
                loop.call_soon_threadsafe(_put)
            except RuntimeError:  # loop closed
                pass
        return len(subs)

    def subscribe(self, channel: str) -> asyncio.Queue:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        with self._lock:
            self._subs.setdefault(str(channel), set()).add((loop, q))
        return q

    def unsubscribe(self, channel: str, q: asyncio.Queue) -> None:
        with self._lock:
            s = self._subs.get(str(channel))
            if s:
                for item in list(s):
                    if item[1] is q:
                        s.discard(item)
                if not s:
                    self._subs.pop(str(channel), None)

    def subscribers(self, channel: str) -> int:
        with self._lock:
            return len(self._subs.get(str(channel), ()))

    def ping(self) -> Dict[str, Any]:
        return {"status": "ok", "latency_ms": 0, "kind": self.kind}


def make_broker(kind: str, redis_url: Optional[str]):
    if kind == "redis" and redis_url:
        try:
            import redis  # noqa: F401
        except ImportError:
            log.warning("redis module not available; using the in-process broker")
    return MemoryBroker()


class Simulator:
    """Bounded async drive simulator (R24).  Each tick publishes the R26 payload for the whole
    remaining route on channel ``driver_name``, pops the first point, sleeps U(tmin, tmax)."""

    def __init__(self, broker: MemoryBroker, tick_min: float = 2.0, tick_max: float = 5.0,
                 max_active: int = 256, delta: bool = False):
        self.broker = broker
        self.tick_min, self.tick_max = tick_min, tick_max
        self.max_active = max_active
        self.delta = delta
        self._tasks: Set[asyncio.Task] = set()

    @property
    def active(self) -> int:
        return len(self._tasks)

    def start(self, data: Dict[str, Any]) -> bool:
        if self.active >= self.max_active:
            return False
        t = asyncio.get_running_loop().create_task(self._run(data))
        self._tasks.add(t)
        t.add_done_callback(self._tasks.discard)
        return True

    def payloads(self, data: Dict[str, Any], pickup: Optional[dt.datetime] = None) -> List[Dict[str, Any]]:
        """All tick payloads (R24's url_data) — used by tests and by :meth:`_run`."""
        pickup = pickup or dt.datetime.now()
        rd = data["route_details"]
        drv = data["driver_details"]
        pts = list(rd["geometry"]["coordinates"])
        summ = rd["properties"]["summary"]
        out = []
        while pts:
            out.append({
                "route_id": drv["driver_name"], "route": list(pts) if not self.delta else pts[:2],
                "destinations": rd["properties"]["destinations"], "driver_name": drv["driver_name"],
                "vehicle_type": drv["vehicle_type"], "duration": summ["duration"],
                "distance": summ["distance"], "trips": summ.get("trips", 1),
                "pickup_time": pickup.isoformat(),
            })
            if self.delta:
                out[-1]["remaining_count"] = len(pts)
            pts.pop(0)
        return out

    async def _run(self, data: Dict[str, Any]) -> None:
        try:
            for p in self.payloads(data):
                msg = format_sse_data(p)
                if "remaining_count" in p:
                    msg["remaining_count"] = p["remaining_count"]
                self.broker.publish(msg, channel=str(p["route_id"]))
                await asyncio.sleep(random.uniform(self.tick_min, self.tick_max))
        except asyncio.CancelledError:
            raise
        except Exception as e:  # bad payloads: the reference's thread would die silently
            log.warning("simulation aborted: %r", e)

    async def shutdown(self) -> None:
        for t in list(self._tasks):
            t.cancel()
        for t in list(self._tasks):
            try:
                await t
            except BaseException:
                pass
