"""Live tracking: SSE pub/sub broker, payload formatter and drive simulator (R06-R08, R24-R26).

Reference: Flask-SSE publishes through Redis ``PUBLISH`` and streams with ``SUBSCRIBE``
(``RO/Flaskr/__init__.py:8,25,28``, ``routes.py:86``); the simulator thread POSTs every tick back
to its own ``/api/update_tracker`` over loopback HTTP with retries (``utils.py:206-251``).

Here the default broker is in-process (asyncio queues, thread-safe ``publish``), so a simulator
tick is a direct publish — no loopback HTTP, no Redis needed.  With ``ROUTEST_BROKER=redis`` and
``REDIS_URL`` set, :class:`RedisBroker` speaks Flask-SSE's Redis format through our own RESP client
(``realtime/redis_resp.py``), so several server processes — or this service and a reference Flask
deployment — share live-tracking channels.
The wire format is Flask-SSE's: ``data:<json>\\n\\n`` (default ``message`` event), which the
dashboard's ``EventSource.onmessage`` consumes (``FE/app/ui/page.jsx:598-650``).
"""
from __future__ import annotations

import asyncio
import datetime as dt
import json
import random
import threading
import time
from typing import Any, Dict, List, Optional, Set, Tuple

from ..utils.logging import get_logger
from ..utils.metrics import REGISTRY
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
        self.dropped = 0         # messages not queued because a subscriber was max_queue behind

    def publish(self, data: Any, channel: str = "sse", type_: Optional[str] = None) -> int:
        msg = sse_message(data, type_)
        with self._lock:
            subs = list(self._subs.get(str(channel), ()))
            self.published += 1
        for loop, q in subs:
            def _put(q=q, msg=msg, channel=channel):
                if q.qsize() < self.max_queue:
                    q.put_nowait(msg)
                else:
                    self.dropped += 1
                    REGISTRY.sse_dropped.inc()
                    if self.dropped & (self.dropped - 1) == 0:   # log at 1, 2, 4, 8, ... drops
                        log.warning("SSE subscriber on channel %r is %d messages behind: dropped "
                                    "(%d dropped so far)", channel, self.max_queue, self.dropped)
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


class RedisBroker:
    """Flask-SSE-compatible broker over Redis pub/sub: ``PUBLISH <channel> {"data":..,"type":..}``;
    each SSE stream holds its own ``SUBSCRIBE`` connection (an asyncio task feeding a queue)."""

    kind = "redis"

    def __init__(self, url: str, max_queue: int = 1024, timeout: float = 2.0):
        from .redis_resp import RespClient
        self.url = url
        self.client = RespClient(url, timeout=timeout)
        self.max_queue = max_queue
        self.published = 0
        self._subs: Dict[int, Tuple[str, Any]] = {}
        self._lock = threading.Lock()

    def publish(self, data: Any, channel: str = "sse", type_: Optional[str] = None) -> int:
        payload: Dict[str, Any] = {"data": data}
        if type_:
            payload["type"] = type_
        try:
            n = self.client.execute("PUBLISH", str(channel), json.dumps(payload))
        except Exception as e:  # best effort, like the reference's publish path
            log.warning("redis publish failed: %r", e)
            return 0
        self.published += 1
        return int(n or 0)

    def subscribe(self, channel: str) -> asyncio.Queue:
        from .redis_resp import subscribe_stream
        q: asyncio.Queue = asyncio.Queue()

        def on_message(raw: bytes) -> None:
            try:
                d = json.loads(raw)
                msg = sse_message(d.get("data"), d.get("type"), d.get("id"))
            except (ValueError, AttributeError):
                return
            if q.qsize() < self.max_queue:
                q.put_nowait(msg)

        async def run():
            try:
                await subscribe_stream(self.url, str(channel), on_message)
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.warning("redis subscribe(%s) ended: %r", channel, e)

        task = asyncio.get_running_loop().create_task(run())
        with self._lock:
            self._subs[id(q)] = (str(channel), task)
        return q

    def unsubscribe(self, channel: str, q: asyncio.Queue) -> None:
        with self._lock:
            item = self._subs.pop(id(q), None)
        if item is not None:
            item[1].cancel()

    def subscribers(self, channel: str) -> int:
        with self._lock:
            return sum(1 for ch, _ in self._subs.values() if ch == str(channel))

    def ping(self) -> Dict[str, Any]:
        t0 = time.time()
        try:
            ms = self.client.ping()
            return {"status": "ok", "latency_ms": int(ms), "kind": self.kind}
        except Exception as e:
            return {"status": "error", "latency_ms": int((time.time() - t0) * 1000), "kind": self.kind,
                    "error": str(e)[:200]}


def make_broker(kind: str, redis_url: Optional[str]):
    if kind == "redis":
        if redis_url:
            return RedisBroker(redis_url)
        log.warning("ROUTEST_BROKER=redis without REDIS_URL; using the in-process broker")
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
