"""Minimal Redis client (RESP2 over TCP/TLS) for the SSE broker — the ``redis`` package is not in
this image, and the broker needs only PING / PUBLISH / SUBSCRIBE.

Wire compatibility with Flask-SSE (the reference's SSE layer, ``RO/Flaskr/__init__.py:8,25,28``):
``sse.publish(data, type=None, channel=...)`` does ``PUBLISH <channel> <json>`` where the JSON is
``{"data": ..., "type": ...}`` (keys only when set), and its stream endpoint ``SUBSCRIBE``s and
renders each message as an SSE event.  :class:`RedisBroker` (realtime/broker.py) publishes and
consumes exactly that format, so this service and a reference Flask deployment can share one Redis.
"""
from __future__ import annotations

import asyncio
import socket
import ssl
import threading
import time
from typing import Any, List, Optional, Tuple
from urllib.parse import unquote, urlparse


class RedisError(RuntimeError):
    pass


def parse_url(url: str) -> Tuple[str, int, Optional[str], Optional[str], int, bool]:
    u = urlparse(url)
    if u.scheme not in ("redis", "rediss"):
        raise ValueError(f"unsupported Redis URL scheme {u.scheme!r}")
    db = int((u.path or "/0").lstrip("/") or 0)
    return (u.hostname or "127.0.0.1", u.port or 6379, unquote(u.username) if u.username else None,
            unquote(u.password) if u.password else None, db, u.scheme == "rediss")


def encode(*args: Any) -> bytes:
    out = [b"*%d\r\n" % len(args)]
    for a in args:
        b = a if isinstance(a, bytes) else str(a).encode()
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


class _Reader:
    """Incremental RESP2 reply parser over a byte source ``read(n) -> bytes``."""

    def __init__(self, read):
        self._read = read
        self._buf = b""

    def _line(self) -> bytes:
        while b"\r\n" not in self._buf:
            chunk = self._read(65536)
            if not chunk:
                raise RedisError("connection closed")
            self._buf += chunk
        line, self._buf = self._buf.split(b"\r\n", 1)
        return line

    def _exact(self, n: int) -> bytes:
        while len(self._buf) < n + 2:
            chunk = self._read(65536)
            if not chunk:
                raise RedisError("connection closed")
            self._buf += chunk
        data, self._buf = self._buf[:n], self._buf[n + 2:]
        return data

    def reply(self) -> Any:
        line = self._line()
        t, rest = line[:1], line[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RedisError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self._exact(n)
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self.reply() for _ in range(n)]
        raise RedisError(f"bad RESP type {t!r}")


class _Conn:
    __slots__ = ("sock", "reader")

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.reader = _Reader(sock.recv)


def _connect(url: str, timeout: float) -> "_Conn":
    host, port, user, pw, db, tls = parse_url(url)
    s = socket.create_connection((host, port), timeout=timeout)
    if tls:
        s = ssl.create_default_context().wrap_socket(s, server_hostname=host)
    s.settimeout(timeout)
    c = _Conn(s)
    if pw:
        s.sendall(encode("AUTH", user, pw) if user else encode("AUTH", pw))
        c.reader.reply()
    if db:
        s.sendall(encode("SELECT", db))
        c.reader.reply()
    return c


class RespClient:
    """Thread-safe request/reply connection (lazy, reconnects once per failed call)."""

    def __init__(self, url: str, timeout: float = 2.0):
        self.url, self.timeout = url, timeout
        self._conn: Optional[_Conn] = None
        self._lock = threading.Lock()

    def _call(self, *args: Any) -> Any:
        if self._conn is None:
            self._conn = _connect(self.url, self.timeout)
        self._conn.sock.sendall(encode(*args))
        return self._conn.reader.reply()

    def execute(self, *args: Any) -> Any:
        with self._lock:
            for attempt in (0, 1):
                try:
                    return self._call(*args)
                except (OSError, RedisError) as e:
                    self.close_locked()
                    if attempt or isinstance(e, RedisError) and "closed" not in str(e):
                        raise

    def close_locked(self) -> None:
        if self._conn is not None:
            try:
                self._conn.sock.close()
            except OSError:
                pass
            self._conn = None

    def close(self) -> None:
        with self._lock:
            self.close_locked()

    def ping(self) -> float:
        t0 = time.perf_counter()
        if self.execute("PING") not in ("PONG", b"PONG"):
            raise RedisError("unexpected PING reply")
        return (time.perf_counter() - t0) * 1e3


async def subscribe_stream(url: str, channel: str, on_message, timeout: float = 5.0) -> None:
    """Run ``SUBSCRIBE channel`` until cancelled; ``on_message(bytes)`` per published payload."""
    host, port, user, pw, db, tls = parse_url(url)
    ctx = ssl.create_default_context() if tls else None
    reader, writer = await asyncio.wait_for(asyncio.open_connection(host, port, ssl=ctx), timeout)
    buf = bytearray()

    async def read(n: int) -> bytes:
        return await reader.read(n)

    async def reply() -> Any:
        nonlocal buf

        async def line() -> bytes:
            nonlocal buf
            while b"\r\n" not in buf:
                chunk = await read(65536)
                if not chunk:
                    raise RedisError("connection closed")
                buf += chunk
            i = buf.index(b"\r\n")
            ln = bytes(buf[:i])
            del buf[:i + 2]
            return ln

        ln = await line()
        t, rest = ln[:1], ln[1:]
        if t in (b"+", b":"):
            return rest
        if t == b"-":
            raise RedisError(rest.decode())
        if t == b"$":
            n = int(rest)
            if n < 0:
                return None
            while len(buf) < n + 2:
                chunk = await read(65536)
                if not chunk:
                    raise RedisError("connection closed")
                buf += chunk
            data = bytes(buf[:n])
            del buf[:n + 2]
            return data
        if t == b"*":
            return [await reply() for _ in range(int(rest))]
        raise RedisError(f"bad RESP type {t!r}")

    try:
        if pw:
            writer.write(encode("AUTH", user, pw) if user else encode("AUTH", pw))
            await reply()
        writer.write(encode("SUBSCRIBE", channel))
        await writer.drain()
        while True:
            msg = await reply()
            if isinstance(msg, list) and len(msg) == 3 and msg[0] == b"message":
                on_message(msg[2])
    finally:
        writer.close()
