"""RedisBroker (own RESP client) against an in-test fake Redis: Flask-SSE message format,
PUBLISH -> SUBSCRIBE fan-out to an SSE queue, PING health, failure behaviour."""
import asyncio
import json
import socket
import socketserver
import threading

import pytest

from routest_amd.realtime.broker import RedisBroker, make_broker, MemoryBroker
from routest_amd.realtime.redis_resp import RespClient, encode, parse_url


class FakeRedis(socketserver.ThreadingTCPServer):
    allow_reuse_address = True
    daemon_threads = True

    def __init__(self):
        super().__init__(("127.0.0.1", 0), Handler)
        self.subs = {}       # channel -> list of sockets
        self.lock = threading.Lock()
        self.published = []


class Handler(socketserver.StreamRequestHandler):
    def _read_cmd(self):
        line = self.rfile.readline()
        if not line:
            return None
        assert line[:1] == b"*"
        args = []
        for _ in range(int(line[1:])):
            n = int(self.rfile.readline()[1:])
            args.append(self.rfile.read(n + 2)[:-2])
        return args

    def handle(self):
        srv = self.server
        while True:
            cmd = self._read_cmd()
            if cmd is None:
                return
            op = cmd[0].upper()
            if op == b"PING":
                self.wfile.write(b"+PONG\r\n")
            elif op in (b"AUTH", b"SELECT"):
                self.wfile.write(b"+OK\r\n")
            elif op == b"PUBLISH":
                ch, msg = cmd[1], cmd[2]
                srv.published.append((ch, msg))
                with srv.lock:
                    targets = list(srv.subs.get(ch, []))
                for w in targets:
                    try:
                        w.write(encode("message", ch, msg))
                        w.flush()
                    except OSError:
                        pass
                self.wfile.write(b":%d\r\n" % len(targets))
            elif op == b"SUBSCRIBE":
                ch = cmd[1]
                with srv.lock:
                    srv.subs.setdefault(ch, []).append(self.wfile)
                self.wfile.write(b"*3\r\n$9\r\nsubscribe\r\n$%d\r\n%s\r\n:1\r\n" % (len(ch), ch))
            else:
                self.wfile.write(b"-ERR unknown\r\n")
            self.wfile.flush()


@pytest.fixture()
def fake_redis():
    srv = FakeRedis()
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield f"redis://:secret@127.0.0.1:{srv.server_address[1]}/0", srv
    srv.shutdown()
    srv.server_close()


def test_parse_url():
    assert parse_url("rediss://u:p%40ss@h.example:6380/2") == ("h.example", 6380, "u", "p@ss", 2, True)
    assert parse_url("redis://localhost") == ("localhost", 6379, None, None, 0, False)


def test_ping_publish_subscribe(fake_redis):
    url, srv = fake_redis
    b = make_broker("redis", url)
    assert isinstance(b, RedisBroker)
    assert b.ping()["status"] == "ok"

    async def main():
        q = b.subscribe("driver-7")
        for _ in range(100):                   # wait until the SUBSCRIBE reached the server
            if srv.subs.get(b"driver-7"):
                break
            await asyncio.sleep(0.01)
        assert b.subscribers("driver-7") == 1
        n = b.publish({"remaining_routes": [[121.0, 14.5]], "assigned_driver": "driver-7"}, channel="driver-7")
        assert n == 1
        msg = await asyncio.wait_for(q.get(), 5)
        b.unsubscribe("driver-7", q)
        return msg
    msg = asyncio.run(main())
    assert msg.startswith("data:") and msg.endswith("\n\n")
    assert json.loads(msg[len("data:"):])["assigned_driver"] == "driver-7"
    # Flask-SSE wire format on the Redis side
    ch, raw = srv.published[-1]
    assert ch == b"driver-7" and json.loads(raw) == {"data": {"remaining_routes": [[121.0, 14.5]],
                                                             "assigned_driver": "driver-7"}}


def test_redis_down_degrades():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    b = RedisBroker(f"redis://127.0.0.1:{port}", timeout=0.5)
    assert b.ping()["status"] == "error"
    assert b.publish({"x": 1}, channel="c") == 0      # best effort, never raises


def test_memory_is_default():
    assert isinstance(make_broker("memory", "redis://x"), MemoryBroker)
    assert isinstance(make_broker("redis", None), MemoryBroker)
