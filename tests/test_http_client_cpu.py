"""Native closed-loop HTTP client (csrc/runtime/http_client.h via _rt.http_load): framing by
Content-Length, keep-alive, warm-up exclusion, request cap, error counting."""
import socketserver
import threading

import pytest

rt = pytest.importorskip("routest_amd._rt")


class _H(socketserver.BaseRequestHandler):
    def handle(self):
        buf = b""
        while True:
            d = self.request.recv(65536)
            if not d:
                return
            buf += d
            while b"\r\n\r\n" in buf:
                head, rest = buf.split(b"\r\n\r\n", 1)
                n = int([ln.split(b":")[1] for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0])
                if len(rest) < n:
                    break
                body, buf = rest[:n], rest[n:]
                status = b"200 OK" if b"ok" in body else b"400 Bad Request"
                out = b'{"eta_minutes_ml": 12.5}'
                self.request.sendall(b"HTTP/1.1 " + status + b"\r\ncontent-type: application/json\r\ncontent-length: "
                                     + str(len(out)).encode() + b"\r\n\r\n" + out)


@pytest.fixture
def server():
    socketserver.ThreadingTCPServer.allow_reuse_address = True
    srv = socketserver.ThreadingTCPServer(("127.0.0.1", 0), _H)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield srv.server_address[1]
    srv.shutdown()
    srv.server_close()


def test_http_load_counts_and_latencies(server):
    r = rt.http_load(server, 1, 10.0, "/api/predict_eta", '{"ok": 1}', 1, 300, 50)
    assert r["errors"] == 0
    assert r["requests"] == 300 == len(r["latencies_us"])
    lat = r["latencies_us"]
    assert (lat[1:] >= lat[:-1]).all() and lat[0] > 0


def test_http_load_multi_connection_and_errors(server):
    r = rt.http_load(server, 4, 0.3, "/api/predict_eta", '{"bad": 1}', 2, 0, 0)
    assert r["requests"] > 0 and r["errors"] == r["requests"]     # every response is a 400
