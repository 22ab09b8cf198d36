#!/usr/bin/env python3
"""End-to-end HTTP benchmark of the ETA API (the reference's /api/predict_eta path, RO/Flaskr/routes.py:365-383).

Starts ``python -m routest_amd serve`` in a child process (uvicorn, synthetic-trained MLP; on a GPU
box the fused HIP kernel serves it), then over loopback HTTP/1.1 keep-alive measures:
  * p50 / p99 latency of single ``POST /api/predict_eta`` requests (sequential client);
  * throughput with C concurrent clients (single-item requests; the micro-batcher coalesces them);
  * throughput of batched ``POST /predict`` (JSON array of B items -> native C++ pack/format path).
The parent never touches the GPU (the server is a separate process started before anything else).
"""
from __future__ import annotations

import argparse
import http.client
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait(port: int, timeout: float = 240.0) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=2)
            c.request("GET", "/api/ping")
            if c.getresponse().status == 200:
                return
        except OSError:
            time.sleep(0.5)
    raise RuntimeError("server did not start")


def _post(conn, path: str, body: bytes):
    conn.request("POST", path, body=body, headers={"Content-Type": "application/json"})
    r = conn.getresponse()
    data = r.read()
    return r.status, data


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=3000)
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--batch", type=int, default=10000)
    ap.add_argument("--device", default="")
    ap.add_argument("--hidden", type=int, default=256)
    a = ap.parse_args()
    port = _free_port()
    env = dict(os.environ, ROUTEST_STORE="none", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "routest_amd", "serve", "--synthetic-model", "--port", str(port),
           "--hidden", str(a.hidden), "--env-file", ""]
    if a.device:
        cmd += ["--device", a.device]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        _wait(port)
        one = json.dumps({"summary": {"distance": 12345}, "pickup_time": "2025-08-25T08:30:00",
                          "driver_age": 34, "weather": "Sunny", "traffic": "Medium"}).encode()
        conn = http.client.HTTPConnection("127.0.0.1", port)
        for _ in range(200):
            _post(conn, "/api/predict_eta", one)
        lat = []
        for _ in range(a.requests):
            t0 = time.perf_counter()
            st, _ = _post(conn, "/api/predict_eta", one)
            lat.append(time.perf_counter() - t0)
            assert st == 200
        lat.sort()
        p50, p99 = lat[len(lat) // 2] * 1e3, lat[int(len(lat) * 0.99)] * 1e3

        # concurrent single-item clients
        done = [0]
        lock = threading.Lock()
        stop = time.perf_counter() + 5.0

        def client():
            c = http.client.HTTPConnection("127.0.0.1", port)
            n = 0
            while time.perf_counter() < stop:
                _post(c, "/api/predict_eta", one)
                n += 1
            with lock:
                done[0] += n
        th = [threading.Thread(target=client) for _ in range(a.concurrency)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        conc_rps = done[0] / (time.perf_counter() - t0)

        # batched /predict (fresh connection: the idle one hit uvicorn's keep-alive timeout)
        conn = http.client.HTTPConnection("127.0.0.1", port)
        items = json.dumps([{"summary": {"distance": 1000 + i}, "pickup_time": "2025-08-25T08:30:00",
                             "traffic": "High"} for i in range(a.batch)]).encode()
        _post(conn, "/predict", items)
        t0 = time.perf_counter()
        nb = 10
        for _ in range(nb):
            st, data = _post(conn, "/predict", items)
            assert st == 200
        batch_pps = a.batch * nb / (time.perf_counter() - t0)
        conn.request("GET", "/api/health")
        health = json.loads(conn.getresponse().read())
        print(json.dumps({"metric": "HTTP /api/predict_eta", "p50_ms": p50, "p99_ms": p99,
                          "concurrent_clients": a.concurrency, "concurrent_req_per_s": conc_rps,
                          "batch_items": a.batch, "batch_predict_preds_per_s": batch_pps,
                          "backend": health["checks"]["model"].get("backend"),
                          "devices": health["checks"]["model"].get("devices")}), flush=True)
    finally:
        srv.terminate()
        try:
            srv.wait(10)
        except subprocess.TimeoutExpired:
            srv.kill()


if __name__ == "__main__":
    main()
