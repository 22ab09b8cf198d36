#!/usr/bin/env python3
"""Where does single-request /predict latency go?  Median of N calls at each layer of the stack
(1 GPU): raw zero-copy kernel + sync, GpuRunner, MicroBatcher (thread hop), EtaService.apredict
(asyncio), and the full FastAPI app over in-process ASGI (httpx) — the bench.py p50 path."""
from __future__ import annotations

import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] * 1e6


def main() -> None:
    import numpy as np
    import torch
    from routest_amd.models.features import RECORD_DTYPE
    from routest_amd.serve.eta_service import EtaService, default_model
    from routest_amd.utils.timeutil import parse_iso
    N = int(os.environ.get("N", "2000"))
    model = default_model(steps=50)
    svc = EtaService(model, devices=[0])
    runner = svc.batcher.runners[0]
    rec_t, _ = svc.make_record(weather="Sunny", traffic="Medium", distance_m=12345,
                               pickup_time="2026-10-15T08:30:00", driver_age=34)
    rec = np.array([rec_t], dtype=RECORD_DTYPE)
    res = {}
    # 1. raw kernel on pinned buffers
    k = runner.kernel
    runner.h_rec_np[:1] = rec
    ts = []
    with torch.cuda.stream(runner.stream):
        for _ in range(N):
            t0 = time.perf_counter()
            k.forward_hostio(runner.h_rec[:1], runner.h_out[:1])
            runner.stream.synchronize()
            ts.append(time.perf_counter() - t0)
    res["kernel_launch_sync_us"] = med(ts)
    ts = []
    for _ in range(N):
        t0 = time.perf_counter()
        runner(rec)
        ts.append(time.perf_counter() - t0)
    res["gpu_runner_us"] = med(ts)
    ts = []
    for _ in range(N):
        t0 = time.perf_counter()
        svc.batcher.predict_sync(rec_t)
        ts.append(time.perf_counter() - t0)
    res["batcher_sync_us"] = med(ts)

    async def amain():
        out = []
        for _ in range(N):
            t0 = time.perf_counter()
            await svc.apredict(weather="Sunny", traffic="Medium", distance_m=12345,
                               pickup_time="2026-10-15T08:30:00", driver_age=34)
            out.append(time.perf_counter() - t0)
        return out
    res["service_apredict_us"] = med(asyncio.run(amain()))

    import httpx
    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    s = load_settings(env={}, dotenv_path=None, devices=[0])
    app = create_app(build_services(s, eta=svc, store=None))
    body = {"summary": {"distance": 12345}, "pickup_time": "2026-10-15T08:30:00", "driver_age": 34,
            "weather": "Sunny", "traffic": "Medium"}

    async def ahttp(path):
        out = []
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://b") as c:
            for _ in range(N):
                t0 = time.perf_counter()
                r = await c.post(path, json=body)
                out.append(time.perf_counter() - t0)
                assert r.status_code == 200
        return out
    res["asgi_predict_eta_us"] = med(asyncio.run(ahttp("/api/predict_eta")))

    async def aping():
        out = []
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://b") as c:
            for _ in range(N):
                t0 = time.perf_counter()
                await c.get("/api/ping")
                out.append(time.perf_counter() - t0)
        return out
    res["asgi_get_ping_us"] = med(asyncio.run(aping()))

    # real HTTP/1.1 over loopback: uvicorn in a background thread of this process, http.client
    import http.client
    import socket
    import threading
    import uvicorn
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning",
                                           access_log=False, lifespan="off"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    while not server.started:
        time.sleep(0.01)
    conn = http.client.HTTPConnection("127.0.0.1", port)
    raw = json.dumps(body).encode()
    hdr = {"Content-Type": "application/json"}
    out = []
    for j in range(N + 200):
        t0 = time.perf_counter()
        conn.request("POST", "/api/predict_eta", body=raw, headers=hdr)
        r = conn.getresponse()
        r.read()
        if j >= 200:
            out.append(time.perf_counter() - t0)
    res["http_loopback_inproc_server_us"] = med(out)
    res["http_loopback_p99_us"] = sorted(out)[int(len(out) * 0.99)] * 1e6
    server.should_exit = True
    th.join(timeout=10)
    svc.close()
    print(json.dumps({"metric": "single-request latency breakdown (median us)", **res}), flush=True)


if __name__ == "__main__":
    main()
