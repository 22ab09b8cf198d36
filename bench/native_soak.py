#!/usr/bin/env python3
"""Soak of the native front end with the resident scorer under MIXED traffic: N single-request
keep-alive connections (resident-scorer rounds) while another client keeps posting large batched
/predict bodies (normal launches, which park the resident kernel first).  Prints one JSON line:
throughput, latency percentiles, server stats; fails if any request errored or the scorer fell
back."""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--connections", type=int, default=32)
    ap.add_argument("--threads", type=int, default=4, help="server reactors")
    ap.add_argument("--batch-items", type=int, default=5000)
    a = ap.parse_args()
    import http.client

    import numpy as np
    from routest_amd.ops import _ext
    from routest_amd.serve.eta_service import default_model
    from routest_amd.serve.native_server import NativePredictServer
    rt = _ext.runtime(required=True)
    body = json.dumps({"summary": {"distance": 12345}, "pickup_time": "2026-10-15T08:30:00",
                       "driver_age": 34, "weather": "Sunny", "traffic": "Medium"})
    items = [{"summary": {"distance": 1000 + 7 * i}, "pickup_time": "2026-10-15T08:30:00",
              "traffic": ["High", "Low", "Jam", "Medium"][i % 4]} for i in range(a.batch_items)]
    big = json.dumps(items).encode()
    model = default_model(steps=30)
    with NativePredictServer(model, device=0, threads=a.threads) as srv:
        stop = time.time() + a.seconds
        big_done = [0, 0]

        def batches():
            c = http.client.HTTPConnection("127.0.0.1", srv.port, timeout=30)
            while time.time() < stop:
                c.request("POST", "/predict", body=big, headers={"Content-Type": "application/json"})
                r = c.getresponse()
                out = json.loads(r.read())
                big_done[0] += 1
                big_done[1] += int(r.status != 200 or len(out["predictions"]) != a.batch_items)

        th = threading.Thread(target=batches)
        th.start()
        res = rt.http_load(srv.port, a.connections, a.seconds, "/api/predict_eta", body, 4, 0, 20)
        th.join()
        st = srv.stats()
    lat = np.asarray(res["latencies_us"])
    out = {"metric": "native front end soak (single requests + concurrent large batches)",
           "seconds": res["seconds"], "connections": a.connections, "reactors": a.threads,
           "single_req_per_s": res["requests"] / res["seconds"], "single_errors": res["errors"],
           "p50_us": float(np.percentile(lat, 50)), "p99_us": float(np.percentile(lat, 99)),
           "p999_us": float(np.percentile(lat, 99.9)), "batch_requests": big_done[0],
           "batch_items": a.batch_items, "batch_errors": big_done[1], "server": st}
    print(json.dumps(out), flush=True)
    ok = res["errors"] == 0 and big_done[1] == 0 and st.get("fallbacks", 0) == 0 and st["errors"] == 0
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
