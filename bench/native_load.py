#!/usr/bin/env python3
"""Native prediction front end under load (1 GPU): closed-loop native load generator
(build/native/loadgen) against NativePredictServer, sweeping client connections and server
reactor threads.  Single-item POST /api/predict_eta (plus one batched /predict run)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    from routest_amd.serve.eta_service import default_model
    from routest_amd.serve.native_server import NativePredictServer
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_ext
    lg = build_ext.build_tools()
    model = default_model(steps=30)
    rows = []
    for threads in (1, 4, 8):
        with NativePredictServer(model, device=0, threads=threads) as srv:
            for conns in (1, 16, 64, 256):
                out = subprocess.run([lg, str(srv.port), str(conns), "2", "/api/predict_eta", "-",
                                      str(min(8, conns))], capture_output=True, text=True, timeout=60)
                d = json.loads(out.stdout.strip().splitlines()[-1])
                d.update(server_threads=threads, launches=srv.stats()["launches"])
                rows.append(d)
                print(json.dumps(d), flush=True)
    # batched /predict: 1000 items per request
    items = [{"summary": {"distance": 1000 + i}, "pickup_time": "2026-10-15T08:30:00", "traffic": "High"}
             for i in range(1000)]
    path = os.path.join(ROOT, "gpurun_out", "batch1000.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(items, f)
    with NativePredictServer(model, device=0, threads=8) as srv:
        out = subprocess.run([lg, str(srv.port), "64", "2", "/predict", path, "8"], capture_output=True,
                             text=True, timeout=60)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        d.update(server_threads=8, items_per_request=1000, preds_per_s=d["req_per_s"] * 1000)
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
