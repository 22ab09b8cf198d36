#!/usr/bin/env python3
"""Config 1 (BASELINE.json): linear-regression ETA trained on a 1k-row synthetic trip CSV, served
by the CPU-only FastAPI /predict (plumbing, no GPU).  Reports p50/p99 of single POST /predict
requests through the app in-process (ASGI; the reference's Flask test-client methodology), the
model's MAE on held-out synthetic trips, and batched /predict throughput."""
from __future__ import annotations

import asyncio
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import httpx
    import numpy as np
    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    from routest_amd.data.synth import synth_trips, write_trips_csv
    from routest_amd.serve.eta_service import EtaService
    from routest_amd.train.trainer import TrainConfig, train_linear
    with tempfile.TemporaryDirectory() as td:
        csv_path = os.path.join(td, "trips_1k.csv")
        write_trips_csv(csv_path, 1000, seed=0)
        t0 = time.perf_counter()
        model = train_linear(TrainConfig(arch="linear", data_csv=csv_path, ckpt_dir=os.path.join(td, "lin")))
        fit_ms = (time.perf_counter() - t0) * 1e3
    x, y = synth_trips(5000, seed=1)
    mae = float(np.abs(model.predict_features(x) - y).mean())
    s = load_settings(env={"ROUTEST_DEVICE": "cpu"}, dotenv_path=None)
    app = create_app(build_services(s, eta=EtaService(model, device="cpu"), store=None))
    body = {"summary": {"distance": 12345}, "pickup_time": "2025-08-25T08:30:00", "driver_age": 34,
            "weather": "Sunny", "traffic": "Medium"}
    items = [dict(body, summary={"distance": 1000 + i}) for i in range(1000)]

    async def run():
        lat = []
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://c1") as c:
            for j in range(2200):
                t1 = time.perf_counter()
                r = await c.post("/predict", json=body)
                if j >= 200:
                    lat.append(time.perf_counter() - t1)
                assert r.status_code == 200
            t1 = time.perf_counter()
            for _ in range(20):
                r = await c.post("/predict", json=items)
                assert r.status_code == 200
            bps = 20 * len(items) / (time.perf_counter() - t1)
        return sorted(lat), bps
    lat, bps = asyncio.run(run())
    print(json.dumps({"metric": "config 1: linear ETA, CPU-only FastAPI /predict", "train_rows": 1000,
                      "fit_ms": fit_ms, "holdout_mae_min": mae, "p50_ms": lat[len(lat) // 2] * 1e3,
                      "p99_ms": lat[int(len(lat) * 0.99)] * 1e3, "batched_1000_preds_per_s": bps,
                      "device": "cpu"}), flush=True)


if __name__ == "__main__":
    main()
