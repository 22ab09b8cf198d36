#!/usr/bin/env python3
"""K4 tree-ensemble throughput: the reference's model family (XGBoost regressor, RO/Flaskr/ml.py:53).

SURVEY §6 proxy: sklearn HistGradientBoostingRegressor, 400 iterations x 63 leaves (2.86 MB pickle,
comparable to the 2.44 MB reference artifact) -> ~359k preds/s bulk on 8 CPU threads.  Here the
same-shaped ensemble is trained on synthetic trips, converted to the packed node format
(models/forest.py) and scored by csrc/forest.hip on one GPU from 16-byte records.  Reports GPU
preds/s (device-resident records), the CPU sklearn bulk number on this host, and max |diff|.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--leaves", type=int, default=63)
    ap.add_argument("--rows", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-rows", type=int, default=200_000)
    a = ap.parse_args()
    import numpy as np
    import torch
    from sklearn.ensemble import HistGradientBoostingRegressor
    from routest_amd.data.synth import synth_records, synth_trips
    from routest_amd.models.features import records_to_features
    from routest_amd.models.forest import ForestModel
    from routest_amd.ops.eta_mlp import records_to_tensor
    from routest_amd.serve.eta_service import ForestKernel

    x, y = synth_trips(200_000, 0)
    t0 = time.perf_counter()
    est = HistGradientBoostingRegressor(max_iter=a.iters, max_leaf_nodes=a.leaves, early_stopping=False,
                                        random_state=0).fit(x, y)
    fit_s = time.perf_counter() - t0
    fm = ForestModel.from_sklearn_hgb(est)
    rec, _ = synth_records(a.rows, 1)
    xr = records_to_features(rec[:a.cpu_rows])
    t0 = time.perf_counter()
    cpu_pred = est.predict(xr)
    cpu_pps = a.cpu_rows / (time.perf_counter() - t0)
    dev = torch.device("cuda", 0)
    rt = records_to_tensor(rec).to(dev)
    res = {}
    for name, lds in (("global", False), ("lds", True)):
        k = ForestKernel(fm, dev, lds=lds)
        out = k(rt)
        torch.cuda.synchronize()
        diff = float(np.abs(out[:a.cpu_rows].cpu().numpy() - cpu_pred).max())
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(a.reps):
            out = k(rt)
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / a.reps
        res[name] = {"ms_per_batch": ms, "gpu_preds_per_s": a.rows / ms * 1e3, "max_abs_diff_vs_sklearn": diff}
    print(json.dumps({"metric": "K4 forest preds/s (1 GPU, device-resident records)", "trees": fm.num_trees,
                      "nodes": int(len(fm.values)), "model_bytes": int(len(fm.values) * 8), "rows": a.rows,
                      "kernels": res, "gpu_preds_per_s": max(r["gpu_preds_per_s"] for r in res.values()),
                      "cpu_sklearn_preds_per_s": cpu_pps, "fit_s": fit_s}), flush=True)


if __name__ == "__main__":
    main()
