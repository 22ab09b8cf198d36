#!/usr/bin/env python3
"""Device-time sweep of the fused ETA kernel: batch x hidden x variant -> us/launch, preds/s,
achieved TFLOP/s.  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="256,4096,65536,262144,1048576,4194304")
    ap.add_argument("--hidden", default="256")
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rec", type=int, default=16, choices=[6, 8, 16], help="wire record bytes")
    a = ap.parse_args()
    import torch
    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import records_to_features
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.models.features import records_to_compact, records_to_compact6
    from routest_amd.ops.eta_mlp import (EtaMlpKernel, records6_to_tensor, records8_to_tensor,
                                         records_to_tensor)

    dev = torch.device("cuda:0")
    res = {}
    for H in [int(x) for x in a.hidden.split(",")]:
        torch.manual_seed(0)
        m = EtaMLP(H)
        r0, y0 = synth_records(8192, 1)
        m.fit_normalization(records_to_features(r0), y0)
        kerns = {v: EtaMlpKernel(m, dev, variant=v) for v in [int(x) for x in a.variants.split(",")]}
        flop_per_row = 2 * (16 * H + H * H + H)
        for B in [int(x) for x in a.batches.split(",")]:
            rec, _ = synth_records(B, 2)
            rt = (records6_to_tensor(records_to_compact6(rec)) if a.rec == 6 else
                  records8_to_tensor(records_to_compact(rec)) if a.rec == 8 else
                  records_to_tensor(rec)).to(dev)
            times = {v: [] for v in kerns}
            for _ in range(a.rounds):
                for v, k in kerns.items():
                    k(rt)
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    s.record()
                    for _ in range(a.iters):
                        k(rt)
                    e.record()
                    torch.cuda.synchronize()
                    times[v].append(s.elapsed_time(e) / a.iters * 1e3)
            for v, ts in times.items():
                us = min(ts)
                row = {"H": H, "B": B, "rec": a.rec, "variant": v, "us": round(us, 2),
                       "preds_per_s": B / us * 1e6, "tflops": flop_per_row * B / us / 1e6}
                print(json.dumps(row), flush=True)
                res[f"{H}/{B}/{v}"] = row
    out = os.environ.get("SWEEP_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
