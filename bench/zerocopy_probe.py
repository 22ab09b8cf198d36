#!/usr/bin/env python3
"""Zero-copy serving throughput vs batch size, record format and number of concurrent streams
(1 GPU).  Answers: is the zero-copy kernel bound by PCIe bandwidth or by reads in flight?"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch
    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import records_to_compact, records_to_features
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.ops.eta_mlp import EtaMlpKernel, records8_to_tensor, records_to_tensor
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = EtaMLP(256)
    r, y = synth_records(65536, 1)
    m.fit_normalization(records_to_features(r), y)
    k = EtaMlpKernel(m, dev)
    rows = []
    rec_all, _ = synth_records(1 << 23, 2)
    for recb in (8, 16):
        host_all = (records8_to_tensor(records_to_compact(rec_all)) if recb == 8 else records_to_tensor(rec_all)).pin_memory()
        dev_all = host_all.to(dev)
        out_h = torch.empty(1 << 23, dtype=torch.float32).pin_memory()
        for B in (1 << 20, 1 << 21, 1 << 22, 1 << 23):
            for mode, ns in (("device", 1), ("zerocopy", 1), ("zerocopy", 2), ("zerocopy", 4)):
                streams = [torch.cuda.Stream(dev) for _ in range(ns)]
                chunk = B // ns

                def run():
                    for i, s in enumerate(streams):
                        with torch.cuda.stream(s):
                            if mode == "device":
                                k(dev_all[i * chunk:(i + 1) * chunk])
                            else:
                                k.forward_hostio(host_all[i * chunk:(i + 1) * chunk], out_h[i * chunk:(i + 1) * chunk])
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                reps = max(3, (1 << 25) // B)
                t0 = time.perf_counter()
                for _ in range(reps):
                    run()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / reps
                rows.append({"rec_bytes": recb, "batch": B, "mode": mode, "streams": ns,
                             "preds_per_s": B / dt, "ms": dt * 1e3,
                             "pcie_GBps": B * (recb + 4) / dt / 1e9 if mode == "zerocopy" else None})
                print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
