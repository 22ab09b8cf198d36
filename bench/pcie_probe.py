#!/usr/bin/env python3
"""Where does the headline's hybrid step lose time?  Times, for B 6-byte records per step:

  copy     : the H2D record DMA alone
  kern_h   : the fused kernel alone, minutes written zero-copy into pinned host memory
  kern_d   : the fused kernel alone, minutes to HBM
  hyb_h    : copy of step k+1 overlapped with the kernel of step k (minutes to host) — bench.py
  hyb_d    : the same with minutes to HBM (no PCIe traffic from the kernel)

for host buffers from torch's pinned allocator (hipHostMalloc, 4 KiB pages) and from
``_C.pinned_host_empty`` (2 MiB-aligned, THP-advised, hipHostRegister'ed).  One JSON line each.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def thp_kb(addr: int) -> int:
    """AnonHugePages (kB) of the mapping holding ``addr``."""
    cur = None
    with open("/proc/self/smaps") as f:
        for line in f:
            parts = line.split()
            if "-" in parts[0] and len(parts) >= 5 and ":" not in parts[0]:
                lo, hi = (int(x, 16) for x in parts[0].split("-"))
                cur = lo <= addr < hi
            elif cur and parts[0] == "AnonHugePages:":
                return int(parts[1])
    return -1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    import torch
    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import records_to_compact6, records_to_features
    from routest_amd.models.mlp3 import EtaMLP
    from routest_amd.ops import _ext
    from routest_amd.ops.eta_mlp import EtaMlpKernel, records6_to_tensor

    from routest_amd.parallel.affinity import bind_to_gpu_numa
    C = _ext.native(required=True)
    dev = torch.device("cuda", 0)
    numa = bind_to_gpu_numa(0)           # host buffers on the GPU's NUMA node, as bench.py
    torch.manual_seed(1234)
    model = EtaMLP(256)
    nr, ny = synth_records(65536, seed=11)
    model.fit_normalization(records_to_features(nr), ny)
    kern = EtaMlpKernel(model, dev)
    B = a.batch
    rec, _ = synth_records(B, seed=100)
    src = records6_to_tensor(records_to_compact6(rec))
    try:
        thp = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        thp = "?"
    print(json.dumps({"thp": thp, "numa": numa}), flush=True)

    def host_buf(kind: str, like: torch.Tensor) -> torch.Tensor:
        if kind == "torch":
            return torch.empty_like(like).pin_memory()
        raw = C.pinned_host_empty(like.numel() * like.element_size(), kind == "thp")
        return raw.view(like.dtype).view(like.shape)

    cs, ks, ds = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    warm = src.to(dev)
    for _ in range(60):                    # clocks ramp over the first ~20 launches
        kern(warm)
    torch.cuda.synchronize()
    del warm

    def timeit(fn, iters):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        # join both streams into the default one before the end event
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.current_stream().wait_stream(ks)
        torch.cuda.current_stream().wait_stream(ds)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    for kind in ("torch", "thp"):
        hrec = host_buf(kind, src)
        hrec.copy_(src)
        hout = [host_buf(kind, torch.empty(B, dtype=torch.float32)) for _ in range(3)]
        drec = [torch.empty_like(src, device=dev) for _ in range(3)]
        dout = [torch.empty(B, dtype=torch.float32, device=dev) for _ in range(3)]
        for d in drec:
            d.copy_(hrec)
        h2d = [torch.cuda.Event() for _ in range(3)]
        done = [torch.cuda.Event() for _ in range(3)]
        out_free = [torch.cuda.Event() for _ in range(3)]
        torch.cuda.synchronize()
        huge_kb = thp_kb(hrec.data_ptr())

        def copy(i):
            with torch.cuda.stream(cs):
                drec[i % 3].copy_(hrec, non_blocking=True)

        def kh(i):
            with torch.cuda.stream(ks):
                kern.forward_hostio(drec[i % 3], hout[i % 3])

        def kd(i):
            with torch.cuda.stream(ks):
                kern.forward_hostio(drec[i % 3], dout[i % 3])

        def hyb(to_host):
            def f(i):
                k = i % 3
                with torch.cuda.stream(cs):
                    cs.wait_event(done[k])
                    drec[k].copy_(hrec, non_blocking=True)
                    h2d[k].record(cs)
                with torch.cuda.stream(ks):
                    ks.wait_event(h2d[k])
                    kern.forward_hostio(drec[k], hout[k] if to_host else dout[k])
                    done[k].record(ks)
            return f

        def d2h(i):
            with torch.cuda.stream(ds):
                hout[i % 3].copy_(dout[i % 3], non_blocking=True)

        def duplex(i):
            copy(i)
            d2h(i)

        def hyb_dma(i):
            # minutes to HBM, then out on a second copy engine (the other link direction)
            k = i % 3
            with torch.cuda.stream(cs):
                cs.wait_event(done[k])
                drec[k].copy_(hrec, non_blocking=True)
                h2d[k].record(cs)
            with torch.cuda.stream(ks):
                ks.wait_event(h2d[k])
                ks.wait_event(out_free[k])
                kern.forward_hostio(drec[k], dout[k])
                done[k].record(ks)
            with torch.cuda.stream(ds):
                ds.wait_event(done[k])
                hout[k].copy_(dout[k], non_blocking=True)
                out_free[k].record(ds)

        res = {"host": kind, "thp_kb_rec": huge_kb, "B": B}
        for name, fn in (("copy", copy), ("d2h", d2h), ("duplex", duplex), ("kern_h", kh),
                         ("kern_d", kd), ("hyb_h", hyb(True)), ("hyb_d", hyb(False)),
                         ("hyb_dma", hyb_dma), ("copy2", copy)):
            ms = timeit(fn, a.iters)
            res[name + "_ms"] = round(ms, 4)
        res["copy_GBps"] = round(src.numel() * 2 / res["copy_ms"] / 1e6, 2)
        res["hyb_h_Gpreds"] = round(B / res["hyb_h_ms"] / 1e6, 3)
        print(json.dumps(res), flush=True)
        del hrec, hout, drec, dout
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
