#!/usr/bin/env python3
"""The wide trainer's dW2|db2 shape (K = batch rows, M = N = H) on its two kernels, for A/B timing
and PMC passes: ``wgrad256`` (256 x 256 output tiles, csrc/wgrad.hip wgrad256_kernel) and the
n-blocked ``wgrad`` (wgrad_kernel<NT>, the trainer's default).  One JSON line per kernel.

    python bench/wgrad_probe.py --hidden 1024 --batch 65536 --iters 20
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kernels", default="wgrad256,wgrad")
    a = ap.parse_args()
    from routest_amd.ops import _ext
    C = _ext.native(required=True)
    dev = torch.device("cuda", 0)
    H, B = a.hidden, a.batch
    ldg = H + 16
    g = torch.Generator(device=dev).manual_seed(0)
    dz2 = torch.randn(B, H, device=dev, generator=g).to(torch.bfloat16)
    h1a = torch.randn(B, ldg, device=dev, generator=g).to(torch.bfloat16)
    ncu = C.num_cus(0)
    ntt = (ldg + 31) // 32
    nsplit = -(-ntt // 9)
    nt = -(-ntt // nsplit)
    nblk = -(-ntt // nt)
    for k in a.kernels.split(","):
        if k == "wgrad256":
            S = max(1, min(B // 64, ncu // ((H // 256) ** 2)))
            slab = torch.zeros(S, H * ldg, device=dev)
            run = lambda: C.wgrad256(dz2, h1a, H, H, slab, ldg, H)  # noqa: E731
        else:
            S = max(1, min(B // 256, ncu // (nblk * (H // 256))))
            slab = torch.empty(S, H * ldg, device=dev)
            run = lambda: C.wgrad(dz2, H, H, h1a, ldg, slab, 0, ldg, nsplit=nsplit)  # noqa: E731
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        flops = 2.0 * B * H * H
        print(json.dumps({"kernel": k, "cfg": os.environ.get("ROUTEST_WGRAD256_CFG", "32x4"), "H": H, "batch": B,
                          "slices": S, "us": us, "tflops": flops / us / 1e6}), flush=True)


if __name__ == "__main__":
    main()
