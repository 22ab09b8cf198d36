"""Wide-trainer GEMM probe: times the layer-2 GEMM (gemm_nt epilogue 1: relu(z + b2) -> h2a + y
partials) and the dgrad GEMM (epilogue 2: store) at the H = 1024 trainer's shape, and checks them
against torch on the same bf16 operands.  The tile is picked by ROUTEST_GEMM_TILE (256 default,
128; read once per process: run once per variant).

    python bench/gemm_probe.py --n 1024 --k 1024 --m 65536
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def hperm(n):
    u = torch.arange(n)
    return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from routest_amd.ops import _ext
    C = _ext.native()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    N, K, M = args.n, args.k, args.m
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(dev)
    X = torch.randn(M, K, generator=g).to(torch.bfloat16).to(dev)
    b2 = (0.1 * torch.randn(N, generator=g)).to(dev)
    w3 = (torch.randn(N, generator=g) / N ** 0.5).to(dev)
    out = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    yp = torch.zeros(M, N // 64, device=dev)
    res = {"tile": int(os.environ.get("ROUTEST_GEMM_TILE", "256")),
           "N": N, "K": K, "M": M}
    flop = 2.0 * N * K * M
    for epi in (2, 1):
        def run():
            if epi == 2:
                C.gemm_nt(2, W, X, N, M, K, out=out)
            else:
                C.gemm_nt(1, W, X, N, M, K, b2=b2, w3=w3, ypart=yp, out=out)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        z = X.float() @ W.float().T
        got = torch.empty(M, N, device=dev)
        got[:, hperm(N).to(dev)] = out.float()
        ref = z if epi == 2 else torch.relu(z + b2)
        err = ((got - ref).abs() / (ref.abs() + 1.0)).max().item()
        res[f"epi{epi}"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1), "max_rel_err": err}
        if epi == 1:
            y = (torch.relu(z + b2) * w3).view(M, N // 64, 64).sum(-1)
            res["epi1"]["ypart_max_err"] = (yp - y).abs().max().item()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
