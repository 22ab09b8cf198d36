"""hipBLASLt (torch.matmul) bf16 throughput on the wide trainer's three GEMM shapes, for comparison
with the in-tree gemm256 / wgrad kernels (bench/gpu_r3v.sh)."""
import json, sys, torch

def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it

H = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
for B in (16384, 65536, 262144):
    d = "cuda"
    h1 = torch.randn(B, H, device=d, dtype=torch.bfloat16)
    w2 = torch.randn(H, H, device=d, dtype=torch.bfloat16)
    dz = torch.randn(B, H, device=d, dtype=torch.bfloat16)
    fl = 2.0 * B * H * H
    res = {"B": B, "H": H}
    res["fwd_ms"] = bench(lambda: h1 @ w2.t())
    res["dgrad_ms"] = bench(lambda: dz @ w2)
    res["wgrad_ms"] = bench(lambda: dz.t() @ h1)
    for k in ("fwd", "dgrad", "wgrad"):
        res[k + "_tflops"] = round(fl / res[k + "_ms"] / 1e9, 1)
    print(json.dumps(res), flush=True)
