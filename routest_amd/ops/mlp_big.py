"""Host side of the wide-MLP path (H = 512, 1024; ``csrc/mlp_big.hip``).

For H <= 256 the whole packed MLP (W2 is 128 KiB at H = 256) lives in each CU's LDS and one fused
kernel scores a batch (``ops/eta_mlp.py``).  At H = 512 / 1024 W2 is 0.5 / 2 MiB: it stays in L2
and streams through LDS tiles, so a batch runs as three launches per chunk of rows:

  big_layer1  : records -> featurize -> layer 1 -> h1 [rows, H] bf16 (hperm() unit order)
  gemm_nt(0)  : relu(W2 h1 + b2) . w3 per (row, 64-unit block) -> partials [rows, H/64]
  big_yreduce : minutes = sum(partials) + b3   (written straight to pinned host memory if asked)

The weights are packed once: W1k fragments exactly as the fused kernel's blob (``pack_mlp3``),
W2 row-major with its K columns in hperm order (h1's stored order), b2 / w3 in natural order with
the target scale folded into w3 / b3.  :func:`emulate_big` mirrors the numerics in PyTorch.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..models.mlp3 import EtaMLP
from . import _ext

BIG_HIDDEN = (512, 1024)


def hperm(H: int) -> torch.Tensor:
    u = torch.arange(H)
    return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1)


def fused_korder(H: int) -> torch.Tensor:
    """Unit feeding K position c of the fused kernel's layer-2 operand: within each 32-chunk,
    p = 8g + 4s + j holds unit 16s + 4g + j."""
    c = torch.arange(H)
    p = c & 31
    return (c & ~31) + 16 * ((p >> 2) & 1) + 4 * (p >> 3) + (p & 3)


class PackedBig:
    def __init__(self, model: EtaMLP, device: torch.device):
        from .eta_mlp import pack_mlp3
        H = model.hidden
        if H % 128:
            raise ValueError("wide path needs H % 128 == 0")
        p = pack_mlp3(model)                 # folded W1k, b1 hi/lo, target scale into w3 / b3
        self.hidden = H
        self.norm = list(p.norm)
        self.b3 = float(p.b3)
        MT = H // 32
        w1_bytes = p.blob[2 * H * H:2 * H * H + 32 * H]          # w1p part of the fused blob
        self.w1p = w1_bytes.view(torch.bfloat16).clone().to(device)
        assert self.w1p.numel() == MT * 64 * 8
        pm = hperm(H)
        self.w2k = p.w2[:, pm].to(torch.bfloat16).contiguous().to(device)      # [n][c] = W2[n][hp(c)]
        self.b2 = p.b2.float().contiguous().to(device)
        self.w3 = p.w3.float().contiguous().to(device)
        self.w1k = p.w1k                                                          # fp32, for emulation
        self.w2 = p.w2
        # fused inference kernel (mlp_big_fused_kernel): W1k as 16x16x16 A fragments
        # w1q[ub][l][j] = W1k[16ub + (l & 15)][4(l >> 4) + j], and W2 with each 32-column K chunk in
        # the order p = 8g + 4s + j <-> unit 16s + 4g + j (the layer-1 MFMA output packing)
        lane = torch.arange(64)
        rows = 16 * torch.arange(H // 16)[:, None, None] + (lane & 15)[None, :, None]
        cols = 4 * (lane >> 4)[None, :, None] + torch.arange(4)[None, None, :]
        self.w1q = p.w1k[rows, cols].to(torch.bfloat16).contiguous().to(device)
        self.w2f = p.w2[:, fused_korder(H)].to(torch.bfloat16).contiguous().to(device)


class EtaMlpBigKernel:
    """Wide-MLP scorer on one GPU; ``__call__(records) -> minutes`` (f32 [B] on the device)."""

    def __init__(self, model: EtaMLP, device: torch.device, chunk_rows: int = 1 << 20):
        self.device = torch.device(device)
        self.hidden = model.hidden
        self._C = _ext.native(required=True)
        self.packed = PackedBig(model.float().cpu().eval(), self.device)
        self.chunk = chunk_rows
        self._ws = None
        self._yp = None

    def _workspace(self, rows: int):
        H = self.hidden
        if self._ws is None or self._ws[0].shape[0] < rows:
            self._ws = (torch.empty(rows, H, dtype=torch.bfloat16, device=self.device),
                        torch.empty(rows, H // 64, dtype=torch.float32, device=self.device))
        return self._ws

    # one launch (featurize + both layers, h1 never in HBM) when H % 256 == 0; ROUTEST_BIG_FUSED=0
    # selects the three-launch path (layer-1 kernel -> h1 in HBM -> GEMM)
    FUSED = os.environ.get("ROUTEST_BIG_FUSED", "1") != "0"

    def _run(self, rec: torch.Tensor, out: torch.Tensor) -> None:
        C, p, H = self._C, self.packed, self.hidden
        B = rec.shape[0]
        fused = self.FUSED and H % 256 == 0
        for s in range(0, B, self.chunk):
            n = min(self.chunk, B - s)
            if fused:
                yp = self._ypart(n)
                C.big_fused(rec[s:s + n], p.w1q, p.w2f, p.b2, p.w3, H, p.norm, yp)
            else:
                h1, yp = self._workspace(n)
                C.big_layer1(rec[s:s + n], p.w1p, H, p.norm, h1[:n])
                C.gemm_nt(0, p.w2k, h1, H, n, H, b2=p.b2, w3=p.w3, ypart=yp)
            C.big_yreduce(yp[:n].reshape(-1), H // 64, p.b3, y=out[s:s + n])

    def _ypart(self, rows: int) -> torch.Tensor:
        if self._yp is None or self._yp.shape[0] < rows:
            self._yp = torch.empty(rows, self.hidden // 64, dtype=torch.float32, device=self.device)
        return self._yp

    def __call__(self, rec: torch.Tensor) -> torch.Tensor:
        out = torch.empty(rec.shape[0], dtype=torch.float32, device=self.device)
        if rec.shape[0]:
            self._run(rec, out)
        return out

    def forward_hostio(self, rec: torch.Tensor, out: torch.Tensor) -> None:
        """records and/or minutes in pinned host memory (zero-copy), like the fused kernel."""
        if rec.shape[0]:
            self._run(rec, out)


def emulate_big(p: PackedBig, rec_i32: torch.Tensor) -> torch.Tensor:
    """PyTorch mirror of the wide path's numerics (bf16 operands, fp32 accumulate, bf16 h1)."""
    from .eta_mlp import PackedMLP3, emulate_kernel  # noqa: F401
    from .eta_mlp import featurize_torch
    x = featurize_torch(rec_i32)
    dev = x.device
    sc = torch.tensor(p.norm[:4], device=dev)
    sh = torch.tensor(p.norm[4:], device=dev)
    num = x[:, 8:12] * sc + sh
    hi = num.to(torch.bfloat16).float()
    f = torch.zeros(x.shape[0], 16, device=dev)
    f[:, :8] = x[:, :8]
    f[:, 8:12] = hi
    f[:, 12] = num[:, 2] - hi[:, 2]
    f[:, 13] = num[:, 3] - hi[:, 3]
    f[:, 14:16] = 1.0
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    h1 = bf(torch.relu(bf(f) @ bf(p.w1k.to(dev)).T))
    h2 = torch.relu(h1 @ bf(p.w2.to(dev)).T + p.b2.to(dev))
    return h2 @ p.w3.to(dev) + p.b3
