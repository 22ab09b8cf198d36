"""Host side of the fused ETA MLP kernel (K1 featurize + K2 forward, ``csrc/eta_mlp_fwd.hip``).

:func:`pack_mlp3` turns an :class:`~routest_amd.models.mlp3.EtaMLP` into the kernel's weight blob:

* ``W1k [H,16]``: W1 on normalised features, with the km/age columns duplicated into the pad
  slots k = 12, 13 (the kernel feeds a bf16 hi/lo split of those two inputs there) and b1 as a
  bf16 hi/lo pair in k = 14, 15 (whose inputs are the constant 1), so layer 1 is one bare MFMA.
* A fragments for ``mfma_f32_32x32x16_bf16``: lane l holds ``A[row l&31][k = 8(l>>5) + j]``.
  For layer 2 the B operand is the layer-1 accumulator, whose element j of lane half h is hidden
  unit ``16ks + 8(j>>2) + 4h + (j&3)`` (cdna_hip_programming.md §3), so W2's columns are permuted
  the same way here, once, on the host.
* bias / w3 vectors in accumulator-register order: ``v[mt][h][i] = v[32mt + (i&3) + 8(i>>2) + 4h]``.
* the target de-normalisation (y_std, y_mean) is folded into w3 / b3.

:func:`emulate_kernel` reproduces the kernel's numerics (bf16 operands, fp32 accumulate) on any
device with plain PyTorch; tests compare the HIP kernel against it and against the fp32 model.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..models.features import RECORD8_DTYPE, RECORD_DTYPE
from ..models.mlp3 import EtaMLP
from . import _ext


def _acc_rows(h: int) -> np.ndarray:
    i = np.arange(16)
    return (i & 3) + 8 * (i >> 2) + 4 * h


def blob_bytes(H: int) -> int:
    """[w2p | w1p | b1p | b2p | w3p | tail(b3,0,0,0)] — csrc/mlp3_tile.h"""
    return 2 * H * H + 44 * H + 16


@dataclass
class PackedMLP3:
    hidden: int
    blob: torch.Tensor          # uint8 [2H^2 + 44H]
    norm: List[float]           # 4 scales + 4 shifts (weekday, hour, km, age)
    b3: float
    # fp32 kernel-view tensors (for emulation / debugging)
    w1k: torch.Tensor
    b1: torch.Tensor
    w2: torch.Tensor
    b2: torch.Tensor
    w3: torch.Tensor

    def to(self, device) -> "PackedMLP3":
        return PackedMLP3(self.hidden, self.blob.to(device), list(self.norm), self.b3,
                          self.w1k, self.b1, self.w2, self.b2, self.w3)


@torch.no_grad()
def pack_mlp3(model: EtaMLP) -> PackedMLP3:
    H = model.hidden
    MT, KS = H // 32, H // 16
    W1 = model.l1.weight.detach().float().cpu()                   # [H,12]
    x_std = model.x_std.detach().float().cpu()
    x_mean = model.x_mean.detach().float().cpu()
    # one-hot inputs are used raw by the kernel: fold any (non-default) one-hot normalisation in
    W1n = W1 / x_std
    b1 = model.l1.bias.detach().float().cpu().clone()
    b1 -= (W1n[:, :8] * x_mean[:8]).sum(1)
    W1eff = W1.clone()
    W1eff[:, :8] = W1n[:, :8]
    w1k = torch.zeros(H, 16)
    w1k[:, :12] = W1eff
    w1k[:, 12] = W1eff[:, 10]
    w1k[:, 13] = W1eff[:, 11]
    b1_hi = b1.to(torch.bfloat16).float()
    w1k[:, 14] = b1_hi            # constant-1 inputs k = 14, 15 carry b1 as bf16 hi + lo
    w1k[:, 15] = b1 - b1_hi
    W2 = model.l2.weight.detach().float().cpu()                   # [H,H] (out, in)
    b2 = model.l2.bias.detach().float().cpu()
    y_std = float(model.y_std)
    y_mean = float(model.y_mean)
    w3 = model.l3.weight.detach().float().cpu().reshape(H) * y_std
    b3 = float(model.l3.bias.detach().float().cpu().reshape(())) * y_std + y_mean

    lane = np.arange(64)
    r = lane & 31
    hh = lane >> 5
    j = np.arange(8)
    # w1p[mt][l][j] = W1k[32mt + r][8h + j]
    rows = (32 * np.arange(MT)[:, None, None] + r[None, :, None])
    cols = (8 * hh[None, :, None] + j[None, None, :])
    w1p = w1k.numpy()[rows, np.broadcast_to(cols, (MT, 64, 8))]
    # w2p[mt][ks][l][j] = W2[32mt + r][16ks + 8(j>>2) + 4h + (j&3)]
    rows2 = 32 * np.arange(MT)[:, None, None, None] + r[None, None, :, None]
    cols2 = (16 * np.arange(KS)[None, :, None, None] + 8 * (j >> 2)[None, None, None, :]
             + 4 * hh[None, None, :, None] + (j & 3)[None, None, None, :])
    rows2 = np.broadcast_to(rows2, (MT, KS, 64, 8))
    cols2 = np.broadcast_to(cols2, (MT, KS, 64, 8))
    w2p = W2.numpy()[rows2, cols2]

    def vec_pack(v: torch.Tensor) -> np.ndarray:
        vv = v.numpy()
        out = np.empty((MT, 2, 16), dtype=np.float32)
        for mt in range(MT):
            for h in range(2):
                out[mt, h] = vv[32 * mt + _acc_rows(h)]
        return out

    def bf16_bytes(a: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16)
        return t.view(torch.int16).numpy().view(np.uint8).reshape(-1)

    parts = [bf16_bytes(w2p), bf16_bytes(w1p),
             vec_pack(b1).view(np.uint8).reshape(-1),
             vec_pack(b2).view(np.uint8).reshape(-1),
             vec_pack(w3).view(np.uint8).reshape(-1),
             np.array([b3, 0.0, 0.0, 0.0], dtype=np.float32).view(np.uint8)]
    blob = torch.from_numpy(np.concatenate(parts).copy())
    assert blob.numel() == blob_bytes(H)
    scale = (1.0 / x_std[8:12]).tolist()
    shift = (-x_mean[8:12] / x_std[8:12]).tolist()
    return PackedMLP3(H, blob, scale + shift, b3, w1k, b1, W2.clone(), b2.clone(), w3)


def blob16_bytes(H: int) -> int:
    """[w2p16 | w1p16 | b2 | w3 | tail(b3,0,0,0) | w3f] — csrc/eta_mlp_fwd.hip Mlp3Layout16"""
    return 2 * H * H + 72 * H + 16


@torch.no_grad()
def pack_mlp3_16(p: PackedMLP3) -> torch.Tensor:
    """Weight blob of the 16x16-MFMA forward kernel (eta_mlp3_fwd16_kernel) from the fp32
    kernel-view tensors of :func:`pack_mlp3` (same folded W1k / target-scaled w3 / b3)."""
    H = p.hidden
    MT, KC = H // 16, H // 32
    lane = np.arange(64)
    i = lane & 15
    q = lane >> 4
    v = np.arange(8)
    # w2p16[t][c][l][v] = W2[16t + i][32c + (v < 4 ? 4q + v : 16 + 4q + v - 4)]
    kslot = np.where(v < 4, 4 * q[:, None] + v[None, :], 16 + 4 * q[:, None] + (v[None, :] - 4))  # [64,8]
    rows = 16 * np.arange(MT)[:, None, None, None] + i[None, None, :, None]
    cols = 32 * np.arange(KC)[None, :, None, None] + kslot[None, None, :, :]
    w2p = p.w2.numpy()[np.broadcast_to(rows, (MT, KC, 64, 8)), np.broadcast_to(cols, (MT, KC, 64, 8))]
    # w1p16[t][l][v] = W1k[16t + i][4q + v]
    v4 = np.arange(4)
    rows1 = np.broadcast_to(16 * np.arange(MT)[:, None, None] + i[None, :, None], (MT, 64, 4))
    cols1 = np.broadcast_to(4 * q[None, :, None] + v4[None, None, :], (MT, 64, 4))
    w1p = p.w1k.numpy()[rows1, cols1]

    def bf16_bytes(a: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16)
        return t.view(torch.int16).numpy().view(np.uint8).reshape(-1)

    # w3f[tp][l][v] = w3[32tp + kslot[l][v]]: w3 as the (row-broadcast) A operand of the layer-3
    # MFMA of variant 23, in the same k order as the relu(z2) pairs of hidden tiles 2tp, 2tp+1
    w3f = p.w3.numpy()[32 * np.arange(H // 32)[:, None, None] + kslot[None, :, :]]
    parts = [bf16_bytes(w2p), bf16_bytes(w1p),
             p.b2.numpy().astype(np.float32).view(np.uint8).reshape(-1),
             p.w3.numpy().astype(np.float32).view(np.uint8).reshape(-1),
             np.array([p.b3, 0.0, 0.0, 0.0], dtype=np.float32).view(np.uint8),
             bf16_bytes(w3f)]
    blob = torch.from_numpy(np.concatenate(parts).copy())
    assert blob.numel() == blob16_bytes(H)
    return blob


def records_to_tensor(rec: np.ndarray) -> torch.Tensor:
    """numpy EtaRecord array -> int32 [B,4] tensor view (16-byte rows)."""
    rec = np.ascontiguousarray(rec, dtype=RECORD_DTYPE)
    return torch.from_numpy(rec.view(np.int32).reshape(-1, 4))


def records8_to_tensor(rec8: np.ndarray) -> torch.Tensor:
    """numpy compact (8-byte) records -> int32 [B,2] tensor view."""
    rec8 = np.ascontiguousarray(rec8, dtype=RECORD8_DTYPE)
    return torch.from_numpy(rec8.view(np.int32).reshape(-1, 2))


def records6_to_tensor(rec6: np.ndarray) -> torch.Tensor:
    """uint16 [B,3] 6-byte records (features.records_to_compact6) -> int16 [B,3] tensor view."""
    return torch.from_numpy(np.ascontiguousarray(rec6, dtype=np.uint16).view(np.int16))


def featurize6_torch(rec6: torch.Tensor) -> torch.Tensor:
    """PyTorch reference of K1 for 6-byte records: int16 [B,3] -> [B,12] fp32."""
    r = rec6.to(torch.int64) & 0xFFFF
    word = r[:, 0] | (r[:, 1] << 16) | (r[:, 2] << 32)
    w = (word >> 42) & 7
    t = (word >> 45) & 7
    ar = torch.arange(4, device=rec6.device)
    km = (word & ((1 << 27) - 1)).float() * (0.125 * 1e-3)
    return torch.cat([(w[:, None] == ar[None]).float(), (t[:, None] == ar[None]).float(),
                      ((word >> 34) & 7).float()[:, None], ((word >> 37) & 31).float()[:, None],
                      km[:, None], ((word >> 27) & 127).float()[:, None]], 1)


def featurize8_torch(rec8_i32: torch.Tensor) -> torch.Tensor:
    """PyTorch reference of K1 for 8-byte wire records: int32 [B,2] -> [B,12] fp32."""
    dist = rec8_i32[:, 0].view(torch.float32)
    pk = rec8_i32[:, 1].to(torch.int64) & 0xFFFFFFFF
    age = (pk & 0xFFFF).to(torch.int16).view(torch.float16).float()
    w = (pk >> 26) & 7
    t = (pk >> 29) & 7
    hrs = (pk >> 16) & 1023
    ar = torch.arange(4, device=rec8_i32.device)
    return torch.cat([(w[:, None] == ar[None]).float(), (t[:, None] == ar[None]).float(),
                      ((hrs // 24) % 7).float()[:, None], (hrs % 24).float()[:, None],
                      (dist / 1000.0)[:, None], age[:, None]], 1)


def featurize_torch(rec_i32: torch.Tensor) -> torch.Tensor:
    """PyTorch reference of K1 on any device: int32 [B,4] (or compact [B,2]) -> [B,12] fp32."""
    if rec_i32.shape[1] == 2:
        return featurize8_torch(rec_i32)
    if rec_i32.shape[1] == 3:
        return featurize6_torch(rec_i32)
    r = rec_i32
    dist = r[:, 0].view(torch.float32) if r.dtype == torch.int32 else r[:, 0]
    age = r[:, 1].view(torch.float32)
    secs = r[:, 2].to(torch.int64)
    w = r[:, 3] & 0xFF
    t = (r[:, 3] >> 8) & 0xFF
    ar = torch.arange(4, device=r.device)
    oh_w = (w[:, None] == ar[None]).float()
    oh_t = (t[:, None] == ar[None]).float()
    days = torch.div(secs, 86400, rounding_mode="floor")
    sod = secs - days * 86400
    wd = torch.remainder(days + 2, 7).float()
    hr = torch.div(sod, 3600, rounding_mode="floor").float()
    return torch.cat([oh_w, oh_t, wd[:, None], hr[:, None], (dist / 1000.0)[:, None],
                      age[:, None]], 1)


def emulate_kernel(p: PackedMLP3, rec_i32: torch.Tensor, variant: int = -1) -> torch.Tensor:
    """Bit-faithful-ish PyTorch emulation of the kernel numerics (bf16 operands, fp32 acc);
    variant 23 runs layer 3 on MFMA, so relu(z2) and w3 are bf16 there."""
    x = featurize_torch(rec_i32)
    dev = x.device
    sc = torch.tensor(p.norm[:4], device=dev)
    sh = torch.tensor(p.norm[4:], device=dev)
    num = x[:, 8:12] * sc + sh
    hi = num.to(torch.bfloat16).float()
    f = torch.zeros(x.shape[0], 16, device=dev)
    f[:, :8] = x[:, :8]
    f[:, 8] = hi[:, 0]
    f[:, 9] = hi[:, 1]
    f[:, 10] = hi[:, 2]
    f[:, 11] = hi[:, 3]
    f[:, 12] = num[:, 2] - hi[:, 2]
    f[:, 13] = num[:, 3] - hi[:, 3]
    f[:, 14] = 1.0
    f[:, 15] = 1.0
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    h1 = torch.relu(bf(f) @ bf(p.w1k.to(dev)).T)
    h2 = torch.relu(bf(h1) @ bf(p.w2.to(dev)).T + p.b2.to(dev))
    if variant in MFMA_L3_VARIANTS:
        return bf(h2) @ bf(p.w3.to(dev)) + p.b3
    return h2 @ p.w3.to(dev) + p.b3


# variants of the 16x16-MFMA kernel (csrc/eta_mlp_fwd.hip eta_mlp3_fwd16_kernel; bindings.cpp
# fwd16_halves): 16/17/18 = 2/4/1 batch halves, 19 = 2 halves at 12 waves/CU, 20 = 4 halves with
# a scalar-FMA layer-3 epilogue, 21 = 20 software-pipelined across hidden tiles, 22 = 21 with 2 halves,
# 23 = 4 halves with layer 3 on MFMA (relu(z2) and w3 in bf16)
FWD16_VARIANTS = (16, 17, 18, 19, 20, 21, 22, 23)
MFMA_L3_VARIANTS = (23,)


class EtaMlpKernel:
    """A packed MLP resident on one device; ``__call__(records_i32) -> minutes``.

    On a GPU device this ALWAYS runs the HIP kernel (raises if the extension is missing): the
    fused K1+K2 kernel for hidden <= 256, the L2-streamed wide path (ops/mlp_big.py) for 512 and
    1024.  On CPU it runs the fp32 PyTorch model (the reference path).

    ``variant``: -1 auto, 0-8 the 32x32-MFMA kernel's variants (csrc/eta_mlp_fwd.hip
    launch_fwd_h), 16/17/18 the 16x16-MFMA kernel with 2/4/1 batch halves per wave-tile (19: 2 halves at
    12 waves per CU) (its own
    weight blob, :func:`pack_mlp3_16`)."""

    def __init__(self, model: EtaMLP, device: Optional[torch.device] = None, variant: int = -1):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.model_cpu = model.float().cpu().eval()
        self._big = None
        if self.device.type == "cuda" and model.hidden > 256:
            # wide MLPs: W2 no longer fits LDS -> the L2-streamed path (ops/mlp_big.py)
            from .mlp_big import BIG_HIDDEN, EtaMlpBigKernel
            if model.hidden not in BIG_HIDDEN:
                raise ValueError(f"HIP MLP kernels support hidden in (64, 128, 256, 512, 1024), "
                                 f"got {model.hidden}")
            self._big = EtaMlpBigKernel(self.model_cpu, self.device)
            self.hidden = model.hidden
            self.variant = variant
            self.packed = pack_mlp3(self.model_cpu)
            self.blob16 = None
            self._C = self._big._C
            return
        self.packed = pack_mlp3(self.model_cpu).to(self.device)
        self.hidden = model.hidden
        self.variant = variant
        # auto (-1): batches of >= AUTO16_MIN_ROWS rows run the 16x16-MFMA kernel with 4 batch
        # halves per wave-tile (variant 17: +4-10 % over the 32x32 kernel's best variant on 16M
        # rows, profiles/eta_fwd16_r1h.jsonl); smaller ones the 32x32 kernel's auto choice
        self.blob16 = (pack_mlp3_16(pack_mlp3(self.model_cpu)).to(self.device)
                       if self.device.type == "cuda" and (variant in FWD16_VARIANTS or variant == -1)
                       else None)
        self._C = _ext.native(required=True) if self.device.type == "cuda" else None
        if self.device.type == "cuda" and self.hidden not in (64, 128, 256):
            raise ValueError(f"HIP MLP kernel supports hidden in (64,128,256), got {self.hidden}")

    def forward_hostio(self, rec_pinned: torch.Tensor, out_pinned: torch.Tensor) -> None:
        """Zero-copy scoring: the kernel reads pinned host records and writes pinned host minutes
        directly over PCIe (asynchronous on the current stream; synchronize before reading)."""
        if self._big is not None:
            return self._big.forward_hostio(rec_pinned, out_pinned)
        v = self._pick(rec_pinned.shape[0])
        self._C.eta_mlp3_forward_hostio(rec_pinned, out_pinned, self._blob(v), self.hidden,
                                        self.packed.norm, v)

    AUTO16_MIN_ROWS = 1 << 17
    # large batches: 4 batch halves per wave-tile, scalar-FMA fp32 layer 3 (variant 20: 1-2 %
    # ahead of the packed-FMA 17, profiles/eta_fwd16_epilogue_ab_r2.jsonl; variant 23, layer 3 on
    # MFMA, is 2.5 % faster still but rounds relu(z2) and w3 to bf16, profiles/eta_fwd16_pmc_r2.md)
    AUTO16_VARIANT = 20

    def _pick(self, rows: int) -> int:
        if self.variant == -1 and rows >= self.AUTO16_MIN_ROWS:
            return self.AUTO16_VARIANT
        return self.variant

    def _blob(self, variant: int) -> torch.Tensor:
        return self.blob16 if variant in FWD16_VARIANTS else self.packed.blob

    def __call__(self, rec: torch.Tensor) -> torch.Tensor:
        if self._big is not None:
            return self._big(rec)
        if self.device.type == "cuda":
            v = self._pick(rec.shape[0])
            return self._C.eta_mlp3_forward(rec, self._blob(v), self.hidden, self.packed.norm, v)
        with torch.no_grad():
            return self.model_cpu(featurize_torch(rec))


class ResidentScorer:
    """The resident single-request scorer (``csrc/persistent_serve.hip``) for one packed MLP: a
    persistent 8-wave workgroup keeps the weights in LDS and takes rounds of up to ``cap``
    16-byte records through a doorbell in pinned host memory — no kernel dispatch and no stream
    synchronisation per request.  It exits after ``idle_ms`` without work or ``life_ms`` of
    residency and is relaunched on demand.  :meth:`score` returns ``None`` when it did not answer
    (the caller then launches the normal kernel); call :meth:`park` before large launches on the
    same GPU."""

    def __init__(self, kernel: "EtaMlpKernel", cap: int = 1024, idle_ms: float = 20.0,
                 life_ms: float = 50.0):
        self._C = kernel._C
        self.cap = cap
        self.h: Optional[int] = self._C.pscore_create(kernel.packed.blob, kernel.hidden,
                                                      list(kernel.packed.norm), cap, idle_ms, life_ms)
        _RESIDENT.add(self)

    def score(self, rec_i32: torch.Tensor, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        n = rec_i32.shape[0]
        if self.h is None or n > self.cap:
            return None
        out = torch.empty(n, dtype=torch.float32) if out is None else out
        return out if self._C.pscore_score(self.h, rec_i32, out) else None

    def park(self) -> None:
        if self.h is not None:
            self._C.pscore_park(self.h)

    def stats(self) -> dict:
        if self.h is None:
            return {}
        l, s, f = self._C.pscore_stats(self.h)
        return {"launches": l, "served": s, "fallbacks": f}

    def close(self) -> None:
        if self.h is not None:
            self._C.pscore_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


def _close_all_resident() -> None:  # pragma: no cover - exit path
    """atexit: stop every live resident scorer before the HIP runtime is torn down."""
    for o in list(_RESIDENT):
        try:
            o.close()
        except Exception:
            pass


import atexit as _atexit  # noqa: E402
import weakref as _weakref  # noqa: E402

_RESIDENT: "_weakref.WeakSet[ResidentScorer]" = _weakref.WeakSet()
_atexit.register(_close_all_resident)
