"""Fused HIP trainer for the ETA MLP (K3) — one rank of data-parallel training.

Per step (all on the current HIP stream, no host synchronisation, HIP-graph capturable):

  eta_mlp3_train_fwd (HIP)  : featurize + layer 1 + ONE pass over layer 2 (relu(z2) kept packed
                            in registers) + layer 3 + MSE grad; G[w3|b3] = dy^T [h2|1] as one fp32
                            row per workgroup (relu(z2) transposed exactly on the MFMA); writes xf
                            and the dz2 fragments (512 B/row) in train_bwd's A-operand order
  G[W2|b2], G[W1k|b1]       : train_bwd (HIP, K = batch): dgrad dh1 = dz2 W2 against an LDS image
                            of W2, relu'(z1) from h1 recomputed on the layer-1 MFMA (h1 is never
                            stored), dW2|db2 and dW1 register-resident over a k-slice; fp32 slabs
                            in the bucket layout, then ONE deterministic reduction of the three
                            slab regions into G
  all_reduce(G)             : ONE RCCL collective (SUM; dy was pre-scaled by 2/global_batch)
  adamw_pack (HIP)          : AdamW on fp32 master params + re-pack of the training blob
No library GEMM runs in the step (csrc/eta_mlp_train.hip).

Training runs in normalised-target space (y' = (y - y_mean)/y_std); :meth:`to_model` writes the
learned weights back into an :class:`EtaMLP` whose buffers carry the scaling.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch

from ..models.mlp3 import EtaMLP
from ..ops import _ext

from ..parallel.dp import allreduce_flat


def flatten_params(model: EtaMLP) -> torch.Tensor:
    H = model.hidden
    parts = [model.l1.weight.detach().reshape(-1), model.l1.bias.detach(),
             model.l2.weight.detach().reshape(-1), model.l2.bias.detach(),
             model.l3.weight.detach().reshape(-1), model.l3.bias.detach()]
    flat = torch.cat([p.float().cpu() for p in parts])
    assert flat.numel() == H * H + 15 * H + 1
    return flat


@torch.no_grad()
def unflatten_into(model: EtaMLP, flat: torch.Tensor) -> None:
    H = model.hidden
    f = flat.detach().float().cpu()
    o = 0
    for t, n in ((model.l1.weight, 12 * H), (model.l1.bias, H), (model.l2.weight, H * H),
                 (model.l2.bias, H), (model.l3.weight, H), (model.l3.bias, 1)):
        t.copy_(f[o:o + n].view_as(t))
        o += n


def hperm(H: int) -> torch.Tensor:
    """Stored hidden-unit order of the fused trainer's activations and gradient bucket (unit u at
    column u with bits 2 and 3 swapped: one 16-byte store per lane, csrc/eta_mlp_train.hip)."""
    u = torch.arange(H)
    return (u & ~12) | ((u & 4) << 1) | ((u & 8) >> 1)


def grads_from_bucket(G: torch.Tensor, H: int):
    """Python mirror of adamw_pack_kernel's bucket -> parameter-gradient mapping (tests)."""
    G = G.detach().float().cpu()
    ldg = H + 16
    pm = hperm(H)
    cols = torch.cat([pm, torch.arange(H, ldg)])
    gW2a = G[:H * ldg].view(H, ldg)[pm][:, cols]
    gW3a = G[H * ldg:H * ldg + ldg][cols]
    gW1a = G[H * ldg + ldg:].view(H, 16)[pm]
    gW1 = gW1a[:, :12].clone()
    gW1[:, 10] += gW1a[:, 12]
    gW1[:, 11] += gW1a[:, 13]
    return {"l1.weight": gW1, "l1.bias": gW1a[:, 14].clone(), "l2.weight": gW2a[:, :H].clone(),
            "l2.bias": gW2a[:, H].clone(), "l3.weight": gW3a[:H].view(1, H).clone(),
            "l3.bias": gW3a[H:H + 1].clone()}


def _w2off(row: np.ndarray, col: np.ndarray) -> np.ndarray:
    """Byte offset of W2[row][col] in the training blob's W2 image (eta_mlp_train.hip w2off:
    512-byte rows, 8-byte chunk k of row R at chunk k ^ w2swz(R))."""
    swz = ((row & 3) << 3) | ((row >> 2) & 7)
    return row * 512 + (((col >> 2) ^ swz) << 3) + 2 * (col & 3)


@torch.no_grad()
def _w2frag_index(u2: np.ndarray, u1: np.ndarray, H: int) -> np.ndarray:
    """bf16 index of W2[u2][u1] in train_bwd_kernel's B-fragment image (eta_mlp_train.hip
    w2frag_index): fragment (u1 // 32, u2 // 16), lane u1 % 32 + 32 h, element j."""
    KS = H // 16
    nb, n, ks, r = u1 >> 5, u1 & 31, u2 >> 4, u2 & 15
    hh, j = (r >> 2) & 1, 4 * (r >> 3) + (r & 3)
    return ((nb * KS + ks) * 64 + n + 32 * hh) * 8 + j


def pack_train_blob(model: EtaMLP) -> torch.Tensor:
    """Host mirror of adamw_pack_kernel(update=False): the training blob of ``model`` — the W2
    image (natural order, swizzled 8-byte chunks) followed by the inference blob's
    w1p | b1p | b2p | w3p | tail (target scale as in the model's buffers), then the backward's
    W2 B-fragment image."""
    from ..ops.eta_mlp import pack_mlp3
    H = model.hidden
    inf = pack_mlp3(model).blob.numpy()
    W2 = model.l2.weight.detach().float().cpu().to(torch.bfloat16).view(torch.int16).numpy()
    img = np.zeros(H * 512, dtype=np.uint8)
    o, c = np.meshgrid(np.arange(H), np.arange(H), indexing="ij")
    src = W2[o, c]
    off = _w2off(o, c)
    img.view(np.int16)[(off // 2).reshape(-1)] = src.reshape(-1)
    tail = inf[2 * H * H:]                   # w1p | b1p | b2p | w3p | tail of the inference blob
    frag = np.zeros(H * H, dtype=np.int16)
    frag[_w2frag_index(o, c, H).reshape(-1)] = src.reshape(-1)
    return torch.from_numpy(np.concatenate([img, tail, frag.view(np.uint8)]))


class FusedMlp3Trainer:
    """One rank of data-parallel training on the hand-written kernels.  H in (64, 128, 256) runs
    the fused LDS-resident step below; H in (512, 1024) is dispatched to
    :class:`FusedMlp3TrainerBig` (L2-streamed GEMMs, csrc/mlp_big.hip)."""

    def __new__(cls, model: EtaMLP, *args, **kw):
        if cls is FusedMlp3Trainer and model.hidden in (512, 1024):
            return super().__new__(FusedMlp3TrainerBig)
        return super().__new__(cls)

    def __init__(self, model: EtaMLP, device: torch.device, batch_local: int, global_batch: int,
                 lr: float = 2e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 warmup: int = 0, total_steps: int = 0, min_lr_ratio: float = 0.1,
                 allreduce: bool = True, comm=None):
        if model.hidden not in self.SUPPORTED:
            raise ValueError(f"{type(self).__name__} supports hidden in {self.SUPPORTED}")
        self.C = _ext.native(required=True)
        self.model = model
        self.H = H = model.hidden
        self.dev = torch.device(device)
        self.B = batch_local
        self.global_batch = global_batch
        self.hp = dict(lr=lr, beta1=betas[0], beta2=betas[1], eps=eps, wd=weight_decay, warmup=warmup,
                       total_steps=total_steps, min_lr_ratio=min_lr_ratio)
        self.allreduce = allreduce
        self.comm = comm          # parallel.comm.DeviceComm: native RCCL / one-shot all-reduce
        xs = model.x_std.float().cpu()
        xm = model.x_mean.float().cpu()
        if (xm[:8] != 0).any() or (xs[:8] != 1).any():
            raise ValueError("one-hot features must not be normalised")
        self.norm = (1.0 / xs[8:12]).tolist() + (-xm[8:12] / xs[8:12]).tolist()
        self.y_mean = float(model.y_mean)
        self.y_std = float(model.y_std)
        d = self.dev
        bf = torch.bfloat16
        self.P = flatten_params(model).to(d)
        self.M = torch.zeros_like(self.P)
        self.V = torch.zeros_like(self.P)
        self.G = torch.zeros(self.C.mlp3_grad_bucket_floats(H), dtype=torch.float32, device=d)
        ldg = H + 16
        self.gW2a = self.G[:H * ldg].view(H, ldg)
        self.gW3a = self.G[H * ldg:H * ldg + ldg].view(1, ldg)
        self.gW1a = self.G[H * ldg + ldg:].view(H, 16)
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=d)
        self._alloc(batch_local)
        self._pack(update=False)

    SUPPORTED = (64, 128, 256)

    def _slices(self, B: int, cap_bytes: int = 0) -> int:
        """Split-K slices of the wgrad kernels: one per CU (256 batch rows each), bounded by
        ``cap_bytes`` of fp32 slabs."""
        ncu = self.C.num_cus(self.dev.index if self.dev.index is not None else 0)
        rows = int(os.environ.get("ROUTEST_WGRAD_ROWS", "256"))     # batch rows per k-slice
        S = max(1, min(ncu, B // rows))
        if cap_bytes:
            S = max(1, min(S, cap_bytes // (4 * self.G.numel())))
        return S

    def _alloc(self, B: int) -> None:
        d, H, bf = self.dev, self.H, torch.bfloat16
        self.blob = torch.zeros(self.C.eta_mlp3_train_blob_bytes(H), dtype=torch.uint8, device=d)
        tiles = (B + 31) // 32
        # feature rows padded to whole 32-row tiles; the pad rows stay zero (the forward only
        # writes rows < B), so the backward's tail tile contributes nothing
        self.xf = torch.zeros(tiles * 32, 16, dtype=bf, device=d)
        # dz2 fragments in train_bwd's A-operand order (per 32-row tile: H/16 x 64 lanes x 16 B):
        # with xf, all the activations that leave the forward kernel
        self.dz2r = torch.empty(tiles * 32 * H, dtype=bf, device=d)
        ldg = H + 16
        # k-slices of the backward kernel (one workgroup per CU at most): dW2|db2 and dW1 partials
        # per slice; dW3|db3 arrives as one row per forward workgroup (w3slab)
        self.S = self.C.train_wgrad_slices(B, d.index or 0, H)
        self.slab2 = torch.empty(self.S, H * ldg, dtype=torch.float32, device=d)
        self.slab = torch.empty(self.S, H * 16, dtype=torch.float32, device=d)
        self.w3slab = torch.empty(self.C.train_fwd_grid(B, d.index or 0), ldg, dtype=torch.float32,
                                  device=d)
        self.sq_err = torch.zeros(B, dtype=torch.float32, device=d)      # per-row squared errors
        self.loss_tiles = self.sq_err                                      # (older name)

    def _pack(self, update: bool) -> None:
        h = self.hp
        self.C.adamw_pack(self.P, self.G, self.M, self.V, self.blob, self.step_ctr, self.H,
                          h["lr"], h["beta1"], h["beta2"], h["eps"], h["wd"], h["warmup"],
                          h["total_steps"], h["min_lr_ratio"], update)

    def normalize_targets(self, y: torch.Tensor) -> torch.Tensor:
        return ((y.float() - self.y_mean) / self.y_std).contiguous()

    def forward_backward(self, rec: torch.Tensor, tgt_norm: torch.Tensor) -> None:
        """Fills the flat gradient bucket G (local contribution, pre-scaled for the global mean)."""
        C, H = self.C, self.H
        C.eta_mlp3_train_fwd(rec, tgt_norm, self.blob, H, self.norm, 2.0 / self.global_batch,
                             self.xf, self.w3slab, self.dz2r, self.sq_err, self.step_ctr)
        ldg = H + 16
        C.train_bwd(self.xf, rec.shape[0], self.blob, H, self.dz2r, self.slab2, self.slab)
        C.wgrad_reduce(self.slab2, self.G[:H * ldg], self.slab, self.G[H * ldg + ldg:],
                       self.w3slab, self.G[H * ldg:H * ldg + ldg], perm_h=H)   # dW2 slabs: register-native

    def _local_only(self) -> bool:
        """No gradient communication this step: no device comm, and all-reduce off or one rank."""
        if self.comm is not None:
            return False
        if not self.allreduce:
            return True
        import torch.distributed as dist
        return not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)

    def step(self, rec: torch.Tensor, tgt_norm: torch.Tensor) -> torch.Tensor:
        """One optimizer step; returns the device tensor of per-row squared errors (no sync).
        Without gradient communication the slab reduction and AdamW run as ONE kernel
        (reduce_adamw: same sums, same update, same bits as wgrad_reduce + adamw_pack);
        ``ROUTEST_FUSED_ADAMW=0`` keeps them apart."""
        if type(self) is FusedMlp3Trainer and self._local_only() and \
                os.environ.get("ROUTEST_FUSED_ADAMW", "1") != "0":
            C, H, h = self.C, self.H, self.hp
            C.eta_mlp3_train_fwd(rec, tgt_norm, self.blob, H, self.norm, 2.0 / self.global_batch,
                                 self.xf, self.w3slab, self.dz2r, self.sq_err, self.step_ctr)
            C.train_bwd(self.xf, rec.shape[0], self.blob, H, self.dz2r, self.slab2, self.slab)
            C.reduce_adamw(self.slab2, self.slab, self.w3slab, self.P, self.G, self.M, self.V, self.blob,
                           self.step_ctr, H, h["lr"], h["beta1"], h["beta2"], h["eps"], h["wd"],
                           h["warmup"], h["total_steps"], h["min_lr_ratio"])
            return self.sq_err
        self.forward_backward(rec, tgt_norm)
        if self.comm is not None:
            self.comm.all_reduce(self.G)
        elif self.allreduce:
            allreduce_flat(self.G, average=False)
        self._pack(update=True)
        return self.sq_err

    def local_mse(self) -> float:
        return float(self.sq_err.sum().item()) / self.B

    @torch.no_grad()
    def to_model(self) -> EtaMLP:
        unflatten_into(self.model, self.P)
        return self.model

    def optimizer_state(self) -> dict:
        return {"exp_avg": self.M.detach().cpu(), "exp_avg_sq": self.V.detach().cpu(),
                "step": self.step_ctr.detach().cpu().to(torch.int64)}

    def load_optimizer_state(self, st: dict) -> None:
        self.M.copy_(st["exp_avg"].to(self.dev))
        self.V.copy_(st["exp_avg_sq"].to(self.dev))
        self.step_ctr.copy_(st["step"].to(torch.int32).to(self.dev))

    def set_params(self, flat: torch.Tensor) -> None:
        self.P.copy_(flat.to(self.dev))
        self._pack(update=False)


class FusedMlp3TrainerBig(FusedMlp3Trainer):
    """Wide MLPs (H = 512, 1024): W2 is 0.5 / 2 MiB, so it no longer lives in LDS.  Per step, all
    on the current stream (no host sync, HIP-graph capturable):

      big_layer1        : featurize + layer 1 -> xf, h1a (hperm order, ones column)
      gemm_nt(H2Y)      : z2 = W2 h1 (W2 streamed from L2 through LDS tiles) -> h2a = relu(z2 + b2)
                          + per-64-unit partials of h2 . w3
      big_dz2y          : y, dy (scaled 2/global_batch), squared errors, dz2 = dy w3 relu'(z2) and
                          the dW3|db3 split-K slab rows, h2a streamed once
      gemm_dgrad_dw1    : dh1 = dz2 W2 (W2^T operand, kept by the optimizer kernel), consumed in its
                          epilogue: per 256-row tile the dW1 partial (dh1 * relu'(h1))^T x (dh1 is
                          never stored)
      wgrad256 + reduce : dW2|db2 on 256 x 256 output tiles; one deterministic slab reduction
      all_reduce(G)     : one collective on the flat bucket (C1: 4.3 MB at H = 1024)
      adamw_pack_big    : AdamW + re-pack of w1p / w2k / w2t / b2 / w3 / b3
    """

    SUPPORTED = (512, 1024)

    def _alloc(self, B: int) -> None:
        d, H, bf = self.dev, self.H, torch.bfloat16
        ldg = H + 16
        self.w1p = torch.zeros(H * 16, dtype=bf, device=d)
        self.w2k = torch.zeros(H, H, dtype=bf, device=d)
        self.w2t = torch.zeros(H, H, dtype=bf, device=d)
        self.b2v = torch.zeros(H, dtype=torch.float32, device=d)
        self.w3v = torch.zeros(H, dtype=torch.float32, device=d)
        self.b3v = torch.zeros(1, dtype=torch.float32, device=d)
        self.xf = torch.empty(B, 16, dtype=bf, device=d)
        self.h1a = torch.empty(B, ldg, dtype=bf, device=d)
        self.h2a = torch.zeros(B, ldg, dtype=bf, device=d)
        self.h2a[:, H] = 1.0                 # ones column (db3 input); kernels never write it
        self.dz2 = torch.empty(B, H, dtype=bf, device=d)
        # dW1 in the dgrad GEMM's epilogue (default; ROUTEST_DW1_EPILOGUE=0: dh1 stored, then a masked
        # wgrad launch): one [H][16] partial per 256-row tile, dh1 never written
        self.dw1_epi = hasattr(self.C, "gemm_dgrad_dw1") and os.environ.get("ROUTEST_DW1_EPILOGUE", "1") != "0"
        if self.dw1_epi:
            self.slab1w = torch.empty((B + 255) // 256, 16 * H, dtype=torch.float32, device=d)
            # relu'(z1) as bits (big_layer1 writes them): 16x less mask traffic than re-reading h1a
            self.h1bits = torch.empty((B + 31) // 32 * 32, H // 32, dtype=torch.int32, device=d)
            self.dh1 = None
        else:
            self.dh1 = torch.empty(B, H, dtype=bf, device=d)
        self.dyb = torch.empty(B, 8, dtype=bf, device=d)
        self.dy = torch.empty(B, dtype=torch.float32, device=d)
        self.ypart = torch.empty(B, H // 64, dtype=torch.float32, device=d)
        self.sq_err = torch.zeros(B, dtype=torch.float32, device=d)
        self.loss_tiles = self.sq_err
        # dW2|db2 ([H, H+16], 4.3 MB at H = 1024) in ONE wgrad launch: ceil(tiles / 9) n-blocks x
        # H/256 m-blocks per k-slice, and only as many k-slices as fill ~one workgroup per CU —
        # 16 slices at H = 1024 (68 MB of slabs) instead of a whole-bucket slab per 256 rows
        ntt = (ldg + 31) // 32
        self.nsplit2 = -(-ntt // 9)
        nt = -(-ntt // self.nsplit2)
        nblk = -(-ntt // nt)
        ncu = self.C.num_cus(d.index if d.index is not None else 0)
        # the 256 x 256 output-tile kernel (wgrad.hip wgrad256_kernel): (H/256)^2 tiles per k-slice and
        # enough slices for one workgroup per CU; db2 rides along.  Default since run r6g: 159-173 us
        # against 214 us for the n-blocked wgrad_kernel at H = 1024, 64k rows (profiles/wgrad256_r6.md);
        # ROUTEST_WGRAD256=0 keeps the latter
        self.wg256 = (H % 256 == 0 and B % 64 == 0 and hasattr(self.C, "wgrad256") and
                      os.environ.get("ROUTEST_WGRAD256", "1") == "1")
        if self.wg256:
            self.S2 = max(1, min(B // 64, ncu // ((H // 256) ** 2)))
            # (zeros: the bucket's pad columns H+1 .. H+15 are never written by the kernel)
            self.slab2 = torch.zeros(self.S2, H * ldg, dtype=torch.float32, device=d)
        else:
            self.S2 = max(1, min(B // 256, ncu // (nblk * (H // 256))))
            self.slab2 = torch.empty(self.S2, H * ldg, dtype=torch.float32, device=d)
        # dW3|db3 and dW1 (small outputs): one k-slice per CU
        self.S = self._slices(B)
        self.slab = torch.empty(self.S, self.G.numel() - H * ldg, dtype=torch.float32, device=d)

    def _pack(self, update: bool) -> None:
        h = self.hp
        self.C.adamw_pack_big(self.P, self.G, self.M, self.V, self.w1p, self.w2k, self.w2t, self.b2v,
                              self.w3v, self.b3v, self.step_ctr, self.H, h["lr"], h["beta1"],
                              h["beta2"], h["eps"], h["wd"], h["warmup"], h["total_steps"],
                              h["min_lr_ratio"], update)

    def forward_backward(self, rec: torch.Tensor, tgt_norm: torch.Tensor) -> None:
        C, H, B = self.C, self.H, rec.shape[0]
        ldg = H + 16
        assert B == self.B, "wide trainer: batch must equal batch_local"
        C.big_layer1(rec, self.w1p, H, self.norm, self.h1a, self.xf, self.h1bits if self.dw1_epi else None)
        C.gemm_nt(1, self.w2k, self.h1a, H, B, H, b2=self.b2v, w3=self.w3v, ypart=self.ypart,
                  out=self.h2a)
        # dy / dyb / squared error + dz2 + the device step counter: one launch
        # ... and dW3|db3 = [h2|1]^T dy into the slab's first H + 16 columns (h2a streamed once)
        C.big_dz2y(self.ypart, H // 64, self.b3v, tgt_norm, 2.0 / self.global_batch, self.dy,
                   self.dyb, self.sq_err, self.h2a, self.w3v, H, self.dz2, self.step_ctr, self.slab)
        if self.dw1_epi:
            C.gemm_dgrad_dw1(self.w2t, self.dz2, H, B, H, self.h1bits, self.xf, self.slab1w)
        else:
            C.gemm_nt(2, self.w2t, self.dz2, H, B, H, out=self.dh1)
        # dW2|db2 = dz2^T [h1|1]: 256 x 256 output tiles (db2 as per-tile-column partial sums folded by
        # the reduce), or one launch of n-blocks of <= 288 columns
        if self.wg256:
            C.wgrad256(self.dz2, self.h1a, H, H, self.slab2, ldg, H)
        else:
            C.wgrad(self.dz2, H, H, self.h1a, ldg, self.slab2, 0, ldg, nsplit=self.nsplit2)
        if self.dw1_epi:
            # dh1 consumed by the dgrad GEMM's epilogue (gemm_dgrad_dw1 above): dW3|db3 from the slab's
            # first ldg columns, dW1 from the per-row-tile partials
            C.wgrad_reduce(self.slab2, self.G[:H * ldg], self.slab, self.G[H * ldg:H * ldg + ldg],
                           self.slab1w, self.G[H * ldg + ldg:],
                           fold_ld=ldg if self.wg256 else 0, fold_col=H if self.wg256 else 0)
            return
        # dW1 = (dh1 * relu'(h1))^T x: dh1 and its mask h1a are both in the hperm order here
        C.wgrad(self.dh1, H, H, self.xf, 16, self.slab, ldg, 16, self.h1a)
        C.wgrad_reduce(self.slab2, self.G[:H * ldg], self.slab, self.G[H * ldg:],
                       fold_ld=ldg if self.wg256 else 0, fold_col=H if self.wg256 else 0)


def lr_at(step: int, lr: float, warmup: int, total: int, min_ratio: float) -> float:
    """Host mirror of adamw_pack_kernel's schedule (for the autograd path and tests)."""
    t = max(1, step)
    out = lr
    if warmup > 0 and t < warmup:
        out *= t / warmup
    if total > 0 and t > warmup:
        prog = min(1.0, (t - warmup) / max(1.0, total - warmup))
        out *= min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * prog))
    return out
