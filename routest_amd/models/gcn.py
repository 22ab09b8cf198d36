"""2-layer GCN road-graph route scorer (north-star config 4).

Per node v a learned *delay factor* (>= 0.5) from the road graph's structure::

    H1 = relu(Â X W1 + b1);  Z = H1 W2;  delay = 0.5 + softplus((Â Z + b2) . wo + bo)

and a candidate route is scored by its delay-weighted length  sum_i delay(v_i) * |v_i v_{i+1}|
(lower is better).  :class:`GcnScorer` is the fp32 PyTorch reference (torch.sparse CSR);
:class:`GcnScorerHip` runs the same math through the gfx950 kernels of ``csrc/gcn.hip`` with two
multi-GPU modes:

* ``replicate``: every rank holds the graph and computes all node delays (no communication);
  the candidate routes are sharded.
* ``partition``: rank r computes layer 1 and the layer-2 transform for its contiguous node range
  only, then ONE ``all_gather`` of Z (N x 32 bf16 = 6.4 MB at 100k nodes, 0.8 MB per rank) before
  the layer-2 aggregation, and one all_gather of the delays (0.4 MB).  With a
  :class:`~routest_amd.parallel.comm.DeviceComm` both gathers are issued in place on the current
  stream (one-shot IPC over xGMI when the shard fits its buffers, else RCCL); without one they go
  through ``torch.distributed.all_gather_into_tensor``.
"""
from __future__ import annotations

import os

from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from ..data.graph import RoadGraph


class GcnScorer(nn.Module):
    def __init__(self, fin: int = 32, fhid: int = 128, fz: int = 32, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.W1 = nn.Parameter(torch.randn(fin, fhid, generator=g) / fin ** 0.5)
        self.b1 = nn.Parameter(torch.randn(fhid, generator=g) * 0.1)
        self.W2 = nn.Parameter(torch.randn(fhid, fz, generator=g) / fhid ** 0.5)
        self.b2 = nn.Parameter(torch.randn(fz, generator=g) * 0.1)
        self.wo = nn.Parameter(torch.randn(fz, generator=g) / fz ** 0.5)
        self.bo = nn.Parameter(torch.zeros(()))

    @staticmethod
    def adjacency(g: RoadGraph) -> torch.Tensor:
        return torch.sparse_csr_tensor(torch.from_numpy(g.gcn_indptr.astype(np.int64)),
                                       torch.from_numpy(g.gcn_indices.astype(np.int64)),
                                       torch.from_numpy(g.gcn_values), size=(g.num_nodes, g.num_nodes))

    def forward(self, A: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        h1 = torch.relu(torch.sparse.mm(A, X) @ self.W1 + self.b1)
        z = h1 @ self.W2
        e = torch.sparse.mm(A, z) + self.b2
        return 0.5 + torch.nn.functional.softplus(e @ self.wo + self.bo)


def score_routes_ref(g: RoadGraph, delay: np.ndarray, routes: Sequence[Sequence[int]]) -> np.ndarray:
    from ..routing.providers import haversine_m
    out = np.zeros(len(routes), dtype=np.float64)
    lat = g.lat.astype(np.float32).astype(np.float64)
    lon = g.lon.astype(np.float32).astype(np.float64)
    for i, r in enumerate(routes):
        r = np.asarray(r)
        if len(r) > 1:
            d = haversine_m(lat[r[:-1]], lon[r[:-1]], lat[r[1:]], lon[r[1:]])
            out[i] = float((delay[r[:-1]] * d).sum())
    return out


def pack_b_frags(W: torch.Tensor) -> torch.Tensor:
    """W [K, N] -> bf16 B fragments [N/32][K/16][64 lanes][8]: lane l holds W[16ks+8(l>>5)+j][32nt+(l&31)]."""
    K, N = W.shape
    KS, NT = K // 16, N // 32
    lane = np.arange(64)
    j = np.arange(8)
    k = 16 * np.arange(KS)[None, :, None, None] + 8 * (lane >> 5)[None, None, :, None] + j[None, None, None, :]
    n = 32 * np.arange(NT)[:, None, None, None] + (lane & 31)[None, None, :, None]
    k, n = np.broadcast_arrays(k, n)
    return W.detach().float().cpu()[torch.from_numpy(k), torch.from_numpy(n)].to(torch.bfloat16).contiguous()


def routes_to_csr(routes: Sequence[Sequence[int]]):
    ptr = np.zeros(len(routes) + 1, dtype=np.int32)
    ptr[1:] = np.cumsum([len(r) for r in routes])
    nodes = np.concatenate([np.asarray(r, dtype=np.int32) for r in routes]) if routes else np.zeros(0, np.int32)
    return ptr, nodes


class GcnScorerHip:
    def __init__(self, model: GcnScorer, g: RoadGraph, device: torch.device, mode: str = "replicate",
                 rank: int = 0, world: int = 1, group=None, comm=None):
        from ..ops import _ext
        self.C = _ext.native(required=True)
        self.dev = d = torch.device(device)
        self.g = g
        self.N = g.num_nodes
        self.mode = mode
        self.rank, self.world, self.group, self.comm = rank, world, group, comm
        self.X = torch.from_numpy(g.features).to(torch.bfloat16).to(d)
        self.indptr = torch.from_numpy(g.gcn_indptr).to(d)
        self.indices = torch.from_numpy(g.gcn_indices).to(d)
        self.values = torch.from_numpy(g.gcn_values).to(d)
        self.w1 = pack_b_frags(model.W1).to(d)
        self.w2 = pack_b_frags(model.W2).to(d)
        self.b1 = model.b1.detach().float().to(d)
        self.b2 = model.b2.detach().float().to(d)
        self.wo = model.wo.detach().float().to(d)
        self.bo = float(model.bo.detach())
        self.fhid = model.W1.shape[1]
        self.fz = model.W2.shape[1]
        if mode == "partition" and world > 1:
            # shard rows rounded up to 4 nodes: every shard of Z and of the delays starts 16-byte
            # aligned and is a 16-byte multiple (one-shot all-gather requirement)
            per = ((self.N + world - 1) // world + 3) // 4 * 4
            self.rows = (rank * per, min(self.N, (rank + 1) * per))
            self.per = per
        else:
            self.rows = (0, self.N)
            self.per = self.N
        npad = self.per * (world if mode == "partition" and world > 1 else 1)
        # fused layer 1 (csrc/gcn.hip gcn_l1_fused_kernel) for the 32 -> 128 -> 32 scorer;
        # ROUTEST_GCN_FUSED=0 selects the two-launch path (H1 materialised in HBM)
        self.fused = (self.X.shape[1], self.fhid, self.fz) == (32, 128, 32) and \
            os.environ.get("ROUTEST_GCN_FUSED", "1") != "0"
        self.H1 = None
        self.Z = torch.empty(npad, self.fz, dtype=torch.bfloat16, device=d)
        self.delay = torch.zeros(npad, dtype=torch.float32, device=d)
        self.lat = torch.from_numpy(g.lat.astype(np.float32)).to(d)
        self.lon = torch.from_numpy(g.lon.astype(np.float32)).to(d)
        # one 8-byte gather per route node in route_score_kernel
        self.latlon = torch.stack([self.lat, self.lon], 1).contiguous()

    def node_delays(self) -> torch.Tensor:
        C, (r0, r1) = self.C, self.rows
        if self.fused:
            # aggregation + W1 + ReLU + W2 in one launch; H1 never leaves LDS
            C.gcn_l1_fused(self.X, self.indptr, self.indices, self.values, self.w1, self.b1, self.w2,
                           self.Z, r0, r1)
        else:
            if self.H1 is None:
                self.H1 = torch.empty(self.Z.shape[0], self.fhid, dtype=torch.bfloat16, device=self.dev)
            C.gcn_agg_gemm(self.X, self.indptr, self.indices, self.values, self.w1, self.b1, self.H1,
                           self.X.shape[1], self.fhid, True, True, r0, r1)
            C.gcn_agg_gemm(self.H1, self.indptr, self.indices, self.values, self.w2, None, self.Z,
                           self.fhid, self.fz, False, False, r0, r1)
        if self.mode == "partition" and self.world > 1:
            self._gather(self.Z)
        C.gcn_spmm_score(self.Z, self.indptr, self.indices, self.values, self.b2, self.wo, self.bo,
                         self.delay, r0, r1)
        if self.mode == "partition" and self.world > 1:
            self._gather(self.delay)
        return self.delay[:self.N]

    def _gather(self, full: torch.Tensor) -> None:
        """In-place all-gather of this rank's row shard of ``full`` (rows [rank*per, (rank+1)*per))."""
        r0 = self.rank * self.per
        own = full[r0:r0 + self.per]
        if self.comm is not None:
            self.comm.all_gather(own, full)
        else:
            import torch.distributed as dist
            if dist.get_backend(self.group) == "gloo":
                # the shared-GPU rehearsal (every rank on one device, gloo rendezvous): staged
                # through host memory; the driver's one-rank-per-GPU runs take the RCCL branch
                h = torch.empty((full.shape[0],) + tuple(full.shape[1:]), dtype=full.dtype)
                dist.all_gather_into_tensor(h, own.cpu(), group=self.group)
                full.copy_(h)
            else:
                dist.all_gather_into_tensor(full, own.clone(), group=self.group)

    def score_routes(self, rptr: torch.Tensor, nodes: torch.Tensor) -> torch.Tensor:
        return self.C.route_score(rptr, nodes, self.latlon, self.delay)
