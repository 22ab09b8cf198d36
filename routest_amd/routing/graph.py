"""Road-graph routing: learned edge costs + batched A* (K9) + a directions provider.

* :func:`edge_costs` — travel time per edge from the ETA MLP: every directed edge becomes one
  request record (distance = edge length, plus the trip context: weather, traffic, pickup time,
  driver age), all scored by ONE fused featurize+MLP launch (the same K1+K2 kernel as
  ``/predict``), scaled by a road-class factor and floored at free-flow time at ``V_MAX`` so the
  A* heuristic stays admissible.
* :class:`BatchedAstar` — many point-to-point queries at once on the GPU (one lane per query,
  ``csrc/astar.hip``); CPU reference = scipy Dijkstra.
* :class:`GraphProvider` — ``directions()`` along road-graph shortest paths (replaces the
  reference's per-trip ORS directions call, ``RO/Flaskr/utils.py:151-156``), ``matrix()`` by
  great-circle distance (the greedy CVRP's max-distance semantics are in metres).
"""
from __future__ import annotations

import os

import datetime as dt
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..data.graph import RoadGraph, synth_road_graph
from ..models.features import RECORD_DTYPE, pack_record
from .providers import HaversineProvider, PROFILE_SPEED_MPS, ProviderError, _bbox, haversine_m

V_MAX_MPS = 130 / 3.6
CLASS_FACTOR = np.array([1.15, 1.0, 0.85, 0.65], dtype=np.float32)   # residential .. highway


TRAFFIC_LEVELS = ("Low", "Medium", "High", "Jam")
L_REF_M = 10_000.0


def edge_traffic(g: RoadGraph, congestion: int = 1) -> np.ndarray:
    """Synthetic per-edge traffic level (index into TRAFFIC_LEVELS): busier on big roads near the
    centre of the box; ``congestion`` (0..3) shifts the whole city."""
    mid_lat, mid_lon = float(g.lat.mean()), float(g.lon.mean())
    src = np.repeat(np.arange(g.num_nodes), np.diff(g.indptr))
    dc = haversine_m(g.lat[src], g.lon[src], mid_lat, mid_lon) / 1000.0
    lvl = (g.road_class.astype(np.int32) >= 2).astype(np.int32) + (dc < 8.0) + (dc < 4.0)
    return np.clip(lvl + congestion - 1, 0, 3).astype(np.int32)


def edge_records(g: RoadGraph, weather: str = "Sunny", congestion: int = 1,
                 pickup: Optional[dt.datetime] = None, driver_age: float = 35.0) -> np.ndarray:
    """Two records per directed edge: (edge traffic, L_REF) and (edge traffic, 0 m)."""
    from ..models.features import traffic_code
    pickup = pickup or dt.datetime(2025, 8, 25, 9, 0)
    proto = np.array([pack_record(weather=weather, traffic="Low", distance_m=0.0, pickup=pickup,
                                  driver_age=driver_age)], dtype=RECORD_DTYPE)
    lvl = edge_traffic(g, congestion)
    codes = np.array([traffic_code(t) for t in TRAFFIC_LEVELS], dtype=np.uint8)[lvl]
    rec = np.repeat(proto, 2 * g.num_edges)
    rec["traffic"][0::2] = codes
    rec["traffic"][1::2] = codes
    rec["distance_m"][0::2] = L_REF_M
    rec["distance_m"][1::2] = 0.0
    return rec


def edge_costs(g: RoadGraph, eta_model, device=None, **ctx: Any) -> np.ndarray:
    """Seconds per directed edge from the ETA MLP: each edge's marginal rate under ITS traffic
    level, measured over a 10 km reference trip so the model's fixed per-trip overhead cancels
    and bf16 rounding stays ~0.1 %:  len/L_REF * (f(ctx_e, L_REF) - f(ctx_e, 0)) minutes, times a
    road-class factor, floored at free-flow time at V_MAX (keeps A*'s heuristic admissible).
    All 2E records go through ONE fused featurize+MLP launch on the GPU."""
    from ..ops.eta_mlp import EtaMlpKernel, featurize_torch, records_to_tensor
    rec = records_to_tensor(edge_records(g, **ctx))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        minutes = EtaMlpKernel(eta_model, dev)(rec.to(dev)).cpu().numpy()
    else:
        with torch.no_grad():
            minutes = eta_model.float().cpu()(featurize_torch(rec)).numpy()
    rate = (minutes[0::2] - minutes[1::2]).astype(np.float32) * np.float32(60.0 / L_REF_M)
    sec = rate * g.length_m * CLASS_FACTOR[g.road_class]
    return np.maximum(sec, g.length_m / V_MAX_MPS).astype(np.float32)


def dijkstra_ref(g: RoadGraph, cost: np.ndarray, src: Sequence[int], dst: Sequence[int]) -> np.ndarray:
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    m = csr_matrix((cost.astype(np.float64), g.indices, g.indptr), shape=(g.num_nodes, g.num_nodes))
    out = np.empty(len(src))
    uniq = np.unique(np.asarray(src))
    d = dijkstra(m, directed=True, indices=uniq)
    row = {int(s): i for i, s in enumerate(uniq)}
    for k, (s, t) in enumerate(zip(src, dst)):
        out[k] = d[row[int(s)], int(t)]
    return out


def _spread16(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32) & 0xFFFF
    x = (x | (x << 8)) & 0x00FF00FF
    x = (x | (x << 4)) & 0x0F0F0F0F
    x = (x | (x << 2)) & 0x33333333
    return (x | (x << 1)) & 0x55555555


def morton_order(lat: np.ndarray, lon: np.ndarray) -> np.ndarray:
    """Node permutation (new id -> old id) sorting nodes by the Z-order key of their coordinates
    quantised to 16 bits per axis."""
    def q(a):
        a = np.asarray(a, dtype=np.float64)
        lo, hi = a.min(), a.max()
        return np.round((a - lo) / max(hi - lo, 1e-12) * 65535.0).astype(np.uint32)
    key = _spread16(q(lat)) << np.uint32(1) | _spread16(q(lon))
    return np.argsort(key, kind="stable").astype(np.int64)


def permute_csr(indptr: np.ndarray, indices: np.ndarray, perm: np.ndarray):
    """Renumber a CSR graph: new node i is old node perm[i].  Returns (perm, inv, indptr', indices',
    edge_perm) with edge_perm[new edge] = old edge, so per-edge arrays permute as a[edge_perm]."""
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(perm), dtype=perm.dtype)
    deg = np.diff(indptr)[perm]
    new_ptr = np.zeros(len(perm) + 1, dtype=indptr.dtype)
    np.cumsum(deg, out=new_ptr[1:])
    # old edge id of every new edge slot: each old node's edge range, nodes in the new order
    edge_perm = np.repeat(indptr[:-1][perm].astype(np.int64) - new_ptr[:-1], deg) + \
        np.arange(new_ptr[-1], dtype=np.int64)
    new_idx = inv[indices[edge_perm]].astype(indices.dtype)
    return perm, inv, new_ptr, new_idx, edge_perm


def landmark_tables(g: RoadGraph, cost: np.ndarray, k: int = 16, seed: int = 0,
                    method: str = "sectors") -> np.ndarray:
    """ALT preprocessing: K landmarks, forward d(L -> v) and backward d(v -> L) shortest-path
    tables, interleaved per node as [N][2K] = (fwd_k, fwd_k+1, bwd_k, bwd_k+1) float4 groups
    (csrc/astar.hip::halt).  ``sectors``: the outermost node of K angular sectors around the centre;
    ``farthest``: greedy farthest-point selection in travel time (each new landmark maximises its
    distance to the chosen set)."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    m = csr_matrix((np.asarray(cost, dtype=np.float64), g.indices, g.indptr), shape=(g.num_nodes,) * 2)
    if method == "farthest":
        rng = np.random.default_rng(seed)
        start = int(rng.integers(0, g.num_nodes))
        d0 = dijkstra(m, directed=True, indices=[start])[0]
        lms = [int(np.argmax(np.where(np.isfinite(d0), d0, -1)))]
        mind = dijkstra(m, directed=True, indices=lms)[0]
        while len(lms) < k:
            nxt = int(np.argmax(np.where(np.isfinite(mind), mind, -1)))
            lms.append(nxt)
            mind = np.minimum(mind, dijkstra(m, directed=True, indices=[nxt])[0])
    else:
        clat, clon = float(g.lat.mean()), float(g.lon.mean())
        ang = np.arctan2(g.lat - clat, (g.lon - clon) * np.cos(np.radians(clat)))
        rad = haversine_m(g.lat, g.lon, clat, clon)
        lms = []
        for i in range(k):
            lo, hi = -np.pi + 2 * np.pi * i / k, -np.pi + 2 * np.pi * (i + 1) / k
            sector = np.where((ang >= lo) & (ang < hi))[0]
            lms.append(int(sector[np.argmax(rad[sector])]) if len(sector) else int(np.argmax(rad)))
    fwd = dijkstra(m, directed=True, indices=lms)
    bwd = dijkstra(m.T.tocsr(), directed=True, indices=lms)
    fwd = np.where(np.isfinite(fwd), fwd, 0.0).astype(np.float32)
    bwd = np.where(np.isfinite(bwd), bwd, 0.0).astype(np.float32)
    out = np.empty((g.num_nodes, k // 2, 4), dtype=np.float32)
    out[:, :, 0] = fwd[0::2].T
    out[:, :, 1] = fwd[1::2].T
    out[:, :, 2] = bwd[0::2].T
    out[:, :, 3] = bwd[1::2].T
    return out.reshape(g.num_nodes, 2 * k)


def median_edge_m(g: RoadGraph, sample: int = 1 << 16) -> float:
    """Median great-circle edge length (metres) over an evenly strided sample of the edges."""
    ip = np.asarray(g.indptr)
    ix = np.asarray(g.indices)
    if ix.size == 0:
        return 0.0
    e = np.arange(0, ix.size, max(1, ix.size // sample))
    u = np.searchsorted(ip, e, side="right") - 1
    v = ix[e]
    la, lb = np.radians(g.lat[u]), np.radians(g.lat[v])
    hv = np.sin(0.5 * (lb - la)) ** 2 + np.cos(la) * np.cos(lb) * np.sin(0.5 * np.radians(g.lon[v] - g.lon[u])) ** 2
    return float(np.median(2 * 6371000.0 * np.arcsin(np.sqrt(np.clip(hv, 0.0, 1.0)))))


def _pow2_bits(n: int) -> int:
    return max(1, int(np.ceil(np.log2(max(2, n)))))


class AstarTier:
    """One tier's workspace (csrc/astar.hip AstarWs): ``slots`` concurrent searches, each with a hash
    table of ``2**tbits`` 16-byte entries (all-ones when idle), a heap row of ``cap`` u64 (the lane
    heap, or the wave tier's near/near/far lists) and a reset list of ``2**(tbits-1)`` slots.  A search
    may touch at most half its table; past that it overflows to the next tier."""

    def __init__(self, slots: int, cap: int, tbits: int, device):
        self.slots, self.cap, self.tbits = int(slots), int(cap), int(tbits)
        ts = 1 << self.tbits
        self.tab = torch.full((self.slots, 2 * ts), -1, dtype=torch.int64, device=device)
        self.heap = torch.empty((self.slots, self.cap), dtype=torch.int64, device=device)
        self.touched = torch.empty((self.slots, ts // 2), dtype=torch.int32, device=device)

    def ws(self):
        return (self.tab, self.heap, self.touched)

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.ws())

    @staticmethod
    def bytes_per_slot(cap: int, tbits: int) -> int:
        return 16 * (1 << tbits) + 8 * cap + 4 * (1 << (tbits - 1))


class BatchedAstar:
    """GPU batched A* (csrc/astar.hip): three tiers of sparse per-search state.

    * lane tier — ``slots`` searches, one lane each, ``lane_pops`` heap pops in small tables;
    * wave tier — ``wave_slots`` searches, one 64-lane wave each, tables of 2**13 entries that grow
      2x at a time into a shared arena (``arena_gb`` / ``ROUTEST_ASTAR_ARENA_GB``, default 4); ``cap`` bounds the
      f-band lists of a search;
    * big tier — ``big_slots`` searches with tables of >= 2N entries for what overflowed the wave tier.

    Workspace is ``slots x ~176 KB + wave_slots x (128 KB + 8 cap) + arena + big_slots x (5-40 MB)``
    — independent of the graph size up to the big tier (the round-2 kernel kept a dense [slots, N]
    state)."""

    def __init__(self, g: RoadGraph, cost: np.ndarray, device, slots: int = 16384, cap: int = 16384,
                 max_path: int = 4096, max_iters: int = 2_000_000, landmarks: int = 32,
                 landmark_method: str = "farthest", wave_slots: Optional[int] = None,
                 big_slots: Optional[int] = None, arena_gb: Optional[float] = None,
                 wave_tbits: Optional[int] = None):
        from ..ops import _ext
        self.C = _ext.native(required=True)
        self.g = g
        self.dev = d = torch.device(device)
        # internal node order: Z-order (Morton) over (lat, lon), so that nodes close on the map are
        # close in memory.  Measured neutral on the 100k-node graph with the dense state (80k legs:
        # 105.1-105.6 ms reordered vs 105.2 ms), so opt-in: ROUTEST_ASTAR_REORDER=1.
        self.reorder = os.environ.get("ROUTEST_ASTAR_REORDER", "0") == "1"
        if self.reorder:
            self.perm, self.inv, indptr, indices, self.edge_perm = permute_csr(
                g.indptr, g.indices, morton_order(g.lat, g.lon))
            self.perm_t = torch.from_numpy(self.perm.astype(np.int32)).to(d)
        else:
            self.perm = self.inv = self.edge_perm = self.perm_t = None
            indptr, indices = g.indptr, g.indices
        self.indptr = torch.from_numpy(np.ascontiguousarray(indptr)).to(d)
        self.indices = torch.from_numpy(np.ascontiguousarray(indices)).to(d)
        self.cost = torch.from_numpy(self._edges(np.asarray(cost, dtype=np.float32))).to(d)
        self.lat = torch.from_numpy(self._nodes(g.lat.astype(np.float32))).to(d)
        self.lon = torch.from_numpy(self._nodes(g.lon.astype(np.float32))).to(d)
        self.slots, self.cap, self.max_path, self.max_iters = slots, cap, max_path, max_iters
        # lane tier budget: the lane-per-query kernel gets `lane_pops` heap pops per query; the
        # searches still open then run one WAVE per query (f-band expansion), so the launch is no
        # longer as long as the single longest search.  ROUTEST_ASTAR_LANE_POPS=0: lane tier only.
        # 80k legs (bench/astar_tail.py, band 10 s, dense state): budget 2000 117 ms, 1000 112 ms,
        # 500 105 ms, 250 108 ms, everything in the wave stage 101 ms; lane only 236 ms.
        self.lane_pops = int(os.environ.get("ROUTEST_ASTAR_LANE_POPS", "500"))
        # interactive batches (a few thousand legs per flush: ~60 lane waves would leave most of the
        # 256 CUs idle) go straight to the wave tier: one 64-lane wave per search fills the chip.
        # Measured on the native route path at 1k concurrency (profiles/superseded/route_http_r3.jsonl): lane
        # budget 500 -> 19.3k req/s, 100 -> 24.1k, 1 (all wave) -> 26.2k, 2000 -> 10.3k.
        self.wave_only_below = int(os.environ.get("ROUTEST_ASTAR_WAVE_ONLY_BELOW", "32768"))
        self.wave_delta = float(os.environ.get("ROUTEST_ASTAR_DELTA", "10"))
        # legs longer than ~8 median edges (great circle) would spend the lane tier's whole pop budget
        # and start over in the wave tier: they skip the lane tier.  Route step, 100k-node graph
        # (profiles/superseded/astar_lane_split_ab_r3x.jsonl): no split 131.7 ms, 1000 m 124.6 ms, 4000 m 129.3 ms
        env_m = os.environ.get("ROUTEST_ASTAR_LANE_MAX_M")
        self.lane_max_m = float(env_m) if env_m is not None else 8.0 * median_edge_m(g)
        if wave_slots is None:
            wave_slots = int(os.environ.get("ROUTEST_ASTAR_WAVE_SLOTS", "16384"))
        self.wave_slots = max(1, min(slots, int(wave_slots)))
        N = g.num_nodes
        big_tbits = min(24, max(_pow2_bits(2 * max(128, (int(cap) + 7) // 8 * 8)) + 1, _pow2_bits(2 * N)))
        big_cap = max(int(cap), min(1 << 20, 1 << _pow2_bits(N // 2)))
        if big_slots is None:
            # as many big-tier searches as ~4 GiB of tables hold (1M nodes: ~100), at most 128
            per = AstarTier.bytes_per_slot(big_cap, big_tbits)
            big_slots = int(os.environ.get("ROUTEST_ASTAR_BIG_SLOTS", str(max(16, min(128, (4 << 30) // per)))))
        # tiers: cap (the wave tier's near/far lists per search) rounded to a multiple of 8; wave
        # tables start at 2**wave_tbits entries and grow 2x at a time into a shared arena, so their
        # memory follows the searches instead of a fixed worst case per slot
        cap = max(128, (int(cap) + 7) // 8 * 8)
        if wave_tbits is None:
            wave_tbits = int(os.environ.get("ROUTEST_ASTAR_WAVE_TBITS", "13"))
        wave_tbits = min(int(wave_tbits), _pow2_bits(2 * cap))
        if self.lane_pops > 0:
            lane_tbits = max(8, _pow2_bits(8 * self.lane_pops))
            lane_cap = max(64, 1 << (lane_tbits - 1))
            self.lane_tier = AstarTier(slots, lane_cap, lane_tbits, d)
            self.wave_tier = AstarTier(self.wave_slots, cap, wave_tbits, d)
        else:
            self.lane_tier = AstarTier(slots, cap, _pow2_bits(2 * cap), d)
            self.wave_tier = None
        if arena_gb is None:
            arena_gb = float(os.environ.get("ROUTEST_ASTAR_ARENA_GB", "4"))
        self.arena = (torch.full((int(arena_gb * (1 << 30)) // 16 * 2,), -1, dtype=torch.int64, device=d)
                      if arena_gb > 0 else None)
        self.arena_ctr = torch.zeros(1, dtype=torch.int64, device=d)
        big_tbits = min(24, max(_pow2_bits(2 * cap) + 1, _pow2_bits(2 * N)))
        big_cap = max(cap, min(1 << 20, 1 << _pow2_bits(N // 2)))
        if big_slots is None:
            # as many big-tier searches as ~4 GiB of tables hold (1M nodes: ~100), at most 128
            per = AstarTier.bytes_per_slot(big_cap, big_tbits)
            big_slots = int(os.environ.get("ROUTEST_ASTAR_BIG_SLOTS", str(max(16, min(128, (4 << 30) // per)))))
        self.big_tier = AstarTier(big_slots, big_cap, big_tbits, d) if big_slots > 0 else None
        self.scratch = torch.empty(1, dtype=torch.int32, device=d)
        # waves per search in the main wave-tier launch / the arena reruns + big tier (1, 2, 4, 8;
        # 0 = ROUTEST_ASTAR_WAVE_WAVES / ROUTEST_ASTAR_RETRY_WAVES, defaults 1 / 4)
        self.wave_nw = 0
        self.retry_nw = 0
        self.last_stats = {}
        # tightest admissible + consistent heuristic: every edge length is 1.15 x its great-circle
        # length (so any path >= 1.15 x the great-circle s-t distance) and every edge is traversed
        # no faster than the fastest edge of the graph
        cost_np = np.asarray(cost, dtype=np.float64)
        self.v_max = float((g.length_m / np.maximum(cost_np, 1e-6)).max()) * 1.0001
        self.inv_vmax = 1.15 / self.v_max
        self.landmark_method = landmark_method
        self.lm = (torch.from_numpy(self._nodes(landmark_tables(g, cost, landmarks,
                                                                method=landmark_method))).to(d)
                   if landmarks else None)

    @property
    def workspace_bytes(self) -> int:
        """Device bytes of the search workspace (all tiers; graph and landmark tables excluded)."""
        return (sum(t.nbytes for t in (self.lane_tier, self.wave_tier, self.big_tier) if t is not None)
                + (self.arena.numel() * 8 if self.arena is not None else 0))

    def _nodes(self, a: np.ndarray) -> np.ndarray:
        return np.ascontiguousarray(a[self.perm]) if self.perm is not None else a

    def _edges(self, a: np.ndarray) -> np.ndarray:
        return np.ascontiguousarray(a[self.edge_perm]) if self.edge_perm is not None else a

    def update_costs(self, cost: np.ndarray) -> None:
        # (heuristics are cached per search in its table and reset after it: nothing to drop)
        cost = np.asarray(cost, dtype=np.float32)
        self.cost.copy_(torch.from_numpy(self._edges(cost)))
        self._csr = None          # the host fallback's CSR was built from the old costs
        self.v_max = float((self.g.length_m / np.maximum(cost.astype(np.float64), 1e-6)).max()) * 1.0001
        self.inv_vmax = 1.15 / self.v_max
        if self.lm is not None:
            self.lm.copy_(torch.from_numpy(self._nodes(landmark_tables(
                self.g, cost, self.lm.shape[1] // 2, method=self.landmark_method))))

    def run(self, src: Sequence[int], dst: Sequence[int], sort: bool = False):
        """Returns (cost_s [Q] tensor, path_len [Q], status [Q], paths [Q, max_path]) on device.

        ``sort``: launch queries ordered by source node (ids are row-major, so this is a spatial
        order); with the kernel's XCD-aware wave mapping each XCD's L2 then serves one region of
        the graph.  Results are scattered back to the caller's order.  Measured neutral (314 vs
        317 ms for 80k legs: the per-slot state, not graph data, dominates), so off by default."""
        d = self.dev
        src = np.asarray(src, dtype=np.int32)
        dst = np.asarray(dst, dtype=np.int32)
        order = None
        if self.inv is not None:
            src, dst = self.inv[src].astype(np.int32), self.inv[dst].astype(np.int32)
        if sort and len(src) > 64:
            order = np.argsort(src, kind="stable")
            src, dst = src[order], dst[order]
        s = torch.as_tensor(src).to(d)
        t = torch.as_tensor(dst).to(d)
        Q = s.numel()
        out_cost = torch.empty(Q, dtype=torch.float32, device=d)
        out_len = torch.empty(Q, dtype=torch.int32, device=d)
        out_status = torch.empty(Q, dtype=torch.int32, device=d)
        out_path = torch.empty((Q, self.max_path), dtype=torch.int32, device=d)
        self.last_iters = torch.empty(Q, dtype=torch.int32, device=d)   # pops / expansions per query
        if self.scratch.numel() < Q + 1:
            self.scratch = torch.empty(Q + 1, dtype=torch.int32, device=d)
        st = self.C.astar_search(self.indptr, self.indices, self.cost, self.lat, self.lon, self.inv_vmax, self.lm,
                                 s, t, self.lane_tier.ws(), self.wave_tier.ws() if self.wave_tier else None,
                                 self.big_tier.ws() if self.big_tier else None, out_cost, out_len, out_status,
                                 out_path, self.last_iters, self.scratch, self.max_iters, self.lane_pops,
                                 self.wave_only_below, self.wave_delta, self.arena, self.arena_ctr,
                                 lane_max_m=self.lane_max_m, wave_nw=self.wave_nw, retry_nw=self.retry_nw)
        self.last_stats = dict(zip(("lane", "wave", "escalated", "lane_ms", "wave_ms", "big_ms", "retried",
                                    "retry_ms"), st))
        self.last_tail = int(st[1])
        self.last_escalated = int(st[2])
        self._exact_fallback(s, t, out_cost, out_len, out_status, out_path)
        if self.perm_t is not None:
            # back to the caller's node ids (entries past path_len are undefined: mask them to -1)
            valid = torch.arange(self.max_path, device=d, dtype=torch.int32)[None, :] < out_len[:, None]
            out_path = torch.where(valid, self.perm_t[out_path.clamp(0, self.g.num_nodes - 1).long()],
                                   torch.full_like(out_path, -1))
        if order is not None:
            idx = torch.from_numpy(order.astype(np.int64)).to(d)
            res = []
            for x in (out_cost, out_len, out_status, out_path):
                y = torch.empty_like(x)
                y[idx] = x
                res.append(y)
            return tuple(res)
        return out_cost, out_len, out_status, out_path

    # searches that ran out of per-slot list capacity (status 2) or of the iteration cap (3) are
    # finished exactly on the host (scipy Dijkstra over the same costs), at most this many per launch
    FALLBACK_MAX = 1024

    def _exact_fallback(self, s, t, out_cost, out_len, out_status, out_path) -> None:
        bad = ((out_status == 2) | (out_status == 3)).nonzero().flatten()
        self.last_fallbacks = int(bad.numel())
        if not self.last_fallbacks or self.last_fallbacks > self.FALLBACK_MAX:
            return
        from scipy.sparse import csr_matrix
        from scipy.sparse.csgraph import dijkstra
        if getattr(self, "_csr", None) is None:
            # the device-order graph (node ids as the kernel sees them)
            self._csr = csr_matrix((self.cost.double().cpu().numpy(), self.indices.cpu().numpy(),
                                    self.indptr.cpu().numpy()), shape=(self.g.num_nodes,) * 2)
        qi = bad.cpu().numpy()
        ss, tt = s[bad].cpu().numpy(), t[bad].cpu().numpy()
        uniq, inv = np.unique(ss, return_inverse=True)
        dist, pred = dijkstra(self._csr, directed=True, indices=uniq, return_predecessors=True)
        cost_h, len_h, st_h = out_cost[bad].cpu(), out_len[bad].cpu(), out_status[bad].cpu()
        for j, (q, sv, tv) in enumerate(zip(qi, ss, tt)):
            row = inv[j]
            if not np.isfinite(dist[row, tv]):
                cost_h[j], len_h[j], st_h[j] = -1.0, 0, 1
                continue
            path = [int(tv)]
            while path[-1] != sv:
                path.append(int(pred[row, path[-1]]))
            if len(path) > self.max_path:
                cost_h[j], len_h[j], st_h[j] = -1.0, 0, 4
                continue
            path.reverse()
            out_path[int(q), :len(path)] = torch.tensor(path, dtype=torch.int32, device=out_path.device)
            cost_h[j], len_h[j], st_h[j] = float(dist[row, tv]), len(path), 0
        out_cost[bad] = cost_h.to(out_cost.device)
        out_len[bad] = len_h.to(out_len.device)
        out_status[bad] = st_h.to(out_status.device)

    def paths(self, src, dst) -> List[Tuple[float, List[int]]]:
        c, n, st, p = self.run(src, dst)
        c, n, st, p = c.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy(), p.cpu().numpy()
        return [(float(c[i]), p[i, :n[i]].tolist()) if st[i] == 0 else (float("nan"), [])
                for i in range(len(c))]


def _path_length(g: RoadGraph, p: np.ndarray) -> float:
    """Sum of the great-circle lengths along a node path: the native route assembler's function
    (csrc/runtime/route_core.h path_length_m) when the C++ runtime is present, so the Python path
    and the native front end produce identical bits."""
    from .providers import _RT
    if _RT is not None:
        return _RT.path_length_m(g.lat, g.lon, np.asarray(p, dtype=np.int32))
    return float(haversine_m(g.lat[p[:-1]], g.lon[p[:-1]], g.lat[p[1:]], g.lon[p[1:]]).sum())


class GraphProvider(HaversineProvider):
    """Directions and road-distance matrices on the road graph (replaces the reference's per-trip
    ORS directions and per-request ORS matrix, ``RO/Flaskr/utils.py:55-62,97-105,151-156``).

    Engines (``ROUTEST_ROUTER``): ``cch`` (default) — :class:`routing.cch.RoadRouter`, the
    context-aware customizable contraction hierarchy (GPU, or the CPU reference without one);
    ``astar`` — the round-3 tiered batched A* / scipy Dijkstra on one fixed cost vector.

    Costs: with ``cost`` given, every request routes on those fixed edge seconds (no context); with
    ``eta_model`` (and no ``cost``), each request's context (weather, traffic, pickup week-hour) gets
    its own edge costs from the model.  ``matrix()`` returns the metre length of the time-shortest
    road path between the points (what the trips will report), not a great-circle estimate.
    Legs are (seconds, metres, node path); ``segments[].steps`` carry maneuvers along the path
    (road names, turn types and "Turn left onto ..." text, csrc/runtime/route_core.h leg_steps)."""

    name = "graph"
    blocking = True        # GPU searches synchronise the device
    FIXED_KEY = 1 << 40    # metric key of the fixed-cost mode

    def __init__(self, g: RoadGraph, cost: Optional[np.ndarray] = None, device=None, eta_model=None,
                 engine: Optional[str] = None):
        super().__init__()
        self.g = g
        self.cost = np.asarray(cost, dtype=np.float32) if cost is not None else None
        self.eta_model = eta_model
        if self.cost is None and self.eta_model is None:
            from ..serve.eta_service import default_model
            self.eta_model = default_model(hidden=64, steps=100)
        self.uses_context = self.cost is None
        self.device = device
        self.engine = (engine or os.environ.get("ROUTEST_ROUTER", "cch")).lower()
        if self.engine == "astar" and self.cost is None:
            self.cost = edge_costs(g, self.eta_model, device)
            self.uses_context = False
        self._astar = None
        self._csr = None
        self._routers: Dict[str, Any] = {}
        from collections import OrderedDict
        self._host_costs: "OrderedDict[int, np.ndarray]" = OrderedDict()   # LRU, HOST_COSTS entries
        import threading
        self._lock = threading.Lock()
        self._steps = None
        from .providers import _RT
        if _RT is not None and hasattr(_RT, "GraphSteps"):
            self._steps = _RT.GraphSteps(g.indptr, g.indices, g.length_m, g.lat, g.lon, g.edge_name,
                                         list(g.names or []))

    @classmethod
    def synthetic(cls, num_nodes: int = 100_000, eta_model=None, device=None) -> "GraphProvider":
        g = synth_road_graph(num_nodes)
        if eta_model is None:
            from ..serve.eta_service import default_model
            eta_model = default_model(hidden=64, steps=100)
        return cls(g, None, device, eta_model=eta_model)

    @classmethod
    def from_path(cls, path: str, eta_model=None, device=None) -> "GraphProvider":
        from ..data.roads import load_graph
        return cls(load_graph(path), None, device, eta_model=eta_model)

    # ---- engines ----
    def router(self, device=None):
        """The CCH router of a device (one per GPU; ``None``: the provider's own device)."""
        from .cch import RoadRouter
        dev = device if device is not None else self.device
        key = str(torch.device(dev)) if dev is not None else "cpu"
        with self._lock:
            r = self._routers.get(key)
            if r is None:
                r = RoadRouter(self.g, self.eta_model, device=dev)
                if self.cost is not None:
                    r.metric_from_costs(self.FIXED_KEY, self.cost)
                self._routers[key] = r
            return r

    HOST_COSTS = 64        # host copies of metrics' edge costs kept (LRU)

    def metric_key(self, ctx=None, device=None) -> int:
        """The metric a request routes on: the fixed one, or its context's (customized on demand).
        The returned key may be evicted again by later customizations: callers that query with it
        hold :meth:`pinned_metric` instead."""
        if not self.uses_context:
            return self.FIXED_KEY
        from .cch import RouteContext
        return self.router(device).metric(ctx or RouteContext())

    def pinned_metric(self, ctx=None, device=None):
        """``with prov.pinned_metric(ctx, dev) as key:`` — the request's metric, usable (not evicted)
        for the whole block."""
        import contextlib
        if not self.uses_context:
            return contextlib.nullcontext(self.FIXED_KEY)
        from .cch import RouteContext
        return self.router(device).pinned(ctx or RouteContext())

    def edge_seconds(self, key: int, device=None) -> np.ndarray:
        """Host copy of a metric's edge costs (maneuver durations); LRU of HOST_COSTS metrics."""
        if key == self.FIXED_KEY and self.cost is not None:
            return self.cost
        with self._lock:
            c = self._host_costs.get(key)
            if c is not None:
                self._host_costs.move_to_end(key)
                return c
        c = np.ascontiguousarray(self.router(device).costs(key), dtype=np.float32)
        with self._lock:
            self._host_costs[key] = c
            while len(self._host_costs) > self.HOST_COSTS:
                self._host_costs.popitem(last=False)
        return c

    def legs(self, pairs: List[Tuple[int, int]], ctx=None, device=None, key: Optional[int] = None):
        """[(seconds, metres, node path)] per (s, t) node pair (nan, nan, [] when not found), and the
        metric key they were computed on (``key``: an already customized metric)."""
        if self.engine == "astar":
            return [(sec, (_path_length(self.g, np.asarray(p)) * 1.15 if len(p) > 1 else 0.0) if p else float("nan"), p)
                    for sec, p in self._shortest_astar(pairs)], self.FIXED_KEY
        r = self.router(device)
        if key is None:
            with self.pinned_metric(ctx, device) as k:
                return self.legs(pairs, device=device, key=k)
        if not pairs:
            return [], key
        sec, met, st, paths = r.route([p[0] for p in pairs], [p[1] for p in pairs], key)
        return [(float(sec[i]), float(met[i]), paths[i].tolist()) if st[i] == 0 else (float("nan"), float("nan"), [])
                for i in range(len(pairs))], key

    def _shortest(self, pairs: List[Tuple[int, int]], ctx=None) -> List[Tuple[float, List[int]]]:
        """(seconds, node path) per pair (the legacy interface of the scorer / alternatives code)."""
        if self.engine == "astar":
            return self._shortest_astar(pairs)
        return [(sec, p) for sec, _, p in self.legs(pairs, ctx)[0]]

    def _shortest_astar(self, pairs: List[Tuple[int, int]]) -> List[Tuple[float, List[int]]]:
        if self.device is not None and torch.device(self.device).type == "cuda":
            # one search workspace per provider: concurrent handler threads take turns
            with self._lock:
                if self._astar is None:
                    self._astar = BatchedAstar(self.g, self.cost, self.device, slots=1024)
                return self._astar.paths([p[0] for p in pairs], [p[1] for p in pairs])
        from scipy.sparse import csr_matrix
        from scipy.sparse.csgraph import dijkstra
        if self._csr is None:
            self._csr = csr_matrix((self.cost.astype(np.float64), self.g.indices, self.g.indptr),
                                   shape=(self.g.num_nodes,) * 2)
        out = []
        for s, t in pairs:
            dist, pred = dijkstra(self._csr, directed=True, indices=s, return_predecessors=True)
            if not np.isfinite(dist[t]):
                out.append((float("nan"), []))
                continue
            path = [t]
            while path[-1] != s:
                path.append(int(pred[path[-1]]))
            out.append((float(dist[t]), path[::-1]))
        return out

    # ---- provider interface ----
    def leg_pairs(self, coords: List[List[float]]):
        """Snap [[lon, lat], ...] to graph nodes; returns (nodes, consecutive (s, t) node pairs)."""
        nodes = self.g.nearest_nodes([c[1] for c in coords], [c[0] for c in coords])
        return nodes, [(int(nodes[k]), int(nodes[k + 1])) for k in range(len(nodes) - 1)]

    def matrix(self, points: List[Dict[str, float]], profile: str, ctx=None) -> np.ndarray:
        """Road metres [n, n] between the snapped points along time-shortest paths (R21's matrix)."""
        nodes = self.g.nearest_nodes([p["lat"] for p in points], [p["lon"] for p in points])
        if self.engine == "astar":
            n = len(nodes)
            pairs = [(int(nodes[i]), int(nodes[j])) for i in range(n) for j in range(n)]
            L, _ = self.legs(pairs)
            D = np.array([m if i != j else 0.0 for (i, j), (_, m, _) in
                          zip([(i, j) for i in range(n) for j in range(n)], L)]).reshape(n, n)
            return np.where(np.isfinite(D), D, np.inf)
        with self.pinned_metric(ctx) as key:
            _, met = self.router().matrix(list(map(int, nodes)), key)
        return met.astype(np.float64)

    def directions(self, coords: List[List[float]], profile: str, ctx=None) -> Dict[str, Any]:
        nodes, pairs = self.leg_pairs(coords)
        with self.pinned_metric(ctx) as key:
            legs, key = self.legs(pairs, key=key)
            return self.feature_from_legs(coords, nodes, legs, profile, key=key)

    def feature_from_legs(self, coords: List[List[float]], nodes, legs, profile: str,
                          key: Optional[int] = None, device=None, ecost=None) -> Dict[str, Any]:
        """ORS-shaped Feature from per-leg (seconds, metres, node path) results (or the legacy
        (seconds, node path)).  A leg the search did not find (disconnected stops) is an explicit
        :class:`ProviderError`, never a silent straight line."""
        speed_scale = PROFILE_SPEED_MPS["driving-car"] / PROFILE_SPEED_MPS.get(profile, PROFILE_SPEED_MPS["driving-car"])
        geometry: List[List[float]] = [[float(coords[0][0]), float(coords[0][1])]]
        segments, way_points = [], [0]
        tot_d = tot_t = 0.0
        if self._steps is None or self.engine == "astar":
            ecost = None
        elif ecost is None and key is not None:
            ecost = self.edge_seconds(key, device)
        for k, leg in enumerate(legs):
            sec, metres, path = leg if len(leg) == 3 else (leg[0], None, leg[1])
            start = len(geometry) - 1
            if not path:
                raise ProviderError(f"no road path found between waypoints {k} and {k + 1} "
                                    f"(graph nodes {int(nodes[k])} -> {int(nodes[k + 1])})")
            p = np.asarray(path)
            if metres is not None:
                dist = float(metres)
            else:
                dist = _path_length(self.g, p) * 1.15 if len(p) > 1 else 0.0
            # node coordinates of the whole leg in one vector op (6 decimals, like ORS)
            geometry.extend(np.round(np.stack([self.g.lon[p], self.g.lat[p]], axis=1)
                                     .astype(np.float64), 6).tolist())
            geometry.append([float(coords[k + 1][0]), float(coords[k + 1][1])])
            end = len(geometry) - 1
            way_points.append(end)
            dur = sec * speed_scale
            arrive = {"distance": 0.0, "duration": 0.0, "type": 10, "instruction": "Arrive at your destination"
                      if k == len(legs) - 1 else f"Arrive at waypoint {k + 1}", "name": "-",
                      "way_points": [end, end]}
            if ecost is not None:
                steps = [{"distance": d, "duration": t, "type": ty, "instruction": ins, "name": nm,
                          "way_points": [w0, w1]}
                         for d, t, ty, ins, nm, w0, w1 in
                         self._steps.steps(p.astype(np.int32), float(sec), ecost, speed_scale, start, end)]
            else:
                steps = [{"distance": round(dist, 1), "duration": round(dur, 1), "type": 11 if k == 0 else 1,
                          "instruction": "Follow the road network", "name": "-", "way_points": [start, end]}]
            segments.append({"distance": round(dist, 1), "duration": round(dur, 1), "steps": steps + [arrive]})
            tot_d += dist
            tot_t += dur
        return {"type": "Feature", "bbox": _bbox(geometry),
                "geometry": {"type": "LineString", "coordinates": geometry},
                "properties": {"segments": segments,
                               "summary": {"distance": round(tot_d, 1), "duration": round(tot_t, 1)},
                               "way_points": way_points}}
