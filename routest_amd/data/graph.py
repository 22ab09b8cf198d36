"""Synthetic road graph for the GCN route scorer (config 4) and batched A* (config 5).

The reference routes over a remote road network (ORS: ``RO/Flaskr/utils.py:55,97,151``; OSRM in the
dashboard).  Offline, we generate a reproducible road-like graph over the Metro-Manila box the seed
locations live in (``LV/database/seeders/LocationsTableSeeder.php:13-34``):

* nodes on a jittered grid (``rows x cols``, 100k nodes by default);
* 4-neighbour streets plus random diagonals; every 8th row/col is a secondary road, every 32nd a
  primary, every 64th a highway (speed limits 30/45/60/80 km/h);
* undirected, stored as directed CSR (both directions), edge lengths by haversine;
* GCN operator Â = D^-1/2 (A + I) D^-1/2 as CSR values (self loops included);
* 32 node features (position, degree, incident road-class mix, fixed random projections).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from ..routing.providers import haversine_m

BBOX = (14.35, 120.90, 14.80, 121.15)   # lat_min, lon_min, lat_max, lon_max
CLASS_SPEED_KMH = np.array([30.0, 45.0, 60.0, 80.0], dtype=np.float32)


@dataclass
class RoadGraph:
    lat: np.ndarray          # [N] f64
    lon: np.ndarray          # [N] f64
    indptr: np.ndarray       # [N+1] i32 (CSR over directed edges, rows = source)
    indices: np.ndarray      # [E] i32 (targets)
    length_m: np.ndarray     # [E] f32
    road_class: np.ndarray   # [E] u8
    gcn_indptr: np.ndarray   # [N+1] i32 (Â incl. self loops)
    gcn_indices: np.ndarray  # [E+N] i32
    gcn_values: np.ndarray   # [E+N] f32
    features: np.ndarray     # [N, F] f32
    rows: int = 0
    cols: int = 0
    edge_name: Optional[np.ndarray] = None   # [E] i32 road name id (-1 unnamed)
    names: Optional[List[str]] = None        # name table

    @property
    def num_nodes(self) -> int:
        return int(self.lat.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.indices.shape[0])

    def degree(self) -> np.ndarray:
        return np.diff(self.indptr)

    #: snapping metric: Euclidean on (lat, lon * cos(14.6 deg)) — Metro Manila's latitude
    SNAP_C = float(np.cos(np.radians(14.6)))

    def _snapper(self):
        """Exact nearest node: the native bucket grid (csrc/runtime/route_core.h NodeGrid, the same
        code the native front end snaps with) when the C++ runtime is present, else a KD-tree."""
        s = getattr(self, "_snap", None)
        if s is None:
            try:
                from ..ops._ext import runtime
                rt = runtime(required=False)
            except Exception:  # pragma: no cover
                rt = None
            if rt is not None:
                s = ("grid", rt.NodeGrid(self.lat.astype(np.float64), self.lon.astype(np.float64), self.SNAP_C))
            else:
                from scipy.spatial import cKDTree
                s = ("kd", cKDTree(np.stack([self.lat, self.lon * self.SNAP_C], 1)))
            self._snap = s
        return s

    def nearest_node(self, lat: float, lon: float) -> int:
        return int(self.nearest_nodes([lat], [lon])[0])

    def nearest_nodes(self, lats, lons) -> np.ndarray:
        kind, s = self._snapper()
        la = np.asarray(lats, dtype=np.float64).reshape(-1)
        lo = np.asarray(lons, dtype=np.float64).reshape(-1)
        if kind == "grid":
            return s.nearest(la, lo)
        _, i = s.query(np.stack([la, lo * self.SNAP_C], 1))
        return i.astype(np.int32)

    def save(self, path: str) -> None:
        extra = {}
        if self.edge_name is not None:
            extra["edge_name"] = self.edge_name
            extra["names"] = np.array(self.names or [], dtype=str)
        np.savez_compressed(path, **{k: getattr(self, k) for k in (
            "lat", "lon", "indptr", "indices", "length_m", "road_class", "gcn_indptr", "gcn_indices",
            "gcn_values", "features")}, rows=self.rows, cols=self.cols, **extra)

    @staticmethod
    def load(path: str) -> "RoadGraph":
        z = np.load(path, allow_pickle=False)
        kw = {k: z[k] for k in z.files if k not in ("rows", "cols", "names")}
        names = [str(x) for x in z["names"]] if "names" in z.files else None
        return RoadGraph(**kw, rows=int(z["rows"]), cols=int(z["cols"]), names=names)

    def name_of_edge(self, e: int) -> str:
        if self.edge_name is None or self.edge_name[e] < 0:
            return "-"
        return self.names[int(self.edge_name[e])]


def _edge_class(r0, c0, r1, c1) -> np.ndarray:
    """Road class of a street segment by the grid line it runs along."""
    horiz = r0 == r1
    line = np.where(horiz, r0, c0)
    straight = (r0 == r1) | (c0 == c1)
    cls = np.zeros(r0.shape, dtype=np.uint8)
    cls = np.where(straight & (line % 8 == 0), 1, cls)
    cls = np.where(straight & (line % 32 == 0), 2, cls)
    cls = np.where(straight & (line % 64 == 0), 3, cls)
    return cls.astype(np.uint8)


def synth_road_graph(num_nodes: int = 100_000, seed: int = 0, feat_dim: int = 32,
                     diag_prob: float = 0.15) -> RoadGraph:
    rng = np.random.default_rng(seed)
    rows = int(np.sqrt(num_nodes))
    cols = int(np.ceil(num_nodes / rows))
    n = rows * cols
    lat0, lon0, lat1, lon1 = BBOX
    rr, cc = np.divmod(np.arange(n), cols)
    dlat = (lat1 - lat0) / max(1, rows - 1)
    dlon = (lon1 - lon0) / max(1, cols - 1)
    lat = lat0 + rr * dlat + rng.uniform(-0.3, 0.3, n) * dlat
    lon = lon0 + cc * dlon + rng.uniform(-0.3, 0.3, n) * dlon

    src, dst = [], []
    ids = np.arange(n).reshape(rows, cols)
    src.append(ids[:, :-1].ravel()); dst.append(ids[:, 1:].ravel())      # east
    src.append(ids[:-1, :].ravel()); dst.append(ids[1:, :].ravel())      # south
    d1 = rng.random((rows - 1, cols - 1)) < diag_prob
    src.append(ids[:-1, :-1][d1]); dst.append(ids[1:, 1:][d1])           # south-east diagonals
    s = np.concatenate(src)
    d = np.concatenate(dst)
    cls = _edge_class(rr[s], cc[s], rr[d], cc[d])
    # road names along the grid lines ("R-<row>" streets run east-west, "C-<col>" north-south, the
    # suffix by class, like Metro Manila's radial / circumferential roads); diagonals are unnamed
    suffix = np.array(["Street", "Avenue", "Boulevard", "Expressway"])
    horiz = rr[s] == rr[d]
    vert = cc[s] == cc[d]
    names = [f"R-{r} {suffix[c]}" for r in range(rows) for c in range(4)] + \
            [f"C-{c} {suffix[k]}" for c in range(cols) for k in range(4)]
    name_id = np.where(horiz, rr[s] * 4 + cls, np.where(vert, rows * 4 + cc[s] * 4 + cls, -1)).astype(np.int32)
    return build_graph(lat, lon, s, d, cls, name_id=name_id, names=names, both_ways=True, rng=rng,
                       feat_dim=feat_dim, rows=rows, cols=cols, bbox=BBOX)


def build_graph(lat: np.ndarray, lon: np.ndarray, s: np.ndarray, d: np.ndarray, cls: np.ndarray,
                length_m: Optional[np.ndarray] = None, name_id: Optional[np.ndarray] = None,
                names: Optional[List[str]] = None, both_ways: bool = False, seed: int = 0,
                feat_dim: int = 32, rows: int = 0, cols: int = 0,
                rng: Optional[np.random.Generator] = None,
                bbox: Optional[Tuple[float, float, float, float]] = None) -> RoadGraph:
    """RoadGraph from a directed edge list (``both_ways``: every edge also in reverse): CSR sorted by
    (source, target) with parallel edges merged (the shortest kept), lengths by haversine x 1.15
    unless given, the GCN operator and node features."""
    n = len(lat)
    lat = np.asarray(lat, dtype=np.float64)
    lon = np.asarray(lon, dtype=np.float64)
    s = np.asarray(s, dtype=np.int64)
    d = np.asarray(d, dtype=np.int64)
    cls = np.asarray(cls, dtype=np.uint8)
    if length_m is None:
        length_m = haversine_m(lat[s], lon[s], lat[d], lon[d]).astype(np.float32) * np.float32(1.15)
    length_m = np.asarray(length_m, dtype=np.float32)
    nid = np.asarray(name_id, dtype=np.int32) if name_id is not None else None
    if both_ways:
        s, d = np.concatenate([s, d]), np.concatenate([d, s])
        cls = np.concatenate([cls, cls])
        length_m = np.concatenate([length_m, length_m])
        nid = np.concatenate([nid, nid]) if nid is not None else None
    keep = s != d                                           # no self loops
    s, d, cls, length_m = s[keep], d[keep], cls[keep], length_m[keep]
    nid = nid[keep] if nid is not None else None
    order = np.lexsort((length_m, d, s))
    s2, d2, cls2, length = s[order], d[order], cls[order], length_m[order]
    nid = nid[order] if nid is not None else None
    first = np.ones(len(s2), dtype=bool)                    # parallel edges: keep the shortest
    first[1:] = (s2[1:] != s2[:-1]) | (d2[1:] != d2[:-1])
    s2, d2, cls2, length = s2[first], d2[first], cls2[first], length[first]
    nid = nid[first] if nid is not None else None
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(indptr, s2 + 1, 1)
    indptr = np.cumsum(indptr).astype(np.int32)

    deg = np.diff(indptr).astype(np.float64) + 1.0
    # Â with self loops, row-sorted CSR (symmetrised: one-way streets still couple their ends)
    us = np.concatenate([s2, d2])
    ud = np.concatenate([d2, s2])
    pair = np.unique(us * n + ud)
    us, ud = pair // n, pair % n
    udeg = np.bincount(us, minlength=n).astype(np.float64) + 1.0
    gs = np.concatenate([us, np.arange(n)])
    gd = np.concatenate([ud, np.arange(n)])
    go = np.lexsort((gd, gs))
    gs, gd = gs[go], gd[go]
    gval = (1.0 / np.sqrt(udeg[gs] * udeg[gd])).astype(np.float32)
    gptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(gptr, gs + 1, 1)
    gptr = np.cumsum(gptr).astype(np.int32)

    # node features
    rng = rng if rng is not None else np.random.default_rng(seed)
    if bbox is None:
        bbox = (float(lat.min()), float(lon.min()), float(lat.max()), float(lon.max()))
    lat0, lon0, lat1, lon1 = bbox
    f = np.zeros((n, feat_dim), dtype=np.float32)
    f[:, 0] = (lat - lat0) / max(lat1 - lat0, 1e-12) * 2 - 1
    f[:, 1] = (lon - lon0) / max(lon1 - lon0, 1e-12) * 2 - 1
    f[:, 2] = (deg - deg.mean()) / max(deg.std(), 1e-12)
    cls_mix = np.zeros((n, 4), dtype=np.float32)
    np.add.at(cls_mix, (s2, np.minimum(cls2, 3)), 1.0)
    f[:, 3:7] = cls_mix / np.maximum(1.0, cls_mix.sum(1, keepdims=True))
    k = feat_dim - 7
    proj = rng.standard_normal((2, k)).astype(np.float32)
    f[:, 7:] = np.sin(f[:, 0:2] @ proj * 3.0)
    return RoadGraph(lat, lon, indptr, d2.astype(np.int32), length.astype(np.float32), cls2, gptr,
                     gd.astype(np.int32), gval, f, rows, cols, edge_name=nid,
                     names=list(names) if names is not None else None)


def synth_route_queries(g: RoadGraph, n: int, seed: int = 0, min_km: float = 1.0,
                        max_km: float = 25.0) -> Tuple[np.ndarray, np.ndarray]:
    """Random (source, target) node pairs with a great-circle distance in [min_km, max_km]."""
    rng = np.random.default_rng(seed)
    out_s, out_t = [], []
    need = n
    while need > 0:
        s = rng.integers(0, g.num_nodes, need * 2)
        t = rng.integers(0, g.num_nodes, need * 2)
        dist = haversine_m(g.lat[s], g.lon[s], g.lat[t], g.lon[t]) / 1000.0
        ok = (dist >= min_km) & (dist <= max_km)
        out_s.append(s[ok][:need])
        out_t.append(t[ok][:need])
        need -= int(ok[:need * 2].sum()) if ok.sum() < need else need
    s = np.concatenate(out_s)[:n].astype(np.int32)
    t = np.concatenate(out_t)[:n].astype(np.int32)
    return s, t
