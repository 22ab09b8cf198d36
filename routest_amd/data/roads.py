"""Real road-network ingest: open formats -> :class:`RoadGraph`.

The reference routes real OSM roads through the remote ORS API (``RO/Flaskr/utils.py:151-156``);
offline, the service routes whatever graph it is given (``serve --graph PATH`` /
``ROUTEST_GRAPH_PATH``):

* **DIMACS** shortest-path challenge format — ``<name>.gr`` (``p sp N M``, ``a u v w`` arcs, 1-based,
  ``w`` = metres here) + ``<name>.co`` (``v id lon*1e6 lat*1e6``).  Arcs are directed, so one-way
  streets are kept as such.
* **Edge CSV** (an OSM export flattened to two tables) — ``<name>.nodes.csv`` with
  ``id,lat,lon`` and ``<name>.edges.csv`` with ``u,v[,length_m][,road_class][,name][,oneway]``
  (ids as in the nodes file; ``road_class`` 0 residential .. 3 highway, or an OSM ``highway=`` tag;
  ``oneway`` 1/yes/true keeps only u -> v).  Road names drive the maneuver text
  ("Turn left onto Shaw Boulevard").
* ``.npz`` — :meth:`RoadGraph.save` output.

Parallel edges are merged (the shortest kept) and self loops dropped by :func:`build_graph`.
"""
from __future__ import annotations

import csv
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from .graph import RoadGraph, build_graph

#: OSM highway tags -> road class (0 residential/other, 1 secondary, 2 primary, 3 motorway/trunk)
OSM_CLASS = {"motorway": 3, "motorway_link": 3, "trunk": 3, "trunk_link": 3, "primary": 2, "primary_link": 2,
             "secondary": 1, "secondary_link": 1, "tertiary": 1, "tertiary_link": 1}


def load_dimacs(gr_path: str, co_path: Optional[str] = None) -> RoadGraph:
    co_path = co_path or os.path.splitext(gr_path)[0] + ".co"
    n = None
    lon = lat = None
    with open(co_path) as f:
        for line in f:
            if line.startswith("p "):
                n = int(line.split()[-1])
                lon = np.zeros(n)
                lat = np.zeros(n)
            elif line.startswith("v "):
                _, i, x, y = line.split()
                lon[int(i) - 1] = int(x) / 1e6
                lat[int(i) - 1] = int(y) / 1e6
    if n is None:
        raise ValueError(f"{co_path}: no 'p' line")
    src: List[int] = []
    dst: List[int] = []
    w: List[float] = []
    with open(gr_path) as f:
        for line in f:
            if line.startswith("a "):
                _, u, v, c = line.split()
                src.append(int(u) - 1)
                dst.append(int(v) - 1)
                w.append(float(c))
    s = np.asarray(src, dtype=np.int64)
    d = np.asarray(dst, dtype=np.int64)
    if len(s) and (s.min() < 0 or d.min() < 0 or s.max() >= n or d.max() >= n):
        raise ValueError(f"{gr_path}: arc endpoint out of range")
    return build_graph(lat, lon, s, d, np.zeros(len(s), dtype=np.uint8), length_m=np.asarray(w, dtype=np.float32))


def _truthy(x: str) -> bool:
    return x.strip().lower() in ("1", "yes", "true", "y", "t")


def load_edge_csv(edges_path: str, nodes_path: Optional[str] = None) -> RoadGraph:
    nodes_path = nodes_path or edges_path.replace(".edges.csv", ".nodes.csv")
    ids: Dict[str, int] = {}
    lat: List[float] = []
    lon: List[float] = []
    with open(nodes_path, newline="", encoding="utf-8") as f:
        for row in csv.DictReader(f):
            ids[row["id"]] = len(lat)
            lat.append(float(row["lat"]))
            lon.append(float(row["lon"]))
    s: List[int] = []
    d: List[int] = []
    length: List[float] = []
    cls: List[int] = []
    name_id: List[int] = []
    names: List[str] = []
    name_ix: Dict[str, int] = {}
    have_len = None
    with open(edges_path, newline="", encoding="utf-8") as f:
        for row in csv.DictReader(f):
            u, v = ids[row["u"]], ids[row["v"]]
            if have_len is None:
                have_len = bool(row.get("length_m"))
            rc = row.get("road_class", "") or "0"
            c = int(rc) if rc.strip().lstrip("-").isdigit() else OSM_CLASS.get(rc.strip(), 0)
            nm = (row.get("name") or "").strip()
            ni = -1
            if nm:
                ni = name_ix.setdefault(nm, len(names))
                if ni == len(names):
                    names.append(nm)
            oneway = _truthy(row.get("oneway", "") or "0")
            ln = float(row["length_m"]) if have_len else np.nan
            for a, b in ((u, v),) if oneway else ((u, v), (v, u)):
                s.append(a)
                d.append(b)
                length.append(ln)
                cls.append(min(max(c, 0), 3))
                name_id.append(ni)
    lat_a = np.asarray(lat)
    lon_a = np.asarray(lon)
    s_a = np.asarray(s, dtype=np.int64)
    d_a = np.asarray(d, dtype=np.int64)
    ln_a = np.asarray(length, dtype=np.float32) if have_len else None
    return build_graph(lat_a, lon_a, s_a, d_a, np.asarray(cls, dtype=np.uint8), length_m=ln_a,
                       name_id=np.asarray(name_id, dtype=np.int32), names=names)


def load_graph(path: str) -> RoadGraph:
    """Any supported format by extension (.npz, .gr [+ .co], .edges.csv [+ .nodes.csv])."""
    if path.endswith(".npz"):
        return RoadGraph.load(path)
    if path.endswith(".gr"):
        return load_dimacs(path)
    if path.endswith(".csv"):
        return load_edge_csv(path)
    raise ValueError(f"unknown road graph format: {path!r} (.npz, .gr + .co, .edges.csv + .nodes.csv)")


# ------------------------------------------------------------------ fixture generator
def irregular_city(n: int = 1500, seed: int = 0, bbox: Tuple[float, float, float, float] = (14.53, 121.00, 14.62, 121.08)):
    """A small road network that is NOT a grid (for the committed fixture): random intersections,
    streets = Delaunay edges no longer than ~2 median edges, ~15 % of streets one-way, names given to
    long, nearly straight chains of streets ("Shaw Boulevard"-style corridors).  Returns
    (lat, lon, edges [(u, v, road_class, name, oneway)])."""
    from scipy.spatial import Delaunay
    rng = np.random.default_rng(seed)
    lat0, lon0, lat1, lon1 = bbox
    lat = rng.uniform(lat0, lat1, n)
    lon = rng.uniform(lon0, lon1, n)
    c = np.cos(np.radians((lat0 + lat1) / 2))
    tri = Delaunay(np.stack([lon * c, lat], 1))
    e = set()
    for t in tri.simplices:
        for a, b in ((t[0], t[1]), (t[1], t[2]), (t[0], t[2])):
            e.add((min(a, b), max(a, b)))
    e = np.array(sorted(e))
    dl = np.hypot((lon[e[:, 0]] - lon[e[:, 1]]) * c, lat[e[:, 0]] - lat[e[:, 1]])
    e = e[dl < 2.0 * np.median(dl)]
    adj: Dict[int, List[int]] = {}
    for a, b in e:
        adj.setdefault(int(a), []).append(int(b))
        adj.setdefault(int(b), []).append(int(a))
    # name corridors: walk straight from random edges
    stems = ["Rizal", "Shaw", "Ortigas", "Katipunan", "Aurora", "Quezon", "Taft", "Roxas", "Espana",
             "Magsaysay", "Bonifacio", "Mabini", "Kalayaan", "Lopez", "Pioneer", "Boni", "Santolan", "Timog"]
    kinds = ["Avenue", "Boulevard", "Street", "Road"]
    edge_name: Dict[Tuple[int, int], str] = {}
    edge_cls: Dict[Tuple[int, int], int] = {}

    def heading(a, b):
        return np.arctan2(lat[b] - lat[a], (lon[b] - lon[a]) * c)

    for k in range(60):
        a, b = (int(x) for x in e[rng.integers(0, len(e))])
        if (min(a, b), max(a, b)) in edge_name:
            continue
        nm = f"{stems[k % len(stems)]} {kinds[(k // len(stems)) % len(kinds)]}" + (f" {k // 72 + 2}" if k >= 72 else "")
        cl = int(rng.choice([1, 2, 3], p=[0.6, 0.3, 0.1]))
        for u, v in ((a, b), (b, a)):          # extend both ways
            prev, cur = u, v
            for _ in range(40):
                key = (min(prev, cur), max(prev, cur))
                if key in edge_name and edge_name[key] != nm:
                    break
                edge_name[key] = nm
                edge_cls[key] = cl
                h = heading(prev, cur)
                best, bd = None, 0.5
                for w in adj[cur]:
                    if w == prev:
                        continue
                    dd = abs((heading(cur, w) - h + np.pi) % (2 * np.pi) - np.pi)
                    if dd < bd:
                        best, bd = w, dd
                if best is None:
                    break
                prev, cur = cur, best
    out = []
    for a, b in e:
        key = (int(a), int(b))
        nm = edge_name.get(key, "")
        oneway = (not nm) and rng.random() < 0.15
        if oneway and rng.random() < 0.5:
            a, b = b, a
        out.append((int(a), int(b), edge_cls.get(key, 0), nm, oneway))
    return lat, lon, out


def write_edge_csv(prefix: str, lat, lon, edges) -> Tuple[str, str]:
    nodes_p, edges_p = prefix + ".nodes.csv", prefix + ".edges.csv"
    with open(nodes_p, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["id", "lat", "lon"])
        for i, (a, b) in enumerate(zip(lat, lon)):
            w.writerow([i, f"{a:.7f}", f"{b:.7f}"])
    with open(edges_p, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["u", "v", "road_class", "name", "oneway"])
        for u, v, cl, nm, ow in edges:
            w.writerow([u, v, cl, nm, 1 if ow else 0])
    return nodes_p, edges_p


def write_dimacs(prefix: str, g: RoadGraph) -> Tuple[str, str]:
    gr, co = prefix + ".gr", prefix + ".co"
    src = np.repeat(np.arange(g.num_nodes), np.diff(g.indptr))
    with open(gr, "w") as f:
        f.write(f"c routest_amd fixture (metres)\np sp {g.num_nodes} {g.num_edges}\n")
        for u, v, w in zip(src, g.indices, g.length_m):
            f.write(f"a {u + 1} {v + 1} {int(round(float(w)))}\n")
    with open(co, "w") as f:
        f.write(f"p aux sp co {g.num_nodes}\n")
        for i, (a, b) in enumerate(zip(g.lat, g.lon)):
            f.write(f"v {i + 1} {int(round(b * 1e6))} {int(round(a * 1e6))}\n")
    return gr, co
