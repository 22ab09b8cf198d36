"""Batched multi-stop trip construction for many concurrent requests (K5 + K6).

``batched_trips(requests)`` packs R requests (each ``[source] + destinations``) into padded fp64
tensors, then on a GPU runs ONE K5 launch (all haversine matrices) and ONE K6 launch (all greedy
trip constructions, a wavefront per request); on CPU it runs the numpy/Python reference.  The
result per request is the trips list (index lists into ``[source]+destinations``) or an
:class:`InfeasibleStops` instance.  Sharding over several GPUs is done by
:class:`routing.route_batcher.RouteBatcher` (one worker thread per device, no collective).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from ..ops import _ext
from .greedy import InfeasibleStops, greedy_trips
from .providers import haversine_matrix

TripsOrError = Union[List[List[int]], InfeasibleStops]


def _f(v: Any, default: float) -> float:
    try:
        return float(v)
    except (TypeError, ValueError):
        return default


def pack_requests(requests: Sequence[Dict[str, Any]]):
    R = len(requests)
    nm = max(1 + len(r["destination_points"]) for r in requests) if R else 1
    lat = np.zeros((R, nm))
    lon = np.zeros((R, nm))
    dem = np.zeros((R, nm))
    npts = np.zeros(R, dtype=np.int32)
    cap = np.zeros(R)
    maxd = np.zeros(R)
    for k, r in enumerate(requests):
        pts = [r["source_point"]] + list(r["destination_points"])
        npts[k] = len(pts)
        lat[k, :len(pts)] = [p["lat"] for p in pts]
        lon[k, :len(pts)] = [p["lon"] for p in pts]
        dem[k, 1:len(pts)] = [_f(p.get("payload", 0), 0.0) for p in pts[1:]]
        drv = r.get("driver_details") or {}
        cap[k] = _f(drv.get("vehicle_capacity", 9e12), 9e12)
        maxd[k] = _f(drv.get("maximum_distance", 9e12), 9e12)
    return lat, lon, dem, npts, cap, maxd


def _unpack(visit: np.ndarray, trip_of: np.ndarray, ntrips: np.ndarray, status: np.ndarray,
            npts: np.ndarray, D: Optional[np.ndarray]) -> List[TripsOrError]:
    out: List[TripsOrError] = []
    for k in range(len(npts)):
        if status[k] != 0:
            placed = set(int(v) for v in visit[k] if v >= 0)
            rest = [i for i in range(1, int(npts[k])) if i not in placed]
            if D is not None:
                rest.sort(key=lambda i: D[k, 0, i])
            out.append(InfeasibleStops([i - 1 for i in rest]))
            continue
        trips: List[List[int]] = [[0] for _ in range(int(ntrips[k]))]
        for v, t in zip(visit[k], trip_of[k]):
            if v < 0:
                break
            trips[t].append(int(v))
        for t in trips:
            t.append(0)
        out.append(trips)
    return out


def batched_trips_device(lat, lon, dem, npts, cap, maxd, circuity: float, device,
                         D: Optional[np.ndarray] = None) -> List[TripsOrError]:
    C = _ext.native(required=True)
    dev = torch.device(device)
    t = lambda a, dt=torch.float64: torch.as_tensor(a, dtype=dt).to(dev)  # noqa: E731
    if D is None:
        D = C.route_haversine_matrix(t(lat), t(lon), t(npts, torch.int32), float(circuity))
    else:
        D = t(np.ascontiguousarray(D, dtype=np.float64))
    visit, trip_of, ntrips, status = C.route_greedy_cvrp(D, t(npts, torch.int32), t(dem), t(cap),
                                                         t(maxd))
    return _unpack(visit.cpu().numpy(), trip_of.cpu().numpy(), ntrips.cpu().numpy(),
                   status.cpu().numpy(), npts, D.cpu().numpy())


def batched_trips_cpu(lat, lon, dem, npts, cap, maxd, circuity: float,
                      D: Optional[np.ndarray] = None) -> List[TripsOrError]:
    out: List[TripsOrError] = []
    for k in range(len(npts)):
        n = int(npts[k])
        d = D[k, :n, :n] if D is not None else haversine_matrix(lat[k, :n], lon[k, :n], circuity)
        try:
            out.append(greedy_trips(d.tolist(), dem[k, :n].tolist(), float(cap[k]), float(maxd[k])))
        except InfeasibleStops as e:
            out.append(e)
    return out


def batched_trips(requests: Sequence[Dict[str, Any]], circuity: float = 1.3,
                  device: Optional[Any] = None, D: Optional[np.ndarray] = None) -> List[TripsOrError]:
    """``D``: given distance matrices [R, nm, nm] (road metres from the CCH router) instead of the
    haversine K5."""
    if not requests:
        return []
    packed = pack_requests(requests)
    if device is not None and torch.device(device).type == "cuda":
        return batched_trips_device(*packed, circuity=circuity, device=device, D=D)
    return batched_trips_cpu(*packed, circuity=circuity, D=D)
