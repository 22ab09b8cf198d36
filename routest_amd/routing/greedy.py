"""Capacity- and distance-constrained multi-trip greedy construction (R21) — CPU reference.

Exact semantics of ``RO/Flaskr/utils.py:111-139``::

    while unvisited:
        trip=[0]; load=0; trip_dist=0; current=0
        for idx in sorted(unvisited, key=lambda i: d[current][i]):   # sorted() runs ONCE, current==0
            if load+demand<=cap and trip_dist + d[current][idx] + d[idx][0] <= max_dist:
                accept: trip.append(idx); load+=demand; trip_dist+=d[current][idx]; current=idx
        trip.append(0); remove trip's stops from unvisited

Note the subtlety the survey's "nearest-first" hides: ``sorted`` is evaluated once per trip while
``current`` is still the depot, so candidates are scanned in order of distance *from the depot*
(stable: ties keep ascending index order) and each trip is a single pass over that order.  Since
the key never changes, the order is the same for every trip.

Fix (Appendix B #3): the reference loops forever when some stop is infeasible on its own (the trip
comes back as ``[0, 0]``).  We detect the no-progress trip and raise :class:`InfeasibleStops`.
The GPU kernel (K6, ``csrc/route_kernels.hip``) implements the same scan with one wavefront per
request; tests check both agree exactly.
"""
from __future__ import annotations

from typing import List, Sequence


class InfeasibleStops(ValueError):
    def __init__(self, stops: Sequence[int]):
        self.stops = list(stops)
        super().__init__("infeasible stop(s) (payload exceeds vehicle capacity or round trip "
                         f"exceeds maximum_distance): destination indices {self.stops}")


def greedy_trips(d: Sequence[Sequence[float]], demand: Sequence[float], cap: float,
                 max_dist: float) -> List[List[int]]:
    """d: (N+1)x(N+1) matrix over [depot] + stops; demand[i] for i in 0..N (demand[0] ignored).
    Returns trips as index lists into [depot]+stops, each starting and ending with 0."""
    n = len(d) - 1
    order = sorted(range(1, n + 1), key=lambda i: d[0][i])
    visited = [False] * (n + 1)
    remaining = n
    trips: List[List[int]] = []
    while remaining:
        trip = [0]
        load = 0.0
        trip_dist = 0.0
        cur = 0
        for idx in order:
            if visited[idx]:
                continue
            dem = float(demand[idx])
            if (load + dem) <= cap and (trip_dist + d[cur][idx] + d[idx][0]) <= max_dist:
                trip.append(idx)
                load += dem
                trip_dist += d[cur][idx]
                cur = idx
        if len(trip) == 1:
            raise InfeasibleStops([i - 1 for i in order if not visited[i]])
        for idx in trip[1:]:
            visited[idx] = True
        remaining -= len(trip) - 1
        trip.append(0)
        trips.append(trip)
    return trips


def greedy_trips_reference_literal(d, demand, cap, max_dist, max_trips: int = 10_000):
    """Line-for-line behaviour of the reference loop (bounded so tests can show the hang)."""
    all_n = len(d)
    trips = []
    unvisited = list(range(1, all_n))
    while unvisited:
        if len(trips) >= max_trips:
            raise RuntimeError("reference loop did not terminate")
        trip = [0]
        load = 0.0
        trip_dist = 0.0
        current = 0
        for idx in sorted(unvisited, key=lambda i: d[current][i]):
            demand_i = float(demand[idx])
            added = d[current][idx] + d[idx][0]
            if (load + demand_i) <= cap and (trip_dist + added) <= max_dist:
                trip.append(idx)
                load += demand_i
                trip_dist += d[current][idx]
                current = idx
        trip.append(0)
        trips.append(trip)
        visited = set(trip[1:-1])
        unvisited = [i for i in unvisited if i not in visited]
    return trips


def optimized_order(trips: List[List[int]]) -> List[int]:
    """R22: destination indices (0-based into destinations[]) in trip order."""
    return [idx - 1 for t in trips for idx in t[1:-1]]
