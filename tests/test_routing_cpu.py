"""Greedy CVRP (R21) parity with a literal transcription of the reference loop, providers, and
the batched-request API on CPU."""
import random

import numpy as np
import pytest

from routest_amd.routing.batched import batched_trips, pack_requests, batched_trips_cpu
from routest_amd.routing.greedy import (InfeasibleStops, greedy_trips, greedy_trips_reference_literal,
                                        optimized_order)
from routest_amd.routing.optimizer import optimize_route
from routest_amd.routing.providers import HaversineProvider, haversine_matrix, profile_for


def _instance(rng, n):
    pts = rng.uniform([14.4, 120.95], [14.7, 121.1], size=(n + 1, 2))
    d = haversine_matrix(pts[:, 0], pts[:, 1], 1.3)
    dem = [0.0] + [float(rng.integers(1, 5)) for _ in range(n)]
    return pts, d, dem


def test_greedy_matches_reference_literal_random():
    rng = np.random.default_rng(0)
    checked = 0
    for trial in range(600):
        n = int(rng.integers(2, 13))
        pts, d, dem = _instance(rng, n)
        cap = float(rng.integers(4, 15))
        maxd = float(rng.uniform(20_000, 120_000))
        dl = d.tolist()
        try:
            ours = greedy_trips(dl, dem, cap, maxd)
        except InfeasibleStops:
            # the reference would loop forever; the bounded literal must report non-termination
            with pytest.raises(RuntimeError):
                greedy_trips_reference_literal(dl, dem, cap, maxd, max_trips=50)
            continue
        assert ours == greedy_trips_reference_literal(dl, dem, cap, maxd)
        checked += 1
    assert checked > 300


def test_greedy_sort_is_by_depot_distance():
    # The reference's sorted() is evaluated once per trip with current == 0, so the scan order is by
    # distance from the DEPOT, not from the current stop (utils.py:125).
    d = [[0, 1, 2, 3], [1, 0, 9, 1], [2, 9, 0, 9], [3, 1, 9, 0]]
    trips = greedy_trips(d, [0, 1, 1, 1], cap=10, max_dist=1e9)
    assert trips == [[0, 1, 2, 3, 0]]
    assert trips == greedy_trips_reference_literal(d, [0, 1, 1, 1], 10, 1e9)


def test_survey_verified_capacity_example():
    # capacity 5, loads 4/3/2 -> optimized_order [1, 2, 0], trips 2
    # (stop 1 nearest the depot, then 2, then 0)
    d = [[0, 3, 1, 2], [3, 0, 2, 1], [1, 2, 0, 1], [2, 1, 1, 0]]
    trips = greedy_trips(d, [0, 4, 3, 2], cap=5, max_dist=1e9)
    assert optimized_order(trips) == [1, 2, 0] and len(trips) == 2


def test_infeasible_stop_reports_indices():
    d = [[0, 1, 2], [1, 0, 1], [2, 1, 0]]
    with pytest.raises(InfeasibleStops) as e:
        greedy_trips(d, [0, 1, 99], cap=5, max_dist=1e9)
    assert e.value.stops == [1]


def test_profile_mapping():
    assert profile_for("Truck ") == "driving-hgv"
    assert profile_for("hgv") == "driving-hgv"
    assert profile_for("motorcycle") == "driving-car"
    assert profile_for("bike") == "cycling-regular"
    assert profile_for("roadbike") == "cycling-road"
    assert profile_for("foot") == "foot-walking"
    assert profile_for("spaceship") == "driving-car"
    assert profile_for(None) == "driving-car"


def test_haversine_provider_directions_shape():
    p = HaversineProvider()
    f = p.directions([[121.0, 14.5], [121.01, 14.51], [121.0, 14.5]], "driving-car")
    coords = f["geometry"]["coordinates"]
    assert f["properties"]["way_points"][0] == 0 and f["properties"]["way_points"][-1] == len(coords) - 1
    assert len(f["properties"]["segments"]) == 2
    s = f["properties"]["summary"]
    assert abs(s["distance"] - sum(seg["distance"] for seg in f["properties"]["segments"])) < 1.0


def test_batched_cpu_matches_single():
    rng = random.Random(1)
    reqs = []
    for _ in range(40):
        n = rng.randint(2, 10)
        reqs.append({"source_point": {"lat": 14.58, "lon": 121.04},
                     "destination_points": [{"lat": 14.4 + rng.random() * 0.3, "lon": 120.95 + rng.random() * 0.15,
                                             "payload": rng.randint(1, 4)} for _ in range(n)],
                     "driver_details": {"vehicle_capacity": rng.randint(4, 12), "maximum_distance": 90_000}})
    res = batched_trips(reqs)
    prov = HaversineProvider()
    for r, t in zip(reqs, res):
        f = optimize_route(r, prov)
        if isinstance(t, InfeasibleStops):
            assert "error" in f
        else:
            assert f["properties"]["optimized_order"] == optimized_order(t)
            assert f["properties"]["summary"]["trips"] == len(t)


def test_morton_permute_csr_preserves_graph():
    """BatchedAstar's internal renumbering (routing/graph.py::permute_csr): the permuted CSR is the
    same graph (same edge set with the same costs) under the node map, and shortest-path costs on it
    match the original graph."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import dijkstra
    from routest_amd.routing.graph import morton_order, permute_csr, synth_road_graph
    g = synth_road_graph(3000)
    rng = np.random.default_rng(1)
    cost = rng.uniform(1, 10, size=len(g.indices)).astype(np.float32)
    perm, inv, ptr, idx, ep = permute_csr(g.indptr, g.indices, morton_order(g.lat, g.lon))
    assert sorted(perm.tolist()) == list(range(g.num_nodes))
    old = {(int(u), int(g.indices[e])): float(cost[e]) for u in range(g.num_nodes)
           for e in range(g.indptr[u], g.indptr[u + 1])}
    new = {(int(perm[i]), int(perm[idx[e]])): float(cost[ep[e]]) for i in range(g.num_nodes)
           for e in range(ptr[i], ptr[i + 1])}
    assert old == new
    n = g.num_nodes
    m0 = csr_matrix((cost.astype(np.float64), g.indices, g.indptr), shape=(n, n))
    m1 = csr_matrix((cost[ep].astype(np.float64), idx, ptr), shape=(n, n))
    src = rng.integers(0, n, 5)
    d0 = dijkstra(m0, indices=src)
    d1 = dijkstra(m1, indices=inv[src])[:, inv]
    np.testing.assert_allclose(d0, d1)
    # Z-order puts map neighbours close in memory: more edges stay within one 128-byte line of
    # 8-byte per-node state (|id gap| < 16)
    near1 = (np.abs(np.repeat(np.arange(n), np.diff(ptr)) - idx) < 16).mean()
    near0 = (np.abs(np.repeat(np.arange(n), np.diff(g.indptr)) - g.indices) < 16).mean()
    assert near1 > near0, (near1, near0)
