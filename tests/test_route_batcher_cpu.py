"""Cross-request optimizer batching (routing/route_batcher.py) on the CPU paths: responses equal
the per-request path request for request, through the batch function, the queue, and concurrent
HTTP requests to /api/optimize_route, /route and /api/request_route."""
import asyncio
import json

import numpy as np
import pytest

from routest_amd.routing.optimizer import optimize_route
from routest_amd.routing.providers import HaversineProvider
from routest_amd.routing.route_batcher import RouteBatcher


def _requests(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = int(rng.integers(1, 11))
        lat0, lon0 = 14.55 + rng.normal(0, 0.03), 121.03 + rng.normal(0, 0.03)
        r = {"source_point": {"lat": lat0, "lon": lon0},
             "destination_points": [{"lat": lat0 + rng.normal(0, 0.05), "lon": lon0 + rng.normal(0, 0.05),
                                     "payload": int(rng.integers(1, 4))} for _ in range(k)],
             "driver_details": {"driver_name": f"d{i}", "vehicle_type": ["car", "truck", "bike"][i % 3],
                                "vehicle_capacity": int(rng.integers(3, 12)),
                                "maximum_distance": float(rng.choice([15000, 40000, 1e6]))}}
        if i % 17 == 0:
            r["destination_points"][0]["payload"] = 999          # infeasible stop -> error, no hang
        if i % 23 == 0:
            r = {"source_point": r["source_point"], "destination_points": []}   # no destinations
        out.append(r)
    return out


def test_run_batch_equals_per_request_haversine():
    prov = HaversineProvider()
    reqs = _requests(300)
    rb = RouteBatcher(prov, devices=[None])
    try:
        got = rb.run_batch(reqs, None)
    finally:
        rb.close()
    ref = [optimize_route(r, prov, "backend:mi355x") for r in reqs]
    assert json.dumps(got, sort_keys=True) == json.dumps(ref, sort_keys=True)
    assert any("error" in g for g in got) and any("geometry" in g for g in got)


def test_queue_two_workers_equals_per_request():
    prov = HaversineProvider()
    reqs = _requests(400, seed=1)
    rb = RouteBatcher(prov, devices=[None, None], batch_max=64, timeout_us=2000)
    try:
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(32) as ex:
            got = list(ex.map(lambda r: rb.optimize_sync(r, 60), reqs))
        assert sum(rb.flushes) >= 2
    finally:
        rb.close()
    ref = [optimize_route(r, prov, "backend:mi355x") for r in reqs]
    for g, r in zip(got, ref):
        assert g == r


def test_graph_provider_batched_legs_equal_per_request():
    from routest_amd.routing.graph import GraphProvider, edge_costs
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.serve.eta_service import default_model
    g = synth_road_graph(3000, seed=2)
    prov = GraphProvider(g, edge_costs(g, default_model(hidden=64, steps=30)))
    lat, lon = g.lat, g.lon
    rng = np.random.default_rng(5)
    reqs = []
    for i in range(40):
        idx = rng.integers(0, g.num_nodes, int(rng.integers(2, 7)))
        reqs.append({"source_point": {"lat": float(lat[idx[0]]), "lon": float(lon[idx[0]])},
                     "destination_points": [{"lat": float(lat[j]), "lon": float(lon[j]), "payload": 1}
                                            for j in idx[1:]],
                     "driver_details": {"driver_name": f"g{i}", "vehicle_capacity": 3,
                                        "maximum_distance": 1e7}})
    rb = RouteBatcher(prov, devices=[None])
    try:
        got = rb.run_batch(reqs, None)
    finally:
        rb.close()
    ref = [optimize_route(r, prov, "backend:mi355x") for r in reqs]
    assert got == ref


def test_http_concurrent_requests_through_batcher():
    import httpx
    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    from routest_amd.serve.eta_service import EtaService
    s = load_settings(env={}, dotenv_path=None, device="cpu", route_batch="1", route_gpu_min_stops=1, route_batch_max=128,
                      route_batch_timeout_us=3000)
    sv = build_services(s, eta=EtaService(None, device="cpu"), store=None)
    assert sv.route_batcher is not None
    app = create_app(sv)
    reqs = _requests(250, seed=3)
    prov = HaversineProvider()

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            paths = ["/api/optimize_route", "/route", "/api/request_route"]
            rs = await asyncio.gather(*[c.post(paths[i % 3], json=r) for i, r in enumerate(reqs)])
            return rs
    try:
        rs = asyncio.run(go())
    finally:
        sv.close()
    for i, (r, req) in enumerate(zip(rs, reqs)):
        ref = optimize_route(req, prov, s.engine_name)
        if "error" in ref:
            assert r.status_code == (200 if i % 3 == 2 else 400)
            assert r.json() == ref
        else:
            assert r.status_code == 200 and r.json() == ref


def test_unfound_leg_is_an_explicit_error():
    """A leg the search did not find is an error response, never a silent straight line."""
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    g = synth_road_graph(2000, seed=6)
    prov = GraphProvider(g, np.ones(g.num_edges, dtype=np.float32))
    prov.legs = lambda pairs, ctx=None, device=None, key=None: (
        [(float("nan"), float("nan"), [])] * len(pairs), prov.FIXED_KEY)
    req = {"source_point": {"lat": float(g.lat[0]), "lon": float(g.lon[0])},
           "destination_points": [{"lat": float(g.lat[500]), "lon": float(g.lon[500])}]}
    out = optimize_route(req, prov)
    assert "error" in out and "no road path" in out["error"]
    rb = RouteBatcher(prov, devices=[None])
    try:
        assert "no road path" in rb.run_batch([req])[0]["error"]
    finally:
        rb.close()


def _ctx_requests(g, n, hours, seed=9):
    rng = np.random.default_rng(seed)
    reqs = []
    for i in range(n):
        idx = rng.integers(0, g.num_nodes, int(rng.integers(2, 6)))
        reqs.append({"source_point": {"lat": float(g.lat[idx[0]]), "lon": float(g.lon[idx[0]])},
                     "destination_points": [{"lat": float(g.lat[j]), "lon": float(g.lon[j]), "payload": 1}
                                            for j in idx[1:]],
                     "driver_details": {"driver_name": f"c{i}", "vehicle_capacity": 3, "maximum_distance": 1e7},
                     "context": {"weather": ["Sunny", "Stormy"][i % 2], "traffic": "Medium",
                                 "pickup_time": f"2026-10-1{i % 3 + 2}T{hours[i % len(hours)]:02d}:15:00"}})
    return reqs


def test_flush_with_more_contexts_than_the_cache_holds():
    """every context group of a flush is planned under a pin of its metric, so
    more distinct contexts than the LRU holds cannot evict a group's metric before it is used."""
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.serve.eta_service import default_model
    g = synth_road_graph(2500, seed=4)
    prov = GraphProvider(g, None, eta_model=default_model(hidden=32, steps=20))
    r = prov.router()
    r.capacity = 2                                   # far fewer than the flush's contexts
    reqs = _ctx_requests(g, 24, hours=[7, 8, 9, 17])
    rb = RouteBatcher(prov, devices=[None])
    try:
        got = rb.run_batch(reqs, None)
    finally:
        rb.close()
    assert all("error" not in x for x in got), [x.get("error") for x in got]
    assert len(r._cpu_metrics) <= 2 and not r._cpu_pins
    ref = [optimize_route(q, prov, "backend:mi355x") for q in reqs]
    assert got == ref


def test_plan_carries_the_context_to_assembly():
    """the context of a request without pickup_time is resolved once, in the
    plan; assembly neither recomputes it from now() nor customizes anything."""
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.serve.eta_service import default_model
    g = synth_road_graph(2000, seed=5)
    prov = GraphProvider(g, None, eta_model=default_model(hidden=32, steps=20))
    req = _ctx_requests(g, 1, hours=[10])[0]
    del req["context"]["pickup_time"]
    rb = RouteBatcher(prov, devices=[None])
    try:
        plan = rb.plan_batch([req], None)[0]
        assert plan[2] is not None and plan[2].key in {k for (k, _, _) in plan[1].legs}

        def boom(*a, **k):
            raise AssertionError("assembly must not customize")
        prov.metric_key = boom
        prov.pinned_metric = boom
        out = rb.assemble(req, plan)
    finally:
        rb.close()
    assert "error" not in out and out["properties"]["summary"]["distance"] > 0


def test_cch_rejects_nan_and_negative_costs():
    """costs are ordered by their float bits; NaN / negative are rejected and
    -0.0 (a zero-length edge) routes like +0.0."""
    rt = pytest.importorskip("routest_amd._rt")
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import dijkstra_ref
    g = synth_road_graph(800, seed=1)
    c = rt.CCH(g.indptr, g.indices, g.lat, g.lon, 2)
    length = g.length_m.astype(np.float32)
    cost = (length / 10.0).astype(np.float32)
    for bad in (np.nan, -1.0, np.inf):
        cb = cost.copy()
        cb[5] = bad
        with pytest.raises(ValueError):
            c.customize(cb, length)
    src = np.arange(0, 60, dtype=np.int32)
    dst = np.arange(400, 460, dtype=np.int32)
    cp, cz = cost.copy(), cost.copy()
    cp[:80] = 0.0
    cz[:80] = -0.0
    sp, _, stp, _ = c.query(c.customize(cp, length), src, dst, False, 4096)
    sz, _, stz, _ = c.query(c.customize(cz, length), src, dst, False, 4096)
    assert np.array_equal(np.asarray(stp), np.asarray(stz)) and np.array_equal(np.asarray(sp), np.asarray(sz))
    ref = dijkstra_ref(g, cost, src, dst)
    s0, _, st0, _ = c.query(c.customize(cost, length), src, dst, False, 4096)
    ok = np.isfinite(ref)
    assert (np.asarray(st0)[ok] == 0).all()
    np.testing.assert_allclose(np.asarray(s0)[ok], ref[ok], rtol=1e-5)
