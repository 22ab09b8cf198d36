"""Routing contexts off the flush's critical path (verdict r4 item 2; SURVEY K9 "precomputed per
(graph, context) and cached").

The native route service (csrc/route_service.hip cch_groups) no longer customizes a new context
inside the flush that first needs it: that request's jobs wait for the router's background build
(csrc/cch.hip builder_loop, lowest-priority stream) while the rest of the flush — and every later
request of a cached context — proceeds.  Contexts of requests routed at "now" are prefetched for
the next week-hour before it begins, and the metric LRU is sized from an HBM budget.
Reference: RO/Flaskr/routes.py:102-104 (the request context read on every optimize call).
"""
import datetime as dt
import http.client
import json
import threading
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _req(port, body, conn=None):
    c = conn or http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request("POST", "/api/optimize_route", body=json.dumps(body).encode(),
              headers={"Content-Type": "application/json"})
    r = c.getresponse()
    return r.status, r.read()


def _pay(g, rng, ctx, stops=4):
    idx = rng.integers(0, g.num_nodes, stops + 1)
    return {"source_point": {"lat": float(g.lat[idx[0]]), "lon": float(g.lon[idx[0]])},
            "destination_points": [{"lat": float(g.lat[j]), "lon": float(g.lon[j]), "payload": 1} for j in idx[1:]],
            "driver_details": {"driver_name": "a", "vehicle_type": "car", "vehicle_capacity": 9999,
                               "maximum_distance": 1e7},
            "context": ctx}


@pytest.fixture(scope="module")
def stack():
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.serve.eta_service import default_model
    from test_frontend_gpu import _stack
    g = synth_road_graph(100_000, seed=0)
    prov = GraphProvider(g, None, device=torch.device("cuda", 0), eta_model=default_model(hidden=64, steps=50))
    st, sv = _stack(prov, None)
    assert st.front.routes
    yield g, prov, st
    st.close()


def test_fresh_context_does_not_delay_cached_context(stack):
    g, prov, st = stack
    rng = np.random.default_rng(0)
    warm = {"weather": "Sunny", "traffic": "Low", "pickup_time": "2025-08-26T03:10:00"}
    pays = [_pay(g, rng, warm) for _ in range(64)]
    conn = http.client.HTTPConnection("127.0.0.1", st.port, timeout=60)
    for p in pays[:8]:
        assert _req(st.port, p, conn)[0] == 200          # context built, chains warm
    base = []
    for p in pays:
        t0 = time.perf_counter()
        assert _req(st.port, p, conn)[0] == 200
        base.append(time.perf_counter() - t0)
    base_p50 = float(np.median(base))
    s0 = st.front.stats()
    # a request under a context never seen, while the cached context keeps being served
    fresh = _pay(g, rng, {"weather": "Stormy", "traffic": "Jam", "pickup_time": "2025-08-29T18:40:00"})
    out = {}

    def fresh_call():
        t0 = time.perf_counter()
        out["fresh"] = _req(st.port, fresh)
        out["fresh_s"] = time.perf_counter() - t0
    th = threading.Thread(target=fresh_call)
    lat = []
    th.start()
    t_end = time.perf_counter() + 0.5
    k = 0
    while th.is_alive() or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        assert _req(st.port, pays[k % len(pays)], conn)[0] == 200
        lat.append(time.perf_counter() - t0)
        k += 1
    th.join()
    s1 = st.front.stats()
    assert out["fresh"][0] == 200
    # the fresh request waited for its build; none of the cached context's requests did
    assert s1["route_ctx_deferred"] - s0["route_ctx_deferred"] == 1, (s0, s1)
    assert s1["route_us_ctx_wait"] > s0["route_us_ctx_wait"]
    build_s = out["fresh_s"]
    assert max(lat) < max(4 * base_p50, 0.5 * build_s), (max(lat), base_p50, build_s)
    # the answer under the fresh context equals the app's (same GPU CCH object)
    b = _req(st.app_server.port, fresh)
    assert b == out["fresh"]


def test_many_contexts_in_one_burst(stack):
    """A burst over 24 fresh contexts: every request answered (byte-identical to the app's), each
    context built once in the background, no flush failed."""
    g, prov, st = stack
    rng = np.random.default_rng(1)
    ctxs = [{"weather": w, "traffic": t, "pickup_time": f"2025-09-0{d}T{h:02d}:05:00"}
            for w in ("Cloudy", "Windy") for t in ("Medium", "High") for d, h in ((1, 6), (2, 11), (3, 15), (4, 20),
                                                                                  (5, 7), (6, 23))]
    pays = [_pay(g, rng, c, stops=int(rng.integers(1, 6))) for c in ctxs for _ in range(3)]
    s0 = st.front.stats()
    res = [None] * len(pays)

    def worker(i0):
        c = http.client.HTTPConnection("127.0.0.1", st.port, timeout=120)
        for i in range(i0, len(pays), 16):
            res[i] = _req(st.port, pays[i], c)
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    s1 = st.front.stats()
    assert all(r is not None and r[0] in (200, 400) for r in res)
    for p, r in zip(pays[::5], res[::5]):
        assert _req(st.app_server.port, p) == r
    assert s1["route_service_fallbacks"] == s0["route_service_fallbacks"]
    stats = prov.router(torch.device("cuda", 0)).stats()
    assert stats["async_failed"] == 0 and stats["cache_capacity"] >= 24, stats


def test_next_hour_is_prefetched(monkeypatch):
    """Requests routed at "now" (no pickup_time): their (weather, traffic) pairs are customized
    for the next week-hour ahead of time (ROUTEST_CCH_PREFETCH_MIN=60: always inside the lead)."""
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.cch import CONGESTION, RouteContext
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.models.features import weather_code
    from routest_amd.serve.eta_service import default_model
    from test_frontend_gpu import _stack
    monkeypatch.setenv("ROUTEST_CCH_PREFETCH_MIN", "60")
    g = synth_road_graph(20_000, seed=3)
    prov = GraphProvider(g, None, device=torch.device("cuda", 0), eta_model=default_model(hidden=64, steps=30))
    st, sv = _stack(prov, None)
    try:
        rng = np.random.default_rng(2)
        for w, t in (("Sunny", "Medium"), ("Stormy", "High")):
            assert _req(st.port, _pay(g, rng, {"weather": w, "traffic": t}))[0] == 200
        now = dt.datetime.now()
        nxt = (now.weekday() * 24 + now.hour + 1) % 168
        want = [RouteContext(weather=weather_code(w), congestion=CONGESTION[t], weekhour=nxt)
                for w, t in (("Sunny", "Medium"), ("Stormy", "High"))]
        r = prov.router(torch.device("cuda", 0))
        t_end = time.time() + 20
        while time.time() < t_end and not all(r.is_cached(c) for c in want):
            time.sleep(0.05)
        if dt.datetime.now().hour != now.hour:
            pytest.skip("the hour turned during the test")
        assert all(r.is_cached(c) for c in want)
        assert st.front.stats()["route_ctx_prefetched"] >= 2
    finally:
        st.close()


def test_lru_is_sized_from_an_hbm_budget(stack):
    """The metric LRU holds as many contexts as fit ROUTEST_CCH_CACHE_GB (default 48 GB), derived
    from the device bytes of a built metric — not a fixed count."""
    g, prov, st = stack
    r = prov.router(torch.device("cuda", 0))
    s = r.stats()
    assert s["cache_gb"] == 48.0 and s["metric_bytes"] > 0, s
    assert s["cache_capacity"] == max(4, int(48.0 * 2 ** 30 // s["metric_bytes"])), s
    r.gpu.set_cache_gb(1.0)
    s1 = r.stats()
    assert s1["cache_capacity"] == max(4, int(2 ** 30 // s["metric_bytes"])) and s1["cached_metrics"] <= s1["cache_capacity"]
    r.gpu.set_cache_gb(48.0)
