"""Contract tests for every reference endpoint (SURVEY Appendix A.1, §4.2 verified behaviours)."""
import json

import pytest
from fastapi.testclient import TestClient

from routest_amd.api.app import build_services, create_app
from routest_amd.config import load_settings
from routest_amd.serve.eta_service import EtaService, default_model
from routest_amd.store.store import SQLiteStore

# The dashboard's canonical request (FE/app/ui/page.jsx:1578-1617, F02)
F02 = {
    "source_point": {"lat": 14.5836, "lon": 121.0409},
    "destination_points": [{"lat": 14.5352, "lon": 120.9822, "payload": 1},
                           {"lat": 14.5833, "lon": 121.0567, "payload": 1},
                           {"lat": 14.6556, "lon": 121.0313, "payload": 1}],
    "driver_details": {"driver_name": "TRK-001", "vehicle_type": "truck", "vehicle_capacity": 9999,
                       "maximum_distance": 100000, "driver_age": 34},
    "meta": {"origin_id": "origin-uuid", "destination_ids": ["a", "b", "c"], "vehicle_id": "TRK-001"},
    "use_ml_eta": True,
    "context": {"weather": "Sunny", "traffic": "Medium"},
}
# RO/tests/test_get_route.py:3-12
SMOKE = {
    "source_point": {"lat": 14.584630, "lon": 121.056885},
    "destination_points": [{"lat": 14.544145, "lon": 121.056617, "payload": 4},
                           {"lat": 14.557855, "lon": 121.066139, "payload": 4}],
    "driver_details": {"driver_name": "John Doe", "vehicle_type": "car", "vehicle_capacity": 5,
                       "maximum_distance": 50000},
}


@pytest.fixture(scope="module")
def model():
    return default_model(seed=0, hidden=64, steps=60)


def _client(model=None, store="memory", **settings_kw):
    s = load_settings(env={}, dotenv_path=None, device="cpu", sim_tick_min_s=0.01, sim_tick_max_s=0.02,
                      **settings_kw)
    eta = EtaService(model, device="cpu") if model is not None else EtaService(None, device="cpu")
    st = SQLiteStore(":memory:") if store == "memory" else None
    sv = build_services(s, eta=eta, store=st)
    return TestClient(create_app(sv))


@pytest.fixture
def client(model):
    with _client(model) as c:
        yield c


def test_url_map_matches_reference(client):
    paths = {(r.path, tuple(sorted(r.methods))) for r in client.app.routes if hasattr(r, "methods")}
    for p, m in [("/api/request_route", "POST"), ("/api/optimize_route", "POST"), ("/api/predict_eta", "POST"),
                 ("/api/confirm_route", "POST"), ("/api/update_tracker", "POST"), ("/api/ping", "GET"),
                 ("/api/health", "GET"), ("/api/history", "GET"), ("/api/history/{req_id}", "GET"),
                 ("/api/history/{req_id}", "DELETE"), ("/api/realtime_feed", "GET"),
                 ("/predict", "POST"), ("/route", "POST")]:
        assert any(pp == p and m in ms for pp, ms in paths), (p, m)


def test_ping(client):
    r = client.get("/api/ping")
    assert r.status_code == 200 and r.json() == {"ok": True, "service": "route-optimizer"}


def test_request_route_multi_stop_shape(client):
    r = client.post("/api/request_route", json=SMOKE)
    assert r.status_code == 200
    f = r.json()
    assert f["type"] == "Feature" and f["geometry"]["type"] == "LineString"
    p = f["properties"]
    # capacity 5, payload 4+4 -> two trips
    assert p["summary"]["trips"] == 2
    assert sorted(p["optimized_order"]) == [0, 1]
    assert p["engine"] == "backend:mi355x" and p["driver_name"] == "John Doe" and p["vehicle_type"] == "car"
    assert len(f["bbox"]) == 4 and f["bbox"][0] <= f["bbox"][2]
    for seg in p["segments"]:
        assert {"distance", "duration", "steps"} <= set(seg)
        for st in seg["steps"]:
            assert {"distance", "duration", "instruction", "name", "type", "way_points"} <= set(st)


def test_request_route_error_is_200_quirk(client):
    r = client.post("/api/request_route", json={"destination_points": []})
    assert r.status_code == 200 and "error" in r.json()


def test_request_route_error_400_without_compat(model):
    with _client(model, compat_request_route_200=False) as c:
        r = c.post("/api/request_route", json={"destination_points": []})
        assert r.status_code == 400


def test_request_route_non_json_415(client):
    r = client.post("/api/request_route", content=b"x", headers={"content-type": "text/plain"})
    assert r.status_code == 415


def test_optimize_route_error_400(client):
    r = client.post("/api/optimize_route", json={})
    assert r.status_code == 400 and r.json() == {"error": "no destination points specified."}


def test_optimize_route_ml_eta_and_persist(client):
    r = client.post("/api/optimize_route", json=F02)
    assert r.status_code == 200
    p = r.json()["properties"]
    assert isinstance(p["eta_minutes_ml"], float) and p["eta_minutes_ml"] > 0
    assert "T" in p["eta_completion_time_ml"]
    assert p["saved"] is True and p["request_id"]
    assert p["vehicle_type"] == "truck"
    h = client.get("/api/history?limit=5").json()["items"]
    assert h[0]["request_id"] == p["request_id"]
    assert h[0]["engine"] == "ml" and h[0]["dest_count"] == 3 and h[0]["optimized"] is True
    assert set(h[0]) == {"request_id", "created_at", "origin_id", "dest_count", "total_distance",
                         "total_duration", "optimized", "engine", "vehicle_id", "eta_minutes_ml",
                         "eta_completion_time_ml"}
    d = client.get(f"/api/history/{p['request_id']}").json()
    assert d["request"]["id"] == p["request_id"] and d["request"]["driver_age"] == 34
    assert d["result"]["geometry"]["type"] == "LineString" and d["result"]["legs"]
    assert client.delete(f"/api/history/{p['request_id']}").status_code == 204
    assert client.get(f"/api/history/{p['request_id']}").status_code == 404


def test_route_alias(client):
    r = client.post("/route", json=dict(F02, use_ml_eta=False))
    assert r.status_code == 200 and "eta_minutes_ml" not in r.json()["properties"]


def test_point_to_point(client):
    body = dict(SMOKE, destination_points=[SMOKE["destination_points"][0]])
    r = client.post("/api/request_route", json=body)
    f = r.json()
    assert f["properties"]["optimized_order"] == [0]
    assert "trips" not in f["properties"]["summary"]  # Appendix B #12
    assert f["properties"]["way_points"][0] == 0
    body["destination_points"] = [dict(SMOKE["destination_points"][0], payload=99)]
    r = client.post("/api/request_route", json=body)
    assert r.json() == {"error": "payload exceeds vehicle capacity"}
    body["driver_details"] = dict(SMOKE["driver_details"], maximum_distance=1)
    r = client.post("/api/request_route", json=body)
    assert r.json()["error"] == "payload exceeds vehicle capacity | route distance exceeds maximum_distance"


def test_multi_stop_infeasible_returns_error_not_hang(client):
    body = json.loads(json.dumps(SMOKE))
    body["destination_points"][1]["payload"] = 50
    r = client.post("/api/optimize_route", json=body)
    assert r.status_code == 400 and "infeasible" in r.json()["error"]


def test_predict_eta(client):
    r = client.post("/api/predict_eta", json={"summary": {"distance": 12000}, "pickup_time": "2025-08-24T08:30:00Z",
                                              "driver_age": 40, "weather": "Stormy", "traffic": "Jam"})
    assert r.status_code == 200
    j = r.json()
    assert set(j) == {"eta_minutes_ml", "eta_completion_time_ml"}
    assert j["eta_completion_time_ml"].startswith("2025-08-24T")
    r = client.post("/api/predict_eta", json={"summary": {"distance": 1000}, "pickup_time": "not-a-date"})
    assert r.status_code == 400


def test_predict_batch_alias(client):
    items = [{"summary": {"distance": d}, "pickup_time": "2025-08-25T17:00:00"} for d in (1000, 5000, 20000)]
    r = client.post("/predict", json=items)
    assert r.status_code == 200
    preds = r.json()["predictions"]
    assert len(preds) == 3 and all("eta_minutes_ml" in p for p in preds)
    assert preds[0]["eta_minutes_ml"] < preds[2]["eta_minutes_ml"]
    r1 = client.post("/predict", json=items[1])
    assert abs(r1.json()["eta_minutes_ml"] - preds[1]["eta_minutes_ml"]) < 1e-4


def test_predict_eta_503_without_model():
    with _client(None) as c:
        r = c.post("/api/predict_eta", json={"summary": {"distance": 1000}})
        assert r.status_code == 503 and r.json() == {"error": "model unavailable"}
        # optimize_route still works, just without ML fields
        r = c.post("/api/optimize_route", json=F02)
        assert r.status_code == 200 and "eta_minutes_ml" not in r.json()["properties"]


def test_health_always_200(client):
    r = client.get("/api/health")
    assert r.status_code == 200
    j = r.json()
    assert {"backend", "checks", "db", "osrm", "redis", "tiles", "status", "version"} <= set(j)
    assert {"engine", "redis", "supabase"} <= set(j["checks"])
    assert j["status"] in ("ok", "degraded")
    # R10 "RCCL ready": collective readiness next to the gpu/model checks
    coll = j["checks"]["collectives"]
    assert coll["status"] in ("ok", "skipped") and "rccl_available" in coll and "dist_initialized" in coll


def test_history_without_store():
    with _client(None, store=None) as c:
        assert c.get("/api/history").status_code == 503
        assert c.get("/api/history/abc").status_code == 503
        assert c.delete("/api/history/abc").status_code == 503
    with _client(None, store=None, compat_history_500=True) as c:
        assert c.get("/api/history").status_code == 500


def test_history_limit_clamp(client):
    for _ in range(3):
        client.post("/api/optimize_route", json=dict(F02, use_ml_eta=False))
    assert len(client.get("/api/history?limit=0").json()["items"]) == 1
    assert len(client.get("/api/history?limit=abc").json()["items"]) >= 3
    assert len(client.get("/api/history?limit=2").json()["items"]) == 2


def test_update_tracker(client):
    assert client.post("/api/update_tracker", json={}).status_code == 400
    data = {"route_id": "drv", "route": [[121.0, 14.5], [121.1, 14.6]], "destinations": [],
            "duration": 600, "distance": 1000, "driver_name": "drv", "vehicle_type": "car",
            "pickup_time": "2025-08-24T10:00:00"}
    r = client.post("/api/update_tracker", json=data)
    assert r.status_code == 200 and r.json() == {"status": "published"}


def test_confirm_route(client):
    feat = client.post("/api/request_route", json=SMOKE).json()
    r = client.post("/api/confirm_route", json={"driver_details": {"driver_name": "d1", "vehicle_type": "car"},
                                                "route_details": feat})
    assert r.status_code == 200 and r.json() == {"status": "route simulation initialized."}


def test_locations(client):
    locs = client.get("/api/locations").json()
    assert len(locs) == 21 and locs[0]["name"] == "Main Warehouse - Mandaluyong"


def test_metrics(client):
    client.get("/api/ping")
    t = client.get("/metrics").text
    assert "routest_requests_total" in t and "routest_request_latency_seconds_bucket" in t


def test_cors_vercel(client):
    r = client.options("/api/ping", headers={"Origin": "https://x.vercel.app",
                                             "Access-Control-Request-Method": "GET"})
    assert r.headers.get("access-control-allow-origin") == "https://x.vercel.app"
    r = client.options("/api/ping", headers={"Origin": "https://evil.example",
                                             "Access-Control-Request-Method": "GET"})
    assert r.headers.get("access-control-allow-origin") is None


def test_batch_optimize(client):
    r = client.post("/api/optimize_routes_batch", json=[SMOKE, F02, {"destination_points": []}])
    res = r.json()["results"]
    assert res[0]["properties"]["summary"]["trips"] == 2
    assert "error" in res[2]
    single = client.post("/api/request_route", json=SMOKE).json()
    assert res[0]["properties"]["optimized_order"] == single["properties"]["optimized_order"]


def test_predict_batch_native_matches_single(client):
    import random
    rng = random.Random(5)
    items = [{"summary": {"distance": rng.uniform(100, 40000)}, "pickup_time": f"2025-08-2{rng.randint(0, 9)}T{rng.randint(0, 23):02d}:15:00",
              "driver_age": rng.randint(18, 70), "weather": rng.choice(["Sunny", "Stormy", "Windy", "Cloudy", "Hail"]),
              "traffic": rng.choice(["Low", "Medium", "High", "Jam"])} for _ in range(50)]
    items.append({"pickup_time": "garbage"})
    r = client.post("/predict", json=items)
    assert r.status_code == 200
    preds = r.json()["predictions"]
    assert "error" in preds[-1]
    for it, p in zip(items[:10], preds[:10]):
        one = client.post("/api/predict_eta", json=it).json()
        assert abs(one["eta_minutes_ml"] - p["eta_minutes_ml"]) < 1e-3
        assert one["eta_completion_time_ml"][:16] == p["eta_completion_time_ml"][:16]
