"""Built-in dashboard (/ui): served by the app and wired to the reference wire contract
(the reference's own Next.js dashboard keeps working unchanged)."""
from fastapi.testclient import TestClient

from routest_amd.api.app import build_services, create_app
from routest_amd.config import load_settings
from routest_amd.serve.eta_service import EtaService
from routest_amd.store.store import SQLiteStore


def _client():
    s = load_settings(env={}, dotenv_path=None, device="cpu")
    sv = build_services(s, eta=EtaService(None, device="cpu"), store=SQLiteStore(":memory:"))
    return TestClient(create_app(sv))


def test_dashboard_pages_served():
    with _client() as c:
        for path in ("/ui", "/ui/", "/ui/history", "/ui/history/abc-123", "/ui/health"):
            r = c.get(path)
            assert r.status_code == 200, path
            assert r.headers["content-type"].startswith("text/html")
            assert "routest_amd dashboard" in r.text


def test_dashboard_uses_reference_contract():
    with _client() as c:
        html = c.get("/ui").text
    # every endpoint the reference dashboard calls, the F02 request fields, the F04 backoff
    for needle in ('"/optimize_route"', '"/confirm_route"', "/realtime_feed?channel=", '"/history?limit=20"',
                   '"/history?limit=100"', '"/locations"', '"/health"', '"/ping"',
                   "vehicle_capacity: 9999", "maximum_distance: 100000", "use_ml_eta", "MAX_STOPS = 10",
                   "Math.min(1000 * 2 ** n, 20000)"):
        assert needle in html, needle


def test_dashboard_flow_endpoints_roundtrip():
    """The calls the page makes, in its order: locations -> optimize (saved) -> history -> detail
    -> delete."""
    with _client() as c:
        locs = c.get("/api/locations").json()
        o, d1, d2 = locs[0], locs[1], locs[2]
        req = {"source_point": {"lat": o["latitude"], "lon": o["longitude"]},
               "destination_points": [{"lat": d["latitude"], "lon": d["longitude"], "payload": 1} for d in (d1, d2)],
               "driver_details": {"driver_name": "ui-1", "vehicle_type": "car", "vehicle_capacity": 9999,
                                  "maximum_distance": 100000, "driver_age": 30},
               "meta": {"origin_id": o["id"], "destination_ids": [d1["id"], d2["id"]], "vehicle_id": "ui-1"},
               "use_ml_eta": False, "context": {"weather": "Sunny", "traffic": "Medium"}}
        feat = c.post("/api/optimize_route", json=req).json()
        rid = feat["properties"]["request_id"]
        items = c.get("/api/history?limit=20").json()["items"]
        assert items[0]["request_id"] == rid and items[0]["dest_count"] == 2
        det = c.get(f"/api/history/{rid}").json()
        assert det["request"]["origin_id"] == o["id"]
        assert c.delete(f"/api/history/{rid}").status_code == 204
