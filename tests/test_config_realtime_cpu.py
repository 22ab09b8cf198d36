"""Config precedence (R01 fix: .env read before any service reads settings) and the SSE path end to
end (R07/R08/R26): a subscriber on /api/realtime_feed receives the R26 payload published by
/api/update_tracker, in Flask-SSE's `data:` wire format."""
import asyncio
import json

from routest_amd.config import load_settings


def test_dotenv_then_env_then_overrides(tmp_path):
    p = tmp_path / ".env"
    p.write_text("OPENROUTESERVICE_API_KEY=from-dotenv\nETA_MODEL_PATH=/m/a\nROUTEST_BATCH_MAX=128\n"
                 "SUPABASE_URL=https://x.supabase.co\nSUPABASE_SERVICE_ROLE_KEY=k\n")
    s = load_settings(env={"ETA_MODEL_PATH": "/m/b"}, dotenv_path=str(p))
    assert s.ors_api_key == "from-dotenv"          # reference alias name accepted
    assert s.eta_model_path == "/m/b"               # process env beats .env
    assert s.batch_max == 128
    assert s.store_url == "postgrest"               # Supabase configured -> PostgREST store
    s2 = load_settings(env={}, dotenv_path=str(p), batch_max=7)
    assert s2.batch_max == 7                        # explicit overrides win
    s3 = load_settings(env={"ORS_API_KEY": "primary"}, dotenv_path=None)
    assert s3.ors_api_key == "primary" and s3.store_url.startswith("sqlite")


def test_route_pipelines_setting():
    """Native route services per GPU: explicit, or auto (2 when the route service persists every
    answer into the SQLite store, else 1; serve/frontend.py route_pipelines_for)."""
    from types import SimpleNamespace
    from routest_amd.serve.frontend import route_pipelines_for
    assert load_settings(env={}, dotenv_path=None).route_pipelines == 0          # auto
    assert load_settings(env={"ROUTEST_ROUTE_PIPELINES": "2"}, dotenv_path=None).route_pipelines == 2
    assert load_settings(env={"ROUTEST_ROUTE_PIPELINES": "-1"}, dotenv_path=None).route_pipelines == 0
    assert load_settings(env={}, dotenv_path=None, route_pipelines=3).route_pipelines == 3
    auto = load_settings(env={}, dotenv_path=None)
    assert route_pipelines_for(SimpleNamespace(settings=auto, store=None)) == 1
    assert route_pipelines_for(SimpleNamespace(settings=auto, store=SimpleNamespace(kind="sqlite"))) == 2
    assert route_pipelines_for(SimpleNamespace(settings=auto, store=SimpleNamespace(kind="postgrest"))) == 1
    three = load_settings(env={}, dotenv_path=None, route_pipelines=3)
    assert route_pipelines_for(SimpleNamespace(settings=three, store=None)) == 3


def test_sse_stream_receives_tracker_update():
    import httpx
    from routest_amd.api.app import build_services, create_app
    from routest_amd.models.mlp3 import LinearETA
    from routest_amd.serve.eta_service import EtaService
    from routest_amd.data.synth import synth_trips
    x, y = synth_trips(500, 0)
    s = load_settings(env={"ROUTEST_DEVICE": "cpu"}, dotenv_path=None)
    sv = build_services(s, eta=EtaService(LinearETA().fit(x, y), device="cpu"), store=None)
    app = create_app(sv)
    data = {"route_id": "drv-9", "route": [[121.0, 14.5], [121.1, 14.6]], "destinations": [{"lat": 14.6}],
            "duration": 600, "distance": 1000, "driver_name": "drv-9", "vehicle_type": "car",
            "pickup_time": "2025-08-24T10:00:00"}

    async def main():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t") as c:
            q = sv.broker.subscribe("drv-9")                 # same broker the feed endpoint uses
            r = await c.post("/api/update_tracker", json=data)
            assert r.status_code == 200
            msg = await asyncio.wait_for(q.get(), 5)
            sv.broker.unsubscribe("drv-9", q)
            return msg
    msg = asyncio.run(main())
    assert msg.startswith("data:") and msg.endswith("\n\n")
    payload = json.loads(msg[len("data:"):].strip())
    assert payload["assigned_driver"] == "drv-9"
    assert payload["overall_estimated_completion_time"] == "2025-08-24T10:10:00"
    assert payload["remaining_routes"] == data["route"]
