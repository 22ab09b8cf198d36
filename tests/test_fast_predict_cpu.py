"""The pure-ASGI native fast path for single predictions returns byte-identical responses to the
FastAPI handler (which stays the owner of every error / quirk case)."""
import json

import pytest
from fastapi.testclient import TestClient

from routest_amd.api.app import build_services, create_app
from routest_amd.config import load_settings
from routest_amd.models.mlp3 import LinearETA
from routest_amd.serve.eta_service import EtaService
from routest_amd.data.synth import synth_trips

BODIES = [
    {"summary": {"distance": 12345}, "pickup_time": "2025-08-25T08:30:00", "driver_age": 34,
     "weather": "Sunny", "traffic": "Medium"},
    {"summary": {"distance": "2500.5"}, "pickup_time": "2024-02-29T23:59:59.999999+05:30", "traffic": "Jam"},
    {"summary": {"distance": 800}, "pickup_time": "2025-01-01T00:00:00Z", "weather": "Hail", "driver_age": 0},
    {"summary": {"distance": True}, "pickup_time": "2025-06-01 12:00", "weather": None},
    {"summary": {"distance": 1e6}, "pickup_time": "2025-08-25T08:30:00", "driver_age": "41"},
    # error / quirk cases: handled by the FastAPI handler in both configurations
    {"summary": {"distance": "abc"}}, {"driver_age": None}, {"pickup_time": "not-a-date"},
    [1, 2], {"items": [{"summary": {"distance": 5}, "pickup_time": "2025-08-25T08:30:00"}]},
]


def _client(fast: bool, model):
    s = load_settings(env={"ROUTEST_FAST_PREDICT": "1" if fast else "0", "ROUTEST_DEVICE": "cpu"}, dotenv_path=None)
    return TestClient(create_app(build_services(s, eta=EtaService(model, device="cpu"), store=None)))


@pytest.fixture(scope="module")
def model():
    x, y = synth_trips(1000, 0)
    return LinearETA().fit(x, y)


@pytest.mark.parametrize("path", ["/api/predict_eta", "/predict"])
def test_fast_path_byte_identical(model, path):
    pytest.importorskip("routest_amd._rt")
    fast, slow = _client(True, model), _client(False, model)
    for b in BODIES:
        if path == "/api/predict_eta" and not isinstance(b, dict):
            continue
        rf = fast.post(path, content=json.dumps(b), headers={"content-type": "application/json"})
        rs = slow.post(path, content=json.dumps(b), headers={"content-type": "application/json"})
        assert rf.status_code == rs.status_code, b
        if "pickup_time" in (b if isinstance(b, dict) else {}) or rf.status_code != 200:
            assert rf.content == rs.content, (b, rf.content, rs.content)
    # non-JSON content type: silent -> {} semantics (distance 0, now())
    rf = fast.post("/api/predict_eta", content=b"hello", headers={"content-type": "text/plain"})
    rs = slow.post("/api/predict_eta", content=b"hello", headers={"content-type": "text/plain"})
    assert rf.status_code == rs.status_code == 200
    assert json.loads(rf.content)["eta_minutes_ml"] == json.loads(rs.content)["eta_minutes_ml"]


def test_fast_path_counts_and_cors(model):
    pytest.importorskip("routest_amd._rt")
    c = _client(True, model)
    r = c.post("/api/predict_eta", json=BODIES[0], headers={"Origin": "http://localhost:3000"})
    assert r.status_code == 200
    assert r.headers.get("access-control-allow-origin") == "http://localhost:3000"
