"""Candidate-route scorer: POST /api/score_routes (CPU reference path) and the HIP path vs CPU."""
import numpy as np
import pytest
import torch
from fastapi.testclient import TestClient

from routest_amd.data.graph import synth_road_graph
from routest_amd.models.gcn import GcnScorer, score_routes_ref
from routest_amd.routing.scorer import RouteScorer


@pytest.fixture(scope="module")
def graph():
    return synth_road_graph(3000, seed=2)


def _routes(g, k=4, n=12, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        idx = rng.integers(0, g.num_nodes, n)
        out.append([[float(g.lon[i]), float(g.lat[i])] for i in idx])
    return out


def test_scorer_cpu_matches_reference(graph):
    sc = RouteScorer(graph)
    routes = _routes(graph)
    res = sc.score(routes)
    with torch.no_grad():
        delay = GcnScorer(seed=0)(GcnScorer.adjacency(graph), torch.from_numpy(graph.features)).numpy()
    nodes = [sc.to_nodes(r) for r in routes]
    ref = score_routes_ref(graph, delay, nodes)
    np.testing.assert_allclose(res["scores"], ref, rtol=1e-5)
    assert res["best"] == int(np.argmin(ref)) and res["engine"] == "gcn-cpu"
    # node-id routes give the same answer as their coordinates
    assert sc.score([{"nodes": nodes[0]}])["scores"][0] == pytest.approx(res["scores"][0], rel=1e-6)


def test_score_routes_endpoint(graph):
    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    from routest_amd.models.mlp3 import LinearETA
    from routest_amd.serve.eta_service import EtaService
    from routest_amd.data.synth import synth_trips
    x, y = synth_trips(300, 0)
    s = load_settings(env={"ROUTEST_DEVICE": "cpu"}, dotenv_path=None)
    sv = build_services(s, eta=EtaService(LinearETA().fit(x, y), device="cpu"), store=None)
    sv.scorer = RouteScorer(graph)
    c = TestClient(create_app(sv))
    routes = _routes(graph, k=3)
    r = c.post("/api/score_routes", json={"routes": routes + [{"geometry": {"coordinates": routes[0]}}]})
    assert r.status_code == 200
    d = r.json()
    assert len(d["scores"]) == 4 and d["scores"][3] == pytest.approx(d["scores"][0])
    assert c.post("/api/score_routes", json={"routes": []}).status_code == 400
    assert c.post("/api/score_routes", json={"routes": [{"nodes": [10 ** 9]}]}).status_code == 400
    assert c.post("/api/score_routes", json={"routes": [[["a", "b"]]]}).status_code == 400


@pytest.mark.gpu
def test_scorer_hip_matches_cpu(graph):
    cpu = RouteScorer(graph)
    gpu = RouteScorer(graph, device="cuda:0")
    routes = _routes(graph, k=64, n=30, seed=3)
    a, b = cpu.score(routes), gpu.score(routes)
    assert b["engine"] == "gcn-hip"
    np.testing.assert_allclose(b["scores"], a["scores"], rtol=3e-2)
