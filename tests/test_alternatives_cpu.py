"""``"alternatives": k`` on /api/optimize_route: every leg chosen among k candidates (shortest path
+ via-node detours) by the trained GCN scorer (routing/alternatives.py; CPU path here, the GPU path
uses the batched A* and the HIP scorer)."""
import json

import numpy as np
from fastapi.testclient import TestClient


def _app():
    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.serve.eta_service import EtaService
    g = synth_road_graph(3000, seed=6)
    cost = (g.length_m / np.array([8.3, 12.5, 16.7, 22.2])[g.road_class]).astype(np.float32)
    s = load_settings(env={}, dotenv_path=None, device="cpu", route_batch="0", warm_scorer=False,
                      scorer_train_steps=40)
    sv = build_services(s, eta=EtaService(None, device="cpu"), provider=GraphProvider(g, cost, device=None),
                        store=None)
    return TestClient(create_app(sv)), g, sv


def test_alternatives_chosen_by_scorer():
    c, g, sv = _app()
    rng = np.random.default_rng(2)
    idx = rng.integers(0, g.num_nodes, 4)
    body = {"source_point": {"lat": float(g.lat[idx[0]]), "lon": float(g.lon[idx[0]])},
            "destination_points": [{"lat": float(g.lat[i]), "lon": float(g.lon[i]), "payload": 1} for i in idx[1:]],
            "driver_details": {"driver_name": "x", "vehicle_type": "car", "vehicle_capacity": 9, "maximum_distance": 1e7},
            "alternatives": 3}
    r = c.post("/api/optimize_route", json=body)
    assert r.status_code == 200, r.text
    p = r.json()["properties"]
    alt = p["alternatives"]
    assert alt["k"] == 3 and alt["scorer"] == "gcn-cpu" and len(alt["legs"]) >= 3
    for leg in alt["legs"]:
        assert leg["candidates"] >= 1 and leg["chosen"] == int(np.argmin(leg["scores"]))
        assert len(leg["seconds"]) == leg["candidates"]
    assert sv.get_scorer().training is not None            # the scorer was trained on the edge times
    # without the flag: the plain optimizer answer (no alternatives block)
    body.pop("alternatives")
    r2 = c.post("/api/optimize_route", json=body)
    assert r2.status_code == 200 and "alternatives" not in r2.json()["properties"]
    # the native route core leaves such requests to the Python app
    from routest_amd.ops import _ext
    rt = _ext.runtime(required=False)
    if rt is not None:
        body["alternatives"] = 3
        assert rt.route_optimize_cpu(json.dumps(body).encode()) is None
