"""Native route assembler (csrc/runtime/route_core.h) == the Python optimize_route path, byte for
byte (the FastAPI JSONResponse body), on the CPU.

The native front end (csrc/native_server.hip) answers /api/optimize_route, /route and
/api/request_route with this assembler; the Python app answers the same requests with
routing/optimizer.py.  The libm-dependent values (haversine, path lengths, snapping) come from one
shared implementation; everything else — request coercions, greedy trips (R21), densified
directions, rounding (builtin round vs numpy.round), float repr, key order, error texts — is
implemented twice and must agree exactly.  Reference: RO/Flaskr/utils.py:10-201,
RO/Flaskr/routes.py:29-50,89-127."""
import json

import numpy as np
import pytest
from starlette.responses import JSONResponse

from routest_amd.ops import _ext
from routest_amd.routing.optimizer import optimize_route
from routest_amd.routing.providers import HaversineProvider

rt = _ext.runtime(required=False)
pytestmark = pytest.mark.skipif(rt is None, reason="routest_amd._rt not built")

VTS = ["car", "Truck ", "bike", "roadbike", "FOOT", "hgv", "motorcycle", None, 5, "spaceship", ""]


def _payloads(n, seed=0, center=(14.55, 121.02), spread=0.05):
    rng = np.random.default_rng(seed)
    out = []
    for it in range(n):
        k = int(rng.integers(1, 12))
        pts = [{"lat": float(center[0] + rng.normal(0, spread)), "lon": float(center[1] + rng.normal(0, spread)),
                "payload": int(rng.integers(0, 4))} for _ in range(k)]
        if it % 7 == 0:
            pts[0]["lat"] = 14                     # int coordinates echo back as ints
        if it % 11 == 0:
            pts[0]["name"] = "Mall é \"x\"\n☃"  # non-ASCII + escapes in an echoed field
        if it % 9 == 0:
            pts[-1]["payload"] = 2.5
        drv = {"driver_name": f"d{it}" if it % 5 else None, "vehicle_type": VTS[it % len(VTS)],
               "vehicle_capacity": int(rng.integers(1, 8)), "maximum_distance": float(rng.uniform(5e3, 8e4))}
        if it % 13 == 0:
            del drv["maximum_distance"]
        if it % 23 == 0:
            drv["vehicle_capacity"] = 0            # every stop infeasible on its own
        p = {"source_point": {"lat": float(center[0] + rng.normal(0, 0.02)), "lon": center[1]},
             "destination_points": pts, "driver_details": drv}
        if it % 29 == 0:
            del p["driver_details"]
        if it % 17 == 0:
            p = {"destination_points": []}
        if it % 19 == 0:
            p["source_point"] = {"lat": 1}
        out.append(p)
    return out


def _python(payload, provider):
    res = optimize_route(payload, provider, "backend:mi355x")
    return (400 if res.get("error") else 200), JSONResponse(res).body


def test_haversine_requests_byte_identical():
    prov = HaversineProvider()
    n = 0
    for p in _payloads(2000):
        body = json.dumps(p).encode()
        got = rt.route_optimize_cpu(body)
        assert got is not None, p
        assert got == _python(json.loads(body), prov), p
        n += 1
    assert n == 2000


def test_silent_body_and_request_route_semantics():
    # optimize_route (silent JSON): a non-JSON body or a non-dict reads as {}
    for body, ok in ((b"not json", False), (b"[1,2]", True), (b"null", True), (b"", True)):
        st, out = rt.route_optimize_cpu(body, json_ok=ok)
        assert st == 400 and json.loads(out) == {"error": "no destination points specified."}
    # request_route: errors answered 200 (reference quirk), non-JSON left to the Python app
    st, out = rt.route_optimize_cpu(b'{"destination_points": []}', is_request_route=True)
    assert st == 200
    assert rt.route_optimize_cpu(b"{bad", is_request_route=True) is None
    assert rt.route_optimize_cpu(b"{}", json_ok=False, is_request_route=True) is None


@pytest.mark.parametrize("payload", [
    {"source_point": {"lat": "14.5", "lon": 121.0}, "destination_points": [{"lat": 14.6, "lon": 121.0}]},
    {"source_point": {"lat": 14.5, "lon": 121.0}, "destination_points": [{"lat": 14.6, "lon": 121.0}],
     "driver_details": ["x"]},
    {"source_point": {"lat": 14.5, "lon": 121.0}, "destination_points": {"a": 1}},
    {"source_point": {"lat": 14.5, "lon": 121.0}, "destination_points": [{"lat": 14.6, "lon": 121.0,
                                                                          "payload": "3"}, {"lat": 14.7, "lon": 121.0}]},
    {"source_point": {"lat": 14.5, "lon": 121.0}, "destination_points": [{"lat": 14.6, "lon": 121.0}],
     "driver_details": {"vehicle_type": "Lastwagenä"}},
])
def test_unmirrored_semantics_fall_back_to_python(payload):
    """Inputs whose Python coercions are not reproduced natively are handed to the Python app."""
    assert rt.route_optimize_cpu(json.dumps(payload).encode()) is None


def test_python_numerics_helpers():
    import math
    for x in (0.25, 0.35, 2.675, 1234.55, -0.05, 1e16 + 2.0, 0.0):
        assert rt.py_round(x, 1) == round(x, 1)
    from routest_amd.routing.providers import _bearing_word
    rng = np.random.default_rng(3)
    for _ in range(500):
        a = rng.uniform(-80, 80, 4)
        assert rt.bearing_word(*a) == _bearing_word(*a)
    assert math.isclose(rt.haversine_m(14.5, 121.0, 14.6, 121.1), 15_000, rel_tol=0.1)


def test_graph_assembly_byte_identical():
    """Road-graph provider: the same trips, snapped nodes and searched legs (seconds, metres, path
    from the CPU CCH) assemble to the same bytes — maneuver steps included — as
    GraphProvider.feature_from_legs + optimize_route."""
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.routing.greedy import InfeasibleStops, greedy_trips
    g = synth_road_graph(3000, seed=1)
    cost = (g.length_m / 9.0).astype(np.float32)
    prov = GraphProvider(g, cost, device=None)
    rng = np.random.default_rng(4)
    checked = 0
    for it, p in enumerate(_payloads(300, seed=5, center=(14.57, 121.02), spread=0.08)):
        body = json.dumps(p).encode()
        want_st, want = _python(json.loads(body), prov)
        r = json.loads(body)
        pts = [r.get("source_point")] + list(r.get("destination_points") or [])
        trips = None
        if isinstance(r.get("destination_points"), list) and len(r["destination_points"]) > 1 and \
                isinstance(r.get("source_point"), dict) and "lon" in r["source_point"]:
            d = prov.matrix(pts, "driving-car")
            drv = r.get("driver_details") or {}
            try:
                trips = greedy_trips(np.asarray(d).tolist(), [0.0] + [float(q.get("payload", 0)) for q in pts[1:]],
                                     float(drv.get("vehicle_capacity", 9e12)), float(drv.get("maximum_distance", 9e12)))
            except InfeasibleStops:
                continue                          # error text covered by the haversine test
        calls = ([[pts[0], pts[1]]] if trips is None and len(pts) == 2 else
                 [[pts[i] for i in t] for t in (trips or [])])
        if want_st != 200 or not calls:
            continue
        nodes = np.concatenate([g.nearest_nodes([q["lat"] for q in c], [q["lon"] for q in c]) for c in calls])
        pairs, o = set(), 0
        for c in calls:
            pairs.update((int(nodes[o + i]), int(nodes[o + i + 1])) for i in range(len(c) - 1))
            o += len(c)
        legs = dict(zip(sorted(pairs), prov.legs(sorted(pairs))[0]))
        got = rt.route_assemble_graph(body, "backend:mi355x", g.lat, g.lon, nodes.astype(np.int32), trips,
                                      {k: tuple(v) for k, v in legs.items()}, prov._steps, prov.cost)
        assert got == (want_st, want), it
        checked += 1
    assert checked > 80


def test_compact_route_record_rebuilds_byte_identical():
    """csrc/runtime/route_record.h: the record the route service persists for a
    graph route — waypoints, per-hop adjacency slots, seconds / metres per leg, step durations in
    tenths — decodes, against the same graph, to exactly the legs and geometry texts the assembly
    wrote; it is a small fraction of their size; another graph is refused."""
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.routing.greedy import InfeasibleStops, greedy_trips
    g = synth_road_graph(3000, seed=1)
    cost = (g.length_m / 9.0).astype(np.float32)
    prov = GraphProvider(g, cost, device=None)
    other = GraphProvider(synth_road_graph(3000, seed=2), cost, device=None)
    checked, rec_bytes, text_bytes = 0, 0, 0
    for it, p in enumerate(_payloads(300, seed=5, center=(14.57, 121.02), spread=0.08)):
        body = json.dumps(p).encode()
        r = json.loads(body)
        pts = [r.get("source_point")] + list(r.get("destination_points") or [])
        if not (isinstance(r.get("source_point"), dict) and "lon" in r["source_point"] and
                isinstance(r.get("destination_points"), list) and r["destination_points"]):
            continue
        if not all(isinstance(q, dict) and isinstance(q.get("lat"), (int, float)) and
                   isinstance(q.get("lon"), (int, float)) for q in pts):
            continue
        trips = None
        if len(pts) > 2:
            d = prov.matrix(pts, "driving-car")
            drv = r.get("driver_details") or {}
            try:
                trips = greedy_trips(np.asarray(d).tolist(), [0.0] + [float(q.get("payload", 0)) for q in pts[1:]],
                                     float(drv.get("vehicle_capacity", 9e12)), float(drv.get("maximum_distance", 9e12)))
            except (InfeasibleStops, TypeError, ValueError):
                continue
        calls = [[pts[0], pts[1]]] if trips is None else [[pts[i] for i in t] for t in trips]
        nodes = np.concatenate([g.nearest_nodes([q["lat"] for q in c], [q["lon"] for q in c]) for c in calls])
        pairs, o = set(), 0
        for c in calls:
            pairs.update((int(nodes[o + i]), int(nodes[o + i + 1])) for i in range(len(c) - 1))
            o += len(c)
        legs = dict(zip(sorted(pairs), prov.legs(sorted(pairs))[0]))
        for with_steps in (True, False):
            got = rt.route_assemble_graph(body, "backend:mi355x", g.lat, g.lon, nodes.astype(np.int32), trips,
                                          {k: tuple(v) for k, v in legs.items()}, prov._steps,
                                          prov.cost if with_steps else None, with_record=True)
            if got is None or got[0] != 200:
                break
            st, resp, rec, seg, geo = got
            assert rec is not None, it
            assert prov._steps.decode_record(rec) == (seg, geo), it
            resp_j = json.loads(resp)
            assert json.loads(seg) == resp_j["properties"]["segments"]
            assert json.loads(geo) == resp_j["geometry"]
            if with_steps:
                rec_bytes += len(rec)
                text_bytes += len(seg) + len(geo)
                checked += 1
                with pytest.raises(ValueError, match="another road graph"):
                    other._steps.decode_record(rec)
                with pytest.raises(ValueError):
                    prov._steps.decode_record(rec[:-3])
                if checked % 10 == 1:        # corrupted rows: refused or decoded, never a crash
                    frng = np.random.default_rng(checked)
                    for _ in range(60):
                        b = bytearray(rec)
                        for _ in range(int(frng.integers(1, 4))):
                            b[int(frng.integers(12, len(b)))] = int(frng.integers(0, 256))
                        if frng.random() < 0.3:
                            b = b[:int(frng.integers(12, len(b)))]
                        try:
                            out = prov._steps.decode_record(bytes(b))
                            assert isinstance(out, tuple) and len(out) == 2
                        except ValueError:
                            pass
    assert checked > 80
    print(f"record {rec_bytes / checked:.0f} B vs text {text_bytes / checked:.0f} B per route")
    assert rec_bytes * 6 < text_bytes, (rec_bytes, text_bytes)


def test_float_fast_paths_match_python():
    """py_round(x, 1) and the JSON float writer take integer-tenths fast paths (route steps): every
    result equals Python's round() / json.dumps, midpoints and large magnitudes included."""
    import json
    import random
    rt = __import__("pytest").importorskip("routest_amd._rt")
    rnd = random.Random(3)
    vals = [0.05, 0.15, 0.25, 2.675, -0.04, -0.05, 1e8 + 0.05, 123456789.95, 0.0, -0.0, 1e-5, 5e-5,
            0.45, 1.45, 2.5, 999999999.95, 1e9 + 0.25, 3e15, 1e16, 1e17]
    for _ in range(20000):
        e = rnd.uniform(-6, 11)
        vals.append(rnd.choice([-1, 1]) * 10 ** e)
        vals.append(round(rnd.uniform(0, 5000), 2) + rnd.choice([0.0, 0.05, 0.049999999, 0.050000001]))
    for v in vals:
        r = rt.py_round(v, 1)
        assert r == round(v, 1) and (str(r) == str(round(v, 1))), v
        assert rt.json_float(r) == json.dumps(r), r
        assert rt.json_float(v) == json.dumps(v), v
