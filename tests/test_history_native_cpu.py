"""Native history / locations reads (csrc/runtime/history_db.h, verdict r3 item 8) are
byte-identical to the FastAPI handlers over the same SQLite database (routest_amd/api/app.py
history, history_detail, delete_history, locations; reference RO/Flaskr/routes.py:185-279,386-406)."""
import numpy as np
import pytest
from fastapi.testclient import TestClient

rt = pytest.importorskip("routest_amd._rt")


@pytest.fixture()
def app_and_db():
    from routest_amd.api.app import build_services, create_app
    from routest_amd.config import load_settings
    from routest_amd.serve.eta_service import EtaService, default_model
    from routest_amd.store.store import SQLiteStore
    s = load_settings(env={}, dotenv_path=None, device="cpu", route_batch="0", warm_scorer=False)
    store = SQLiteStore(":memory:")
    sv = build_services(s, eta=EtaService(default_model(hidden=64, steps=20), device="cpu"), store=store)
    c = TestClient(create_app(sv))
    rng = np.random.default_rng(0)
    for i in range(25):
        n = int(rng.integers(1, 5))
        p = {"source_point": {"lat": 14.58 + rng.random() * 0.02, "lon": 121.05 + rng.random() * 0.02},
             "destination_points": [{"lat": 14.55 + rng.random() * 0.03, "lon": 121.03 + rng.random() * 0.03,
                                     "payload": 1} for _ in range(n)],
             "driver_details": {"driver_name": f"drv{i}" if i % 4 else None, "vehicle_type": "car",
                                "driver_age": [30, 41.5, None][i % 3]},
             "meta": {"origin_id": None if i % 2 else f"o{i}",
                      "destination_ids": [f"d{i}_{k}" for k in range(n)] if i % 5 else []},
             "use_ml_eta": i % 3 == 0, "context": {"weather": "Sunny", "traffic": "Medium"}}
        r = c.post("/api/optimize_route", json=p)
        assert r.status_code == 200, r.text
    db = rt.HistoryDb(store.sqlite_uri)
    yield c, db
    sv.close() if hasattr(sv, "close") else None


def test_history_list_and_limits(app_and_db):
    c, db = app_and_db
    for lim in (None, "5", "1", "0", "250", "abc", " 7 ", "-3", ""):
        ref = c.get("/api/history" + ("" if lim is None else f"?limit={lim}"))
        got = db.history(lim)
        assert got is not None, lim
        assert got == (ref.status_code, ref.content), (lim, got[1][:200], ref.content[:200])


def test_history_detail_delete_and_locations(app_and_db):
    c, db = app_and_db
    items = c.get("/api/history?limit=100").json()["items"]
    assert len(items) == 25
    for it in items[:10]:
        rid = it["request_id"]
        ref = c.get(f"/api/history/{rid}")
        assert db.detail(rid) == (200, ref.content)
    assert db.detail("nope") == (404, c.get("/api/history/nope").content)
    rid = items[0]["request_id"]
    assert db.delete(rid) == (204, b"")
    assert c.get(f"/api/history/{rid}").status_code == 404          # the app sees the native delete
    assert db.history("100")[1] == c.get("/api/history?limit=100").content
    assert db.locations() == (200, c.get("/api/locations").content)


def test_native_reads_see_later_writes_and_deletes(app_and_db):
    """No statement is left open between calls: a held read transaction would pin an old WAL
    snapshot, so rows the app writes or deletes afterwards would be missing / still listed."""
    c, db = app_and_db
    items = c.get("/api/history?limit=100").json()["items"]
    assert db.detail(items[0]["request_id"])[0] == 200          # leaves nothing open
    assert db.history("3")[0] == 200
    assert c.delete(f"/api/history/{items[1]['request_id']}").status_code == 204
    p = {"source_point": {"lat": 14.58, "lon": 121.05}, "destination_points": [{"lat": 14.56, "lon": 121.04}],
         "driver_details": {"driver_name": "late", "vehicle_type": "car"}, "meta": {"origin_id": "late-1"}}
    assert c.post("/api/optimize_route", json=p).status_code == 200
    assert db.history("100")[1] == c.get("/api/history?limit=100").content
    assert db.detail(items[1]["request_id"])[0] == 404


def test_side_file_references_resolve_identically(app_and_db):
    """Rows written by the native route service keep legs / geometry in <db>.blobs (a reference in
    the column, store.py BLOB_REF): the app and the native reader resolve them to the same bytes,
    and the detail is identical to the inline row it replaces."""
    import sqlite3
    from routest_amd.store.store import BLOB_REF
    c, db = app_and_db
    store = c.app.state.services.store
    items = c.get("/api/history?limit=100").json()["items"]
    before = {it["request_id"]: c.get(f"/api/history/{it['request_id']}").content for it in items[:8]}
    con = sqlite3.connect(store.sqlite_uri, isolation_level=None)
    with open(store.blob_path, "ab") as f:
        off = f.tell()
        for rid in before:
            legs, geom = con.execute("SELECT legs, geometry FROM route_results WHERE request_id=?", (rid,)).fetchone()
            lb, gb = legs.encode(), geom.encode()
            f.write(b"xx" + lb + gb)                 # (some unrelated bytes first)
            ref_l = f"{BLOB_REF}{off + 2}:{len(lb)}"
            ref_g = f"{BLOB_REF}{off + 2 + len(lb)}:{len(gb)}"
            con.execute("UPDATE route_results SET legs=?, geometry=? WHERE request_id=?", (ref_l, ref_g, rid))
            off += 2 + len(lb) + len(gb)
    con.close()
    for rid, ref in before.items():
        app = c.get(f"/api/history/{rid}")
        assert app.status_code == 200 and app.content == ref
        assert db.detail(rid) == (200, ref)
    assert db.history("100")[1] == c.get("/api/history?limit=100").content


def test_compact_route_records_read_back_identically(tmp_path):
    """the native route service persists a graph route as a compact record (a
    BLOB in route_results.legs, geometry NULL; csrc/runtime/route_record.h).  The app (through the
    provider's GraphSteps) and the native history reader rebuild history detail byte-identically to
    the same route stored as text — and a reader without the graph relays / refuses instead of
    answering something else."""
    import json
    import sqlite3
    from routest_amd.data.graph import synth_road_graph
    from routest_amd.routing.graph import GraphProvider
    from routest_amd.routing.greedy import InfeasibleStops, greedy_trips
    from routest_amd.store.store import RECORD_MAGIC, SQLiteStore, StoreUnavailable
    g = synth_road_graph(3000, seed=1)
    prov = GraphProvider(g, (g.length_m / 9.0).astype(np.float32), device=None)
    store = SQLiteStore(str(tmp_path / "r.db"))
    store.set_record_graph(prov._steps)
    rng = np.random.default_rng(7)
    recs = {}
    for i in range(40):
        k = int(rng.integers(1, 8))
        pts = [{"lat": 14.57 + rng.normal(0, 0.05), "lon": 121.02 + rng.normal(0, 0.05), "payload": 1}
               for _ in range(k + 1)]
        p = {"source_point": pts[0], "destination_points": pts[1:],
             "driver_details": {"driver_name": f"d{i}", "vehicle_type": "car", "vehicle_capacity": 99,
                                "maximum_distance": 1e7, "driver_age": 30 + i},
             "meta": {"origin_id": f"o{i}", "destination_ids": [f"x{j}" for j in range(k)]}, "use_ml_eta": False}
        trips = None
        if k > 1:
            try:
                trips = greedy_trips(np.asarray(prov.matrix(pts, "driving-car")).tolist(), [0.0] + [1.0] * k, 99.0, 1e7)
            except InfeasibleStops:
                continue
        calls = [[pts[0], pts[1]]] if trips is None else [[pts[j] for j in t] for t in trips]
        nodes = np.concatenate([g.nearest_nodes([q["lat"] for q in c], [q["lon"] for q in c]) for c in calls])
        pairs, o = set(), 0
        for c in calls:
            pairs.update((int(nodes[o + j]), int(nodes[o + j + 1])) for j in range(len(c) - 1))
            o += len(c)
        legs = dict(zip(sorted(pairs), prov.legs(sorted(pairs))[0]))
        st, resp, rec, seg, geo = rt.route_assemble_graph(json.dumps(p).encode(), "backend:mi355x", g.lat, g.lon,
                                                          nodes.astype(np.int32), trips,
                                                          {kk: tuple(v) for kk, v in legs.items()}, prov._steps,
                                                          prov.cost, with_record=True)
        assert st == 200 and rec is not None and rec[:4] == RECORD_MAGIC
        rid = store.persist_request_and_result(p, json.loads(resp))
        recs[rid] = rec
    assert len(recs) > 25
    native = rt.HistoryDb(store.sqlite_uri, graph=prov._steps)
    text_detail = {rid: native.detail(rid) for rid in recs}
    app_text = {rid: json.dumps(store.history_detail(rid)) for rid in recs}
    con = sqlite3.connect(store.sqlite_uri, isolation_level=None)
    for rid, rec in recs.items():
        con.execute("UPDATE route_results SET legs=?, geometry=NULL WHERE request_id=?", (rec, rid))
    con.close()
    for rid in recs:
        assert native.detail(rid) == text_detail[rid]
        assert json.dumps(store.history_detail(rid)) == app_text[rid]
    # no graph: the native reader relays to the app, which refuses rather than answering wrongly
    assert rt.HistoryDb(store.sqlite_uri).detail(next(iter(recs))) is None
    store.set_record_graph(None)
    with pytest.raises(StoreUnavailable):
        store.history_detail(next(iter(recs)))
    store.close()
