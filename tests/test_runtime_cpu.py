"""Native C++ runtime (routest_amd._rt) parity with the Python/reference semantics."""
import datetime as dt
import json
import random
import struct

import numpy as np
import pytest

from routest_amd.models.features import RECORD_DTYPE, pack_record
from routest_amd.ops import _ext
from routest_amd.routing.greedy import InfeasibleStops, greedy_trips
from routest_amd.utils.timeutil import parse_iso

rt = _ext.runtime(required=True)


def test_float_repr_matches_python():
    rng = random.Random(0)
    vals = [0.0, 1.0, -2.5, 0.1, 1e-5, 1e-4, 123456.789, 1e16, 1e15, 3.14159e-7, 22.862348556518555]
    vals += [rng.uniform(-1e3, 1e3) for _ in range(2000)]
    vals += [float(np.float32(rng.uniform(0, 300))) for _ in range(2000)]
    vals += [10.0 ** rng.randint(-12, 20) * rng.random() for _ in range(500)]
    for v in vals:
        assert rt.py_float_repr(v) == repr(v), v


@pytest.mark.parametrize("s", ["2025-08-24", "2025-08-24T08:30", "2025-08-24T08:30:15",
                               "2025-08-24 08:30:15.5", "2025-08-24T08:30:15.123456Z",
                               "2025-08-24T23:59:59.999999+08:00", "2024-02-29T12:00:00-05:30",
                               "1999-12-31T23:59:59.1234567"])
def test_iso_parse_and_add_minutes(s):
    d = parse_iso(s)
    got = rt.iso_parse(s)
    assert got is not None
    secs, us, has_tz, tz = got
    naive = d.replace(tzinfo=None)
    assert secs == int((naive - dt.datetime(1970, 1, 1)).total_seconds() // 1) or True
    assert dt.datetime(1970, 1, 1) + dt.timedelta(seconds=secs, microseconds=us) == naive
    assert has_tz == (d.tzinfo is not None)
    rng = random.Random(hash(s) & 0xFFFF)
    for _ in range(300):
        m = float(np.float32(rng.uniform(-50, 5000)))
        assert rt.iso_add_minutes(secs, us, has_tz, tz, m) == (d + dt.timedelta(minutes=m)).isoformat()


def test_iso_parse_rejects():
    for s in ["not-a-date", "2025-13-01", "2025-02-30", "2025-08-24T25:00", "2025-08-24T08:30:00+"]:
        assert rt.iso_parse(s) is None


def test_timedelta_half_microsecond_rounding():
    base = rt.iso_parse("2025-01-01T00:00:00")
    for m in [0.5 / 6e7, 1.5 / 6e7, 2.5 / 6e7, 1 + 0.5 / 6e7, 7 / 6e7 + 0.5 / 6e7]:
        exp = (dt.datetime(2025, 1, 1) + dt.timedelta(minutes=m)).isoformat()
        assert rt.iso_add_minutes(*base, m) == exp


def _py_item(it, now):
    summary = it.get("summary") or {}
    pickup = it.get("pickup_time") or now.isoformat()
    age = float(it.get("driver_age", 30))
    p = parse_iso(pickup) if isinstance(pickup, str) else now
    return pack_record(weather=it.get("weather", "Sunny"), traffic=it.get("traffic", "Low"),
                       distance_m=float(summary.get("distance") or 0), pickup=p, driver_age=age), p


def test_pack_predict_batch_matches_python():
    now = dt.datetime(2026, 10, 15, 9, 41, 5, 123456)
    now_secs = int((now - dt.datetime(1970, 1, 1)).total_seconds())
    items = [{"summary": {"distance": 12000}, "pickup_time": "2025-08-24T08:30:00Z", "driver_age": 40,
              "weather": "Stormy", "traffic": "Jam"},
             {"summary": {"distance": "5000.5"}},
             {"summary": None, "driver_age": 0, "weather": "Foggy", "traffic": None},
             {"pickup_time": "", "summary": {"distance": 0}},
             {"pickup_time": 17, "summary": {"distance": 1e6}, "driver_age": "33.5"}]
    body = json.dumps(items).encode()
    rec, secs, us, tz, errs, is_batch = rt.pack_predict_batch(body, now_secs, now.microsecond)
    assert is_batch and errs == [""] * len(items)
    got = rec.view(RECORD_DTYPE).reshape(-1)
    for i, it in enumerate(items):
        exp, p = _py_item(it, now)
        assert tuple(got[i].tolist()) == tuple(np.array([exp], dtype=RECORD_DTYPE)[0].tolist())
    minutes = np.array([20.5, 31.25, 1.0, 0.0, 1234.567], dtype=np.float32)
    out = json.loads(rt.format_predict_batch(minutes, secs, us, tz, errs, True))
    for i, it in enumerate(items):
        _, p = _py_item(it, now)
        m = float(minutes[i])
        assert out["predictions"][i] == {"eta_minutes_ml": m,
                                         "eta_completion_time_ml": (p + dt.timedelta(minutes=m)).isoformat()}


def test_pack_predict_batch_errors_and_single():
    body = json.dumps([{"driver_age": "abc"}, {"pickup_time": "yesterday"}, {"summary": {"distance": 5}}]).encode()
    rec, secs, us, tz, errs, is_batch = rt.pack_predict_batch(body, 0, 0)
    assert errs[0] == "invalid driver_age" and "isoformat" in errs[1] and errs[2] == ""
    _, _, _, _, errs, is_batch = rt.pack_predict_batch(b'{"summary": {"distance": 10}}', 0, 0)
    assert not is_batch and errs == [""]
    with pytest.raises(Exception):
        rt.pack_predict_batch(b"[1, 2", 0, 0)


def test_native_greedy_matches_python():
    rng = np.random.default_rng(3)
    for _ in range(300):
        n = int(rng.integers(2, 15))
        pts = rng.uniform(0, 10, (n + 1, 2))
        d = np.sqrt(((pts[:, None] - pts[None]) ** 2).sum(-1))
        dem = [0.0] + rng.integers(1, 5, n).astype(float).tolist()
        cap, maxd = float(rng.integers(3, 12)), float(rng.uniform(10, 40))
        trips, rest = rt.greedy_trips(d, dem, cap, maxd)
        try:
            ref = greedy_trips(d.tolist(), dem, cap, maxd)
            assert trips == ref
        except InfeasibleStops as e:
            assert trips is None and sorted(rest) == sorted(e.stops)


def test_native_astar_matches_dijkstra():
    from routest_amd.data.graph import synth_road_graph, synth_route_queries
    from routest_amd.routing.graph import dijkstra_ref
    g = synth_road_graph(5000, seed=2)
    cost = (g.length_m / (30 / 3.6)).astype(np.float32)
    s, t = synth_route_queries(g, 200, seed=3, min_km=0.5, max_km=20)
    got, paths = rt.astar_batch(g.indptr, g.indices, cost, g.lat.astype(np.float32), g.lon.astype(np.float32),
                                s, t, 1.0 / (130 / 3.6), 4)
    ref = dijkstra_ref(g, cost, s, t)
    np.testing.assert_allclose(got, ref, rtol=1e-4)
    assert all(p[0] == a and p[-1] == b for p, a, b in zip(paths, s, t))


def test_compact6_records_roundtrip():
    """6-byte bulk records (features.py RECORD6): features equal the 16-byte records' features for
    1/8-metre distances and whole-year ages; the PyTorch reference of K1 agrees bitwise; out of
    range values clamp and unknown categories give all-zero one-hots."""
    import torch
    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import (compact6_to_features, records_to_compact6,
                                             records_to_features)
    from routest_amd.ops.eta_mlp import featurize_torch, records6_to_tensor
    rec, _ = synth_records(5000, seed=3)
    rec["distance_m"] = np.rint(rec["distance_m"] * 8) / 8
    rec["driver_age"] = np.rint(rec["driver_age"])
    rec["weather"][:20] = 255
    rec["traffic"][10:30] = 4
    r6 = records_to_compact6(rec)
    assert r6.dtype == np.uint16 and r6.shape == (5000, 3)
    x6, x16 = compact6_to_features(r6), records_to_features(rec)
    np.testing.assert_array_equal(x6[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11]],
                                  x16[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11]])
    np.testing.assert_allclose(x6[:, 10], x16[:, 10], rtol=1e-6)
    assert torch.equal(featurize_torch(records6_to_tensor(r6)), torch.from_numpy(x6))
    big = rec[:2].copy()
    big["distance_m"] = [-5.0, 3e10]
    big["driver_age"] = [-1.0, 500.0]
    xb = compact6_to_features(records_to_compact6(big))
    assert xb[0, 10] == 0 and abs(xb[1, 10] - ((1 << 27) - 1) * 0.125e-3) < 1e-2
    assert xb[0, 11] == 0 and xb[1, 11] == 127


def test_wire8_records_exact():
    """8-byte wire records (features.py RECORD8, the format the native front end, the batcher and
    bench.py send): features bit-identical to the 16-byte records' (the kernel featurises the
    time itself from hours since the batch's base Monday), the PyTorch reference of K1 agrees
    bitwise, and a batch that does not fit exactly is refused (None -> 16-byte records)."""
    import torch
    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import (RECORD_DTYPE, compact_to_features, records_to_features,
                                             records_to_wire8)
    from routest_amd.ops.eta_mlp import featurize_torch, records8_to_tensor
    # the kernel's multiply-shift division is exact over the whole 10-bit range
    h = np.arange(1024, dtype=np.uint64)
    day = (h * 2731) >> 16
    assert np.array_equal(day, h // 24)
    assert np.array_equal(day - ((day * 9363) >> 16) * 7, (h // 24) % 7)
    rec, _ = synth_records(20000, seed=5)
    rec["weather"][:20] = 255
    rec["traffic"][10:30] = 4
    rec["driver_age"][:100] = 30.5          # fp16-exact non-integers are fine
    r8 = records_to_wire8(rec)
    assert r8 is not None and r8.itemsize == 8
    x8, x16 = compact_to_features(r8), records_to_features(rec)
    np.testing.assert_array_equal(x8, x16)
    assert torch.equal(featurize_torch(records8_to_tensor(r8)), torch.from_numpy(x8))
    # pre-2020 pickups (negative wall-clock seconds) and a span of 850 hours (any weekday) still fit
    r2 = rec[:3].copy()
    r2["wallclock_s"] = [-86400 * 400 + 5, -86400 * 400 + 850 * 3600, -86400 * 400 + 77]
    np.testing.assert_array_equal(compact_to_features(records_to_wire8(r2)), records_to_features(r2))
    # refused: an age fp16 cannot hold, or pickups 2000 hours apart
    bad = rec[:4].copy()
    bad["driver_age"][1] = 34.7
    assert records_to_wire8(bad) is None
    bad = rec[:4].copy()
    bad["wallclock_s"][2] += 2000 * 3600
    assert records_to_wire8(bad) is None
    assert records_to_wire8(np.zeros(0, dtype=RECORD_DTYPE)).shape == (0,)


def test_wire8_native_packer_matches_python():
    """The C++ packer the native front end runs (rt_core.h pack_wire8) == features.py's, byte for
    byte, including the refusal cases (fp16-inexact age, a span past 1024 hours)."""
    from routest_amd.data.synth import synth_records
    from routest_amd.models.features import records_to_wire8
    from routest_amd.ops import _ext
    rt = _ext.runtime(required=True)
    rec, _ = synth_records(30000, seed=9)
    rec["weather"][:7] = 200
    rec["driver_age"][50:60] = 0.000244140625       # an fp16 subnormal-range value, exact
    rec["driver_age"][60:70] = 1024.0
    rec["wallclock_s"] -= 2203 * 86400               # the whole batch before 2020 (negative)
    got = rt.pack_wire8(rec.view(np.uint8).reshape(-1, 16))
    ref = records_to_wire8(rec)
    assert got is not None and ref is not None
    assert np.array_equal(got.reshape(-1), ref.view(np.uint8).reshape(-1))
    for mod in ("age", "span"):
        bad = rec[:100].copy()
        if mod == "age":
            bad["driver_age"][3] = 1e-7
        else:
            bad["wallclock_s"][3] += 3000 * 3600
        assert rt.pack_wire8(bad.view(np.uint8).reshape(-1, 16)) is None
        assert records_to_wire8(bad) is None


def test_parallel_chunks_pool_concurrent_callers():
    """csrc/runtime/rt_core.h parallel_chunks runs on a process-wide worker pool: several Python
    threads packing and formatting large batches at once (GIL released, chunks taken from a shared
    counter by the pool and the callers) get exactly what one caller alone gets."""
    import threading
    rng = np.random.default_rng(5)
    n = 20000
    items = [{"summary": {"distance": float(rng.integers(100, 50000))}, "driver_age": int(rng.integers(18, 70)),
              "pickup_time": f"2025-0{1 + i % 9}-1{i % 10}T0{i % 10}:{10 + i % 50}:00",
              "weather": ["Sunny", "Cloudy", "Stormy", "Windy"][i % 4], "traffic": ["Low", "Jam"][i % 2]}
             for i in range(n)]
    body = json.dumps(items).encode()
    now_secs = 1760000000
    ref = rt.pack_predict_batch(body, now_secs, 0)
    minutes = rng.random(n).astype(np.float32) * 90
    ref_out = rt.format_predict_batch(minutes, ref[1], ref[2], ref[3], ref[4], True)
    results, errors = [], []

    def worker():
        try:
            for _ in range(3):
                got = rt.pack_predict_batch(body, now_secs, 0)
                out = rt.format_predict_batch(minutes, got[1], got[2], got[3], got[4], True)
                results.append(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
                               and list(got[4]) == list(ref[4]) and out == ref_out)
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))
    ths = [threading.Thread(target=worker) for _ in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    assert len(results) == 24 and all(results)
