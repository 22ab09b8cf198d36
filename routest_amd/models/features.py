"""ETA feature schema (R16) — CPU reference implementation and the packed record format
that the GPU featurize kernel (K1, ``csrc/eta_mlp.hip``) consumes.

Reference: ``RO/Flaskr/ml.py:35-51`` builds exactly 12 columns in this order::

    weather_{Cloudy,Stormy,Sunny,Windy}, traffic_{High,Jam,Low,Medium},
    weekday_ordered (Mon=0), hour_ordered, distance_km = distance_m/1000, driver_age (default 30)

Unknown categories produce all-zero one-hots (`==` comparisons).  Instead of building a pandas
DataFrame per request we pack each request into one 16-byte record (one ``dwordx4`` load per row
on the GPU)::

    struct EtaRecord { float distance_m; float driver_age; int32 wallclock_s; u8 weather; u8 traffic; u16 pad; }

``wallclock_s`` is the pickup wall-clock time in seconds since 2020-01-01 (tz ignored, exactly like
``datetime.weekday()``/``.hour``), from which the kernel derives weekday and hour.
"""
from __future__ import annotations

import datetime as dt
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple  # noqa: F401

import numpy as np

from ..utils.timeutil import KERNEL_EPOCH_WEEKDAY, coerce_pickup, wallclock_seconds

FEATURE_COLUMNS: List[str] = [
    "weather_Cloudy", "weather_Stormy", "weather_Sunny", "weather_Windy",
    "traffic_High", "traffic_Jam", "traffic_Low", "traffic_Medium",
    "weekday_ordered", "hour_ordered", "distance_km", "driver_age",
]
NUM_FEATURES = len(FEATURE_COLUMNS)
WEATHERS: Tuple[str, ...] = ("Cloudy", "Stormy", "Sunny", "Windy")
TRAFFICS: Tuple[str, ...] = ("High", "Jam", "Low", "Medium")
UNKNOWN_CODE = 255
_W = {w: i for i, w in enumerate(WEATHERS)}
_T = {t: i for i, t in enumerate(TRAFFICS)}

RECORD_DTYPE = np.dtype([("distance_m", "<f4"), ("driver_age", "<f4"), ("wallclock_s", "<i4"),
                         ("weather", "u1"), ("traffic", "u1"), ("pad", "<u2")])
assert RECORD_DTYPE.itemsize == 16

#: Compact 8-byte wire record (12 B per prediction with the f32 output instead of 20), used by the
#: native front end, the Python batcher and bench.py alike for every batch it represents EXACTLY:
#:   word0 = distance_m (f32, the same value as the 16-byte record's)
#:   word1 = fp16(driver_age) | hours << 16 | weather << 26 | traffic << 29
#: ``hours`` (10 bits) is the pickup's wall-clock hour counted from 00:00 of the Monday that starts
#: the batch's earliest pickup week (the per-batch base, kept by the host for the response).  The
#: kernel derives weekday = (hours / 24) % 7 and hour = hours % 24 itself — hour is the finest unit
#: any R16 feature reads, so the record is lossless for the model.  Category code 7 = unknown
#: (all-zero one-hot).  :func:`records_to_wire8` returns None when a batch cannot be represented
#: exactly (an age that fp16 does not hold, or pickups spanning more than 1024 hours from the
#: base); callers then send the 16-byte records.
RECORD8_DTYPE = np.dtype([("distance_m", "<f4"), ("packed", "<u4")])
assert RECORD8_DTYPE.itemsize == 8
WIRE8_HOURS = 1 << 10
#: 2020-01-01 (the records' wall-clock epoch) is a Wednesday: day d has weekday (d + 2) % 7
#: 6-byte bulk wire record (10 B per prediction with the f32 output): one little-endian 48-bit word
#: stored as 3 x u16 — bits 0-26 distance in eighths of a metre (to 16,777 km; exact in f32 below
#: 2,097 km), 27-33 driver age in whole years (0-127), 34-36 weekday, 37-41 hour, 42-44 weather,
#: 45-47 traffic (code 7 = unknown -> all-zero one-hot).  Distance is kept to 1/8 m (ORS reports
#: 0.1 m) and age to a year (the reference's column is an integer); both are finer than what the
#: kernel's bf16 hi/lo operand split resolves after normalisation.
RECORD6_WORDS = 3
DIST6_MAX_Q = (1 << 27) - 1


def weather_code(w: Any) -> int:
    return _W.get(w, UNKNOWN_CODE) if isinstance(w, str) else UNKNOWN_CODE


def traffic_code(t: Any) -> int:
    return _T.get(t, UNKNOWN_CODE) if isinstance(t, str) else UNKNOWN_CODE


def feature_dict(*, weather: Any, traffic: Any, distance_m: Any, pickup_time: Any,
                 driver_age: Any = 30.0) -> Tuple[Dict[str, Any], dt.datetime]:
    """Exact R16 feature dict (same Python types as the reference's DataFrame row)."""
    p = coerce_pickup(pickup_time)
    feats = {
        "weather_Cloudy": weather == "Cloudy",
        "weather_Stormy": weather == "Stormy",
        "weather_Sunny": weather == "Sunny",
        "weather_Windy": weather == "Windy",
        "traffic_High": traffic == "High",
        "traffic_Jam": traffic == "Jam",
        "traffic_Low": traffic == "Low",
        "traffic_Medium": traffic == "Medium",
        "weekday_ordered": p.weekday(),
        "hour_ordered": p.hour,
        "distance_km": float(distance_m or 0) / 1000.0,
        "driver_age": float(driver_age or 30.0),
    }
    return feats, p


def features_row(**kw: Any) -> np.ndarray:
    feats, _ = feature_dict(**kw)
    return np.array([float(feats[c]) for c in FEATURE_COLUMNS], dtype=np.float32)


def pack_record(*, weather: Any, traffic: Any, distance_m: Any, pickup: dt.datetime,
                driver_age: Any = 30.0) -> Tuple:
    return (float(distance_m or 0), float(driver_age or 30.0), wallclock_seconds(pickup),
            weather_code(weather), traffic_code(traffic), 0)


def pack_records(rows: Sequence[Dict[str, Any]]) -> np.ndarray:
    """Pack request dicts (weather, traffic, distance_m, pickup(datetime), driver_age)."""
    out = np.empty(len(rows), dtype=RECORD_DTYPE)
    for i, r in enumerate(rows):
        out[i] = pack_record(**r)
    return out


def wire8_base_hour(wallclock_s: np.ndarray) -> int:
    """Per-batch base: 00:00 of the Monday on or before the earliest pickup (hours since epoch)."""
    h0 = int(np.floor_divide(np.asarray(wallclock_s, dtype=np.int64).min(), 3600))
    d0 = h0 // 24
    monday = d0 - (d0 + KERNEL_EPOCH_WEEKDAY) % 7
    return monday * 24


def records_to_wire8(rec: np.ndarray) -> Optional[np.ndarray]:
    """16-byte records -> 8-byte wire records, or None if the batch does not fit exactly."""
    rec = np.asarray(rec, dtype=RECORD_DTYPE)
    out = np.empty(rec.shape[0], dtype=RECORD8_DTYPE)
    if rec.shape[0] == 0:
        return out
    age = rec["driver_age"]
    age16 = age.astype(np.float16)
    if not np.array_equal(age16.astype(np.float32).view(np.uint32), age.view(np.uint32)):
        return None
    hrs = np.floor_divide(rec["wallclock_s"].astype(np.int64), 3600) - wire8_base_hour(rec["wallclock_s"])
    if hrs.max() >= WIRE8_HOURS:
        return None
    w = rec["weather"].astype(np.uint32)
    t = rec["traffic"].astype(np.uint32)
    w = np.where(w > 3, 7, w)
    t = np.where(t > 3, 7, t)
    out["distance_m"] = rec["distance_m"]
    out["packed"] = (age16.view(np.uint16).astype(np.uint32) | (hrs.astype(np.uint32) << 16)
                     | (w << 26) | (t << 29))
    return out


def records_to_compact(rec: np.ndarray) -> np.ndarray:
    """:func:`records_to_wire8`, raising if the batch is not exactly representable."""
    out = records_to_wire8(rec)
    if out is None:
        raise ValueError("batch not representable as 8-byte wire records (age not fp16-exact or "
                         "pickups span >= 1024 hours)")
    return out


def records_to_compact6(rec: np.ndarray) -> np.ndarray:
    """16-byte records -> 6-byte bulk records, uint16 [B,3] (see RECORD6_WORDS)."""
    rec = np.asarray(rec, dtype=RECORD_DTYPE)
    q = np.clip(np.rint(rec["distance_m"].astype(np.float64) * 8.0), 0, DIST6_MAX_Q).astype(np.uint64)
    age = np.clip(np.rint(rec["driver_age"].astype(np.float64)), 0, 127).astype(np.uint64)
    secs = rec["wallclock_s"].astype(np.int64)
    days = np.floor_divide(secs, 86400)
    wd = ((days + KERNEL_EPOCH_WEEKDAY) % 7).astype(np.uint64)
    hr = ((secs - days * 86400) // 3600).astype(np.uint64)
    w = rec["weather"].astype(np.uint64)
    t = rec["traffic"].astype(np.uint64)
    w = np.where(w > 3, 7, w)
    t = np.where(t > 3, 7, t)
    word = q | (age << 27) | (wd << 34) | (hr << 37) | (w << 42) | (t << 45)
    out = np.empty((rec.shape[0], RECORD6_WORDS), dtype=np.uint16)
    for k in range(RECORD6_WORDS):
        out[:, k] = (word >> (16 * k)) & 0xFFFF
    return out


def compact6_to_features(rec6: np.ndarray) -> np.ndarray:
    """CPU reference of the K1 featurize kernel for 6-byte records."""
    r = np.asarray(rec6, dtype=np.uint16).astype(np.uint64)
    word = r[:, 0] | (r[:, 1] << 16) | (r[:, 2] << 32)
    x = np.zeros((r.shape[0], NUM_FEATURES), dtype=np.float32)
    w = (word >> 42) & 7
    t = (word >> 45) & 7
    for i in range(4):
        x[:, i] = (w == i)
        x[:, 4 + i] = (t == i)
    x[:, 8] = (word >> 34) & 7
    x[:, 9] = (word >> 37) & 31
    x[:, 10] = (word & DIST6_MAX_Q).astype(np.float32) * np.float32(np.float32(0.125) * np.float32(1e-3))
    x[:, 11] = (word >> 27) & 127
    return x


def compact_to_features(rec8: np.ndarray) -> np.ndarray:
    """CPU reference of the K1 featurize kernel for 8-byte wire records."""
    rec8 = np.asarray(rec8, dtype=RECORD8_DTYPE)
    pk = rec8["packed"].astype(np.uint32)
    x = np.zeros((rec8.shape[0], NUM_FEATURES), dtype=np.float32)
    w = (pk >> 26) & 7
    t = (pk >> 29) & 7
    for i in range(4):
        x[:, i] = (w == i)
        x[:, 4 + i] = (t == i)
    hrs = (pk >> 16) & (WIRE8_HOURS - 1)
    x[:, 8] = (hrs // 24) % 7
    x[:, 9] = hrs % 24
    x[:, 10] = rec8["distance_m"].astype(np.float32) / np.float32(1000.0)
    x[:, 11] = (pk & 0xFFFF).astype(np.uint16).view(np.float16).astype(np.float32)
    return x


def records_to_features(rec: np.ndarray) -> np.ndarray:
    """CPU reference of the K1 featurize kernel: records -> [B,12] float32 (R16 order)."""
    rec = np.asarray(rec, dtype=RECORD_DTYPE)
    b = rec.shape[0]
    x = np.zeros((b, NUM_FEATURES), dtype=np.float32)
    w = rec["weather"].astype(np.int64)
    t = rec["traffic"].astype(np.int64)
    for i in range(4):
        x[:, i] = (w == i)
        x[:, 4 + i] = (t == i)
    secs = rec["wallclock_s"].astype(np.int64)
    days = np.floor_divide(secs, 86400)
    sod = secs - days * 86400
    x[:, 8] = (days + KERNEL_EPOCH_WEEKDAY) % 7
    x[:, 9] = sod // 3600
    x[:, 10] = rec["distance_m"].astype(np.float32) / np.float32(1000.0)
    x[:, 11] = rec["driver_age"]
    return x


def dataframe_to_features(df: Any) -> np.ndarray:
    """Accept a reference-style pandas DataFrame (12 named columns) -> [B,12] float32."""
    cols = list(df.columns)
    if cols != FEATURE_COLUMNS:
        missing = [c for c in FEATURE_COLUMNS if c not in cols]
        if missing:
            raise ValueError(f"missing feature columns: {missing}")
        df = df[FEATURE_COLUMNS]
    return df.to_numpy(dtype=np.float32)


def features_to_records(x: np.ndarray, base_day: int = 0) -> np.ndarray:
    """Inverse map for synthetic data: [B,12] features -> records (weekday/hour re-encoded)."""
    x = np.asarray(x, dtype=np.float32)
    rec = np.zeros(x.shape[0], dtype=RECORD_DTYPE)
    w = np.where(x[:, 0:4].max(1) > 0.5, x[:, 0:4].argmax(1), UNKNOWN_CODE)
    t = np.where(x[:, 4:8].max(1) > 0.5, x[:, 4:8].argmax(1), UNKNOWN_CODE)
    wd = x[:, 8].astype(np.int64)
    hr = x[:, 9].astype(np.int64)
    # choose a day whose weekday matches: day d has weekday (d + EPOCH_WD) % 7
    day = base_day + ((wd - KERNEL_EPOCH_WEEKDAY - base_day) % 7)
    rec["wallclock_s"] = (day * 86400 + hr * 3600).astype(np.int32)
    rec["distance_m"] = x[:, 10] * 1000.0
    rec["driver_age"] = x[:, 11]
    rec["weather"] = w.astype(np.uint8)
    rec["traffic"] = t.astype(np.uint8)
    return rec
