"""Synthetic data generators (the reference ships no data: ``data/.gitkeep``, ``notebooks/.gitkeep``).

* :func:`synth_trips` — seeded trip table in the exact R16 12-feature schema plus an
  ``eta_minutes`` target generated from a plausible travel-time model (speed depends on
  traffic/weather/hour; small driver-age effect; noise).  Used for config 1 (1k-row CSV,
  linear regression) and to train the MLP (configs 2-3).
* :func:`synth_records` — the same, directly as packed 16-byte records for the GPU benches.
* :func:`seed_locations` — the 21 Metro-Manila rows of the reference's seeder
  (``LV/database/seeders/LocationsTableSeeder.php:13-44``).
"""
from __future__ import annotations

import csv
import uuid
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..models.features import FEATURE_COLUMNS, RECORD_DTYPE, features_to_records

# (name, lat, lon) — LocationsTableSeeder.php:13-34
SEED_LOCATIONS: List[Tuple[str, float, float]] = [
    ("Main Warehouse - Mandaluyong", 14.5836, 121.0409),
    ("SM Mall of Asia", 14.5352, 120.9822),
    ("Greenbelt Mall", 14.5516, 121.0233),
    ("SM Megamall", 14.5833, 121.0567),
    ("Market! Market!", 14.5536, 121.0546),
    ("Robinsons Galleria", 14.5896, 121.0614),
    ("SM North EDSA", 14.6556, 121.0313),
    ("Trinoma Mall", 14.6537, 121.0321),
    ("Gateway Mall", 14.6206, 121.0526),
    ("SM City Manila", 14.5881, 120.9814),
    ("Lucky Chinatown Mall", 14.6054, 120.9734),
    ("SM Aura Premier", 14.5456, 121.0559),
    ("Robinsons Place Manila", 14.5730, 120.9820),
    ("Ayala Malls Vertis North", 14.6543, 121.0327),
    ("Fisher Mall", 14.6300, 121.0045),
    ("SM City Sta. Mesa", 14.6031, 121.0275),
    ("Alabang Town Center", 14.4269, 121.0314),
    ("Festival Mall Alabang", 14.4143, 121.0438),
    ("Eastwood Mall", 14.6101, 121.0791),
    ("Robinsons Magnolia", 14.6162, 121.0336),
    ("Venice Grand Canal Mall", 14.5404, 121.0530),
]


def seed_locations() -> List[Dict[str, object]]:
    """Deterministic UUIDs (uuid5 of the name) so history rows can reference them stably."""
    ns = uuid.UUID("5b0a9e52-7a3c-4c2e-9a53-1f2d3c4b5a69")
    return [{"id": str(uuid.uuid5(ns, n)), "name": n, "latitude": la, "longitude": lo}
            for n, la, lo in SEED_LOCATIONS]


_BASE_SPEED_KMH = {"High": 22.0, "Jam": 12.0, "Low": 38.0, "Medium": 28.0}
_WEATHER_FACTOR = {"Cloudy": 0.95, "Stormy": 0.7, "Sunny": 1.0, "Windy": 0.9}


def eta_ground_truth(x: np.ndarray, rng: Optional[np.random.Generator] = None,
                     noise: float = 0.05) -> np.ndarray:
    """Synthetic target (minutes) as a function of the 12 R16 features."""
    x = np.asarray(x, dtype=np.float64)
    speeds = np.array([_BASE_SPEED_KMH[t] for t in ("High", "Jam", "Low", "Medium")])
    wf = np.array([_WEATHER_FACTOR[w] for w in ("Cloudy", "Stormy", "Sunny", "Windy")])
    t_oh, w_oh = x[:, 4:8], x[:, 0:4]
    speed = np.where(t_oh.sum(1) > 0, t_oh @ speeds, 30.0)
    speed = speed * np.where(w_oh.sum(1) > 0, w_oh @ wf, 1.0)
    hour = x[:, 9]
    rush = 1.0 - 0.25 * (np.exp(-((hour - 8.0) ** 2) / 4.0) + np.exp(-((hour - 18.0) ** 2) / 4.0))
    weekend = np.where(x[:, 8] >= 5, 1.1, 1.0)
    speed = speed * rush * weekend
    age = x[:, 11]
    age_f = 1.0 + 0.004 * np.abs(age - 35.0)
    minutes = 4.0 + 60.0 * x[:, 10] / speed * age_f
    if rng is not None and noise > 0:
        minutes = minutes * (1.0 + noise * rng.standard_normal(minutes.shape))
    return minutes.astype(np.float32)


def synth_features(n: int, seed: int = 0, unknown_frac: float = 0.02) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = np.zeros((n, 12), dtype=np.float32)
    w = rng.integers(0, 4, n)
    t = rng.integers(0, 4, n)
    wu = rng.random(n) < unknown_frac
    tu = rng.random(n) < unknown_frac
    x[np.arange(n)[~wu], w[~wu]] = 1.0
    x[np.arange(n)[~tu], 4 + t[~tu]] = 1.0
    x[:, 8] = rng.integers(0, 7, n)
    x[:, 9] = rng.integers(0, 24, n)
    x[:, 10] = np.round(rng.gamma(2.0, 6.0, n), 3)   # km, mean 12
    x[:, 11] = rng.integers(18, 70, n).astype(np.float32)
    return x


def synth_trips(n: int, seed: int = 0, noise: float = 0.05) -> Tuple[np.ndarray, np.ndarray]:
    """Returns (X [n,12] float32 in R16 order, y minutes [n] float32)."""
    x = synth_features(n, seed)
    y = eta_ground_truth(x, np.random.default_rng(seed + 1), noise)
    return x, y


def synth_records(n: int, seed: int = 0, noise: float = 0.05) -> Tuple[np.ndarray, np.ndarray]:
    """Packed 16-byte records; pickups carry a random minute/second inside their hour, like real
    ISO timestamps (only weekday and hour reach the model)."""
    x, y = synth_trips(n, seed, noise)
    rec = features_to_records(x, base_day=2200)
    rec["wallclock_s"] += np.random.default_rng(seed + 7).integers(0, 3600, n).astype(np.int32)
    return rec, y


def write_trips_csv(path: str, n: int = 1000, seed: int = 0) -> None:
    """Config 1 input: a 1k-row CSV with the 12 feature columns + ``eta_minutes``."""
    x, y = synth_trips(n, seed)
    with open(path, "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(FEATURE_COLUMNS + ["eta_minutes"])
        for i in range(n):
            row = [bool(v) if j < 8 else (int(v) if j in (8, 9) else float(v))
                   for j, v in enumerate(x[i])]
            wr.writerow(row + [float(y[i])])


def read_trips_csv(path: str) -> Tuple[np.ndarray, np.ndarray]:
    with open(path, newline="") as f:
        rd = csv.reader(f)
        header = next(rd)
        idx = [header.index(c) for c in FEATURE_COLUMNS]
        yi = header.index("eta_minutes")
        xs, ys = [], []
        for row in rd:
            xs.append([1.0 if row[i] == "True" else 0.0 if row[i] == "False" else float(row[i])
                       for i in idx])
            ys.append(float(row[yi]))
    return np.asarray(xs, dtype=np.float32), np.asarray(ys, dtype=np.float32)
