"""Distance / directions providers.

The reference calls the remote OpenRouteService API for the distance matrix
(``RO/Flaskr/utils.py:93-109``) and for per-trip directions (``utils.py:53-66,147-160``).  This
service is self-contained by default:

* :class:`HaversineProvider` — great-circle distance x a circuity factor, profile-dependent speed,
  straight-line polylines densified every ~``step_m`` metres, ORS-shaped ``segments``/``steps``
  (``RO/sample_get_route_response.json``).  Batched matrices for many requests run on the GPU
  (K5, ``csrc/route_kernels.hip``).
* :class:`GraphProvider` (``routing/graph.py``) — shortest paths on a synthetic road graph with
  learned edge costs (K9).
* :class:`ORSProvider` — the reference's remote calls, kept for wire compatibility when an ORS key
  is configured and ``ROUTEST_PROVIDER=ors``.

All providers raise :class:`ProviderError` with the reference's error strings.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Sequence

import numpy as np

from ..utils.faults import maybe_fail

EARTH_R = 6_371_000.0

#: ORS profile per vehicle type (R19, utils.py:22-29)
VEHICLE_PROFILES = {
    "car": "driving-car",
    "truck": "driving-hgv", "hgv": "driving-hgv",
    "motorcycle": "driving-car",
    "bike": "cycling-regular",
    "roadbike": "cycling-road",
    "foot": "foot-walking",
}
#: mean speeds (m/s) used for durations by the offline providers
PROFILE_SPEED_MPS = {
    "driving-car": 30 / 3.6,
    "driving-hgv": 24 / 3.6,
    "cycling-regular": 15 / 3.6,
    "cycling-road": 22 / 3.6,
    "foot-walking": 5 / 3.6,
}


class ProviderError(RuntimeError):
    pass


def profile_for(vehicle_type: Any) -> str:
    vt = (vehicle_type or "car")
    vt = vt.lower().strip() if isinstance(vt, str) else "car"
    return VEHICLE_PROFILES.get(vt, "driving-car")


def haversine_m(lat1, lon1, lat2, lon2):
    p1, p2 = np.radians(lat1), np.radians(lat2)
    dphi = p2 - p1
    dl = np.radians(lon2) - np.radians(lon1)
    a = np.sin(dphi / 2) ** 2 + np.cos(p1) * np.cos(p2) * np.sin(dl / 2) ** 2
    return 2 * EARTH_R * np.arcsin(np.sqrt(np.clip(a, 0.0, 1.0)))


def _native_rt():
    try:
        from ..ops._ext import runtime
        return runtime(required=False)
    except Exception:  # pragma: no cover
        return None


_RT = _native_rt()


def haversine_scalar(lat1: float, lon1: float, lat2: float, lon2: float) -> float:
    """One great-circle distance.  With the C++ runtime present this is the native route
    assembler's own function (csrc/runtime/route_core.h), so the Python path and the native front
    end produce identical bits; numpy's vectorised sin/cos may differ from libm in the last ulp."""
    if _RT is not None:
        return _RT.haversine_m(float(lat1), float(lon1), float(lat2), float(lon2))
    return float(haversine_m(lat1, lon1, lat2, lon2))


def haversine_matrix(lats: Sequence[float], lons: Sequence[float], circuity: float = 1.0) -> np.ndarray:
    la = np.asarray(lats, dtype=np.float64)
    lo = np.asarray(lons, dtype=np.float64)
    if _RT is not None and la.shape[0] <= 4096:
        return _RT.haversine_matrix(la, lo, float(circuity))
    return haversine_m(la[:, None], lo[:, None], la[None, :], lo[None, :]) * circuity


def _bearing_word(lat1, lon1, lat2, lon2) -> str:
    y = math.sin(math.radians(lon2 - lon1)) * math.cos(math.radians(lat2))
    x = (math.cos(math.radians(lat1)) * math.sin(math.radians(lat2))
         - math.sin(math.radians(lat1)) * math.cos(math.radians(lat2)) * math.cos(math.radians(lon2 - lon1)))
    b = (math.degrees(math.atan2(y, x)) + 360.0) % 360.0
    return ["north", "northeast", "east", "southeast", "south", "southwest", "west",
            "northwest"][int((b + 22.5) // 45) % 8]


class HaversineProvider:
    name = "haversine"
    blocking = False       # pure CPU, sub-millisecond: handlers call it inline (no thread hop)

    def __init__(self, circuity: float = 1.3, step_m: float = 150.0):
        self.circuity = circuity
        self.step_m = step_m

    def matrix(self, points: List[Dict[str, float]], profile: str) -> np.ndarray:
        maybe_fail("provider_timeout")
        return haversine_matrix([p["lat"] for p in points], [p["lon"] for p in points],
                                self.circuity)

    def directions(self, coords: List[List[float]], profile: str) -> Dict[str, Any]:
        """coords: [[lon, lat], ...] -> ORS-shaped GeoJSON Feature."""
        maybe_fail("provider_timeout")
        speed = PROFILE_SPEED_MPS.get(profile, PROFILE_SPEED_MPS["driving-car"])
        geometry: List[List[float]] = [[float(coords[0][0]), float(coords[0][1])]]
        segments = []
        way_points = [0]
        tot_d = 0.0
        for k in range(len(coords) - 1):
            lon1, lat1 = float(coords[k][0]), float(coords[k][1])
            lon2, lat2 = float(coords[k + 1][0]), float(coords[k + 1][1])
            dist = haversine_scalar(lat1, lon1, lat2, lon2) * self.circuity
            n = max(1, int(math.ceil(dist / self.step_m)))
            start_wp = len(geometry) - 1
            t = np.arange(1, n + 1, dtype=np.float64) / n          # densify in one vector op
            pts = np.round(np.stack([lon1 + (lon2 - lon1) * t, lat1 + (lat2 - lat1) * t], axis=1), 6)
            geometry.extend(pts.tolist())
            end_wp = len(geometry) - 1
            way_points.append(end_wp)
            dur = dist / speed
            d_r, t_r = round(dist, 1), round(dur, 1)
            segments.append({
                "distance": d_r, "duration": t_r,
                "steps": [
                    {"distance": d_r, "duration": t_r, "type": 11 if k == 0 else 1,
                     "instruction": f"Head {_bearing_word(lat1, lon1, lat2, lon2)}",
                     "name": "-", "way_points": [start_wp, end_wp]},
                    {"distance": 0.0, "duration": 0.0, "type": 10,
                     "instruction": "Arrive at your destination" if k == len(coords) - 2
                     else f"Arrive at waypoint {k + 1}",
                     "name": "-", "way_points": [end_wp, end_wp]},
                ],
            })
            tot_d += dist
        tot_t = tot_d / speed
        return {
            "type": "Feature",
            "bbox": _bbox(geometry),
            "geometry": {"type": "LineString", "coordinates": geometry},
            "properties": {"segments": segments,
                           "summary": {"distance": round(tot_d, 1), "duration": round(tot_t, 1)},
                           "way_points": way_points},
        }


def _bbox(coords: List[List[float]]) -> List[float]:
    lons = [c[0] for c in coords]
    lats = [c[1] for c in coords]
    return [min(lons), min(lats), max(lons), max(lats)]


class ORSProvider:
    """The reference's remote calls (utils.py:55-62, 97-103, 151-156), same timeouts/errors."""

    name = "ors"
    blocking = True        # remote HTTPS: handlers offload it to the thread pool
    BASE = "https://api.openrouteservice.org"

    def __init__(self, api_key: str, timeout: float = 30.0, session: Any = None):
        import requests
        self.key = api_key
        self.timeout = timeout
        self.http = session or requests.Session()

    def _headers(self) -> Dict[str, str]:
        return {"Authorization": self.key, "Content-Type": "application/json"}

    def matrix(self, points: List[Dict[str, float]], profile: str) -> np.ndarray:
        import requests
        maybe_fail("provider_timeout")
        body = {"locations": [[p["lon"], p["lat"]] for p in points], "metrics": ["distance"],
                "units": "m"}
        try:
            r = self.http.post(f"{self.BASE}/v2/matrix/{profile}", json=body, headers=self._headers(),
                               timeout=self.timeout)
            r.raise_for_status()
            dm = r.json().get("distances")
        except requests.RequestException as e:
            status = getattr(e.response, "status_code", "n/a")
            text = getattr(e.response, "text", str(e))
            raise ProviderError(f"ORS matrix error (status {status}): {text}")
        if not dm:
            raise ProviderError("ORS matrix returned no distances")
        return np.asarray(dm, dtype=np.float64)

    def directions(self, coords: List[List[float]], profile: str) -> Dict[str, Any]:
        import requests
        maybe_fail("provider_timeout")
        try:
            r = self.http.post(f"{self.BASE}/v2/directions/{profile}/geojson",
                               json={"coordinates": coords}, headers=self._headers(),
                               timeout=self.timeout)
            r.raise_for_status()
            return r.json()["features"][0]
        except requests.RequestException as e:
            status = getattr(e.response, "status_code", "n/a")
            text = getattr(e.response, "text", str(e))
            raise ProviderError(f"ORS directions error (status {status}): {text}")
