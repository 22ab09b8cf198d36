"""Route optimizer: dispatcher + point-to-point + multi-stop + trip assembly (R19-R23).

Reference: ``optimize_route`` (``RO/Flaskr/utils.py:10-48``), ``_point_to_point`` (``:53-82``),
``_multi_stop`` (``:85-193``), ``_annotate_common_props`` (``:196-201``).  Behaviour kept:

* ``{"error": "no destination points specified."}`` on empty input;
* vehicle_type -> profile mapping (lower-cased, stripped; default ``driving-car``);
* one destination: route first, *then* the payload/max-distance feasibility check with the
  reference's ``" | "``-joined messages; ``optimized_order=[0]``, ``source``, ``destinations``;
* many destinations: distance matrix over ``[source]+destinations``, greedy multi-trip
  construction (:mod:`routing.greedy`), per-trip directions concatenated, bbox, summary with
  ``trips``; ``optimized_order`` as 0-based destination indices;
* metadata ``vehicle_type``, ``driver_name``, ``engine``.

Fixed: infeasible stops return an error instead of hanging (Appendix B #3).
The batched GPU path for many concurrent requests (K5 + K6) is :func:`optimize_many`.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from .greedy import InfeasibleStops, greedy_trips, optimized_order
from .providers import ProviderError, _bbox, profile_for


def _annotate(feature: Dict[str, Any], driver: Dict[str, Any], vehicle_type: str, engine: str) -> None:
    p = feature.setdefault("properties", {})
    p["vehicle_type"] = vehicle_type
    p["driver_name"] = driver.get("driver_name")
    p["engine"] = engine


def _vehicle_type(driver: Dict[str, Any]) -> str:
    vt = driver.get("vehicle_type") or "car"
    return vt.lower().strip() if isinstance(vt, str) else "car"


def _float(v: Any, default: float) -> float:
    try:
        return float(v)
    except (TypeError, ValueError):
        return default


def _ctx_kw(ctx) -> Dict[str, Any]:
    """Routing context for context-aware providers (routing/cch.py); others take no such argument."""
    return {"ctx": ctx} if ctx is not None else {}


def point_to_point(provider, source, dest, profile: str, driver: Dict[str, Any], ctx=None) -> Dict[str, Any]:
    coords = [[source["lon"], source["lat"]], [dest["lon"], dest["lat"]]]
    try:
        feature = provider.directions(coords, profile, **_ctx_kw(ctx))
    except ProviderError as e:
        return {"error": str(e)}
    payload = dest.get("payload", 0)
    cap = driver.get("vehicle_capacity", 999999)
    max_dist = _float(driver.get("maximum_distance", 9e12), 9e12)
    dist_m = float(feature["properties"]["summary"]["distance"])
    errors = []
    try:
        if payload > cap:
            errors.append("payload exceeds vehicle capacity")
    except TypeError:
        pass
    if dist_m > max_dist:
        errors.append("route distance exceeds maximum_distance")
    if errors:
        return {"error": " | ".join(errors)}
    return feature


def assemble_trips(provider, all_points: List[Dict[str, Any]], trips: List[List[int]],
                   profile: str, source, destinations, ctx=None) -> Dict[str, Any]:
    geometry: List[List[float]] = []
    segments: List[Any] = []
    tot_d = 0.0
    tot_t = 0.0
    for trip in trips:
        coords = [[all_points[i]["lon"], all_points[i]["lat"]] for i in trip]
        try:
            f = provider.directions(coords, profile, **_ctx_kw(ctx))
        except ProviderError as e:
            return {"error": str(e)}
        geometry += f["geometry"]["coordinates"]
        segments += f["properties"].get("segments", [])
        tot_d += float(f["properties"]["summary"]["distance"])
        tot_t += float(f["properties"]["summary"]["duration"])
    return {
        "bbox": _bbox(geometry),
        "type": "Feature",
        "geometry": {"type": "LineString", "coordinates": geometry},
        "properties": {
            "source": source,
            "destinations": destinations,
            "optimized_order": optimized_order(trips),
            "segments": segments,
            "summary": {"distance": tot_d, "duration": tot_t, "trips": len(trips)},
        },
    }


def multi_stop(provider, source, destinations, profile: str, driver: Dict[str, Any],
               trips: Optional[List[List[int]]] = None, ctx=None) -> Dict[str, Any]:
    all_points = [source] + list(destinations)
    if trips is None:
        try:
            d = provider.matrix(all_points, profile, **_ctx_kw(ctx))
        except ProviderError as e:
            return {"error": str(e)}
        cap = _float(driver.get("vehicle_capacity", 9e12), 9e12)
        max_dist = _float(driver.get("maximum_distance", 9e12), 9e12)
        demand = [0.0] + [_float(p.get("payload", 0), 0.0) for p in destinations]
        try:
            trips = greedy_trips(np.asarray(d, dtype=np.float64).tolist(), demand, cap, max_dist)
        except InfeasibleStops as e:
            return {"error": str(e)}
    return assemble_trips(provider, all_points, trips, profile, source, destinations, ctx)


def optimize_route(input_data: Any, provider, engine: str = "backend:mi355x",
                   trips: Optional[List[List[int]]] = None, ctx=None) -> Dict[str, Any]:
    """Pure function: GeoJSON Feature on success, ``{"error": ...}`` on failure (R19).  ``ctx``:
    the request's routing context as resolved when its legs were planned (the batcher), so a
    request without ``pickup_time`` is assembled under the same week-hour it was routed in."""
    if not input_data or not isinstance(input_data, dict) or not input_data.get("destination_points"):
        return {"error": "no destination points specified."}
    driver = input_data.get("driver_details") or {}
    vehicle_type = _vehicle_type(driver)
    profile = profile_for(vehicle_type)
    source = input_data.get("source_point")
    if not isinstance(source, dict) or "lat" not in source or "lon" not in source:
        return {"error": "source_point with lat/lon is required."}
    destinations = input_data["destination_points"]
    # road providers route under the request's context (weather, traffic, pickup week-hour)
    if not getattr(provider, "uses_context", False):
        ctx = None
    elif ctx is None:
        from .cch import RouteContext
        ctx = RouteContext.from_request(input_data)
    if len(destinations) == 1:
        feature = point_to_point(provider, source, destinations[0], profile, driver, ctx)
        if "error" in feature:
            return feature
        p = feature.setdefault("properties", {})
        p["optimized_order"] = [0]
        p["source"] = source
        p["destinations"] = [destinations[0]]
        _annotate(feature, driver, vehicle_type, engine)
        return feature
    feature = multi_stop(provider, source, destinations, profile, driver, trips, ctx)
    if "error" in feature:
        return feature
    _annotate(feature, driver, vehicle_type, engine)
    return feature


def optimize_many(requests: Sequence[Dict[str, Any]], provider, engine: str = "backend:mi355x",
                  device=None) -> List[Dict[str, Any]]:
    """Batched optimizer for many concurrent requests: the distance matrices and greedy trips of
    every multi-stop request are computed in ONE pair of GPU launches (K5 + K6) when a GPU device
    is given (haversine provider only); assembly stays on the host."""
    from .batched import batched_trips
    multi = [i for i, r in enumerate(requests)
             if isinstance(r, dict) and isinstance(r.get("destination_points"), list)
             and len(r["destination_points"]) > 1 and isinstance(r.get("source_point"), dict)]
    trip_map: Dict[int, Any] = {}
    if multi and getattr(provider, "name", "") == "haversine":
        res = batched_trips([requests[i] for i in multi], circuity=provider.circuity, device=device)
        trip_map = dict(zip(multi, res))
    out = []
    for i, r in enumerate(requests):
        t = trip_map.get(i)
        if isinstance(t, InfeasibleStops):
            out.append({"error": str(t)})
            continue
        out.append(optimize_route(r, provider, engine, trips=t))
    return out
