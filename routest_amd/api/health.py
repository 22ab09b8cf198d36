"""``GET /api/health`` payload (R10, ``RO/Flaskr/routes.py:282-363``): always HTTP 200, overall
``ok``/``degraded``; per-check ``status`` + ``latency_ms``.  Adds ``gpu`` (device count, HBM
free/total, native kernels loaded), ``model`` (ETA backend) and ``native`` (the native front end
that owns the main port: GPU-slot quarantine, served model and epoch) checks."""
from __future__ import annotations

import os
import time
from typing import Any, Dict


def _check_engine(provider: Any) -> Dict[str, Any]:
    t0 = time.time()
    name = getattr(provider, "name", "unknown")
    if name != "ors":
        return {"status": "ok", "latency_ms": 0, "engine": name}
    import requests
    try:
        head = requests.head("https://api.openrouteservice.org", timeout=2)
        code = head.status_code
        status = "ok" if 200 <= code < 400 else "degraded"
        if provider.key:
            try:
                r = requests.get("https://api.openrouteservice.org/health",
                                 headers={"Authorization": provider.key}, timeout=2)
                status = "ok" if 200 <= r.status_code < 300 else "degraded"
                code = r.status_code
            except Exception:
                pass
        return {"status": status, "latency_ms": int((time.time() - t0) * 1000), "engine": "ors", "code": code}
    except Exception as e:
        return {"status": "error", "latency_ms": int((time.time() - t0) * 1000), "engine": "ors",
                "error": str(e)[:200]}


def _check_gpu(sv: Any) -> Dict[str, Any]:
    t0 = time.time()
    try:
        import torch
        if not torch.cuda.is_available():
            return {"status": "skipped", "latency_ms": 0, "reason": "no GPU visible", "devices": 0}
        from ..ops import _ext
        C = _ext.native(required=False)
        devs = []
        for i in range(torch.cuda.device_count()):
            free, total = torch.cuda.mem_get_info(i)
            devs.append({"index": i, "name": torch.cuda.get_device_name(i), "hbm_free_gb": round(free / 2**30, 2),
                         "hbm_total_gb": round(total / 2**30, 2)})
        status = "ok" if C is not None else "error"
        out = {"status": status, "latency_ms": int((time.time() - t0) * 1000), "devices": len(devs),
               "detail": devs, "native_kernels": C is not None}
        if C is None:
            out["error"] = "routest_amd._C not loaded"
        return out
    except Exception as e:
        return {"status": "error", "latency_ms": int((time.time() - t0) * 1000), "error": str(e)[:200]}


def _check_collectives(sv: Any) -> Dict[str, Any]:
    """RCCL / collective readiness (SURVEY R10 "RCCL ready"): the RCCL library our native comm
    links (torch's bundled librccl), the torch.distributed state of this process, and any native
    DeviceComm the services hold (one-shot buffers mapped, no pending peer-wait error)."""
    t0 = time.time()
    try:
        import torch
        import torch.distributed as dist
        out: Dict[str, Any] = {"rccl_available": bool(dist.is_available() and dist.is_nccl_available())}
        from ..ops import _ext
        C = _ext.native(required=False)
        if C is not None and torch.cuda.is_available():
            out["rccl_version"] = int(C.rccl_version())
        init = dist.is_available() and dist.is_initialized()
        out["dist_initialized"] = bool(init)
        if init:
            out["backend"] = dist.get_backend()
            out["world_size"] = dist.get_world_size()
            out["rank"] = dist.get_rank()
        comm = getattr(sv, "comm", None)
        status = "ok" if out["rccl_available"] else "skipped"
        if comm is not None:
            out["device_comm"] = comm.ready()
            if out["device_comm"].get("error"):
                status = "degraded"
        out["status"] = status
        out["latency_ms"] = int((time.time() - t0) * 1000)
        return out
    except Exception as e:
        return {"status": "error", "latency_ms": int((time.time() - t0) * 1000), "error": str(e)[:200]}


def _check_native(sv: Any) -> Dict[str, Any]:
    """The process that serves the main port (serve/frontend.py ServingStack): per-GPU-slot health
    of the native front end (quarantine, failures, the model each slot serves, the model epoch after
    hot swaps), its request counters and the native route services' (CCH contexts built)."""
    front = getattr(sv, "native", None)
    if front is None:
        return {"status": "skipped", "latency_ms": 0, "reason": "no native front end in this process"}
    t0 = time.time()
    try:
        h = front.health()
        h["status"] = "degraded" if h.get("degraded") else "ok"
        h["latency_ms"] = int((time.time() - t0) * 1000)
        h["routes_native"] = bool(getattr(front, "routes", None))
        return h
    except Exception as e:
        return {"status": "error", "latency_ms": int((time.time() - t0) * 1000), "error": str(e)[:200]}


def health_payload(sv: Any) -> Dict[str, Any]:
    s = sv.settings
    redis_res = sv.broker.ping()
    engine_res = _check_engine(sv.provider)
    if sv.store is None:
        db_res = {"status": "skipped", "latency_ms": 0, "reason": "SUPABASE not configured"}
    else:
        db_res = sv.store.ping()
    gpu_res = _check_gpu(sv)
    coll_res = _check_collectives(sv)
    native_res = _check_native(sv)
    model = sv.eta.describe()
    model_res = {"status": ("degraded" if model.get("degraded") else "ok") if sv.eta.batcher is not None
                 else "skipped", **model}
    parts = (redis_res["status"], engine_res["status"], db_res["status"], gpu_res["status"], model_res["status"],
             coll_res["status"], native_res["status"])
    overall = "degraded" if any(p in ("error", "degraded") for p in parts) else "ok"
    return {
        "backend": True,
        "checks": {"engine": engine_res, "redis": redis_res, "supabase": db_res, "gpu": gpu_res,
                   "model": model_res, "collectives": coll_res, "native": native_res},
        "db": db_res["status"] == "ok",
        "osrm": engine_res["status"] in ("ok", "degraded"),
        "redis": redis_res["status"] == "ok",
        "tiles": True,
        "status": overall,
        "version": s.version or os.getenv("RENDER_GIT_COMMIT") or os.getenv("GIT_COMMIT_SHA"),
        "uptime_s": round(time.time() - sv.started, 1),
    }
