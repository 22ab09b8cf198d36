"""Typed settings for the whole service, loaded once *before* any module reads them.

Reference parity: the reference reads env vars at module import time
(``RO/Flaskr/routes.py:11-17``, ``RO/Flaskr/utils.py:8,206-208``) and only afterwards runs
``load_dotenv()`` (``RO/app.py:1-4``), so `.env`-only values never reach those constants
(Appendix B #2).  Here every consumer calls :func:`get_settings`, which parses `.env` first,
then the process environment, then explicit overrides.  All of the reference's env-var names are
accepted unchanged; new knobs use the ``ROUTEST_`` prefix.
"""
from __future__ import annotations

import dataclasses
import os
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


def _parse_dotenv(path: str) -> Dict[str, str]:
    """Minimal `.env` reader (python-dotenv is not available offline)."""
    out: Dict[str, str] = {}
    try:
        with open(path, "r", encoding="utf-8") as f:
            for raw in f:
                line = raw.strip()
                if not line or line.startswith("#") or "=" not in line:
                    continue
                if line.startswith("export "):
                    line = line[len("export "):]
                k, v = line.split("=", 1)
                k, v = k.strip(), v.strip()
                if len(v) >= 2 and v[0] == v[-1] and v[0] in "'\"":
                    v = v[1:-1]
                out[k] = v
    except OSError:
        pass
    return out


def _as_bool(v: Optional[str], default: bool = False) -> bool:
    if v is None or v == "":
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


@dataclass
class Settings:
    # ---- reference env names (RO/Flaskr/*.py) ----
    ors_api_key: Optional[str] = None            # ORS_API_KEY / OPENROUTESERVICE_API_KEY
    redis_url: Optional[str] = None              # REDIS_URL
    supabase_url: Optional[str] = None           # SUPABASE_URL
    supabase_service_key: Optional[str] = None   # SUPABASE_SERVICE_ROLE_KEY
    eta_model_path: Optional[str] = None         # ETA_MODEL_PATH
    running_in_render: bool = False              # RENDER / RENDER_SERVICE_ID
    dev_api_base: str = "http://127.0.0.1:5000"  # DEV_API_BASE
    prod_api_base: str = ""                      # API_BASE_URL / RENDER_EXTERNAL_URL
    version: Optional[str] = None                # RENDER_GIT_COMMIT / GIT_COMMIT_SHA

    # ---- new knobs ----
    device: str = "auto"                 # ROUTEST_DEVICE: auto|cpu|cuda
    devices: List[int] = field(default_factory=list)  # ROUTEST_DEVICES: "0,1,..." (empty = all)
    batch_max: int = 4096                # ROUTEST_BATCH_MAX: micro-batch cap (rows)
    batch_timeout_us: int = 200          # ROUTEST_BATCH_TIMEOUT_US: flush deadline
    dtype: str = "bf16"                  # ROUTEST_DTYPE
    provider: str = "haversine"          # ROUTEST_PROVIDER: haversine|graph|ors
    store_url: str = "sqlite:///:memory:"  # ROUTEST_STORE: sqlite:///path | postgrest | none
    broker: str = "memory"               # ROUTEST_BROKER: memory|redis
    engine_name: str = "backend:mi355x"  # ROUTEST_ENGINE_NAME (R23: reference writes "backend:ors")
    compat_request_route_200: bool = True  # ROUTEST_COMPAT_REQUEST_ROUTE_200 (Appendix B #1)
    compat_history_500: bool = False     # ROUTEST_COMPAT_HISTORY_500 (Appendix B #6)
    sse_delta: bool = False              # ROUTEST_SSE_DELTA (Appendix B #7)
    fast_predict: bool = True            # ROUTEST_FAST_PREDICT: pure-ASGI native single-predict path
    graph_nodes: int = 100_000           # ROUTEST_GRAPH_NODES: synthetic road graph for the route scorer
    graph_path: str = ""                 # ROUTEST_GRAPH_PATH / serve --graph: a real road graph
                                         # (.gr + .co DIMACS, .edges.csv + .nodes.csv, .npz)
    route_batch: str = "auto"            # ROUTEST_ROUTE_BATCH: auto (on with a GPU) | 1 | 0
    route_batch_max: int = 1024          # ROUTEST_ROUTE_BATCH_MAX: requests per optimizer flush
    route_batch_timeout_us: int = 500    # ROUTEST_ROUTE_BATCH_TIMEOUT_US
    route_pipelines: int = 0             # ROUTEST_ROUTE_PIPELINES: native route services per GPU (each
                                         # its own GPU / assembly / persistence threads, so one flush's
                                         # host stages overlap another's GPU stages); 0 = auto:
                                         # serve/frontend.py route_pipelines_for
    route_gpu_min_stops: int = 32        # ROUTEST_ROUTE_GPU_MIN_STOPS: haversine requests with fewer
                                         # destinations stay inline (profiles/superseded/route_http_r2.jsonl)
    warm_scorer: bool = True             # ROUTEST_WARM_SCORER: build the GCN scorer at startup
    scorer_train_steps: int = 300        # ROUTEST_SCORER_TRAIN_STEPS: training steps of the GCN scorer
    # ROUTEST_SCORER_TARGET: "observed" (trip observations: hidden delays the edge costs lack,
    # models/gcn_observed.py) or "edge" (round 3: the learned edge times themselves)
    scorer_target: str = "observed"
    scorer_trips: int = 20000            # ROUTEST_SCORER_TRIPS: observed trips to train on
    sim_tick_min_s: float = 2.0          # ROUTEST_SIM_TICK_MIN (reference: U(2,5) s, utils.py:251)
    sim_tick_max_s: float = 5.0          # ROUTEST_SIM_TICK_MAX
    max_simulations: int = 256           # ROUTEST_MAX_SIMULATIONS (reference: unbounded threads)
    fault: str = ""                      # ROUTEST_FAULT: provider_timeout|gpu_fail|rccl_timeout
    default_model_dir: str = ""          # ROUTEST_MODEL_DIR: native checkpoint dir
    cors_origins: List[str] = field(default_factory=lambda: [
        "http://localhost:3000", "http://127.0.0.1:3000"])
    cors_origin_regex: str = r"https://.*\.vercel\.app"
    port: int = 5000                     # Appendix B #8: serve on 5000
    log_json: bool = False               # ROUTEST_LOG_JSON

    @property
    def api_base(self) -> str:
        """R25: loopback base URL (prod when running on Render, else DEV)."""
        if self.running_in_render and self.prod_api_base:
            return self.prod_api_base
        return self.dev_api_base

    @property
    def supabase_configured(self) -> bool:
        return bool(self.supabase_url and self.supabase_service_key)

    def replace(self, **kw: Any) -> "Settings":
        return dataclasses.replace(self, **kw)


def load_settings(env: Optional[Dict[str, str]] = None, dotenv_path: Optional[str] = ".env",
                  **overrides: Any) -> Settings:
    """Build Settings from `.env` < process env (or `env`) < overrides."""
    merged: Dict[str, str] = {}
    if dotenv_path:
        merged.update(_parse_dotenv(dotenv_path))
    merged.update(os.environ if env is None else env)
    g = merged.get

    def _int(name: str, default: int) -> int:
        try:
            return int(g(name) or default)
        except ValueError:
            return default

    def _float(name: str, default: float) -> float:
        try:
            return float(g(name) or default)
        except ValueError:
            return default

    devs = [int(x) for x in (g("ROUTEST_DEVICES") or "").split(",") if x.strip().isdigit()]
    s = Settings(
        ors_api_key=g("ORS_API_KEY") or g("OPENROUTESERVICE_API_KEY"),
        redis_url=g("REDIS_URL"),
        supabase_url=g("SUPABASE_URL"),
        supabase_service_key=g("SUPABASE_SERVICE_ROLE_KEY"),
        eta_model_path=g("ETA_MODEL_PATH"),
        running_in_render=bool(g("RENDER") or g("RENDER_SERVICE_ID")),
        dev_api_base=(g("DEV_API_BASE") or "http://127.0.0.1:5000").rstrip("/"),
        prod_api_base=(g("API_BASE_URL") or g("RENDER_EXTERNAL_URL") or "").rstrip("/"),
        version=g("RENDER_GIT_COMMIT") or g("GIT_COMMIT_SHA"),
        device=(g("ROUTEST_DEVICE") or "auto").lower(),
        devices=devs,
        batch_max=_int("ROUTEST_BATCH_MAX", 4096),
        batch_timeout_us=_int("ROUTEST_BATCH_TIMEOUT_US", 200),
        dtype=(g("ROUTEST_DTYPE") or "bf16").lower(),
        provider=(g("ROUTEST_PROVIDER") or ("ors" if g("ROUTEST_USE_ORS") else "haversine")).lower(),
        store_url=g("ROUTEST_STORE") or ("postgrest" if (g("SUPABASE_URL") and g("SUPABASE_SERVICE_ROLE_KEY"))
                                          else "sqlite:///:memory:"),
        broker=(g("ROUTEST_BROKER") or "memory").lower(),
        engine_name=g("ROUTEST_ENGINE_NAME") or "backend:mi355x",
        compat_request_route_200=_as_bool(g("ROUTEST_COMPAT_REQUEST_ROUTE_200"), True),
        compat_history_500=_as_bool(g("ROUTEST_COMPAT_HISTORY_500"), False),
        sse_delta=_as_bool(g("ROUTEST_SSE_DELTA"), False),
        fast_predict=_as_bool(g("ROUTEST_FAST_PREDICT"), True),
        graph_nodes=_int("ROUTEST_GRAPH_NODES", 100_000),
        graph_path=g("ROUTEST_GRAPH_PATH") or "",
        route_batch=(g("ROUTEST_ROUTE_BATCH") or "auto").lower(),
        route_batch_max=_int("ROUTEST_ROUTE_BATCH_MAX", 1024),
        route_batch_timeout_us=_int("ROUTEST_ROUTE_BATCH_TIMEOUT_US", 500),
        route_pipelines=max(0, _int("ROUTEST_ROUTE_PIPELINES", 0)),
        route_gpu_min_stops=_int("ROUTEST_ROUTE_GPU_MIN_STOPS", 32),
        warm_scorer=_as_bool(g("ROUTEST_WARM_SCORER"), True),
        scorer_train_steps=_int("ROUTEST_SCORER_TRAIN_STEPS", 300),
        scorer_target=(g("ROUTEST_SCORER_TARGET") or "observed").lower(),
        scorer_trips=_int("ROUTEST_SCORER_TRIPS", 20000),
        sim_tick_min_s=_float("ROUTEST_SIM_TICK_MIN", 2.0),
        sim_tick_max_s=_float("ROUTEST_SIM_TICK_MAX", 5.0),
        max_simulations=_int("ROUTEST_MAX_SIMULATIONS", 256),
        fault=(g("ROUTEST_FAULT") or "").lower(),
        default_model_dir=g("ROUTEST_MODEL_DIR") or "",
        port=_int("ROUTEST_PORT", 5000),
        log_json=_as_bool(g("ROUTEST_LOG_JSON"), False),
    )
    if overrides:
        s = s.replace(**overrides)
    return s


_lock = threading.Lock()
_settings: Optional[Settings] = None


def get_settings() -> Settings:
    global _settings
    with _lock:
        if _settings is None:
            _settings = load_settings()
        return _settings


def set_settings(s: Optional[Settings]) -> None:
    global _settings
    with _lock:
        _settings = s
