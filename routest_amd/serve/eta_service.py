"""ETA prediction service (R15-R17 + the north-star batched GPU path).

Reference: ``predict_eta_minutes`` (``RO/Flaskr/ml.py:23-58``) lazily unpickles one model on the
first call, caches a load error *forever* as the string ``"ERROR:<e>"`` (never retried), builds a
one-row DataFrame per request and returns ``(minutes, iso)`` or ``(None, None)``.

Here the model is loaded once at startup under a lock; a failed load is retried (at most every
``retry_s`` seconds, and on ``/api/admin/reload_model``) instead of being cached forever
(Appendix B #4).  Requests are packed into 16-byte records and scored by the micro-batcher:
on GPUs every batch is one fused featurize+MLP HIP launch per device; on CPU the fp32 PyTorch
model (or the linear / tree-ensemble model) runs the same batches.
"""
from __future__ import annotations

import datetime as dt
import os
import threading
import time
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.features import RECORD_DTYPE, pack_record, records_to_features
from ..models.mlp3 import EtaMLP, LinearETA
from ..utils.logging import get_logger
from ..utils.timeutil import coerce_pickup
from .batcher import GpuRunner, MicroBatcher

log = get_logger("eta")


def _cpu_runner(model: Any):
    if isinstance(model, EtaMLP):
        import copy
        m = copy.deepcopy(model).float().cpu().eval()

        def run(rec: np.ndarray) -> np.ndarray:
            with torch.no_grad():
                return m(torch.from_numpy(records_to_features(rec))).numpy()
        return run
    if isinstance(model, LinearETA):
        return lambda rec: model.predict_features(records_to_features(rec))
    if hasattr(model, "predict_features"):
        return lambda rec: np.asarray(model.predict_features(records_to_features(rec)), dtype=np.float32)

    def run_df(rec: np.ndarray) -> np.ndarray:  # reference-style .predict(DataFrame) models
        import pandas as pd
        from ..models.features import FEATURE_COLUMNS
        x = records_to_features(rec)
        df = pd.DataFrame({c: (x[:, j] > 0.5) if j < 8 else x[:, j] for j, c in enumerate(FEATURE_COLUMNS)})
        return np.asarray(model.predict(df), dtype=np.float32)
    return run_df


class ForestKernel:
    """Tree ensemble resident on one GPU (K4: fused featurize + traversal, csrc/forest.hip)."""

    def __init__(self, model, device, lds: bool = True):
        from ..ops import _ext
        self.C = _ext.native(required=True)
        self.m = model
        self.values, self.info, self.roots = model.device_arrays(device)
        tab = model.chunk_table() if lds else None
        self.chunks = torch.from_numpy(tab).to(device) if tab is not None else None
        self.nodes2 = torch.from_numpy(model.nodes2()).to(device) if tab is not None else None

    def __call__(self, rec: torch.Tensor) -> torch.Tensor:
        if self.chunks is not None:   # whole trees fit the LDS chunk: staged kernel
            return self.C.forest_predict_lds(rec, self.nodes2, self.roots, self.chunks, self.m.base_score,
                                             self.m.le, list(self.m.feature_map))
        return self.C.forest_predict(rec, self.values, self.info, self.roots, self.m.base_score, self.m.le,
                                     list(self.m.feature_map))


class EtaService:
    def __init__(self, model: Any = None, model_path: Optional[str] = None, device: str = "auto",
                 devices: Sequence[int] = (), batch_max: int = 4096, timeout_us: int = 200,
                 allow_pickle: bool = False, retry_s: float = 30.0):
        self.model = model
        self.model_path = model_path
        self.device_pref = device
        self.device_ids = list(devices)
        self.batch_max = batch_max
        self.timeout_us = timeout_us
        self.allow_pickle = allow_pickle
        self.retry_s = retry_s
        self.error: Optional[str] = None
        self.on_activate: List[Any] = []   # callbacks(model) after a (re)load: the native front end's hot swap
        self._last_try = 0.0
        self._lock = threading.Lock()
        self.batcher: Optional[MicroBatcher] = None
        self.devices: List[torch.device] = []
        self.backend = "none"
        if model is not None:
            self._activate(model)
        elif model_path:
            self.reload()

    # ---- lifecycle ----
    def _gpu_devices(self) -> List[torch.device]:
        if self.device_pref == "cpu" or not torch.cuda.is_available():
            return []
        ids = self.device_ids or list(range(torch.cuda.device_count()))
        return [torch.device("cuda", i) for i in ids]

    def _activate(self, model: Any) -> None:
        from ..ops.eta_mlp import EtaMlpKernel
        runners = []
        devs: List[torch.device] = []
        from ..models.forest import ForestModel
        if isinstance(model, EtaMLP) and model.hidden in (64, 128, 256, 512, 1024):
            for d in self._gpu_devices():
                runners.append(GpuRunner(EtaMlpKernel(model, d), d, self.batch_max))
                devs.append(d)
        elif isinstance(model, ForestModel):
            for d in self._gpu_devices():
                runners.append(GpuRunner(ForestKernel(model, d), d, self.batch_max))
                devs.append(d)
        fallback = None
        if not runners:
            runners = [_cpu_runner(model)]
            self.backend = "cpu"
        else:
            self.backend = "hip"
            fallback = _cpu_runner(model)   # failed GPU batches are re-run here
        old = self.batcher
        self.batcher = MicroBatcher(runners, self.batch_max, self.timeout_us, fallback=fallback)
        self.devices = devs
        self.model = model
        self.error = None
        if old is not None:
            old.close()
        log.info("ETA model active: %s on %s", getattr(model, "arch", type(model).__name__),
                 [str(d) for d in devs] or "cpu")
        for cb in list(self.on_activate):
            try:
                cb(model)
            except Exception as e:  # noqa: BLE001 - a hook failure must not undo the Python reload
                log.error("model activation hook failed: %r", e)

    def reload(self, path: Optional[str] = None) -> bool:
        from ..models.checkpoint import load_any
        with self._lock:
            path = path or self.model_path
            self._last_try = time.time()
            if not path:
                self.error = "no model configured"
                return False
            try:
                self._activate(load_any(path, allow_pickle=self.allow_pickle))
                self.model_path = path
                return True
            except Exception as e:
                self.error = f"ERROR:{e}"
                log.warning("model load failed: %s", self.error)
                return False

    @property
    def available(self) -> bool:
        if self.batcher is not None:
            return True
        if self.model_path and time.time() - self._last_try > self.retry_s:
            return self.reload()
        return False

    def close(self) -> None:
        if self.batcher is not None:
            self.batcher.close()
            self.batcher = None

    # ---- request path ----
    @staticmethod
    def make_record(*, weather: Any, traffic: Any, distance_m: Any, pickup_time: Any,
                    driver_age: Any = 30.0) -> Tuple[tuple, dt.datetime]:
        pickup = coerce_pickup(pickup_time)
        return pack_record(weather=weather, traffic=traffic, distance_m=distance_m, pickup=pickup,
                           driver_age=driver_age), pickup

    @staticmethod
    def finish(minutes: float, pickup: dt.datetime) -> Tuple[float, str]:
        return minutes, (pickup + dt.timedelta(minutes=minutes)).isoformat()

    def predict_eta_minutes(self, **kw: Any) -> Tuple[Optional[float], Optional[str]]:
        """Blocking R17 signature: (minutes, iso) or (None, None)."""
        if not self.available:
            return None, None
        try:
            rec, pickup = self.make_record(**kw)
            return self.finish(self.batcher.predict_sync(rec), pickup)
        except Exception as e:
            log.warning("predict failed: %r", e)
            return None, None

    async def apredict(self, **kw: Any) -> Tuple[Optional[float], Optional[str]]:
        if not self.available:
            return None, None
        try:
            rec, pickup = self.make_record(**kw)
            return self.finish(await self.batcher.submit(rec), pickup)
        except Exception as e:
            log.warning("predict failed: %r", e)
            return None, None

    def predict_records(self, rec: np.ndarray) -> np.ndarray:
        """Bulk path: records straight to one runner (bypasses the request queue)."""
        if not self.available:
            raise RuntimeError(self.error or "model unavailable")
        return self.batcher.runners[0](np.asarray(rec, dtype=RECORD_DTYPE))

    def describe(self) -> dict:
        return {"backend": self.backend, "devices": [str(d) for d in self.devices],
                "arch": getattr(self.model, "arch", type(self.model).__name__ if self.model else None),
                "hidden": getattr(self.model, "hidden", None), "error": self.error,
                "batch_max": self.batch_max, "timeout_us": self.timeout_us,
                "runners": self.batcher.health() if self.batcher is not None else [],
                "degraded": bool(self.batcher is not None and self.batcher.degraded)}


def default_model(seed: int = 0, hidden: int = 256, steps: int = 300) -> EtaMLP:
    """A quickly-trained MLP on synthetic trips (used by `routest serve --synthetic-model`)."""
    from ..data.synth import synth_trips
    torch.manual_seed(seed)
    x, y = synth_trips(20000, seed)
    m = EtaMLP(hidden)
    m.fit_normalization(x, y)
    opt = torch.optim.AdamW(m.parameters(), lr=2e-3)
    xt, yt = torch.from_numpy(x), torch.from_numpy((y - float(m.y_mean)) / float(m.y_std))
    for i in range(steps):
        idx = torch.randint(0, len(xt), (1024,))
        loss = torch.nn.functional.mse_loss(m.forward_normalized(xt[idx]), yt[idx])
        opt.zero_grad()
        loss.backward()
        opt.step()
    return m.eval()
