"""On-disk model format + compatibility loaders.

Native checkpoint = a directory::

    config.json          {"arch": "mlp3"|"linear", "hidden", "feature_columns", "target",
                          "dtype", "version", "framework": "routest_amd"}
    model.safetensors    weights + normalisation buffers
    optimizer.safetensors / trainer_state.json   (training resume, optional)

Compatibility:
* :class:`EtaPredictor` is a picklable wrapper exposing ``.predict(pandas.DataFrame[12 R16 cols])``
  -> minutes, so the *reference* Flask service can load a routest_amd model unchanged through
  ``ETA_MODEL_PATH`` (``RO/Flaskr/ml.py:6-21,53``).
* :func:`load_any` also accepts a pickle exposing ``.predict(DataFrame)`` (e.g. the reference's
  ``XGBRegressor``; needs ``xgboost``, which is not installed here) — only when the caller opts in
  (``allow_pickle=True``), since unpickling executes code — and an XGBoost JSON model dump
  (``model.save_model("m.json")``) which is parsed without xgboost and evaluated by the
  tree-ensemble kernel (K4, ``models/forest.py``).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch
from safetensors.torch import load_file, save_file

from .features import FEATURE_COLUMNS, dataframe_to_features
from .mlp3 import EtaMLP, LinearETA

FORMAT_VERSION = 1


def save_checkpoint(path: str, model: Any, optimizer_state: Optional[Dict[str, torch.Tensor]] = None,
                    trainer_state: Optional[Dict[str, Any]] = None, extra_config: Optional[dict] = None) -> None:
    os.makedirs(path, exist_ok=True)
    cfg = {"arch": model.arch, "feature_columns": FEATURE_COLUMNS, "target": "eta_minutes",
           "version": FORMAT_VERSION, "framework": "routest_amd",
           "dtype": "bf16-kernel/fp32-master" if model.arch == "mlp3" else "fp64"}
    if model.arch == "mlp3":
        cfg["hidden"] = model.hidden
        sd = {k: v.detach().float().cpu().contiguous() for k, v in model.state_dict().items()}
    else:
        sd = {k: v.contiguous() for k, v in model.state_dict().items()}
    if extra_config:
        cfg.update(extra_config)
    # every file is written under a temporary name first and only then renamed into place, in one
    # tight sequence ending with trainer_state.json (the resume step) and config.json: a rank killed
    # while saving (torchrun tears the job down when a peer dies) leaves the previous checkpoint's
    # files intact instead of a half-written one
    staged = []
    tmp = os.path.join(path, ".tmp_opt.safetensors")
    if optimizer_state is not None:
        save_file({k: v.detach().cpu().contiguous() for k, v in optimizer_state.items()}, tmp)
        staged.append((tmp, os.path.join(path, "optimizer.safetensors")))
    tmp = os.path.join(path, ".tmp_model.safetensors")
    save_file(sd, tmp)
    staged.append((tmp, os.path.join(path, "model.safetensors")))
    if trainer_state is not None:
        tmp = os.path.join(path, ".tmp_trainer_state.json")
        with open(tmp, "w") as f:
            json.dump(trainer_state, f)
        staged.append((tmp, os.path.join(path, "trainer_state.json")))
    tmp = os.path.join(path, ".tmp_config.json")
    with open(tmp, "w") as f:
        json.dump(cfg, f, indent=1)
    staged.append((tmp, os.path.join(path, "config.json")))
    for src, dst in staged:
        os.replace(src, dst)


def load_checkpoint(path: str) -> Tuple[Any, Dict[str, Any]]:
    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    if cfg.get("feature_columns", FEATURE_COLUMNS) != FEATURE_COLUMNS:
        raise ValueError("checkpoint feature schema differs from R16")
    sd = load_file(os.path.join(path, "model.safetensors"))
    if cfg["arch"] == "mlp3":
        m = EtaMLP(int(cfg["hidden"]))
        m.load_state_dict(sd)
        m.eval()
    elif cfg["arch"] == "linear":
        m = LinearETA()
        m.load_state_dict(sd)
    else:
        raise ValueError(f"unknown arch {cfg['arch']!r}")
    return m, cfg


def load_training_state(path: str) -> Tuple[Optional[Dict[str, torch.Tensor]], Optional[Dict[str, Any]]]:
    opt = ts = None
    p = os.path.join(path, "optimizer.safetensors")
    if os.path.exists(p):
        opt = load_file(p)
    p = os.path.join(path, "trainer_state.json")
    if os.path.exists(p):
        with open(p) as f:
            ts = json.load(f)
    return opt, ts


class EtaPredictor:
    """Picklable ``.predict(DataFrame) -> minutes`` wrapper (reference-loader compatible)."""

    def __init__(self, model: Any):
        self.arch = model.arch
        if self.arch == "mlp3":
            self.hidden = model.hidden
            self.state = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
        else:
            self.hidden = 0
            self.state = {k: v.numpy() for k, v in model.state_dict().items()}
        self._model = None

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_model"] = None
        return d

    def _get(self):
        if self._model is None:
            if self.arch == "mlp3":
                m = EtaMLP(self.hidden)
                m.load_state_dict({k: torch.from_numpy(v) for k, v in self.state.items()})
                self._model = m.eval()
            else:
                m = LinearETA()
                m.load_state_dict({k: torch.from_numpy(v) for k, v in self.state.items()})
                self._model = m
        return self._model

    def predict_features(self, x: np.ndarray) -> np.ndarray:
        m = self._get()
        if self.arch == "mlp3":
            with torch.no_grad():
                return m(torch.as_tensor(np.asarray(x, dtype=np.float32))).numpy()
        return m.predict_features(x)

    def predict(self, df: Any) -> np.ndarray:
        if hasattr(df, "columns"):
            x = dataframe_to_features(df)
        else:
            x = np.asarray(df, dtype=np.float32)
        return self.predict_features(x)


def export_predictor_pickle(model: Any, path: str) -> None:
    import pickle
    with open(path, "wb") as f:
        pickle.dump(EtaPredictor(model), f)


def load_any(path: str, allow_pickle: bool = False) -> Any:
    """Checkpoint dir | XGBoost JSON dump | (opt-in) pickle with ``.predict(DataFrame)``."""
    if os.path.isdir(path):
        return load_checkpoint(path)[0]
    if path.endswith(".json"):
        from .forest import ForestModel
        return ForestModel.from_xgboost_json(path)
    if allow_pickle:
        import pickle
        with open(path, "rb") as f:
            obj = pickle.load(f)  # noqa: S301 - explicit opt-in (ROUTEST_ALLOW_PICKLE=1)
        if not hasattr(obj, "predict"):
            raise ValueError("pickled object has no .predict")
        return obj
    raise ValueError(f"refusing to unpickle {path!r} (set ROUTEST_ALLOW_PICKLE=1 to opt in)")
