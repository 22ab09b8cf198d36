"""On-disk model format + compatibility loaders.

Native checkpoint = a directory holding versioned snapshots and one pointer::

    <path>/LATEST                   text: name of the current snapshot directory (e.g. step_00000120)
    <path>/step_00000120/
        config.json                 {"arch": "mlp3"|"linear", "hidden", "feature_columns", "target",
                                     "dtype", "version", "framework": "routest_amd", "step"}
        model.safetensors           weights + normalisation buffers
        optimizer.safetensors       flat AdamW moments (training resume, optional)
        trainer_state.json          {"step", "config", "world"} (training resume, optional)

A save writes a complete snapshot into a private staging directory, fsyncs every file and the
directory, renames it to ``step_N`` (``step_N.<pid>_<ns>`` when that step already has a snapshot,
so a re-save never moves the directory ``LATEST`` names) and only then swaps ``LATEST`` with ONE
``os.replace`` (fsynced as well).  Staging directories of saves whose process died are removed by
the next save.  A rank killed at any point leaves either the previous snapshot or the new one as
``LATEST`` — never new weights beside an old step counter (round-2 ADVICE: the per-file renames
could mix them).  The two most recent snapshots are kept.  A flat legacy directory
(``config.json`` + ``model.safetensors`` directly inside) still loads.

Compatibility:
* :func:`export_predictor_pickle` (``models/export.py``) writes a by-value pickle exposing
  ``.predict(pandas.DataFrame[12 R16 cols])`` -> minutes that the *reference* Flask service loads
  unchanged through ``ETA_MODEL_PATH`` with numpy + pandas only (``RO/Flaskr/ml.py:6-21,53``).
* :func:`load_any` also accepts a pickle exposing ``.predict(DataFrame)`` (e.g. the reference's
  ``XGBRegressor``; needs ``xgboost``, which is not installed here) — only when the caller opts in
  (``allow_pickle=True``), since unpickling executes code — and an XGBoost JSON model dump
  (``model.save_model("m.json")``) which is parsed without xgboost and evaluated by the
  tree-ensemble kernel (K4, ``models/forest.py``).
"""
from __future__ import annotations

import json
import os
import re
import shutil
import time
from typing import Any, Dict, Optional, Tuple

import torch
from safetensors.torch import load_file, save_file

from .export import EtaPredictor, export_predictor_pickle, make_predictor  # noqa: F401 (re-export)
from .features import FEATURE_COLUMNS
from .mlp3 import EtaMLP, LinearETA

FORMAT_VERSION = 2
LATEST = "LATEST"
KEEP = 2
_SNAP_RE = re.compile(r"^step_(\d+)(\.\d+_\d+)?$")
_TMP_RE = re.compile(r"^\.(?:staging|old)_(\d+)_")


def _fsync_file(p: str) -> None:
    fd = os.open(p, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _fsync_dir(p: str) -> None:
    try:
        fd = os.open(p, os.O_RDONLY | os.O_DIRECTORY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def resolve_checkpoint(path: str) -> Optional[str]:
    """The snapshot directory ``path`` currently designates, or None if there is none."""
    ptr = os.path.join(path, LATEST)
    if os.path.isfile(ptr):
        with open(ptr) as f:
            name = f.read().strip()
        d = os.path.join(path, name)
        if name and os.path.basename(name) == name and os.path.isfile(os.path.join(d, "config.json")):
            return d
        raise ValueError(f"checkpoint pointer {ptr} names a missing snapshot {name!r}")
    if os.path.isfile(os.path.join(path, "config.json")):
        return path                                   # flat legacy layout
    return None


def checkpoint_exists(path: Optional[str]) -> bool:
    return bool(path) and os.path.isdir(path) and resolve_checkpoint(path) is not None


def save_checkpoint(path: str, model: Any, optimizer_state: Optional[Dict[str, torch.Tensor]] = None,
                    trainer_state: Optional[Dict[str, Any]] = None, extra_config: Optional[dict] = None) -> str:
    """Write one complete snapshot and atomically make it ``LATEST``; returns its directory."""
    os.makedirs(path, exist_ok=True)
    step = int((trainer_state or {}).get("step", 0))
    cfg = {"arch": model.arch, "feature_columns": FEATURE_COLUMNS, "target": "eta_minutes",
           "version": FORMAT_VERSION, "framework": "routest_amd", "step": step,
           "dtype": "bf16-kernel/fp32-master" if model.arch == "mlp3" else "fp64"}
    if model.arch == "mlp3":
        cfg["hidden"] = model.hidden
        sd = {k: v.detach().float().cpu().contiguous() for k, v in model.state_dict().items()}
    else:
        sd = {k: v.contiguous() for k, v in model.state_dict().items()}
    if extra_config:
        cfg.update(extra_config)
    _clean_stale(path)
    stage = os.path.join(path, f".staging_{os.getpid()}_{step}")
    shutil.rmtree(stage, ignore_errors=True)
    os.makedirs(stage)
    files = []
    if optimizer_state is not None:
        p = os.path.join(stage, "optimizer.safetensors")
        save_file({k: v.detach().cpu().contiguous() for k, v in optimizer_state.items()}, p)
        files.append(p)
    p = os.path.join(stage, "model.safetensors")
    save_file(sd, p)
    files.append(p)
    if trainer_state is not None:
        p = os.path.join(stage, "trainer_state.json")
        with open(p, "w") as f:
            json.dump(trainer_state, f)
        files.append(p)
    p = os.path.join(stage, "config.json")
    with open(p, "w") as f:
        json.dump(cfg, f, indent=1)
    files.append(p)
    for p in files:
        _fsync_file(p)
    _fsync_dir(stage)
    name = f"step_{step:08d}"
    if os.path.exists(os.path.join(path, name)):
        # re-save of a step that already has a snapshot: the new copy gets a name of its own and
        # the LATEST swap below stays the ONLY commit point (a crash at any moment leaves LATEST on
        # a complete snapshot); the superseded copy is removed only after the swap
        name = f"{name}.{os.getpid()}_{time.time_ns()}"
    final = os.path.join(path, name)
    os.replace(stage, final)
    _fsync_dir(path)
    tmp = os.path.join(path, f".{LATEST}.{os.getpid()}")
    with open(tmp, "w") as f:
        f.write(name + "\n")
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, os.path.join(path, LATEST))       # the commit point
    _fsync_dir(path)
    _prune(path, keep_name=name)
    return final


def _snap_step(d: str) -> Optional[int]:
    m = _SNAP_RE.match(d)
    return int(m.group(1)) if m else None


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def _clean_stale(path: str) -> None:
    """Remove staging / superseded directories left by saves that died mid-write (their writer
    process is gone); a live writer's directories are left alone."""
    for d in os.listdir(path):
        m = _TMP_RE.match(d)
        if m and int(m.group(1)) != os.getpid() and not _pid_alive(int(m.group(1))):
            shutil.rmtree(os.path.join(path, d), ignore_errors=True)


def _prune(path: str, keep_name: str) -> None:
    """Keep the snapshots of the KEEP most recent steps (one copy per step: the LATEST one for its
    step, else the newest) and never ``keep_name``."""
    by_step: Dict[int, list] = {}
    for d in os.listdir(path):
        st = _snap_step(d)
        if st is not None and os.path.isdir(os.path.join(path, d)):
            by_step.setdefault(st, []).append(d)
    keep_step = _snap_step(keep_name)
    steps = sorted(by_step)
    kept = set(steps[-KEEP:])
    for st in steps:
        names = sorted(by_step[st], key=lambda d: os.stat(os.path.join(path, d)).st_mtime_ns)
        if st == keep_step:
            survivors = {keep_name}
        elif st in kept:
            survivors = {names[-1]}
        else:
            survivors = set()
        for d in names:
            if d not in survivors:
                shutil.rmtree(os.path.join(path, d), ignore_errors=True)
    _clean_stale(path)


def load_checkpoint(path: str) -> Tuple[Any, Dict[str, Any]]:
    d = resolve_checkpoint(path)
    if d is None:
        raise FileNotFoundError(f"no checkpoint in {path!r}")
    with open(os.path.join(d, "config.json")) as f:
        cfg = json.load(f)
    if cfg.get("feature_columns", FEATURE_COLUMNS) != FEATURE_COLUMNS:
        raise ValueError("checkpoint feature schema differs from R16")
    sd = load_file(os.path.join(d, "model.safetensors"))
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
    d = resolve_checkpoint(path)
    opt = ts = None
    if d is None:
        return opt, ts
    p = os.path.join(d, "optimizer.safetensors")
    if os.path.exists(p):
        opt = load_file(p)
    p = os.path.join(d, "trainer_state.json")
    if os.path.exists(p):
        with open(p) as f:
            ts = json.load(f)
    return opt, ts


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
