"""Model export for the reference's own Flask service.

The reference loads ``ETA_MODEL_PATH`` with a bare ``pickle.load`` and calls
``float(model.predict(df)[0])`` on a 12-column pandas DataFrame (``RO/Flaskr/ml.py:11-21,53``).
Its environment is numpy / pandas / xgboost — no torch, no safetensors and no routest_amd
(``RO/requirements.txt:15-16,24``).  A pickle of a routest_amd class would need ``routest_amd``
(and whatever that imports) at load time, so the exported predictor is pickled **by value**:

* the predictor's class source (:data:`PREDICTOR_SOURCE`, numpy only) travels inside the pickle;
  on load, ``builtins.eval`` of a small expression ``exec``s it into a fresh namespace and returns
  the class — nothing outside the standard library and numpy is imported;
* the weights travel as ``(dtype, shape, raw little-endian bytes)`` tuples of builtins, never as
  numpy-pickled arrays (numpy 2 pickles name ``numpy._core``, which numpy 1.26 — the reference's
  pin — may not resolve).

The forward is the fp32 model: ``relu(relu(norm(x) W1ᵀ + b1) W2ᵀ + b2) w3 + b3`` rescaled to minutes
(``models/mlp3.py`` :class:`EtaMLP`), or the least-squares model of config 1 (:class:`LinearETA`).
Column handling follows R16: the DataFrame's 12 named columns are selected in reference order
(``RO/Flaskr/ml.py:35-48``); a plain 2-D array is taken as already in that order.

Unpickling executes code — exactly like the reference's own ``pickle.load`` of its XGBoost file.
Load only exports you made.
"""
from __future__ import annotations

import pickle
from typing import Any, Dict, Tuple

import numpy as np

from .features import FEATURE_COLUMNS

#: numpy-only predictor class, shipped by value inside every exported pickle
PREDICTOR_SOURCE = r'''
import numpy as _np


class EtaPredictor:
    """routest_amd ETA model export: .predict(DataFrame[12 R16 columns]) -> minutes (fp32 forward)."""

    FEATURE_COLUMNS = %(cols)r

    def __init__(self, arch, hidden, tensors):
        self.arch = arch
        self.hidden = hidden
        self._raw = dict(tensors)
        self.p = {k: _np.frombuffer(buf, dtype=_np.dtype(dt)).reshape(shape).copy()
                  for k, (dt, shape, buf) in tensors.items()}

    def __reduce__(self):
        return (_ROUTEST_LOADER, (self.arch, self.hidden, self._raw))

    def _features(self, df):
        if hasattr(df, "columns"):
            cols = list(df.columns)
            missing = [c for c in self.FEATURE_COLUMNS if c not in cols]
            if missing:
                raise ValueError("missing feature columns: %%s" %% missing)
            return df[self.FEATURE_COLUMNS].to_numpy(dtype=_np.float64)
        x = _np.asarray(df, dtype=_np.float64)
        return x.reshape(1, -1) if x.ndim == 1 else x

    def predict(self, df):
        x = self._features(df)
        p = self.p
        if self.arch == "linear":
            return (x @ p["coef"] + p["intercept"][0]).astype(_np.float32)
        f = lambda k: p[k].astype(_np.float32)
        xn = ((x.astype(_np.float32) - f("x_mean")) / f("x_std")).astype(_np.float32)
        h = _np.maximum(xn @ f("l1.weight").T + f("l1.bias"), 0.0)
        h = _np.maximum(h @ f("l2.weight").T + f("l2.bias"), 0.0)
        y = h @ f("l3.weight").reshape(-1) + f("l3.bias")[0]
        return (y * f("y_std").reshape(()) + f("y_mean").reshape(())).astype(_np.float32)
''' % {"cols": list(FEATURE_COLUMNS)}

# eval()'d by pickle on load: exec the class source in a fresh namespace and return the class
_CLASS_EXPR = ("(lambda g: (exec(compile(%r, '<routest_amd EtaPredictor export>', 'exec'), g), "
               "g.__setitem__('_ROUTEST_LOADER', g['EtaPredictor']), g['EtaPredictor'])[2])"
               "({'__name__': 'routest_amd_eta_export'})") % PREDICTOR_SOURCE


class _ClassByValue:
    """Pickles as ``eval(_CLASS_EXPR)``: the unpickled object IS the predictor class."""

    def __reduce__(self):
        import builtins
        return (builtins.eval, (_CLASS_EXPR,))

    def __call__(self, *args):              # pickle requires the reduce callable to be callable
        return EtaPredictor(*args)


def _ns() -> Dict[str, Any]:
    g: Dict[str, Any] = {"__name__": "routest_amd_eta_export"}
    exec(compile(PREDICTOR_SOURCE, "<routest_amd EtaPredictor export>", "exec"), g)
    g["_ROUTEST_LOADER"] = _ClassByValue()
    return g


#: the same class in this process (for tests / in-process use)
EtaPredictor = _ns()["EtaPredictor"]


def _tensors(model: Any) -> Tuple[str, int, Dict[str, Tuple[str, Tuple[int, ...], bytes]]]:
    out = {}
    for k, v in model.state_dict().items():
        a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        a = np.ascontiguousarray(a, dtype="<f8" if model.arch == "linear" else "<f4")
        out[k] = (a.dtype.str, tuple(int(s) for s in a.shape), a.tobytes())
    return model.arch, int(getattr(model, "hidden", 0)), out


def make_predictor(model: Any) -> Any:
    """An in-process :data:`EtaPredictor` holding ``model``'s weights (EtaMLP or LinearETA)."""
    arch, hidden, tensors = _tensors(model)
    if arch not in ("mlp3", "linear"):
        raise ValueError(f"cannot export arch {arch!r}")
    return EtaPredictor(arch, hidden, tensors)


def export_predictor_pickle(model: Any, path: str) -> None:
    """Write ``model`` as a by-value pickle the reference service loads with ``pickle.load``."""
    pred = make_predictor(model)
    with open(path, "wb") as f:
        pickle.dump(pred, f, protocol=4)
