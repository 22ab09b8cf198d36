"""ETA regressors.

* :class:`EtaMLP` — the 3-layer MLP ``12 -> H -> H -> 1`` (configs 2-3).  Replaces the reference's
  pickled XGBoost regressor (``RO/Flaskr/ml.py:11-21,53``; ``RO/xgb_eta_model.pkl``) with a model
  whose hot path is a single fused HIP launch (``csrc/eta_mlp_fwd.hip``).  Input normalisation
  (numeric features only) and target scaling are buffers of the module, so a checkpoint is
  self-contained.
* :class:`LinearETA` — closed-form least-squares ETA (config 1, CPU plumbing).

Both accept raw R16 features ``[B, 12]`` (``models/features.py``) and return minutes.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from .features import NUM_FEATURES

NUMERIC = slice(8, 12)   # weekday, hour, distance_km, driver_age


class EtaMLP(nn.Module):
    arch = "mlp3"

    def __init__(self, hidden: int = 256):
        super().__init__()
        if hidden % 32 != 0:
            raise ValueError("hidden must be a multiple of 32 (MFMA 32x32 tiles)")
        self.hidden = hidden
        self.l1 = nn.Linear(NUM_FEATURES, hidden)
        self.l2 = nn.Linear(hidden, hidden)
        self.l3 = nn.Linear(hidden, 1)
        self.register_buffer("x_mean", torch.zeros(NUM_FEATURES))
        self.register_buffer("x_std", torch.ones(NUM_FEATURES))
        self.register_buffer("y_mean", torch.zeros(()))
        self.register_buffer("y_std", torch.ones(()))

    @torch.no_grad()
    def fit_normalization(self, x: np.ndarray, y: Optional[np.ndarray] = None) -> None:
        x = torch.as_tensor(np.asarray(x, dtype=np.float32))
        mean = torch.zeros(NUM_FEATURES)
        std = torch.ones(NUM_FEATURES)
        mean[NUMERIC] = x[:, NUMERIC].mean(0)
        std[NUMERIC] = x[:, NUMERIC].std(0).clamp_min(1e-3)
        self.x_mean.copy_(mean)
        self.x_std.copy_(std)
        if y is not None:
            yt = torch.as_tensor(np.asarray(y, dtype=np.float32))
            self.y_mean.copy_(yt.mean())
            self.y_std.copy_(yt.std().clamp_min(1e-3))

    def normalize_x(self, x: torch.Tensor) -> torch.Tensor:
        return (x - self.x_mean) / self.x_std

    def forward_normalized(self, x: torch.Tensor) -> torch.Tensor:
        h = torch.relu(self.l1(self.normalize_x(x)))
        h = torch.relu(self.l2(h))
        return self.l3(h).squeeze(-1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward_normalized(x) * self.y_std + self.y_mean

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())


class LinearETA:
    """Config 1: ordinary least squares with a bias, numpy only (no GPU)."""

    arch = "linear"

    def __init__(self) -> None:
        self.coef = np.zeros(NUM_FEATURES, dtype=np.float64)
        self.intercept = 0.0

    def fit(self, x: np.ndarray, y: np.ndarray, l2: float = 1e-6) -> "LinearETA":
        x = np.asarray(x, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        a = np.hstack([x, np.ones((x.shape[0], 1))])
        reg = l2 * np.eye(a.shape[1])
        reg[-1, -1] = 0.0
        w = np.linalg.solve(a.T @ a + reg, a.T @ y)
        self.coef, self.intercept = w[:-1], float(w[-1])
        return self

    def predict_features(self, x: np.ndarray) -> np.ndarray:
        return (np.asarray(x, dtype=np.float64) @ self.coef + self.intercept).astype(np.float32)

    def state_dict(self) -> dict:
        return {"coef": torch.tensor(self.coef, dtype=torch.float64),
                "intercept": torch.tensor([self.intercept], dtype=torch.float64)}

    def load_state_dict(self, sd: dict) -> None:
        self.coef = sd["coef"].double().numpy()
        self.intercept = float(sd["intercept"].double().numpy()[0])
