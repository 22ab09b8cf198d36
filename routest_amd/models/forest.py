"""Tree-ensemble ETA models (K4) — compatibility with the reference's XGBoost regressor.

The reference serves a pickled sklearn-API ``XGBRegressor`` (``RO/Flaskr/ml.py:11-21,53``;
``RO/xgb_eta_model.pkl`` is only a Git-LFS pointer in the mount).  Unpickling needs ``xgboost``
(not installed) and executes code, so instead we load XGBoost's portable JSON dump
(``model.save_model("eta.json")``) with a plain JSON parser, or convert an sklearn
``HistGradientBoostingRegressor``.  Trees are re-laid out breadth-first so both children of a node
are adjacent, and packed into 8-byte nodes for the GPU kernel (``csrc/forest.hip``):

    node = (float value_or_threshold, u32 info)
    info = is_leaf << 31 | default_left << 30 | feature << 24 | left_child_offset (24 bits)

Decision rule per model: XGBoost ``x < thr`` goes left, sklearn ``x <= thr`` goes left; missing
(NaN) goes the node's default direction.  Prediction = base_score + sum of leaf values.
"""
from __future__ import annotations

import json
from collections import deque
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from .features import FEATURE_COLUMNS


class ForestModel:
    arch = "forest"

    def __init__(self, values: np.ndarray, info: np.ndarray, roots: np.ndarray, base_score: float,
                 le: bool, feature_map: Optional[Sequence[int]] = None):
        self.values = np.asarray(values, dtype=np.float32)
        self.info = np.asarray(info, dtype=np.uint32)
        self.roots = np.asarray(roots, dtype=np.int32)
        self.base_score = float(base_score)
        self.le = bool(le)                      # True: x <= thr goes left (sklearn)
        self.feature_map = list(feature_map) if feature_map is not None else list(range(12))

    @property
    def num_trees(self) -> int:
        return int(self.roots.shape[0])

    # ------------------------------------------------------------------ builders
    @staticmethod
    def _pack(trees: List[Dict[str, np.ndarray]], base: float, le: bool, feature_map) -> "ForestModel":
        vals, infos, roots = [], [], []
        off = 0
        for t in trees:
            left, right, feat = t["left"], t["right"], t["feat"]
            thr, leafv, dleft = t["thr"], t["leaf"], t["default_left"]
            order, pos = [], {}
            q = deque([0])
            while q:                              # BFS: children of a node are emitted adjacently
                n = q.popleft()
                pos[n] = len(order)
                order.append(n)
                if left[n] != -1:
                    q.append(int(left[n]))
                    q.append(int(right[n]))
            roots.append(off)
            for n in order:
                if left[n] == -1:
                    vals.append(float(leafv[n]))
                    infos.append(1 << 31)
                else:
                    lo = pos[int(left[n])]
                    assert pos[int(right[n])] == lo + 1
                    f = int(feat[n])
                    if not 0 <= f < 64 or lo >= (1 << 24):
                        raise ValueError("tree too large for the packed node format")
                    vals.append(float(thr[n]))
                    infos.append((int(bool(dleft[n])) << 30) | (f << 24) | lo)
            off += len(order)
        return ForestModel(np.array(vals, np.float32), np.array(infos, np.uint32), np.array(roots, np.int32),
                           base, le, feature_map)

    @classmethod
    def from_xgboost_json(cls, path_or_dict: Any) -> "ForestModel":
        d = path_or_dict
        if isinstance(d, str):
            with open(d) as f:
                d = json.load(f)
        learner = d["learner"]
        names = learner.get("feature_names") or FEATURE_COLUMNS
        # model feature j -> R16 column index
        fmap = [FEATURE_COLUMNS.index(n) for n in names]
        base = float(learner["learner_model_param"]["base_score"])
        gb = learner["gradient_booster"]
        model = gb["model"] if "model" in gb else gb["gbtree"]["model"]
        trees = []
        for t in model["trees"]:
            left = np.asarray(t["left_children"], np.int64)
            trees.append({"left": left, "right": np.asarray(t["right_children"], np.int64),
                          "feat": np.asarray(t["split_indices"], np.int64),
                          "thr": np.asarray(t["split_conditions"], np.float32),
                          "leaf": np.asarray(t["split_conditions"], np.float32),
                          "default_left": np.asarray(t["default_left"], np.int64)})
        m = cls._pack(trees, base, le=False, feature_map=fmap)
        return m

    @classmethod
    def from_sklearn_hgb(cls, est) -> "ForestModel":
        trees = []
        for (pred,) in est._predictors:
            n = pred.nodes
            leaf = n["is_leaf"].astype(bool)
            left = np.where(leaf, -1, n["left"].astype(np.int64))
            right = np.where(leaf, -1, n["right"].astype(np.int64))
            thr64 = n["num_threshold"].astype(np.float64)
            thr32 = thr64.astype(np.float32)
            # largest float32 <= the float64 threshold: `x <= thr` is then exact for float32 x
            thr32 = np.where(thr32.astype(np.float64) > thr64, np.nextafter(thr32, np.float32(-np.inf)), thr32)
            trees.append({"left": left, "right": right, "feat": n["feature_idx"].astype(np.int64),
                          "thr": thr32, "leaf": n["value"].astype(np.float32),
                          "default_left": n["missing_go_to_left"].astype(np.int64)})
        base = float(np.asarray(est._baseline_prediction).reshape(-1)[0])
        return cls._pack(trees, base, le=True, feature_map=list(range(12)))

    def to_xgboost_json(self) -> Dict[str, Any]:
        """Write this forest in XGBoost's JSON schema (x < thr semantics; `<=` thresholds are
        nudged to the next float32 up).  Used to build parser fixtures without xgboost."""
        trees = []
        for ti, r in enumerate(self.roots):
            end = self.roots[ti + 1] if ti + 1 < len(self.roots) else len(self.values)
            L, R, F, S, D = [], [], [], [], []
            for k in range(r, end):
                inf = int(self.info[k])
                if inf >> 31:
                    L.append(-1); R.append(-1); F.append(0); S.append(float(self.values[k])); D.append(0)
                else:
                    lo = inf & 0xFFFFFF
                    L.append(int(lo)); R.append(int(lo + 1))
                    F.append((inf >> 24) & 63)
                    t = np.float32(self.values[k])
                    S.append(float(np.nextafter(t, np.float32(np.inf)) if self.le else t))
                    D.append((inf >> 30) & 1)
            trees.append({"left_children": L, "right_children": R, "split_indices": F,
                          "split_conditions": S, "default_left": D, "base_weights": S})
        names = [FEATURE_COLUMNS[j] for j in self.feature_map]
        return {"learner": {"feature_names": names,
                            "learner_model_param": {"base_score": repr(self.base_score), "num_feature": "12"},
                            "gradient_booster": {"name": "gbtree", "model": {"trees": trees}}},
                "version": [2, 1, 1]}

    # ------------------------------------------------------------------ inference
    def predict_features(self, x: np.ndarray) -> np.ndarray:
        """CPU reference traversal (vectorised over rows, per tree)."""
        x = np.asarray(x, dtype=np.float32)
        xm = x[:, self.feature_map] if self.feature_map != list(range(12)) else x
        b = x.shape[0]
        out = np.full(b, self.base_score, dtype=np.float64)
        rows = np.arange(b)
        for r in self.roots:
            node = np.full(b, r, dtype=np.int64)
            while True:
                inf = self.info[node]
                leaf = (inf >> 31) == 1
                if leaf.all():
                    break
                f = (inf >> 24) & 63
                v = xm[rows, np.where(leaf, 0, f)]
                thr = self.values[node]
                go_left = np.where(np.isnan(v), ((inf >> 30) & 1) == 1, (v <= thr) if self.le else (v < thr))
                child = self.roots_offset(node) + (inf & 0xFFFFFF) + np.where(go_left, 0, 1)
                node = np.where(leaf, node, child)
            out += self.values[node]
        return out.astype(np.float32)

    def roots_offset(self, node: np.ndarray) -> np.ndarray:
        idx = np.searchsorted(self.roots, node, side="right") - 1
        return self.roots[idx]

    def validate(self) -> None:
        """Host check of the packed format (children in range, features < 12) before any launch."""
        M = len(self.values)
        if len(self.info) != M or not len(self.roots) or self.roots[0] != 0 or np.any(np.diff(self.roots) <= 0):
            raise ValueError("malformed forest arrays")
        inner = (self.info >> 31) == 0
        idx = np.nonzero(inner)[0]
        child = self.roots_offset(idx) + (self.info[idx] & 0xFFFFFF).astype(np.int64)
        if np.any(child + 1 >= M) or np.any(((self.info[idx] >> 24) & 63) >= 12):
            raise ValueError("forest node references out of range")

    def device_arrays(self, device):
        import torch
        self.validate()
        d = torch.device(device)
        return (torch.from_numpy(self.values).to(d), torch.from_numpy(self.info.view(np.int32)).to(d),
                torch.from_numpy(self.roots).to(d))

    LDS_NODES = 12288      # csrc/forest.hip FOREST_LDS_NODES (96 KB of 8-byte nodes per chunk)

    def chunk_table(self, cap: int = LDS_NODES) -> Optional[np.ndarray]:
        """Greedy cut of the tree list into chunks of <= cap nodes at tree boundaries:
        int32 [C+1, 2] of (first tree, first node).  None if one tree alone exceeds cap."""
        ends = np.append(self.roots[1:], len(self.values)).astype(np.int64)
        sizes = ends - self.roots
        if len(sizes) == 0 or sizes.max() > cap:
            return None
        rows = [(0, 0)]
        cur = 0
        for t, sz in enumerate(sizes):
            if cur + sz > cap:
                rows.append((t, int(self.roots[t])))
                cur = 0
            cur += int(sz)
        rows.append((len(sizes), len(self.values)))
        return np.asarray(rows, dtype=np.int32)

    def nodes2(self) -> np.ndarray:
        """(value bits, info) interleaved int32 [M, 2] for the LDS kernel's 8-byte node loads."""
        return np.stack([self.values.view(np.int32), self.info.view(np.int32)], axis=1).copy()

    def predict(self, df: Any) -> np.ndarray:
        from .features import dataframe_to_features
        x = dataframe_to_features(df) if hasattr(df, "columns") else np.asarray(df, dtype=np.float32)
        return self.predict_features(x)
