"""K4 tree-ensemble compatibility path: sklearn parity, XGBoost-JSON round trip, GPU kernel."""
import json

import numpy as np
import pytest
import torch

from routest_amd.data.synth import synth_records, synth_trips
from routest_amd.models.features import records_to_features
from routest_amd.models.forest import ForestModel


@pytest.fixture(scope="module")
def hgb():
    from sklearn.ensemble import HistGradientBoostingRegressor
    x, y = synth_trips(20000, 0)
    x[::97, 10] = np.nan  # exercise missing-value routing
    return HistGradientBoostingRegressor(max_iter=120, max_leaf_nodes=31, random_state=0).fit(x, y)


def test_sklearn_conversion_matches_sklearn(hgb):
    m = ForestModel.from_sklearn_hgb(hgb)
    x, _ = synth_trips(5000, 1)
    x[::50, 10] = np.nan
    np.testing.assert_allclose(m.predict_features(x), hgb.predict(x), rtol=1e-5, atol=1e-4)


def test_xgboost_json_roundtrip(hgb, tmp_path):
    m = ForestModel.from_sklearn_hgb(hgb)
    p = tmp_path / "eta_xgb.json"
    p.write_text(json.dumps(m.to_xgboost_json()))
    m2 = ForestModel.from_xgboost_json(str(p))
    assert not m2.le
    x, _ = synth_trips(3000, 2)
    np.testing.assert_allclose(m2.predict_features(x), m.predict_features(x), rtol=1e-6, atol=1e-5)
    # load_any dispatches .json to the forest loader
    from routest_amd.models.checkpoint import load_any
    assert isinstance(load_any(str(p)), ForestModel)


def test_xgboost_feature_name_reorder(hgb):
    m = ForestModel.from_sklearn_hgb(hgb)
    d = m.to_xgboost_json()
    names = d["learner"]["feature_names"]
    perm = list(reversed(range(12)))
    # re-express the same model with features declared in reversed order
    d["learner"]["feature_names"] = [names[i] for i in perm]
    inv = {old: new for new, old in enumerate(perm)}
    for t in d["learner"]["gradient_booster"]["model"]["trees"]:
        t["split_indices"] = [inv[f] for f in t["split_indices"]]
    m3 = ForestModel.from_xgboost_json(d)
    x, _ = synth_trips(2000, 3)
    np.testing.assert_allclose(m3.predict_features(x), m.predict_features(x), rtol=1e-6, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("lds", [False, True])
@pytest.mark.parametrize("fmt", ["xgb", "sklearn"])
def test_forest_kernel_vs_cpu(hgb, lds, fmt):
    from routest_amd.ops.eta_mlp import records_to_tensor
    from routest_amd.serve.eta_service import ForestKernel
    m = ForestModel.from_sklearn_hgb(hgb)
    if fmt == "xgb":
        m = ForestModel.from_xgboost_json(m.to_xgboost_json())
    rec, _ = synth_records(100_003, 4)
    k = ForestKernel(m, "cuda:0", lds=lds)
    assert (k.chunks is not None) == lds
    got = k(records_to_tensor(rec).cuda()).cpu().numpy()
    ref = m.predict_features(records_to_features(rec))
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)


def test_chunk_table():
    rng = np.random.default_rng(0)
    sizes = rng.integers(1, 300, size=200) * 2 - 1          # odd node counts (full binary trees)
    roots = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int32)
    M = int(sizes.sum())
    m = ForestModel(np.zeros(M, np.float32), np.full(M, 1 << 31, np.uint32), roots, 0.0, True)
    tab = m.chunk_table(cap=1000)
    assert tab[0].tolist() == [0, 0] and tab[-1].tolist() == [200, M]
    for (t0, n0), (t1, n1) in zip(tab[:-1], tab[1:]):
        assert n1 - n0 <= 1000 and roots[t0] == n0 and t1 > t0
    assert m.chunk_table(cap=10) is None


def test_service_serves_forest_on_cpu(hgb):
    from routest_amd.serve.eta_service import EtaService
    m = ForestModel.from_sklearn_hgb(hgb)
    svc = EtaService(model=m, device="cpu")
    try:
        minutes, iso = svc.predict_eta_minutes(weather="Sunny", traffic="High", distance_m=8000,
                                               pickup_time="2025-08-25T08:30:00", driver_age=30)
        assert minutes is not None and minutes > 0 and iso.startswith("2025-08-25T")
    finally:
        svc.close()


def test_corrupt_forest_rejected_before_launch(hgb):
    m = ForestModel.from_sklearn_hgb(hgb)
    bad = ForestModel(m.values, m.info.copy(), m.roots, m.base_score, m.le)
    bad.info[0] = (bad.info[0] & ~np.uint32(0xFFFFFF)) | np.uint32(len(bad.values) + 5)
    with pytest.raises(ValueError):
        bad.validate()
