"""Checkpoint format: atomic versioned snapshots + the reference-loadable export.

* a save is one ``LATEST`` pointer swap: a crash before it leaves the previous snapshot whole
  (weights, optimizer moments and step agree), never a mix (round-2 ADVICE, checkpoint.py:70);
* the export pickle loads in a process where ``torch``, ``safetensors`` and ``routest_amd`` cannot
  be imported — the reference's environment (``RO/requirements.txt:15-16,24``) — and its
  ``.predict(DataFrame)`` matches the checkpoint model (``RO/Flaskr/ml.py:11-21,53``).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from routest_amd.models import checkpoint as ck
from routest_amd.models.features import FEATURE_COLUMNS
from routest_amd.models.mlp3 import EtaMLP, LinearETA


def _model(seed, hidden=64):
    torch.manual_seed(seed)
    m = EtaMLP(hidden)
    x = np.random.default_rng(seed).normal(size=(256, 12)).astype(np.float32) * 3 + 10
    m.fit_normalization(x, x[:, 10] * 2 + 5)
    return m


def test_snapshots_and_pointer(tmp_path):
    d = str(tmp_path / "ck")
    m1, m2, m3 = _model(1), _model(2), _model(3)
    opt = {"exp_avg": torch.ones(10), "exp_avg_sq": torch.ones(10) * 2, "step": torch.tensor([10])}
    ck.save_checkpoint(d, m1, optimizer_state=opt, trainer_state={"step": 10})
    ck.save_checkpoint(d, m2, optimizer_state=opt, trainer_state={"step": 20})
    ck.save_checkpoint(d, m3, optimizer_state=opt, trainer_state={"step": 30})
    assert open(os.path.join(d, "LATEST")).read().strip() == "step_00000030"
    # two snapshots kept
    assert sorted(x for x in os.listdir(d) if x.startswith("step_")) == ["step_00000020", "step_00000030"]
    m, cfg = ck.load_checkpoint(d)
    assert cfg["step"] == 30
    assert torch.equal(m.l2.weight, m3.l2.weight)
    o, ts = ck.load_training_state(d)
    assert ts["step"] == 30 and torch.equal(o["exp_avg"], opt["exp_avg"])
    # re-saving the same step replaces it (under a name of its own) and the pointer stays valid
    ck.save_checkpoint(d, m1, trainer_state={"step": 30})
    m, _ = ck.load_checkpoint(d)
    assert torch.equal(m.l2.weight, m1.l2.weight)
    snaps = sorted(x for x in os.listdir(d) if x.startswith("step_"))
    assert len(snaps) == 2 and snaps[0] == "step_00000020"      # one copy per step
    assert open(os.path.join(d, "LATEST")).read().strip() == snaps[1]


def test_crash_during_same_step_resave_keeps_a_loadable_snapshot(tmp_path, monkeypatch):
    """a re-save of the step LATEST names used to move that directory away before the
    new one took its place; a crash between the two renames left LATEST naming nothing.  Now a
    crash at ANY rename of the re-save leaves LATEST on a complete snapshot."""
    for crash_at in range(2):          # the snapshot rename, the pointer swap
        d = str(tmp_path / f"ck{crash_at}")
        m1, m2 = _model(1), _model(2)
        ck.save_checkpoint(d, m1, trainer_state={"step": 10})
        real_replace = os.replace
        calls = []

        def dying_replace(src, dst):
            calls.append(dst)
            if len(calls) > crash_at:
                raise KeyboardInterrupt("killed mid re-save")
            return real_replace(src, dst)
        monkeypatch.setattr(ck.os, "replace", dying_replace)
        with pytest.raises(KeyboardInterrupt):
            ck.save_checkpoint(d, m2, trainer_state={"step": 10})
        monkeypatch.setattr(ck.os, "replace", real_replace)
        m, cfg = ck.load_checkpoint(d)                 # never a ValueError: LATEST names a snapshot
        assert cfg["step"] == 10
        assert torch.equal(m.l2.weight, m1.l2.weight) or torch.equal(m.l2.weight, m2.l2.weight)


def test_stale_staging_directories_are_removed(tmp_path):
    d = str(tmp_path / "ck")
    os.makedirs(d)
    # a save by a process that no longer exists died mid-write
    dead = subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True,
                          text=True).stdout.strip()
    stale = os.path.join(d, f".staging_{dead}_7")
    os.makedirs(stale)
    open(os.path.join(stale, "model.safetensors"), "w").write("x" * 100)
    ck.save_checkpoint(d, _model(1), trainer_state={"step": 8})
    assert not os.path.exists(stale)
    assert ck.load_checkpoint(d)[1]["step"] == 8


def test_crash_before_pointer_swap_keeps_previous_snapshot(tmp_path, monkeypatch):
    d = str(tmp_path / "ck")
    m1, m2 = _model(1), _model(2)
    ck.save_checkpoint(d, m1, optimizer_state={"exp_avg": torch.zeros(3)}, trainer_state={"step": 10})
    real_replace = os.replace

    def dying_replace(src, dst):
        if os.path.basename(dst) == "LATEST":
            raise KeyboardInterrupt("killed between the snapshot rename and the pointer swap")
        return real_replace(src, dst)
    monkeypatch.setattr(ck.os, "replace", dying_replace)
    with pytest.raises(KeyboardInterrupt):
        ck.save_checkpoint(d, m2, optimizer_state={"exp_avg": torch.ones(3)}, trainer_state={"step": 20})
    monkeypatch.setattr(ck.os, "replace", real_replace)
    m, cfg = ck.load_checkpoint(d)
    o, ts = ck.load_training_state(d)
    # weights, moments and step all from the step-10 snapshot: a consistent set
    assert cfg["step"] == 10 and ts["step"] == 10
    assert torch.equal(m.l2.weight, m1.l2.weight) and torch.equal(o["exp_avg"], torch.zeros(3))


def test_legacy_flat_directory_loads(tmp_path):
    from safetensors.torch import save_file
    m = _model(4)
    d = tmp_path / "flat"
    d.mkdir()
    save_file({k: v.contiguous() for k, v in m.state_dict().items()}, str(d / "model.safetensors"))
    (d / "config.json").write_text(json.dumps({"arch": "mlp3", "hidden": 64, "feature_columns": FEATURE_COLUMNS}))
    m2, _ = ck.load_checkpoint(str(d))
    assert torch.equal(m2.l1.weight, m.l1.weight)
    assert ck.checkpoint_exists(str(d)) and not ck.checkpoint_exists(str(tmp_path / "none"))


_LOADER = r'''
import sys, pickle, json
for mod in ("torch", "safetensors", "safetensors.torch", "routest_amd"):
    sys.modules[mod] = None                      # the reference env has none of these
import pandas as pd
rows = json.loads(sys.argv[2])
with open(sys.argv[1], "rb") as f:
    model = pickle.load(f)                       # RO/Flaskr/ml.py:11-21 (bare pickle.load)
cols = %r
df = pd.DataFrame(rows, columns=cols)
out = [float(model.predict(df.iloc[[i]])[0]) for i in range(len(df))]   # ml.py:53, batch 1
out_b = [float(v) for v in model.predict(df)]
assert not any(m.startswith("routest_amd") for m in sys.modules if sys.modules[m] is not None)
print(json.dumps({"one": out, "batch": out_b}))
''' % (FEATURE_COLUMNS,)


@pytest.mark.parametrize("arch", ["mlp3", "linear"])
def test_export_loads_without_torch_or_routest(tmp_path, arch):
    if arch == "mlp3":
        m = _model(5, hidden=128)
    else:
        rng = np.random.default_rng(0)
        x = rng.normal(size=(500, 12))
        m = LinearETA().fit(x, x @ rng.normal(size=12) + 3.0)
    ck.save_checkpoint(str(tmp_path / "ck"), m, trainer_state={"step": 1})
    model, _ = ck.load_checkpoint(str(tmp_path / "ck"))
    pkl = str(tmp_path / "eta.pkl")
    ck.export_predictor_pickle(model, pkl)
    rows = []
    for i, (w, t) in enumerate([("Sunny", "Low"), ("Stormy", "Jam"), ("Fog", "Medium"), ("Windy", "High")]):
        feats = {c: False for c in FEATURE_COLUMNS}
        if f"weather_{w}" in feats:
            feats[f"weather_{w}"] = True
        feats[f"traffic_{t}"] = True
        feats.update(weekday_ordered=i, hour_ordered=7 + 3 * i, distance_km=1.5 + 7.25 * i, driver_age=30.0 + i)
        rows.append([feats[c] for c in FEATURE_COLUMNS])
    env = dict(os.environ, PYTHONPATH="")
    r = subprocess.run([sys.executable, "-c", _LOADER, pkl, json.dumps(rows)], capture_output=True,
                       text=True, timeout=120, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    x = np.array(rows, dtype=np.float32)
    if arch == "mlp3":
        with torch.no_grad():
            ref = model(torch.from_numpy(x)).numpy()
    else:
        ref = model.predict_features(x)
    np.testing.assert_allclose(got["one"], ref, atol=1e-4, rtol=0)
    np.testing.assert_allclose(got["batch"], ref, atol=1e-4, rtol=0)
