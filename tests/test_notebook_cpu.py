"""The notebook training entrypoint (notebooks/train_eta.ipynb) executes end to end on CPU."""
import json
import os

import pytest


def test_train_notebook_runs(tmp_path, monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU variant of the notebook")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nb = json.load(open(os.path.join(root, "notebooks", "train_eta.ipynb")))
    nbdir = tmp_path / "notebooks"
    nbdir.mkdir()
    monkeypatch.chdir(nbdir)
    monkeypatch.syspath_prepend(root)
    g = {"__name__": "__notebook__"}
    for cell in nb["cells"]:
        if cell["cell_type"] == "code":
            src = "".join(cell["source"]).replace("os.path.abspath('..')", repr(root))
            exec(compile(src, "train_eta.ipynb", "exec"), g)
    from routest_amd.models.checkpoint import checkpoint_exists
    assert checkpoint_exists(str(nbdir / "out" / "mlp3_ckpt"))
    assert (nbdir / "out" / "train_log.jsonl").exists()
