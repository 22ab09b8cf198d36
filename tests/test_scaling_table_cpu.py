"""tools/scaling_table.py: efficiency table from bench.py lines at several GPU counts."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import scaling_table  # noqa: E402


def _line(n, v, dp, shared=False):
    return json.dumps({"n_gpus": n, "value": v, "shared_gpu": shared,
                       "dp_training": {"samples_per_s": dp}, "gcn": {"replicate": {"routes_per_s": 1e8 * n}},
                       "route_optimizer": None})


def test_weak_scaling_efficiency_rows():
    lines = [_line(1, 9e9, 8e8), _line(2, 18e9, 1.5e9), "not json", _line(8, 68.4e9, 5.6e9)]
    t = scaling_table.table(scaling_table.load(lines))
    assert "| config 2: ETA preds/s (headline) | preds/s | 9e+09 | 1.8e+10 | 6.84e+10 | 95.0 % |" in t
    assert "87.5 %" in t                 # 5.6e9 / (8 * 8e8)
    assert "route optimizer" not in t    # absent everywhere -> no row
    assert "SHARED" not in t


def test_shared_gpu_runs_are_flagged():
    t = scaling_table.table(scaling_table.load([_line(1, 9e9, 8e8), _line(2, 8e9, 3e8, shared=True)]))
    assert "SHARED one GPU" in t
