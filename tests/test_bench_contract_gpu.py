"""The driver's bench.py contract: one JSON line with the agreed keys, run as a subprocess."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


@pytest.mark.parametrize("io", ["hybrid", "zerocopy"])
def test_bench_json_line(io):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--batch", "262144", "--io", io, "--p50", "0", "--route-steps", "0"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 1e8 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["dtype"] == "bf16" and d["finite"] is True
    assert d["config"]["global_batch"] == 262144 and d["config"]["io"] == io
    assert abs(d["value"] - 262144 * 3 / (d["ms_per_step"] * 3 / 1e3)) / d["value"] < 1e-6


def test_bench_spawns_ranks_itself_shared_gpu():
    """``python bench.py --gpus 2`` (no WORLD_SIZE) launches the 2 ranks itself; on the 1-GPU box
    both share GPU 0 (gloo rendezvous) and the line says so."""
    env = dict(os.environ, ROUTEST_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--batch", "262144", "--p50", "0", "--rec16-steps", "2",
                        "--gcn-steps", "0", "--route-steps", "0"],
                       capture_output=True, text=True, timeout=115, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["shared_gpu"] is True and d["finite"] is True
    assert d["schema_problems"] == [], d["schema_problems"]
    assert d["config"]["global_batch"] == 2 * 262144
    # two ranks time-sharing one GPU through gloo barriers: a sanity floor, not a rate claim
    assert d["preds_per_s_rec16"] > 1e7
    # the DP-training probe on the native one-shot all-reduce: every rank ends on the same params
    os_ = d["dp_training_oneshot"]
    assert os_ and "error" not in os_, os_
    assert os_["params_identical_across_ranks"] is True and os_["comm_error"] is False
    assert abs(os_["final_local_mse_normalized"] - d["dp_training"]["final_local_mse_normalized"]) < 1e-3


def test_bench_route_optimizer_probe():
    """Config 5 inside bench.py: road matrices + K6 + the legs on the CCH per step, every leg found."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--batch", "262144", "--p50", "0", "--rec16-steps", "0", "--train-steps", "0",
                        "--gcn-steps", "0", "--route-requests", "2000", "--route-steps", "2"],
                       capture_output=True, text=True, timeout=115, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    ro = d["route_optimizer"]
    assert ro["requests_per_step"] == 2000 and ro["steps"] == 2
    assert ro["engine"] == "cch" and ro["unfound_legs"] == 0 and ro["requests_per_s"] > 1e3
    assert d["schema_problems"] == [], d["schema_problems"]


def test_bench_fails_loud_on_too_many_gpus():
    import torch
    n = torch.cuda.device_count()
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("ROUTEST_BENCH_SHARE_GPU", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1),
                        "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
    assert r.returncode == 2 and "visible" in r.stderr
