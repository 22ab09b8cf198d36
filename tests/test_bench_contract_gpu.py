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
                        "--batch", "262144", "--io", io, "--p50", "0"],
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
