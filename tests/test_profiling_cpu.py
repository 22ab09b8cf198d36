"""Profiling helpers: Chrome-trace export, debug env, /metrics scrape never fails."""
import json
import os

from routest_amd.utils.profiling import apply_debug_env, chrome_trace


def test_chrome_trace_cpu(tmp_path):
    import torch
    p = tmp_path / "t.json"
    with chrome_trace(str(p)):
        torch.randn(64, 64) @ torch.randn(64, 64)
    d = json.loads(p.read_text())
    assert "traceEvents" in d and len(d["traceEvents"]) > 0


def test_debug_env():
    env = {"ROUTEST_DEBUG_SYNC": "1"}
    assert apply_debug_env(env)
    assert env["AMD_SERIALIZE_KERNEL"] == "3" and env["HIP_LAUNCH_BLOCKING"] == "1"
    assert not apply_debug_env({})


def test_metrics_render():
    from routest_amd.utils.metrics import REGISTRY
    txt = REGISTRY.render()
    assert "routest_requests_total" in txt or "routest_eta_predictions_total" in txt
