"""Elastic recovery end to end ("DP training that resumes from the last checkpoint with
torchrun --max-restarts"): a 2-rank Gloo job whose last rank dies hard mid-run (``ROUTEST_FAULT=
rank_crash@25``, first attempt only) is relaunched by the real launcher, resumes from the step-20
checkpoint and finishes at the absolute ``--max-steps``."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(backend: str, extra_env=None):
    with tempfile.TemporaryDirectory() as d:
        ck = os.path.join(d, "ckpt")
        env = dict(os.environ, ROUTEST_FAULT="rank_crash@25", PYTHONPATH=ROOT, OMP_NUM_THREADS="2",
                   **(extra_env or {}))
        env.pop("WORLD_SIZE", None)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
               "--max-restarts", "1", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               "-m", "routest_amd.train", "--hidden", "64", "--batch-local", "512", "--steps", "40",
               "--max-steps", "40", "--rows-per-rank", "4096", "--eval-rows", "1024", "--log-every", "10",
               "--ckpt-dir", ck, "--ckpt-every", "10", "--backend", backend, "--dist-backend", "gloo",
               "--warmup", "5"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=d, env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-8000:])
        # the first attempt really died at step 25; the relaunch resumed from the step-20 checkpoint
        assert "exits hard at step 25" in r.stderr, r.stderr[-3000:]
        res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        assert res["start_step"] == 20 and res["end_step"] == 40 and res["world"] == 2
        from routest_amd.models.checkpoint import load_training_state
        _, ts = load_training_state(ck)
        assert ts["step"] == 40


def test_torchrun_max_restarts_resumes_after_rank_crash():
    _run("autograd")


@pytest.mark.gpu
def test_torchrun_max_restarts_fused_hip_trainer_shared_gpu():
    """The same on the fused HIP trainer: both ranks on GPU 0 (gloo), the relaunch restores the
    flat fp32 params and the AdamW moments into the kernels' buffers and finishes."""
    _run("fused", {"ROUTEST_BENCH_SHARE_GPU": "1"})
