"""bench.py argument contract checks that need no GPU: it refuses to run with a world size other
than --gpus, and refuses --gpus N when fewer than N GPUs are visible (here: none)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_over):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ROUTEST_BENCH_SHARE_GPU"):
        env.pop(k, None)
    env.update(env_over)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)


def test_world_size_mismatch_exits_2():
    r = _run(["--gpus", "4", "--steps", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_too_many_gpus_exits_2():
    import torch
    if torch.cuda.device_count() >= 8:
        return
    r = _run(["--gpus", "8", "--steps", "1"])
    assert r.returncode == 2 and "visible" in r.stderr
