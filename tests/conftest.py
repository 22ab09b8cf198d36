import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "multigpu: needs >=2 GPUs")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "run_first: timing-sensitive GPU child process; collected ahead "
                            "of every other test, before this runner holds queues on the GPU")


def _cuda_count() -> int:
    try:
        import torch
        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:
        return 0


def pytest_collection_modifyitems(config, items):
    n = _cuda_count()
    skip_gpu = pytest.mark.skip(reason="no GPU visible")
    skip_multi = pytest.mark.skip(reason="needs >=2 GPUs")
    # a test that times a child process on the one shared GPU runs before the runner itself has
    # created streams / hardware queues there (the child's 32 queues plus the runner's exceed the
    # hardware queue slots, and the scheduler then time-slices them: ~100 ms stalls that are the
    # rehearsal's, not the code's).  Stable: the rest keep their order.
    first = [it for it in items if "run_first" in it.keywords]
    if first:
        items[:] = first + [it for it in items if "run_first" not in it.keywords]
    for it in items:
        if "gpu" in it.keywords and n == 0:
            it.add_marker(skip_gpu)
        if "multigpu" in it.keywords and n < 2:
            it.add_marker(skip_multi)
