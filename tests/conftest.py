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
    for it in items:
        if "gpu" in it.keywords and n == 0:
            it.add_marker(skip_gpu)
        if "multigpu" in it.keywords and n < 2:
            it.add_marker(skip_multi)
