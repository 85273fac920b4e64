import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")


# Whole-network training trajectories run after every kernel / op test, so a trajectory bound can
# never keep (under -x) the op-level numerics tests from running.
_LAST = ("test_convergence_gpu.py",)


def pytest_collection_modifyitems(config, items):
    import torch

    items.sort(key=lambda it: os.path.basename(str(it.fspath)) in _LAST)  # stable
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
