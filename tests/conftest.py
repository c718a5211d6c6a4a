"""Shared pytest setup: import paths, the `gpu` marker, common fixtures."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "single-stable-dreamfusion_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _gpu_selected(config):
    """True when the run was asked for the GPU tests (`-m gpu`, not `-m "not
    gpu"`): then a missing device is a failure, not a skip, so a box whose GPU
    is not visible cannot report a green GPU suite with nothing run."""
    expr = (config.getoption("markexpr") or "").replace(" ", "")
    return "gpu" in expr and "notgpu" not in expr


@pytest.fixture(scope="session")
def gpu(request):
    import torch
    if not torch.cuda.is_available():
        if _gpu_selected(request.config):
            pytest.fail("-m gpu selected but no HIP device is visible (torch.cuda.is_available() "
                        "is False)", pytrace=False)
        pytest.skip("no GPU")
    import _dfhip
    _dfhip.load()
    return torch.device("cuda:0")


@pytest.fixture
def rng():
    return np.random.default_rng(0)
