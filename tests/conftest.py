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


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import _dfhip
    _dfhip.load()
    return torch.device("cuda:0")


@pytest.fixture
def rng():
    return np.random.default_rng(0)
