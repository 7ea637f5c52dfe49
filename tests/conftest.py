"""Test configuration.

Markers: `gpu` tests need an MI355X and run on the GPU box
(`pytest -m gpu`); everything else runs on CPU (`pytest -m "not gpu"`).
GPU tests never skip silently: without a device they fail.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-baselines_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)

    return load


@pytest.fixture(scope="session")
def gpu():
    import torch

    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X"
    import mmb_lib

    mmb_lib.load()
    return torch.device("cuda", 0)
