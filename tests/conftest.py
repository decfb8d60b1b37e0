"""Shared pytest configuration.

Markers: ``gpu`` (needs an MI355X; run with ``-m gpu``), ``slow`` and
``integration`` (real servers / subprocesses; run on demand).
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
os.environ.setdefault("OMP_NUM_THREADS", "4")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950) and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "integration: spawns real servers / processes")


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def models():
    from inference_arena_amd.models.zoo import default_models

    return default_models(0)


@pytest.fixture()
def rng():
    return np.random.default_rng(1234)
