"""Shared test setup.

Markers: ``gpu`` — needs a real MI355X (run with ``-m gpu``); everything else
runs on CPU.  The oracle (oracle/, test infrastructure) is the parity
checker; libtensorium_hip.so is the product under test.
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X (gfx950) GPU")


def _ensure_oracle():
    # always ask make: oracle/Makefile knows every source and header the
    # checker depends on (a no-op when libtns_oracle.so is current)
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


def _ensure_hip():
    from tensorium_amd import build
    if not build.LIB.exists():
        build.build_hip()


@pytest.fixture(scope="session")
def ora():
    _ensure_oracle()
    from oracle import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def hiplib():
    _ensure_hip()
    from tensorium_amd import _abi
    return _abi.load()


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(ROOT / "tests" / "golden" / "golden.npz"))


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but torch.cuda.is_available() is False")
    return torch


@pytest.fixture(scope="session")
def hip(hiplib, torch_cuda):
    from tensorium_amd.nnhip import TNNHip
    h = TNNHip(0)
    yield h
    h.finish()
    h.close()
