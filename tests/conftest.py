"""pytest configuration.

Markers: `gpu` -- needs a real MI355X (run with `-m gpu` on the GPU box); everything else runs
on the CPU-only build container.  The oracle (tests' checker) is built on demand.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    from pyoracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"))
    return load


@pytest.fixture(scope="session")
def ti():
    """The native library, on a GPU: fails loudly if the HIP build or the device is missing."""
    import turboinfer_amd as T
    if not os.path.exists(T.LIB_PATH):
        T.build()
    T.init(0)
    return T


@pytest.fixture(scope="session")
def ti_host():
    """The native library for its host-only entry points (no device bound): CPU tests."""
    import turboinfer_amd as T
    if not os.path.exists(T.LIB_PATH):
        T.build()
    T.lib()
    return T


def inp(seed: int, shape, scale: float = 1.0) -> np.ndarray:
    """Same seeded inputs as tests/golden/gen_golden.py."""
    return (np.random.RandomState(seed).standard_normal(shape) * scale).astype(np.float32)
