"""Test configuration: import paths, the ``gpu`` marker and fixture loaders.

``-m "not gpu"`` (CPU, the build container): oracle restatements against the
reference-generated fixtures in tests/golden/, host-side logic, library
load/exports, and the world_size-2 gloo sharding test.
``-m gpu`` (MI355X): parity of the HIP path through the C ABI.
"""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ska-sdp-func-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture
def load_golden():
    return golden


def rel_rms(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2)) / max(np.sqrt(np.mean(np.abs(b) ** 2)), 1e-300))
