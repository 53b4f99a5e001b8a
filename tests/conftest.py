import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libdamvs.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def bn_from_golden(g, prefix="bn::"):
    return {k[len(prefix):]: g[k] for k in g.files if k.startswith(prefix)}


def rel_max(a, b):
    """max |a-b| / max |b| (float64)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def pixel_rel(a, b):
    """per-pixel |a-b| / |b| (float64)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-12)


@pytest.fixture(scope="session")
def golden_loader():
    return golden
