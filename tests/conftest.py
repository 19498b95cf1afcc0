import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def block_fixtures():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "block_*.npz")))


def rel_to_max(a, b):
    """max|a-b| / max|b|  (the tolerance measure used throughout)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    denom = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / denom)


@pytest.fixture(scope="session")
def pkg():
    from stgcn_loader import load
    return load()
