import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dlrm-yx_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: multi-process or long-running CPU test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        have_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def fp32_close(a, b, rtol=1e-5, atol=1e-5):
    """The north-star tolerance: |a - b| <= 1e-5 * max(1, |ref|)."""
    import numpy as np
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    tol = atol * np.maximum(1.0, np.abs(b))
    bad = np.abs(a - b) > tol
    if bad.any():
        i = np.unravel_index(np.argmax(np.abs(a - b) - tol), a.shape)
        return False, f"max excess at {i}: got {a[i]!r} ref {b[i]!r} ({bad.sum()} bad)"
    return True, ""


@pytest.fixture
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load
