import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def gpu_available():
    import torch  # noqa: F401  (plumbing only: device presence)
    return torch.cuda.is_available()
