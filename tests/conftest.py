import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "image-processing-suite_amd")
for p in (PKG_ROOT, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libcpx on a HIP device)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def dev():
    """One libcpx Device for the whole GPU session (a single process drives the card)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpx.device import Device
    d = Device(0)
    yield d
    d.close()
