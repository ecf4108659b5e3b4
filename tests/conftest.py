import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dct-carver_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def ctx():
    """One dctenergy context for the GPU tests (fails loudly if the HIP
    library or the device is missing -- there is no CPU fallback)."""
    import dctenergy
    c = dctenergy.Context(ngpus=1)
    yield c
    c.close()
