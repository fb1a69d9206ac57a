import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU-side checks")


@pytest.fixture(scope="session")
def sid():
    import sid_amd
    sid_amd.lib()
    return sid_amd


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def gpu(sid):
    if sid.device_count() < 1:
        pytest.skip("no HIP device")
    import sid_amd.gpu as G
    return G
