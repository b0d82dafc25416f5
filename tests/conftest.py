import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ctypes

    oracle_ctypes.lib()
    return oracle_ctypes


@pytest.fixture(scope="session")
def device():
    import raytracingtherestofyourlife_amd as rtp

    dev = rtp.Device(0)
    yield dev
    dev.close()
