import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nzcb-circom_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def engine():
    import nzcb
    if nzcb.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible")
    e = nzcb.Engine(0, max_log_ntt=14, max_msm_points=1 << 14)
    yield e
    e.close()
