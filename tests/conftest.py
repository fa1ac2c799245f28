import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "passport-zk-circuits_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session", autouse=True)
def _torch_device_first(request):
    """When GPU tests are selected, torch's HIP runtime takes the device before libpzkwit's does
    (the order bench.py uses). With the native library first and worker pools forked in between
    (PassportGen key generation), torch's later lazy init found no device."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    yield
