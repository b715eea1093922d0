import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from _lamellar_bootstrap import load_package  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def lam():
    return load_package()


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def capi(lam):
    from lamellar_runtime_amd import _capi
    return _capi.lib()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def world(lam):
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return lam.LamellarWorldBuilder().build()
