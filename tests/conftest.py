import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP kernels")


@pytest.fixture(scope="session")
def lib():
    from koordinator_amd import abi
    return abi.load_library()


@pytest.fixture(scope="session")
def gpu(lib):
    """The HIP path must be the one that runs: on a GPU box a missing device is a failure."""
    assert lib.ke_device_available() == 1, "no HIP device visible: GPU tests cannot run on the CPU"
    return lib
