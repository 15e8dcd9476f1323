import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def gpu_lib():
    """Loads libband_hip.so and asserts a gfx950 device is present (fails loudly)."""
    from band_amd import _abi, device
    lib = _abi.load()
    n = device.device_count()
    assert n > 0, "no HIP device visible"
    assert device.device_arch(0).startswith("gfx950"), device.device_arch(0)
    return lib
