import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import helpers  # noqa: E402,F401  (sets sys.path for lcv / oracle)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X and the HIP library liblcv.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_verifier():
    """The PRODUCT library on cuda:0 (fails loudly if liblcv.so or the GPU is missing).
    LCV_TEST_HOSTSIM=1 dry-runs the GPU tests on the host simulation (CPU development only)."""
    if os.environ.get("LCV_TEST_HOSTSIM") == "1":
        return helpers.hostsim_verifier()
    from lcv.device import Verifier
    return Verifier(0)


@pytest.fixture(scope="session")
def sim_verifier():
    """The host simulation of the same per-item kernel code (CPU-only tests)."""
    return helpers.hostsim_verifier()
