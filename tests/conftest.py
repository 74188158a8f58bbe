import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import helpers  # noqa: E402,F401  (sets sys.path for lcv / oracle)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X and the HIP library liblcv.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "no_sop: the test's calls run no SOP program (engine_verifier checks less)")


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


@pytest.fixture(params=["fan", "batch"])
def engine_verifier(request, gpu_verifier):
    """gpu_verifier with every call of the test on ONE engine: "fan" = latency mode 64, lcv_init's default for
    <= 64-row batches (fan-engine SOP programs, the fused Miller program, one-item-per-wave SSWU / signature
    twins); "batch" = latency mode 0, the batch engine bench.py measures (one op per lane, 64 / TEAM items per
    wave, one lane per SSWU map / signature).  Afterwards the device's engine log (lcv_debug_engine_log) must
    show that the chosen engine took every launch and the other none."""
    v = gpu_verifier
    prev = v.latency_mode
    v.set_latency_mode(64 if request.param == "fan" else 0)
    v.engine_log(reset=True)
    try:
        yield v
        log = v.engine_log(reset=True)
        mine, other = (("fan", "twin"), ("batch", "lane")) if request.param == "fan" else (("batch", "lane"), ("fan", "twin"))
        assert log[other[0]] == 0 and log[other[1]] == 0, log
        if request.node.get_closest_marker("no_sop") is None:
            assert log[mine[0]] > 0, log
    finally:
        v.set_latency_mode(prev)
