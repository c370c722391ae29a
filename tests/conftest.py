"""Shared fixtures.  `-m gpu` tests need a visible MI355X and call librps.so through the
C ABI; everything else runs on the CPU (oracle vs golden vectors, ABI symbol checks, gloo
multi-process sharding)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "rust-particle-system_amd", "python"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs librps.so kernels)")
    config.addinivalue_line("markers", "perf: wall-clock bound, not correctness; runs only with RPS_PERF_TESTS=1")


def pytest_collection_modifyitems(config, items):
    """Timing bounds depend on machine load: kept out of the correctness suite unless asked for."""
    if os.environ.get("RPS_PERF_TESTS") == "1":
        return
    skip = pytest.mark.skip(reason="perf bound: set RPS_PERF_TESTS=1 to run")
    for item in items:
        if "perf" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def rps():
    import rps_amd

    rps_amd.lib()  # raises if the HIP extension is missing: no fallback
    return rps_amd


@pytest.fixture(scope="session")
def orc():
    import oracle as orc_mod

    orc_mod.lib()
    return orc_mod


@pytest.fixture(scope="session")
def gpu(rps):
    if rps.device_count() < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return rps
