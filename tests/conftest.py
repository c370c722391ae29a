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
