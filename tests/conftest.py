"""Shared test setup: import paths, markers, build of the oracle and engine."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kube-batch-1_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def kbgen_mod():
    import kbgen
    return kbgen


@pytest.fixture(scope="session")
def engine():
    """The HIP engine; fails (does not skip) when the library or device is missing."""
    import kbhip
    if not os.path.exists(kbhip.LIB_PATH):
        kbhip.build()
    n = kbhip.device_count()
    assert n >= 1, "no gfx950 device visible to libkbhip.so"
    return kbhip


@pytest.fixture(scope="session")
def engine_lib():
    """libkbhip.so loaded through the binding (built if needed); no device required."""
    import kbhip
    if not os.path.exists(kbhip.LIB_PATH):
        kbhip.build()
    return kbhip.lib()
