import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "mast3r-slam-ysh_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def knobs():
    """knobs(name, value): set a solver knob (m3s_set_knob) for this test;
    every knob set is restored at teardown."""
    import mast3r_slam_backends as be

    saved = []

    def set_(name, value):
        saved.append((be._lib, name, be.set_knob(name, int(value))))

    yield set_
    for lib, name, old in reversed(saved):  # on the library it was set on (see test_lib)
        lib.m3s_set_knob(name.encode(), int(old))


@pytest.fixture
def test_lib():
    """Run this test on the test build of the library (libm3s_gn_test.so:
    -DM3S_TEST_PATHS, the A/B reference solver paths and the bounded-wait
    hook); the product library is restored afterwards."""
    import mast3r_slam_backends as be

    prod = be._lib
    be._lib = be.load_test_library()
    yield be._lib
    be._lib = prod
