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
        saved.append((name, be.set_knob(name, int(value))))

    yield set_
    for name, old in reversed(saved):
        be.set_knob(name, old)
