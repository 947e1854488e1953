import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "yet-another-raytracer_amd"))
sys.path.insert(0, str(REPO / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libyart.so on the device)")


@pytest.fixture(scope="session")
def repo():
    return REPO


@pytest.fixture
def opt():
    """opt("world_bvh", 1): sets a library option (yart_debug_set_option, include/yart.h YART_OPT_*)
    for this test and restores every option it touched afterwards."""
    import yart
    saved = {}

    def set_(name, value):
        old = yart.set_option(name, value)
        saved.setdefault(name, old)

    yield set_
    for k, v in saved.items():
        yart.set_option(k, v)
