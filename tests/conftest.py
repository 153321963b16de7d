import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfgv.so on cuda:0)")


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on device 0.  No skip: a gpu test without the library or GPU fails."""
    from fabric_amd import _lib
    eng = _lib.Engine(0)
    yield eng
    eng.close()
