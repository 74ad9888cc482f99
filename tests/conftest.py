import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def golden():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session")
def ctx():
    """The engine context on cuda:0 -- GPU tests only; no fallback."""
    from lime_amd import Context
    c = Context(0)
    yield c
    c.close()
