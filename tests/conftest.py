import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dune-eigensolver_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP path")


@pytest.fixture(scope="session")
def ctx():
    import eigmi
    c = eigmi.Context(0)  # raises (no fallback) when no device is visible
    yield c
    c.close()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
