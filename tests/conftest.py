import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nanopore-barcoding-orc_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
# drop-in calls run in their own process unless a test asks for the resident server
os.environ.setdefault("DMX_DAEMON", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libdmx.so")


@pytest.fixture(scope="session")
def ctx():
    """One HIP context for the whole GPU session (tests run in one process)."""
    from dmx import lib
    c = lib.Context(0)
    yield c
    c.close()
