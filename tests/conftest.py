import os
import sys

# before the HIP runtime initialises in this process (see exo_amd/__init__.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.hookimpl(trylast=True)
def pytest_sessionstart(session):
    """A native SIGSEGV handler (tools/segv_trace.c, built by build()) ahead
    of faulthandler's, so a host crash inside the HIP runtime prints its frames
    as library+offset, then the Python stack (the r05
    capture_end faults left Python stacks only).  EXO_SEGV_TRACE=0: off."""
    so = os.path.join(REPO, "tools", "_segv_trace.so")
    if os.environ.get("EXO_SEGV_TRACE", "1") != "0" and os.path.exists(so):
        import ctypes
        try:
            ctypes.CDLL(so).segv_trace_install()
        except OSError:
            pass


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
