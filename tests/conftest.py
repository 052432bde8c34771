import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: long-running (large scenes)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the in-tree libraries once (no-op when up to date)."""
    from pnraytracing_amd import build
    build.build_host()
    if os.path.exists(build.HIPCC):
        build.build_device()
        build.build_diag_variants()
    build.build_oracle()
    yield
