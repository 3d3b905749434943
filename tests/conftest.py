import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU; run with -m gpu")


def gpu_available():
    try:
        import pyPhantom as ph
        return ph.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device / libfhespear_hip.so is available")


@pytest.fixture(scope="module")
def orc():
    """The CPU parity oracle (oracle/ckks_oracle.c via oracle/oracle.py), built in-tree."""
    from oracle import oracle
    oracle.build()
    return oracle
