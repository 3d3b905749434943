import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
# reproducible encryption randomness (encryption counters from 0, public-key masks from the secret key
# alone) so seeded keys reproduce the oracle's ciphertexts; inherited by the tools the tests start
os.environ.setdefault("FHESPEAR_PARITY_RNG", "1")
sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU; run with -m gpu")


# Oracle-comparing (limb-parity) files first, so a `-x` stop later in the GPU suite still leaves the
# core rows proven; the remaining files keep pytest's order.
_FIRST = ["test_gpu_parity.py", "test_golden_replay.py", "test_seal_mode.py", "test_full_size.py",
          "test_fri_ring.py", "test_bootstrap.py", "test_giant_shard.py"]


def pytest_collection_modifyitems(session, config, items):
    rank = {name: i for i, name in enumerate(_FIRST)}
    items.sort(key=lambda it: rank.get(Path(str(it.fspath)).name, len(_FIRST)))   # stable: in-file order kept


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
