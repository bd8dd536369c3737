import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden_files(prefix="g"):
    return sorted(f for f in os.listdir(GOLDEN)
                  if f.startswith(prefix) and f.endswith(".npz")
                  and not f.startswith(("g7_", "g9_", "g10_", "g11_", "g12_", "g13_")))


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
