import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU oracle case")


def pytest_collection_modifyitems(config, items):
    # nothing is skipped silently: gpu tests fail loudly on a box without the HIP path
    pass


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
