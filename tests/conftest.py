import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_collection_modifyitems(config, items):
    # A GPU test never silently passes on a machine without a GPU: it is
    # skipped only when deselected; when selected without a device it fails.
    pass


@pytest.fixture(scope="session")
def native_lib():
    from madrona_basketball_amd import build
    build.build()
    from madrona_basketball_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle.lib()
