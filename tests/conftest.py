import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the tests drive libgvstore_test.so: the production engine plus the dump and
# raw-store hooks of include/gvstore_test.h (grapevine_amd/store.py)
os.environ.setdefault("GVS_TEST_HOOKS", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import ffi
    return ffi.lib()
