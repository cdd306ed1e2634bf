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


@pytest.hookimpl(trylast=True)  # after -m deselection
def pytest_collection_modifyitems(config, items):
    """GPU sessions start torch's HIP runtime before libgvstore's.  torch
    bundles its own libamdhip64; when the engine's runtime (/opt/rocm) has
    opened the device first, torch's finds no device ("No HIP GPUs are
    available") and the tests that hand the engine torch tensors fail, while
    the other order works.  CPU sessions do not import torch here."""
    if not any(it.get_closest_marker("gpu") for it in items):
        return
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
