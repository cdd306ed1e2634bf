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


# Whole-pipeline property tests (byte counters, kernel durations) run after
# every parity test: under `pytest -x` a failing property must not keep the
# oracle-parity evidence from being collected.  Inside each module the file's
# own order holds.
PROPERTY_MODULES = ("test_oblivious.py", "test_timing.py")


def _property_rank(item):
    name = os.path.basename(str(item.fspath))
    return PROPERTY_MODULES.index(name) + 1 if name in PROPERTY_MODULES else 0


@pytest.hookimpl(trylast=True)  # after -m deselection
def pytest_collection_modifyitems(config, items):
    items.sort(key=_property_rank)  # stable: file order kept inside each rank
    _torch_first(items)


def _torch_first(items):
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
