"""gvstore: MI355X-native batched oblivious message store for grapevine's CRUD path.

The product is libgvstore.so (HIP/gfx950 kernels behind the C ABI of
include/gvstore.h); this package holds its ctypes mirror.
"""
from . import abi  # noqa: F401
from .store import ObliviousStore, GvsError, load_library  # noqa: F401

__version__ = "0.1.0"
