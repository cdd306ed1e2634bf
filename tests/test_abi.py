"""The C-ABI library loads and exports every entry point include/gvstore.h
declares; POD sizes agree between the header, ctypes and numpy.  No compute
calls (CPU container)."""
import ctypes
import os
import re

from grapevine_amd import abi
from grapevine_amd.store import EXPORTED, TEST_EXPORTED, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header="gvstore.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(gvs_\w+)\s*\(", src, flags=re.M)))


def test_every_declared_symbol_is_exported():
    decl = declared_functions()
    assert len(decl) >= 12
    assert set(decl) == set(EXPORTED)
    assert set(declared_functions("gvstore_test.h")) == set(TEST_EXPORTED)
    prod = load_library(os.path.join(ROOT, "grapevine_amd", "libgvstore.so"))
    test = load_library(os.path.join(ROOT, "grapevine_amd", "libgvstore_test.so"))
    for name in decl:
        assert hasattr(prod, name) and hasattr(test, name), name
    for name in TEST_EXPORTED:  # the production library has no test hooks
        assert hasattr(test, name), name
        assert not hasattr(prod, name), name


def test_library_contains_gfx950_code():
    for lib in ("libgvstore.so", "libgvstore_test.so"):
        path = os.path.join(ROOT, "grapevine_amd", lib)
        # the embedded HIP fat binary names its code object target
        assert b"amdgcn-amd-amdhsa--gfx950" in open(path, "rb").read()


def test_pod_sizes_match_header():
    hdr = open(os.path.join(ROOT, "include", "gvstore.h")).read()
    assert "GVS_PAYLOAD_BYTES 936" in hdr and "GVS_MAILBOX_SLOTS 62" in hdr
    assert abi.REQUEST_DTYPE.itemsize == 1040 and abi.RESPONSE_DTYPE.itemsize == 1040
    assert ctypes.sizeof(abi.GvsConfig) == 8 + 4 * 4 + 32 + 4 + 28
    assert ctypes.sizeof(abi.GvsStats) == 12 * 8


def test_config_init_and_version_without_gpu():
    lib = load_library()
    cfg = abi.GvsConfig()
    assert lib.gvs_config_init(ctypes.byref(cfg), 1 << 24) == 0
    assert cfg.msg_capacity == 1 << 24
    assert cfg.mailbox_partitions * cfg.mailbox_partition_slots == 1 << 20  # R = N/16
    assert cfg.max_batch == 65536
    assert lib.gvs_config_init(ctypes.byref(cfg), 1000) == abi.GVS_ERR_INVALID_ARG
    assert lib.gvs_version().startswith(b"gvstore")


def test_invalid_configs_rejected_before_device_use():
    lib = load_library()
    h = ctypes.c_void_p()
    bad = abi.make_config(4096, max_batch=100)  # not a power of two
    assert lib.gvs_create(ctypes.byref(bad), ctypes.byref(h)) == abi.GVS_ERR_INVALID_ARG
    bad = abi.make_config(4096, mailbox_partition_slots=2048)
    assert lib.gvs_create(ctypes.byref(bad), ctypes.byref(h)) == abi.GVS_ERR_INVALID_ARG


def test_invalid_sharded_configs_rejected_before_device_use():
    lib = load_library()
    h = ctypes.c_void_p()
    bad = abi.make_config(4096, max_batch=1024, shard_count=65)  # more than kShardsMax
    assert lib.gvs_create(ctypes.byref(bad), ctypes.byref(h)) == abi.GVS_ERR_INVALID_ARG
    bad = abi.make_config(4096, max_batch=1024, shard_count=2, route_capacity=2048)  # C > B
    assert lib.gvs_create(ctypes.byref(bad), ctypes.byref(h)) == abi.GVS_ERR_INVALID_ARG
    bad = abi.make_config(4096, max_batch=1024, rows_per_partition=100)
    assert lib.gvs_create(ctypes.byref(bad), ctypes.byref(h)) == abi.GVS_ERR_INVALID_ARG


def test_sealed_mailbox_partition_limit():
    """Sealed stores keep a mailbox partition's per-row values in the AES
    window's holes (gvs_mauth.h kSrAuth): more than 256 rows per partition is
    refused at create, before any device use; 256 passes validation (on a box
    without a GPU it then fails with GVS_ERR_NO_DEVICE)."""
    lib = load_library()
    h = ctypes.c_void_p()
    bad = abi.make_config(65536, mailbox_partitions=16, mailbox_partition_slots=512, max_batch=1024,
                          auth_storage=True)
    assert lib.gvs_create(ctypes.byref(bad), ctypes.byref(h)) == abi.GVS_ERR_INVALID_ARG
    plain = abi.make_config(65536, mailbox_partitions=16, mailbox_partition_slots=512, max_batch=1024)
    ok = abi.make_config(65536, mailbox_partitions=16, mailbox_partition_slots=256, max_batch=1024,
                         auth_storage=True)
    for cfg in (plain, ok):
        rc = lib.gvs_create(ctypes.byref(cfg), ctypes.byref(h))
        assert rc in (0, abi.GVS_ERR_NO_DEVICE), rc
        if rc == 0:
            lib.gvs_destroy(h)
