"""GPU: the key-value map (gvs_omap_*, the mc-oblivious-traits
ObliviousHashMap surface) bit-exact against the sequential
oracle (oracle/gvs_kv.c, test infrastructure, pinned on CPU to a plain-Python
restatement in tests/test_kv_oracle.py): every op's status and value, and the
map's contents read back through the same API."""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import GvsError, KeyValueMap
from oracle import ffi

from test_kv_oracle import SECRET, key_pool, random_map_ops

pytestmark = pytest.mark.gpu


def make(cap, B):
    cfg = abi.make_oram_config(cap, max_batch=B, secret_key=SECRET)
    return KeyValueMap(cfg), ffi.OmapModel(cap, SECRET)


def same(got, want, where):
    bad = np.nonzero((got["status"] != want["status"]) | (got["value"] != want["value"]).any(1))[0]
    assert len(bad) == 0, f"{where}: {len(bad)} ops differ, first {bad[:5]}: " \
                          f"got {got['status'][bad[:5]]} want {want['status'][bad[:5]]}"


def read_back(store, model, pool, B):
    for lo in range(0, len(pool), B):
        keys = pool[lo:lo + B]
        ops = np.zeros(len(keys), dtype=abi.OMAP_OP_DTYPE)
        ops["key"] = keys
        ops["op"] = abi.OMAP_READ
        same(store.access(ops), model.access(ops), f"read-back [{lo}, {lo + len(keys)})")


def run(cap, B, batches, seed, nkeys, sizes=None, p_ops=(0.3, 0.3, 0.25, 0.15)):
    store, model = make(cap, B)
    rng = np.random.default_rng(seed)
    pool = key_pool(rng, nkeys)
    seen = set()
    try:
        for b in range(batches):
            n = sizes[b % len(sizes)] if sizes else B
            ops = random_map_ops(rng, n, pool, p_ops=p_ops)
            got, want = store.access(ops), model.access(ops)
            same(got, want, f"batch {b}")
            seen |= set(int(x) for x in want["status"])
        read_back(store, model, pool, B)
    finally:
        store.close()
        model.close()
    return seen


def test_map_mixed_hot_keys_and_partial_batches():
    seen = run(4096, 1024, 8, 31, 400, sizes=[1024, 1000, 1, 0, 333])
    assert {abi.OMAP_FOUND, abi.OMAP_NOT_FOUND, abi.OMAP_INVALID_KEY} <= seen, seen


def test_map_overflow_admission():
    # 16 partitions of 256 rows, 20000 keys: partitions fill, new keys
    # overflow (2048-op batches keep each partition's distinct keys per batch
    # within its 256 group slots)
    seen = run(4096, 2048, 8, 32, 20000, p_ops=(0.1, 0.4, 0.45, 0.05))
    assert abi.OMAP_OVERFLOW in seen, seen


def test_map_single_key_chain():
    store, model = make(4096, 1024)
    rng = np.random.default_rng(33)
    pool = key_pool(rng, 1)
    for b in range(3):
        ops = random_map_ops(rng, 1024, pool, p_invalid=0.0)
        same(store.access(ops), model.access(ops), f"batch {b}")
    store.close()


def test_map_unknown_op_applies_nothing():
    store, model = make(4096, 1024)
    rng = np.random.default_rng(34)
    pool = key_pool(rng, 300)
    ops = random_map_ops(rng, 1024, pool)
    same(store.access(ops), model.access(ops), "batch 0")
    bad = random_map_ops(rng, 1024, pool)
    bad[7]["op"] = 9
    with pytest.raises(GvsError) as ei:
        store.access(bad)
    assert ei.value.code == abi.GVS_ERR_INVALID_ARG
    read_back(store, model, pool, 1024)
    store.close()


def test_map_c3_shape():
    """2^20 rows, 64K-op batches over 2^17 keys: bit-exact."""
    run(1 << 20, 65536, 3, 35, 1 << 17)
