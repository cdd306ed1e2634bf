"""GPU: the block store (gvs_oram_*, the mc-oblivious-traits ORAM::access
surface) bit-exact against the sequential oracle
(oracle/gvs_kv.c, test infrastructure): every block each op saw, and the whole
table read back through the same API at the end."""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import BlockStore, GvsError
from oracle import ffi

from test_kv_oracle import random_ops

pytestmark = pytest.mark.gpu

SECRET = bytes((0x33 + 7 * i) & 0xFF for i in range(32))


def read_all(store, model, cap, B):
    for lo in range(0, cap, B):
        ops = np.zeros(B, dtype=abi.BLOCK_OP_DTYPE)
        ops["index"] = np.arange(lo, lo + B)
        got, want = store.access(ops), model.access(ops)
        assert (got == want).all(), f"blocks [{lo}, {lo + B})"


def run(cap, B, batches, seed, auth=False, sizes=None, hot=None):
    store = BlockStore(abi.make_oram_config(cap, max_batch=B, secret_key=SECRET, auth_storage=auth))
    model = ffi.OramModel(cap)
    rng = np.random.default_rng(seed)
    try:
        for b in range(batches):
            n = sizes[b % len(sizes)] if sizes else B
            ops = random_ops(rng, n, cap, hot=hot if b % 2 else None)
            got, want = store.access(ops), model.access(ops)
            assert got.shape == want.shape
            bad = np.nonzero((got != want).any(1))[0]
            assert len(bad) == 0, f"batch {b}: {len(bad)} ops differ, first {bad[:5]}"
        read_all(store, model, cap, B)
    finally:
        store.close()
        model.close()


def test_oram_small_hot_and_partial_batches():
    # 300 hot blocks: many ops per block in one batch (chains of reads and writes)
    run(4096, 1024, 8, 11, sizes=[1024, 1000, 1, 0, 517], hot=300)


def test_oram_authenticated():
    run(4096, 1024, 6, 12, auth=True, hot=200)


def test_oram_single_block_chain():
    store = BlockStore(abi.make_oram_config(4096, max_batch=1024))
    model = ffi.OramModel(4096)
    rng = np.random.default_rng(13)
    for b in range(3):
        ops = random_ops(rng, 1024, 4096)
        ops["index"] = 77  # every op on one block: a 1024-long chain
        got, want = store.access(ops), model.access(ops)
        assert (got == want).all(), f"batch {b}"
    store.close()


def test_oram_invalid_batch_applies_nothing():
    cap = 4096
    store = BlockStore(abi.make_oram_config(cap, max_batch=1024))
    model = ffi.OramModel(cap)
    rng = np.random.default_rng(14)
    ops = random_ops(rng, 1024, cap)
    assert (store.access(ops) == model.access(ops)).all()
    bad = random_ops(rng, 1024, cap, p_write=1.0)
    bad[500]["index"] = cap
    with pytest.raises(GvsError) as ei:
        store.access(bad)
    assert ei.value.code == abi.GVS_ERR_INVALID_ARG
    bad[500]["index"] = 3
    bad[20]["op"] = 7
    with pytest.raises(GvsError):
        store.access(bad)
    read_all(store, model, cap, 1024)  # nothing was applied
    store.close()


def test_oram_c3_shape():
    """2^20 blocks, 64K-op batches (the message store's C3 batch): bit-exact."""
    run(1 << 20, 65536, 4, 15, hot=1 << 14)
