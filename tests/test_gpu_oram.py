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


# ---- sealed block store (GVS_FLAG_AUTH_STORAGE): the message table's XMACC
# format and k_rpass2<AUTH>; tamper, replay and swap of a
# block row, its tag or a pending final state fail the next batch with
# GVS_ERR_INTEGRITY and the handle stays dead.

def sealed_pair(seed, batches=2, cap=4096, B=1024):
    store = BlockStore(abi.make_oram_config(cap, max_batch=B, secret_key=SECRET, auth_storage=True))
    model = ffi.OramModel(cap)
    rng = np.random.default_rng(seed)
    for _ in range(batches):
        ops = random_ops(rng, B, cap, hot=200)
        assert (store.access(ops) == model.access(ops)).all()
    return store, model, rng


def expect_integrity(store, rng, cap=4096, B=1024):
    for _ in range(2):  # the failing batch, then the dead handle
        with pytest.raises(GvsError) as ei:
            store.access(random_ops(rng, B, cap))
        assert ei.value.code == abi.ERR_INTEGRITY


@pytest.mark.parametrize("region,offset", [
    (abi.RAW_MESSAGES, 1234 * 1024 + 17),  # a block row's ciphertext
    (abi.RAW_MSG_TAGS, 345 * 16 + 9),      # a block row's tag
    (abi.RAW_PENDING, 100 * 1024 + 3),     # a pending final state
    (abi.RAW_PENDING_SIDE, 40 * 128 + 1),  # its side entry (target row)
    (abi.RAW_PENDING_TAGS, 700 * 16),      # its tag
])
def test_sealed_block_tamper_is_detected(region, offset):
    store, model, rng = sealed_pair(60)
    try:
        b = store.dump_raw(region, offset, 1)
        store.store_raw(region, offset, bytes([int(b[0]) ^ 0x04]))
        expect_integrity(store, rng)
    finally:
        store.close()
        model.close()


def test_sealed_block_replay_and_swap_are_detected():
    for kind in ("replay", "swap"):
        store, model, rng = sealed_pair(61)
        try:
            if kind == "replay":
                old = store.dump_raw(abi.RAW_MESSAGES, 77 * 1024, 1024).tobytes()
                old_tag = store.dump_raw(abi.RAW_MSG_TAGS, 77 * 16, 16).tobytes()
                ops = random_ops(rng, 1024, 4096)
                assert (store.access(ops) == model.access(ops)).all()  # every row re-sealed
                store.store_raw(abi.RAW_MESSAGES, 77 * 1024, old)
                store.store_raw(abi.RAW_MSG_TAGS, 77 * 16, old_tag)
            else:
                rows = [store.dump_raw(abi.RAW_MESSAGES, r * 1024, 1024).tobytes() for r in (10, 11)]
                tags = [store.dump_raw(abi.RAW_MSG_TAGS, r * 16, 16).tobytes() for r in (10, 11)]
                for r, k in ((10, 1), (11, 0)):
                    store.store_raw(abi.RAW_MESSAGES, r * 1024, rows[k])
                    store.store_raw(abi.RAW_MSG_TAGS, r * 16, tags[k])
            expect_integrity(store, rng)
        finally:
            store.close()
            model.close()


def test_sealed_block_store_staged_pass():
    """65536 blocks in 256-row partitions: 40 transaction slots, so the sealed
    pass stages every slot line in LDS (gvs_spass.h); hot and uniform batches
    bit-exact, then every block read back, then a tampered row detected."""
    cap, B = 65536, 1024
    store, model, rng = sealed_pair(63, batches=4, cap=cap, B=B)
    try:
        for _ in range(3):
            ops = random_ops(rng, B, cap, hot=64)
            assert (store.access(ops) == model.access(ops)).all()
        read_all(store, model, cap, B)
        b = store.dump_raw(abi.RAW_MESSAGES, 4321 * 1024 + 100, 1)
        store.store_raw(abi.RAW_MESSAGES, 4321 * 1024 + 100, bytes([int(b[0]) ^ 0x01]))
        expect_integrity(store, rng, cap=cap, B=B)
    finally:
        store.close()
        model.close()


def test_sealed_block_rows_are_the_storage_format():
    """Rows that the last batch did not touch hold the message table's format
    (table 0) at the epoch = batches applied: the oracle's seal of the model's
    block gives the stored ciphertext and tag byte for byte."""
    cap, B, batches = 4096, 1024, 3
    store, model, rng = sealed_pair(62, batches=batches)
    try:
        side = store.dump_raw(abi.RAW_PENDING_SIDE, 0, B * 128).reshape(B, 128)
        # side entries are sealed; a row the batch touched is pending (table 0x100): skip
        # rows that appear in the last batch's ops by comparing against both formats
        W = cap // 256  # 256-row partitions at this size
        checked = 0
        for index in (0, 1, 5, 999, 2048, cap - 1):
            row = (index % W) * 256 + index // W
            ct = store.dump_raw(abi.RAW_MESSAGES, row * 1024, 1024).tobytes()
            tag = store.dump_raw(abi.RAW_MSG_TAGS, row * 16, 16).tobytes()
            ops = np.zeros(1, dtype=abi.BLOCK_OP_DTYPE)
            ops["index"] = index
            pt = model.access(ops)[0].tobytes()
            c0, _, t0 = ffi.seal_row(SECRET, 0, row, batches, pt)
            if (ct, tag) == (c0, t0):
                checked += 1
        assert checked >= 3, checked
        del side
    finally:
        store.close()
        model.close()
