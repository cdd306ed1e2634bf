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


# ---- sealed map (GVS_FLAG_AUTH_STORAGE): the value table is the block store's
# sealed table (k_rpass2<AUTH>); the key directory is sealed in
# 1-KiB rows of 32 entries (k_okey<true>: AES-CTR + BLAKE2b tag over the row,
# its index, the epoch and table 3), re-sealed by every batch.  Tamper, replay
# and swap of a directory row or its tag, or of a value row, fail the next
# batch with GVS_ERR_INTEGRITY and the handle stays dead.

def sealed_pair(seed, batches=3, cap=4096, B=1024, nkeys=600):
    cfg = abi.make_oram_config(cap, max_batch=B, secret_key=SECRET, auth_storage=True)
    store, model = KeyValueMap(cfg), ffi.OmapModel(cap, SECRET)
    rng = np.random.default_rng(seed)
    pool = key_pool(rng, nkeys)
    for b in range(batches):
        ops = random_map_ops(rng, B, pool)
        same(store.access(ops), model.access(ops), f"sealed batch {b}")
    return store, model, rng, pool


def expect_integrity(store, rng, pool, B=1024):
    for _ in range(2):  # the failing batch, then the dead handle
        with pytest.raises(GvsError) as ei:
            store.access(random_map_ops(rng, B, pool))
        assert ei.value.code == abi.ERR_INTEGRITY


def test_sealed_map_matches_the_oracle():
    """Sealed and plain maps give the same results over mixed batches, hot
    keys and partial batches, and the contents read back the same."""
    store, model, rng, pool = sealed_pair(70, batches=6)
    try:
        for n in (1000, 1, 0, 333):
            ops = random_map_ops(rng, n, pool)
            same(store.access(ops), model.access(ops), f"sealed partial {n}")
        read_back(store, model, pool, 1024)
    finally:
        store.close()
        model.close()


def test_sealed_map_staged_pass():
    """A 65536-row map (256-row partitions, 40 transaction slots): the value
    table's sealed pass stages every slot line in LDS (gvs_spass.h)."""
    store, model, rng, pool = sealed_pair(74, batches=5, cap=65536, nkeys=3000)
    try:
        for n in (1024, 7, 512):
            ops = random_map_ops(rng, n, pool)
            same(store.access(ops), model.access(ops), f"staged sealed {n}")
        read_back(store, model, pool, 1024)
    finally:
        store.close()
        model.close()


def test_sealed_map_directory_is_not_plaintext():
    """No stored key appears in the sealed directory's bytes."""
    store, model, rng, pool = sealed_pair(71)
    try:
        raw = store.dump_raw(abi.RAW_KEY_DIR, 0, 4096 * 32).tobytes()
        assert not any(bytes(k) in raw for k in pool[:200])
    finally:
        store.close()
        model.close()


@pytest.mark.parametrize("region,offset", [
    (abi.RAW_KEY_DIR, 37 * 1024 + 5),      # a directory row's ciphertext
    (abi.RAW_KEY_DIR_TAGS, 64 * 16 + 3),   # a directory row's tag
    (abi.RAW_MESSAGES, 1234 * 1024 + 17),  # a value row
])
def test_sealed_map_tamper_is_detected(region, offset):
    store, model, rng, pool = sealed_pair(72)
    try:
        b = store.dump_raw(region, offset, 1)
        store.store_raw(region, offset, bytes([int(b[0]) ^ 0x10]))
        expect_integrity(store, rng, pool)
    finally:
        store.close()
        model.close()


def test_sealed_map_replay_and_swap_are_detected():
    for kind in ("replay", "swap"):
        store, model, rng, pool = sealed_pair(73)
        try:
            if kind == "replay":  # a directory row and its tag from one batch earlier
                old = store.dump_raw(abi.RAW_KEY_DIR, 21 * 1024, 1024).tobytes()
                old_tag = store.dump_raw(abi.RAW_KEY_DIR_TAGS, 21 * 16, 16).tobytes()
                ops = random_map_ops(rng, 1024, pool)
                same(store.access(ops), model.access(ops), "before the replay")
                store.store_raw(abi.RAW_KEY_DIR, 21 * 1024, old)
                store.store_raw(abi.RAW_KEY_DIR_TAGS, 21 * 16, old_tag)
            else:  # two directory rows exchanged, tags with them
                rows = [store.dump_raw(abi.RAW_KEY_DIR, r * 1024, 1024).tobytes() for r in (8, 9)]
                tags = [store.dump_raw(abi.RAW_KEY_DIR_TAGS, r * 16, 16).tobytes() for r in (8, 9)]
                for r, k in ((8, 1), (9, 0)):
                    store.store_raw(abi.RAW_KEY_DIR, r * 1024, rows[k])
                    store.store_raw(abi.RAW_KEY_DIR_TAGS, r * 16, tags[k])
            expect_integrity(store, rng, pool)
        finally:
            store.close()
            model.close()


def test_sealed_map_rejects_oversized_partitions():
    """The sealed key pass holds the AES tables in LDS: at most 1024 rows and
    256 group slots per partition; larger shapes are refused."""
    cfg = abi.make_oram_config(1 << 23, max_batch=1024, secret_key=SECRET, auth_storage=True)
    with pytest.raises(GvsError) as ei:
        KeyValueMap(cfg)
    assert ei.value.code == abi.GVS_ERR_INVALID_ARG
