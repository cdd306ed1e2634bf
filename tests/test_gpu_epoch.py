"""GPU: the storage epoch limit of authenticated mode.

Every sealed row is bound to (row, epoch, table); a wrapped 32-bit epoch would
reuse AES-CTR keystream and let old rows verify again (gvs_crypto.h).  Every
batch entry point of every sealed store kind therefore refuses work with
GVS_ERR_EPOCH_EXHAUSTED once the epoch reaches the limit (2^32 - 256), before
any kernel runs: the message store, the block store and the key-value map
(the map's entry points lacked the check).  The epoch is set
through the test hook gvs_test_set_epoch (include/gvstore_test.h)."""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import BlockStore, GvsError, KeyValueMap, ObliviousStore
from oracle import ffi

from test_kv_oracle import SECRET, key_pool, random_map_ops

pytestmark = pytest.mark.gpu

LIMIT = 0xFFFFFF00


def refused(fn):
    with pytest.raises(GvsError) as ei:
        fn()
    assert ei.value.code == abi.GVS_ERR_EPOCH_EXHAUSTED


def test_message_store_refuses_at_epoch_limit():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024,
                          secret_key=SECRET, auth_storage=True)
    store, model = ObliviousStore(cfg), ffi.Model(cfg)
    try:
        model.seed(5)
        reqs = model.gen_batch(1024, ffi.gen_params(n_identities=100))
        store.process_batch(reqs)  # a batch below the limit runs
        store._check(store.lib.gvs_test_set_epoch(store.h, LIMIT))
        refused(lambda: store.process_batch(reqs))
    finally:
        store.close()
        model.close()


def test_block_store_refuses_at_epoch_limit():
    cfg = abi.make_oram_config(4096, max_batch=1024, secret_key=SECRET, auth_storage=True)
    store = BlockStore(cfg)
    try:
        ops = np.zeros(16, dtype=abi.BLOCK_OP_DTYPE)
        ops["index"] = np.arange(16)
        store.access(ops)
        store._check(store.lib.gvs_test_set_epoch(store._raw_handle(), LIMIT))
        refused(lambda: store.access(ops))
    finally:
        store.close()


def test_key_value_map_refuses_at_epoch_limit():
    cfg = abi.make_oram_config(4096, max_batch=1024, secret_key=SECRET, auth_storage=True)
    store = KeyValueMap(cfg)
    try:
        rng = np.random.default_rng(3)
        pool = key_pool(rng, 100)
        store.access(random_map_ops(rng, 256, pool))
        store._check(store.lib.gvs_test_set_epoch(store._raw_handle(), LIMIT))
        refused(lambda: store.access(random_map_ops(rng, 256, pool)))
        # the device-pointer entry point refuses before touching its arguments
        refused(lambda: store._check(store.lib.gvs_omap_access_batch_device(store.h, None, 0, None)))
        # one epoch below the limit still runs (the refusal is the limit, not the hook)
        store._check(store.lib.gvs_test_set_epoch(store._raw_handle(), LIMIT - 1))
        with pytest.raises(GvsError) as ei:  # rows were sealed at the real epoch: tags fail
            store.access(random_map_ops(rng, 256, pool))
        assert ei.value.code == abi.ERR_INTEGRITY
    finally:
        store.close()
