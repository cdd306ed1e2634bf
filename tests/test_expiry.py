"""Message expiry sweep (README.md:86-99).

The host supplies a cutoff; messages whose timestamp is older are recorded by
one batch's message pass (a fixed number per workgroup) and deleted by the
next batch's trailing expiry slots, as if their recipient had deleted them
(row, mailbox entry and slot freed), unless an UPDATE refreshed them since.

CPU tests exercise the oracle's restatement of that rule; GPU tests check the
HIP engine against it bit-exactly (responses, table bytes, counts) while the
cutoff moves.  The reference leaves expiry unimplemented in its MVP
(README.md:99), so this behaviour is "parity unpinned": it is pinned only to
the repo's own rule, which the oracle states.
"""
import numpy as np
import pytest

from grapevine_amd import abi
from oracle import ffi

from parity import diff_responses, diff_tables

TS0 = 1_700_000_000


def model(n_msgs=4096, Q=16, Sr=32, B=1024, X=128, **kw):
    cfg = abi.make_config(n_msgs, mailbox_partitions=Q, mailbox_partition_slots=Sr,
                          max_batch=B, expiry_per_batch=X, **kw)
    return cfg, ffi.Model(cfg)


def fill(m, n, batches=1, identities=64):
    for _ in range(batches):
        m.process_batch(m.gen_batch(n, ffi.gen_params(create=100, read=0, update=0, delete=0,
                                                      miss=0, bad_auth=0, bad_recipient=0,
                                                      hard_error=0, zero_recipient=0,
                                                      n_identities=identities)))


def empty(m):
    return m.process_batch(np.zeros(0, dtype=abi.REQUEST_DTYPE))


def test_config_rules():
    with pytest.raises(ValueError):
        model(X=300)            # not a power of two
    with pytest.raises(ValueError):
        model(B=1024, X=1024)   # more than half the batch
    with pytest.raises(ValueError):
        model(B=1024, X=256)    # 16 records per workgroup (W = 16): more than 8
    _, m = model(B=1024, X=128)
    with pytest.raises(ValueError):
        m.process_batch(np.zeros(1024 - 128 + 1, dtype=abi.REQUEST_DTYPE))  # n > B - X


def test_everything_old_expires_and_frees_mailboxes():
    _, m = model()
    fill(m, 768, batches=2)
    n0 = m.messages
    assert n0 > 1000 and m.mailboxes > 0
    m.set_expiry_cutoff(TS0 + 10**6)  # everything is older
    counts = []
    for _ in range(24):
        empty(m)
        counts.append(m.messages)
    # W = 16 partitions x 8 records per batch: one sweep (batch 0) then
    # 128 deletes per batch from batch 1 on
    assert counts[0] == n0
    assert counts[1] == n0 - 128
    assert counts[-1] == 0 and m.mailboxes == 0, counts


def test_no_cutoff_no_expiry():
    _, m = model()
    fill(m, 768)
    n0 = m.messages
    for _ in range(3):
        empty(m)
    assert m.messages == n0
    m.set_expiry_cutoff(TS0)  # older than every message: still nothing
    for _ in range(3):
        empty(m)
    assert m.messages == n0


def test_only_older_messages_expire():
    _, m = model()
    fill(m, 768)       # ops 0..767
    fill(m, 768)       # ops 768..1535
    m.set_expiry_cutoff(TS0 + 768)
    for _ in range(8):
        empty(m)
    recs = m.dump_messages()
    live = recs[recs["msg_id"].any(axis=1)]
    assert len(live) > 0
    assert (live["timestamp"] >= TS0 + 768).all()
    assert m.messages == len(live)


def test_update_after_sweep_keeps_message():
    """A message swept for expiry but UPDATEd before its delete runs survives;
    only messages that were not refreshed are deleted."""
    cfg, m = model()
    fill(m, 768)
    m.set_expiry_cutoff(TS0 + 10**6)
    empty(m)  # batch 0: the sweep records 8 messages per partition (128)
    recs = m.dump_messages()
    live = recs[recs["msg_id"].any(axis=1)]
    # refresh every other live message; the recorded deletes run after the
    # updates in the next batch (by-id class, last slots)
    upd = live[::2]
    reqs = np.zeros(len(upd), dtype=abi.REQUEST_DTYPE)
    reqs["msg_id"] = upd["msg_id"]
    reqs["auth_identity"] = upd["sender"]
    reqs["recipient"] = upd["recipient"]
    reqs["timestamp"] = TS0 + 2 * 10**6
    reqs["request_type"] = abi.REQUEST_TYPE_UPDATE
    out = m.process_batch(reqs)
    assert (out["status_code"] == 1).all()
    after = m.dump_messages()
    alive = {bytes(r["msg_id"]) for r in after if r["msg_id"].any()}
    updated = {bytes(r["msg_id"]) for r in upd}
    gone = {bytes(r["msg_id"]) for r in live} - alive
    assert updated <= alive                 # every refreshed message survived
    assert gone and not (gone & updated)    # only unrefreshed ones were deleted
    assert len(gone) <= 128
    # exactly the swept ones: the first 8 live rows of each of the 16
    # partitions (slot s lives in partition s mod 16 at offset s div 16; the
    # dump is in slot order), minus the refreshed ones
    swept = set()
    for w in range(16):
        part = recs[w::16]
        swept |= {bytes(r["msg_id"]) for r in part[part["msg_id"].any(axis=1)][:8]}
    assert len(swept) == 128 and gone == swept - updated


def test_rotating_workgroups_when_X_below_W():
    # N = 2^16: 256 partitions of 256 rows; X = 64 -> one record per
    # partition, a quarter of the partitions per batch
    _, m = model(n_msgs=1 << 16, Q=64, Sr=64, B=1024, X=64)
    fill(m, 960, batches=3)
    n0 = m.messages
    m.set_expiry_cutoff(TS0 + 10**7)
    empty(m)
    seen = []
    for _ in range(8):
        empty(m)
        seen.append(n0 - m.messages)
        n0 = m.messages
    assert all(0 < d <= 64 for d in seen), seen


@pytest.mark.gpu
@pytest.mark.parametrize("n_msgs,Q,Sr,X,auth", [
    (4096, 16, 32, 128, False),      # X >= W: 8 records per workgroup
    (1 << 16, 64, 64, 64, False),    # X < W: one record, rotating workgroups
    (4096, 16, 32, 64, True),        # authenticated storage, 4 records per workgroup
])
def test_gpu_expiry_parity(n_msgs, Q, Sr, X, auth):
    from grapevine_amd.store import ObliviousStore
    B = 1024
    cfg = abi.make_config(n_msgs, mailbox_partitions=Q, mailbox_partition_slots=Sr, max_batch=B,
                          expiry_per_batch=X, auth_storage=auth)
    store, m = ObliviousStore(cfg), ffi.Model(cfg)
    m.seed(41)
    n = B - X
    params = ffi.gen_params(create=40, read=20, update=20, delete=20, n_identities=200)
    expired = 0
    for b in range(14):
        # messages untouched for ~1.5 batches of ops expire
        cutoff = TS0 + max(0, m.ops - int(1.5 * n)) if b >= 2 else 0
        m.set_expiry_cutoff(cutoff)
        store.set_expiry_cutoff(cutoff)
        before = m.messages
        reqs = m.gen_batch(n, params)
        want = m.process_batch(reqs)
        got = store.process_batch(reqs)
        d = diff_responses(got, want, reqs)
        assert not d, f"batch {b}: " + "\n".join(d)
        st = store.stats()
        assert st["messages"] == m.messages, (b, st["messages"], m.messages)
        assert st["mailboxes"] == m.mailboxes, (b, st["mailboxes"], m.mailboxes)
        creates = int(((reqs["request_type"] == 1) & (want["status_code"] == 1)).sum())
        deletes = int(((reqs["request_type"] == 4) & (want["status_code"] == 1)).sum())
        expired += before + creates - deletes - m.messages
    dt = diff_tables(store.dump_messages(), m.dump_messages())
    assert not dt, "\n".join(dt)
    assert expired > 0


def cluster(S=2, n_msgs=4096, Q=16, Sr=32, B=1024, X=128, C=0):
    cfg = abi.make_config(n_msgs, mailbox_partitions=Q, mailbox_partition_slots=Sr, max_batch=B,
                          expiry_per_batch=X, shard_count=S, route_capacity=C)
    return cfg, ffi.Cluster(cfg)


def test_sharded_expiry_every_shard_sweeps_its_own_table():
    """Sharded stores: each shard's pipeline carries its own X expiry slots
    after the S*C routed ones, so callers still submit S*B requests."""
    S, B, X = 2, 1024, 128
    cfg, cl = cluster(S=S, B=B, X=X)
    assert ffi.shard_batch(S * cl.capacity + X) >= S * cl.capacity + X
    cl.seed(5)
    fill_p = ffi.gen_params(create=100, read=0, update=0, delete=0, miss=0, bad_auth=0,
                            bad_recipient=0, hard_error=0, zero_recipient=0, n_identities=128)
    for _ in range(2):
        assert cl.process_batch(cl.gen_batch(S * B, fill_p)) is not None
    n0 = cl.messages
    per_shard0 = [cl.shard(k).messages for k in range(S)]
    assert min(per_shard0) > 200
    cl.set_expiry_cutoff(TS0 + 10**7)
    for _ in range(3):
        assert cl.process_batch(np.zeros(0, dtype=abi.REQUEST_DTYPE)) is not None
    # one sweep, then X deletes per shard and batch (W = 16 x 8 records)
    assert n0 - cl.messages == 2 * S * X
    assert all(per_shard0[k] - cl.shard(k).messages == 2 * X for k in range(S))


def test_shard_batch_rule():
    # the smaller of the next power of two and the next multiple of 8192
    assert ffi.shard_batch(1536) == 2048
    assert ffi.shard_batch(5376) == 8192
    assert ffi.shard_batch(72192) == 73728      # C3 routed 8 ways: not 131072
    assert ffi.shard_batch(18048) == 24576
    assert ffi.shard_batch(100) == 1024


@pytest.mark.gpu
@pytest.mark.parametrize("S,B,X", [(2, 1024, 128), (4, 1024, 64)])
def test_gpu_sharded_expiry_parity(S, B, X):
    from grapevine_amd.store import ObliviousStore
    cfg, cl = cluster(S=S, B=B, X=X)
    store = ObliviousStore(cfg)
    assert store.stats()["shard_batch"] == ffi.shard_batch(S * cl.capacity + X)
    cl.seed(43 + S)
    n = S * B
    params = ffi.gen_params(create=40, read=20, update=20, delete=20, n_identities=300)
    expired = 0
    for b in range(12):
        cutoff = TS0 + max(0, cl.ops - int(1.5 * n)) if b >= 2 else 0
        cl.set_expiry_cutoff(cutoff)
        store.set_expiry_cutoff(cutoff)
        before = cl.messages
        reqs = cl.gen_batch(n, params)
        want = cl.process_batch(reqs)
        got = store.process_batch(reqs)
        d = diff_responses(got, want, reqs)
        assert not d, f"batch {b}: " + "\n".join(d)
        st = store.stats()
        assert (st["messages"], st["mailboxes"]) == (cl.messages, cl.mailboxes), b
        creates = int(((reqs["request_type"] == 1) & (want["status_code"] == 1)).sum())
        deletes = int(((reqs["request_type"] == 4) & (want["status_code"] == 1)).sum())
        expired += before + creates - deletes - cl.messages
    dt = diff_tables(store.dump_messages(), cl.dump_messages())
    assert not dt, "\n".join(dt)
    assert expired > 0


def test_expiry_deletes_must_fit_group_slots():
    """with few mailbox partitions the group slots are capped
    (kGroupMax), and X expiry deletes could overflow a partition on their own;
    every later batch would then fail with its records.  gvs_create refuses
    such a configuration before touching the device."""
    import ctypes
    from grapevine_amd.store import load_library
    lib = load_library()
    ok_codes = (abi.GVS_OK, abi.GVS_ERR_NO_DEVICE)

    def create(**kw):
        cfg = abi.make_config(8192, mailbox_partition_slots=256, max_batch=4096, **kw)
        h = ctypes.c_void_p()
        rc = lib.gvs_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc == 0:
            lib.gvs_destroy(h)
        return rc

    assert create(mailbox_partitions=2, expiry_per_batch=1024) == abi.GVS_ERR_INVALID_ARG
    assert create(mailbox_partitions=2, expiry_per_batch=256) in ok_codes
    assert create(mailbox_partitions=2, expiry_per_batch=0) in ok_codes
