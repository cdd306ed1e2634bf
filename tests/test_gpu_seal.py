"""GPU: the authenticated-storage mode (GVS_FLAG_AUTH_STORAGE).

* Responses, live counts and the (host-unsealed) message table stay bit-exact
  with the oracle, which knows nothing about sealing: sealing must not change
  what the store computes.
* What sits in HBM is exactly the format of oracle/gvs_seal.c: every raw
  message row, mailbox row, side entry and tag equals the oracle's sealing of
  the plaintext at the store's current epoch.
* Tampering with any stored byte, tag or side entry, or replaying an older
  sealed row, fails the next batch with GVS_ERR_INTEGRITY, and the handle then
  refuses further work.
"""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import GvsError, ObliviousStore
from oracle import ffi

from parity import run_stream

pytestmark = pytest.mark.gpu

SECRET = bytes((0x67 + 31 * i) & 0xFF for i in range(32))


def make_pair(n_msgs=4096, Q=16, Sr=32, B=1024, rpp=0):
    """The sealed message pass (gvs_spass.h k_spass) stages a partition's slot
    lines in LDS when it has at most 64 transaction slots: with 1024-request
    batches that needs 64 partitions or more (n_msgs = 65536 and rpp <= 1024
    here, the staged pass; 12 waves per workgroup from 1024-row partitions).
    The small default tables (4096 messages, 16 partitions of 256 rows, 144
    slots) run the fallback that keeps slot lines in HBM."""
    cfg = abi.make_config(n_msgs, mailbox_partitions=Q, mailbox_partition_slots=Sr,
                          max_batch=B, secret_key=SECRET, auth_storage=True, rows_per_partition=rpp)
    return ObliviousStore(cfg), ffi.Model(cfg)


def physical_row(st, slot):
    W, S = st["msg_partitions"], st["msg_partition_slots"]
    return (slot % W) * S + slot // W


def unseal(table, row, epoch, ct, side_ct=None):
    """Decrypt with the oracle's keystream (the sealing of a zero row)."""
    z = ffi.seal_row(SECRET, table, row, epoch, bytes(1024), bytes(16) if side_ct is not None else None)
    pt = bytes(np.frombuffer(ct, np.uint8) ^ np.frombuffer(z[0], np.uint8))
    spt = bytes(np.frombuffer(side_ct, np.uint8) ^ np.frombuffer(z[1], np.uint8)) if side_ct is not None else None
    return pt, spt


STAGED = dict(n_msgs=65536, rpp=256)  # the staged pass, 8 waves


@pytest.mark.parametrize("n_msgs,rpp,waves", [(4096, 0, 8), (4096, 512, 4), (65536, 256, 8), (65536, 512, 4),
                                              (65536, 1024, 12), (65536, 1024, 0)])
def test_auth_mode_parity_stream(n_msgs, rpp, waves):
    store, model = make_pair(n_msgs=n_msgs, rpp=rpp)
    store.set_option("sealed_pass_waves", waves)
    model.seed(31)
    seen = run_stream(store, model, ffi.gen_params(n_identities=300), batches=8, n=1024)
    assert {0, 1, 2} <= set(seen), seen
    assert store.stats()["epoch"] == 8


def test_auth_mode_hot_recipient_and_capacity():
    store, model = make_pair(n_msgs=512, Q=4, Sr=16, B=1024)
    model.seed(32)
    seen = run_stream(store, model, ffi.gen_params(create=60, read=15, update=10, delete=15,
                                                   hot=40, n_identities=60), batches=6, n=1024)
    assert seen[5] > 0 and seen[7] > 0, seen


def pending_states(store, ep):
    """The final states the last batch left pending: {physical row: (position,
    plaintext)}, each checked against the oracle format of table 2 (a P entry,
    bound to its position and, through its side entry, to its target row)."""
    B = store.config.max_batch
    P = store.dump_raw(abi.RAW_PENDING, 0, B * 1024).reshape(B, 1024)
    side = store.dump_raw(abi.RAW_PENDING_SIDE, 0, B * 128).reshape(B, 128)[:, :16]
    tags = store.dump_raw(abi.RAW_PENDING_TAGS, 0, B * 16).reshape(B, 16)
    out = {}
    for p in range(B):
        pt, spt = unseal(abi.TABLE_PENDING_STATE, p, ep, P[p].tobytes(), side[p].tobytes())
        want = ffi.seal_row(SECRET, abi.TABLE_PENDING_STATE, p, ep, pt, spt)
        assert (P[p].tobytes(), side[p].tobytes(), tags[p].tobytes()) == want, f"P position {p}"
        row, valid = int.from_bytes(spt[:8], "little"), spt[8] & 1
        if valid:
            assert row not in out, f"two final states for row {row}"
            out[row] = (p, pt)
    return out


@pytest.mark.parametrize("n_msgs,rpp", [(4096, 0), (4096, 512), (65536, 256)])
def test_stored_bytes_are_the_oracle_format(n_msgs, rpp):
    store, model = make_pair(n_msgs=n_msgs, rpp=rpp)
    model.seed(33)
    run_stream(store, model, ffi.gen_params(n_identities=200), batches=3, n=1024)
    st = store.stats()
    ep = st["epoch"]
    N = store.config.msg_capacity
    want_tab = model.dump_messages()
    raw = store.dump_raw(abi.RAW_MESSAGES, 0, N * 1024).reshape(N, 1024)
    tags = store.dump_raw(abi.RAW_MSG_TAGS, 0, N * 16).reshape(N, 16)
    pend = pending_states(store, ep)
    assert 0 < len(pend) <= 1024
    rng = np.random.default_rng(0)
    live = [s for s in range(N) if want_tab[s]["msg_id"].any()]
    slots = sorted(set(rng.choice(live, 24, replace=False).tolist()) | {0, N - 1}
                   | {s for s in range(N) if physical_row(st, s) in pend})
    n_pend = 0
    for s in slots:
        r = physical_row(st, s)
        if r in pend:
            # the row holds its state before the last batch, sealed as pending;
            # its final state is the P entry
            n_pend += 1
            assert pend[r][1] == want_tab[s:s + 1].tobytes(), f"slot {s}: pending final state"
            pt, _ = unseal(0, r, ep, raw[r].tobytes())
            ct, _, tag = ffi.seal_row(SECRET, abi.TABLE_PENDING_ROW, r, ep, pt)
        else:
            ct, _, tag = ffi.seal_row(SECRET, 0, r, ep, want_tab[s:s + 1].tobytes())
        assert raw[r].tobytes() == ct, f"slot {s} row {r}: ciphertext differs"
        assert tags[r].tobytes() == tag, f"slot {s} row {r}: tag differs"
    assert n_pend == len(pend)
    # mailbox rows: decrypt, re-seal with the oracle, compare bytes and tag
    R = store.config.mailbox_partitions * store.config.mailbox_partition_slots
    mb = store.dump_raw(abi.RAW_MAILBOXES, 0, R * 1024).reshape(R, 1024)
    side = store.dump_raw(abi.RAW_SIDE, 0, R * 16).reshape(R, 16)
    btag = store.dump_raw(abi.RAW_MBOX_TAGS, 0, R * 16).reshape(R, 16)
    occupied = 0
    for r in range(R):
        pt, spt = unseal(1, r, ep, mb[r].tobytes(), side[r].tobytes())
        occupied += spt[8] & 1
        ct, sct, tag = ffi.seal_row(SECRET, 1, r, ep, pt, spt)
        assert (mb[r].tobytes(), side[r].tobytes(), btag[r].tobytes()) == (ct, sct, tag), f"mailbox row {r}"
    assert occupied == model.mailboxes


def run_one(store, model, params, n=1024):
    reqs = model.gen_batch(n, params)
    return store.process_batch(reqs), model.process_batch(reqs)


@pytest.mark.parametrize("region,offset", [
    (abi.RAW_MESSAGES, 5 * 1024 + 700),   # a byte of a message row
    (abi.RAW_MSG_TAGS, 77 * 16 + 3),      # a message tag
    (abi.RAW_MAILBOXES, 9 * 1024 + 40),   # a mailbox row
    (abi.RAW_SIDE, 3 * 16 + 1),           # a mailbox side entry
    (abi.RAW_MBOX_TAGS, 200 * 16 + 15),   # a mailbox tag
    (abi.RAW_PENDING, 300 * 1024 + 5),    # a pending final state
    (abi.RAW_PENDING_SIDE, 17 * 128 + 2),  # its side entry (target row)
    (abi.RAW_PENDING_SIDE, 17 * 128 + 12),  # its side entry (the slot its state goes to)
    (abi.RAW_PENDING_TAGS, 900 * 16),     # its tag
])
@pytest.mark.parametrize("staged", [False, True])
def test_tamper_is_detected(region, offset, staged):
    store, model = make_pair(**(STAGED if staged else {}))
    model.seed(34)
    params = ffi.gen_params(n_identities=200)
    run_stream(store, model, params, batches=2, n=1024)
    b = store.dump_raw(region, offset, 1)
    store.store_raw(region, offset, bytes([int(b[0]) ^ 0x10]))
    with pytest.raises(GvsError) as ei:
        run_one(store, model, params)
    assert ei.value.code == abi.ERR_INTEGRITY
    with pytest.raises(GvsError) as ei:  # the handle stays dead
        run_one(store, model, params)
    assert ei.value.code == abi.ERR_INTEGRITY


@pytest.mark.parametrize("staged", [False, True])
def test_replayed_row_is_detected(staged):
    store, model = make_pair(**(STAGED if staged else {}))
    model.seed(35)
    params = ffi.gen_params(n_identities=200)
    run_stream(store, model, params, batches=2, n=1024)
    row = 123
    old = store.dump_raw(abi.RAW_MESSAGES, row * 1024, 1024).tobytes()
    old_tag = store.dump_raw(abi.RAW_MSG_TAGS, row * 16, 16).tobytes()
    run_stream(store, model, params, batches=1, n=1024)  # every row re-sealed at a new epoch
    store.store_raw(abi.RAW_MESSAGES, row * 1024, old)
    store.store_raw(abi.RAW_MSG_TAGS, row * 16, old_tag)
    with pytest.raises(GvsError) as ei:
        run_one(store, model, params)
    assert ei.value.code == abi.ERR_INTEGRITY


@pytest.mark.parametrize("staged", [False, True])
def test_swapped_rows_are_detected(staged):
    store, model = make_pair(**(STAGED if staged else {}))
    model.seed(36)
    params = ffi.gen_params(n_identities=200)
    run_stream(store, model, params, batches=2, n=1024)
    a = [store.dump_raw(abi.RAW_MESSAGES, r * 1024, 1024).tobytes() for r in (10, 11)]
    t = [store.dump_raw(abi.RAW_MSG_TAGS, r * 16, 16).tobytes() for r in (10, 11)]
    store.store_raw(abi.RAW_MESSAGES, 10 * 1024, a[1])
    store.store_raw(abi.RAW_MSG_TAGS, 10 * 16, t[1])
    store.store_raw(abi.RAW_MESSAGES, 11 * 1024, a[0])
    store.store_raw(abi.RAW_MSG_TAGS, 11 * 16, t[0])
    with pytest.raises(GvsError) as ei:
        run_one(store, model, params)
    assert ei.value.code == abi.ERR_INTEGRITY


def test_sharded_local_auth_parity():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024,
                          secret_key=SECRET, auth_storage=True, shard_count=2)
    store = ObliviousStore(cfg)
    cl = ffi.Cluster(cfg)
    cl.seed(37)
    p = ffi.gen_params(n_identities=300)
    for b in range(4):
        reqs = cl.gen_batch(2048, p)
        want = cl.process_batch(reqs)
        got = store.process_batch(reqs)
        assert got.tobytes() == want.tobytes(), f"batch {b}"


def live_slot_descriptors(store):
    """Indices of the slot descriptors of the last batch: {row, stamp, position}
    records carrying the newest stamp."""
    st = store.stats()
    n = store.dump_raw_size(abi.RAW_SLOTS) // 128
    d = store.dump_raw(abi.RAW_SLOTS, 0, n * 128).view(np.uint32).reshape(n, 32)[:, :4]
    S = st["msg_partition_slots"]
    stamp = int(d[:, 1].max())
    live = np.nonzero((d[:, 1] == stamp) & (d[:, 0] < S))[0]
    return d, live


@pytest.mark.parametrize("word,delta", [
    (1, 1),   # the stamp: the row's pending final state is hidden
    (0, 1),   # the row: the final state is applied to another row
])
@pytest.mark.parametrize("staged", [False, True])
def test_tampered_slot_descriptor_is_detected(word, delta, staged):
    store, model = make_pair(**(STAGED if staged else {}))
    model.seed(38)
    params = ffi.gen_params(n_identities=200)
    run_stream(store, model, params, batches=2, n=1024)
    d, live = live_slot_descriptors(store)
    assert len(live) > 100
    k = int(live[len(live) // 2])
    rec = d[k].copy()
    rec[word] = (int(rec[word]) + delta) % (1 << 32)
    store.store_raw(abi.RAW_SLOTS, k * 128, rec.tobytes())
    with pytest.raises(GvsError) as ei:
        run_one(store, model, params)
    assert ei.value.code == abi.ERR_INTEGRITY


@pytest.mark.parametrize("word", [2, 3])
def test_descriptor_positions_are_not_trusted(word):
    """The previous batch's descriptor positions (its last op's P position,
    word 2; its first op's, word 3) are not consulted by the pass: the final
    states reach their slots through the authenticated P side entries
    (k_pseal), so changing them changes nothing."""
    store, model = make_pair()
    model.seed(40)
    params = ffi.gen_params(n_identities=200)
    run_stream(store, model, params, batches=2, n=1024)
    d, live = live_slot_descriptors(store)
    for k in live[:50]:
        rec = d[k].copy()
        rec[word] = (int(rec[word]) + 1) % (1 << 32)
        store.store_raw(abi.RAW_SLOTS, int(k) * 128, rec.tobytes())
    run_stream(store, model, params, batches=2, n=1024)


def test_replayed_pending_state_is_detected():
    """An older P entry (same position, previous epoch) in place of the current one."""
    store, model = make_pair()
    model.seed(39)
    params = ffi.gen_params(n_identities=200)
    run_stream(store, model, params, batches=2, n=1024)
    old = [store.dump_raw(r, 0, n).tobytes() for r, n in
           ((abi.RAW_PENDING, 1024 * 1024), (abi.RAW_PENDING_SIDE, 1024 * 128), (abi.RAW_PENDING_TAGS, 1024 * 16))]
    run_stream(store, model, params, batches=1, n=1024)
    for r, b in zip((abi.RAW_PENDING, abi.RAW_PENDING_SIDE, abi.RAW_PENDING_TAGS), old):
        store.store_raw(r, 0, b)
    with pytest.raises(GvsError) as ei:
        run_one(store, model, params)
    assert ei.value.code == abi.ERR_INTEGRITY


def test_joint_slot_overflow_over_two_batches():
    """the sealed pass stages the previous batch's and this
    batch's rows of a partition in the same 86 LDS buffers (gvs_spass.h), so
    k_sjoint fails a batch whose rows plus the previous batch's rows in one
    partition exceed them, even when the batch fits its own c slots.  Two
    batches of 45 by-id reads in one partition (c = 64 here: 4096-request
    batches over 256 partitions): the first is applied, the second fails with
    GVS_ERR_BATCH_OVERFLOW and its own message before anything changes, and a
    smaller batch after it (45 + 10 rows) is applied bit-exact with the oracle,
    which never saw the failed batch; so is a random batch after that."""
    store, model = make_pair(n_msgs=65536, Q=64, Sr=64, B=4096, rpp=256)
    assert store.get_option("txn_slots") == 64 and store.get_option("fixed_schedule_pass") == 1
    W = store.stats()["msg_partitions"]
    model.seed(5)
    fill = ffi.gen_params(create=100, read=0, update=0, delete=0, n_identities=1000)
    live = []
    for _ in range(7):
        reqs = model.gen_batch(4096, fill)
        got, want = store.process_batch(reqs), model.process_batch(reqs)
        assert got.tobytes() == want.tobytes()
        for r, o in zip(reqs, got):
            if o["status_code"] == 1:
                live.append((bytes(o["record"]["msg_id"]), r["auth_identity"].copy()))
    part = {}
    for mid, who in live:
        slot, _ = ffi.id_decode(SECRET[:16], mid, 65536)
        part.setdefault(slot % W, []).append((mid, who))
    q, msgs = max(part.items(), key=lambda kv: len(kv[1]))
    assert len(msgs) >= 100, len(msgs)

    def reads(sel):
        reqs = np.zeros(len(sel), dtype=abi.REQUEST_DTYPE)
        for i, (mid, who) in enumerate(sel):
            reqs[i]["request_type"] = 2
            reqs[i]["msg_id"] = np.frombuffer(mid, np.uint8)
            reqs[i]["auth_identity"] = who
            reqs[i]["timestamp"] = 1_800_000_000 + i
        return reqs

    a, b, c = reads(msgs[:45]), reads(msgs[45:90]), reads(msgs[90:100])
    got, want = store.process_batch(a), model.process_batch(a)
    assert got.tobytes() == want.tobytes() and (got["status_code"] == 1).all()
    before = store.stats()["messages"]
    with pytest.raises(GvsError) as ei:
        store.process_batch(b)
    assert ei.value.code == abi.GVS_ERR_BATCH_OVERFLOW and "previous batch" in str(ei.value), str(ei.value)
    assert store.stats()["messages"] == before
    got, want = store.process_batch(c), model.process_batch(c)
    assert got.tobytes() == want.tobytes() and (got["status_code"] == 1).all()
    got, want = run_one(store, model, ffi.gen_params(n_identities=1000), n=4096)
    assert got.tobytes() == want.tobytes()


def test_fixed_schedule_pass_option():
    """gvs_get_option("fixed_schedule_pass"): 1 where the message pass stages
    every slot line in LDS (c <= 64), 0 past that: B = 16384
    over 256 partitions gives c = 64 + 8 * 8 + 16 = 144."""
    for auth in (False, True):
        for B, want in ((1024, 1), (16384, 0)):
            cfg = abi.make_config(65536, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=B,
                                  secret_key=SECRET, auth_storage=auth, rows_per_partition=256)
            st = ObliviousStore(cfg)
            assert st.get_option("fixed_schedule_pass") == want, (auth, B, st.get_option("txn_slots"))
            st.close()
