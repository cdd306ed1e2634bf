"""Hypothesis property tests, CPU only.

Properties that must hold for every input, not just the seeded streams:
  * wire codec: QueryRequest / QueryResponse slabs survive encode -> decode
    unchanged and always encode to the pinned constant sizes
    (api/tests/grapevine_types.rs:13-55);
  * the sequential model's batch result equals applying the requests one at a
    time in the class order of DESIGN.md §2.8, whatever the mix;
  * the Path ORAM restatement of the reference's CPU path returns the same
    bytes as the sequential model on any small stream;
  * the sharded cluster model gives the unsharded model's statuses;
  * the authenticated-storage format: decryption inverts encryption, and any
    single flipped bit of the ciphertext, side entry, row index, epoch or table
    changes the tag.
"""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from grapevine_amd import abi, wire
from oracle import ffi

SETTINGS = settings(max_examples=25, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])

b16, b32, b64 = (st.binary(min_size=n, max_size=n) for n in (16, 32, 64))
payload = st.binary(min_size=abi.PAYLOAD_BYTES, max_size=abi.PAYLOAD_BYTES)


@st.composite
def request_slabs(draw):
    n = draw(st.integers(1, 6))
    q = np.zeros(n, abi.REQUEST_DTYPE)
    sig = np.zeros((n, 64), np.uint8)
    for k in range(n):
        q[k]["request_type"] = draw(st.integers(1, 2**32 - 1))
        q[k]["auth_identity"] = np.frombuffer(draw(b32), np.uint8)
        q[k]["msg_id"] = np.frombuffer(draw(b16), np.uint8)
        q[k]["recipient"] = np.frombuffer(draw(b32), np.uint8)
        q[k]["payload"] = np.frombuffer(draw(payload), np.uint8)
        sig[k] = np.frombuffer(draw(b64), np.uint8)
    return q, sig


@SETTINGS
@given(request_slabs())
def test_request_wire_round_trip(slab):
    q, sig = slab
    enc = wire.encode_requests(q, sig)
    assert enc.shape[1] == wire.REQUEST_WIRE_BYTES == 1099
    q2, sig2 = wire.decode_requests(enc)
    assert q2.tobytes() == q.tobytes() and sig2.tobytes() == sig.tobytes()
    # the generic field reader agrees with the canonical slicer
    q3, sig3 = wire.decode_requests([bytes(r) for r in enc])
    assert q3.tobytes() == q.tobytes() and sig3.tobytes() == sig.tobytes()


@st.composite
def response_slabs(draw):
    n = draw(st.integers(1, 6))
    r = np.zeros(n, abi.RESPONSE_DTYPE)
    for k in range(n):
        rec = r[k]["record"]
        rec["msg_id"] = np.frombuffer(draw(b16), np.uint8)
        rec["sender"] = np.frombuffer(draw(b32), np.uint8)
        rec["recipient"] = np.frombuffer(draw(b32), np.uint8)
        rec["timestamp"] = draw(st.integers(1, 2**64 - 1))
        rec["payload"] = np.frombuffer(draw(payload), np.uint8)
        r[k]["status_code"] = draw(st.integers(1, 2**32 - 1))
    return r


@SETTINGS
@given(response_slabs())
def test_response_wire_round_trip(r):
    enc = wire.encode_responses(r)
    assert enc.shape[1] == wire.RESPONSE_WIRE_BYTES == 1042
    assert wire.decode_responses([bytes(x) for x in enc]).tobytes() == r.tobytes()


mixes = st.fixed_dictionaries({
    "create": st.integers(0, 60), "read": st.integers(0, 40), "update": st.integers(0, 30),
    "delete": st.integers(0, 40), "nxt": st.integers(0, 100), "miss": st.integers(0, 30),
    "bad_auth": st.integers(0, 20), "bad_recipient": st.integers(0, 20),
    "hard_error": st.integers(0, 5), "zero_recipient": st.integers(0, 5),
    "hot": st.integers(0, 60), "n_identities": st.integers(2, 120),
}).filter(lambda m: m["create"] + m["read"] + m["update"] + m["delete"] > 0)


def small_cfg(sr=16):
    return abi.make_config(256, mailbox_partitions=2, mailbox_partition_slots=sr, max_batch=1024)


def class_of(r):
    t = int(r["request_type"])
    hard = t < 1 or t > 4 or not r["auth_identity"].any() or (t == 3 and not r["msg_id"].any())
    if hard:
        return 2
    if t == 1:
        return 1
    return 0 if t in (2, 4) and not r["msg_id"].any() else 2


@SETTINGS
@given(mixes, st.integers(0, 2**32 - 1), st.lists(st.integers(1, 300), min_size=1, max_size=4))
def test_batch_equals_class_ordered_single_steps(mix, seed, sizes):
    batched, single = ffi.Model(small_cfg()), ffi.Model(small_cfg())
    batched.seed(seed)
    p = ffi.gen_params(**mix)
    for n in sizes:
        reqs = batched.gen_batch(n, p)
        got = batched.process_batch(reqs)
        order = sorted(range(n), key=lambda i: (class_of(reqs[i]), i))
        want = np.zeros(n, abi.RESPONSE_DTYPE)
        for i in order:
            want[i] = single.apply_one(reqs[i])
        assert got.tobytes() == want.tobytes()
    assert (batched.messages, batched.mailboxes) == (single.messages, single.mailboxes)


@SETTINGS
@given(mixes, st.integers(0, 2**32 - 1), st.lists(st.integers(1, 400), min_size=1, max_size=3))
def test_path_oram_equals_sequential_model(mix, seed, sizes):
    cfg = small_cfg()
    seq, oram = ffi.Model(cfg), ffi.PathOramModel(cfg)
    seq.seed(seed)
    p = ffi.gen_params(**mix)
    for n in sizes:
        reqs = seq.gen_batch(n, p)
        assert oram.process_batch(reqs).tobytes() == seq.process_batch(reqs).tobytes()
    assert (oram.messages, oram.mailboxes) == (seq.messages, seq.mailboxes)


@SETTINGS
@given(mixes, st.integers(0, 2**32 - 1), st.sampled_from([2, 4]))
def test_cluster_statuses_equal_unsharded(mix, seed, S):
    """Routing across S shards changes ids (they carry the shard) but no
    outcome: statuses and counts equal the single store's, the requests the
    router sheds (a source's ops past their routing key's cap) aside: those
    are INTERNAL_ERROR and reach the single store as hard errors."""
    cfg = abi.make_config(1024, mailbox_partitions=4, mailbox_partition_slots=32, max_batch=1024,
                          shard_count=S, route_capacity=1024)
    one = ffi.Model(abi.make_config(1024 * S, mailbox_partitions=4 * S, mailbox_partition_slots=32,
                                    max_batch=1024 * S))
    cl = ffi.Cluster(cfg)
    cl.seed(seed)
    p = ffi.gen_params(**{**mix, "miss": 0, "bad_auth": 0, "n_identities": min(mix["n_identities"], 48)})
    reqs = cl.gen_batch(S * 256, p)
    shed = ffi.route_shed(cfg, reqs)
    got = cl.process_batch(reqs)
    ones = reqs.copy()
    ones["request_type"][shed] = 0
    want = one.process_batch(ones)
    assert got is not None
    want["status_code"][shed] = abi.STATUS_CODE_INTERNAL_ERROR
    assert list(got["status_code"]) == list(want["status_code"])
    assert cl.messages == one.messages


SECRET = bytes((0x67 + 31 * i) & 0xFF for i in range(32))


@SETTINGS
@given(st.sampled_from([0, 1]), st.integers(0, 2**40), st.integers(0, 2**32 - 1),
       st.binary(min_size=1024, max_size=1024), st.binary(min_size=16, max_size=16),
       st.integers(0, 1024 * 8 + 16 * 8 - 1))
def test_sealing_inverts_and_binds(table, row, epoch, pt, side, bit):
    side_pt = side if table == 1 else None
    ct, sct, tag = ffi.seal_row(SECRET, table, row, epoch, pt, side_pt)
    ks, sks, _ = ffi.seal_row(SECRET, table, row, epoch, bytes(1024), bytes(16) if side_pt else None)
    assert bytes(a ^ b for a, b in zip(ct, ks)) == pt                 # CTR decrypts
    if side_pt:
        assert bytes(a ^ b for a, b in zip(sct, sks)) == side_pt
    # a flipped plaintext bit flips exactly that ciphertext bit, and the tag changes
    if bit < 1024 * 8:
        pt2 = bytearray(pt)
        pt2[bit // 8] ^= 1 << (bit % 8)
        ct2, _, tag2 = ffi.seal_row(SECRET, table, row, epoch, bytes(pt2), side_pt)
        assert bytes(a ^ b for a, b in zip(ct, ct2)) == bytes(a ^ b for a, b in zip(pt, pt2))
        assert tag2 != tag
    elif side_pt:
        s2 = bytearray(side_pt)
        k = bit - 1024 * 8
        s2[(k // 8) % 16] ^= 1 << (k % 8)
        assert ffi.seal_row(SECRET, table, row, epoch, pt, bytes(s2))[2] != tag
    # the tag binds the row index, the epoch and the table
    assert ffi.seal_row(SECRET, table, row ^ 1, epoch, pt, side_pt)[2] != tag
    assert ffi.seal_row(SECRET, table, row, epoch ^ 1, pt, side_pt)[2] != tag
    other = ffi.seal_row(SECRET, 1 - table, row, epoch, pt, bytes(16) if table == 0 else None)
    assert other[2] != tag
