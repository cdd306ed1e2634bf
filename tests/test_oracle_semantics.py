"""Known-answer tests of the oracle's handler semantics, written line by line
from api/proto/grapevine.proto:57-122 and README.md:73-175, plus the batch
linearisation rule of DESIGN.md §2."""
import numpy as np
import pytest

from grapevine_amd import abi
from oracle import ffi

A, B_, C = ffi.identity(1), ffi.identity(2), ffi.identity(3)
ZERO32, ZERO16 = bytes(32), bytes(16)
TS = 1_700_000_000


def cfg(n=256, Q=1, Sr=16, B=1024):
    return abi.make_config(n, mailbox_partitions=Q, mailbox_partition_slots=Sr, max_batch=B)


def req(t, auth, msg_id=ZERO16, recipient=ZERO32, payload=b"", ts=TS):
    r = np.zeros(1, dtype=abi.REQUEST_DTYPE)[0]
    r["request_type"] = t
    r["auth_identity"] = np.frombuffer(auth, np.uint8)
    r["msg_id"] = np.frombuffer(msg_id, np.uint8)
    r["recipient"] = np.frombuffer(recipient, np.uint8)
    p = (payload * (936 // max(len(payload), 1) + 1))[:936] if payload else bytes(936)
    r["payload"] = np.frombuffer(p, np.uint8)
    r["timestamp"] = ts
    return r


def create(m, auth, rcpt, payload=b"x", ts=TS):
    return m.apply_one(req(1, auth, recipient=rcpt, payload=payload, ts=ts))


def mid(resp):
    return bytes(resp["record"]["msg_id"])


def test_create_returns_full_record_with_server_fields():
    m = ffi.Model(cfg())
    r = create(m, A, B_, b"hello", ts=TS + 5)
    assert r["status_code"] == abi.STATUS_CODE_SUCCESS
    rec = r["record"]
    assert mid(r) != ZERO16                                  # random nonzero id (proto:66-79)
    assert bytes(rec["sender"]) == A                         # sender = auth_identity
    assert bytes(rec["recipient"]) == B_
    assert rec["timestamp"] == TS + 5                        # server time (README:143-144)
    assert bytes(rec["payload"])[:5] == b"hello"


def test_create_ignores_client_id_and_rejects_zero_recipient():
    m = ffi.Model(cfg())
    r1 = m.apply_one(req(1, A, msg_id=b"\x01" * 16, recipient=B_))
    assert mid(r1) != b"\x01" * 16
    r2 = create(m, A, ZERO32)
    assert r2["status_code"] == abi.STATUS_CODE_INVALID_RECIPIENT  # proto:72
    assert r2["record"]["timestamp"] == TS and not r2["record"]["msg_id"].any()


def test_read_by_id_requires_sender_or_recipient():
    m = ffi.Model(cfg())
    i = mid(create(m, A, B_))
    for who in (A, B_):
        assert m.apply_one(req(2, who, msg_id=i))["status_code"] == abi.STATUS_CODE_SUCCESS
    assert m.apply_one(req(2, C, msg_id=i))["status_code"] == abi.STATUS_CODE_NOT_FOUND  # proto:84
    assert m.apply_one(req(2, A, msg_id=b"\x05" * 16))["status_code"] == abi.STATUS_CODE_NOT_FOUND


def test_read_next_is_fifo_per_recipient_and_nondestructive():
    m = ffi.Model(cfg())
    ids = [mid(create(m, A, B_, bytes([k]))) for k in range(3)]
    for _ in range(2):
        r = m.apply_one(req(2, B_))
        assert r["status_code"] == 1 and mid(r) == ids[0]
    assert m.apply_one(req(2, A))["status_code"] == abi.STATUS_CODE_NOT_FOUND  # sender has no mailbox


def test_update_rules():
    m = ffi.Model(cfg())
    i = mid(create(m, A, B_, b"old"))
    r = m.apply_one(req(3, A, msg_id=i, recipient=C, payload=b"new"))
    assert r["status_code"] == abi.STATUS_CODE_INVALID_RECIPIENT            # proto:99-101
    r = m.apply_one(req(3, C, msg_id=i, recipient=B_, payload=b"new"))
    assert r["status_code"] == abi.STATUS_CODE_NOT_FOUND                    # proto:97
    r = m.apply_one(req(3, B_, msg_id=i, recipient=B_, payload=b"new", ts=TS + 9))
    assert r["status_code"] == 1 and bytes(r["record"]["payload"])[:3] == b"new"
    assert r["record"]["timestamp"] == TS + 9 and bytes(r["record"]["sender"]) == A
    r = m.apply_one(req(2, A, msg_id=i))
    assert bytes(r["record"]["payload"])[:3] == b"new"
    assert m.apply_one(req(3, A))["status_code"] == abi.STATUS_HARD_ERROR    # zero id (proto:95)


def test_delete_by_id_and_next():
    m = ffi.Model(cfg())
    ids = [mid(create(m, A, B_, bytes([k]))) for k in range(3)]
    assert m.apply_one(req(4, A, msg_id=ids[1], recipient=C))["status_code"] == 4
    r = m.apply_one(req(4, A, msg_id=ids[1], recipient=B_))
    assert r["status_code"] == 1 and mid(r) == ids[1]
    assert m.apply_one(req(2, A, msg_id=ids[1]))["status_code"] == 2
    r = m.apply_one(req(4, B_))                                              # delete-next pops head
    assert r["status_code"] == 1 and mid(r) == ids[0]
    r = m.apply_one(req(2, B_))
    assert mid(r) == ids[2]
    assert m.apply_one(req(4, B_))["status_code"] == 1
    assert m.apply_one(req(4, B_))["status_code"] == 2
    assert m.messages == 0 and m.mailboxes == 0


def test_limits_62_per_recipient_and_capacity():
    m = ffi.Model(cfg(n=256, Q=1, Sr=16))
    st = [create(m, A, B_)["status_code"] for _ in range(63)]
    assert st[:62] == [1] * 62 and st[62] == abi.STATUS_CODE_TOO_MANY_MESSAGES_FOR_RECIPIENT
    # 16 mailbox rows in the single partition: the 17th recipient is refused
    st = [create(m, A, ffi.identity(100 + k))["status_code"] for k in range(16)]
    assert st[:15] == [1] * 15 and st[15] == abi.STATUS_CODE_TOO_MANY_RECIPIENTS
    m2 = ffi.Model(cfg(n=256, Q=1, Sr=256))
    st = [create(m2, A, ffi.identity(k % 200))["status_code"] for k in range(300)]
    assert st[:256] == [1] * 256 and set(st[256:]) == {abi.STATUS_CODE_TOO_MANY_MESSAGES}
    # precedence [D]: TOO_MANY_MESSAGES before the per-recipient checks
    assert create(m2, A, ffi.identity(5))["status_code"] == abi.STATUS_CODE_TOO_MANY_MESSAGES


def test_hard_errors():
    m = ffi.Model(cfg())
    assert m.apply_one(req(1, ZERO32, recipient=B_))["status_code"] == 0   # zero auth (proto:60)
    assert m.apply_one(req(0, A))["status_code"] == 0
    assert m.apply_one(req(9, A))["status_code"] == 0
    r = m.apply_one(req(7, A))
    assert not any(r.tobytes())


def test_batch_is_class_ordered_linearisation():
    """process_batch == apply_one over (next ops, creates, rest), each in order."""
    c = cfg(n=4096, Q=4, Sr=64, B=1024)
    m1, m2 = ffi.Model(c), ffi.Model(c)
    m1.seed(3)
    p = ffi.gen_params(n_identities=50, hot=20)
    for _ in range(5):
        reqs = m1.gen_batch(1024, p)
        got = m1.process_batch(reqs)
        order = []
        for cls in range(3):
            for i, r in enumerate(reqs):
                t = int(r["request_type"])
                hard = t not in (1, 2, 3, 4) or not r["auth_identity"].any() or (t == 3 and not r["msg_id"].any())
                k = 2 if hard else (1 if t == 1 else (0 if t in (2, 4) and not r["msg_id"].any() else 2))
                if k == cls:
                    order.append(i)
        want = np.zeros_like(got)
        for i in order:
            want[i] = m2.apply_one(reqs[i])
        assert got.tobytes() == want.tobytes()
    assert m1.digest() == m2.digest()


def test_generator_is_deterministic():
    c = cfg(n=4096, Q=4, Sr=64, B=1024)
    outs = []
    for _ in range(2):
        m = ffi.Model(c)
        m.seed(42)
        p = ffi.gen_params()
        h = []
        for _ in range(3):
            r = m.gen_batch(512, p)
            h.append(m.process_batch(r).tobytes())
        outs.append((b"".join(h), m.digest()))
    assert outs[0] == outs[1]
