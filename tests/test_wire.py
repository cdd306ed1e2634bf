"""Wire-level parity, mirroring api/tests/grapevine_types.rs:
round trips against an independent protobuf implementation (google.protobuf,
messages built from the field numbers/types of api/proto/grapevine.proto:
123-176) and the constant encoded sizes that test file pins (1099 / 1042 B),
plus the enum values of types/src/lib.rs:16-22,122-137."""
import random

import numpy as np
import pytest

from grapevine_amd import abi, wire

pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402

F = descriptor_pb2.FieldDescriptorProto


def _classes():
    fd = descriptor_pb2.FileDescriptorProto(name="gv_test.proto", package="grapevine", syntax="proto3")

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=F.LABEL_OPTIONAL)
            if tname:
                f.type_name = tname

    msg("RequestRecord", [("msg_id", 1, F.TYPE_BYTES, None), ("recipient", 2, F.TYPE_BYTES, None),
                          ("payload", 3, F.TYPE_BYTES, None)])
    msg("Record", [("msg_id", 1, F.TYPE_BYTES, None), ("sender", 2, F.TYPE_BYTES, None),
                   ("recipient", 3, F.TYPE_BYTES, None), ("timestamp", 4, F.TYPE_FIXED64, None),
                   ("payload", 5, F.TYPE_BYTES, None)])
    msg("QueryRequest", [("request_type", 1, F.TYPE_FIXED32, None), ("auth_identity", 2, F.TYPE_BYTES, None),
                         ("auth_signature", 3, F.TYPE_BYTES, None),
                         ("record", 4, F.TYPE_MESSAGE, ".grapevine.RequestRecord")])
    msg("QueryResponse", [("record", 1, F.TYPE_MESSAGE, ".grapevine.Record"),
                          ("status_code", 2, F.TYPE_FIXED32, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return (get(pool.FindMessageTypeByName("grapevine.QueryRequest")),
            get(pool.FindMessageTypeByName("grapevine.QueryResponse")))


QueryRequest, QueryResponse = _classes()


def rb(rng, n):
    return bytes(rng.randrange(256) for _ in range(n))


def random_request(rng):
    # like QueryRequest::from_random, types/src/lib.rs:167-176
    return QueryRequest(request_type=rng.randrange(4) + 1, auth_identity=rb(rng, 32),
                        auth_signature=rb(rng, 64),
                        record=dict(msg_id=rb(rng, 16), recipient=rb(rng, 32), payload=rb(rng, 936)))


def random_response(rng):
    # QueryResponse::from_random draws status 1..9 (types/src/lib.rs:182)
    return QueryResponse(record=dict(msg_id=rb(rng, 16), sender=rb(rng, 32), recipient=rb(rng, 32),
                                     timestamp=rng.getrandbits(64) | 1, payload=rb(rng, 936)),
                         status_code=rng.randrange(9) + 1)


@pytest.mark.parametrize("seed", range(4))
def test_request_round_trip_and_constant_size(seed):
    rng = random.Random(seed)
    msgs = [random_request(rng) for _ in range(16)]
    raw = np.stack([np.frombuffer(m.SerializeToString(), np.uint8) for m in msgs])
    assert raw.shape[1] == wire.REQUEST_WIRE_BYTES == 1099
    q, sig = wire.decode_requests(raw)
    again = wire.encode_requests(q, sig)
    assert again.tobytes() == raw.tobytes()
    for k, m in enumerate(msgs):
        assert q[k]["request_type"] == m.request_type
        assert bytes(q[k]["recipient"]) == m.record.recipient
    # generic reader agrees with the canonical slicer
    q2, sig2 = wire.decode_requests([m.SerializeToString() for m in msgs])
    assert q2.tobytes() == q.tobytes() and sig2.tobytes() == sig.tobytes()


@pytest.mark.parametrize("seed", range(4))
def test_response_round_trip_and_constant_size(seed):
    rng = random.Random(100 + seed)
    msgs = [random_response(rng) for _ in range(16)]
    raw = [m.SerializeToString() for m in msgs]
    assert {len(x) for x in raw} == {wire.RESPONSE_WIRE_BYTES} == {1042}
    r = wire.decode_responses(raw)
    enc = wire.encode_responses(r)
    assert [bytes(x) for x in enc] == raw
    back = QueryResponse.FromString(bytes(enc[3]))
    assert back == msgs[3]


def test_engine_failure_responses_stay_constant_size():
    """The engine's non-success responses (zero fields, nonzero timestamp and
    status) encode to the same 1042 bytes; status 0 / ts 0 would not."""
    r = np.zeros(3, abi.RESPONSE_DTYPE)
    r["record"]["timestamp"] = 1_700_000_000
    r["status_code"] = [abi.STATUS_CODE_NOT_FOUND, abi.STATUS_CODE_INVALID_RECIPIENT,
                        abi.STATUS_CODE_TOO_MANY_MESSAGES]
    enc = wire.encode_responses(r)
    for row in enc:
        m = QueryResponse.FromString(bytes(row))
        assert len(m.SerializeToString()) == 1042
    def size(ts, st):
        return len(QueryResponse(record=dict(msg_id=bytes(16), sender=bytes(32), recipient=bytes(32),
                                             timestamp=ts, payload=bytes(936)),
                                 status_code=st).SerializeToString())
    # zero timestamp -> 1033 B, zero status -> 1037 B
    assert (size(1, 1), size(0, 1), size(1, 0)) == (1042, 1033, 1037)


def test_enum_values():
    # api/tests/grapevine_types.rs:58-113
    assert (abi.REQUEST_TYPE_CREATE, abi.REQUEST_TYPE_READ, abi.REQUEST_TYPE_UPDATE,
            abi.REQUEST_TYPE_DELETE) == (1, 2, 3, 4)
    assert [abi.STATUS_CODE_SUCCESS, abi.STATUS_CODE_NOT_FOUND, abi.STATUS_CODE_MESSAGE_ID_ALREADY_IN_USE,
            abi.STATUS_CODE_INVALID_RECIPIENT, abi.STATUS_CODE_TOO_MANY_MESSAGES_FOR_RECIPIENT,
            abi.STATUS_CODE_TOO_MANY_RECIPIENTS, abi.STATUS_CODE_TOO_MANY_MESSAGES,
            abi.STATUS_CODE_INTERNAL_ERROR] == list(range(1, 9))


# ---- prost decoding rules (the device codec's rule, gvs_process_wire_batch) ----

from wire_cases import all_variants  # noqa: E402


def test_prost_rules_match_google_protobuf_on_valid_variants():
    """Reordered, repeated (last wins), merged-record, unknown-field and
    non-minimal-varint encodings decode to the same fields under the host
    codec's prost rules and under google.protobuf."""
    cases = all_variants(7, 6)
    good = [(n, m) for n, m in cases if not n.startswith("bad_")]
    assert any(n == "step_cap_exact" for n, _ in good)
    q, sig, st = wire.decode_requests([m for _, m in good], timestamps=5, strict=False)
    for k, (name, m) in enumerate(good):
        ref = QueryRequest.FromString(m)
        assert st[k] == wire.WIRE_OK, name
        assert q[k]["request_type"] == ref.request_type, name
        assert bytes(q[k]["auth_identity"]) == ref.auth_identity, name
        assert bytes(sig[k]) == ref.auth_signature, name
        assert bytes(q[k]["msg_id"]) == ref.record.msg_id, name
        assert bytes(q[k]["recipient"]) == ref.record.recipient, name
        assert bytes(q[k]["payload"]) == ref.record.payload, name
        assert q[k]["timestamp"] == 5


def test_malformed_variants_are_rejected():
    cases = all_variants(8, 4)
    bad = [(n, m) for n, m in cases if n.startswith("bad_")]
    q, sig, st = wire.decode_requests([m for _, m in bad], timestamps=5, strict=False)
    for k, (name, m) in enumerate(bad):
        assert st[k] in (wire.WIRE_DECODE_ERROR, wire.WIRE_BAD_FIELD), name
        assert q[k].tobytes() == bytes(abi.REQUEST_DTYPE.itemsize), name  # type 0: a hard error
        assert not sig[k].any()
    # structural errors google.protobuf also refuses
    for name, m in bad:
        if name in ("bad_varint_11_bytes", "bad_length_past_end", "bad_record_past_end",
                    "bad_field_zero", "bad_wire_type_6", "bad_fixed_past_end"):
            with pytest.raises(Exception):
                QueryRequest.FromString(m)
        if name.startswith("bad_") and name[4:] in ("auth_short", "sig_long", "payload_short"):
            assert wire.decode_requests([m], strict=False)[2][0] == wire.WIRE_BAD_FIELD
    with pytest.raises(ValueError):
        wire.decode_requests([bad[0][1]], strict=True)


def test_encode_response_matches_google_protobuf():
    rng = random.Random(11)
    r = np.zeros(24, abi.RESPONSE_DTYPE)
    for k in range(24):
        r[k]["record"]["msg_id"] = np.frombuffer(rb(rng, 16), np.uint8)
        r[k]["record"]["sender"] = np.frombuffer(rb(rng, 32), np.uint8)
        r[k]["record"]["recipient"] = np.frombuffer(rb(rng, 32), np.uint8)
        r[k]["record"]["payload"] = np.frombuffer(rb(rng, 936), np.uint8)
        r[k]["record"]["timestamp"] = 0 if k % 5 == 0 else rng.getrandbits(64)
        r[k]["status_code"] = 0 if k % 7 == 3 else rng.randrange(1, 9)
    for k in range(24):
        enc = wire.encode_response(r[k])
        if r[k]["status_code"] == 0:
            assert enc == b""
            continue
        rec = r[k]["record"]
        ref = QueryResponse(record=dict(msg_id=bytes(rec["msg_id"]), sender=bytes(rec["sender"]),
                                        recipient=bytes(rec["recipient"]), timestamp=int(rec["timestamp"]),
                                        payload=bytes(rec["payload"])),
                            status_code=int(r[k]["status_code"])).SerializeToString()
        assert enc == ref
        assert len(enc) == (1042 if rec["timestamp"] else 1033)
