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
