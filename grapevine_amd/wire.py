"""Batched constant-size protobuf codec for QueryRequest / QueryResponse.

Encodes/decodes the wire form of api/proto/grapevine.proto:123-176 (prost
structs types/src/lib.rs:27-120) directly to/from the engine's POD slabs
(include/gvstore.h), vectorised over a whole batch with numpy.

Every field of these messages has a fixed size (README.md:148: payloads are
exactly 936 bytes), so a fully populated QueryRequest is 1099 bytes and a
QueryResponse with nonzero timestamp and status is 1042 bytes: the
constant-size property pinned by api/tests/grapevine_types.rs:22-31,46-55.
Messages in that canonical form are handled by slicing; anything else goes
through a small generic protobuf reader.
"""
import numpy as np

from . import abi

REQUEST_WIRE_BYTES = 1099
RESPONSE_WIRE_BYTES = 1042

# canonical QueryRequest: (offset, tag bytes) of each field header
_REQ_HDR = [
    (0, b"\x0d"),                 # 1: request_type fixed32
    (5, b"\x12\x20"),             # 2: auth_identity, 32 B
    (39, b"\x1a\x40"),            # 3: auth_signature, 64 B
    (105, b"\x22\xdf\x07"),       # 4: record (RequestRecord, 991 B)
    (108, b"\x0a\x10"),           #    1: msg_id, 16 B
    (126, b"\x12\x20"),           #    2: recipient, 32 B
    (160, b"\x1a\xa8\x07"),       #    3: payload, 936 B
]
_RESP_HDR = [
    (0, b"\x0a\x8a\x08"),         # 1: record (Record, 1034 B)
    (3, b"\x0a\x10"),             #    1: msg_id
    (21, b"\x12\x20"),            #    2: sender
    (55, b"\x1a\x20"),            #    3: recipient
    (89, b"\x21"),                #    4: timestamp fixed64
    (98, b"\x2a\xa8\x07"),        #    5: payload
    (1037, b"\x15"),              # 2: status_code fixed32
]


def _put_headers(buf, hdrs):
    for off, tag in hdrs:
        buf[:, off:off + len(tag)] = np.frombuffer(tag, np.uint8)


def encode_responses(resps):
    """gvs_response slab -> (n, 1042) uint8 wire messages.

    Requires nonzero timestamp and status (what the engine emits for every
    non-hard-error response); raises otherwise, since proto3 would then omit
    the field and the message would not be constant-size."""
    r = np.asarray(resps, dtype=abi.RESPONSE_DTYPE)
    if (r["record"]["timestamp"] == 0).any() or (r["status_code"] == 0).any():
        raise ValueError("zero timestamp/status is not constant-size on the wire")
    n = len(r)
    out = np.zeros((n, RESPONSE_WIRE_BYTES), np.uint8)
    _put_headers(out, _RESP_HDR)
    rec = r["record"]
    out[:, 5:21] = rec["msg_id"]
    out[:, 23:55] = rec["sender"]
    out[:, 57:89] = rec["recipient"]
    out[:, 90:98] = rec["timestamp"].astype("<u8").view(np.uint8).reshape(n, 8)
    out[:, 101:1037] = rec["payload"]
    out[:, 1038:1042] = r["status_code"].astype("<u4").view(np.uint8).reshape(n, 4)
    return out


def encode_requests(reqs, signatures=None):
    """gvs_request slab (+ optional (n, 64) signatures) -> (n, 1099) wire messages."""
    q = np.asarray(reqs, dtype=abi.REQUEST_DTYPE)
    if (q["request_type"] == 0).any():
        raise ValueError("request_type 0 is not constant-size on the wire")
    n = len(q)
    out = np.zeros((n, REQUEST_WIRE_BYTES), np.uint8)
    _put_headers(out, _REQ_HDR)
    out[:, 1:5] = q["request_type"].astype("<u4").view(np.uint8).reshape(n, 4)
    out[:, 7:39] = q["auth_identity"]
    if signatures is not None:
        out[:, 41:105] = signatures
    out[:, 110:126] = q["msg_id"]
    out[:, 128:160] = q["recipient"]
    out[:, 163:1099] = q["payload"]
    return out


class DecodeError(ValueError):
    """The bytes are not a message prost would decode."""


# field number -> wire type of the known fields (prost structs,
# types/src/lib.rs:27-120): 0 varint, 1 fixed64, 2 length-delimited, 5 fixed32
_REQ_SPEC = {1: 5, 2: 2, 3: 2, 4: 2}
_REQREC_SPEC = {1: 2, 2: 2, 3: 2}
_RESP_SPEC = {1: 2, 2: 5}
_REC_SPEC = {1: 2, 2: 2, 3: 2, 4: 1, 5: 2}

WIRE_OK, WIRE_DECODE_ERROR, WIRE_BAD_FIELD = abi.WIRE_OK, abi.WIRE_DECODE_ERROR, abi.WIRE_BAD_FIELD


def _varint(b, i, end):
    """prost decode_varint: at most 10 bytes, the 10th at most 1."""
    v = 0
    for c in range(10):
        if i >= end:
            break
        x = b[i]
        i += 1
        v |= (x & 0x7F) << (7 * c)
        if x < 0x80:
            if c == 9 and x > 1:
                raise DecodeError("invalid varint")
            return v, i
    raise DecodeError("invalid varint")


WIRE_STEPS = 32  # gvs_wire.h kWireSteps: fields + embedded records + 1 per request


def _walk(b, i, end, spec, out, nested=None, steps=None):
    """Decode fields in b[i:end) the way prost's generated merge does: a known
    field must carry its wire type, unknown fields are skipped, the last
    occurrence of a scalar / bytes field wins, and an embedded message named in
    `nested` ({field: (spec, dict)}) is merged over all its occurrences.
    [D] Groups (wire types 3/4) are rejected (prost would skip unknown ones)."""
    while i < end:
        if steps is not None:
            steps[0] += 1
        key, i = _varint(b, i, end)
        if key > 0xFFFFFFFF:
            raise DecodeError("invalid key value")
        f, wt = key >> 3, key & 7
        if f == 0 or wt in (3, 4) or wt > 5:
            raise DecodeError(f"invalid tag {f} / wire type {wt}")
        if f in spec and spec[f] != wt:
            raise DecodeError(f"field {f}: wire type {wt}, expected {spec[f]}")
        if wt == 0:
            _, i = _varint(b, i, end)
        elif wt in (1, 5):
            sz = 8 if wt == 1 else 4
            if end - i < sz:
                raise DecodeError("buffer underflow")
            if f in spec:
                out[f] = int.from_bytes(bytes(b[i:i + sz]), "little")
            i += sz
        else:
            ln, i = _varint(b, i, end)
            if ln > end - i:
                raise DecodeError("buffer underflow")
            if f in spec:
                if nested and f in nested:
                    _walk(b, i, i + ln, nested[f][0], nested[f][1], steps=steps)
                    if steps is not None:
                        steps[0] += 1  # leaving the embedded message
                else:
                    out[f] = bytes(b[i:i + ln])
            i += ln
    return out


def _fixed(v, size, name):
    v = v if v is not None else b""
    if len(v) != size:
        raise ValueError(f"{name} must be exactly {size} bytes, got {len(v)}")
    return np.frombuffer(v, np.uint8)


def decode_request(m):
    """One wire QueryRequest -> (fields, record fields) with prost semantics;
    raises DecodeError.  [D] Like the device decoder, a request needing more
    than WIRE_STEPS steps (fields + embedded records + 1) is refused."""
    f, rec = {}, {}
    steps = [1]
    _walk(bytes(m), 0, len(m), _REQ_SPEC, f, {4: (_REQREC_SPEC, rec)}, steps=steps)
    if steps[0] > WIRE_STEPS:
        raise DecodeError(f"{steps[0]} decode steps, more than {WIRE_STEPS}")
    return f, rec


def decode_requests(msgs, timestamps=None, strict=True):
    """Wire QueryRequests -> (gvs_request slab, (n, 64) signatures[, status]).

    `msgs` is a list of bytes or an (n, 1099) uint8 array; `timestamps` is the
    server time to stamp on each request (README.md:143-144).  strict: a
    message that fails to decode or has a field of the wrong size raises.
    Otherwise it becomes an all-zero request of type 0 (a hard error in the
    store) and a per-message GVS_WIRE_* status array is returned too: the
    device codec's rule (gvs_process_wire_batch, include/gvstore.h)."""
    canon = strict and isinstance(msgs, np.ndarray) and msgs.ndim == 2 and msgs.shape[1] == REQUEST_WIRE_BYTES
    if canon:
        for off, tag in _REQ_HDR:
            if not (msgs[:, off:off + len(tag)] == np.frombuffer(tag, np.uint8)).all():
                canon = False
                break
    if canon:
        n = len(msgs)
        q = np.zeros(n, abi.REQUEST_DTYPE)
        q["request_type"] = msgs[:, 1:5].copy().view("<u4").reshape(n)
        q["auth_identity"] = msgs[:, 7:39]
        sig = msgs[:, 41:105].copy()
        q["msg_id"] = msgs[:, 110:126]
        q["recipient"] = msgs[:, 128:160]
        q["payload"] = msgs[:, 163:1099]
        status = np.zeros(n, np.uint32)
    else:
        rows = [bytes(m) for m in msgs]
        n = len(rows)
        q = np.zeros(n, abi.REQUEST_DTYPE)
        sig = np.zeros((n, 64), np.uint8)
        status = np.zeros(n, np.uint32)
        for k, m in enumerate(rows):
            try:
                f, rec = decode_request(m)
            except DecodeError:
                if strict:
                    raise
                status[k] = WIRE_DECODE_ERROR
                continue
            try:
                vals = (_fixed(f.get(2), 32, "auth_identity"), _fixed(f.get(3), 64, "auth_signature"),
                        _fixed(rec.get(1), 16, "msg_id"), _fixed(rec.get(2), 32, "recipient"),
                        _fixed(rec.get(3), abi.PAYLOAD_BYTES, "payload"))
            except ValueError:
                if strict:
                    raise
                status[k] = WIRE_BAD_FIELD
                continue
            q[k]["request_type"] = f.get(1, 0)
            q[k]["auth_identity"], sig[k], q[k]["msg_id"], q[k]["recipient"], q[k]["payload"] = vals
    if timestamps is not None:
        q["timestamp"] = np.where(status == 0, timestamps, 0)
    return (q, sig) if strict else (q, sig, status)


def encode_response(r):
    """One gvs_response -> the bytes prost writes for its QueryResponse, or b""
    for a hard error (status 0: the handler answers with a gRPC error).  A zero
    timestamp is omitted (1033 B); otherwise 1042 B."""
    if int(r["status_code"]) == 0:
        return b""
    rec = r["record"]
    ts = int(rec["timestamp"])
    body = (b"\x0a\x10" + bytes(rec["msg_id"]) + b"\x12\x20" + bytes(rec["sender"]) +
            b"\x1a\x20" + bytes(rec["recipient"]) +
            (b"\x21" + ts.to_bytes(8, "little") if ts else b"") +
            b"\x2a\xa8\x07" + bytes(rec["payload"]))
    ln = len(body)
    return (b"\x0a" + bytes([(ln & 0x7F) | 0x80, ln >> 7]) + body + b"\x15" +
            int(r["status_code"]).to_bytes(4, "little"))


def decode_responses(msgs):
    """Wire QueryResponses -> gvs_response slab (prost rules, strict)."""
    n = len(msgs)
    r = np.zeros(n, abi.RESPONSE_DTYPE)
    for k, m in enumerate(msgs):
        f, rec = {}, {}
        _walk(bytes(m), 0, len(m), _RESP_SPEC, f, {1: (_REC_SPEC, rec)})
        r[k]["record"]["msg_id"] = _fixed(rec.get(1), 16, "msg_id")
        r[k]["record"]["sender"] = _fixed(rec.get(2), 32, "sender")
        r[k]["record"]["recipient"] = _fixed(rec.get(3), 32, "recipient")
        r[k]["record"]["timestamp"] = rec.get(4, 0)
        r[k]["record"]["payload"] = _fixed(rec.get(5), abi.PAYLOAD_BYTES, "payload")
        r[k]["status_code"] = f.get(2, 0)
    return r
