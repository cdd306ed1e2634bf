"""Wire-level request variants for the codec tests (CPU and GPU).

Each variant is a QueryRequest encoding that prost (types/src/lib.rs:27-78)
treats in a defined way: canonical, reordered, with unknown fields, with
repeated fields (last wins) or a RequestRecord split over several occurrences
(merged), with non-minimal varints -- and malformed ones (truncated, bad
varints, wrong wire types, field number 0, groups, lengths past the end,
fields of the wrong size).  Built by hand from the field numbers and wire
types, so they do not depend on any protobuf library's choices.
"""
import random

REQUEST_TYPES = (1, 2, 3, 4)


def varint(v, pad=0):
    """Minimal varint of v, plus `pad` redundant continuation bytes."""
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v or pad:
            out.append(b | 0x80)
            if not v:
                break
        else:
            out.append(b)
            return bytes(out)
    for k in range(pad):
        out.append(0x80 if k < pad - 1 else 0x00)
    return bytes(out)


def key(field, wt, pad=0):
    return varint(field << 3 | wt, pad)


def ld(field, data, pad=0):
    return key(field, 2) + varint(len(data), pad) + data


def fx32(field, v):
    return key(field, 5) + v.to_bytes(4, "little")


def fx64(field, v):
    return key(field, 1) + v.to_bytes(8, "little")


def rb(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def fields(rng, rtype=None):
    return dict(rt=rtype if rtype is not None else rng.choice(REQUEST_TYPES), auth=rb(rng, 32),
                sig=rb(rng, 64), id=rb(rng, 16) if rng.random() < 0.7 else bytes(16),
                rc=rb(rng, 32), pl=rb(rng, 936))


def record(f, order=(1, 2, 3), pad=0):
    parts = {1: ld(1, f["id"], pad), 2: ld(2, f["rc"], pad), 3: ld(3, f["pl"], pad)}
    return b"".join(parts[k] for k in order)


def canonical(f):
    return fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"]) + ld(4, record(f))


def variants(rng):
    """-> list of (name, bytes).  Names starting with "bad_" are malformed or
    carry wrong-size fields; the rest decode to `f`'s values."""
    f = fields(rng)
    g = fields(rng)  # decoy values, overridden later in the message
    rec = record(f)
    unknown = varint(9 << 3 | 0) + varint(rng.getrandbits(40)) + fx64(10, rng.getrandbits(64)) + \
        ld(11, rb(rng, rng.randrange(0, 40))) + fx32(12, rng.getrandbits(32))
    v = [
        ("canonical", canonical(f)),
        ("reordered", ld(4, record(f, (3, 1, 2))) + ld(3, f["sig"]) + fx32(1, f["rt"]) + ld(2, f["auth"])),
        ("unknown_fields", unknown + fx32(1, f["rt"]) + ld(2, f["auth"]) + unknown + ld(3, f["sig"]) +
         ld(4, unknown + rec + unknown)),
        ("repeated_last_wins", fx32(1, g["rt"]) + ld(2, g["auth"]) + ld(3, g["sig"]) + ld(2, f["auth"]) +
         fx32(1, f["rt"]) + ld(3, f["sig"]) + ld(4, rec)),
        ("record_merged", canonical(dict(f, id=g["id"], rc=g["rc"], pl=g["pl"])) +
         ld(4, ld(1, f["id"]) + ld(3, f["pl"])) + ld(4, ld(2, f["rc"]))),
        ("record_repeated_field", fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"]) +
         ld(4, ld(1, g["id"]) + ld(2, g["rc"]) + rec)),
        ("nonminimal_varints", key(1, 5, pad=2) + f["rt"].to_bytes(4, "little") + ld(2, f["auth"], pad=3) +
         ld(3, f["sig"], pad=1) + key(4, 2, pad=1) + varint(len(record(f, pad=2)), pad=2) + record(f, pad=2)),
        ("type_zero_explicit", canonical(dict(f, rt=0))),
        ("type_out_of_range", canonical(dict(f, rt=rng.choice((5, 9, 0xFFFFFFFF))))),
        ("type_absent", ld(2, f["auth"]) + ld(3, f["sig"]) + ld(4, rec)),
        # 9 steps for the canonical fields + 23 one-step unknown fields: exactly the step cap
        ("step_cap_exact", canonical(f) + (key(9, 0) + varint(1)) * 23),
        ("empty_record_then_full", fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"]) + ld(4, b"") +
         ld(4, rec) + ld(4, b"")),
        # malformed: prost returns DecodeError
        ("bad_truncated", canonical(f)[:rng.randrange(1, 1098)]),
        ("bad_type_as_varint", key(1, 0) + varint(f["rt"]) + canonical(f)[5:]),
        ("bad_auth_as_fixed32", canonical(f) + fx32(2, 7)),
        ("bad_record_as_varint", canonical(f) + key(4, 0) + varint(3)),
        ("bad_record_field_wt", fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"]) +
         ld(4, rec + fx64(2, 1))),
        ("bad_field_zero", canonical(f) + key(0, 0) + varint(1)),
        ("bad_group", canonical(f) + key(13, 3) + key(13, 4)),
        ("bad_wire_type_6", canonical(f) + key(14, 6)),
        ("bad_length_past_end", canonical(f) + key(11, 2) + varint(50) + rb(rng, 10)),
        ("bad_record_past_end", fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"]) +
         key(4, 2) + varint(len(rec) + 5) + rec),
        ("bad_nested_overrun", fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"]) +
         key(4, 2) + varint(len(rec) - 3) + rec),
        ("bad_varint_11_bytes", canonical(f) + key(9, 0) + b"\xff" * 10 + b"\x01"),
        ("bad_varint_10th_byte", canonical(f) + key(9, 0) + b"\xff" * 9 + b"\x02"),
        ("bad_key_above_u32", canonical(f) + varint((1 << 32) | 0) + varint(1)),
        ("bad_over_step_cap", canonical(f) + (key(9, 0) + varint(1)) * 24),  # [D] prost has no cap
        ("bad_fixed_past_end", canonical(f) + key(10, 1) + b"\x01\x02\x03"),
        # decodes, but a field has the wrong size: a hard error for the handler
        ("bad_auth_short", canonical(dict(f, auth=f["auth"][:31]))),
        ("bad_sig_long", canonical(dict(f, sig=f["sig"] + b"\x00"))),
        ("bad_payload_short", canonical(dict(f, pl=f["pl"][:935]))),
        ("bad_msg_id_empty", canonical(dict(f, id=b""))),
        ("bad_record_absent", fx32(1, f["rt"]) + ld(2, f["auth"]) + ld(3, f["sig"])),
        ("bad_empty", b""),
    ]
    return v


def all_variants(seed, rounds):
    rng = random.Random(seed)
    out = []
    for _ in range(rounds):
        out.extend(variants(rng))
    return out
