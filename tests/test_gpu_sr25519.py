"""GPU parity of the batched schnorrkel challenge check (SURVEY.md §8(f)
rank 3; include/gvstore.h gvs_sr25519_verify, gvs_process_wire_batch with
challenges) against the CPU restatement oracle/sr25519.py (pinned in
tests/test_sr25519.py).  Every verdict must equal the oracle's: valid
signatures, every tampered field, unmarked and non-canonical scalars,
non-canonical and off-curve keys, other contexts and message lengths."""
import random

import numpy as np
import pytest

from grapevine_amd import abi, wire
from grapevine_amd.store import ObliviousStore
from oracle import ffi
from oracle import sr25519 as sr

import wire_cases

pytestmark = pytest.mark.gpu


def small_store():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024)
    return ObliviousStore(cfg), ffi.Model(cfg)


def cases(rng, n, msg_len, context):
    """(pk, msg, sig) triples: valid ones and every kind of invalid one."""
    out = []
    keys = [rng.randrange(1, sr.L) for _ in range(8)]
    pks = [sr.public_key(x) for x in keys]
    for i in range(n):
        j = i % len(keys)
        msg = rng.randbytes(msg_len)
        sig = bytearray(sr.sign(keys[j], msg, rng.randrange(1, sr.L), context))
        pk = bytearray(pks[j])
        kind = i % 12
        if kind == 1:
            sig[rng.randrange(32)] ^= 1 << rng.randrange(8)         # R
        elif kind == 2:
            sig[32 + rng.randrange(31)] ^= 1 << rng.randrange(8)    # s
        elif kind == 3:
            sig[63] &= 0x7F                                         # no schnorrkel marker
        elif kind == 4:
            s = int.from_bytes(sig[32:], "little") & ((1 << 255) - 1)
            big = s + sr.L                                          # same scalar, not canonical
            if big < 1 << 255:
                sig[32:] = (big | 1 << 255).to_bytes(32, "little")
        elif kind == 5:
            pk = bytearray(pks[(j + 1) % len(keys)])                # another signer's key
        elif kind == 6:
            pk[0] |= 1                                              # negative field element
        elif kind == 7 and msg_len:
            msg = bytes([msg[0] ^ 0x80]) + msg[1:]                  # another message
        elif kind == 8:
            pk = bytearray((sr.P + rng.randrange(19) // 2 * 2).to_bytes(32, "little"))  # >= p
        elif kind == 9:
            pk = bytearray(rng.randbytes(32))                       # random bytes
        elif kind == 10:
            sig = bytearray(rng.randbytes(64))
        out.append((bytes(pk), msg, bytes(sig)))
    return out


@pytest.mark.parametrize("msg_len,context", [(32, b"grapevine-challenge"), (0, b""),
                                             (200, b"substrate"), (400, bytes(range(64)))])
def test_verify_matches_oracle(msg_len, context):
    store, _ = small_store()
    rng = random.Random(msg_len * 7 + len(context))
    cs = cases(rng, 96, msg_len, context)
    want = np.array([sr.verify(pk, msg, sig, context) for pk, msg, sig in cs])
    got = store.sr25519_verify(np.frombuffer(b"".join(c[0] for c in cs), np.uint8).reshape(-1, 32),
                               np.frombuffer(b"".join(c[1] for c in cs), np.uint8).reshape(len(cs), msg_len),
                               np.frombuffer(b"".join(c[2] for c in cs), np.uint8).reshape(-1, 64),
                               context)
    bad = np.nonzero(got != want)[0]
    assert not len(bad), [(int(k), k % 12, bool(got[k]), bool(want[k])) for k in bad[:8]]
    assert want.sum() >= 96 // 12 * 2  # valid signatures and the no-op tampers are in the mix
    store.close()


def test_verify_many_valid():
    """A full wave of blocks: 700 valid signatures across 7 keys all pass."""
    store, _ = small_store()
    rng = random.Random(5)
    keys = [rng.randrange(1, sr.L) for _ in range(7)]
    pks = [sr.public_key(x) for x in keys]
    n = 700
    msgs = [rng.randbytes(32) for _ in range(n)]
    sigs = [sr.sign(keys[i % 7], msgs[i], rng.randrange(1, sr.L)) for i in range(n)]
    assert sr.verify(pks[3], msgs[3], sigs[3])
    got = store.sr25519_verify(np.frombuffer(b"".join(pks[i % 7] for i in range(n)), np.uint8).reshape(n, 32),
                               np.frombuffer(b"".join(msgs), np.uint8).reshape(n, 32),
                               np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 64))
    assert got.all(), np.nonzero(~got)[0][:10]
    store.close()


def test_wire_batch_with_challenges():
    """Wire requests signed by their auth identity over per-request challenges:
    the device decodes, verifies, runs the store and encodes; a request with a
    bad signature is a hard error (empty response, status GVS_WIRE_BAD_SIGNATURE)."""
    store, model = small_store()
    model.seed(41)
    params = ffi.gen_params(n_identities=60, hot=5)
    rng = random.Random(77)
    keymap = {}

    def key_for(ident):
        if ident not in keymap:
            x = rng.randrange(1, sr.L)
            keymap[ident] = (x, sr.public_key(x))
        return keymap[ident]

    for b in range(2):
        reqs = model.gen_batch(1024, params)
        for q in reqs:  # identities and recipients become real ristretto keys
            for f in ("auth_identity", "recipient"):
                v = bytes(q[f])
                if any(v):
                    q[f] = np.frombuffer(key_for(v)[1], np.uint8)
        inv = {pk: x for x, pk in keymap.values()}
        chal = np.frombuffer(rng.randbytes(32 * len(reqs)), np.uint8).reshape(-1, 32)
        msgs, forged = [], []
        for k, q in enumerate(reqs):
            pk = bytes(q["auth_identity"])
            x = inv.get(pk, 1)
            sig = bytearray(sr.sign(x, bytes(chal[k]), rng.randrange(1, sr.L)))
            if k % 9 == 4:
                sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
                forged.append(k)
            f = dict(rt=int(q["request_type"]), auth=pk, sig=bytes(sig), id=bytes(q["msg_id"]),
                     rc=bytes(q["recipient"]), pl=bytes(q["payload"]))
            msgs.append(wire_cases.canonical(f))
        times = reqs["timestamp"].copy()
        q, sig, st = wire.decode_requests(msgs, timestamps=times, strict=False)
        valid = np.ones(len(reqs), bool)
        unknown = [k for k in range(len(reqs)) if bytes(reqs[k]["auth_identity"]) not in inv]
        for k in forged + unknown:  # oracle verdicts where validity is not by construction
            valid[k] = sr.verify(bytes(reqs[k]["auth_identity"]), bytes(chal[k]), bytes(sig[k]))
        for k in np.nonzero(~valid)[0]:
            q[k]["request_type"] = 0
            st[k] = st[k] or abi.WIRE_BAD_SIGNATURE
        want = [wire.encode_response(r) for r in model.process_batch(q)]
        got, got_sig, got_st = store.process_wire_batch(msgs, times, challenges=chal)
        assert (got_st == st).all(), np.nonzero(got_st != st)[0][:10]
        diff = [k for k in range(len(want)) if got[k] != want[k]]
        assert not diff, f"batch {b}: {len(diff)} responses differ (first {diff[:5]})"
        assert (~valid).sum() > 50
        s = store.stats()
        assert (s["messages"], s["mailboxes"]) == (model.messages, model.mailboxes)
    store.close()
