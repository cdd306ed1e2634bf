"""The CPU restatement of grapevine's challenge check (oracle/sr25519.py),
pinned piece by piece:

  * Keccak-f[1600]: SHAKE128 built on it equals hashlib.shake_128;
  * merlin Transcript: the published "test protocol" vector (the one the
    merlin crate and its ports check);
  * ristretto255: the encodings of 0..8 times the base point, RFC 9496
    Appendix A.1, and the RFC's INVSQRT_A_MINUS_D; decode(encode(P)) = P;
    non-canonical and negative encodings rejected (RFC 9496 §4.3.1);
  * edwards25519 arithmetic: Ed25519 signatures made by the openssl CLI
    verify (tests/golden/ed25519_openssl.json, tests/golden/make_ed25519.py);
  * schnorrkel: sign/verify round trips; every tampered field rejected.
The schnorrkel composition itself has no upstream vector in the image
("parity unpinned")."""
import hashlib
import json
import os
import random

import pytest

from oracle import sr25519 as sr

HERE = os.path.dirname(os.path.abspath(__file__))

RFC9496_MULTIPLES = [
    "0000000000000000000000000000000000000000000000000000000000000000",
    "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76",
    "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919",
    "94741f5d5d52755ece4f23f044ee27d5d1ea1e2bd196b462166b16152a9d0259",
    "da80862773358b466ffadfe0b3293ab3d9fd53c5ea6c955358f568322daf6a57",
    "e882b131016b52c1d3337080187cf768423efccbb517bb495ab812c4160ff44e",
    "f64746d3c92b13050ed8d80236a7f0007c3b3f962f5ba793d19a601ebb1df403",
    "44f53520926ec81fbd5a387845beb7df85a96a24ece18738bdcfa6a7822a176d",
    "903293d8f2287ebe10e2374dc1a53e0bc887e592699f02d077d5263cdd55601c",
]


@pytest.mark.parametrize("n", [0, 1, 167, 168, 169, 500])
def test_keccak_is_shake128(n):
    data = bytes(range(256))[: (n * 7) % 256] * (1 + n // 100)
    assert sr.shake128(data, n + 32) == hashlib.shake_128(data).digest(n + 32)


def test_merlin_published_vector():
    t = sr.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == \
        "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_ristretto_rfc9496_vectors():
    for k, want in enumerate(RFC9496_MULTIPLES):
        p = sr.scalar_mult(k, sr.BASE)
        assert sr.ristretto_encode(p).hex() == want, k
        q = sr.ristretto_decode(bytes.fromhex(want))
        assert q is not None and sr.ristretto_encode(q).hex() == want
    assert sr.INVSQRT_A_MINUS_D == \
        54469307008909316920995813868745141605393597292927456921205312896311721017578


def test_ristretto_rejects_bad_encodings():
    rng = random.Random(4)
    for _ in range(20):
        s = rng.randrange(sr.P) | 1  # negative field element
        assert sr.ristretto_decode(s.to_bytes(32, "little")) is None
    for s in (sr.P, sr.P + 2, 2 ** 255 - 2):  # not canonical
        assert sr.ristretto_decode(s.to_bytes(32, "little")) is None
    # random even field elements decode about half of the time, never wrongly
    ok = 0
    for _ in range(40):
        b = (rng.randrange(sr.P) & ~1).to_bytes(32, "little")
        p = sr.ristretto_decode(b)
        if p is not None:
            ok += 1
            assert sr.ristretto_encode(p) == b
    assert 5 < ok < 35


def test_curve_arithmetic_verifies_openssl_ed25519():
    with open(os.path.join(HERE, "golden", "ed25519_openssl.json")) as f:
        vecs = json.load(f)
    assert len(vecs) >= 8
    for v in vecs:
        pk, msg, sig = (bytes.fromhex(v[k]) for k in ("pk", "msg", "sig"))
        assert sr.ed25519_verify(pk, msg, sig)
        bad = bytearray(sig)
        bad[5] ^= 1
        assert not sr.ed25519_verify(pk, msg, bytes(bad))


def test_schnorrkel_round_trip_and_tampering():
    rng = random.Random(9)
    for _ in range(6):
        x = rng.randrange(1, sr.L)
        msg = rng.randbytes(32)
        sig = sr.sign(x, msg, rng.randrange(1, sr.L))
        pk = sr.public_key(x)
        assert sr.verify(pk, msg, sig)
        assert not sr.verify(pk, msg, sig, context=b"grapevine-challengf")
        assert not sr.verify(pk, bytes([msg[0] ^ 1]) + msg[1:], sig)
        for i in (0, 31, 32, 62):
            bad = bytearray(sig)
            bad[i] ^= 0x04
            assert not sr.verify(pk, msg, bytes(bad)), i
        unmarked = bytearray(sig)
        unmarked[63] &= 0x7F
        assert not sr.verify(pk, msg, bytes(unmarked))
        s = int.from_bytes(sig[32:], "little") & ((1 << 255) - 1)
        big = (s + sr.L).to_bytes(32, "little")  # the same scalar, not canonical
        if big[31] < 0x80:
            assert not sr.verify(pk, msg, sig[:32] + big[:31] + bytes([big[31] | 0x80]))
        assert not sr.verify(sr.public_key(x + 1), msg, sig)
