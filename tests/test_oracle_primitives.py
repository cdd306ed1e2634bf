"""Pins the oracle's primitives against independent sources:
SipHash-2-4 against the SipHash paper's vectors and against CPython's own
siphash24 (sys.hash_info.algorithm == 'siphash24'; PYTHONHASHSEED=0 zeroes its
key), and the id PRP against its inverse."""
import os
import random
import subprocess
import sys

import pytest

from oracle import ffi

KEY = bytes(range(16))


def test_siphash_paper_vectors():
    # Aumasson & Bernstein, "SipHash: a fast short-input PRF", Appendix A
    assert ffi.siphash24(KEY, bytes(range(15))) == 0xA129CA6149BE45E5
    # reference implementation vectors.h, first entry (empty message)
    assert ffi.siphash24(KEY, b"") == 0x726FDB47DD0E0E31


@pytest.mark.skipif(sys.hash_info.algorithm != "siphash24", reason="CPython not using siphash24")
def test_siphash_matches_cpython_builtin():
    rnd = random.Random(5)
    msgs = [bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 80))) for _ in range(200)]
    msgs += [bytes(range(n)) for n in range(1, 40)]
    code = "import sys\nfor h in sys.argv[1:]: print(hash(bytes.fromhex(h)))"
    env = dict(os.environ, PYTHONHASHSEED="0")
    out = subprocess.run([sys.executable, "-c", code] + [m.hex() for m in msgs],
                         env=env, capture_output=True, text=True, check=True).stdout.split()
    for m, h in zip(msgs, out):
        want = int(h) & 0xFFFFFFFFFFFFFFFF
        got = ffi.siphash24(bytes(16), m)
        if got == 0xFFFFFFFFFFFFFFFF:  # CPython maps -1 to -2
            got = 0xFFFFFFFFFFFFFFFE
        assert got == want, m.hex()


def test_id_prp_roundtrip_and_uniqueness():
    key = bytes(range(100, 116))
    seen = set()
    for slot in (0, 1, 255, 4095, (1 << 20) - 1):
        for ctr in (0, 1, 2, 1 << 40):
            i = ffi.id_encode(key, slot, ctr)
            assert i != bytes(16)
            assert ffi.id_decode(key, i, 1 << 20) == (slot, ctr)
            assert ffi.id_decode(key, i, slot) is None  # slot out of range
            seen.add(i)
    assert len(seen) == 20
    # random ids almost never decode (32-bit tag)
    rnd = random.Random(1)
    bad = sum(ffi.id_decode(key, bytes(rnd.randrange(256) for _ in range(16)), 1 << 32) is not None
              for _ in range(2000))
    assert bad == 0
