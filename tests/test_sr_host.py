"""The arithmetic of the device signature check (gvs_sr25519.h: field
multiply and square, ristretto255 decode / encode, the joint scalar
multiplication s*B - k*A, the wide reduction mod l), built for the CPU
(tests/libsrhost.so from tests/sr_host.cpp) and checked against the oracle
(oracle/sr25519.py, pinned in tests/test_sr25519.py) on random and edge
inputs.  The GPU tests (tests/test_gpu_sr25519.py) check the kernel itself."""
import ctypes
import os
import random

import pytest

from oracle import sr25519 as sr

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libsrhost.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("tests/libsrhost.so not built (make)")
    return ctypes.CDLL(LIB)


def b32(x):
    return (x % (1 << 256)).to_bytes(32, "little")


def test_field_mul_and_square(lib):
    rng = random.Random(1)
    edge = [0, 1, 2, sr.P - 1, sr.P, sr.P + 1, 2 ** 255, 2 ** 256 - 1, 2 ** 256 - 38, 2 ** 256 - 39]
    vals = edge + [rng.getrandbits(256) for _ in range(300)]
    prod, sq = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    for i, a in enumerate(vals):
        b = vals[(i * 7 + 3) % len(vals)]
        lib.sr_host_mul(b32(a), b32(b), prod, sq)
        assert int.from_bytes(prod.raw, "little") == a * b % sr.P, (a, b)
        assert int.from_bytes(sq.raw, "little") == a * a % sr.P, a


def test_decode_encode_roundtrip(lib):
    rng = random.Random(2)
    out = ctypes.create_string_buffer(32)
    for k in range(9):
        enc = sr.ristretto_encode(sr.scalar_mult(k, sr.BASE))
        assert lib.sr_host_roundtrip(enc, out) == 1 and out.raw == enc
    for _ in range(200):
        b = rng.randbytes(32)
        want = sr.ristretto_decode(b)
        ok = lib.sr_host_roundtrip(b, out)
        assert ok == (want is not None), b.hex()
        if ok:
            assert out.raw == b


def test_double_scalar_mul(lib):
    rng = random.Random(3)
    out = ctypes.create_string_buffer(32)
    for i in range(40):
        x = rng.randrange(1, sr.L)
        pk = sr.public_key(x)
        s = rng.randrange(sr.L) if i % 10 else (0 if i == 0 else sr.L - 1)
        k = rng.randrange(sr.L) if i % 7 else (0 if i == 7 else sr.L - 1)
        assert lib.sr_host_combine(b32(s), b32(k), pk, out) == 1
        a = sr.ristretto_decode(pk)
        want = sr.ristretto_encode(sr.point_add(sr.scalar_mult(s, sr.BASE),
                                                sr.scalar_mult(k, sr.point_neg(a))))
        assert out.raw == want, i


def test_reduce_wide(lib):
    rng = random.Random(4)
    out = ctypes.create_string_buffer(32)
    for v in [0, sr.L - 1, sr.L, 2 ** 512 - 1] + [rng.getrandbits(512) for _ in range(300)]:
        lib.sr_host_reduce_wide(v.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw, "little") == v % sr.L, v
