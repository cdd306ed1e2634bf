"""The authenticated-storage format on CPU.

Three independent implementations must agree:
  * oracle/gvs_seal.c (byte-oriented AES per FIPS-197, BLAKE2b per RFC 7693);
  * a pure-Python composition of the openssl CLI (AES-128-ECB over the counter
    blocks = the CTR keystream) and hashlib.blake2b;
  * the product library's host-side implementation (gvs_storage_seal_row,
    the same gvs_crypto.h code the gfx950 kernels run).
Known-answer vectors: FIPS-197 Appendix C.1, SP 800-38A F.5.1, RFC 7693
Appendix A.  Tag: H ^ L_0 ^ .. ^ L_3 (XOR-MAC with a counter term, gvs_crypto.h)."""
import ctypes
import hashlib
import shutil
import subprocess

import numpy as np
import pytest

from oracle import ffi

SECRET = bytes((0x67 + 31 * i) & 0xFF for i in range(32))
HAVE_OPENSSL = shutil.which("openssl") is not None


def openssl_ecb(key16, data):
    r = subprocess.run(["openssl", "enc", "-aes-128-ecb", "-nopad", "-K", key16.hex()],
                       input=data, capture_output=True, check=True)
    return r.stdout


def py_keys(secret):
    a = hashlib.blake2b(b"gvs storage aes", key=secret, digest_size=16).digest()
    m = hashlib.blake2b(b"gvs storage mac", key=secret, digest_size=32).digest()
    return a, m


def counter_block(table, row, epoch, j):
    return (row.to_bytes(8, "little") + epoch.to_bytes(4, "little") + bytes([table & 0xFF, 0])
            + j.to_bytes(2, "big"))


def py_seal_rows(secret, table, rows, epoch, pts, side_pts=None):
    """Reference sealing of many rows at once (one openssl call)."""
    ak, mk = py_keys(secret)
    nb = 65 if side_pts is not None else 64
    ctr = b"".join(counter_block(table, r, epoch, j) for r in rows for j in range(nb))
    ks = np.frombuffer(openssl_ecb(ak, ctr), np.uint8).reshape(len(rows), nb * 16)
    out = []
    for k, r in enumerate(rows):
        ct = bytes(np.frombuffer(pts[k], np.uint8) ^ ks[k, :1024])
        sct = bytes(np.frombuffer(side_pts[k], np.uint8) ^ ks[k, 1024:]) if side_pts is not None else None
        hdr = r.to_bytes(8, "little") + epoch.to_bytes(4, "little") + table.to_bytes(4, "little")
        hdr += sct if sct is not None else bytes(16)
        tag = int.from_bytes(hashlib.blake2b(hdr, key=mk, digest_size=16,
                                             person=b"gvs-head" + bytes(8)).digest(), "little")
        nl = 4 if table & 1 else 8  # mailbox rows: 4 leaves of 256 B; message tables: 8 of 128 B
        lb = 1024 // nl
        for i in range(nl):
            person = b"gvs-leaf" + i.to_bytes(4, "little") + (table & 1).to_bytes(4, "little")
            tag ^= int.from_bytes(hashlib.blake2b(ct[lb * i:lb * i + lb], key=mk, digest_size=16,
                                                  person=person).digest(), "little")
        out.append((ct, sct, tag.to_bytes(16, "little")))
    return out


def test_aes128_fips197_and_sp800_38a():
    key = bytes(range(16))
    assert ffi.aes128_encrypt(key, bytes.fromhex("00112233445566778899aabbccddeeff")).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"
    k2 = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    ks = ffi.aes128_encrypt(k2, bytes.fromhex("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff"))
    ct = bytes(a ^ b for a, b in zip(ks, bytes.fromhex("6bc1bee22e409f96e93d7e117393172a")))
    assert ct.hex() == "874d6191b620e3261bef6864990db6ce"


@pytest.mark.skipif(not HAVE_OPENSSL, reason="openssl CLI absent")
def test_aes128_matches_openssl_on_random_blocks():
    rng = np.random.default_rng(1)
    for _ in range(4):
        key = rng.bytes(16)
        blocks = rng.bytes(16 * 64)
        want = openssl_ecb(key, blocks)
        got = b"".join(ffi.aes128_encrypt(key, blocks[i:i + 16]) for i in range(0, len(blocks), 16))
        assert got == want


def test_blake2b_rfc7693_and_hashlib():
    assert ffi.blake2b(b"abc").hex().startswith("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b7")
    rng = np.random.default_rng(2)
    for n in (0, 1, 127, 128, 129, 255, 256, 1000):
        msg = rng.bytes(n)
        for ds, key, person in ((64, b"", None), (16, b"", b"gvs-leaf" + bytes(8)),
                                (16, rng.bytes(32), None), (32, rng.bytes(64), rng.bytes(16))):
            want = hashlib.blake2b(msg, digest_size=ds, key=key,
                                   person=person if person else b"").digest()
            assert ffi.blake2b(msg, ds, key, person) == want, (n, ds, len(key))


# 0 messages, 1 mailboxes, 2 pending final states (side: target row), 0x100 a
# message row whose final state is pending
TABLES = [0, 1, 2, 0x100]


def has_side(table):
    return table in (1, 2)


@pytest.mark.skipif(not HAVE_OPENSSL, reason="openssl CLI absent")
@pytest.mark.parametrize("table", TABLES)
def test_seal_row_matches_reference(table):
    rng = np.random.default_rng(3 + table)
    rows = [0, 1, 4095, (1 << 24) - 1, 123456789]
    pts = [rng.bytes(1024) for _ in rows]
    sides = [rng.bytes(16) for _ in rows] if has_side(table) else None
    ref = py_seal_rows(SECRET, table, rows, 7, pts, sides)
    for k, r in enumerate(rows):
        got = ffi.seal_row(SECRET, table, r, 7, pts[k], sides[k] if sides else None)
        assert got == ref[k], (table, r)
    assert ffi.storage_keys(SECRET) == py_keys(SECRET)


def test_seal_binds_row_epoch_and_table():
    pt = bytes(1024)
    base = ffi.seal_row(SECRET, 0, 5, 3, pt)
    assert ffi.seal_row(SECRET, 0, 6, 3, pt)[2] != base[2]
    assert ffi.seal_row(SECRET, 0, 5, 4, pt)[2] != base[2]
    assert ffi.seal_row(SECRET, 1, 5, 3, pt, bytes(16))[2] != base[2]
    assert ffi.seal_row(SECRET, 2, 5, 3, pt, bytes(16))[2] != base[2]
    pend = ffi.seal_row(SECRET, 0x100, 5, 3, pt)
    assert pend[0] == base[0] and pend[2] != base[2]  # same ciphertext, another tag
    assert ffi.seal_row(SECRET, 0, 5, 3, pt)[0] != ffi.seal_row(SECRET, 0, 5, 4, pt)[0]


def library_seal(table, row, epoch, pt, side=None):
    from grapevine_amd.store import load_library
    lib = load_library()
    ct, sct, tag = (ctypes.create_string_buffer(1024), ctypes.create_string_buffer(16),
                    ctypes.create_string_buffer(16))
    rc = lib.gvs_storage_seal_row(SECRET, table, row, epoch, pt, side, ct, sct, tag)
    assert rc == 0
    return ct.raw, (sct.raw if side is not None else None), tag.raw


@pytest.mark.parametrize("table", TABLES)
def test_library_host_sealing_matches_oracle(table):
    rng = np.random.default_rng(10 + table)
    for row in (0, 77, (1 << 20) + 3):
        pt = rng.bytes(1024)
        side = rng.bytes(16) if has_side(table) else None
        assert library_seal(table, row, 9, pt, side) == ffi.seal_row(SECRET, table, row, 9, pt, side)
