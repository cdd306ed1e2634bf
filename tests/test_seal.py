"""The authenticated-storage format on CPU.

Three independent implementations must agree:
  * oracle/gvs_seal.c (byte-oriented AES per FIPS-197, BLAKE2b per RFC 7693);
  * a pure-Python composition of the openssl CLI (AES-128-ECB over the counter
    blocks = the CTR keystream) and hashlib.blake2b;
  * the product library's host-side implementation (gvs_storage_seal_row,
    the same gvs_crypto.h code the gfx950 kernels run).
Known-answer vectors: FIPS-197 Appendix C.1, SP 800-38A F.5.1, RFC 7693
Appendix A.  Tag: H ^ G, H the header PRF (AES-128 of the row's nonce for the
message tables, keyed BLAKE2b for the mailbox table); G the row hash of the message
tables (UHASH-128 layers: NH, the one-block L2, the p36 L3; restated below in
Python from its definition) or, for the mailbox table, the XOR of its four leaf
PRFs (gvs_crypto.h).  The row hash has no published vector of its own (UMAC's
are for its full byte layout and the AES-based key derivation): the Python and
C restatements and the library's host code are checked against each other, and
its properties (every word and every tag bit depend on the data, key
separation, linearity of NH) are checked below."""
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


P36 = (1 << 36) - 5


def py_uhash_keys(secret):
    """The row hash's keys from BLAKE2b-512(key = mac_key, "gvs-uhash-" | j)."""
    _, mk = py_keys(secret)
    kb = b"".join(hashlib.blake2b(b"gvs-uhash-" + bytes([j]), key=mk, digest_size=64).digest()
                  for j in range(19))
    nh = [int.from_bytes(kb[4 * w:4 * w + 4], "little") for w in range(268)]
    l3k = []
    for i in range(16):
        k = int.from_bytes(kb[1072 + 8 * i:1080 + 8 * i], "little") & ((1 << 36) - 1)
        l3k.append(k - P36 if k >= P36 else k)
    l3p = [int.from_bytes(kb[1200 + 4 * t:1204 + 4 * t], "little") for t in range(4)]
    return nh, l3k, l3p


def py_row_hash(keys, ct):
    """NH over the row's 256 little-endian words, key shifted 4 words per
    iteration; L3: the 16-bit chunks of S_t (most significant first) against
    l3k mod p36, mod 2^32, xor l3p."""
    nh, l3k, l3p = keys
    m = [int.from_bytes(ct[4 * w:4 * w + 4], "little") for w in range(256)]
    out = b""
    for t in range(4):
        s = 0
        for j in range(128):
            a = (m[2 * j] + nh[4 * t + 2 * j]) & 0xFFFFFFFF
            b = (m[2 * j + 1] + nh[4 * t + 2 * j + 1]) & 0xFFFFFFFF
            s = (s + a * b) & ((1 << 64) - 1)
        y = sum(((s >> (48 - 16 * c)) & 0xFFFF) * l3k[4 * t + c] for c in range(4)) % P36
        out += ((y & 0xFFFFFFFF) ^ l3p[t]).to_bytes(4, "little")
    return out


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
        if table == 3:  # map directory rows
            hdr += sct if sct is not None else bytes(16)
            tag = int.from_bytes(hashlib.blake2b(hdr, key=mk, digest_size=16,
                                                 person=b"gvs-head" + bytes(8)).digest(), "little")
        else:  # AES-128 under kh of the nonce (then of it ^ side ct)
            kh = hashlib.blake2b(b"gvs storage head", key=secret, digest_size=16).digest()
            h = openssl_ecb(kh, hdr)
            if sct is not None:
                h = openssl_ecb(kh, bytes(a ^ b for a, b in zip(h, sct)))
            tag = int.from_bytes(h, "little")
        if table == 3:  # map directory rows: 4 leaf PRFs of 256 B
            for i in range(4):
                person = b"gvs-leaf" + i.to_bytes(4, "little") + (1).to_bytes(4, "little")
                tag ^= int.from_bytes(hashlib.blake2b(ct[256 * i:256 * i + 256], key=mk, digest_size=16,
                                                      person=person).digest(), "little")
        else:  # every other table: the row hash
            tag ^= int.from_bytes(py_row_hash(py_uhash_keys(secret), ct), "little")
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


def test_row_hash_c_matches_python():
    keys_c, keys_py = ffi.uhash_keys(SECRET), py_uhash_keys(SECRET)
    assert list(keys_c[0]) == keys_py[0] and list(keys_c[1]) == keys_py[1] and list(keys_c[2]) == keys_py[2]
    assert all(k < P36 for k in keys_py[1])
    rng = np.random.default_rng(11)
    for ct in (bytes(1024), b"\xff" * 1024, rng.bytes(1024), rng.bytes(1024)):
        assert ffi.row_hash(keys_c, ct) == py_row_hash(keys_py, ct)


def test_row_hash_properties():
    """Every 4-byte word of the row and every tag word depend on the data;
    other secrets give other keys; NH is linear in the key offset as stated
    (the Toeplitz shift: iteration t reads key words 4t .. 4t + 255)."""
    keys = ffi.uhash_keys(SECRET)
    rng = np.random.default_rng(12)
    ct = bytearray(rng.bytes(1024))
    g0 = ffi.row_hash(keys, bytes(ct))
    for w in range(0, 256, 17):
        c2 = bytearray(ct)
        c2[4 * w] ^= 1
        g1 = ffi.row_hash(keys, bytes(c2))
        assert all(g0[4 * t:4 * t + 4] != g1[4 * t:4 * t + 4] for t in range(4)), w
    other = ffi.uhash_keys(bytes(31) + b"\x01")
    assert ffi.row_hash(other, bytes(ct)) != g0
    nh, l3k, l3p = keys
    shifted = (np.concatenate([nh[4:], np.zeros(4, np.uint32)]), l3k.copy(), l3p.copy())
    # iteration 1 of the original keys is iteration 0 of keys shifted by 4 words, given its L3 keys
    shifted[1][0:4] = l3k[4:8]
    shifted[2][0] = l3p[1]
    assert ffi.row_hash(shifted, bytes(ct))[0:4] == g0[4:8]
