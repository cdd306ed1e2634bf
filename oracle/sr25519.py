"""CPU restatement of grapevine's challenge check (TEST INFRASTRUCTURE ONLY:
only tests/, smoke() and bench.py's cpu_baseline may use it; the product path
is the HIP kernel in grapevine_amd/csrc/gvs_sr25519.h).

What the reference does (README.md:187-200, types/src/lib.rs:13,
api/proto/grapevine.proto:20-25,126-131): a client signs each 32-byte
challenge with its Ristretto key using mc-crypto-keys' `sign_schnorrkel`
under the signing context b"grapevine-challenge"; the enclave verifies the
signature against `auth_identity` before serving the request.  Those crates
(schnorrkel, merlin, curve25519-dalek, pinned through mc-crypto-keys) are
absent from /root/reference and not in its Cargo.lock, so this file restates
their published algorithms:

  * Keccak-f[1600] (FIPS 202) -- pinned against hashlib.shake_128 (same
    permutation, rate 168 = STROBE-128's) in tests/test_sr25519.py;
  * STROBE-128 as merlin's minimal strobe.rs implements it (meta_ad / ad /
    prf only), and merlin 2's Transcript (label b"Merlin v1.0",
    append_message = meta_ad(label) + meta_ad(le32 len, more) + ad(msg),
    challenge_bytes = meta_ad(label) + meta_ad(le32 len, more) + prf);
  * ristretto255 (RFC 9496 §4.3: decode, encode, SQRT_RATIO_M1) over
    edwards25519 (RFC 8032 §5.1) -- the encoding of the base point and its
    small multiples is pinned against RFC 9496 Appendix A.1, and the curve
    arithmetic against Ed25519 signatures made by the openssl CLI;
  * schnorrkel 0.11 verify: transcript = Transcript("SigningContext"),
    append_message(b"", context), append_message(b"sign-bytes", msg),
    append_message(b"proto-name", b"Schnorr-sig"),
    append_message(b"sign:pk", A), append_message(b"sign:R", R),
    k = challenge_bytes(b"sign:c", 64) mod l; accept iff the signature's
    high bit (schnorrkel's marker) is set, s < l, A decodes, and
    encode(s*B - k*A) == R byte for byte.

The composition (merlin transcript over schnorrkel's labels) has no vector in
the image: "parity unpinned" against upstream for the full signature check.
"""
import hashlib

# ---------------------------------------------------------------- Keccak-f[1600]

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56],
        [27, 20, 39, 8, 14]]
_M64 = (1 << 64) - 1


def _rol(v, r):
    return ((v << r) | (v >> (64 - r))) & _M64 if r else v


def keccak_f1600(state):
    """In place on a bytearray(200) (lanes little-endian, lane (x, y) at 8*(x+5y))."""
    a = [[int.from_bytes(state[8 * (x + 5 * y):8 * (x + 5 * y) + 8], "little") for y in range(5)]
         for x in range(5)]
    for rc in _RC:
        c = [a[x][0] ^ a[x][1] ^ a[x][2] ^ a[x][3] ^ a[x][4] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        a = [[a[x][y] ^ d[x] for y in range(5)] for x in range(5)]
        b = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                b[y][(2 * x + 3 * y) % 5] = _rol(a[x][y], _ROT[x][y])
        a = [[b[x][y] ^ ((~b[(x + 1) % 5][y]) & b[(x + 2) % 5][y]) for y in range(5)] for x in range(5)]
        a[0][0] ^= rc
    for x in range(5):
        for y in range(5):
            state[8 * (x + 5 * y):8 * (x + 5 * y) + 8] = a[x][y].to_bytes(8, "little")


def shake128(data, n):
    """SHAKE128 from keccak_f1600 (the pin against hashlib)."""
    rate = 168
    st = bytearray(200)
    msg = bytearray(data) + b"\x1f"
    msg += bytes((-len(msg)) % rate)
    msg[-1] |= 0x80
    for i in range(0, len(msg), rate):
        for j in range(rate):
            st[j] ^= msg[i + j]
        keccak_f1600(st)
    out = bytearray()
    while len(out) < n:
        out += st[:rate]
        keccak_f1600(st)
    return bytes(out[:n])


# ------------------------------------------------------------------ STROBE-128

STROBE_R = 166
FLAG_I, FLAG_A, FLAG_C, FLAG_T, FLAG_M, FLAG_K = 1, 2, 4, 8, 16, 32


class Strobe128:
    def __init__(self, protocol_label):
        st = bytearray(200)
        st[0:6] = bytes([1, STROBE_R + 2, 1, 0, 1, 96])
        st[6:18] = b"STROBEv1.0.2"
        keccak_f1600(st)
        self.st, self.pos, self.pos_begin, self.cur_flags = st, 0, 0, 0
        self.meta_ad(protocol_label, False)

    def copy(self):
        c = Strobe128.__new__(Strobe128)
        c.st, c.pos, c.pos_begin, c.cur_flags = bytearray(self.st), self.pos, self.pos_begin, self.cur_flags
        return c

    def _run_f(self):
        self.st[self.pos] ^= self.pos_begin
        self.st[self.pos + 1] ^= 0x04
        self.st[STROBE_R + 1] ^= 0x80
        keccak_f1600(self.st)
        self.pos = 0
        self.pos_begin = 0

    def _absorb(self, data):
        for b in data:
            self.st[self.pos] ^= b
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()

    def _squeeze(self, n):
        out = bytearray(n)
        for i in range(n):
            out[i] = self.st[self.pos]
            self.st[self.pos] = 0
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()
        return bytes(out)

    def _begin_op(self, flags, more):
        if more:
            assert self.cur_flags == flags
            return
        assert not flags & FLAG_T
        old_begin = self.pos_begin
        self.pos_begin = self.pos + 1
        self.cur_flags = flags
        self._absorb(bytes([old_begin, flags]))
        if flags & (FLAG_C | FLAG_K) and self.pos != 0:
            self._run_f()

    def meta_ad(self, data, more):
        self._begin_op(FLAG_M | FLAG_A, more)
        self._absorb(data)

    def ad(self, data, more):
        self._begin_op(FLAG_A, more)
        self._absorb(data)

    def prf(self, n, more):
        self._begin_op(FLAG_I | FLAG_A | FLAG_C, more)
        return self._squeeze(n)


class Transcript:
    """merlin::Transcript."""

    def __init__(self, label):
        self.s = Strobe128(b"Merlin v1.0")
        self.append_message(b"dom-sep", label)

    def copy(self):
        t = Transcript.__new__(Transcript)
        t.s = self.s.copy()
        return t

    def append_message(self, label, message):
        self.s.meta_ad(label, False)
        self.s.meta_ad(len(message).to_bytes(4, "little"), True)
        self.s.ad(message, False)

    def challenge_bytes(self, label, n):
        self.s.meta_ad(label, False)
        self.s.meta_ad(n.to_bytes(4, "little"), True)
        return self.s.prf(n, False)


# ------------------------------------------------------- edwards25519 / ristretto255

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)


def _neg(x):
    return x & 1  # IS_NEGATIVE on a reduced value


def _abs(x):
    return (P - x) % P if _neg(x) else x


def sqrt_ratio_m1(u, v):
    """RFC 9496 §4.2 SQRT_RATIO_M1 -> (was_square, r)."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (P - u) % P
    flipped_i = check == (P - u) * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    return correct or flipped, _abs(r)


INVSQRT_A_MINUS_D = sqrt_ratio_m1(1, (-1 - D) % P)[1]
BASE_Y = 4 * pow(5, P - 2, P) % P


def _recover_x(y, sign):
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    ok, x = sqrt_ratio_m1(u, v)
    assert ok
    return (P - x) % P if (x & 1) != sign else x


BASE = (_recover_x(BASE_Y, 0), BASE_Y, 1, _recover_x(BASE_Y, 0) * BASE_Y % P)
IDENTITY = (0, 1, 1, 0)


def point_add(p, q):
    """Extended twisted Edwards coordinates, a = -1 (add-2008-hwcd-3)."""
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = 2 * D * t1 * t2 % P
    d = 2 * z1 * z2 % P
    e, f, g, h = (b - a) % P, (d - c) % P, (d + c) % P, (b + a) % P
    return e * f % P, g * h % P, f * g % P, e * h % P


def point_neg(p):
    x, y, z, t = p
    return (P - x) % P, y, z, (P - t) % P


def scalar_mult(k, p):
    acc = IDENTITY
    for i in reversed(range(k.bit_length())):
        acc = point_add(acc, acc)
        if k >> i & 1:
            acc = point_add(acc, p)
    return acc


def ristretto_decode(b):
    """RFC 9496 §4.3.1; None if invalid."""
    if len(b) != 32:
        return None
    s = int.from_bytes(b, "little")
    if s >= P or _neg(s):
        return None
    ss = s * s % P
    u1, u2 = (1 - ss) % P, (1 + ss) % P
    u2_sqr = u2 * u2 % P
    v = (-(D * u1 % P * u1) - u2_sqr) % P
    was_square, invsqrt = sqrt_ratio_m1(1, v * u2_sqr % P)
    den_x = invsqrt * u2 % P
    den_y = invsqrt * den_x % P * v % P
    x = _abs(2 * s * den_x % P)
    y = u1 * den_y % P
    t = x * y % P
    if not was_square or _neg(t) or y == 0:
        return None
    return x, y, 1, t


def ristretto_encode(p):
    """RFC 9496 §4.3.2."""
    x0, y0, z0, t0 = p
    u1 = (z0 + y0) * (z0 - y0) % P
    u2 = x0 * y0 % P
    _, invsqrt = sqrt_ratio_m1(1, u1 * u2 % P * u2 % P)
    den1, den2 = invsqrt * u1 % P, invsqrt * u2 % P
    z_inv = den1 * den2 % P * t0 % P
    ix0, iy0 = x0 * SQRT_M1 % P, y0 * SQRT_M1 % P
    enchanted = den1 * INVSQRT_A_MINUS_D % P
    rotate = _neg(t0 * z_inv % P)
    x, y, den_inv = (iy0, ix0, enchanted) if rotate else (x0, y0, den2)
    if _neg(x * z_inv % P):
        y = (P - y) % P
    s = _abs(den_inv * (z0 - y) % P)
    return s.to_bytes(32, "little")


# ------------------------------------------------------------------ schnorrkel

CHALLENGE_CONTEXT = b"grapevine-challenge"  # types/src/lib.rs:13


def signing_transcript(context, message):
    t = Transcript(b"SigningContext")
    t.append_message(b"", context)
    t.append_message(b"sign-bytes", message)
    return t


def challenge_scalar(t, pk, r_bytes):
    t.append_message(b"proto-name", b"Schnorr-sig")
    t.append_message(b"sign:pk", pk)
    t.append_message(b"sign:R", r_bytes)
    return int.from_bytes(t.challenge_bytes(b"sign:c", 64), "little") % L


def public_key(secret_scalar):
    return ristretto_encode(scalar_mult(secret_scalar, BASE))


def sign(secret_scalar, message, nonce, context=CHALLENGE_CONTEXT):
    """A schnorrkel signature with an explicit nonce scalar (the real signer
    derives it from a transcript RNG; any nonce gives a valid signature)."""
    pk = public_key(secret_scalar)
    r_bytes = ristretto_encode(scalar_mult(nonce % L, BASE))
    k = challenge_scalar(signing_transcript(context, message), pk, r_bytes)
    s = (k * secret_scalar + nonce) % L
    sb = bytearray(s.to_bytes(32, "little"))
    sb[31] |= 0x80  # schnorrkel's marker bit
    return r_bytes + bytes(sb)


def verify(pk, message, sig, context=CHALLENGE_CONTEXT):
    if len(sig) != 64 or len(pk) != 32 or not sig[63] & 0x80:
        return False
    r_bytes = bytes(sig[:32])
    sb = bytearray(sig[32:])
    sb[31] &= 0x7F
    s = int.from_bytes(sb, "little")
    if s >= L:
        return False
    a = ristretto_decode(bytes(pk))
    if a is None:
        return False
    k = challenge_scalar(signing_transcript(context, bytes(message)), bytes(pk), r_bytes)
    rr = point_add(scalar_mult(s, BASE), scalar_mult(k, point_neg(a)))
    return ristretto_encode(rr) == r_bytes


# ------------------------------------------------- Ed25519 (pin of the curve code)

def _ed_encode(p):
    x, y, z, _ = p
    zi = pow(z, P - 2, P)
    x, y = x * zi % P, y * zi % P
    return (y | (x & 1) << 255).to_bytes(32, "little")


def _ed_decode(b):
    v = int.from_bytes(b, "little")
    y, sign = v & ((1 << 255) - 1), v >> 255
    if y >= P:
        return None
    u, w = (y * y - 1) % P, (D * y * y + 1) % P
    ok, x = sqrt_ratio_m1(u, w)
    if not ok or (x == 0 and sign):
        return None
    if (x & 1) != sign:
        x = P - x
    return x, y, 1, x * y % P


def ed25519_verify(pk, msg, sig):
    """RFC 8032 §5.1.7 (cofactorless), on this file's point arithmetic."""
    a = _ed_decode(pk)
    r = _ed_decode(sig[:32])
    s = int.from_bytes(sig[32:], "little")
    if a is None or r is None or s >= L:
        return False
    h = int.from_bytes(hashlib.sha512(sig[:32] + pk + msg).digest(), "little") % L
    lhs = _ed_encode(scalar_mult(s, BASE))
    rhs = _ed_encode(point_add(r, scalar_mult(h, a)))
    return lhs == rhs
