/*
 * gvs_seal.c — TEST INFRASTRUCTURE ONLY (see gvs_oracle.h).
 *
 * Plain C restatement of the authenticated-storage format of DESIGN.md §8
 * (the config-5 mode that mirrors mc-oblivious's untrusted ORAM storage:
 * AES-CTR encryption plus a BLAKE2b MAC per stored row).  Written from the
 * primary specs, independently of the engine's table-driven kernels:
 *   AES-128: FIPS-197 §5.1-5.2 (byte-oriented SubBytes/ShiftRows/MixColumns);
 *   BLAKE2b: RFC 7693 §3 (parameter block per BLAKE2 spec §2.8).
 * Pinned by tests/test_seal.py against FIPS-197 Appendix C.1, SP 800-38A
 * F.5.1, the openssl CLI and Python's hashlib.blake2b.
 */
#include <stdint.h>
#include <string.h>

#include "gvs_oracle.h"

/* ---------------------------------------------------------------- AES-128 */

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  while (b) {
    if (b & 1) p ^= a;
    a = xtime(a);
    b >>= 1;
  }
  return p;
}

/* S-box from its definition (FIPS-197 §5.1.1): multiplicative inverse in
 * GF(2^8) followed by the affine transform. */
static uint8_t sbox(uint8_t x) {
  uint8_t inv = 0;
  if (x) {
    for (int c = 1; c < 256; ++c)
      if (gmul(x, (uint8_t)c) == 1) {
        inv = (uint8_t)c;
        break;
      }
  }
  uint8_t s = inv, r = inv;
  for (int i = 0; i < 4; ++i) {
    r = (uint8_t)((r << 1) | (r >> 7));
    s ^= r;
  }
  return (uint8_t)(s ^ 0x63);
}

static uint8_t SBOX[256];
static int sbox_ready = 0;
static void sbox_init(void) {
  if (sbox_ready) return;
  for (int i = 0; i < 256; ++i) SBOX[i] = sbox((uint8_t)i);
  sbox_ready = 1;
}

void gvo_aes128_expand(const uint8_t key[16], uint8_t rk[176]) {
  sbox_init();
  memcpy(rk, key, 16);
  uint8_t rcon = 1;
  for (int i = 4; i < 44; ++i) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % 4 == 0) {
      uint8_t u = t[0];
      t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
      t[1] = SBOX[t[2]];
      t[2] = SBOX[t[3]];
      t[3] = SBOX[u];
      rcon = xtime(rcon);
    }
    for (int k = 0; k < 4; ++k) rk[4 * i + k] = (uint8_t)(rk[4 * (i - 4) + k] ^ t[k]);
  }
}

void gvo_aes128_encrypt(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
  sbox_init();
  uint8_t s[16];
  for (int k = 0; k < 16; ++k) s[k] = (uint8_t)(in[k] ^ rk[k]);
  for (int r = 1; r <= 10; ++r) {
    uint8_t t[16];
    /* SubBytes + ShiftRows: state is column-major, s[4c + row] */
    for (int c = 0; c < 4; ++c)
      for (int row = 0; row < 4; ++row) t[4 * c + row] = SBOX[s[4 * ((c + row) % 4) + row]];
    if (r < 10) {
      for (int c = 0; c < 4; ++c) { /* MixColumns */
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c] = (uint8_t)(xtime(a0) ^ (xtime(a1) ^ a1) ^ a2 ^ a3);
        s[4 * c + 1] = (uint8_t)(a0 ^ xtime(a1) ^ (xtime(a2) ^ a2) ^ a3);
        s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xtime(a2) ^ (xtime(a3) ^ a3));
        s[4 * c + 3] = (uint8_t)((xtime(a0) ^ a0) ^ a1 ^ a2 ^ xtime(a3));
      }
    } else {
      memcpy(s, t, 16);
    }
    for (int k = 0; k < 16; ++k) s[k] ^= rk[16 * r + k];
  }
  memcpy(out, s, 16);
}

/* ---------------------------------------------------------------- BLAKE2b */

static const uint64_t B2IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static uint64_t rotr64(uint64_t x, int r) { return (x >> r) | (x << (64 - r)); }
static uint64_t le64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

typedef struct {
  uint64_t h[8];
  uint64_t t;
  uint8_t buf[128];
  size_t n;
  size_t outlen;
} b2ctx;

static void b2_F(b2ctx *c, int last) {
  uint64_t v[16], m[16];
  for (int i = 0; i < 16; ++i) m[i] = le64(c->buf + 8 * i);
  for (int i = 0; i < 8; ++i) {
    v[i] = c->h[i];
    v[i + 8] = B2IV[i];
  }
  v[12] ^= c->t;
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; ++r) {
    const uint8_t *s = SIGMA[r];
#define G(a, b, cc, d, x, y)          \
  v[a] = v[a] + v[b] + (x);           \
  v[d] = rotr64(v[d] ^ v[a], 32);     \
  v[cc] = v[cc] + v[d];               \
  v[b] = rotr64(v[b] ^ v[cc], 24);    \
  v[a] = v[a] + v[b] + (y);           \
  v[d] = rotr64(v[d] ^ v[a], 16);     \
  v[cc] = v[cc] + v[d];               \
  v[b] = rotr64(v[b] ^ v[cc], 63);
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
#undef G
  }
  for (int i = 0; i < 8; ++i) c->h[i] ^= v[i] ^ v[i + 8];
}

static void b2_update(b2ctx *c, const uint8_t *p, size_t len) {
  while (len) {
    if (c->n == 128) { /* a full buffered block that is not the last one */
      c->t += 128;
      b2_F(c, 0);
      c->n = 0;
    }
    size_t k = 128 - c->n < len ? 128 - c->n : len;
    memcpy(c->buf + c->n, p, k);
    c->n += k;
    p += k;
    len -= k;
  }
}

/* BLAKE2b with digest length outlen, optional key, optional 16-byte person */
void gvo_blake2b(const uint8_t *key, size_t keylen, const uint8_t *person, const uint8_t *msg,
                 size_t len, uint8_t *out, size_t outlen) {
  b2ctx c;
  memset(&c, 0, sizeof c);
  uint8_t pb[64];
  memset(pb, 0, 64);
  pb[0] = (uint8_t)outlen;
  pb[1] = (uint8_t)keylen;
  pb[2] = 1; /* fanout */
  pb[3] = 1; /* depth */
  if (person) memcpy(pb + 48, person, 16);
  for (int i = 0; i < 8; ++i) c.h[i] = B2IV[i] ^ le64(pb + 8 * i);
  c.outlen = outlen;
  if (keylen) {
    uint8_t kb[128];
    memset(kb, 0, 128);
    memcpy(kb, key, keylen);
    b2_update(&c, kb, 128);
  }
  b2_update(&c, msg, len);
  c.t += c.n;
  memset(c.buf + c.n, 0, 128 - c.n);
  b2_F(&c, 1);
  uint8_t full[64];
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 8; ++k) full[8 * i + k] = (uint8_t)(c.h[i] >> (8 * k));
  memcpy(out, full, outlen);
}

/* ------------------------------------------------------ storage format [D] */

void gvo_storage_keys(const uint8_t secret[32], uint8_t aes_key[16], uint8_t mac_key[32]) {
  static const char a[] = "gvs storage aes", m[] = "gvs storage mac";
  gvo_blake2b(secret, 32, NULL, (const uint8_t *)a, sizeof a - 1, aes_key, 16);
  gvo_blake2b(secret, 32, NULL, (const uint8_t *)m, sizeof m - 1, mac_key, 32);
}

static void put_le(uint8_t *p, uint64_t v, int n) {
  for (int i = 0; i < n; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

/* Row-hash keys of the message tables (round 6): 1216 bytes, blocks j = 0..18
 * of BLAKE2b-512(key = mac_key, "gvs-uhash-" | byte j).  Words 0..267 are the
 * NH key (little-endian u32), then 16 L3 keys (le64 mod 2^36, minus p36 when
 * at least p36 = 2^36 - 5) and 4 L3 pads (le32). */
#define GVO_P36 ((1ull << 36) - 5)
void gvo_uhash_keys(const uint8_t secret[32], uint32_t nh[268], uint64_t l3k[16], uint32_t l3p[4]) {
  uint8_t ak[16], mk[32], kb[19 * 64];
  gvo_storage_keys(secret, ak, mk);
  for (int j = 0; j < 19; ++j) {
    uint8_t msg[11] = {'g', 'v', 's', '-', 'u', 'h', 'a', 's', 'h', '-', (uint8_t)j};
    gvo_blake2b(mk, 32, NULL, msg, sizeof msg, kb + 64 * j, 64);
  }
  for (int w = 0; w < 268; ++w)
    nh[w] = (uint32_t)kb[4 * w] | (uint32_t)kb[4 * w + 1] << 8 | (uint32_t)kb[4 * w + 2] << 16 |
            (uint32_t)kb[4 * w + 3] << 24;
  for (int i = 0; i < 16; ++i) {
    uint64_t k = le64(kb + 1072 + 8 * i) & ((1ull << 36) - 1);
    l3k[i] = k >= GVO_P36 ? k - GVO_P36 : k;
  }
  for (int t = 0; t < 4; ++t) {
    const uint8_t *q = kb + 1200 + 4 * t;
    l3p[t] = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
  }
}

/* G(ct), the 128-bit hash of a 1024-byte message-table ciphertext: the
 * layers of UMAC's UHASH-128 (RFC 4418 §5) for a message of one 1024-byte
 * block, four iterations t with the NH key shifted by 4 words (16 bytes) each:
 *   S_t = sum_j ((m[2j] + k[4t + 2j]) mod 2^32) * ((m[2j+1] + k[4t + 2j+1]) mod 2^32)
 *         mod 2^64 over the 256 little-endian words m of the ciphertext (NH);
 *   Y_t = ((sum_c chunk_c(S_t) * l3k[4t + c]) mod p36) mod 2^32, xor l3p[t]
 *         with chunk_c the 16-bit pieces of S_t, most significant first (L3;
 *         L2 of a one-block message is the identity, its upper 64 bits zero);
 *   G = le32(Y_0) | le32(Y_1) | le32(Y_2) | le32(Y_3). */
void gvo_row_hash(const uint32_t nh[268], const uint64_t l3k[16], const uint32_t l3p[4],
                  const uint8_t ct[1024], uint8_t out[16]) {
  uint32_t m[256];
  for (int w = 0; w < 256; ++w)
    m[w] = (uint32_t)ct[4 * w] | (uint32_t)ct[4 * w + 1] << 8 | (uint32_t)ct[4 * w + 2] << 16 |
           (uint32_t)ct[4 * w + 3] << 24;
  for (int t = 0; t < 4; ++t) {
    uint64_t s = 0;
    for (int j = 0; j < 128; ++j)
      s += (uint64_t)(uint32_t)(m[2 * j] + nh[4 * t + 2 * j]) * (uint64_t)(uint32_t)(m[2 * j + 1] + nh[4 * t + 2 * j + 1]);
    uint64_t y = 0;
    for (int c = 0; c < 4; ++c) {
      const uint64_t chunk = (s >> (48 - 16 * c)) & 0xffffu;
      y = (y + chunk * l3k[4 * t + c]) % GVO_P36;
    }
    put_le(out + 4 * t, (uint32_t)y ^ l3p[t], 4);
  }
}

/* Seal one row: ct = pt ^ AES-CTR keystream; tag = H ^ G, with
 *   H   = every table but the map directory: AES-128_kh(le64(row) | le32(epoch) | le32(table)),
 *         for the tables with a side entry (1, 2) AES-128_kh(that ^ side ct);
 *         map directory (3): BLAKE2b-128(key = mac_key, person = "gvs-head" | 0^8,
 *                     le64(row) | le32(epoch) | le32(table) | 0^16)
 *   G   = gvo_row_hash(ct) for every table but the map directory (a
 *         Carter-Wegman MAC, H the PRF of a nonce never sealed twice; the
 *         mailbox table since the end of round 6);
 *         for the map directory (table 3) the XOR of its 4 leaf PRFs
 *         L_i = BLAKE2b-128(key = mac_key, person = "gvs-leaf" | le32(i) | le32(1), leaf i of 256 B)
 * table: 0 message rows, 1 mailbox rows, 2 pending final states (P, by
 * position, side = target row), 3 the key-value map's directory rows,
 * 0x100 a message row whose final state is
 * pending in P (header only: its keystream and leaves are table 0's; the CTR
 * block carries the table's low byte). 
 * side_pt may be NULL (message rows); then side_ct is not written and 16 zero
 * bytes stand in for it. */
void gvo_seal_row(const uint8_t secret[32], uint32_t table, uint64_t row, uint32_t epoch,
                  const uint8_t pt[1024], const uint8_t *side_pt, uint8_t ct[1024],
                  uint8_t *side_ct, uint8_t tag[16]) {
  uint8_t ak[16], mk[32], rk[176];
  gvo_storage_keys(secret, ak, mk);
  gvo_aes128_expand(ak, rk);
  uint8_t blk[16], ks[16];
  const uint32_t nblk = side_pt ? 65 : 64;
  for (uint32_t j = 0; j < nblk; ++j) {
    put_le(blk, row, 8);
    put_le(blk + 8, epoch, 4);
    blk[12] = (uint8_t)table;
    blk[13] = 0;
    blk[14] = (uint8_t)(j >> 8);
    blk[15] = (uint8_t)j;
    gvo_aes128_encrypt(rk, blk, ks);
    const uint8_t *src = j < 64 ? pt + 16 * j : side_pt;
    uint8_t *dst = j < 64 ? ct + 16 * j : side_ct;
    for (int k = 0; k < 16; ++k) dst[k] = (uint8_t)(src[k] ^ ks[k]);
  }
  uint8_t hdr[32], head_person[16] = {'g', 'v', 's', '-', 'h', 'e', 'a', 'd'};
  memset(hdr, 0, sizeof hdr);
  put_le(hdr, row, 8);
  put_le(hdr + 8, epoch, 4);
  put_le(hdr + 12, table, 4);
  if (side_pt) memcpy(hdr + 16, side_ct, 16);
  if (table != 3) {
    /* H = AES_kh(nonce), or AES_kh(AES_kh(nonce) ^ side ct) for the tables
     * with a side entry (mailboxes, table 1; P, table 2): a PRF of a
     * fixed-length input per table, kh = BLAKE2b-128(key = secret, "gvs storage head") */
    static const char hk[] = "gvs storage head";
    uint8_t kh[16], rkh[176];
    gvo_blake2b(secret, 32, NULL, (const uint8_t *)hk, sizeof hk - 1, kh, 16);
    gvo_aes128_expand(kh, rkh);
    gvo_aes128_encrypt(rkh, hdr, tag);
    if (side_pt) {
      uint8_t x[16];
      for (int k = 0; k < 16; ++k) x[k] = (uint8_t)(tag[k] ^ side_ct[k]);
      gvo_aes128_encrypt(rkh, x, tag);
    }
  } else {
    gvo_blake2b(mk, 32, head_person, hdr, sizeof hdr, tag, 16);
  }
  if (table != 3) { /* every table but the map directory: the row hash */
    uint32_t nh[268], l3p[4];
    uint64_t l3k[16];
    uint8_t g[16];
    gvo_uhash_keys(secret, nh, l3k, l3p);
    gvo_row_hash(nh, l3k, l3p, ct, g);
    for (int k = 0; k < 16; ++k) tag[k] ^= g[k];
    return;
  }
  /* map directory: 4 leaves of 256 B */
  const uint32_t nl = 4, lb = 1024 / nl;
  for (uint32_t i = 0; i < nl; ++i) {
    uint8_t person[16] = {'g', 'v', 's', '-', 'l', 'e', 'a', 'f'}, l[16];
    put_le(person + 8, i, 4);
    put_le(person + 12, table & 1, 4);
    gvo_blake2b(mk, 32, person, ct + lb * i, lb, l, 16);
    for (int k = 0; k < 16; ++k) tag[k] ^= l[k];
  }
}
