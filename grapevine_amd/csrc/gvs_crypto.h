// gvs_crypto.h — primitives of the authenticated-storage mode:
// AES-128 (FIPS-197) in counter mode and BLAKE2b (RFC 7693), written for gfx950
// and shared with the host (key schedule, tables, the precomputed MAC key
// state, host-side unsealing for test dumps).
//
// Storage format of one row (message row: 1024 B; mailbox row: 1024 B + its
// 16-B side entry), sealed at epoch e (the number of batches the store has
// applied; every row is rewritten every batch, so e is also its version):
//   keystream block j = AES_k(le64(row) | le32(e) | table | 0 | be16(j))
//                       (standard CTR, counter in the last two bytes)
//   ct_j = pt_j ^ keystream_j          (j = 0..63 row, j = 64 side entry)
//   H    = every table but the map directory: AES-128_kh(le64(row) | le32(e) |
//          le32(table)), then AES-128_kh of that ^ side_ct for the tables with a
//          side entry, 1 and 2 (head_aes; kh = BLAKE2b-128(key = secret,
//          "gvs storage head"));
//          map directory (3): BLAKE2b-128(key = mac_key, person = "gvs-head" | 0^8,
//                      le64(row) | le32(e) | le32(table) | 0^16)
//   tag  = H ^ G(ct)
//   G    = every table but the map directory (tables 0, 1, 2 and 0x100): the
//          row hash (round 6): the layers of UMAC's UHASH-128 (RFC 4418 §5) for
//          one 1024-byte block, four NH iterations over the row's 256
//          little-endian words with the key shifted 16 bytes per iteration,
//          each reduced to 32 bits by the p36 inner product (L3) and padded:
//            S_t = sum_j ((m[2j] + k[4t+2j]) mod 2^32)((m[2j+1] + k[4t+2j+1]) mod 2^32) mod 2^64
//            Y_t = ((sum_c chunk_c(S_t) l3k[4t+c]) mod (2^36 - 5)) mod 2^32 ^ l3p[t]
//          (chunk_c the 16-bit pieces of S_t, most significant first), keys
//          from BLAKE2b-512(key = mac_key, "gvs-uhash-" | byte j), j < 19;
//          map directory (3): the XOR of its four leaf PRFs
//            L_i = BLAKE2b-128(key = mac_key, person = "gvs-leaf" | le32(i) | le32(1),
//                              leaf i of ct, 256 B)
// The row-hash tables' tag is a Carter-Wegman MAC: H is the PRF of a value
// that is never sealed twice, (row, e, table), and G an almost-XOR-universal
// hash of the row (UHASH-128's bound, ~2^-120 per forgery attempt; a store
// stops at its first bad tag).  NH costs one 32x32->64 multiply-add per 8
// bytes where BLAKE2b costs ~15 three-source operations: the sealed message
// pass is bound by VALU issue.  The map directory keeps the
// XOR-MAC with a counter term (Bellare-Guerin-Rogaway's XMACC).  The tag binds
// row, table and epoch, so a replayed, moved or spliced row fails.  The key block of each keyed hash
// depends only on (key, person): its state is computed once (SealCtx), so a
// 128-B leaf costs one compression, a 256-B leaf two and the header one; the
// header depends on no row data, so the message pass computes it for 64 rows
// at a time.  Message rows use 128-B leaves so that a wave of 8 rows hashes
// its 64 leaves in 64 lanes (the message pass runs 8 rows per wave, 2 waves
// per SIMD, gvs_txn.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gvs {

// ------------------------------------------------------------------ AES-128

struct AesRk {
  uint32_t w[44];  // expanded encryption key, big-endian words (FIPS-197 §5.2)
};

__host__ __device__ inline uint32_t ror32(uint32_t x, int r) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, (uint32_t)r);
#else
  return (x >> r) | (x << (32 - r));
#endif
}
__host__ __device__ inline uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96)
__host__ __device__ inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// te0[x] = S[x]*{02} | S[x] | S[x] | S[x]*{03} (big-endian bytes); the other
// three round tables are byte rotations of it, S[x] = (te0[x] >> 8) & 0xff.
// te_at(tab, s, k) = te0[byte k of s] (k = 3 is the most significant byte).
// Host: a plain 256-word array.  Device: the LDS replicas of gvs_seal_dev.h.
__host__ __device__ inline uint32_t te_at(const uint32_t* tab, uint32_t s, int k) {
  return tab[(s >> (8 * k)) & 0xffu];
}

template <typename Tab>
__host__ __device__ __attribute__((always_inline)) inline void aes128_encrypt_words(const AesRk& rk, const Tab& te0, uint32_t s0,
                                                     uint32_t s1, uint32_t s2, uint32_t s3,
                                                     uint32_t out[4]) {
  s0 ^= rk.w[0];
  s1 ^= rk.w[1];
  s2 ^= rk.w[2];
  s3 ^= rk.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    const uint32_t t0 = xor3(xor3(te_at(te0, s0, 3), ror32(te_at(te0, s1, 2), 8),
                                  ror32(te_at(te0, s2, 1), 16)),
                             ror32(te_at(te0, s3, 0), 24), rk.w[4 * r]);
    const uint32_t t1 = xor3(xor3(te_at(te0, s1, 3), ror32(te_at(te0, s2, 2), 8),
                                  ror32(te_at(te0, s3, 1), 16)),
                             ror32(te_at(te0, s0, 0), 24), rk.w[4 * r + 1]);
    const uint32_t t2 = xor3(xor3(te_at(te0, s2, 3), ror32(te_at(te0, s3, 2), 8),
                                  ror32(te_at(te0, s0, 1), 16)),
                             ror32(te_at(te0, s1, 0), 24), rk.w[4 * r + 2]);
    const uint32_t t3 = xor3(xor3(te_at(te0, s3, 3), ror32(te_at(te0, s0, 2), 8),
                                  ror32(te_at(te0, s1, 1), 16)),
                             ror32(te_at(te0, s2, 0), 24), rk.w[4 * r + 3]);
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
#define GVS_SB(x, k) ((te_at(te0, (x), (k)) >> 8) & 0xffu)
  out[0] = (GVS_SB(s0, 3) << 24 | GVS_SB(s1, 2) << 16 | GVS_SB(s2, 1) << 8 | GVS_SB(s3, 0)) ^ rk.w[40];
  out[1] = (GVS_SB(s1, 3) << 24 | GVS_SB(s2, 2) << 16 | GVS_SB(s3, 1) << 8 | GVS_SB(s0, 0)) ^ rk.w[41];
  out[2] = (GVS_SB(s2, 3) << 24 | GVS_SB(s3, 2) << 16 | GVS_SB(s0, 1) << 8 | GVS_SB(s1, 0)) ^ rk.w[42];
  out[3] = (GVS_SB(s3, 3) << 24 | GVS_SB(s0, 2) << 16 | GVS_SB(s1, 1) << 8 | GVS_SB(s2, 0)) ^ rk.w[43];
#undef GVS_SB
}

// keystream block j of (table, row, epoch) as four little-endian data words
template <typename Tab>
__host__ __device__ inline uint4 ctr_keystream(const AesRk& rk, const Tab& te0, uint32_t table,
                                               uint64_t row, uint32_t epoch, uint32_t j) {
  uint32_t o[4];
  aes128_encrypt_words(rk, te0, bswap32((uint32_t)row), bswap32((uint32_t)(row >> 32)),
                       bswap32(epoch), (table << 24) | j, o);
  return make_uint4(bswap32(o[0]), bswap32(o[1]), bswap32(o[2]), bswap32(o[3]));
}

// H of a row of every table but the map directory: AES-128 under kh of the
// nonce le64(row) | le32(epoch) | le32(table), and for the tables with a side
// entry (mailboxes 1, P 2) AES again of that XOR the side ciphertext: a PRF of a fixed-
// length input per table.  out = H as two little-endian 64-bit words.
template <typename Tab>
__host__ __device__ __attribute__((always_inline)) inline void head_aes_w(const AesRk& rkh, const Tab& te0,
                                                                         uint64_t row, uint32_t epoch,
                                                                         uint32_t table, bool with_side,
                                                                         uint64_t s0, uint64_t s1,
                                                                         uint64_t out[2]) {
  uint32_t o[4];
  aes128_encrypt_words(rkh, te0, bswap32((uint32_t)row), bswap32((uint32_t)(row >> 32)), bswap32(epoch),
                       bswap32(table), o);
  if (with_side)
    aes128_encrypt_words(rkh, te0, o[0] ^ bswap32((uint32_t)s0), o[1] ^ bswap32((uint32_t)(s0 >> 32)),
                         o[2] ^ bswap32((uint32_t)s1), o[3] ^ bswap32((uint32_t)(s1 >> 32)), o);
  out[0] = (uint64_t)bswap32(o[0]) | ((uint64_t)bswap32(o[1]) << 32);
  out[1] = (uint64_t)bswap32(o[2]) | ((uint64_t)bswap32(o[3]) << 32);
}
template <typename Tab>
__host__ __device__ __attribute__((always_inline)) inline void head_aes(const AesRk& rkh, const Tab& te0, uint64_t row,
                                                                       uint32_t epoch, uint32_t table,
                                                                       const uint64_t* side, uint64_t out[2]) {
  head_aes_w(rkh, te0, row, epoch, table, side != nullptr, side ? side[0] : 0ull, side ? side[1] : 0ull, out);
}

// --------------------------------------------------------------- BLAKE2b

struct B2State {
  uint64_t h[8];
};

// 64-bit rotate right by a constant; on the device two v_alignbit_b32 (a
// rotate by 32 is a register swap)
__host__ __device__ inline uint64_t b2_rotr(uint64_t x, int r) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (r >= 32) {
    const uint32_t t = lo;
    lo = hi;
    hi = t;
    r -= 32;
  }
  if (r == 0) return ((uint64_t)hi << 32) | lo;
  const uint32_t nlo = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)r);
  const uint32_t nhi = __builtin_amdgcn_alignbit(lo, hi, (uint32_t)r);
  return ((uint64_t)nhi << 32) | nlo;
#else
  return (x >> r) | (x << (64 - r));
#endif
}

__host__ __device__ inline void b2_iv(uint64_t iv[8]) {
  iv[0] = 0x6a09e667f3bcc908ULL;
  iv[1] = 0xbb67ae8584caa73bULL;
  iv[2] = 0x3c6ef372fe94f82bULL;
  iv[3] = 0xa54ff53a5f1d36f1ULL;
  iv[4] = 0x510e527fade682d1ULL;
  iv[5] = 0x9b05688c2b3e6c1fULL;
  iv[6] = 0x1f83d9abfb41bd6bULL;
  iv[7] = 0x5be0cd19137e2179ULL;
}

#define GVS_B2G(a, b, c, d, x, y)    \
  do {                               \
    v[a] = v[a] + v[b] + (x);        \
    v[d] = b2_rotr(v[d] ^ v[a], 32); \
    v[c] = v[c] + v[d];              \
    v[b] = b2_rotr(v[b] ^ v[c], 24); \
    v[a] = v[a] + v[b] + (y);        \
    v[d] = b2_rotr(v[d] ^ v[a], 16); \
    v[c] = v[c] + v[d];              \
    v[b] = b2_rotr(v[b] ^ v[c], 63); \
  } while (0)

// message schedule sigma[r] (RFC 7693 §2.7); rounds 10 and 11 reuse rows 0, 1
__host__ __device__ constexpr int b2_sigma(int r, int i) {
  constexpr uint8_t S[10][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
  return S[r % 10][i];
}

// One round with compile-time message indices: every m[] access is static,
// so the message block stays in registers (a runtime index would make the
// compiler move the array to scratch or LDS).
template <int R>
__host__ __device__ __attribute__((always_inline)) inline void b2_round(uint64_t (&v)[16], const uint64_t* m) {
  GVS_B2G(0, 4, 8, 12, m[b2_sigma(R, 0)], m[b2_sigma(R, 1)]);
  GVS_B2G(1, 5, 9, 13, m[b2_sigma(R, 2)], m[b2_sigma(R, 3)]);
  GVS_B2G(2, 6, 10, 14, m[b2_sigma(R, 4)], m[b2_sigma(R, 5)]);
  GVS_B2G(3, 7, 11, 15, m[b2_sigma(R, 6)], m[b2_sigma(R, 7)]);
  GVS_B2G(0, 5, 10, 15, m[b2_sigma(R, 8)], m[b2_sigma(R, 9)]);
  GVS_B2G(1, 6, 11, 12, m[b2_sigma(R, 10)], m[b2_sigma(R, 11)]);
  GVS_B2G(2, 7, 8, 13, m[b2_sigma(R, 12)], m[b2_sigma(R, 13)]);
  GVS_B2G(3, 4, 9, 14, m[b2_sigma(R, 14)], m[b2_sigma(R, 15)]);
}

// RFC 7693 §3.2 compression F; t = byte offset after this block, last = final block
__host__ __device__ __attribute__((always_inline)) inline void b2_compress(B2State& s, const uint64_t m[16], uint64_t t,
                                            bool last) {
  uint64_t v[16], iv[8];
  b2_iv(iv);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = s.h[i];
    v[i + 8] = iv[i];
  }
  v[12] ^= t;
  v[14] ^= last ? ~0ull : 0ull;  // a select: `last` may differ across lanes
  b2_round<0>(v, m);
  b2_round<1>(v, m);
  b2_round<2>(v, m);
  b2_round<3>(v, m);
  b2_round<4>(v, m);
  b2_round<5>(v, m);
  b2_round<6>(v, m);
  b2_round<7>(v, m);
  b2_round<8>(v, m);
  b2_round<9>(v, m);
  b2_round<10>(v, m);
  b2_round<11>(v, m);
#pragma unroll
  for (int i = 0; i < 8; ++i) s.h[i] ^= v[i] ^ v[i + 8];
}
#undef GVS_B2G

// initial state from the parameter block: digest length nn, key length kk,
// sequential mode, personalisation (p0, p1) (RFC 7693 §2.5, BLAKE2 §2.8)
__host__ __device__ inline B2State b2_init(uint32_t nn, uint32_t kk, uint64_t p0, uint64_t p1) {
  B2State s;
  b2_iv(s.h);
  s.h[0] ^= 0x01010000ULL ^ ((uint64_t)kk << 8) ^ nn;
  s.h[6] ^= p0;
  s.h[7] ^= p1;
  return s;
}

constexpr uint64_t kLeafPerson0 = 0x6661656c2d737667ULL;  // "gvs-leaf" little-endian
constexpr uint64_t kHeadPerson0 = 0x646165682d737667ULL;  // "gvs-head" little-endian

// state of keyed BLAKE2b-128 (32-byte key) with personalisation (p0, p1)
// after its key block
__host__ __device__ inline B2State b2_keyed_state(const uint8_t key[32], uint64_t p0, uint64_t p1) {
  B2State s = b2_init(16, 32, p0, p1);
  uint64_t m[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint64_t w = 0;
    if (k < 4)
      for (int b = 7; b >= 0; --b) w = (w << 8) | key[8 * k + b];
    m[k] = w;
  }
  b2_compress(s, m, 128, false);
  return s;
}

// L_i over one 256-byte leaf (m = its 32 little-endian words), from the
// keyed state of leaf i (mailbox table)
__host__ __device__ __attribute__((always_inline)) inline void leaf_prf(const B2State& k,
                                                                       const uint64_t m[32],
                                                                       uint64_t out[2]) {
  B2State s = k;
  b2_compress(s, m, 128 + 128, false);
  b2_compress(s, m + 16, 128 + 256, true);
  out[0] = s.h[0];
  out[1] = s.h[1];
}

// the 32-byte header message block
__host__ __device__ inline void header_block(uint64_t row, uint32_t epoch, uint32_t table,
                                             const uint64_t side[2], uint64_t m[16]) {
  m[0] = row;
  m[1] = (uint64_t)epoch | ((uint64_t)table << 32);
  m[2] = side[0];
  m[3] = side[1];
#pragma unroll
  for (int k = 4; k < 16; ++k) m[k] = 0;
}

// ------------------------------------------------------- message row hash

constexpr uint32_t kNhWords = 268;            // NH key: 256 words + 3 shifts of 4
constexpr uint64_t kP36 = (1ull << 36) - 5;

// NH of 16 word pairs w[0..31] against key words k(o + 4t + i) for the four
// iterations t: s[t] += sum over pairs (mod 2^64).  `k` is any indexable key
// (LDS, global or host array); o = 32 * leaf for a 128-B leaf of the row.
template <typename K>
__host__ __device__ __attribute__((always_inline)) inline void nh_words(const K& k, uint32_t o,
                                                                       const uint32_t (&w)[32],
                                                                       uint64_t s[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t a = w[2 * j] + k[o + 4 * t + 2 * j], b = w[2 * j + 1] + k[o + 4 * t + 2 * j + 1];
      s[t] += (uint64_t)a * (uint64_t)b;  // one v_mad_u64_u32
    }
  }
}

// L3 of the four NH sums: out = G as two little-endian 64-bit words
__host__ __device__ inline void row_hash_fin(const uint64_t s[4], const uint64_t l3k[16], const uint32_t l3p[4],
                                             uint64_t out[2]) {
  uint32_t y[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    uint64_t acc = 0;  // < 4 * 2^16 * 2^36
#pragma unroll
    for (int c = 0; c < 4; ++c) acc += ((s[t] >> (48 - 16 * c)) & 0xffffull) * l3k[4 * t + c];
    uint64_t x = (acc & ((1ull << 36) - 1)) + 5ull * (acc >> 36);  // 2^36 = 5 mod p36
    x = x >= kP36 ? x - kP36 : x;
    y[t] = (uint32_t)x ^ l3p[t];
  }
  out[0] = (uint64_t)y[0] | ((uint64_t)y[1] << 32);
  out[1] = (uint64_t)y[2] | ((uint64_t)y[3] << 32);
}

// Everything a sealing kernel needs, passed by value.
struct SealCtx {
  AesRk rk;
  AesRk rkh;            // message tables' header PRF (head_aes)
  B2State leafk1[4];    // keyed states after the key block: map-directory leaves (256 B)
  B2State headk;        // keyed state of the header PRF
  const uint32_t* nhk;  // the row hash's NH key (kNhWords words, device memory)
  uint64_t l3k[16];     // its L3 keys (< p36)
  uint32_t l3p[4];      // its L3 pads
  uint32_t epoch;       // rows are read at `epoch`, written at `epoch + 1`
  uint32_t on;          // authenticated-storage mode enabled
};

}  // namespace gvs
