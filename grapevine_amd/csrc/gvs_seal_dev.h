// gvs_seal_dev.h — wave-level sealing of table rows for the authenticated-
// storage mode (format in gvs_crypto.h).
//
// A wave holds U consecutive rows, 16 B per lane (lane l = AES block l of
// each row).  Decryption/encryption is lane-parallel: lane l runs AES for
// block l of every row.  The tag needs each row's 4 leaf digests: the rows
// are staged in the wave's LDS area so that lane L can hash leaf (L & 3) of
// row (L >> 2) mod U from 16 conflict-free ds_read_b128 (each 256-B leaf
// segment is padded by 16 B).  Every lane then gathers its row's leaves
// with shuffles and computes the row's tag (4 lanes per row, redundantly).
// No branch depends on data; the same instructions run for every chunk.
#pragma once
#include "gvs_crypto.h"
#include "gvs_device.h"

namespace gvs {

constexpr uint32_t kSegU4 = 17;  // 256-B leaf segment + 16 B padding, in uint4

// LDS bytes per wave for U rows: 4 segments per row + U side slots
__host__ __device__ constexpr uint32_t stage_u4(int U) { return (uint32_t)U * 4 * kSegU4 + (uint32_t)U; }

// stage slot of block `lane` of row u: 256-B leaf segments padded by 16 B
__device__ inline uint32_t stage_slot(int u, uint32_t lane) {
  return ((uint32_t)u * 4 + (lane >> 4)) * kSegU4 + (lane & 15);
}


// The AES table lives in LDS as 32 interleaved replicas: entry x of replica
// r at byte x * 256 + 4 r (r < 32).  Lane l reads replica l mod 32: a
// ds_read_b32 is serviced in two half-waves {0-31}, {32-63}, banked by
// (address / 4) mod 32 (MI355X_MICROARCH.md "LDS"), so the 32 lanes of a half
// always hit 32 distinct banks whatever the (secret, data-dependent) indices
// are: no bank conflicts, and no timing that depends on the key or the
// plaintext through conflicts.  The table's 64-KiB window is 64 KiB-aligned,
// which puts it at LDS address 0, so a lookup address is a single v_perm_b32:
// byte 1 = the state byte, byte 0 = 4 (l mod 32).  Bytes [128, 256) of every
// 256-B entry row are not part of the table: 256 holes of 128 B (32 KiB) that
// the sealed message pass uses as staging space (gvs_spass.h).
constexpr uint32_t kTeRep = 32;
constexpr uint32_t kTeWords = 256 * 64;  // the 64-KiB window (table + holes)
#define GVS_TE_LDS __shared__ __attribute__((aligned(65536))) uint32_t

__device__ inline void load_te(uint32_t* s_te, const uint32_t* g_te) {
  for (uint32_t i = threadIdx.x; i < 256 * kTeRep; i += blockDim.x)
    s_te[(i / kTeRep) * 64 + (i % kTeRep)] = g_te[i / kTeRep];
}

struct LdsTe {
  const uint32_t* base;  // s_te (at LDS address 0)
  uint32_t lane4;        // 4 * (lane mod 32)
};

__device__ inline LdsTe lds_te(const uint32_t* s_te) { return LdsTe{s_te, (lane_id() & 31u) * 4u}; }

__device__ inline uint32_t te_at(const LdsTe& t, uint32_t s, int k) {
  const uint32_t off = __builtin_amdgcn_perm(s, t.lane4, 0x0c0c0400u | ((uint32_t)(4 + k) << 8));
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(t.base) + off);
}

__device__ inline uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__device__ inline uint64_t shfl_u64(uint64_t x, int src) {
  const uint32_t lo = __shfl((uint32_t)x, src), hi = __shfl((uint32_t)(x >> 32), src);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// S-box bytes of four lookups (byte 1 of each te0 entry) packed big-endian:
// three v_perm_b32
__device__ inline uint32_t sbox_pack(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3) {
  const uint32_t hi = __builtin_amdgcn_perm(l0, l1, 0x05010c0cu);  // l0.b1 | l1.b1 | 0 | 0
  const uint32_t lo = __builtin_amdgcn_perm(l2, l3, 0x0c0c0501u);  // 0 | 0 | l2.b1 | l3.b1
  return hi | lo;
}

// AES-128 rounds R0..10 of two blocks at once (the device form of
// aes128_encrypt_words; a[], b[] hold the state entering round R0).  Each
// round first issues all 32 table lookups of both blocks, then combines them:
// sched_barrier keeps the compiler from interleaving loads and uses (which it
// does under register pressure, leaving one LDS latency exposed per lookup).
template <int R0>
__device__ inline void aes128_rounds2(const AesRk& rk, const LdsTe& te, uint32_t (&a)[4],
                                      uint32_t (&b)[4]) {
#pragma unroll
  for (int r = R0; r < 10; ++r) {
    uint32_t la[16], lb[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        la[4 * i + k] = te_at(te, a[(i + k) & 3], 3 - k);
        lb[4 * i + k] = te_at(te, b[(i + k) & 3], 3 - k);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = xor3(xor3(la[4 * i], ror32(la[4 * i + 1], 8), ror32(la[4 * i + 2], 16)),
                  ror32(la[4 * i + 3], 24), rk.w[4 * r + i]);
      b[i] = xor3(xor3(lb[4 * i], ror32(lb[4 * i + 1], 8), ror32(lb[4 * i + 2], 16)),
                  ror32(lb[4 * i + 3], 24), rk.w[4 * r + i]);
    }
  }
  uint32_t la[16], lb[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      la[4 * i + k] = te_at(te, a[(i + k) & 3], 3 - k);
      lb[4 * i + k] = te_at(te, b[(i + k) & 3], 3 - k);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // last round: SubBytes + ShiftRows (S-box = te0 byte 1), AddRoundKey
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = sbox_pack(la[4 * i], la[4 * i + 1], la[4 * i + 2], la[4 * i + 3]) ^ rk.w[40 + i];
    b[i] = sbox_pack(lb[4 * i], lb[4 * i + 1], lb[4 * i + 2], lb[4 * i + 3]) ^ rk.w[40 + i];
  }
}

// Counter blocks of one lane over a chunk of rows row0 .. row0 + U - 1 (U
// divides 256, row0 a multiple of U) differ only in the low byte of the row,
// which AES round 1 reads once (the byte-3 lookup of word 0).  Round 1 is
// therefore computed once per chunk without that term; per block it costs one
// lookup (ctr_round1_finish).
struct CtrRound1 {
  uint32_t t[4];  // round-1 output, t[0] still missing T0[x0.b3]
  uint32_t x0b3;  // byte 3 of x0 = bswap(row0 lo) ^ rk0, for the low row byte
};

__device__ inline CtrRound1 ctr_round1_chunk(const AesRk& rk, const LdsTe& te, uint32_t table,
                                             uint64_t row0, uint32_t epoch, uint32_t j) {
  const uint32_t x0 = bswap32((uint32_t)row0) ^ rk.w[0];
  const uint32_t x1 = bswap32((uint32_t)(row0 >> 32)) ^ rk.w[1];
  const uint32_t x2 = bswap32(epoch) ^ rk.w[2];
  const uint32_t x3 = ((table << 24) | j) ^ rk.w[3];
  const uint32_t x[4] = {x0, x1, x2, x3};
  uint32_t l[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) l[4 * i + k] = (i == 0 && k == 0) ? 0u : te_at(te, x[(i + k) & 3], 3 - k);
  CtrRound1 c;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    c.t[i] = xor3(xor3(l[4 * i], ror32(l[4 * i + 1], 8), ror32(l[4 * i + 2], 16)),
                  ror32(l[4 * i + 3], 24), rk.w[4 + i]);
  c.x0b3 = x0 >> 24;
  return c;
}

// keystream blocks j of rows row0 + u and row0 + u + 1 as little-endian words
__device__ inline void ctr_keystream2(const AesRk& rk, const LdsTe& te, const CtrRound1& c1,
                                      uint32_t u, uint4& ka, uint4& kb) {
  const uint32_t ta = te_at(te, (c1.x0b3 ^ u) << 24, 3);
  const uint32_t tb = te_at(te, (c1.x0b3 ^ (u + 1)) << 24, 3);
  uint32_t a[4] = {c1.t[0] ^ ta, c1.t[1], c1.t[2], c1.t[3]};
  uint32_t b[4] = {c1.t[0] ^ tb, c1.t[1], c1.t[2], c1.t[3]};
  aes128_rounds2<2>(rk, te, a, b);
  ka = make_uint4(bswap32(a[0]), bswap32(a[1]), bswap32(a[2]), bswap32(a[3]));
  kb = make_uint4(bswap32(b[0]), bswap32(b[1]), bswap32(b[2]), bswap32(b[3]));
}

// Counter blocks j = j0 + i (i < 8, j0 a multiple of 8) of one row: they
// differ only in byte 0 of the last word, which round 1 reads once (the
// byte-0 lookup of word 3, into t[0]).  Round 1 once per row without that
// term; per block one lookup (the leaf-major message pass, gvs_spass.h: lane L
// holds blocks 8 (L & 7) .. + 7 of one row).
struct CtrRound1J {
  uint32_t t[4];  // round-1 output, t[0] still missing T0[x3.b0] >>> 24
  uint32_t x3b0;  // byte 0 of x3 for j0 (x3 = (table << 24 | j) ^ rk3)
};

__device__ inline CtrRound1J ctr_round1_row(const AesRk& rk, const LdsTe& te, uint32_t table,
                                            uint64_t row, uint32_t epoch, uint32_t j0) {
  const uint32_t x0 = bswap32((uint32_t)row) ^ rk.w[0];
  const uint32_t x1 = bswap32((uint32_t)(row >> 32)) ^ rk.w[1];
  const uint32_t x2 = bswap32(epoch) ^ rk.w[2];
  const uint32_t x3 = ((table << 24) | j0) ^ rk.w[3];
  const uint32_t x[4] = {x0, x1, x2, x3};
  uint32_t l[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) l[4 * i + k] = (i == 0 && k == 3) ? 0u : te_at(te, x[(i + k) & 3], 3 - k);
  CtrRound1J c;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    c.t[i] = xor3(xor3(l[4 * i], ror32(l[4 * i + 1], 8), ror32(l[4 * i + 2], 16)),
                  ror32(l[4 * i + 3], 24), rk.w[4 + i]);
  c.x3b0 = x3 & 0xffu;
  return c;
}

// keystream blocks j0 + i and j0 + i + 1 of the row as little-endian words
__device__ inline void ctr_keystream2_j(const AesRk& rk, const LdsTe& te, const CtrRound1J& c1,
                                        uint32_t i, uint4& ka, uint4& kb) {
  const uint32_t ta = te_at(te, c1.x3b0 ^ i, 0);
  const uint32_t tb = te_at(te, c1.x3b0 ^ (i + 1), 0);
  uint32_t a[4] = {c1.t[0] ^ ror32(ta, 24), c1.t[1], c1.t[2], c1.t[3]};
  uint32_t b[4] = {c1.t[0] ^ ror32(tb, 24), c1.t[1], c1.t[2], c1.t[3]};
  aes128_rounds2<2>(rk, te, a, b);
  ka = make_uint4(bswap32(a[0]), bswap32(a[1]), bswap32(a[2]), bswap32(a[3]));
  kb = make_uint4(bswap32(b[0]), bswap32(b[1]), bswap32(b[2]), bswap32(b[3]));
}

// The same for NB independent blocks at once: each round issues all 16 NB
// lookups before combining them, so a lane waits for NB / 2 times fewer LDS
// round trips per block (the sealed pass is bound by that latency).
template <int R0, int NB, bool ROLL = false>
__device__ inline void aes128_rounds_n(const AesRk& rk, const LdsTe& te, uint32_t (&s)[NB][4]) {
  // ROLL: one copy of the round (round keys read by index, scalar loads), for
  // the sealed mailbox passes (gvs_mauth.h)
  constexpr int kUnroll = ROLL ? 1 : 10;
#pragma unroll kUnroll
  for (int r = R0; r < 10; ++r) {
    uint32_t l[NB][16];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) l[b][4 * i + k] = te_at(te, s[b][(i + k) & 3], 3 - k);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        s[b][i] = xor3(xor3(l[b][4 * i], ror32(l[b][4 * i + 1], 8), ror32(l[b][4 * i + 2], 16)),
                       ror32(l[b][4 * i + 3], 24), rk.w[4 * r + i]);
  }
  uint32_t l[NB][16];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) l[b][4 * i + k] = te_at(te, s[b][(i + k) & 3], 3 - k);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      s[b][i] = sbox_pack(l[b][4 * i], l[b][4 * i + 1], l[b][4 * i + 2], l[b][4 * i + 3]) ^ rk.w[40 + i];
}

// keystream blocks j0 + i0 .. j0 + i0 + NB - 1 of the row (ctr_round1_row)
template <int NB, bool ROLL = false>
__device__ inline void ctr_keystream_jn(const AesRk& rk, const LdsTe& te, const CtrRound1J& c1, uint32_t i0,
                                        uint4 (&ks)[NB]) {
  uint32_t s[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint32_t t = te_at(te, c1.x3b0 ^ (i0 + (uint32_t)b), 0);
    s[b][0] = c1.t[0] ^ ror32(t, 24);
    s[b][1] = c1.t[1];
    s[b][2] = c1.t[2];
    s[b][3] = c1.t[3];
  }
  aes128_rounds_n<2, NB, ROLL>(rk, te, s);
#pragma unroll
  for (int b = 0; b < NB; ++b) ks[b] = make_uint4(bswap32(s[b][0]), bswap32(s[b][1]), bswap32(s[b][2]), bswap32(s[b][3]));
}

// Two tables in the 64-KiB window (the sealed message pass, gvs_spass.h):
// T0 as above, and T1 = T0 rotated right by 8 in the holes (entry x of
// replica r at byte 256 x + 128 + 4 r: the same bank as T0's entry, so a
// half-wave is still conflict-free).  A round column is then
// T0[a] ^ T1[b] ^ ror16(T0[c] ^ T1[d]) ^ rk (FIPS-197 §5.2.1's T-table
// identities): one rotation instead of three.  The pass is bound by the issue
// of its three-source instructions (DESIGN.md §8 "Issue rates"), and the
// rotations were 28 % of them.
__device__ inline void load_te2(uint32_t* s_te, const uint32_t* g_te) {
  for (uint32_t i = threadIdx.x; i < 256 * kTeRep; i += blockDim.x) {
    const uint32_t t = g_te[i / kTeRep];
    s_te[(i / kTeRep) * 64 + (i % kTeRep)] = t;
    s_te[(i / kTeRep) * 64 + 32 + (i % kTeRep)] = (t >> 8) | (t << 24);
  }
}

__device__ inline uint32_t te1_at(const LdsTe& t, uint32_t s, int k) {
  const uint32_t off = __builtin_amdgcn_perm(s, t.lane4, 0x0c0c0400u | ((uint32_t)(4 + k) << 8));
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(t.base) + 128u + off);
}

// aes128_rounds_n on the two-table window.  The rounds are rolled: unrolled,
// the sealed pass's loop body did not fit the instruction cache (15.8 M
// instruction requests to L2 per 2^20-row launch, a count that followed the
// request mix, and refetched code lines made its FETCH_SIZE noisy: ~900 64-B
// reads between two seeds of one mix); rolled, 133 K requests, the same under
// every mix, read requests within 13 of each other, 2.5 % slower
// (profiles/r05ai_spass_inst_requests.txt, r05aj_spass_roll_ab.txt)
template <int R0, int NB>
__device__ inline void aes128_rounds_n2(const AesRk& rk, const LdsTe& te, uint32_t (&s)[NB][4]) {
#pragma unroll 1
  for (int r = R0; r < 10; ++r) {
    uint32_t l[NB][16];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        l[b][4 * i + 0] = te_at(te, s[b][i], 3);
        l[b][4 * i + 1] = te1_at(te, s[b][(i + 1) & 3], 2);
        l[b][4 * i + 2] = te_at(te, s[b][(i + 2) & 3], 1);
        l[b][4 * i + 3] = te1_at(te, s[b][(i + 3) & 3], 0);
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        s[b][i] = xor3(l[b][4 * i], l[b][4 * i + 1], ror32(l[b][4 * i + 2] ^ l[b][4 * i + 3], 16)) ^ rk.w[4 * r + i];
  }
  uint32_t l[NB][16];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) l[b][4 * i + k] = te_at(te, s[b][(i + k) & 3], 3 - k);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      s[b][i] = sbox_pack(l[b][4 * i], l[b][4 * i + 1], l[b][4 * i + 2], l[b][4 * i + 3]) ^ rk.w[40 + i];
}

template <int NB>
__device__ inline void ctr_keystream_jn2(const AesRk& rk, const LdsTe& te, const CtrRound1J& c1, uint32_t i0,
                                         uint4 (&ks)[NB]) {
  uint32_t s[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint32_t t = te_at(te, c1.x3b0 ^ (i0 + (uint32_t)b), 0);
    s[b][0] = c1.t[0] ^ ror32(t, 24);
    s[b][1] = c1.t[1];
    s[b][2] = c1.t[2];
    s[b][3] = c1.t[3];
  }
  aes128_rounds_n2<2, NB>(rk, te, s);
#pragma unroll
  for (int b = 0; b < NB; ++b) ks[b] = make_uint4(bswap32(s[b][0]), bswap32(s[b][1]), bswap32(s[b][2]), bswap32(s[b][3]));
}

// Round 2 cached as well (the two-table window): after round 1 only word 0
// of the state differs between a lane's blocks, and each round-2 column reads
// exactly one byte of word 0 (column 0: T0[w0.b3]; 1: T1[w0.b0] in the ror16
// pair; 2: T0[w0.b1] in the ror16 pair; 3: T1[w0.b2]).  The other twelve
// lookups and the round key are folded once per row into f[]; per block,
// round 2 costs four lookups instead of sixteen (the sealed message pass is
// bound by its LDS lookups).
struct CtrRound2J {
  uint32_t f[4];  // round-2 columns without their word-0 terms
  uint32_t t0;    // round-1 word 0 without its block term (CtrRound1J::t[0])
  uint32_t x3b0;  // as CtrRound1J
};

__device__ inline CtrRound2J ctr_round2_row(const AesRk& rk, const LdsTe& te, const CtrRound1J& c1) {
  const uint32_t s1 = c1.t[1], s2 = c1.t[2], s3 = c1.t[3];
  CtrRound2J c;
  c.f[0] = te1_at(te, s1, 2) ^ ror32(te_at(te, s2, 1) ^ te1_at(te, s3, 0), 16) ^ rk.w[8];
  c.f[1] = te_at(te, s1, 3) ^ te1_at(te, s2, 2) ^ ror32(te_at(te, s3, 1), 16) ^ rk.w[9];
  c.f[2] = te_at(te, s2, 3) ^ te1_at(te, s3, 2) ^ ror32(te1_at(te, s1, 0), 16) ^ rk.w[10];
  c.f[3] = te_at(te, s3, 3) ^ ror32(te_at(te, s1, 1) ^ te1_at(te, s2, 0), 16) ^ rk.w[11];
  c.t0 = c1.t[0];
  c.x3b0 = c1.x3b0;
  return c;
}

// keystream blocks j0 + i0 .. j0 + i0 + NB - 1 of the row from round 3 on
template <int NB>
__device__ inline void ctr_keystream_jn3(const AesRk& rk, const LdsTe& te, const CtrRound2J& c2, uint32_t i0,
                                         uint4 (&ks)[NB]) {
  uint32_t w0[NB], l[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) w0[b] = c2.t0 ^ ror32(te_at(te, c2.x3b0 ^ (i0 + (uint32_t)b), 0), 24);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    l[b][0] = te_at(te, w0[b], 3);
    l[b][1] = te1_at(te, w0[b], 0);
    l[b][2] = te_at(te, w0[b], 1);
    l[b][3] = te1_at(te, w0[b], 2);
  }
  __builtin_amdgcn_sched_barrier(0);
  uint32_t s[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    s[b][0] = c2.f[0] ^ l[b][0];
    s[b][1] = c2.f[1] ^ ror32(l[b][1], 16);
    s[b][2] = c2.f[2] ^ ror32(l[b][2], 16);
    s[b][3] = c2.f[3] ^ l[b][3];
  }
  aes128_rounds_n2<3, NB>(rk, te, s);
#pragma unroll
  for (int b = 0; b < NB; ++b) ks[b] = make_uint4(bswap32(s[b][0]), bswap32(s[b][1]), bswap32(s[b][2]), bswap32(s[b][3]));
}

// The same for the one-table window (the sealed mailbox passes, gvs_mauth.h):
// a column is T0[a] ^ ror8(T0[b]) ^ ror16(T0[c]) ^ ror24(T0[d]), word 0's
// byte entering column 0 direct, column 1 as d, column 2 as c, column 3 as b.
__device__ inline CtrRound2J ctr_round2_row1(const AesRk& rk, const LdsTe& te, const CtrRound1J& c1) {
  const uint32_t s1 = c1.t[1], s2 = c1.t[2], s3 = c1.t[3];
  CtrRound2J c;
  c.f[0] = xor3(ror32(te_at(te, s1, 2), 8), ror32(te_at(te, s2, 1), 16), ror32(te_at(te, s3, 0), 24)) ^ rk.w[8];
  c.f[1] = xor3(te_at(te, s1, 3), ror32(te_at(te, s2, 2), 8), ror32(te_at(te, s3, 1), 16)) ^ rk.w[9];
  c.f[2] = xor3(te_at(te, s2, 3), ror32(te_at(te, s3, 2), 8), ror32(te_at(te, s1, 0), 24)) ^ rk.w[10];
  c.f[3] = xor3(te_at(te, s3, 3), ror32(te_at(te, s1, 1), 16), ror32(te_at(te, s2, 0), 24)) ^ rk.w[11];
  c.t0 = c1.t[0];
  c.x3b0 = c1.x3b0;
  return c;
}

template <int NB, bool ROLL = false>
__device__ inline void ctr_keystream_jn3_1(const AesRk& rk, const LdsTe& te, const CtrRound2J& c2, uint32_t i0,
                                           uint4 (&ks)[NB]) {
  uint32_t w0[NB], l[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) w0[b] = c2.t0 ^ ror32(te_at(te, c2.x3b0 ^ (i0 + (uint32_t)b), 0), 24);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    l[b][0] = te_at(te, w0[b], 3);
    l[b][1] = te_at(te, w0[b], 0);
    l[b][2] = te_at(te, w0[b], 1);
    l[b][3] = te_at(te, w0[b], 2);
  }
  __builtin_amdgcn_sched_barrier(0);
  uint32_t s[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    s[b][0] = c2.f[0] ^ l[b][0];
    s[b][1] = c2.f[1] ^ ror32(l[b][1], 24);
    s[b][2] = c2.f[2] ^ ror32(l[b][2], 16);
    s[b][3] = c2.f[3] ^ ror32(l[b][3], 8);
  }
  aes128_rounds_n<3, NB, ROLL>(rk, te, s);
#pragma unroll
  for (int b = 0; b < NB; ++b) ks[b] = make_uint4(bswap32(s[b][0]), bswap32(s[b][1]), bswap32(s[b][2]), bswap32(s[b][3]));
}

// The tile layout of a sealed message (or block) table: rows in tiles of 8
// (8 KiB); inside a tile, 16-B unit i * 64 + L holds block 8 (L & 7) + i of
// row L >> 3.  A wave's coalesced load of unit i into lane L (8 whole-KiB
// instructions) then leaves leaf L & 7 (128 B) of row L >> 3 in lane L's
// registers: the leaf hashes need no transposition through LDS.
__host__ __device__ constexpr uint64_t tile_unit(uint64_t row, uint32_t block) {
  return (row >> 3) * 512 + (uint64_t)(block & 7u) * 64 + (row & 7) * 8 + (block >> 3);
}

// The tile layout of a sealed mailbox table: rows in tiles of 16 (16 KiB);
// inside a tile, 16-B unit i * 64 + L holds block 16 (L & 3) + i of row L >> 2.
// A wave's 16 coalesced 1-KiB loads leave leaf L & 3 (256 B) of row L >> 2 in
// lane L's registers (gvs_mauth.h).
__host__ __device__ constexpr uint64_t mtile_unit(uint64_t row, uint32_t block) {
  return (row >> 4) * 1024 + (uint64_t)(block & 15u) * 64 + (row & 15) * 4 + (block >> 4);
}

template <int U>
__device__ inline void stage_rows(const uint4 (&v)[U], uint4* st) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < U; ++u) st[stage_slot(u, lane)] = v[u];
  wave_lds_sync();
}

template <int U>
__device__ inline void unstage_rows(uint4 (&v)[U], const uint4* st) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = st[stage_slot(u, lane)];
  wave_lds_sync();
}

// c ? a : b for a whole BLAKE2b state (per-lane selects)
__device__ inline B2State b2_sel(bool c, const B2State& a, const B2State& b) {
  B2State r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.h[i] = c ? a.h[i] : b.h[i];
  return r;
}

// Tag of row row0 + (lane >> 2) % U, over the ciphertext rows already in the
// stage: tag = H ^ L_0 ^ .. ^ L_(NL-1) (gvs_crypto.h).
//  * NL = 4 (map directory rows, 256-B leaves): lane L computes leaf L & 3 of row
//    (L >> 2) % U; the quad XORs its four leaves by shuffles.
//    - U <= 8 (side entries staged at st[U*4*kSegU4 + u]): lanes 32 + u
//      compute H of row u in the same instructions (their first compression
//      takes the header block instead of leaf data), so the header costs no
//      extra time.  htab: the header's table field in this lane's header row.
//    - U = 16: every lane hashes a leaf; `hdr` is H of the lane's row.
//  * NL = 8 (the row hash: message and mailbox tables, 128-B leaves): lane L
//    computes leaf L & 7 of row L >> 3 (U = 8), or of rows L >> 3 and
//    (L >> 3) + 8 (U = 16); the 8 lanes of a row add their NH sums, and every
//    lane then takes its row's sum.  `hdr` is H of the lane's row (the
//    message pass computes it for 64 rows at once).
// Valid in lanes < 4U.
template <int U, int NL = 4>
__device__ inline void wave_tags(const SealCtx& c, uint32_t table, uint64_t row0, uint32_t epoch,
                                 bool with_side, const uint4* st, const uint64_t* hdr,
                                 uint64_t out[2], uint32_t htab) {
  const uint32_t lane = lane_id();
  if constexpr (NL == 8) {
    static_assert(U == 8 || U == 16, "8 or 16 rows of 8 leaves");
    // the row hash (gvs_crypto.h): lane L's leaf L & 7 against its window of
    // the NH key (global, read once per call), the sums added over the row's
    // 8 lanes, then L3 on each lane's row
    const uint32_t leaf = lane & 7;
    uint32_t k[44];
    const uint4* kp = reinterpret_cast<const uint4*>(c.nhk + 32u * leaf);
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      const uint4 x = kp[q];
      k[4 * q] = x.x;
      k[4 * q + 1] = x.y;
      k[4 * q + 2] = x.z;
      k[4 * q + 3] = x.w;
    }
    uint64_t acc[U / 8][4];
#pragma unroll
    for (int set = 0; set < U / 8; ++set) {
      const uint32_t ur = (lane >> 3) + 8u * (uint32_t)set;
      const uint4* seg = st + (ur * 4 + (leaf >> 1)) * kSegU4 + (leaf & 1) * 8;
      uint32_t w[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint4 x = seg[q];
        w[4 * q] = x.x;
        w[4 * q + 1] = x.y;
        w[4 * q + 2] = x.z;
        w[4 * q + 3] = x.w;
      }
      uint64_t sm[4] = {0, 0, 0, 0};
      nh_words(k, 0u, w, sm);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sm[t] += shfl_u64(sm[t], (int)(lane ^ 1u));
        sm[t] += shfl_u64(sm[t], (int)(lane ^ 2u));
        sm[t] += shfl_u64(sm[t], (int)(lane ^ 4u));
        acc[set][t] = sm[t];
      }
    }
    const uint32_t row = (lane >> 2) % (uint32_t)U;
    const int src = (int)(8u * (row & 7u));
    uint64_t sm[4], g[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // both shuffles in every lane (a shuffle under a divergent branch would
      // read lanes that are switched off), then a per-lane select
      const uint64_t lo = shfl_u64(acc[0][t], src);
      const uint64_t hi = shfl_u64(acc[U / 8 - 1][t], src);
      sm[t] = U == 16 && row >= 8 ? hi : lo;
    }
    row_hash_fin(sm, c.l3k, c.l3p, g);
    out[0] = g[0] ^ hdr[0];
    out[1] = g[1] ^ hdr[1];
    (void)table, (void)row0, (void)epoch, (void)with_side, (void)htab;
    return;
  } else {
    constexpr bool kInlineHdr = U <= 8;
    const uint32_t ur = (lane >> 2) % (uint32_t)U, leaf = lane & 3;
    uint64_t m[32];
    const uint4* seg = st + (ur * 4 + leaf) * kSegU4;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint4 x = seg[k];
      m[2 * k] = u4lo(x);
      m[2 * k + 1] = u4hi(x);
    }
    uint64_t res[2];
    if (kInlineHdr) {
      const bool hl = lane >= 32;
      const uint32_t hrow = (lane - 32) % (uint32_t)U;
      uint64_t sd[2] = {0, 0};
      if (with_side) {
        const uint4 x = st[U * 4 * kSegU4 + hrow];
        sd[0] = u4lo(x);
        sd[1] = u4hi(x);
      }
      uint64_t hb[16];
      header_block(row0 + hrow, epoch, htab, sd, hb);
#pragma unroll
      for (int k = 0; k < 16; ++k) hb[k] = hl ? hb[k] : m[k];
      B2State s = b2_sel(hl, c.headk, c.leafk1[0]);
#pragma unroll
      for (uint32_t i = 1; i < 4; ++i) s = b2_sel(!hl && leaf == i, c.leafk1[i], s);
      b2_compress(s, hb, hl ? 128 + 32 : 128 + 128, hl);
      const uint64_t h0 = s.h[0], h1 = s.h[1];
      b2_compress(s, m + 16, 128 + 256, true);
      res[0] = hl ? h0 : s.h[0];
      res[1] = hl ? h1 : s.h[1];
    } else {
      B2State s = c.leafk1[0];
#pragma unroll
      for (uint32_t i = 1; i < 4; ++i) s = b2_sel(leaf == i, c.leafk1[i], s);
      leaf_prf(s, m, res);
    }
    // H of the lane's row: taken before the quad reduction below, which would
    // fold four rows' headers together in the header lanes
    uint64_t h[2];
#pragma unroll
    for (int w = 0; w < 2; ++w) h[w] = kInlineHdr ? shfl_u64(res[w], (int)(32 + ur)) : hdr[w];
    // XOR of the row's four leaves (lanes 4ur .. 4ur + 3), then H
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      res[w] ^= shfl_u64(res[w], (int)(lane ^ 1u));
      res[w] ^= shfl_u64(res[w], (int)(lane ^ 2u));
      out[w] = res[w] ^ h[w];
    }
  }
}

// XOR the CTR keystream of (table, row0 + u, epoch) block `lane` into the
// staged rows, in place.  A rolled loop (one copy of the AES code, two
// independent blocks per step); the rows are not held in registers meanwhile,
// which leaves the AES lookups room to be issued back to back.
template <int U>
__device__ inline void stage_ctr(const SealCtx& c, const uint32_t* s_te, uint32_t table,
                                 uint64_t row0, uint32_t epoch, uint4* st) {
  static_assert(U % 2 == 0 && 256 % U == 0, "rows come in pairs; a chunk stays in one 256-row block");
  const uint32_t lane = lane_id();
  const LdsTe te = lds_te(s_te);
  const CtrRound1 c1 = ctr_round1_chunk(c.rk, te, table, row0, epoch, lane);
#pragma unroll 1
  for (int u = 0; u < U; u += 2) {
    uint4 k0, k1;
    ctr_keystream2(c.rk, te, c1, (uint32_t)u, k0, k1);
    uint4* p0 = st + stage_slot(u, lane);
    uint4* p1 = st + stage_slot(u + 1, lane);
    *p0 = xor4(*p0, k0);
    *p1 = xor4(*p1, k1);
  }
  wave_lds_sync();
}

// Verify and decrypt U rows read at c.epoch.  `tags` is the table's tag
// array (indexed by row); side ciphertexts (mailbox rows) must already be in
// the stage's side slots.  Returns false (wave-uniform) on any mismatch.
template <int U, int NL = 4>
__device__ inline bool wave_unseal(const SealCtx& c, const uint32_t* s_te, uint32_t table,
                                   uint64_t row0, uint4 (&v)[U], const uint4* tags, bool with_side,
                                   uint4* st, const uint64_t* hdr = nullptr, uint32_t htab = ~0u) {
  stage_rows<U>(v, st);
  uint64_t t[2];
  wave_tags<U, NL>(c, table, row0, c.epoch, with_side, st, hdr, t, htab == ~0u ? table : htab);
  const uint32_t lane = lane_id(), ur = (lane >> 2) % (uint32_t)U;
  const uint4 want = tags[row0 + ur];
  const bool bad = lane < 4u * U && (u4lo(want) != t[0] || u4hi(want) != t[1]);
  stage_ctr<U>(c, s_te, table, row0, c.epoch, st);
  unstage_rows<U>(v, st);
  return __ballot(bad) == 0ull;
}

// Encrypt U plaintext rows at epoch `ep` (c.epoch + 1 for a pass's writes)
// and store their tags (side ciphertexts, if any, already staged).
template <int U, int NL = 4>
__device__ inline void wave_seal(const SealCtx& c, const uint32_t* s_te, uint32_t table,
                                 uint64_t row0, uint32_t ep, uint4 (&v)[U], uint4* tags,
                                 bool with_side, uint4* st, const uint64_t* hdr = nullptr,
                                 uint32_t htab = ~0u) {
  stage_rows<U>(v, st);
  stage_ctr<U>(c, s_te, table, row0, ep, st);
  unstage_rows<U>(v, st);
  uint64_t t[2];
  wave_tags<U, NL>(c, table, row0, ep, with_side, st, hdr, t, htab == ~0u ? table : htab);
  wave_lds_sync();  // the stage is reused by the caller
  const uint32_t lane = lane_id();
  if ((lane & 3u) == 0 && (lane >> 2) < (uint32_t)U)
    tags[row0 + (lane >> 2)] = make_uint4((uint32_t)t[0], (uint32_t)(t[0] >> 32), (uint32_t)t[1],
                                          (uint32_t)(t[1] >> 32));
}

// Keystream block 64 (the mailbox side entry) of `row` at `ep`.
__device__ inline uint4 side_keystream(const SealCtx& c, const uint32_t* s_te, uint64_t row,
                                       uint32_t ep) {
  return ctr_keystream(c.rk, lds_te(s_te), 1u, row, ep, 64u);
}


// Seal freshly initialised (all-zero) rows of a table at epoch 0; one wave
// per 16 rows, grid-stride.  side != nullptr: mailbox table (+ side array).
__global__ __launch_bounds__(256) void k_seal_init(SealCtx c, const uint32_t* g_te, uint4* rows,
                                                   uint4* tags, uint4* side, uint32_t table,
                                                   uint64_t n_rows) {
  constexpr int U = 16;
  GVS_TE_LDS s_te[kTeWords];
  __shared__ uint4 s_st[4 * stage_u4(U)];
  load_te(s_te, g_te);
  __syncthreads();
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  uint4* st = s_st + wave * stage_u4(U);
  for (uint64_t r0 = ((uint64_t)blockIdx.x * 4 + wave) * U; r0 < n_rows;
       r0 += (uint64_t)gridDim.x * 4 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = make_uint4(0, 0, 0, 0);
    if (side) {
      if (lane < (uint32_t)U) {
        const uint4 sct = side_keystream(c, s_te, r0 + lane, 0u);  // zero plaintext
        side[r0 + lane] = sct;
        st[U * 4 * kSegU4 + lane] = sct;
      }
      wave_lds_sync();
    }
    uint64_t sd[2] = {0, 0}, hdr[2];
    if (side) {
      const uint4 x = st[U * 4 * kSegU4 + ((lane >> 2) % U)];
      sd[0] = u4lo(x);
      sd[1] = u4hi(x);
    }
    // (two call sites rather than a pointer select, which would put sd in scratch)
    if (side)
      head_aes(c.rkh, lds_te(s_te), r0 + ((lane >> 2) % U), 0u, table, sd, hdr);
    else
      head_aes(c.rkh, lds_te(s_te), r0 + ((lane >> 2) % U), 0u, table, nullptr, hdr);
    // the row hash (NH over 8 leaves of 128 B) for the message tables and,
    // since round 6, the mailbox table
    wave_seal<U, 8>(c, s_te, table, r0, 0u, v, tags, side != nullptr, st, hdr);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (side)  // the mailbox table: 16-row tiles (mtile_unit)
        rows[mtile_unit(r0 + u, lane)] = v[u];
      else  // message and block tables: the tile layout (tile_unit)
        rows[tile_unit(r0 + u, lane)] = v[u];
    }
  }
}

}  // namespace gvs
