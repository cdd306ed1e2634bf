// gvs_seal_fused.h — the sealed message pass's crypto with the LDS and VALU
// work of one wave interleaved (DESIGN.md §8 "Interleaved AES and BLAKE2b").
//
// Per 8-row chunk a lane runs 16 AES blocks (CTR keystream at the read and at
// the write epoch) and 2 BLAKE2b compressions (the 128-B leaf it hashes for
// the read tag and for the write tag).  AES by T-tables is bound by LDS
// lookups (16 ds_read_b32 per block-round, 2 LDS-array cycles each), BLAKE2b
// is pure VALU.  Run one after the other, and with all waves of a workgroup
// in the same phase, the CU alternates between an LDS-bound and a VALU-bound
// stretch and the two never overlap (the measured pass time was about the sum
// of the two).  Here one fused step issues the 32 table lookups of an AES
// pair-round, runs 2-3 BLAKE2b G functions while they are in flight, then
// combines the lookups: every step keeps both pipes busy.
//
// A fused iteration = 4 AES block pairs (rows 2p, 2p+1 of the lane's block,
// rounds 2..10 after the shared round 1 of ctr_round1_chunk) = 36 steps, and
// one BLAKE2b compression (96 G functions, 8 per round): G functions
// [8T/3, 8(T+1)/3) run in step T.  Everything is compile-time indexed, so the
// message block, the state and the lookups stay in registers.
#pragma once
#include <utility>

#include "gvs_seal_dev.h"

namespace gvs {

// the keyed BLAKE2b state of message-table leaf `leaf` (128-B leaves), per lane
__device__ inline B2State leaf_key128(const SealCtx& c, uint32_t leaf) {
  B2State k = c.leafk0[0];
#pragma unroll
  for (uint32_t i = 1; i < 8; ++i) k = b2_sel(leaf == i, c.leafk0[i], k);
  return k;
}

struct FusedState {
  // AES: the pair in flight
  uint32_t a[4], b[4];
  // BLAKE2b working vector
  uint64_t v[16];
};

__device__ __attribute__((always_inline)) inline void b2g(uint64_t (&v)[16], int a, int b, int c,
                                                          int d, uint64_t x, uint64_t y) {
  v[a] = v[a] + v[b] + x;
  v[d] = b2_rotr(v[d] ^ v[a], 32);
  v[c] = v[c] + v[d];
  v[b] = b2_rotr(v[b] ^ v[c], 24);
  v[a] = v[a] + v[b] + y;
  v[d] = b2_rotr(v[d] ^ v[a], 16);
  v[c] = v[c] + v[d];
  v[b] = b2_rotr(v[b] ^ v[c], 63);
}

// G function g (0..95) of a compression: round g / 8, columns then diagonals
template <int g>
__device__ __attribute__((always_inline)) inline void b2g_at(uint64_t (&v)[16], const uint64_t (&m)[16]) {
  constexpr int R = g / 8, i = g % 8;
  constexpr int a = i < 4 ? i : i - 4;
  constexpr int b = i < 4 ? 4 + i : 4 + ((i - 3) & 3);
  constexpr int c = i < 4 ? 8 + i : 8 + ((i - 2) & 3);
  constexpr int d = i < 4 ? 12 + i : 12 + ((i - 1) & 3);
  b2g(v, a, b, c, d, m[b2_sigma(R, 2 * i)], m[b2_sigma(R, 2 * i + 1)]);
}

template <int G0, int... Is>
__device__ __attribute__((always_inline)) inline void b2g_range(uint64_t (&v)[16], const uint64_t (&m)[16],
                                                                std::integer_sequence<int, Is...>) {
  (b2g_at<G0 + Is>(v, m), ...);
}

// the 16 lookups of one block-round (state s entering the round)
__device__ __attribute__((always_inline)) inline void aes_issue(const LdsTe& te, const uint32_t (&s)[4],
                                                                uint32_t (&l)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) l[4 * i + k] = te_at(te, s[(i + k) & 3], 3 - k);
}

template <int R>  // R = 2..9: full round; 10: the last (SubBytes, ShiftRows, AddRoundKey)
__device__ __attribute__((always_inline)) inline void aes_combine(const AesRk& rk, uint32_t (&s)[4],
                                                                  const uint32_t (&l)[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (R < 10)
      s[i] = xor3(xor3(l[4 * i], ror32(l[4 * i + 1], 8), ror32(l[4 * i + 2], 16)), ror32(l[4 * i + 3], 24),
                  rk.w[4 * R + i]);
    else
      s[i] = sbox_pack(l[4 * i], l[4 * i + 1], l[4 * i + 2], l[4 * i + 3]) ^ rk.w[40 + i];
  }
}

// start pair p: rows 2p, 2p + 1 from the chunk's round 1 (one lookup each)
__device__ __attribute__((always_inline)) inline void pair_start(const LdsTe& te, const CtrRound1& c1, int p,
                                                                 FusedState& x) {
  const uint32_t ta = te_at(te, (c1.x0b3 ^ (uint32_t)(2 * p)) << 24, 3);
  const uint32_t tb = te_at(te, (c1.x0b3 ^ (uint32_t)(2 * p + 1)) << 24, 3);
  x.a[0] = c1.t[0] ^ ta;
  x.b[0] = c1.t[0] ^ tb;
#pragma unroll
  for (int i = 1; i < 4; ++i) x.a[i] = x.b[i] = c1.t[i];
}

template <int T>
__device__ __attribute__((always_inline)) inline void fused_step(const AesRk& rk, const LdsTe& te,
                                                                 const CtrRound1& c1, const uint64_t (&m)[16],
                                                                 FusedState& x, uint4 (&ks)[8]) {
  constexpr int p = T / 9, R = 2 + T % 9;
  constexpr int g0 = 8 * T / 3, g1 = 8 * (T + 1) / 3;
  if constexpr (R == 2) pair_start(te, c1, p, x);
  uint32_t la[16], lb[16];
  aes_issue(te, x.a, la);
  aes_issue(te, x.b, lb);
  __builtin_amdgcn_sched_barrier(0);
  b2g_range<g0>(x.v, m, std::make_integer_sequence<int, g1 - g0>{});
  __builtin_amdgcn_sched_barrier(0);
  aes_combine<R>(rk, x.a, la);
  aes_combine<R>(rk, x.b, lb);
  if constexpr (R == 10) {
    ks[2 * p] = make_uint4(bswap32(x.a[0]), bswap32(x.a[1]), bswap32(x.a[2]), bswap32(x.a[3]));
    ks[2 * p + 1] = make_uint4(bswap32(x.b[0]), bswap32(x.b[1]), bswap32(x.b[2]), bswap32(x.b[3]));
  }
}

template <int... Ts>
__device__ __attribute__((always_inline)) inline void fused_steps(const AesRk& rk, const LdsTe& te,
                                                                  const CtrRound1& c1, const uint64_t (&m)[16],
                                                                  FusedState& x, uint4 (&ks)[8],
                                                                  std::integer_sequence<int, Ts...>) {
  (fused_step<Ts>(rk, te, c1, m, x, ks), ...);
}

// One fused iteration: ks[u] = keystream block `lane` of row row0 + u (u < 8)
// at `epoch`, and dig = BLAKE2b-128 of the 128-B message m under the keyed
// state k (leaf_prf128: final block, t = 256).
__device__ inline void fused_ks8_leaf(const SealCtx& c, const LdsTe& te, uint32_t table, uint64_t row0,
                                      uint32_t epoch, const B2State& k, const uint64_t (&m)[16],
                                      uint4 (&ks)[8], uint64_t (&dig)[2]) {
  const CtrRound1 c1 = ctr_round1_chunk(c.rk, te, table, row0, epoch, lane_id());
  FusedState x;
  uint64_t iv[8];
  b2_iv(iv);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x.v[i] = k.h[i];
    x.v[i + 8] = iv[i];
  }
  x.v[12] ^= 256ull;
  x.v[14] = ~x.v[14];
  fused_steps(c.rk, te, c1, m, x, ks, std::make_integer_sequence<int, 36>{});
  dig[0] = k.h[0] ^ x.v[0] ^ x.v[8];
  dig[1] = k.h[1] ^ x.v[1] ^ x.v[9];
}

// the 128-B leaf (lane & 7) of staged row lane >> 3 (U = 8 rows per stage)
__device__ inline void stage_leaf8(const uint4* st, uint64_t (&m)[16]) {
  const uint32_t lane = lane_id(), leaf = lane & 7, ur = lane >> 3;
  const uint4* seg = st + (ur * 4 + (leaf >> 1)) * kSegU4 + (leaf & 1) * 8;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 x = seg[q];
    m[2 * q] = u4lo(x);
    m[2 * q + 1] = u4hi(x);
  }
}

// tag of row (lane >> 2) & 7 from the lanes' leaf digests (8 lanes per row)
// and H of the lane's row (wave_tags, NL = 8, U = 8)
__device__ inline void tag_finish8(uint64_t (&r)[2], const uint64_t (&hdr)[2], uint64_t (&out)[2]) {
  const uint32_t lane = lane_id();
  const int src = (int)(8u * ((lane >> 2) & 7u));
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    r[w] ^= shfl_u64(r[w], (int)(lane ^ 1u));
    r[w] ^= shfl_u64(r[w], (int)(lane ^ 2u));
    r[w] ^= shfl_u64(r[w], (int)(lane ^ 4u));
    out[w] = shfl_u64(r[w], src) ^ hdr[w];
  }
}

}  // namespace gvs
