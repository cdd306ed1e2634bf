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

__device__ inline void load_te(uint32_t* s_te, const uint32_t* g_te) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_te[i] = g_te[i];
}

__device__ inline uint64_t shfl_u64(uint64_t x, int src) {
  const uint32_t lo = __shfl((uint32_t)x, src), hi = __shfl((uint32_t)(x >> 32), src);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Tag of row row0 + ur, ur = (lane >> 2) % U, over the ciphertext rows v[]
// and (mailbox rows) side ciphertexts staged at st[U*4*kSegU4 + u].
template <int U>
__device__ inline void wave_tags(const SealCtx& c, uint32_t table, uint64_t row0, uint32_t epoch,
                                 const uint4 (&v)[U], bool with_side, uint4* st, uint64_t out[2]) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < U; ++u) st[(u * 4 + (lane >> 4)) * kSegU4 + (lane & 15)] = v[u];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t ur = (lane >> 2) % (uint32_t)U, leaf = lane & 3;
  uint64_t m[32];
  const uint4* seg = st + (ur * 4 + leaf) * kSegU4;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint4 x = seg[k];
    m[2 * k] = u4lo(x);
    m[2 * k + 1] = u4hi(x);
  }
  uint64_t d[2];
  leaf_digest(m, leaf, d);
  uint64_t lv[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int src = (int)((lane & ~3u) | (uint32_t)k);
    lv[2 * k] = shfl_u64(d[0], src);
    lv[2 * k + 1] = shfl_u64(d[1], src);
  }
  uint64_t sd[2] = {0, 0};
  if (with_side) {
    const uint4 x = st[U * 4 * kSegU4 + ur];
    sd[0] = u4lo(x);
    sd[1] = u4hi(x);
  }
  row_tag(c.keyed, row0 + ur, epoch, table, sd, lv, out);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();  // the stage is reused by the caller
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XOR the CTR keystream of (table, row0 + u, epoch) block `lane` into v[u]
template <int U>
__device__ inline void wave_ctr(const SealCtx& c, const uint32_t* s_te, uint32_t table,
                                uint64_t row0, uint32_t epoch, uint4 (&v)[U]) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint4 k = ctr_keystream(c.rk, s_te, table, row0 + u, epoch, lane);
    v[u] = make_uint4(v[u].x ^ k.x, v[u].y ^ k.y, v[u].z ^ k.z, v[u].w ^ k.w);
  }
}

// Verify and decrypt U rows read at c.epoch.  `tags` is the table's tag
// array (indexed by row); side ciphertexts (mailbox rows) must already be in
// the stage's side slots.  Returns false (wave-uniform) on any mismatch.
template <int U>
__device__ inline bool wave_unseal(const SealCtx& c, const uint32_t* s_te, uint32_t table,
                                   uint64_t row0, uint4 (&v)[U], const uint4* tags, bool with_side,
                                   uint4* st) {
  uint64_t t[2];
  wave_tags<U>(c, table, row0, c.epoch, v, with_side, st, t);
  const uint32_t ur = (lane_id() >> 2) % (uint32_t)U;
  const uint4 want = tags[row0 + ur];
  const bool bad = u4lo(want) != t[0] || u4hi(want) != t[1];
  wave_ctr<U>(c, s_te, table, row0, c.epoch, v);
  return __ballot(bad) == 0ull;
}

// Encrypt U plaintext rows at epoch `ep` (c.epoch + 1 for a pass's writes)
// and store their tags (side ciphertexts, if any, already staged).
template <int U>
__device__ inline void wave_seal(const SealCtx& c, const uint32_t* s_te, uint32_t table,
                                 uint64_t row0, uint32_t ep, uint4 (&v)[U], uint4* tags,
                                 bool with_side, uint4* st) {
  wave_ctr<U>(c, s_te, table, row0, ep, v);
  uint64_t t[2];
  wave_tags<U>(c, table, row0, ep, v, with_side, st, t);
  const uint32_t lane = lane_id();
  if ((lane & 3u) == 0 && (lane >> 2) < (uint32_t)U)
    tags[row0 + (lane >> 2)] = make_uint4((uint32_t)t[0], (uint32_t)(t[0] >> 32), (uint32_t)t[1],
                                          (uint32_t)(t[1] >> 32));
}

// Keystream block 64 (the mailbox side entry) of `row` at `ep`.
__device__ inline uint4 side_keystream(const SealCtx& c, const uint32_t* s_te, uint64_t row,
                                       uint32_t ep) {
  return ctr_keystream(c.rk, s_te, 1u, row, ep, 64u);
}

__device__ inline uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// Seal freshly initialised (all-zero) rows of a table at epoch 0; one wave
// per 16 rows, grid-stride.  side != nullptr: mailbox table (+ side array).
__global__ __launch_bounds__(256) void k_seal_init(SealCtx c, const uint32_t* g_te, uint4* rows,
                                                   uint4* tags, uint4* side, uint32_t table,
                                                   uint64_t n_rows) {
  constexpr int U = 16;
  __shared__ uint32_t s_te[256];
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
    }
    wave_seal<U>(c, s_te, table, r0, 0u, v, tags, side != nullptr, st);
#pragma unroll
    for (int u = 0; u < U; ++u) rows[(r0 + u) * 64 + lane] = v[u];
  }
}

}  // namespace gvs
