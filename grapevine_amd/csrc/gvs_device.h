// gvs_device.h — device-side definitions shared by the gvstore kernels.
//
// Layouts:
//   * message table: N rows of 1024 B (gvs_record layout, README.md:132-136),
//     partition-major: slot s lives in partition w = s % W at offset o = s / W,
//     row index w*S + o (S = N/W).  An all-zero msg_id marks an empty row
//     (README.md:159-160: the zero id is invalid).
//   * mailbox table: R = Q*S_r rows of 1024 B = recipient[32] + 62 ids x 16 B
//     (README.md:78-80); lane l>=2 of a wave holds id l-2.  Side array of 16 B
//     per row holds the recipient hash and the mailbox length.
//   * request image: the first 1024 B of gvs_request are the Record a CREATE
//     stores (sender = auth_identity), so images and rows share lane mapping.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gvs {

constexpr uint32_t kIdTag = 0x47565331u;  // "GVS1", must match oracle
constexpr uint32_t kPending = 0xFFu;      // internal status: decided later
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kGroupMax = 512;            // distinct recipients per mailbox partition per batch
constexpr int kStash = 2048;              // per-partition ops kept in LDS (beyond: re-read)
constexpr int kRowsMax = 4096;            // message rows per partition (S)
constexpr int kBinsMax = 32768;           // histogram bins (Q+1, W+1) kept in LDS
constexpr int kSrMax = 1024;              // mailbox rows per partition
constexpr int kTile = 256;                // message rows per R-pass tile
constexpr int kSeqBits = 20;              // seq <= B <= 2^19 (seq B = shared dummy record)
constexpr uint32_t kSeqMask = (1u << kSeqBits) - 1;

enum Kind : uint32_t {
  KIND_PAD = 0,
  KIND_HARD = 1,
  KIND_NEXT_READ = 2,
  KIND_NEXT_DEL = 3,
  KIND_CREATE = 4,
  KIND_READ = 5,
  KIND_UPDATE = 6,
  KIND_DELETE = 7,
};

// cflag bits written by M1 (one u32 per op)
constexpr uint32_t CF_POP = 1u;     // delete-next that pops a message
constexpr uint32_t CF_MBOX_OK = 2u; // create passes the mailbox checks

// Per-op records are 128 B (one L2 line) and written whole by one thread, so
// no two ops ever share a line: scattered per-op traffic then touches a fixed
// set of lines whatever order the data imposes (obliviousness).
// 16-B store that drops the line from the XCD's L2 (buffer_store ... nt sc1:
// the bytes are written through and the L2 drops the line,
// MI355X_MICROARCH.md:174; with nt the line is not kept on the memory side
// either: with sc1 alone, the readers of such records ran 4-7 us faster when
// the batch had just written more of them, k_vscan_a<M1rOp> / k_m1r_c at C3,
// profiles/r04j_timing_*).  Every record or row that a LATER kernel reads in
// an order or pairing that depends on the data is stored this way, so that the
// reader fetches it from HBM whatever the data, instead of hitting lines that
// happen to still sit in some XCD's L2 (FETCH_SIZE would then depend on the
// data; DESIGN.md §3 rule 3).  `base` is an array base (wave-uniform); the
// byte offset 16 * i must be below 2^32.
#ifndef GVS_DIAG_DROP_AUX
#define GVS_DIAG_DROP_AUX (2 | 16)  // nt sc1 (diagnostic builds may change it)
#endif
__device__ inline void st_drop(const void* base, uint64_t i, uint4 x) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const u4v v = {x.x, x.y, x.z, x.w};
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (uint32_t)(i * 16u), 0, GVS_DIAG_DROP_AUX);
}

// 16-B streaming store of a table or mailbox row (buffer_store ... nt sc1:
// non-temporal and written through).  The row passes store every row of the
// table whatever the batch; with plain non-temporal stores the number of
// 64-B HBM write requests (TCC_EA0_WRREQ) moved by thousands per 2^20-row
// pass with the timing of the batch's slot traffic, and the reads around them
// picked up DRAM bubbles (TCC_BUBBLE); written through, both are fixed
// (profiles/r04d_store_policy.txt) and the pass runs 3% faster.  Same
// contract as st_drop: `base` wave-uniform, 16 * i below 2^32.
__device__ inline void st_stream(const void* base, uint64_t i, uint4 x) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const u4v v = {x.x, x.y, x.z, x.w};
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (uint32_t)(i * 16u), 0, 2 /* nt */ | 16 /* sc1 */);
}

// a whole 128-B record of one thread (8 such stores)
template <class T>
__device__ inline void st_drop_rec(T* base, uint64_t i, const T& rec) {
  static_assert(sizeof(T) == 128, "128-B records");
  const uint4* w = reinterpret_cast<const uint4*>(&rec);
#pragma unroll
  for (int c = 0; c < 8; ++c) st_drop(base, i * 8 + c, w[c]);
}

struct alignas(128) OpState {  // seq-indexed, written by k_meta
  uint32_t kind, pre_status, slot, q;
  uint64_t ts, h_hi, h_lo;
  uint32_t id[4];
  uint32_t x[8];  // mailbox key (recipient / auth) for mailbox-touching ops
  uint32_t pad[10];
};
static_assert(sizeof(OpState) == 128, "OpState");

struct alignas(128) M1Out {  // seq-indexed, written by the M1 pass
  uint32_t status, slot, flags, pad;
  uint32_t id[4];
  uint32_t pad2[24];
};
static_assert(sizeof(M1Out) == 128, "M1Out");

struct alignas(128) ROp {  // seq-indexed: everything the R and M2 passes need
  uint32_t status, slot, kind, flags;
  uint32_t id[4];
  uint32_t x[8];
  uint32_t pad[16];
};
static_assert(sizeof(ROp) == 128, "ROp");

struct alignas(128) RRes {  // seq-indexed result of the message pass
  uint32_t status, pad0, pad1, pad2;
  uint32_t pad[28];
};
static_assert(sizeof(RRes) == 128, "RRes");

constexpr uint32_t kRespSlot = 1152;  // internal response slot: 9 whole 128-B lines

struct alignas(16) Key128 {
  uint64_t hi, lo;
};

struct alignas(128) Scal {  // persistent device scalars + per-batch temporaries
  // The error word has a line of its own: every workgroup of every kernel
  // reads it first (a scalar load), and the counters below are written by
  // atomics and single threads during the batch, so sharing their line made
  // the scalar reads' L2 hits depend on what else touched it.
  uint32_t error, pad0[31];
  uint64_t count, ctr, head, tail, n_mailboxes, batches;
  // per batch
  uint64_t pops, scnt, m, count1, head0, tail0, nd;
  uint64_t pad1[3];
};
static_assert(sizeof(Scal) == 256, "Scal: two lines");

struct KeyCtx {
  uint64_t pk0, pk1, hk0, hk1;
  uint32_t tag;     // id plaintext tag of this shard: kIdTag ^ shard << 8
  uint32_t nshards; // S (1 when unsharded)
};

// Plaintext tag of the ids a shard issues (shard < 2^16; shard 0 = kIdTag).
__host__ __device__ inline uint32_t shard_tag(uint32_t shard) { return kIdTag ^ (shard << 8); }

// ------------------------------------------------------------- SipHash-2-4

__host__ __device__ inline uint64_t rotl64(uint64_t x, int b) {
  return (x << b) | (x >> (64 - b));
}

#define GVS_SIPROUND                                                          \
  do {                                                                        \
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);             \
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                                  \
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                                  \
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);             \
  } while (0)

// SipHash-2-4 over full 8-byte blocks m[0..nb) followed by a final block
// carrying `tail` (already packed little-endian) and total length `len`.
__host__ __device__ inline uint64_t siphash24_blocks(uint64_t k0, uint64_t k1,
                                                      const uint64_t* m, int nb,
                                                      uint64_t tail, uint64_t len) {
  uint64_t v0 = 0x736f6d6570736575ULL ^ k0;
  uint64_t v1 = 0x646f72616e646f6dULL ^ k1;
  uint64_t v2 = 0x6c7967656e657261ULL ^ k0;
  uint64_t v3 = 0x7465646279746573ULL ^ k1;
  for (int i = 0; i < nb; ++i) {
    v3 ^= m[i];
    GVS_SIPROUND;
    GVS_SIPROUND;
    v0 ^= m[i];
  }
  uint64_t b = (len << 56) | tail;
  v3 ^= b;
  GVS_SIPROUND;
  GVS_SIPROUND;
  v0 ^= b;
  v2 ^= 0xff;
  GVS_SIPROUND;
  GVS_SIPROUND;
  GVS_SIPROUND;
  GVS_SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

__host__ __device__ inline uint64_t feistel_f(const KeyCtx& k, int r, uint64_t x) {
  uint64_t m[2] = {x, (uint64_t)r};
  return siphash24_blocks(k.pk0, k.pk1, m, 2, 0, 16);
}

// id = PRP(slot | tag<<32, ctr); bytes [0:8) = L, [8:16) = R little-endian
__host__ __device__ inline void id_encode(const KeyCtx& k, uint32_t slot, uint64_t ctr,
                                          uint64_t& L, uint64_t& R) {
  L = (uint64_t)slot | ((uint64_t)k.tag << 32);
  R = ctr;
  for (int r = 0; r < 4; ++r) {
    uint64_t nl = R, nr = L ^ feistel_f(k, r, R);
    L = nl;
    R = nr;
  }
}

__host__ __device__ inline uint64_t id_plain_lo(const KeyCtx& k, uint64_t L, uint64_t R) {
  for (int r = 3; r >= 0; --r) {
    uint64_t nl = R ^ feistel_f(k, r, L), nr = L;
    L = nl;
    R = nr;
  }
  return L;
}

// returns the slot, or kNone when the id does not decode to a valid slot of
// this shard
__host__ __device__ inline uint32_t id_decode(const KeyCtx& k, uint64_t L, uint64_t R,
                                              uint64_t n_slots) {
  L = id_plain_lo(k, L, R);
  if ((uint32_t)(L >> 32) != k.tag) return kNone;
  if ((uint64_t)(uint32_t)L >= n_slots) return kNone;
  return (uint32_t)L;
}

// shard that issued the id, or kNone when it decodes to no valid (shard, slot)
__host__ __device__ inline uint32_t id_shard(const KeyCtx& k, uint64_t L, uint64_t R,
                                             uint64_t n_slots) {
  L = id_plain_lo(k, L, R);
  const uint32_t t = (uint32_t)(L >> 32) ^ kIdTag;
  if ((t & 0xFF0000FFu) != 0u) return kNone;
  const uint32_t s = t >> 8;
  if (s >= k.nshards || (uint64_t)(uint32_t)L >= n_slots) return kNone;
  return s;
}

// recipient PRF over the 32-byte key given as 4 little-endian words
__host__ __device__ inline void recipient_hash(const KeyCtx& k, const uint64_t x[4],
                                               uint64_t& hi, uint64_t& lo) {
  hi = siphash24_blocks(k.hk0, k.hk1, x, 4, 1, 33);
  lo = siphash24_blocks(k.hk0, k.hk1, x, 4, 2, 33);
}

// shard owning the mailbox of recipient key x (and every message addressed to
// it): low 16 bits of h_lo, which neither the mailbox partition (top bits of
// h_hi) nor the group key (h_lo >> 23) uses
__host__ __device__ inline uint32_t shard_of_hash(uint64_t h_lo, uint32_t nshards) {
  return (uint32_t)(h_lo & 0xFFFFu) % nshards;
}

// S1 (mailbox) sort key: hi = h_hi; lo = h_lo[63:23] | class<<21 | seq<<1 | sub
__host__ __device__ inline uint64_t s1_lo(uint64_t h_lo, uint32_t cls, uint32_t seq,
                                          uint32_t sub) {
  return (h_lo & ~((1ull << 23) - 1)) | ((uint64_t)cls << 21) | ((uint64_t)seq << 1) |
         (uint64_t)sub;
}
__host__ __device__ inline uint64_t s1_group(uint64_t lo) { return lo >> 23; }
__host__ __device__ inline uint32_t s1_class(uint64_t lo) { return (uint32_t)(lo >> 21) & 3u; }
__host__ __device__ inline uint32_t s1_seq(uint64_t lo) { return (uint32_t)(lo >> 1) & kSeqMask; }
__host__ __device__ inline uint32_t s1_sub(uint64_t lo) { return (uint32_t)lo & 1u; }

// R-pass sort key: slot' (partition-major row) << 22 | class << 20 | seq
constexpr uint64_t kRNullRow = (1ull << 42) - 1;
__host__ __device__ inline uint64_t r_key(uint64_t row, uint32_t cls, uint32_t seq) {
  return (row << 22) | ((uint64_t)cls << 20) | (uint64_t)seq;
}

// ------------------------------------------------------------- wave helpers

__device__ inline uint32_t lane_id() { return threadIdx.x & 63u; }
// order the wave's LDS stores before its later LDS loads (and vice versa)
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Eight 1040-B records (the caller's gvs_request / gvs_response layout) of one
// wave to `out` (= the first record; i0 a multiple of 8, so the 8320 B are 65
// whole 128-B lines): record r's 1 KiB in v[r], lane r < 8 holds record r's
// 16-B tail word.  Staged in the wave's LDS (`st`, 520 x 16 B) and written
// line by line, each line by one store instruction and written through
// (st_stream): records written one by one left the line two records share to
// two instructions, and its partial write-backs moved WRITE_SIZE with the
// timing.  Records >= nrec are not written.
__device__ inline void wave_put_rec8(uint4* out, uint4* st, const uint4 (&v)[8], uint4 tail, uint32_t nrec) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (uint32_t r = 0; r < 8; ++r) st[r * 65 + lane] = v[r];
  if (lane < 8) st[lane * 65 + 64] = tail;
  wave_lds_sync();
#pragma unroll
  for (uint32_t j = 0; j < 9; ++j) {
    const uint32_t o = j * 64 + lane;
    if (o < 520 && o / 65 < nrec) st_stream(out, o, st[o]);
  }
  wave_lds_sync();
}

__device__ inline uint32_t mbcnt64(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ inline uint4 shfl4(uint4 v, int src) {
  uint4 r;
  r.x = __shfl(v.x, src);
  r.y = __shfl(v.y, src);
  r.z = __shfl(v.z, src);
  r.w = __shfl(v.w, src);
  return r;
}

// bitwise, not &&: a short-circuit chain may compile to exec-mask branches
// that skip code by the data (instruction fetch shows in FETCH_SIZE)
__device__ inline bool eq4(uint4 a, uint4 b) {
  return ((a.x ^ b.x) | (a.y ^ b.y) | (a.z ^ b.z) | (a.w ^ b.w)) == 0u;
}
__host__ __device__ inline bool nz4(uint4 a) { return (a.x | a.y | a.z | a.w) != 0u; }

__host__ __device__ inline uint64_t u4lo(uint4 v) { return (uint64_t)v.x | ((uint64_t)v.y << 32); }
__host__ __device__ inline uint64_t u4hi(uint4 v) { return (uint64_t)v.z | ((uint64_t)v.w << 32); }

// Pin a loaded value: the load must happen here even if the value is only
// used on a rarely taken path (keeps full-table read passes full).
__device__ inline void keep4(uint4& x) {
  asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w));
}

// c ? x : y per component through a mask the optimiser cannot turn back into
// an indexed access (which would move a register array to scratch)
// c ? x : y as mask arithmetic the compiler cannot turn into a branch
__device__ inline uint32_t selu32(bool c, uint32_t x, uint32_t y) {
  uint32_t m = 0u - (uint32_t)c;
  asm volatile("" : "+v"(m));
  return (x & m) | (y & ~m);
}
__device__ inline uint64_t selu64(bool c, uint64_t x, uint64_t y) {
  uint32_t m = 0u - (uint32_t)c;
  asm volatile("" : "+v"(m));
  const uint64_t mm = ((uint64_t)m << 32) | m;
  return (x & mm) | (y & ~mm);
}

__device__ inline uint4 sel4(uint32_t c, uint4 x, uint4 y) {
  uint32_t m = 0u - c;
  asm volatile("" : "+v"(m));
  return make_uint4((x.x & m) | (y.x & ~m), (x.y & m) | (y.y & ~m), (x.z & m) | (y.z & ~m),
                    (x.w & m) | (y.w & ~m));
}

}  // namespace gvs
