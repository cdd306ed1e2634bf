// gvs_kernels.h — gfx950 HIP kernels of the batched oblivious store pipeline.
//
// Per batch (DESIGN.md §3 has the pipeline, §3 "Obliviousness" the rules):
//   k_copy        request AoS (ABI layout) -> 1 KiB request images + type words
//   k_meta        classify, recipient PRF, id decode, mailbox sort keys
//   sort128       LDS-staged bitonic sort of the mailbox keys (S1)
//   (gvs_mtx.h)   group slots, mailbox read pass k_m1x and its scans
//   k_alloc_sum   seq-order flags + block sums (pops, mailbox-ok creates)
//   k_alloc_ring  one workgroup: pops -> free ring; allocation window -> creates
//   k_alloc_b     capacity cutoff, id PRP, message-pass keys
//   sort64        bitonic sort of the message-pass keys
//   (gvs_txn.h)   transaction slots, message table pass k_rpass2 and its scans
//   k_post_sum / k_post_ring   by-id deletes -> free ring, scalar commit
//   (gvs_mtx.h)   mailbox result scans and the write pass k_m2x
//   k_out         internal 1152-B response slots -> caller's 1040-B responses
//
// Every kernel keeps a fixed per-op footprint (same reads and writes for an op
// whatever its kind or outcome), reads/writes every table row exactly once,
// uses 128-B per-op records, and does data-dependent permutations of sub-line
// data only inside a single workgroup.
#pragma once
#include "gvs_device.h"
#include "gvs_seal_dev.h"

namespace gvs {

// ------------------------------------------------------------ sort (bitonic)

template <typename K>
__device__ inline bool key_lt(const K& a, const K& b);
template <>
__device__ inline bool key_lt<uint64_t>(const uint64_t& a, const uint64_t& b) {
  return a < b;
}
// bitwise & and |: a short-circuit || / && may compile to a branch on the
// keys (tests/test_code_object.py checks the sort kernels for any)
template <>
__device__ inline bool key_lt<Key128>(const Key128& a, const Key128& b) {
  return (a.hi < b.hi) | ((a.hi == b.hi) & (a.lo < b.lo));
}

// c ? a : b per component (a select of whole structs goes through scratch)
__device__ inline uint64_t key_sel(bool c, uint64_t a, uint64_t b) { return c ? a : b; }
__device__ inline Key128 key_sel(bool c, const Key128& a, const Key128& b) {
  return Key128{c ? a.hi : b.hi, c ? a.lo : b.lo};
}

__device__ inline uint64_t shfl_xor_key(uint64_t a, uint32_t m) {
  const uint32_t lo = __shfl_xor((uint32_t)a, (int)m), hi = __shfl_xor((uint32_t)(a >> 32), (int)m);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ inline Key128 shfl_xor_key(const Key128& a, uint32_t m) {
  return Key128{shfl_xor_key(a.hi, m), shfl_xor_key(a.lo, m)};
}

// compare-exchange of one element with its partner's copy: keep the smaller
// key if this element is the lower one of an ascending pair (or the upper
// one of a descending pair), else the larger
template <typename K>
__device__ inline K cmpex_keep(const K& mine, const K& other, bool keep_min) {
  const bool lt = key_lt(other, mine);
  return key_sel(lt == keep_min, other, mine);
}

// Bitonic sort of n keys, n a multiple of the tile size L = 1024 * E (not
// necessarily a power of two).  Tiles are sorted ascending by the classic
// network (full = 1: direction of element i at level k from bit k of its
// index inside the tile, so every tile ends ascending).  Merge levels k > L
// use the all-ascending form: the first step of a level pairs i with its
// mirror i ^ (k - 1) in the k-block, the later steps pair i with i + j.  The
// keys past n count as +inf: every comparator puts the smaller key at the
// lower index, so a pair whose upper index is >= n never exchanges and those
// keys are neither read nor written.
//
// k_bitonic_tile: a whole tile sort (full = 1), or the last steps j = L/2 .. 1
// of merge level kmerge (full = 0, ascending).  Thread t holds keys
// t*E .. t*E + E - 1 in registers: steps j < E are register compare-exchanges,
// steps E <= j < 64 E exchange with lane t ^ (j / E) by shuffles, and only
// steps j >= 64 E go through LDS with a barrier each (Key128, 4096-key tiles:
// 10 of the 78 steps of a full tile sort).  The sequence of operations does
// not depend on the keys (a sorting network).
template <typename K, int E>
__global__ __launch_bounds__(1024) void k_bitonic_tile(K* data, uint32_t kmerge, int full) {
  constexpr uint32_t L = 1024u * E;
  __shared__ K s[L];
  const uint32_t t = threadIdx.x, lane = lane_id();
  const uint32_t base = blockIdx.x * L;
  K r[E];
#pragma unroll
  for (int e = 0; e < E; ++e) r[e] = data[base + t * E + e];
  const uint32_t k_lo = full ? 2u : kmerge, k_hi = full ? L : kmerge;
  for (uint32_t k = k_lo; k <= k_hi; k <<= 1) {
    const uint32_t j_top = full ? (k >> 1) : (L >> 1);
    // steps through LDS
    if (j_top >= 64u * E) {
#pragma unroll
      for (int e = 0; e < E; ++e) s[t * E + e] = r[e];
      __syncthreads();
      for (uint32_t j = j_top; j >= 64u * E; j >>= 1) {
        for (uint32_t p = t; p < (L >> 1); p += 1024u) {
          const uint32_t i = ((p / j) * 2u * j) + (p % j);
          const bool asc = !full || (i & k) == 0u;
          const K a = s[i], b = s[i + j];
          const bool sw = asc ? key_lt(b, a) : key_lt(a, b);
          s[i] = key_sel(sw, b, a);
          s[i + j] = key_sel(sw, a, b);
        }
        __syncthreads();
      }
#pragma unroll
      for (int e = 0; e < E; ++e) r[e] = s[t * E + e];
      __syncthreads();  // s is rewritten by the next level
    }
    // steps across lanes
    for (uint32_t m = min(j_top, 32u * E) / E; m >= 1u; m >>= 1) {
      const bool lower = (lane & m) == 0u;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const bool asc = !full || ((t * E + e) & k) == 0u;
        r[e] = cmpex_keep(r[e], shfl_xor_key(r[e], m), lower == asc);
      }
    }
    // steps inside the thread's registers
#pragma unroll
    for (uint32_t j = E / 2; j >= 1u; j >>= 1) {
      if (j <= j_top) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if ((e & j) == 0u) {
            const bool asc = !full || ((t * E + e) & k) == 0u;
            const K a = r[e], b = r[e | j];
            const bool sw = asc ? key_lt(b, a) : key_lt(a, b);
            r[e] = key_sel(sw, b, a);
            r[e | j] = key_sel(sw, a, b);
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) data[base + t * E + e] = r[e];
}

// Two steps (j, j/2) of merge level k over the array: each thread owns the
// four keys whose lowest index is x0 = (block of 2j) + o, o < j/2.  First
// step of the level (flip, j = k/2): quadruple {x0, x0 + h, m - h, m} with
// m = x0 ^ (2j - 1) its mirror; else {x0, x0 + h, x0 + j, x0 + j + h}.
// nq = quadruples with x0 < n.
//
// Every index into x[] / v[] is a compile-time constant and the flip is a
// select, so the four keys stay in registers: a runtime index (the partner
// chosen by flip) put them in scratch, whose loads the compiler then placed
// under branches on the key comparisons (scratch traffic is HBM traffic, and
// it showed in FETCH_SIZE under regular key orders).
template <typename K>
__device__ inline void cx_static(K& a, K& b, bool live) {  // a at the lower index
  const bool sw = live & key_lt(b, a);
  const K ta = a;
  a = key_sel(sw, b, a);
  b = key_sel(sw, ta, b);
}

template <typename K>
__global__ __launch_bounds__(256) void k_bitonic_global2(K* data, uint32_t n, uint32_t k,
                                                         uint32_t j, uint32_t nq) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nq) return;
  const uint32_t h = j >> 1;
  const uint32_t g = p / h, o = p % h;
  const uint32_t x0 = g * 2u * j + o;
  const bool flip = (j << 1) == k;
  const uint32_t m = x0 ^ (2u * j - 1u);
  const uint32_t x1 = x0 + h, x2 = flip ? m - h : x0 + j, x3 = flip ? m : x0 + j + h;
  const bool l1 = x1 < n, l2 = x2 < n, l3 = x3 < n;  // x0 < n: nq counts those
  K v0 = data[x0];
  K v1 = data[l1 ? x1 : x0];
  K v2 = data[l2 ? x2 : x0];
  K v3 = data[l3 ? x3 : x0];
  // first step: pairs (0, 2), (1, 3), or (0, 3), (1, 2) on a level's first step
  K b0 = key_sel(flip, v3, v2), b1 = key_sel(flip, v2, v3);
  cx_static(v0, b0, flip ? l3 : l2);
  cx_static(v1, b1, flip ? l2 : l3);
  v2 = key_sel(flip, b1, b0);
  v3 = key_sel(flip, b0, b1);
  cx_static(v0, v1, l1);
  cx_static(v2, v3, l3);
  data[x0] = v0;
  if (l1) data[x1] = v1;
  if (l2) data[x2] = v2;
  if (l3) data[x3] = v3;
}

// Four steps (j .. j/8) of merge level k: each thread owns the 16 keys of a
// block of 2j at offsets o + a q (q = j/8, o < q, a < 16); on a level's first
// step (flip) the upper eight are the mirrors of the lower eight, stored in
// ascending order (v[8 + b] = mirror of lower key 7 - b), so that the three
// later steps are the same for both.  nq = groups whose lowest key is < n.
// Static indices only, flip as selects (see k_bitonic_global2).
template <typename K>
__global__ __launch_bounds__(256) void k_bitonic_global4(K* data, uint32_t n, uint32_t k,
                                                         uint32_t j, uint32_t nq) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nq) return;
  const uint32_t q = j >> 3;
  const uint32_t base = (p / q) * 2u * j, o = p % q;
  const bool flip = (j << 1) == k;
  uint32_t x[16];
  bool l[16];
#pragma unroll
  for (uint32_t a = 0; a < 16; ++a) {
    // flip: upper key b = mirror of lower key 7 - b = base + j + (q - 1 - o) + b q
    const uint32_t up = base + j + (flip ? q - 1u - o : o) + (a - 8u) * q;
    x[a] = a < 8 ? base + o + a * q : up;
    l[a] = x[a] < n;
  }
  K v[16];
#pragma unroll
  for (uint32_t a = 0; a < 16; ++a) v[a] = data[l[a] ? x[a] : x[0]];
  // step j: (a, a + 8), or on a flip (a, 15 - a)
  K t[8];
#pragma unroll
  for (uint32_t a = 0; a < 8; ++a) {
    t[a] = key_sel(flip, v[15 - a], v[8 + a]);
    cx_static(v[a], t[a], flip ? l[15 - a] : l[8 + a]);
  }
#pragma unroll
  for (uint32_t a = 0; a < 8; ++a) v[8 + a] = key_sel(flip, t[7 - a], t[a]);
  // steps j/2, j/4, j/8 inside each half
#pragma unroll
  for (uint32_t s = 4; s >= 1; s >>= 1)
#pragma unroll
    for (uint32_t a = 0; a < 16; ++a)
      if ((a & s) == 0u) cx_static(v[a], v[a + s], l[a + s]);
#pragma unroll
  for (uint32_t a = 0; a < 16; ++a)
    if (l[a]) data[x[a]] = v[a];
}

// One step j of merge level k: pair (i, i ^ (2j - 1)) on the level's first
// step, else (i, i + j); np = pairs with i < n.
template <typename K>
__global__ __launch_bounds__(256) void k_bitonic_global(K* data, uint32_t n, uint32_t k,
                                                        uint32_t j, uint32_t np) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= np) return;
  const uint32_t i = ((p / j) * 2u * j) + (p % j);
  const uint32_t pj = (j << 1) == k ? i ^ (2u * j - 1u) : i + j;
  if (pj >= n) return;  // +inf partner: no exchange (depends on n only)
  const K a = data[i], b = data[pj];
  const bool sw = key_lt(b, a);
  // both keys are stored whatever the comparison says: a store only on a
  // swap would make the written bytes depend on the key order
  data[i] = key_sel(sw, b, a);
  data[pj] = key_sel(sw, a, b);
}

// ------------------------------------------------------------ block helpers

// Exclusive prefix of a per-thread flag over a 1024-thread block.  Returns the
// prefix; *total gets the block count.  Uses s_w[16].
__device__ inline uint32_t block1024_prefix(bool f, uint32_t* s_w, uint32_t* total) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint64_t m = __ballot(f);
  if (lane == 0) s_w[wave] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (uint32_t w = 0; w < 16; ++w) {
    off += w < wave ? s_w[w] : 0u;
    tot += s_w[w];
  }
  __syncthreads();
  *total = tot;
  return off + mbcnt64(m);
}

// ------------------------------------------------------------------ k_copy

// One wave per request: 64 x 16 B of image + the type word.  Rows >= n are
// padding (zero image, type 0).  `stride` is the input record pitch in 16-B
// units: 65 for the caller's gvs_request array, 72 for routed slots.
//
// Rows >= xbase (expiry sweep on) are the expiry deletes the
// previous message pass recorded: record k = i - xbase becomes a DELETE image
// of msg id with auth = recipient = the stored recipient, internal type
// kTypeExpire if the record is valid, else padding.
constexpr uint32_t kTypeExpire = 0x45585031u;  // never a valid request_type
constexpr uint32_t kCopyPerWave = 8;  // requests per wave in k_copy / k_out (loads in flight together)
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint32_t stride,
                                              uint32_t n, uint32_t B, uint4* __restrict__ img,
                                              uint32_t* __restrict__ types, const uint4* xbuf,
                                              uint32_t xbase) {
  constexpr uint32_t R = kCopyPerWave;
  const uint32_t i0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  const uint32_t lane = lane_id();
  __shared__ uint4 s_rec[4][R * 65];
  if (i0 >= B) return;
  uint4 v[R];
  uint32_t t;
  const uint32_t live = min(n, xbase);
  if (stride == 65) {
    // 1040-B records: the wave's R = 8 of them are 65 whole 128-B lines
    // (aligned: i0 is a multiple of 8), read once each, line by line, and
    // handed out through LDS.  Record by record, the line two records share
    // was requested twice, and whether the second request found it in L2
    // followed the timing (FETCH_SIZE noise of ~50 KiB per batch).
    uint4* st = s_rec[threadIdx.x >> 6];
    const uint4* base = in + (uint64_t)i0 * 65;
#pragma unroll
    for (uint32_t j = 0; j < (R * 65 + 63) / 64; ++j) {
      const uint32_t o = j * 64 + lane;
      if (o < R * 65) st[o] = (i0 + o / 65 < live) ? base[o] : make_uint4(0, 0, 0, 0);
    }
    wave_lds_sync();
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) v[r] = st[r * 65 + lane];
    t = lane < R ? st[min(lane, R - 1u) * 65 + 64].x : 0u;
  } else {  // whole-line records (routed slots: 72 x 16 B)
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {  // wave-uniform conditions
      const uint32_t i = i0 + r;
      v[r] = i < live ? in[(uint64_t)i * stride + lane] : make_uint4(0, 0, 0, 0);
    }
    // type words: lane r < R holds request i0 + r's
    const uint32_t ti = i0 + min(lane, R - 1u);
    t = (lane < R && ti < live) ? in[(uint64_t)ti * stride + 64].x : 0u;
  }
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = i0 + r;
    if (i >= xbase) {
      // lanes 0..5 <- record words id, rcpt lo, rcpt hi, rcpt lo, rcpt hi, valid
      const uint32_t src = lane == 0 ? 0u : (lane < 5 ? 2u - (lane & 1u) : 3u);
      const uint4 x = xbuf[(uint64_t)(i - xbase) * 8 + src];
      const uint32_t tx = __shfl(x.x, 5) ? kTypeExpire : 0u;
      v[r] = lane < 5 ? x : (lane == 5 ? make_uint4(1u, 0, 0, 0) : make_uint4(0, 0, 0, 0));  // nonzero server time
      t = lane == r ? tx : t;
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) img[(uint64_t)(i0 + r) * 64 + lane] = v[r];
  if (lane < R) types[i0 + lane] = t;
}

// ------------------------------------------------------------------ k_meta

struct MetaArgs {
  const uint4* img;
  const uint32_t* types;
  OpState* ops;
  uint32_t* kinds;
  Key128* s1keys;
  uint32_t n, B, Q, logQ;
  uint64_t N;
  KeyCtx kc;
  uint32_t xbase;  // ops >= xbase: expiry deletes (type kTypeExpire) or padding
  uint4* idn;      // B x 128 B: the image's first 80 B (id, sender, recipient), for k_rr1
};

__global__ __launch_bounds__(256) void k_meta(MetaArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* row = a.img + (uint64_t)i * 64;
  uint4 c0 = row[0], c1 = row[1], c2 = row[2], c3 = row[3], c4 = row[4], c5 = row[5];
  {  // the identity words k_rr1 gathers (so that it never re-reads image lines)
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint4 w[8] = {c0, c1, c2, c3, c4, z, z, z};
#pragma unroll
    for (int c = 0; c < 8; ++c) st_drop(a.idn, (uint64_t)i * 8 + c, w[c]);
  }
  const uint32_t raw = a.types[i];
  const bool is_x = i >= a.xbase;
  const uint32_t type = selu32(is_x & (raw == kTypeExpire), 4u, raw);  // DELETE
  OpState o = {};
  o.id[0] = c0.x; o.id[1] = c0.y; o.id[2] = c0.z; o.id[3] = c0.w;
  o.ts = u4lo(c5);
  o.slot = kNone;
  const bool id_zero = !nz4(c0);
  const bool auth_zero = !nz4(c1) && !nz4(c2);
  const bool rcpt_zero = !nz4(c3) && !nz4(c4);
  // Classification without branches: every op runs the same instructions
  // (a skipped branch would leave its code lines unfetched, and instruction
  // fetch shows up in FETCH_SIZE; DESIGN.md §3 rule 6).  Conditions combine
  // with bitwise operators (no short-circuit control flow) and every select
  // chooses between values already computed.
  const bool pad = (is_x & (raw != kTypeExpire)) | (!is_x & (i >= a.n));
  const bool hard = (type < 1u) | (type > 4u) | auth_zero | ((type == 3u) & id_zero);
  const bool create = type == 1u;
  const bool next = ((type == 2u) | (type == 4u)) & id_zero;
  const uint32_t dec = id_decode(a.kc, u4lo(c0), u4hi(c0), a.N);  // every op: fixed work
  const bool nodec = dec == kNone;
  const uint32_t byid_kind =
      selu32(type == 2u, KIND_READ, selu32(type == 3u, KIND_UPDATE, KIND_DELETE));
  const uint32_t next_kind = selu32(type == 2u, KIND_NEXT_READ, KIND_NEXT_DEL);
  const bool fail = pad | hard;
  const bool byid = !fail & !create & !next;
  uint32_t kind = selu32(next, next_kind, byid_kind);
  kind = selu32(create, KIND_CREATE, kind);
  kind = selu32(hard, KIND_HARD, kind);
  kind = selu32(pad, KIND_PAD, kind);
  // grapevine.proto:57-64, :95 fail-fast; :72 INVALID_RECIPIENT; NOT_FOUND
  // when the id names no slot
  uint32_t pre = selu32(byid & nodec, 2u, kPending);
  pre = selu32(create, selu32(rcpt_zero, 4u, kPending), pre);
  pre = selu32(fail, 0u, pre);
  uint32_t cls = selu32((byid_kind == KIND_DELETE) & !nodec & !rcpt_zero, 2u, 3u);
  cls = selu32(next, 0u, cls);
  cls = selu32(create, selu32(rcpt_zero, 3u, 1u), cls);
  cls = selu32(fail, 3u, cls);
  const uint32_t sub = (uint32_t)(next & (type == 4u));
  o.slot = selu32(byid, dec, kNone);
  const uint4 xa = sel4(next, c1, c3), xb = sel4(next, c2, c4);  // mailbox key: recipient, or auth
  o.x[0] = xa.x; o.x[1] = xa.y; o.x[2] = xa.z; o.x[3] = xa.w;
  o.x[4] = xb.x; o.x[5] = xb.y; o.x[6] = xb.z; o.x[7] = xb.w;
  Key128 key;
  uint32_t q;
  {
    // the PRF runs for every op (fixed work); only participants use it
    const uint64_t x[4] = {u4lo(xa), u4hi(xa), u4lo(xb), u4hi(xb)};
    uint64_t hi, lo;
    recipient_hash(a.kc, x, hi, lo);
    const bool part = cls < 3u;
    const uint32_t q_part = a.logQ ? (uint32_t)(hi >> (64 - a.logQ)) : 0u;
    const uint64_t lo_part = s1_lo(lo, cls, i, sub);
    const uint64_t lo_none = (~0ull << 21) | ((uint64_t)i << 1);
    o.h_hi = selu64(part, hi, 0ull);
    o.h_lo = selu64(part, lo, 0ull);
    q = selu32(part, q_part, a.Q);
    key.hi = selu64(part, hi, ~0ull);
    key.lo = selu64(part, lo_part, lo_none);
  }
  o.kind = kind;
  o.pre_status = pre;
  o.q = q;
  st_drop_rec(a.ops, i, o);  // read by the scans in sorted order
  a.kinds[i] = kind;
  a.s1keys[i] = key;
}

// ------------------------------------------------------ mailbox passes M1/M2

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#ifndef GVS_DIAG_NT
#define GVS_DIAG_NT 0  // diagnostic builds only: every ld_row non-temporal
#endif
template <bool NT>
__device__ inline uint4 ld_row(const uint4* p) {
  if (NT || GVS_DIAG_NT) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
template <bool NT>
__device__ inline void st_row(uint4* p, uint4 x) {
  if (NT) {
    v4u v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  } else {
    *p = x;
  }
}

constexpr int kMU = 8;  // mailbox rows per wave and chunk in the M1/M2 row passes
constexpr uint32_t kMDryU4 = 512;  // a mailbox partition's dry block: 8 x 1 KiB (k_m1x 0..3, k_m2x 4..7)

// One chunk of kMU rows (16 B per lane each), loads issued back to back
// without branches; a chunk that runs past Sr (Sr not a multiple of 4 kMU)
// re-reads the last row for the missing ones, a fixed per-config footprint.
__device__ inline void load_rows(uint4 (&v)[kMU], const uint4* part, uint32_t j0, uint32_t Sr) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < kMU; ++u)
    v[u] = ld_row<true>(&part[(uint64_t)min(j0 + u, Sr - 1u) * 64 + lane]);
}


struct MArgs {
  const Key128* keys;
  uint4* mbox;             // R rows x 64 uint4
  uint4* side;             // R entries
  M1Out* m1out;
  const ROp* rop;          // M2
  const RRes* rres;        // M2
  Scal* scal;
  uint32_t Q, Sr, B;
  uint64_t N;
  KeyCtx kc;
  SealCtx sc;          // authenticated storage (AUTH instantiations)
  const uint32_t* te;  // AES table (256 words)
  uint4* btag;         // R mailbox row tags
  // fixed-slot mailbox passes (gvs_mtx.h)
  const uint4* gtx;    // Q*cm group descriptors (128 B) of this batch
  const uint4* m2tx;   // Q*cm group results (1152 B) for the write pass
  uint4* msnap;        // Q*cm x 1 KiB: the read pass's sink for unused group slots
  uint4* msnapp;       // B x 1 KiB: group snapshots at their heads' sorted positions
  uint4* mdry;         // Q x 8 KiB: each workgroup's dry-run lines (gvs_mtx.h: one 1 KiB per use)
  uint32_t stamp, cm;
  uint32_t sink_mul;   // MSNAP sink line of global slot x: x * sink_mul mod Q*cm (a permutation)
};

// ---------------------------------------------------------- allocation

struct AllocArgs {
  const uint32_t* kinds;
  const M1Out* m1out;
  const OpState* ops;
  uint32_t* pflag;  // bit0 pop, bit1 mailbox-ok create
  uint32_t* pslot;  // popped slot
  uint32_t* bsum;   // 2 per block
  uint32_t* cslot;  // allocated slot per op (kNone if not a successful create)
  uint32_t* ring;
  ROp* rop;
  uint64_t* rkeys;
  Scal* scal;
  uint32_t B, nblk, W, S;
  uint64_t N, ring_size;
  KeyCtx kc;
};

constexpr uint32_t kWinGroup = 8;      // blocks per allocation-window refill
constexpr uint32_t kWinRing = 16384;  // LDS window ring: one group + one chunk fits

// Free-ring index of entry `off` after the ring counter whose residue is
// `base` (= counter mod m, computed once per kernel from the wave-uniform
// counter), off < 2m (window reads run up to B + 1023 past the counter):
// two selects.  A per-element 64-bit `%` expands to a branch
// on the high word of its operand, so the code fetched would follow the data
// (instruction fetch shows in FETCH_SIZE; DESIGN.md §3 rule 6).
__device__ inline uint32_t ring_at(uint32_t base, uint32_t off, uint32_t m) {
  uint32_t x = base + off;
  x = x >= m ? x - m : x;
  return x >= m ? x - m : x;
}

// seq-order compact flags (coalesced, fixed) + per-block counts; pflag holds
// bit 0 pop, bit 1 mailbox-ok create, bits 2..11 / 12..21 their in-block
// exclusive prefixes
__global__ __launch_bounds__(1024) void k_alloc_sum(AllocArgs a) {
  __shared__ uint32_t s_w[16];
  if (a.scal->error) return;
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const M1Out m1 = a.m1out[i];
  const uint32_t kind = a.kinds[i];
  const bool pop = (m1.flags & CF_POP) != 0u;
  const bool s = (m1.flags & CF_MBOX_OK) != 0u && kind == KIND_CREATE;
  a.pslot[i] = m1.slot;
  uint32_t tp, ts;
  const uint32_t pp = block1024_prefix(pop, s_w, &tp);
  const uint32_t ps = block1024_prefix(s, s_w, &ts);
  a.pflag[i] = (pop ? 1u : 0u) | (s ? 2u : 0u) | (pp << 2) | (ps << 12);
  if (threadIdx.x == 0) {
    a.bsum[2 * blockIdx.x] = tp;
    a.bsum[2 * blockIdx.x + 1] = ts;
  }
}

// One workgroup: (1) delete-next pops -> free ring window [tail, tail+B) in seq
// order (a permutation of the window); (2) the allocation window
// [head, head+B) is read in order, exactly once, and its first m entries are
// handed to the successful creates in seq order (TOO_MANY_MESSAGES cutoff).
__global__ __launch_bounds__(1024) void k_alloc_ring(AllocArgs a) {
  __shared__ uint32_t s_off[2][1024];
  __shared__ uint32_t s_win[kWinRing];
  __shared__ uint32_t s_stage[kWinGroup][1024];
  const uint32_t tid = threadIdx.x;
  if (a.scal->error) return;
  // block offsets (nblk <= 1024)
  uint32_t vp = tid < a.nblk ? a.bsum[2 * tid] : 0u, vs = tid < a.nblk ? a.bsum[2 * tid + 1] : 0u;
  s_off[0][tid] = vp;
  s_off[1][tid] = vs;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint32_t x = tid >= off ? s_off[0][tid - off] : 0u, y = tid >= off ? s_off[1][tid - off] : 0u;
    __syncthreads();
    s_off[0][tid] += x;
    s_off[1][tid] += y;
    __syncthreads();
  }
  const uint32_t pops = s_off[0][1023], scnt = s_off[1][1023];
  Scal* sc = a.scal;
  const uint64_t tail0 = sc->tail, head0 = sc->head;
  const uint32_t rs = (uint32_t)a.ring_size;
  const uint32_t tbase = (uint32_t)(tail0 % a.ring_size), hbase = (uint32_t)(head0 % a.ring_size);
  const uint64_t count1 = sc->count - pops;
  const uint64_t room = a.N - count1;
  const uint64_t m = scnt < room ? scnt : room;
  // (1) pops -> ring.  In-block prefixes come from k_alloc_sum (pflag bits
  // 2..11), so the blocks are independent: no barrier, loads in flight
  // together.
  for (uint32_t c0 = 0; c0 < a.nblk; c0 += kWinGroup) {
    uint32_t f[kWinGroup], slot[kWinGroup];  // loads of 8 blocks in flight together
#pragma unroll
    for (uint32_t u = 0; u < kWinGroup; ++u) {
      const uint32_t i = (c0 + u) * 1024 + tid;
      f[u] = c0 + u < a.nblk ? a.pflag[i] : 0u;
      slot[u] = c0 + u < a.nblk ? a.pslot[i] : 0u;
    }
    // each block's 1024 entries staged in LDS in window order (its pops,
    // then the rest) and written by consecutive threads: written straight
    // from the lanes, a wave's stores formed one run or two by the data, and
    // batches with pops ran 2-4 us slower (profiles/r05n_timing_c3_store.txt;
    // the free ring's other writer, k_post_ring, rule 13)
#pragma unroll
    for (uint32_t u = 0; u < kWinGroup; ++u) {
      const uint32_t c = c0 + u;
      if (c < a.nblk) {
        const bool pop = f[u] & 1u;
        const uint32_t pp = (f[u] >> 2) & 1023u, P0 = c ? s_off[0][c - 1] : 0u, tp = s_off[0][c] - P0;
        s_stage[u][pop ? pp : tp + (tid - pp)] = pop ? slot[u] : kNone;
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < kWinGroup; ++u) {
      const uint32_t c = c0 + u;
      if (c < a.nblk) {
        const uint32_t P0 = c ? s_off[0][c - 1] : 0u, tp = s_off[0][c] - P0;
        const uint32_t pos = tid < tp ? P0 + tid : pops + (c * 1024 - P0) + (tid - tp);
        a.ring[ring_at(tbase, pos, rs)] = s_stage[u][tid];
      }
    }
    __syncthreads();  // the stage is refilled by the next group
  }
  __threadfence_block();
  __syncthreads();
  // (2) allocation window [head, head + B), read in order in 1024-entry
  // chunks through an LDS ring; groups of 8 blocks (8192 ops) share one
  // refill and two barriers
  uint32_t loaded = 0;  // window entries loaded so far (multiple of 1024)
  for (uint32_t c0 = 0; c0 < a.nblk; c0 += kWinGroup) {
    const uint32_t c1 = min(c0 + kWinGroup, a.nblk);
    const uint32_t need = (uint32_t)min((uint64_t)s_off[1][c1 - 1], m);
    // refill: up to kWinGroup + 1 chunks, all loads issued before the stores
    uint32_t w[kWinGroup + 1];
#pragma unroll
    for (uint32_t k = 0; k <= kWinGroup; ++k) {
      const uint32_t pos = loaded + k * 1024;
      w[k] = pos < need ? a.ring[ring_at(hbase, pos + tid, rs)] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k <= kWinGroup; ++k) {
      const uint32_t pos = loaded + k * 1024;
      if (pos < need) s_win[(pos + tid) & (kWinRing - 1u)] = w[k];
    }
    while (loaded < need) loaded += 1024;  // uniform across the block
    __syncthreads();
    uint32_t f[kWinGroup];
#pragma unroll
    for (uint32_t u = 0; u < kWinGroup; ++u) f[u] = c0 + u < c1 ? a.pflag[(c0 + u) * 1024 + tid] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < kWinGroup; ++u) {
      const uint32_t c = c0 + u, i = c * 1024 + tid;
      if (c < c1) {
        const uint32_t Si = (c ? s_off[1][c - 1] : 0u) + ((f[u] >> 12) & 1023u);
        const bool success = (f[u] & 2u) && (uint64_t)Si < m;
        a.cslot[i] = success ? s_win[Si & (kWinRing - 1u)] : kNone;
      }
    }
    __syncthreads();  // the next refill overwrites the ring
  }
  // read the rest of the window (fixed B entries per batch), 8 chunks in flight
  for (; loaded < a.B; loaded += 8 * 1024) {
    uint32_t v[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t pos = loaded + k * 1024;
      v[k] = pos < a.B ? a.ring[ring_at(hbase, pos + tid, rs)] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) asm volatile("" ::"v"(v[k]));
  }
  if (tid == 0) {
    sc->pops = pops;
    sc->scnt = scnt;
    sc->count1 = count1;
    sc->m = m;
    sc->head0 = head0;
    sc->tail0 = tail0;
  }
}

// Per op: statuses, ids, message-pass routing keys, partition histogram.
// 256-thread workgroups: in 1024-thread ones the kernel ran on a quarter of
// the CUs (B / 1024 = 64 workgroups at C3), as k_meta did
__global__ __launch_bounds__(256) void k_alloc_b(AllocArgs a) {
  const uint32_t tid = threadIdx.x;
  if (a.scal->error) return;
  // S_i: offset of the op's 1024-op block + its in-block prefix of
  // mailbox-ok creates (k_alloc_sum, pflag bits 12..21)
  const uint32_t i = blockIdx.x * 256 + tid, c = i >> 10;
  uint32_t boff = 0;
  for (uint32_t b = 0; b < c; ++b) boff += a.bsum[2 * b + 1];
  const uint32_t f = a.pflag[i];
  const uint32_t S_i = boff + ((f >> 12) & 1023u);
  const uint32_t kind = a.kinds[i];
  const OpState os = a.ops[i];
  const M1Out m1 = a.m1out[i];
  const uint32_t cs = a.cslot[i];
  const Scal* sc = a.scal;
  const uint64_t count1 = sc->count1, ctr0 = sc->ctr;

  // every case computed, the op's own selected (no branch over op kinds: a
  // block of padding ops would skip the code, and instruction fetch shows in
  // FETCH_SIZE)
  uint64_t L, R;
  id_encode(a.kc, cs == kNone ? 0u : cs, ctr0 + S_i, L, R);  // fixed work for every op
  const bool c_cr = kind == KIND_CREATE && os.pre_status == kPending;
  const bool cr_full = count1 + S_i >= a.N, cr_ok = !cr_full && cs != kNone;
  const bool c_nx = kind == KIND_NEXT_READ || kind == KIND_NEXT_DEL;
  const bool nx_ok = m1.status == kPending;
  const bool c_id = kind == KIND_READ || kind == KIND_UPDATE || kind == KIND_DELETE;
  ROp r = {};
  r.kind = kind;
  // CREATE: TOO_MANY_MESSAGES (7) checked before 5/6 from the mailbox pass
  const uint32_t st_cr = selu32(cr_full, 7u, selu32(cs == kNone, m1.status, kPending));
  r.status = selu32(c_cr, st_cr, selu32(c_nx, m1.status, os.pre_status));
  r.slot = selu32(c_cr && cr_ok, cs, selu32(c_nx && nx_ok, m1.slot, selu32(c_id, os.slot, kNone)));
  const uint32_t nid[4] = {(uint32_t)L, (uint32_t)(L >> 32), (uint32_t)R, (uint32_t)(R >> 32)};
  for (int k = 0; k < 4; ++k)
    r.id[k] = selu32(c_cr && cr_ok, nid[k], selu32(c_nx && nx_ok, m1.id[k], os.id[k]));
  for (int k = 0; k < 8; ++k) r.x[k] = os.x[k];
  const bool c_id_ok = c_id && os.slot != kNone;
  const uint32_t cls = selu32(c_cr && cr_ok, 1u, selu32(c_nx && nx_ok, 0u, selu32(c_id_ok, 2u, 3u)));
  st_drop_rec(a.rop, i, r);  // read by the scans in sorted order
  const bool real = cls < 3u;
  const uint32_t sl = r.slot;
  const uint64_t rowc = (uint64_t)(sl % a.W) * a.S + sl / a.W;  // computed for every op
  const uint64_t rowp = real ? rowc : kRNullRow;
  const uint32_t rcls = selu32(real, cls, 0u);
  a.rkeys[i] = r_key(rowp, rcls, i);
}

constexpr uint32_t kXepMax = 8;  // expiry records per workgroup (one store instruction)

// ------------------------------------------------------------ post-R commit

struct PostArgs {
  const uint32_t* kinds;
  const RRes* rres;
  const ROp* rop;
  uint32_t* dflag;
  uint32_t* dslot;
  uint32_t* bsum;
  uint32_t* ring;
  Scal* scal;
  uint32_t B, nblk;
  uint64_t ring_size;
};

__global__ __launch_bounds__(1024) void k_post_sum(PostArgs a) {
  __shared__ uint32_t s_w[16];
  if (a.scal->error) return;
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t st = a.rres[i].status, slot = a.rop[i].slot;
  const bool d = a.kinds[i] == KIND_DELETE && st == 1u;
  a.dslot[i] = slot;
  uint32_t tot;
  const uint32_t pre = block1024_prefix(d, s_w, &tot);
  a.dflag[i] = (d ? 1u : 0u) | (pre << 1);  // flag + in-block exclusive prefix
  if (threadIdx.x == 0) a.bsum[blockIdx.x] = tot;
}

// one workgroup: by-id deletes -> free ring in seq order; commit scalars.
// Block c's entries go to two runs of the ring window, its deletes' and the
// rest's; they are staged in LDS in run order and written by consecutive
// threads, so that every wave writes consecutive ring entries whatever the
// split (scattered straight from the lanes, a wave's writes formed one run or
// two by the data: k_post_ring 2.7 us faster at C3 without by-id deletes).
__global__ __launch_bounds__(1024) void k_post_ring(PostArgs a) {
  __shared__ uint32_t s_off[1024];
  __shared__ uint32_t s_run[8][1024];
  const uint32_t tid = threadIdx.x;
  if (a.scal->error) return;
  s_off[tid] = tid < a.nblk ? a.bsum[tid] : 0u;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint32_t x = tid >= off ? s_off[tid - off] : 0u;
    __syncthreads();
    s_off[tid] += x;
    __syncthreads();
  }
  const uint32_t nd = s_off[1023];
  Scal* sc = a.scal;
  const uint32_t rs = (uint32_t)a.ring_size;
  const uint32_t tbase = (uint32_t)((sc->tail0 + sc->pops) % a.ring_size);
  for (uint32_t c0 = 0; c0 < a.nblk; c0 += 8) {  // no barrier: blocks are independent
    uint32_t f[8], slot[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      const uint32_t i = (c0 + u) * 1024 + tid;
      f[u] = c0 + u < a.nblk ? a.dflag[i] : 0u;
      slot[u] = c0 + u < a.nblk ? a.dslot[i] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {  // run order: the block's deletes, then the rest
      const uint32_t c = c0 + u;
      const bool d = f[u] & 1u;
      const uint32_t Dc = c < a.nblk ? s_off[c] - (c ? s_off[c - 1] : 0u) : 0u, r = f[u] >> 1;
      s_run[u][d ? r : Dc + (tid - r)] = d ? slot[u] : kNone;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      const uint32_t c = c0 + u;
      if (c < a.nblk) {
        const uint32_t P0 = c ? s_off[c - 1] : 0u, Dc = s_off[c] - P0;
        const uint32_t pos = tid < Dc ? P0 + tid : nd + c * 1024 - P0 + (tid - Dc);
        a.ring[ring_at(tbase, pos, rs)] = s_run[u][tid];
      }
    }
    __syncthreads();  // the next group restages
  }
  if (tid == 0) {
    sc->nd = nd;
    sc->count = sc->count1 + sc->m - nd;
    sc->head = sc->head0 + sc->m;
    sc->tail = sc->tail0 + sc->pops + nd;
    sc->ctr += sc->m;
    sc->batches += 1;
  }
}

// block-wide exclusive prefix of a per-index flag over [0, n) (n <= 1024),
// result in out[0..n], out[n] = total.  All 256 threads must call.
__device__ inline void block_flag_scan(const uint8_t* flag, uint32_t n, uint16_t* out,
                                       uint32_t* s_w) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n || base == 0; base += 256) {  // runs even for n = 0
    const uint32_t i = base + tid;
    const bool f = i < n && flag[i];
    const uint64_t m = __ballot(f);
    if (lane == 0) s_w[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (uint32_t w = 0; w < 4; ++w) {
      off += w < wave ? s_w[w] : 0u;
      tot += s_w[w];
    }
    if (i < n) out[i] = (uint16_t)(carry + off + mbcnt64(m));
    carry += tot;
    __syncthreads();
  }
  if (tid == 0) out[n] = (uint16_t)carry;
  __syncthreads();
}
// ------------------------------------------------------------------ k_out

// internal response slots (kRespSlot B, whole lines) -> caller layout (1040 B),
// kCopyPerWave responses per wave, written as whole lines (wave_put_rec8)
__global__ __launch_bounds__(256) void k_out(const uint4* __restrict__ resp, uint32_t n,
                                             uint4* __restrict__ out) {
  constexpr uint32_t R = kCopyPerWave;
  static_assert(R == 8, "wave_put_rec8");
  __shared__ uint4 s_rec[4][R * 65];
  const uint32_t i0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  const uint32_t lane = lane_id();
  if (i0 >= n) return;
  uint4 v[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r)
    v[r] = i0 + r < n ? resp[(uint64_t)(i0 + r) * (kRespSlot / 16) + lane] : make_uint4(0, 0, 0, 0);
  const uint32_t si = i0 + min(lane, R - 1u);
  const uint4 st = (lane < R && si < n) ? resp[(uint64_t)si * (kRespSlot / 16) + 64] : make_uint4(0, 0, 0, 0);
  wave_put_rec8(out + (uint64_t)i0 * 65, s_rec[threadIdx.x >> 6], v, st, n - i0);
}

}  // namespace gvs
