// gvs_kernels.h — gfx950 HIP kernels of the batched oblivious store pipeline.
//
// Per batch (DESIGN.md §3 has the pipeline, §3 "Obliviousness" the rules):
//   k_copy        request AoS (ABI layout) -> 1 KiB request images + type words
//   k_meta        classify, recipient PRF, id decode, mailbox sort keys, histogram
//   sort128       LDS-staged bitonic sort of the mailbox keys (S1)
//   k_m1          mailbox read pass: resolve next-message ops, create admission
//   k_alloc_sum   seq-order flags + block sums (pops, mailbox-ok creates)
//   k_alloc_ring  one workgroup: pops -> free ring; allocation window -> creates
//   k_alloc_b     capacity cutoff, id PRP, message-pass keys + histogram
//   sort64        bitonic sort of the message-pass keys
//   k_rpass       message table pass: stream every row, apply ops, emit responses
//   k_post_sum / k_post_ring   by-id deletes -> free ring, scalar commit
//   k_m2          mailbox write pass: pops, appends, removals, new mailboxes
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
template <>
__device__ inline bool key_lt<Key128>(const Key128& a, const Key128& b) {
  return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
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

// Bitonic sort inside tiles of L = 1024 * E keys (full = 1), or the last
// steps j = L/2 .. 1 of merge level kmerge (full = 0).  Thread t holds keys
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
          const bool asc = ((base + i) & k) == 0u;
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
        const bool asc = ((base + t * E + e) & k) == 0u;
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
            const bool asc = ((base + t * E + e) & k) == 0u;
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

// Two steps (j, j/2) of merge level k over the whole array: each thread owns
// the four keys i0, i0 + j/2, i0 + j, i0 + 3j/2.
template <typename K>
__global__ __launch_bounds__(256) void k_bitonic_global2(K* data, uint32_t n, uint32_t k,
                                                         uint32_t j) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (n >> 2)) return;
  const uint32_t h = j >> 1;
  // a group of 2j indices holds h quadruples x0, x0 + h, x0 + j, x0 + j + h
  const uint32_t g = p / h, o = p % h;
  const uint32_t x0 = g * 2u * j + o;  // bits h and j of x0 are zero
  const uint32_t x1 = x0 + h, x2 = x0 + j, x3 = x0 + j + h;
  const bool asc = (x0 & k) == 0u;
  K v0 = data[x0], v1 = data[x1], v2 = data[x2], v3 = data[x3];
  auto cx = [&](K& a, K& b) {
    const bool sw = asc ? key_lt(b, a) : key_lt(a, b);
    const K ta = a;
    a = key_sel(sw, b, a);
    b = key_sel(sw, ta, b);
  };
  cx(v0, v2);
  cx(v1, v3);
  cx(v0, v1);
  cx(v2, v3);
  data[x0] = v0;
  data[x1] = v1;
  data[x2] = v2;
  data[x3] = v3;
}

template <typename K>
__global__ __launch_bounds__(256) void k_bitonic_global(K* data, uint32_t n, uint32_t k,
                                                        uint32_t j) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (n >> 1)) return;
  uint32_t i = ((p / j) * 2u * j) + (p % j);
  uint32_t pj = i + j;
  bool asc = ((i & k) == 0u);
  const K a = data[i], b = data[pj];
  const bool sw = asc ? key_lt(b, a) : key_lt(a, b);
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

// out[i] = sum(in[0..i)), out[n] = total.  One block of 1024 threads; n is
// small (histogram bins).
__global__ __launch_bounds__(1024) void k_scan_excl(const uint32_t* in, uint32_t* out,
                                                    uint32_t n) {
  __shared__ uint32_t s[1024];
  const uint32_t T = blockDim.x, t = threadIdx.x;
  const uint32_t per = (n + T - 1) / T;
  const uint32_t lo = t * per, hi = min(n, lo + per);
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += in[i];
  s[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < T; off <<= 1) {
    uint32_t v = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  uint32_t run = s[t] - sum;
  for (uint32_t i = lo; i < hi; ++i) {
    uint32_t v = in[i];
    out[i] = run;
    run += v;
  }
  if (t == T - 1) out[n] = s[T - 1];
}

// LDS histogram of one 1024-op block, then every bin (zeros included) added to
// the global histogram: a fixed set of atomics whatever the bins' contents.
__device__ inline void hist_flush(uint32_t* s_hist, uint32_t nbins, uint32_t* g_hist) {
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x) atomicAdd(&g_hist[b], s_hist[b]);
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
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint32_t stride,
                                              uint32_t n, uint32_t B, uint4* __restrict__ img,
                                              uint32_t* __restrict__ types, const uint4* xbuf,
                                              uint32_t xbase) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  if (i >= B) return;
  uint4 v = make_uint4(0, 0, 0, 0);
  uint32_t t = 0;
  if (i >= xbase) {
    // lanes 0..5 <- record words id, rcpt lo, rcpt hi, rcpt lo, rcpt hi, valid
    const uint32_t src = lane == 0 ? 0u : (lane < 5 ? 2u - (lane & 1u) : 3u);
    const uint4* rec = xbuf + (uint64_t)(i - xbase) * 8;
    const uint4 x = rec[src];
    t = __shfl(x.x, 5) ? kTypeExpire : 0u;
    if (lane < 5) v = x;
    if (lane == 5) v = make_uint4(1u, 0, 0, 0);  // nonzero server time (response unused)
  } else {
    if (i < n) v = in[(uint64_t)i * stride + lane];
    if (i < n && lane == 0) t = in[(uint64_t)i * stride + 64].x;
  }
  img[(uint64_t)i * 64 + lane] = v;
  if (lane == 0) types[i] = t;
}

// ------------------------------------------------------------------ k_meta

struct MetaArgs {
  const uint4* img;
  const uint32_t* types;
  OpState* ops;
  uint32_t* kinds;
  Key128* s1keys;
  uint32_t* qcount;  // Q+1 counters
  uint32_t n, B, Q, logQ;
  uint64_t N;
  KeyCtx kc;
  uint32_t xbase;  // ops >= xbase: expiry deletes (type kTypeExpire) or padding
};

__global__ __launch_bounds__(1024) void k_meta(MetaArgs a) {
  __shared__ uint32_t s_hist[kBinsMax];
  for (uint32_t b = threadIdx.x; b <= a.Q; b += blockDim.x) s_hist[b] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* row = a.img + (uint64_t)i * 64;
  uint4 c0 = row[0], c1 = row[1], c2 = row[2], c3 = row[3], c4 = row[4], c5 = row[5];
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
  a.ops[i] = o;
  a.kinds[i] = kind;
  a.s1keys[i] = key;
  atomicAdd(&s_hist[q], 1u);
  hist_flush(s_hist, a.Q + 1, a.qcount);
}

// ------------------------------------------------------ mailbox passes M1/M2

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ inline uint4 ld_row(const uint4* p) {
  if (NT) {
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

// One chunk of kMU rows (16 B per lane each), loads issued back to back
// without branches; a chunk that runs past Sr (Sr not a multiple of 4 kMU)
// re-reads the last row for the missing ones, a fixed per-config footprint.
__device__ inline void load_rows(uint4 (&v)[kMU], const uint4* part, uint32_t j0, uint32_t Sr) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < kMU; ++u)
    v[u] = ld_row<true>(&part[(uint64_t)min(j0 + u, Sr - 1u) * 64 + lane]);
}


struct GroupL {  // 64 B LDS descriptor of one recipient group
  uint64_t hi, glo;
  uint32_t first, n_next, n_del, n_create;
  uint32_t n_x, fcs, len, flags;
  int32_t slot;
  uint32_t n_succ, n_delok, fl;
};

struct MArgs {
  const Key128* keys;
  const uint32_t* qstart;  // Q+2 entries
  uint4* mbox;             // R rows x 64 uint4
  uint4* side;             // R entries
  M1Out* m1out;
  const ROp* rop;          // M2
  const RRes* rres;        // M2
  Scal* scal;
  uint32_t Q, Sr, B, dummy_blocks;
  uint64_t N;
  KeyCtx kc;
  SealCtx sc;          // authenticated storage (AUTH instantiations)
  const uint32_t* te;  // AES table (256 words)
  uint4* btag;         // R mailbox row tags
  // fixed-slot mailbox passes (gvs_mtx.h)
  const uint4* gtx;    // Q*cm group descriptors (128 B) of this batch
  const uint4* m2tx;   // Q*cm group results (1152 B) for the write pass
  uint4* msnap;        // Q*cm group snapshots (1 KiB) from the read pass
  uint4* mdry;         // Q x 1 KiB: each workgroup's dry-run line
  uint32_t stamp, cm;
};

// packed per-op info kept in LDS: seq | class<<20 | sub<<22 | success<<23
__device__ inline uint32_t pack_s1(uint64_t lo, uint32_t succ) {
  return s1_seq(lo) | (s1_class(lo) << 20) | (s1_sub(lo) << 22) | (succ << 23);
}
__device__ inline uint32_t pk_seq(uint32_t p) { return p & kSeqMask; }
__device__ inline uint32_t pk_sub(uint32_t p) { return (p >> 22) & 1u; }
__device__ inline uint32_t pk_succ(uint32_t p) { return (p >> 23) & 1u; }

// Per-op info of sorted position m of the partition starting at `start`.
// Positions beyond the LDS stash (a partition with > kStash ops in one batch)
// re-read the key (and for M2 the status): correct, but a data-dependent read.
template <bool kM2>
__device__ inline uint32_t op_info(const MArgs& a, const uint32_t* stash, uint32_t start,
                                   uint32_t m) {
  const uint32_t k = m - start;
  if (k < (uint32_t)kStash) return stash[k];
  const Key128 key = a.keys[m];
  uint32_t succ = 0;
  if (kM2) succ = a.rres[s1_seq(key.lo)].status == 1u ? 1u : 0u;
  return pack_s1(key.lo, succ);
}

// Phase A shared by M1 and M2: discover the groups of the sorted key range
// [start, end) into LDS and stash each op's packed info.  Each key (and for M2
// each op's status) is read exactly once.  Returns the group count, or
// kGroupMax+1 on overflow.
template <bool kM2>
__device__ uint32_t discover_groups(const MArgs& a, uint32_t start, uint32_t end,
                                    GroupL* g, uint32_t* stash, Key128* s_key,
                                    uint32_t* s_w, uint32_t* s_ng) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  if (tid == 0) *s_ng = 0;
  Key128 last = {~0ull, ~0ull};
  // at least one (possibly empty) iteration: the same code runs in every workgroup
  for (uint32_t base = start; base < end || base == start; base += 256) {
    const uint32_t i = base + tid;
    const bool valid = i < end;
    Key128 key = {~0ull, ~0ull};
    uint32_t succ = 0;
    if (valid) {
      key = a.keys[i];
      if (kM2) succ = a.rres[s1_seq(key.lo)].status == 1u ? 1u : 0u;
    }
    s_key[tid] = key;
    __syncthreads();
    const Key128 prev = tid > 0 ? s_key[tid - 1] : last;
    last = s_key[255];
    const bool head = valid && (i == start || key.hi != prev.hi ||
                                s1_group(key.lo) != s1_group(prev.lo));
    const uint64_t bm = __ballot(head);
    const uint32_t pre = mbcnt64(bm);
    if (lane == 0) s_w[wave] = (uint32_t)__popcll(bm);
    __syncthreads();
    uint32_t woff = 0, tot = 0;
    for (uint32_t w = 0; w < 4; ++w) {
      woff += w < wave ? s_w[w] : 0u;
      tot += s_w[w];
    }
    const uint32_t ng0 = *s_ng;
    const uint32_t incl = ng0 + woff + pre + (head ? 1u : 0u);
    if (head && incl - 1 < (uint32_t)kGroupMax) {
      GroupL& G = g[incl - 1];
      G.hi = key.hi;
      G.glo = s1_group(key.lo);
      G.first = i;
      G.n_next = G.n_del = G.n_create = G.n_x = 0;
      G.fcs = 0xFFFFFFFFu;
      G.len = 0;
      G.flags = 0;
      G.slot = -1;
      G.n_succ = G.n_delok = G.fl = 0;
    }
    if (valid && i - start < (uint32_t)kStash) stash[i - start] = pack_s1(key.lo, succ);
    __syncthreads();
    if (valid && incl >= 1 && incl - 1 < (uint32_t)kGroupMax) {
      GroupL& G = g[incl - 1];
      const uint32_t cls = s1_class(key.lo), seq = s1_seq(key.lo);
      if (cls == 0) {
        atomicAdd(&G.n_next, 1u);
        if (s1_sub(key.lo)) atomicAdd(&G.n_del, 1u);
      } else if (cls == 1) {
        atomicAdd(&G.n_create, 1u);
        atomicMin(&G.fcs, seq);
        if (kM2 && succ) atomicAdd(&G.n_succ, 1u);
      } else {
        atomicAdd(&G.n_x, 1u);
        if (kM2 && succ) atomicAdd(&G.n_delok, 1u);
      }
    }
    __syncthreads();
    if (tid == 0) *s_ng = ng0 + tot;
    __syncthreads();
  }
  __syncthreads();
  uint32_t ng = *s_ng;
  return ng > (uint32_t)kGroupMax ? (uint32_t)kGroupMax + 1 : ng;
}

// Group of (hi, glo) among g[0, ng), or -1: a fixed-step lower bound (the same
// ten steps whatever ng is; g has kGroupMax + 1 entries).
__device__ inline int find_group(const GroupL* g, uint32_t ng, uint64_t hi, uint64_t glo) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t step = kGroupMax; step > 0; step >>= 1) {
    const uint32_t c = pos + step;
    const GroupL& G = g[min(c - 1, (uint32_t)kGroupMax)];
    const bool less = G.hi < hi || (G.hi == hi && G.glo < glo);
    pos = (c <= ng && less) ? c : pos;
  }
  const GroupL& G = g[min(pos, (uint32_t)kGroupMax)];
  return (pos < ng && G.hi == hi && G.glo == glo) ? (int)pos : -1;
}

// Sink descriptor g[ng] that follows the real groups: every per-group loop
// also visits it (with all of its ops masked off), so each loop body runs in
// every workgroup, empty partitions included.
__device__ inline void init_sink(GroupL* g, uint32_t ng, uint32_t start) {
  if (threadIdx.x == 0) {
    GroupL& G = g[ng];
    G.hi = ~0ull;
    G.glo = ~0ull;
    G.first = start;
    G.n_next = G.n_del = G.n_create = G.n_x = 1;
    G.fcs = 0xFFFFFFFFu;
    G.len = 0;
    G.flags = 0;
    G.slot = -1;
    G.n_succ = G.n_delok = G.fl = 0;
  }
}

// Phase B shared: map occupied mailbox rows of the partition to groups (and
// cache each row's occupied bit).  AUTH: side entries are decrypted here;
// they are authenticated with their row in phase C.
template <bool AUTH>
__device__ inline void side_prepass(const MArgs& a, uint32_t q, GroupL* g, uint32_t ng,
                                    int16_t* s_sg, uint8_t* s_occb, uint32_t* s_occ,
                                    const uint32_t* s_te) {
  for (uint32_t j = threadIdx.x; j < a.Sr; j += 256) {
    const uint64_t row = (uint64_t)q * a.Sr + j;
    uint4 sd = a.side[row];
    if (AUTH) sd = xor4(sd, side_keystream(a.sc, s_te, row, a.sc.epoch));
    uint64_t hi = u4lo(sd), w1 = u4hi(sd);
    const bool occ = (w1 & 1u) != 0;
    const int k = occ ? find_group(g, ng, hi, w1 >> 23) : -1;
    if (occ) atomicAdd(s_occ, 1u);
    if (k >= 0) {
      g[k].slot = (int32_t)j;
      g[k].len = (uint32_t)(w1 >> 1) & 63u;
    }
    s_sg[j] = (int16_t)k;
    s_occb[j] = occ ? 1 : 0;
  }
}

// AUTH, phase C: stage the side ciphertexts of rows j0 .. j0+kMU-1 and verify
// and decrypt the chunk's rows; a mismatch fails the batch for good.
template <int U>
__device__ inline void m_unseal_chunk(const MArgs& a, const uint32_t* s_te, uint32_t q,
                                      uint32_t j0, uint4 (&v)[U], uint4* st) {
  const uint32_t lane = lane_id();
  const uint64_t r0 = (uint64_t)q * a.Sr + j0;
  if (lane < (uint32_t)U) st[U * 4 * kSegU4 + lane] = a.side[r0 + lane];
  if (!wave_unseal<U>(a.sc, s_te, 1u, r0, v, a.btag, true, st) && lane == 0)
    atomicOr(&a.scal->error, 8u);
}

// Wave-cooperative write of up to 64 M1Out records (one per lane): each store
// instruction covers 8 whole 128-B records, so no record line is ever left
// partially written in L2 (partial lines make write-back traffic depend on
// eviction timing).  All 64 lanes must call.
__device__ inline void m1_write_wave(const MArgs& a, bool valid, uint32_t seq, uint32_t status,
                                     uint32_t slot, uint32_t flags, uint4 id) {
  const uint32_t lane = lane_id();
  uint4* base = reinterpret_cast<uint4*>(a.m1out);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int src = it * 8 + (int)(lane >> 3);
    const uint32_t chunk = lane & 7u;
    const uint32_t v = __shfl((uint32_t)valid, src), sq = __shfl(seq, src);
    const uint4 hdr = make_uint4(__shfl(status, src), __shfl(slot, src), __shfl(flags, src), 0u);
    const uint4 sid = shfl4(id, src);
    const uint4 d = chunk == 0 ? hdr : (chunk == 1 ? sid : make_uint4(0, 0, 0, 0));
    if (v) base[(uint64_t)sq * 8 + chunk] = d;
  }
}

// Resolve the next-message ops (class 0) of group G against its mailbox row v
// (lane 2+k holds id k): the op that has d delete-nexts before it reads id d.
// It has a single call site, which every workgroup also runs once in "dry"
// mode (one fake op writing the shared dummy record `dry_seq` = B), so the
// code executed does not depend on the request mix.
__device__ __forceinline__ void m1_resolve_next(const MArgs& a, const GroupL& G, uint4 v,
                                                const uint32_t* stash, uint32_t start,
                                                uint32_t dry_seq) {
  const uint32_t lane = lane_id();
  const bool dry = dry_seq != kNone;
  const uint32_t len = dry ? 62u : G.len;
  const uint32_t n_next = dry ? 1u : G.n_next;
  uint32_t carry = 0;
  for (uint32_t c = 0; c < n_next; c += 64) {
    const bool valid = c + lane < n_next;
    uint32_t p = 0;
    if (valid) p = op_info<false>(a, stash, start, (dry ? start : G.first) + c + lane);
    if (dry) p = dry_seq | (1u << 22);
    const uint32_t seq = pk_seq(p), sub = pk_sub(p);
    const uint64_t dm = __ballot(valid && sub);
    const uint32_t d = carry + mbcnt64(dm);
    carry += (uint32_t)__popcll(dm);
    const uint4 id = shfl4(v, 2 + (int)min(d, 61u));
    const bool found = d < len;
    const uint32_t slot = found ? id_decode(a.kc, u4lo(id), u4hi(id), a.N) : kNone;
    m1_write_wave(a, valid, seq, found ? kPending : 2u, slot, (found && sub) ? CF_POP : 0u,
                  found ? id : make_uint4(0, 0, 0, 0));
  }
}

// ops that touch no mailbox: the same per-op footprint as participants
// (one key read [+ status read, ROp read for M2] and the same writes)
template <bool kM2>
__device__ void dummy_partition(const MArgs& a, uint32_t b) {
  const uint32_t start = a.qstart[a.Q], end = a.qstart[a.Q + 1];
  const uint32_t nb = a.dummy_blocks;
  const uint32_t len = end - start, per = (len + nb - 1) / nb;
  const uint32_t lo = start + b * per, hi = min(end, lo + per);
  for (uint32_t base = lo; base < hi; base += 256) {
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < hi;
    uint32_t seq = 0;
    if (valid) seq = s1_seq(a.keys[i].lo);
    if (kM2) {
      if (valid) {
        const uint32_t st = a.rres[seq].status;
        const ROp r = a.rop[seq];
        asm volatile("" ::"v"(st), "v"(r.id[0]), "v"(r.x[0]));
      }
    } else {
      m1_write_wave(a, valid, seq, kPending, kNone, 0u, make_uint4(0, 0, 0, 0));
    }
  }
}

template <bool AUTH>
__global__ __launch_bounds__(256) void k_m1(MArgs a) {
  __shared__ GroupL g[kGroupMax + 1];
  __shared__ uint32_t stash[kStash];
  __shared__ Key128 s_key[256];
  __shared__ int16_t s_sg[kSrMax];
  __shared__ uint8_t s_occb[kSrMax];
  __shared__ uint32_t s_w[4], s_ng, s_occ, s_empt;
  GVS_TE_LDS s_te[AUTH ? kTeWords : 1];
  __shared__ uint4 s_st[AUTH ? 4 * stage_u4(kMU) : 1];
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar branches
  const uint32_t q = blockIdx.x;
  if (q >= a.Q) {
    dummy_partition<false>(a, q - a.Q);
    return;
  }
  if (AUTH) load_te(s_te, a.te);
  uint4* st = s_st + (AUTH ? wave * stage_u4(kMU) : 0u);
  // the wave's first chunk of rows is in flight during the group discovery
  const uint4* part = a.mbox + (uint64_t)q * a.Sr * 64;
  uint4 va[kMU], vb[kMU];
  load_rows(va, part, wave * kMU, a.Sr);
  const uint32_t start = a.qstart[q], end = a.qstart[q + 1];
  const uint32_t ng = discover_groups<false>(a, start, end, g, stash, s_key, s_w, &s_ng);
  if (ng > (uint32_t)kGroupMax) {
    if (tid == 0) atomicOr(&a.scal->error, 1u);
    return;
  }
  if (tid == 0) {
    s_occ = 0;
    s_empt = 0;
  }
  init_sink(g, ng, start);
  __syncthreads();
  side_prepass<AUTH>(a, q, g, ng, s_sg, s_occb, &s_occ, s_te);
  __syncthreads();

  // Phase C: stream every mailbox row of the partition (read-only pass).  Rows
  // owned by a group go one at a time (branch-free select) through the single
  // copy of m1_resolve_next; wave 0's first chunk also runs it once dry.  The
  // next chunk is loaded while the current one is worked on.
  for (uint32_t j0 = wave * kMU; j0 < a.Sr; j0 += 4 * kMU) {
    if (j0 + 4 * kMU < a.Sr) load_rows(vb, part, j0 + 4 * kMU, a.Sr);
    uint4 v[kMU];
    uint32_t mm = 0;
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      v[u] = va[u];
      keep4(v[u]);  // every row is read, used or not
      mm |= (j0 + u < a.Sr && s_sg[j0 + u] >= 0) ? (1u << u) : 0u;
    }
    if (AUTH) m_unseal_chunk<kMU>(a, s_te, q, j0, v, st);
    mm = __builtin_amdgcn_readfirstlane(mm);
    bool dry = j0 == 0;
    while (mm || dry) {
      const uint32_t bit = dry ? 1u : (mm & (0u - mm));
      if (!dry) mm &= mm - 1u;
      uint4 cur = v[0];
#pragma unroll
      for (int uu = 1; uu < kMU; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
      const int k = s_sg[j0 + (uint32_t)__builtin_ctz(bit)];
      m1_resolve_next(a, g[(!dry && k >= 0) ? (uint32_t)k : ng], cur, stash, start,
                      dry ? a.B : kNone);
      dry = false;
    }
#pragma unroll
    for (int u = 0; u < kMU; ++u) va[u] = vb[u];
  }
  __syncthreads();

  // Phase D: free rows after pops, admission of new recipients by the seq of
  // their first create (grapevine.proto:74 TOO_MANY_RECIPIENTS).  Loops run
  // over the sink g[ng] too (see init_sink).
  for (uint32_t k = tid; k <= ng; k += 256) {
    const GroupL& G = g[k];
    if (G.slot >= 0 && G.len == min(G.n_del, G.len)) atomicAdd(&s_empt, 1u);
  }
  __syncthreads();
  const uint32_t freeq = (a.Sr - s_occ) + s_empt;
  for (uint32_t k = tid; k <= ng; k += 256) {
    GroupL& G = g[k];
    const uint32_t len1 = G.slot >= 0 ? G.len - min(G.n_del, G.len) : 0u;
    const bool exists1 = len1 > 0;
    const bool isnew = !exists1 && G.n_create > 0;
    uint32_t rank = 0;
    if (isnew) {
      for (uint32_t k2 = 0; k2 <= ng; ++k2) {
        const GroupL& H = g[k2];
        const uint32_t hl = H.slot >= 0 ? H.len - min(H.n_del, H.len) : 0u;
        if (hl == 0 && H.n_create > 0 && H.fcs < G.fcs) ++rank;
      }
    }
    G.fl = len1;
    G.flags = (exists1 ? 1u : 0u) | ((isnew && rank < freeq) ? 2u : 0u);
  }
  __syncthreads();

  // Phase E: creates get their mailbox verdict; every remaining op is visited once.
  for (uint32_t k = wave; k <= ng; k += 4) {
    const GroupL& G = g[k];
    const bool real = k < ng;  // the sink's ops are all masked off
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (G.slot < 0) {
      for (uint32_t c = 0; c < G.n_next; c += 64) {
        const bool valid = real && c + lane < G.n_next;
        const uint32_t p = valid ? op_info<false>(a, stash, start, G.first + c + lane) : 0u;
        m1_write_wave(a, valid, pk_seq(p), 2u, kNone, 0u, z);
      }
    }
    const bool exists1 = G.flags & 1u, admitted = G.flags & 2u;
    for (uint32_t c = 0; c < G.n_create; c += 64) {
      const uint32_t r = c + lane;
      const bool valid = real && r < G.n_create;
      const uint32_t p = valid ? op_info<false>(a, stash, start, G.first + G.n_next + r) : 0u;
      const bool ok = exists1 ? (G.fl + r < GVS_MAILBOX_SLOTS) : (admitted && r < GVS_MAILBOX_SLOTS);
      const uint32_t st = ok ? kPending : ((exists1 || admitted) ? 5u : 6u);
      m1_write_wave(a, valid, pk_seq(p), st, kNone, ok ? CF_MBOX_OK : 0u, z);
    }
    for (uint32_t c = 0; c < G.n_x; c += 64) {
      const bool valid = real && c + lane < G.n_x;
      const uint32_t p =
          valid ? op_info<false>(a, stash, start, G.first + G.n_next + G.n_create + c + lane) : 0u;
      m1_write_wave(a, valid, pk_seq(p), kPending, kNone, 0u, z);
    }
  }
}

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
  uint32_t* pcount;  // W+1 partition counters
  Scal* scal;
  uint32_t B, nblk, W, S;
  uint64_t N, ring_size;
  KeyCtx kc;
};

constexpr uint32_t kWinGroup = 8;      // blocks per allocation-window refill
constexpr uint32_t kWinRing = 16384;  // LDS window ring: one group + one chunk fits

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
#pragma unroll
    for (uint32_t u = 0; u < kWinGroup; ++u) {
      const uint32_t c = c0 + u, i = c * 1024 + tid;
      if (c < a.nblk) {
        const bool pop = f[u] & 1u;
        const uint32_t P = (c ? s_off[0][c - 1] : 0u) + ((f[u] >> 2) & 1023u);
        const uint64_t pos = pop ? (uint64_t)P : (uint64_t)pops + (i - P);
        a.ring[(tail0 + pos) % a.ring_size] = pop ? slot[u] : kNone;
      }
    }
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
      w[k] = pos < need ? a.ring[(head0 + pos + tid) % a.ring_size] : 0u;
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
      v[k] = pos < a.B ? a.ring[(head0 + pos + tid) % a.ring_size] : 0u;
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
__global__ __launch_bounds__(1024) void k_alloc_b(AllocArgs a) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_hist[kBinsMax];
  const uint32_t tid = threadIdx.x;
  if (a.scal->error) return;
  for (uint32_t b = tid; b <= a.W; b += 1024) s_hist[b] = 0;
  // S_i: block offset + in-block prefix of mailbox-ok creates
  uint32_t boff = 0;
  for (uint32_t b = 0; b < blockIdx.x; ++b) boff += a.bsum[2 * b + 1];
  const uint32_t i = blockIdx.x * 1024 + tid;
  const uint32_t f = a.pflag[i];
  uint32_t tot;
  const uint32_t S_i = boff + block1024_prefix((f & 2u) != 0u, s_w, &tot);
  const uint32_t kind = a.kinds[i];
  const OpState os = a.ops[i];
  const M1Out m1 = a.m1out[i];
  const uint32_t cs = a.cslot[i];
  const Scal* sc = a.scal;
  const uint64_t count1 = sc->count1, ctr0 = sc->ctr;

  ROp r = {};
  r.kind = kind;
  r.status = os.pre_status;
  r.slot = kNone;
  r.id[0] = os.id[0]; r.id[1] = os.id[1]; r.id[2] = os.id[2]; r.id[3] = os.id[3];
  for (int k = 0; k < 8; ++k) r.x[k] = os.x[k];
  uint32_t cls = 3;
  uint64_t L, R;
  id_encode(a.kc, cs == kNone ? 0u : cs, ctr0 + S_i, L, R);  // fixed work for every op
  if (kind == KIND_CREATE && os.pre_status == kPending) {
    if (count1 + S_i >= a.N) r.status = 7;  // TOO_MANY_MESSAGES (checked before 5/6)
    else if (cs == kNone) r.status = m1.status;  // 5 or 6 from the mailbox pass
    else {
      r.slot = cs;
      r.status = kPending;
      r.id[0] = (uint32_t)L; r.id[1] = (uint32_t)(L >> 32);
      r.id[2] = (uint32_t)R; r.id[3] = (uint32_t)(R >> 32);
      cls = 1;
    }
  } else if (kind == KIND_NEXT_READ || kind == KIND_NEXT_DEL) {
    r.status = m1.status;
    if (m1.status == kPending) {
      r.slot = m1.slot;
      r.id[0] = m1.id[0]; r.id[1] = m1.id[1]; r.id[2] = m1.id[2]; r.id[3] = m1.id[3];
      cls = 0;
    }
  } else if (kind == KIND_READ || kind == KIND_UPDATE || kind == KIND_DELETE) {
    r.slot = os.slot;
    if (os.slot != kNone) cls = 2;
  }
  a.rop[i] = r;
  uint64_t rowp = kRNullRow;
  uint32_t part = a.W;
  if (cls < 3) {
    const uint32_t sl = r.slot;
    part = sl % a.W;
    rowp = (uint64_t)part * a.S + sl / a.W;
  } else {
    cls = 0;
  }
  a.rkeys[i] = r_key(rowp, cls, i);
  atomicAdd(&s_hist[part], 1u);
  hist_flush(s_hist, a.W + 1, a.pcount);
}

// ---------------------------------------------------------------- R pass

struct RArgs {
  uint4* table;             // N rows x 64 uint4, partition-major
  const uint64_t* rkeys;    // sorted
  const uint32_t* pstart;   // W+2
  const ROp* rop;
  const uint4* img;
  uint4* resp;              // B internal slots of kRespSlot bytes
  RRes* rres;
  Scal* scal;
  uint32_t n, B, W, S, null_blocks;
  SealCtx sc;               // authenticated storage (AUTH instantiations)
  const uint32_t* te;       // AES table (256 words)
  uint4* mtag;              // N row tags
  // expiry sweep: ops with seq >= xbase are expiry deletes
  // (succeed only if the row's timestamp < cutoff); with xon, workgroups
  // w = xrot (mod xk) record their partition's first xep expired rows after
  // the batch's ops into xbuf[(w / xk) * xep ..], one 128-B record each
  uint32_t xbase, xon, xk, xrot, xep;
  uint64_t cutoff;
  uint4* xbuf;
};

constexpr uint32_t kXepMax = 8;  // expiry records per workgroup (one store instruction)

__device__ inline void write_response(const RArgs& a, uint32_t seq, uint4 rec, uint32_t status) {
  const uint32_t lane = lane_id();
  uint4* dst = a.resp + (uint64_t)seq * (kRespSlot / 16);
  dst[lane] = rec;
  if (lane < 8) {
    const uint4 t = make_uint4(lane == 0 ? status : 0u, 0, 0, 0);
    dst[64 + lane] = t;                                        // status line of the slot
    reinterpret_cast<uint4*>(a.rres)[(uint64_t)seq * 8 + lane] = t;  // whole RRes line
  }
}

// failure record: all zero but the request's server timestamp (lane 5 low 8 B)
__device__ inline uint4 fail_record(uint4 q, uint32_t status) {
  const uint32_t lane = lane_id();
  const uint4 ts = shfl4(q, 5);
  uint4 r = make_uint4(0, 0, 0, 0);
  if (lane == 5 && status != 0u) {
    r.x = ts.x;
    r.y = ts.y;
  }
  return r;
}

// packed R-pass op: row offset in partition << 20 | seq
__device__ inline uint32_t r_op_at(const RArgs& a, const uint32_t* stash, uint32_t start,
                                   uint32_t k, uint64_t rowbase) {
  if (k < (uint32_t)kStash) return stash[k];
  const uint64_t key = a.rkeys[start + k];
  return ((uint32_t)((key >> 22) - rowbase) << 20) | ((uint32_t)key & kSeqMask);
}

// Apply the ops routed to one row, in (class, seq) order, to the row held in v
// (16 B per lane).  Branch-free over op kinds (lane-wise selects), so every op
// runs the same instructions.  With `dry` set, a first fake op (the shared
// dummy record `dry_seq` = B) runs on a zero row whose result is discarded:
// wave 0 of every workgroup runs each inlined copy of this code once, so the
// instruction fetch does not depend on the request mix.
__device__ inline void r_apply(const RArgs& a, uint4& v, const uint32_t* stash, uint32_t start,
                               uint64_t rowbase, uint32_t first, uint32_t cnt, bool dry,
                               uint32_t dry_seq) {
  const uint32_t lane = lane_id();
  const uint32_t n = cnt + (dry ? 1u : 0u);
  for (uint32_t k = 0; k < n; ++k) {
    const bool isdry = dry && k == 0;
    const uint32_t kidx = isdry ? 0u : first + k - (dry ? 1u : 0u);  // dry: stash[0], in LDS
    const uint32_t pk = r_op_at(a, stash, start, kidx, rowbase);
    const uint32_t seq = isdry ? dry_seq : (pk & kSeqMask);
    const ROp r = a.rop[seq];
    const uint4 q = a.img[(uint64_t)seq * 64 + lane];
    const uint32_t kind = __builtin_amdgcn_readfirstlane(r.kind);
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint4 cur = isdry ? z : v;
    const uint4 vr = shfl4(cur, (int)lane + 2);  // lanes 1,2 see the row's recipient
    const uint64_t m_eq = __ballot(eq4(q, cur));
    const uint64_t m_eqr = __ballot(eq4(q, vr));
    const bool exists = (__ballot(nz4(cur)) & 1ull) != 0;
    const uint4 rid = make_uint4(r.id[0], r.id[1], r.id[2], r.id[3]);
    const bool rid_match = (__ballot(lane == 0 && eq4(cur, rid)) & 1ull) != 0;
    const bool id_match = (m_eq & 1ull) != 0;
    const bool auth_ok = ((m_eq & 6ull) == 6ull) || ((m_eqr & 6ull) == 6ull);
    const bool rcpt_ok = (m_eq & 0x18ull) == 0x18ull;
    const bool is_next = kind == KIND_NEXT_READ || kind == KIND_NEXT_DEL;
    const bool is_create = kind == KIND_CREATE;
    // next ops were resolved by M1 (mismatch = internal error); the allocator
    // only hands out free rows to creates; by-id ops check existence, auth
    // (grapevine.proto:84,97,107) and then the recipient (:99-101,:110-112)
    const uint32_t st_next = (exists && rid_match) ? 1u : 8u;
    const uint32_t st_create = exists ? 8u : 1u;
    // expiry deletes (seq >= xbase) also need the row's timestamp (lane 5,
    // low 8 B) below the cutoff: a row updated since its sweep is kept
    const uint64_t row_ts = ((uint64_t)__shfl(cur.y, 5) << 32) | __shfl(cur.x, 5);
    const bool fresh = seq >= a.xbase && !(row_ts < a.cutoff);
    const bool found = exists && id_match && auth_ok && !fresh;
    const uint32_t st_byid = !found ? 2u : ((kind != KIND_READ && !rcpt_ok) ? 4u : 1u);
    const uint32_t status = is_next ? st_next : (is_create ? st_create : st_byid);
    const bool ok = status == 1u;
    const bool del = ok && (kind == KIND_NEXT_DEL || kind == KIND_DELETE);
    const bool cre = ok && is_create;
    const bool upd = ok && kind == KIND_UPDATE;
    const uint4 v_create = lane == 0 ? rid : q;  // sender = auth, recipient, ts, payload
    const uint4 v_upd = lane >= 5 ? q : cur;     // timestamp (lane 5 low half) + payload
    const uint4 nv = del ? z : (cre ? v_create : (upd ? v_upd : cur));
    const uint4 resp = ok ? ((cre || upd) ? nv : cur) : fail_record(q, status);
    write_response(a, seq, resp, status);
    if (!isdry) v = nv;
  }
}

// Expiry sweep, per chunk of U rows after their ops: rows that hold a message
// (nonzero id, lane 0) with timestamp (lane 5) < cutoff are appended, in row
// order, to the wave's LDS list (id, recipient lo, recipient hi); entries past
// xep go to a spare slot.  Branch-free and on-die only.  Returns the count.
template <int U>
__device__ inline uint32_t x_detect(const RArgs& a, const uint4 (&v)[U], uint4* buf, uint32_t xc) {
  const uint32_t lane = lane_id();
  const uint32_t part = lane == 0 ? 0u : lane - 2u;  // lanes 0, 3, 4 -> list words 0, 1, 2
  const bool writer = lane == 0 || lane == 3 || lane == 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t ts = ((uint64_t)v[u].y << 32) | v[u].x;
    const uint64_t m_old = __ballot(lane == 5 && ts < a.cutoff);
    const uint64_t m_msg = __ballot(lane == 0 && nz4(v[u]));
    const uint32_t hit = (uint32_t)((m_old >> 5) & m_msg & 1ull);
    const uint32_t slot = min(xc, a.xep);
    if (writer) buf[slot * 3 + part] = v[u];
    xc += hit;
  }
  return xc;
}

// After a tile: append the waves' lists (wave order = row order) to the
// partition's list s_xp of up to xep entries; s_xt is its length.  Threads
// < 3 xep each fill one word with selects; the caller syncs, then thread 0
// stores the returned length.
__device__ inline uint32_t x_merge(const RArgs& a, const uint4* s_xw, const uint32_t* s_xc,
                                   uint4* s_xp, uint32_t tot) {
  const uint32_t tid = threadIdx.x, cap = a.xep;
  uint32_t add = 0;
  if (tid < 3 * cap) {
    const uint32_t k = tid / 3, c = tid % 3;
    uint32_t off = k - tot, src = kNone;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t cw = min(s_xc[w], cap);
      const bool take = k >= tot && src == kNone && off < cw;
      src = selu32(take, ((uint32_t)w * (kXepMax + 1) + off) * 3 + c, src);
      off -= cw;
    }
    if (src != kNone) s_xp[k * 3 + c] = s_xw[src];
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) add += min(s_xc[w], cap);
  return min(tot + add, cap);
}

template <int U, bool NTL, bool NTS, int MINW, bool AUTH = false>
__global__ __launch_bounds__(256, MINW) void k_rpass(RArgs a) {
  __shared__ uint32_t stash[kStash];
  __shared__ uint32_t s_first[kTile], s_cnt[kTile];
  __shared__ uint32_t s_tile[kRowsMax / kTile + 1];
  GVS_TE_LDS s_te[AUTH ? kTeWords : 1];
  __shared__ uint4 s_st[AUTH ? 4 * stage_u4(U) : 1];
  __shared__ uint4 s_xw[4 * (kXepMax + 1) * 3];  // expiry: per-wave lists of a tile
  __shared__ uint4 s_xp[kXepMax * 3];            //         the partition's list
  __shared__ uint32_t s_xc[4], s_xt;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t w = blockIdx.x;
  if (a.scal->error) return;
  if (w >= a.W) {
    // ops that touch no row: same footprint (key, ROp, image, response, result)
    const uint32_t start = a.pstart[a.W], end = a.pstart[a.W + 1];
    const uint32_t nb = a.null_blocks, b = w - a.W;
    const uint32_t len = end - start, per = (len + nb - 1) / nb;
    const uint32_t lo = start + b * per, hi = min(end, lo + per);
    // wave 0 first runs a fake op on the shared dummy record: fixed code path
    const uint32_t i0 = wave == 0 ? lo - 4 : lo + wave;
    for (uint32_t i = i0; i < hi || (wave == 0 && i == i0); i += 4) {
      const bool isdry = wave == 0 && i == i0;
      const uint32_t seq = isdry ? a.B : ((uint32_t)a.rkeys[i] & kSeqMask);
      const ROp r = a.rop[seq];
      const uint32_t st = __builtin_amdgcn_readfirstlane(r.status);
      asm volatile("" ::"v"(r.id[0]), "v"(r.kind));
      const uint4 q = a.img[(uint64_t)seq * 64 + lane];
      write_response(a, seq, fail_record(q, st), st);
    }
    return;
  }
  const uint32_t start = a.pstart[w], end = a.pstart[w + 1];
  const uint32_t cnt = end - start;
  const uint64_t rowbase = (uint64_t)w * a.S;
  if (AUTH) load_te(s_te, a.te);
  uint4* st = s_st + (AUTH ? wave * stage_u4(U) : 0u);
  // stash this partition's ops (each key read once): row offset << 20 | seq
  for (uint32_t k = tid; k < cnt && k < (uint32_t)kStash; k += 256) {
    const uint64_t key = a.rkeys[start + k];
    stash[k] = ((uint32_t)((key >> 22) - rowbase) << 20) | ((uint32_t)key & kSeqMask);
  }
  __syncthreads();
  const uint32_t tiles = a.S / kTile;
  // first op of each tile: lower bound over the sorted stash
  for (uint32_t t = tid; t <= tiles; t += 256) {
    uint32_t lo = 0, hi = cnt;
    const uint32_t target = t * kTile;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((r_op_at(a, stash, start, mid, rowbase) >> 20) < target) lo = mid + 1;
      else hi = mid;
    }
    s_tile[t] = lo;
  }
  __syncthreads();
  uint4* part = a.table + rowbase * 64;
  for (uint32_t t = 0; t < tiles; ++t) {
    const uint32_t lo = s_tile[t], hi = s_tile[t + 1];
    s_cnt[tid] = 0;
    s_first[tid] = 0xFFFFFFFFu;
    if (t == 0 && tid == 0) s_xt = 0;
    __syncthreads();
    uint32_t xc = 0;  // expiry: this wave's hits in this tile
    for (uint32_t k = lo + tid; k < hi; k += 256) {
      const uint32_t o = (r_op_at(a, stash, start, k, rowbase) >> 20) - t * kTile;
      atomicAdd(&s_cnt[o], 1u);
      atomicMin(&s_first[o], k);
    }
    __syncthreads();
    const uint32_t rb = t * kTile + wave * 64;
    // AUTH: the header PRF of the wave's 64 rows at both epochs, one row per
    // lane (it depends on no row data); each chunk takes its rows' by shuffle
    uint64_t hv[2] = {0, 0}, hs[2] = {0, 0};
    if (AUTH) {
      const uint64_t z[2] = {0, 0};
      header_prf(a.sc.headk, rowbase + rb + lane, a.sc.epoch, 0u, z, hv);
      header_prf(a.sc.headk, rowbase + rb + lane, a.sc.epoch + 1u, 0u, z, hs);
    }
    for (uint32_t j = 0; j < 64; j += U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld_row<NTL>(&part[(uint64_t)(rb + j + u) * 64 + lane]);
      const uint64_t r0 = rowbase + rb + j;  // physical row of v[0]
      const uint32_t hsrc = j + ((lane >> 2) & (uint32_t)(U - 1));  // lane holding the header
      if (AUTH) {
        const uint64_t hvr[2] = {shfl_u64(hv[0], (int)hsrc), shfl_u64(hv[1], (int)hsrc)};
        if (!wave_unseal<U>(a.sc, s_te, 0u, r0, v, a.mtag, false, st, hvr) && lane == 0)
          atomicOr(&a.scal->error, 8u);  // integrity failure: the batch and the handle are dead
      }
      // rows of this chunk that have ops (wave-uniform); wave 0's first chunk
      // also runs the dry op, so the single copy of the apply code below is
      // executed by every workgroup whatever the batch holds (see r_apply)
      const bool dry = (t == 0 && j == 0 && wave == 0);
      uint32_t mm = dry ? 1u : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) mm |= s_cnt[wave * 64 + j + u] ? (1u << u) : 0u;
      mm = __builtin_amdgcn_readfirstlane(mm);
      bool first_dry = dry;
      while (mm) {
        const uint32_t u = (uint32_t)__builtin_ctz(mm);
        const uint32_t bit = mm & (0u - mm);
        mm &= mm - 1u;
        // branch-free select of row u (keeps v[] in registers)
        uint4 cur = v[0];
#pragma unroll
        for (int uu = 1; uu < U; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
        const uint32_t o = wave * 64 + j + u;
        r_apply(a, cur, stash, start, rowbase, s_first[o], s_cnt[o], first_dry, a.B);
        first_dry = false;
#pragma unroll
        for (int uu = 0; uu < U; ++uu) v[uu] = sel4((bit >> uu) & 1u, cur, v[uu]);
      }
      if (a.xon) xc = x_detect<U>(a, v, s_xw + wave * (kXepMax + 1) * 3, xc);
      if (AUTH) {
        const uint64_t hsr[2] = {shfl_u64(hs[0], (int)hsrc), shfl_u64(hs[1], (int)hsrc)};
        wave_seal<U>(a.sc, s_te, 0u, r0, a.sc.epoch + 1u, v, a.mtag, false, st, hsr);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st_row<NTS>(&part[(uint64_t)(rb + j + u) * 64 + lane], v[u]);
    }
    if (lane == 0) s_xc[wave] = xc;
    __syncthreads();
    if (a.xon) {
      const uint32_t tot = x_merge(a, s_xw, s_xc, s_xp, s_xt);
      __syncthreads();
      if (tid == 0) s_xt = tot;
    }
  }
  if (a.xon && w % a.xk == a.xrot) {
    // the partition's expiry records: 8 lanes per 128-B record (id, recipient,
    // valid word, zeros), all written by one store instruction of wave 0
    __syncthreads();
    if (wave == 0 && lane < 8 * a.xep) {
      const uint32_t k = lane >> 3, part8 = lane & 7;
      const bool valid = k < s_xt;
      uint4 val = make_uint4(part8 == 3 && valid ? 1u : 0u, 0, 0, 0);
      if (part8 < 3) val = valid ? s_xp[k * 3 + part8] : make_uint4(0, 0, 0, 0);
      a.xbuf[((uint64_t)(w / a.xk) * a.xep + k) * 8 + part8] = val;
    }
  }
}

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

// one workgroup: by-id deletes -> free ring in seq order; commit scalars
__global__ __launch_bounds__(1024) void k_post_ring(PostArgs a) {
  __shared__ uint32_t s_off[1024];
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
  const uint64_t tail = sc->tail0 + sc->pops;
  for (uint32_t c0 = 0; c0 < a.nblk; c0 += 8) {  // no barrier: blocks are independent
    uint32_t f[8], slot[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      const uint32_t i = (c0 + u) * 1024 + tid;
      f[u] = c0 + u < a.nblk ? a.dflag[i] : 0u;
      slot[u] = c0 + u < a.nblk ? a.dslot[i] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      const uint32_t c = c0 + u, i = c * 1024 + tid;
      if (c < a.nblk) {
        const bool d = f[u] & 1u;
        const uint32_t P = (c ? s_off[c - 1] : 0u) + (f[u] >> 1);
        const uint64_t pos = d ? (uint64_t)P : (uint64_t)nd + (i - P);
        a.ring[(tail + pos) % a.ring_size] = d ? slot[u] : kNone;
      }
    }
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

// ----------------------------------------------------------------- M2 pass

// Build the new state of one mailbox row: pop D' ids, append the ids of the
// successful creates (a prefix of the class-1 members), remove ids of
// successful by-id deletes, clear the row if it ends empty.  Each member's
// ROp is read exactly once here.
// With `dry` (G = the sink), one fake member of each class reads the shared
// dummy record B instead and the caller discards v: every workgroup runs the
// single copy of this code once whatever the batch holds.
__device__ __forceinline__ void m2_apply(const MArgs& a, const GroupL& G, uint4& v, bool matched,
                                         const uint32_t* stash, uint32_t start, bool dry) {
  const uint32_t lane = lane_id();
  const uint32_t len = matched ? G.len : 0u;
  const uint32_t dp = min(G.n_del, len);
  for (uint32_t c = 0; c < G.n_next; c += 64) {  // visit pops (state needs only the count)
    if (c + lane < G.n_next) {
      const uint32_t p = dry ? a.B : op_info<true>(a, stash, start, G.first + c + lane);
      const ROp r = a.rop[pk_seq(p)];
      asm volatile("" ::"v"(r.id[0]), "v"(r.x[0]));
    }
  }
  if (dp) {
    const uint32_t src = lane + dp;
    const uint4 s = shfl4(v, (int)min(src, 63u));
    if (lane >= 2) v = src < 64 ? s : make_uint4(0, 0, 0, 0);
  }
  uint32_t cur = len - dp;
  for (uint32_t c = 0; c < G.n_create; c += 64) {
    const bool valid = c + lane < G.n_create;
    ROp r = {};
    uint32_t p = 0;
    if (valid) {
      p = dry ? a.B : op_info<true>(a, stash, start, G.first + G.n_next + c + lane);
      r = a.rop[pk_seq(p)];
    }
    const uint64_t ms = __ballot(valid && pk_succ(p));
    const uint32_t ns = (uint32_t)__popcll(ms);
    if (!matched && c == 0) {
      const uint4 x0 = shfl4(make_uint4(r.x[0], r.x[1], r.x[2], r.x[3]), 0);
      const uint4 x1 = shfl4(make_uint4(r.x[4], r.x[5], r.x[6], r.x[7]), 0);
      if (lane == 0) v = x0;
      if (lane == 1) v = x1;
    }
    const int rel = (int)lane - 2 - (int)cur;
    const uint4 nid = shfl4(make_uint4(r.id[0], r.id[1], r.id[2], r.id[3]),
                            rel < 0 ? 0 : (rel > 63 ? 63 : rel));
    if (lane >= 2 && rel >= 0 && rel < (int)ns) v = nid;
    cur += ns;
  }
  for (uint32_t c = 0; c < G.n_x; c += 64) {
    const bool valid = c + lane < G.n_x;
    ROp r = {};
    uint32_t p = 0;
    if (valid) {
      p = dry ? a.B : op_info<true>(a, stash, start, G.first + G.n_next + G.n_create + c + lane);
      r = a.rop[pk_seq(p)];
    }
    uint64_t md = __ballot(valid && pk_succ(p));
    const uint4 myid = make_uint4(r.id[0], r.id[1], r.id[2], r.id[3]);
    while (md) {
      const int b = __builtin_ctzll(md);
      md &= md - 1;
      const uint4 did = shfl4(myid, b);
      const uint64_t hit = __ballot(lane >= 2 && eq4(v, did));
      if (hit) {
        const uint32_t pos = (uint32_t)__builtin_ctzll(hit);
        const uint4 nxt = shfl4(v, (int)min(lane + 1, 63u));
        if (lane >= pos) v = lane < 63 ? nxt : make_uint4(0, 0, 0, 0);
        cur -= 1;
      }
    }
  }
  if (cur == 0) v = make_uint4(0, 0, 0, 0);
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

template <bool AUTH>
__global__ __launch_bounds__(256) void k_m2(MArgs a) {
  __shared__ GroupL g[kGroupMax + 1];
  __shared__ uint32_t stash[kStash];
  __shared__ Key128 s_key[256];
  __shared__ int16_t s_sg[kSrMax];
  __shared__ uint8_t s_occb[kSrMax];
  GVS_TE_LDS s_te[AUTH ? kTeWords : 1];
  __shared__ uint4 s_st[AUTH ? 4 * stage_u4(kMU) : 1];
  __shared__ int16_t s_place[kSrMax];
  __shared__ uint8_t s_flag[kSrMax];
  __shared__ uint16_t s_pfx[kSrMax + 1];
  __shared__ uint16_t s_gpfx[kGroupMax + 1];
  __shared__ uint8_t s_gflag[kGroupMax + 1];
  __shared__ int16_t s_pend[kGroupMax];
  __shared__ uint32_t s_w[4], s_ng, s_occ, s_delta;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar branches
  const uint32_t q = blockIdx.x;
  if (a.scal->error) return;
  if (q >= a.Q) {
    dummy_partition<true>(a, q - a.Q);
    return;
  }
  if (AUTH) load_te(s_te, a.te);
  uint4* st = s_st + (AUTH ? wave * stage_u4(kMU) : 0u);
  // the wave's first chunk of rows is in flight during the group discovery
  uint4* part = a.mbox + (uint64_t)q * a.Sr * 64;
  uint4* side = a.side + (uint64_t)q * a.Sr;
  uint4 va[kMU], vb[kMU];
  load_rows(va, part, wave * kMU, a.Sr);
  const uint32_t start = a.qstart[q], end = a.qstart[q + 1];
  const uint32_t ng = discover_groups<true>(a, start, end, g, stash, s_key, s_w, &s_ng);
  if (ng > (uint32_t)kGroupMax) return;  // M1 already flagged the batch
  if (tid == 0) {
    s_occ = 0;
    s_delta = 0;
  }
  init_sink(g, ng, start);
  __syncthreads();
  side_prepass<AUTH>(a, q, g, ng, s_sg, s_occb, &s_occ, s_te);
  __syncthreads();
  // final lengths; pending = groups with no row that end non-empty (the sink
  // g[ng] gets fl = 0, flag 0)
  for (uint32_t k = tid; k <= ng; k += 256) {
    GroupL& G = g[k];
    const uint32_t len = G.slot >= 0 ? G.len : 0u;
    const uint32_t dp = min(G.n_del, len);
    G.fl = len - dp + G.n_succ - G.n_delok;
    s_gflag[k] = (G.slot < 0 && G.fl > 0) ? 1 : 0;
  }
  __syncthreads();
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int k = s_sg[j];
    const bool occ = s_occb[j] != 0;
    s_flag[j] = (!occ || (k >= 0 && g[k].fl == 0)) ? 1 : 0;
  }
  __syncthreads();
  block_flag_scan(s_flag, a.Sr, s_pfx, s_w);
  block_flag_scan(s_gflag, ng, s_gpfx, s_w);
  for (uint32_t k = tid; k <= ng; k += 256)
    if (k < ng && s_gflag[k]) s_pend[s_gpfx[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t npend = s_gpfx[ng];
  if (tid == 0 && npend > s_pfx[a.Sr]) atomicOr(&a.scal->error, 2u);
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    int16_t p = -1;
    if (s_flag[j] && s_pfx[j] < npend) p = s_pend[s_pfx[j]];
    s_place[j] = p;
    const int k = s_sg[j];
    if (k >= 0 && g[k].fl == 0) atomicSub(&s_delta, 1u);
  }
  if (tid == 0) atomicAdd(&s_delta, npend);
  __syncthreads();

  // Phase C: rewrite every row of the partition exactly once.  Rows with work
  // go one at a time (branch-free select) through the single copy of
  // m2_apply; wave 0's first chunk also runs it once dry on the sink.  The
  // next chunk is loaded while the current one is worked on.
  for (uint32_t j0 = wave * kMU; j0 < a.Sr; j0 += 4 * kMU) {
    if (j0 + 4 * kMU < a.Sr) load_rows(vb, part, j0 + 4 * kMU, a.Sr);
    uint4 v[kMU], sd[kMU];
    uint32_t mm = 0;
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      const bool in = j0 + u < a.Sr;  // wave-uniform
      v[u] = va[u];
      sd[u] = in ? side[j0 + u] : make_uint4(0, 0, 0, 0);
      mm |= (in && (s_sg[j0 + u] >= 0 || s_place[j0 + u] >= 0)) ? (1u << u) : 0u;
    }
    if (AUTH) {
      // verify + decrypt the rows (side ciphertexts staged), then the side
      // entries: lane u < kMU decrypts row u's and every lane takes them all
      m_unseal_chunk<kMU>(a, s_te, q, j0, v, st);
      const uint64_t r0 = (uint64_t)q * a.Sr + j0;
      uint4 mine = make_uint4(0, 0, 0, 0);
      if (lane < (uint32_t)kMU)
        mine = xor4(st[kMU * 4 * kSegU4 + lane], side_keystream(a.sc, s_te, r0 + lane, a.sc.epoch));
#pragma unroll
      for (int u = 0; u < kMU; ++u) sd[u] = shfl4(mine, u);
    }
    mm = __builtin_amdgcn_readfirstlane(mm);
    bool dry = j0 == 0;
    while (mm || dry) {
      const uint32_t bit = dry ? 1u : (mm & (0u - mm));
      if (!dry) mm &= mm - 1u;
      uint4 cur = v[0];
#pragma unroll
      for (int uu = 1; uu < kMU; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
      const uint32_t j = j0 + (uint32_t)__builtin_ctz(bit);
      const int k = dry ? -1 : s_sg[j], p = dry ? -1 : s_place[j];
      // pass 0: the row's own group; pass 1: a new mailbox placed in the row
      // (one that is, or became, empty)
#pragma unroll 1
      for (uint32_t pass = 0; pass < 2; ++pass) {
        const int gi = pass == 0 ? k : p;
        if (gi < 0 && !(dry && pass == 0)) continue;
        if (pass == 1) cur = make_uint4(0, 0, 0, 0);
        m2_apply(a, g[gi >= 0 ? (uint32_t)gi : ng], cur, pass == 0 && !dry, stash, start, dry);
      }
      const GroupL& G = g[p >= 0 ? (uint32_t)p : (k >= 0 ? (uint32_t)k : ng)];
      const uint64_t w1 = (G.glo << 23) | ((uint64_t)G.fl << 1) | 1ull;
      const uint4 nsd = G.fl > 0 ? make_uint4((uint32_t)G.hi, (uint32_t)(G.hi >> 32), (uint32_t)w1,
                                              (uint32_t)(w1 >> 32))
                                 : make_uint4(0, 0, 0, 0);
      if (!dry) {
#pragma unroll
        for (int uu = 0; uu < kMU; ++uu) {
          v[uu] = sel4((bit >> uu) & 1u, cur, v[uu]);
          sd[uu] = sel4((bit >> uu) & 1u, nsd, sd[uu]);
        }
      }
      dry = false;
    }
    if (AUTH) {
      // new side entries: lane u < kMU encrypts row u's at epoch + 1 and
      // stages it for the tag; then the rows are sealed at epoch + 1
      const uint64_t r0 = (uint64_t)q * a.Sr + j0;
      const uint32_t ep = a.sc.epoch + 1u;
      uint4 mine = sd[0];
#pragma unroll
      for (int u = 1; u < kMU; ++u) mine = sel4(lane == (uint32_t)u, sd[u], mine);
      if (lane < (uint32_t)kMU) {
        const uint4 ct = xor4(mine, side_keystream(a.sc, s_te, r0 + lane, ep));
        st[kMU * 4 * kSegU4 + lane] = ct;
        side[j0 + lane] = ct;
      }
      wave_seal<kMU>(a.sc, s_te, 1u, r0, ep, v, a.btag, true, st);
    }
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      if (j0 + u < a.Sr) {
        st_row<true>(&part[(uint64_t)(j0 + u) * 64 + lane], v[u]);
        if (!AUTH && lane == 0) side[j0 + u] = sd[u];
      }
      va[u] = vb[u];
    }
  }
  // Phase D: members of groups that own no row (misses, failed creates) are
  // visited too; the sink's three fake members read the dummy record B.
  for (uint32_t k = wave; k <= ng; k += 4) {
    const GroupL& G = g[k];
    const bool real = k < ng;
    if (real && (G.slot >= 0 || s_gflag[k])) continue;
    const uint32_t cnt = G.n_next + G.n_create + G.n_x;
    for (uint32_t c = lane; c < cnt; c += 64) {
      const uint32_t p = real ? op_info<true>(a, stash, start, G.first + c) : a.B;
      const ROp r = a.rop[pk_seq(p)];
      asm volatile("" ::"v"(r.id[0]), "v"(r.x[0]));
    }
  }
  if (tid == 0 && s_delta) atomicAdd((unsigned long long*)&a.scal->n_mailboxes,
                                     (unsigned long long)(int64_t)(int32_t)s_delta);
}

// ------------------------------------------------------------------ k_out

// internal response slots (kRespSlot B, whole lines) -> caller layout (1040 B)
__global__ __launch_bounds__(256) void k_out(const uint4* __restrict__ resp, uint32_t n,
                                             uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t lane = lane_id();
  if (i >= n) return;
  const uint4* src = resp + (uint64_t)i * (kRespSlot / 16);
  out[(uint64_t)i * 65 + lane] = src[lane];
  if (lane == 0) out[(uint64_t)i * 65 + 64] = src[64];
}

}  // namespace gvs
