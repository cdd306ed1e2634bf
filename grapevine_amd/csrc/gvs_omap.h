// gvs_omap.h — the key-value map (gvs_omap_*): mc-oblivious-traits
// ObliviousHashMap<16, 1024> (access_and_insert / read / remove), batched
// (DESIGN.md §10).
//
// Rows of the value table are found by key in a key directory K (per row: the
// 16-B key, zero when free, and its 128-bit keyed hash).  A key lives in the
// partition q = the top log2(W) bits of its hash; a partition's S rows hold at
// most S keys (OMAP_OVERFLOW beyond, the cuckoo table's overflow analogue).
// Per batch:
//   k_ocopy              ops -> images, 128-B op lines, (hash, seq) sort keys
//   sort128              by (hash, seq): a key's ops are contiguous, in order
//   k_ogather            position records (kind, key, hash) read once
//   k_scan_*<OgtOp>      keys -> group slots of their partition (c per
//                        partition), each group's composed transform
//   k_okey               per partition: stream its S directory entries, match
//                        the groups' keys, admit new keys into free rows,
//                        rewrite every entry; each group's row -> its head's
//                        position
//   k_scan_*<OrowOp>     the row to every op of the group; row keys and the
//                        per-op lines of the table pass
// then the block store's table pass and (exists, value) copy-forward
// (gvs_kv.h) with OMAP statuses, and k_out.
#pragma once
#include "gvs_kv.h"

namespace gvs {

// keyed hash of a 16-B key (domain bytes 3 / 4; recipients use 1 / 2)
__host__ __device__ inline void omap_hash(const KeyCtx& k, uint64_t k0, uint64_t k1, uint64_t& hi,
                                          uint64_t& lo) {
  const uint64_t m[2] = {k0, k1};
  hi = siphash24_blocks(k.hk0, k.hk1, m, 2, 3, 17);
  lo = siphash24_blocks(k.hk0, k.hk1, m, 2, 4, 17);
}
constexpr uint64_t kOHashMask = ~(uint64_t)kSeqMask;  // hash bits kept in the sort key's low word

// ------------------------------------------------------------- k_ocopy
//
// gvs_omap_op (1056 B: key, op, value) -> image (value), op line {kind,
// invalid, 0, 0} + key, sort key (hash hi, hash lo | seq); an all-zero key
// (OMAP_INVALID_KEY) and padding sort last.  An op code > 3 fails the batch.

struct OcopyArgs {
  const uint4* in;   // n x 66 uint4
  uint4* img;        // B x 64
  uint4* meta;       // B x 8: {kind, e0, overflow, invalid}, key
  Key128* skeys;     // B
  Scal* scal;
  KeyCtx kc;
  uint32_t n, B;
};

__global__ __launch_bounds__(256) void k_ocopy(OcopyArgs a) {
  __shared__ uint4 stage[4 * 64 * 8];
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t i0 = (blockIdx.x * 4 + wave) * 64;
  uint4 my_h = make_uint4(0, 0, 0, 0), my_k = make_uint4(0, 0, 0, 0);
  for (uint32_t j = 0; j < 64; ++j) {
    const uint32_t i = i0 + j;
    const bool real = i < a.n;
    const uint4* src = a.in + (uint64_t)min(i, a.n ? a.n - 1 : 0u) * 66;
    const uint4 v = real ? src[2 + lane] : make_uint4(0, 0, 0, 0);
    a.img[(uint64_t)i * 64 + lane] = v;
    const uint4 key = real ? uni4(src[0]) : make_uint4(0, 0, 0, 0);
    const uint4 h = real ? uni4(src[1]) : make_uint4(0, 0, 0, 0);
    if (real && h.x > KV_REMOVE && lane == 0) atomicOr(&a.scal->error, kKvErr);
    my_h = sel4(lane == j, h, my_h);
    my_k = sel4(lane == j, key, my_k);
  }
  // lane l: op i0 + l
  const uint32_t i = i0 + lane;
  const bool real = i < a.n;
  const bool invalid = !nz4(my_k);
  uint64_t hi, lo;
  omap_hash(a.kc, u4lo(my_k), u4hi(my_k), hi, lo);
  const bool null = !real || invalid;
  Key128 sk;
  sk.hi = null ? ~0ull : hi;
  sk.lo = (null ? kOHashMask : (lo & kOHashMask)) | i;
  a.skeys[i] = sk;
  uint4 rec[8];
  rec[0] = make_uint4(my_h.x, 0u, 0u, (real && invalid) ? 1u : 0u);
  rec[1] = my_k;
  rec[2] = make_uint4((uint32_t)hi, (uint32_t)(hi >> 32), (uint32_t)lo, (uint32_t)(lo >> 32));
#pragma unroll
  for (int c = 3; c < 8; ++c) rec[c] = make_uint4(0, 0, 0, 0);
  wave_store128(stage + wave * 64 * 8, a.meta, i, rec);
}

// ------------------------------------------------------------- k_ogather
// position p's op line, read once per batch into a position-indexed copy

struct OposArgs {
  const Key128* skeys;  // sorted
  const uint4* meta;
  uint4* opr;           // B x 128 B: {kind, invalid, seq, null}, key, {hash}
  uint32_t B;
};

__global__ __launch_bounds__(256) void k_ogather(OposArgs a) {
  __shared__ uint4 stage[4 * 64 * 8];
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  uint4* st = stage + (threadIdx.x >> 6) * 64 * 8;
  const Key128 k = a.skeys[p];
  const uint32_t seq = (uint32_t)k.lo & kSeqMask;
  const bool null = k.hi == ~0ull;
  uint4 l[8], rec[8];
  wave_load128(st, a.meta + (uint64_t)seq * 8, l);
  rec[0] = make_uint4(l[0].x, l[0].w, seq, null ? 1u : 0u);
  rec[1] = l[1];
  rec[2] = l[2];
#pragma unroll
  for (int c = 3; c < 8; ++c) rec[c] = make_uint4(0, 0, 0, 0);
  wave_store128(st, a.opr, p, rec);
}

// ------------------------------------------------------------- OgtOp scan
//
// Segmented by partition (group slots) and by key (the composed transform of
// the key's ops, whether any op creates it).  The key's last op writes the
// 128-B group record {stamp, transform kind, e, creates}, key, hash, {head
// position}; every other op a dummy line.

struct OgtV {
  uint32_t preset, gcnt;   // partition segments: group heads
  uint32_t greset, fk, fe, cr, g0, pad;  // group segments
};

struct OgtArgs {
  const uint4* opr;   // B position records
  uint4* opos;        // B: {seq | head | last | null, slot, q, 0}
  uint4* ogt;         // (W*c + B) x 128 B group records
  OgtV* agg;
  OgtV* carry;
  Scal* scal;
  uint32_t B, W, logW, c, nblk, stamp;
};

struct OgtOp {
  using V = OgtV;
  using Args = OgtArgs;
  __device__ static bool stop(const Args&) { return false; }  // phase A
  __device__ static V identity() { return V{0, 0, 0, kTId, 0, 0, 0, 0}; }
  __device__ static V combine(const V& a, const V& b) {
    V r;
    r.preset = selu32(b.preset != 0u, 1u, a.preset);
    r.gcnt = selu32(b.preset != 0u, b.gcnt, a.gcnt + b.gcnt);
    const bool g = b.greset != 0u;
    const uint4 f = KvOp::f_combine(make_uint4(a.fk, a.fe, 0, 0), make_uint4(b.fk, b.fe, 0, 0));
    r.greset = selu32(g, 1u, a.greset);
    r.fk = selu32(g, b.fk, f.x);
    r.fe = selu32(g, b.fe, f.y);
    r.cr = selu32(g, b.cr, a.cr | b.cr);
    r.g0 = selu32(g, b.g0, a.g0);
    r.pad = 0;
    return r;
  }
  __device__ static uint4 rec0(const Args& a, uint32_t p) { return a.opr[(uint64_t)p * 8]; }
  __device__ static uint4 hash(const Args& a, uint32_t p) { return a.opr[(uint64_t)p * 8 + 2]; }
  __device__ static uint32_t part(const Args& a, uint4 h, bool null) {
    const uint64_t hi = (uint64_t)h.x | ((uint64_t)h.y << 32);
    return null ? a.W : (a.logW ? (uint32_t)(hi >> (64 - a.logW)) : 0u);
  }
  __device__ static bool same_key(uint4 x, uint4 y) {
    return (x.x == y.x) & (x.y == y.y) & ((x.z & ~kSeqMask) == (y.z & ~kSeqMask)) & (x.w == y.w);
  }
  __device__ static V local(const Args& a, uint32_t p, uint4*) {
    const uint4 r = rec0(a, p), h = hash(a, p);
    const bool null = r.w != 0u;
    uint4 hp = make_uint4(~0u, ~0u, ~0u, ~0u), rp = make_uint4(0, 0, 0, 1u);
    if (p) {
      hp = hash(a, p - 1);
      rp = rec0(a, p - 1);
    }
    const bool pnull = rp.w != 0u;
    const uint32_t q = part(a, h, null), pq = p ? part(a, hp, pnull) : ~0u;
    const bool head = !null & ((p == 0) | pnull | !same_key(h, hp));
    // own transform: READ id, WRITE const(1), REMOVE const(0), INSERT ifabsent
    const uint32_t kind = r.x;
    uint32_t fk = kTId, fe = 0;
    fk = selu32((kind == KV_WRITE) | (kind == KV_REMOVE), kTConst, fk);
    fe = selu32(kind == KV_WRITE, 1u, fe);
    fk = selu32(kind == KV_INSERT, kTIfAbsent, fk);
    return V{(uint32_t)((p == 0) | (q != pq)), head ? 1u : 0u, (head | null) ? 1u : 0u, fk, fe,
             ((kind == KV_WRITE) | (kind == KV_INSERT)) ? 1u : 0u, p, 0u};
  }
  __device__ static void emit(const Args& a, uint32_t p, const V& ex, const V& loc, uint4* stage) {
    const uint4 r = rec0(a, p), h = hash(a, p);
    const bool null = r.w != 0u;
    uint4 hn = make_uint4(~0u, ~0u, ~0u, ~0u), rn = make_uint4(0, 0, 0, 1u);
    if (p + 1 < a.B) {
      hn = hash(a, p + 1);
      rn = rec0(a, p + 1);
    }
    const bool last = !null & ((p + 1 == a.B) | (rn.w != 0u) | !same_key(h, hn));
    const V in = combine(ex, loc);
    const bool head = loc.gcnt != 0u;
    const uint32_t before = loc.preset ? 0u : ex.gcnt;
    const uint32_t k = head ? before : before - 1u;
    if (head && k >= a.c) atomicOr(&a.scal->error, 1u);
    const uint32_t kk = min(k, a.c - 1u);
    const uint32_t q = part(a, h, null);
    a.opos[p] = make_uint4(r.z | (head ? kPosHead : 0u) | (last ? kPosLast : 0u) | (null ? kPosNull : 0u),
                           null ? kNone : q * a.c + kk, q, 0u);
    uint4 rec[8];
    rec[0] = make_uint4(a.stamp, in.fk, in.fe, in.cr);
    rec[1] = a.opr[(uint64_t)p * 8 + 1];  // key
    rec[2] = h;
    rec[3] = make_uint4(in.g0, 0u, 0u, 0u);
#pragma unroll
    for (int c = 4; c < 8; ++c) rec[c] = make_uint4(0, 0, 0, 0);
    const uint64_t idx = last ? (uint64_t)q * a.c + kk : (uint64_t)a.W * a.c + p;
    wave_store128(stage, a.ogt, idx, rec);
  }
};

// ------------------------------------------------------------- k_okey
//
// One workgroup per partition: its c group records (fixed), its S directory
// entries (fixed, rewritten).  Row j's key is matched against the groups by
// hash (binary search over the partition's groups, log2(c) fixed steps) and
// then by key.  Groups that need a row (key absent, some op creates it) are
// admitted in group (hash) order into the partition's free rows, as many as
// there are; the rest overflow.  Each group's result {physical row or none,
// e0, overflow} goes to its head op's position.

struct OkeyArgs {
  const uint4* ogt;   // group records
  uint4* kdir;        // N x 32 B: key, hash
  uint4* ogp;         // (B + W*c) x 128 B: group results by head position (dummies after B)
  Scal* scal;
  uint32_t W, S, c, B, stamp;
  // sealed map (AUTH): the directory as N/32 rows of 1 KiB (32 entries each),
  // sealed like the mailbox rows (AES-CTR, BLAKE2b tag over the row, its
  // index, the epoch and table kDirTable), one 16-B tag per row
  SealCtx sc;
  const uint32_t* te;
  uint4* ktag;
};

constexpr uint32_t kDirTable = 3;        // seal domain of the key directory rows
constexpr uint32_t kOkeySealedSlots = 256;  // group slots per partition, sealed map (LDS: the AES tables)
constexpr uint32_t kOkeySealedRows = 1024;  // rows per partition, sealed map (entries held in registers)

struct GroupO {
  uint64_t hi, lo;  // hash (lo with the seq bits cleared)
  uint32_t key[4];
  uint32_t fk, fe, cr, real;
  int32_t row;      // row in the partition: matched or placed
  uint32_t e0, head, pad;
};

__device__ inline int find_group_o(const GroupO* g, uint32_t ng, uint32_t c, uint64_t hi, uint64_t lo) {
  // first group >= (hi, lo) among g[0, ng): fixed log2(c) + 1 steps
  uint32_t pos = 0, top = 1;
  while (top < c) top <<= 1;  // depends on c only
  for (uint32_t step = top; step > 0; step >>= 1) {
    const uint32_t t = pos + step;
    const GroupO& G = g[min(t - 1, c - 1)];
    // both words read at every step, bitwise (no short-circuit branch that
    // skips the compare by the data; find_group_m's rule)
    uint64_t ghi = G.hi, glo = G.lo;
    asm volatile("" : "+v"(ghi), "+v"(glo));
    const bool lt = (t <= ng) & ((ghi < hi) | ((ghi == hi) & (glo < lo)));
    pos = lt ? t : pos;
  }
  const GroupO& G = g[min(pos, c - 1)];
  uint64_t ghi = G.hi, glo = G.lo;
  asm volatile("" : "+v"(ghi), "+v"(glo));
  return ((pos < ng) & (ghi == hi) & (glo == lo)) ? (int)pos : -1;
}

template <bool AUTH>
__global__ __launch_bounds__(256) void k_okey(OkeyArgs a) {
  constexpr uint32_t kG = AUTH ? kOkeySealedSlots : kSlotMax;  // group slots at most; g[kG]: the sink
  GVS_TE_LDS s_te[AUTH ? kTeWords : 1];
  __shared__ uint4 s_st[AUTH ? 4 * stage_u4(2) : 1];
  __shared__ GroupO g[kG + 1];
  __shared__ int16_t s_m[kRowsMax];    // row -> matched group, or -1
  __shared__ uint8_t s_free[kRowsMax];
  __shared__ uint16_t s_fpfx[kRowsMax + 1];
  __shared__ uint8_t s_need[kG + 1];
  __shared__ uint16_t s_npfx[kG + 1];
  __shared__ int16_t s_pend[kG + 1];
  __shared__ uint32_t s_w[4], s_ng;
  const uint32_t tid = threadIdx.x, w = blockIdx.x, lane = lane_id(), wave = tid >> 6;
  if (a.scal->error) return;
  if (AUTH) load_te(s_te, a.te);
  uint4* st = s_st + (AUTH ? wave * stage_u4(2) : 0u);
  if (tid == 0) s_ng = 0;
  __syncthreads();
  // Global reads cover whole 128-B lines in one instruction (a line read in
  // parts by several instructions is fetched whole or in halves depending on
  // timing): a group record by 8 lanes, words 1..3 shuffled to its first lane.
  for (uint32_t k0 = wave * 8; k0 < a.c; k0 += 32) {  // c only
    const uint32_t k = k0 + (lane >> 3);
    const uint4 x = a.ogt[((uint64_t)w * a.c + min(k, a.c - 1u)) * 8 + (lane & 7u)];
    const int l0 = (int)(lane & ~7u);
    const uint4 r0 = x, r1 = shfl4(x, l0 + 1), r2 = shfl4(x, l0 + 2), r3 = shfl4(x, l0 + 3);
    if ((lane & 7u) == 0u && k < a.c) {
      GroupO G;
      G.hi = u4lo(r2);
      G.lo = u4hi(r2) & kOHashMask;
      G.key[0] = r1.x;
      G.key[1] = r1.y;
      G.key[2] = r1.z;
      G.key[3] = r1.w;
      G.fk = r0.y;
      G.fe = r0.z;
      G.cr = r0.w;
      G.real = r0.x == a.stamp ? 1u : 0u;
      G.row = -1;
      G.e0 = 0;
      G.head = r3.x;
      G.pad = 0;
      g[k] = G;
      atomicAdd(&s_ng, G.real);
    }
  }
  __syncthreads();
  const uint32_t ng = s_ng;
  uint4* kd = a.kdir + (uint64_t)w * a.S * 2;
  // match every row's key.  The directory entries are read once and kept in
  // registers for the rewrite (a line read twice hits or misses L2 depending
  // on the traffic in between: FETCH_SIZE would depend on the keys)
  // Each wave reads its 64 entries (2 KiB) as two whole-line loads, entry
  // j = tid + 256 it to lane tid % 64 by shuffles (S >= 256, a power of two).
  constexpr uint32_t kIt = AUTH ? kOkeySealedRows / 256 : kRowsMax / 256;
  uint4 dkey[kIt], dh[kIt];
  const int se = (int)((2u * lane) & 63u);
#pragma unroll
  for (uint32_t it = 0; it < kIt; ++it) {
    const uint32_t j0 = it * 256 + wave * 64;
    if (j0 >= a.S) break;  // S only
    uint4 lo = kd[(uint64_t)j0 * 2 + lane], hi = kd[(uint64_t)j0 * 2 + 64 + lane];
    if (AUTH) {  // directory rows r0, r0 + 1: verified and decrypted at the epoch
      uint4 v[2] = {lo, hi};
      const uint64_t r0 = ((uint64_t)w * a.S + j0) / 32;
      if (!wave_unseal<2>(a.sc, s_te, kDirTable, r0, v, a.ktag, false, st) && lane == 0)
        atomicOr(&a.scal->error, 8u);
      lo = v[0];
      hi = v[1];
    }
    const uint4 klo = shfl4(lo, se), khi = shfl4(hi, se), hlo = shfl4(lo, se + 1), hhi = shfl4(hi, se + 1);
    dkey[it] = sel4(lane < 32u, klo, khi);
    dh[it] = sel4(lane < 32u, hlo, hhi);
  }
#pragma unroll
  for (uint32_t it = 0; it < kIt; ++it) {
    const uint32_t j = tid + it * 256;
    if (j >= a.S) break;
    const uint4 key = dkey[it], h = dh[it];
    const bool used = nz4(key);
    const int k = find_group_o(g, ng, a.c, u4lo(h), u4hi(h) & kOHashMask);
    const GroupO& G = g[k >= 0 ? k : 0];
    // bitwise: a short-circuit && skipped the key compares (code) for rows
    // without a hash match, i.e. by how many keys the batch misses; the
    // instruction fetch showed in FETCH_SIZE (+20-40 KiB under the miss and
    // insert-of-new-key mixes, profiles/r06f_oblivious_FETCH_SIZE_omap.txt)
    const bool match = used & (k >= 0) & (key.x == G.key[0]) & (key.y == G.key[1]) & (key.z == G.key[2]) &
                       (key.w == G.key[3]);
    const uint32_t kk = match ? (uint32_t)k : kG;  // sink entry otherwise
    g[kk].row = (int32_t)j;
    g[kk].e0 = 1u;
    s_m[j] = match ? (int16_t)k : (int16_t)-1;
    s_free[j] = used ? 0 : 1;
  }
  __syncthreads();
  for (uint32_t k = tid; k < a.c; k += 256) {
    const GroupO& G = g[k];
    s_need[k] = ((k < ng) & !G.e0 & (G.cr != 0u)) ? 1 : 0;
  }
  __syncthreads();
  block_flag_scan(s_free, a.S, s_fpfx, s_w);
  block_flag_scan(s_need, a.c, s_npfx, s_w);
  const uint32_t nfree = s_fpfx[a.S], nneed = s_npfx[a.c];
  const uint32_t nadm = min(nfree, nneed);
  for (uint32_t k = tid; k < a.c; k += 256)  // admitted groups in order; the rest write the sink
    s_pend[((s_need[k] != 0) & (s_npfx[k] < nadm)) ? s_npfx[k] : kG] = (int16_t)k;
  __syncthreads();
  // the r-th free row takes the r-th admitted group
  for (uint32_t j = tid; j < a.S; j += 256) {
    const bool take = (s_free[j] != 0) & (s_fpfx[j] < nadm);
    const int16_t k = s_pend[min((uint32_t)s_fpfx[j], kG)];
    const uint32_t kk = take ? (uint32_t)k : kG;
    g[kk].row = (int32_t)j;
    s_m[j] = take ? (int16_t)(k | 0x4000) : s_m[j];  // placed: bit 14
  }
  __syncthreads();
  // the directory after the batch: a group's key stays or arrives where its
  // final state exists (transform applied to e0; an overflowed group never
  // exists)
#pragma unroll
  for (uint32_t it = 0; it < kIt; ++it) {
    const uint32_t j = tid + it * 256;
    if (j >= a.S) break;
    const int16_t m = s_m[j];
    const uint32_t k = (uint32_t)(m & 0x3fff);
    const GroupO& G = g[m >= 0 ? k : 0u];
    // every field read, then selected (a ternary over fields compiled to a
    // branch per row on its group's transform kind)
    uint32_t gfk = G.fk, ge0 = G.e0, gfe = G.fe;
    asm volatile("" : "+v"(gfk), "+v"(ge0), "+v"(gfe));
    const uint32_t efin = selu32(gfk == kTId, ge0, selu32(gfk == kTConst, gfe, 1u));
    uint4 key = dkey[it], h = dh[it];
    const uint4 gk = make_uint4(G.key[0], G.key[1], G.key[2], G.key[3]);
    const uint4 gh = make_uint4((uint32_t)G.hi, (uint32_t)(G.hi >> 32), (uint32_t)G.lo, (uint32_t)(G.lo >> 32));
    key = sel4(m >= 0, sel4(efin != 0u, gk, make_uint4(0, 0, 0, 0)), key);
    h = sel4(m >= 0, sel4(efin != 0u, gh, make_uint4(0, 0, 0, 0)), h);
    // back as two whole-line stores: word 2e + b of a half is entry e's key (b = 0) or hash
    const int e = (int)(lane >> 1);
    const uint4 klo = shfl4(key, e), khi = shfl4(key, 32 + e), hlo = shfl4(h, e), hhi = shfl4(h, 32 + e);
    const uint64_t j0 = (uint64_t)j - lane;
    uint4 v[2] = {sel4(lane & 1u, hlo, klo), sel4(lane & 1u, hhi, khi)};
    if (AUTH)  // sealed at the next epoch, tags with them
      wave_seal<2>(a.sc, s_te, kDirTable, ((uint64_t)w * a.S + j0) / 32, a.sc.epoch + 1u, v, a.ktag, false, st);
    kd[j0 * 2 + lane] = v[0];
    kd[j0 * 2 + 64 + lane] = v[1];
  }
  // each group's result to its head position (slots without a group:
  // dummies), a record by 8 lanes: one whole-line store
  for (uint32_t k0 = wave * 8; k0 < a.c; k0 += 32) {  // c only
    const uint32_t k = min(k0 + (lane >> 3), a.c - 1u);
    const GroupO& G = g[k];
    const bool real = k < ng;
    const bool ovf = real & (s_need[k] != 0) & (s_npfx[k] >= nadm);
    uint32_t grow = (uint32_t)G.row, ghead = G.head;  // read whatever `real` is, then selected
    asm volatile("" : "+v"(grow), "+v"(ghead));
    const uint64_t prow = (int32_t)grow >= 0 ? (uint64_t)w * a.S + grow : ~0ull;
    const uint64_t idx = real ? ghead : (uint64_t)a.B + (uint64_t)w * a.c + k;
    const uint4 rec0 = make_uint4((uint32_t)prow, (uint32_t)(prow >> 32), (G.e0 ? 1u : 0u) | (ovf ? 2u : 0u), 0u);
    if (k0 + (lane >> 3) < a.c) st_drop(a.ogp, idx * 8 + (lane & 7u), sel4((lane & 7u) == 0u, rec0, make_uint4(0, 0, 0, 0)));
  }
}

// A sealed map's directory at creation: N/32 all-zero rows sealed at epoch 0,
// one wave per two rows (grid-stride).
__global__ __launch_bounds__(256) void k_kdir_seal_init(SealCtx c, const uint32_t* g_te, uint4* kdir,
                                                        uint4* ktag, uint64_t n_rows) {
  GVS_TE_LDS s_te[kTeWords];
  __shared__ uint4 s_st[4 * stage_u4(2)];
  load_te(s_te, g_te);
  __syncthreads();
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  uint4* st = s_st + wave * stage_u4(2);
  for (uint64_t r0 = ((uint64_t)blockIdx.x * 4 + wave) * 2; r0 < n_rows; r0 += (uint64_t)gridDim.x * 8) {
    uint4 v[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    wave_seal<2>(c, s_te, kDirTable, r0, 0u, v, ktag, false, st);
    kdir[r0 * 64 + lane] = v[0];
    kdir[r0 * 64 + 64 + lane] = v[1];
  }
}

// ------------------------------------------------------------- OrowOp scan
//
// The group's result (read at its head position) copied forward to every op
// of the group: each op's row key for the table pass and its op line {kind,
// e0, overflow, invalid} for KvOp.

struct OrowV {
  uint32_t reset, row_lo, row_hi, flags;
};

struct OrowArgs {
  const uint4* opos;
  const uint4* opr;
  const uint4* ogp;
  uint64_t* rkeys;    // B row keys for the table pass
  uint4* meta;        // B x 128 B by seq (KvOp's op lines)
  OrowV* agg;
  OrowV* carry;
  Scal* scal;
  uint32_t B, nblk;
};

struct OrowOp {
  using V = OrowV;
  using Args = OrowArgs;
  __device__ static bool stop(const Args& a) { return a.scal->error != 0u; }
  __device__ static V identity() { return V{0, 0, 0, 0}; }
  __device__ static V combine(const V& a, const V& b) {
    const bool r = b.reset != 0u;
    return V{selu32(r, 1u, a.reset), selu32(r, b.row_lo, a.row_lo), selu32(r, b.row_hi, a.row_hi),
             selu32(r, b.flags, a.flags)};
  }
  __device__ static V local(const Args& a, uint32_t p, uint4*) {
    const uint4 op = a.opos[p];
    const uint4 g = a.ogp[(uint64_t)p * 8];  // meaningful at heads only; read at every position
    const bool head = op.x & kPosHead, null = op.x & kPosNull;
    return V{(head | null) ? 1u : 0u, head ? g.x : ~0u, head ? g.y : ~0u, head ? g.z : 0u};
  }
  __device__ static void emit(const Args& a, uint32_t p, const V& ex, const V& loc, uint4* stage) {
    const V in = combine(ex, loc);
    const uint4 op = a.opos[p];
    const uint4 r = a.opr[(uint64_t)p * 8];
    const uint32_t seq = op.x & kSeqMask;
    const bool null = op.x & kPosNull;
    const uint64_t prow = ((uint64_t)in.row_hi << 32) | in.row_lo;
    const bool has_row = !null & (prow != ~0ull);
    a.rkeys[p] = r_key(has_row ? prow : kRNullRow, 0u, seq);
    uint4 rec[8];
    rec[0] = make_uint4(r.x, null ? 0u : (in.flags & 1u), null ? 0u : (in.flags >> 1) & 1u, r.y);
#pragma unroll
    for (int c = 1; c < 8; ++c) rec[c] = make_uint4(0, 0, 0, 0);
    wave_store128(stage, a.meta, seq, rec);
  }
};

}  // namespace gvs
