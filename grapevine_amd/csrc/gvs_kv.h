// gvs_kv.h — block and key-value access on the fixed-slot table pass: the
// mc-oblivious-traits surfaces of SURVEY.md §8 a10 (ObliviousHashMap) and a11
// (ORAM::access), batched.
//
// A batch of B ops over a table of N 1 KiB rows (partition-major, as the
// message table) runs:
//   k_bcopy          ops -> 1 KiB images, 128-B per-op meta lines, row keys
//   sort64           row keys (row, seq)
//   k_scan_*<RtxOp>  rows -> transaction slots (gvs_txn.h)
//   k_rpass2         table pass: apply the previous batch's final states,
//                    snapshot this batch's rows (gvs_txn.h)
//   k_vscan_*<KvOp>  (exists, value) copy-forward along each row's ops
//   k_kv_c           per op: status, the value it saw; the final states (P)
// Each op's state transform is one of id (READ), const(e, v) (WRITE: (1, v),
// REMOVE: (0, 0)) and ifabsent(v) (INSERT).  The class is closed under
// composition, so a row's ops fold associatively and the scan is op-parallel.
#pragma once
#include "gvs_txn.h"

namespace gvs {

enum KvKind : uint32_t { KV_READ = 0, KV_WRITE = 1, KV_INSERT = 2, KV_REMOVE = 3 };
// per-op status (mc-oblivious-traits OMAP_* codes)
constexpr uint32_t kOmapFound = 0, kOmapNotFound = 1, kOmapOverflow = 2, kOmapInvalidKey = 3;
// transform kinds in the scan flags F = {kind, e, 0, 0}
constexpr uint32_t kTId = 0, kTConst = 1, kTIfAbsent = 2;

// ------------------------------------------------------------- k_bcopy
//
// ORAM ops (gvs_block_op, 1040 B: index, op, data) -> image (data), meta line
// {kind, e0 = 1, 0, 0} and row key.  Ops >= n are padding (null row).  An
// index >= N or an op code > 1 fails the batch (error bit kKvErr) before any
// state changes.
constexpr uint32_t kKvErr = 64;

struct BcopyArgs {
  const uint4* in;   // n x 65 uint4
  uint4* img;        // B x 64
  uint4* meta;       // B x 8
  uint64_t* rkeys;   // B
  Scal* scal;
  uint64_t N;
  uint32_t n, B, W, S;
};

__global__ __launch_bounds__(256) void k_bcopy(BcopyArgs a) {
  __shared__ uint4 stage[4 * 64 * 8];
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t i0 = (blockIdx.x * 4 + wave) * 64;  // 64 ops per wave: meta lines by wave_store128
  uint4 rec[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) rec[c] = make_uint4(0, 0, 0, 0);
  uint32_t my_kind = 0;
  uint64_t my_key = 0;
  for (uint32_t j = 0; j < 64; ++j) {
    const uint32_t i = i0 + j;
    const bool real = i < a.n;
    const uint4* src = a.in + (uint64_t)min(i, a.n ? a.n - 1 : 0u) * 65;
    uint4 v = real ? src[1 + lane] : make_uint4(0, 0, 0, 0);
    a.img[(uint64_t)i * 64 + lane] = v;
    const uint4 h = real ? uni4(src[0]) : make_uint4(0, 0, 0, 0);
    const uint64_t index = (uint64_t)h.x | ((uint64_t)h.y << 32);
    const bool bad = real && (index >= a.N || h.z > 1u);
    if (bad && lane == 0) atomicOr(&a.scal->error, kKvErr);
    // 32-bit division (index < N < 2^32 when it counts): a 64-bit one branches
    // on the dividend's high word
    const uint32_t ix = (real && !bad) ? (uint32_t)index : 0u;
    const uint64_t row = (real && !bad) ? (uint64_t)(ix % a.W) * a.S + ix / a.W : kRNullRow;
    my_key = lane == j ? r_key(row, 0u, i) : my_key;
    my_kind = lane == j ? h.z : my_kind;
  }
  a.rkeys[i0 + lane] = my_key;  // the wave's 64 keys in one store: whole lines
  rec[0] = make_uint4(my_kind, 1u, 0u, 0u);
  wave_store128(stage + wave * 64 * 8, a.meta, i0 + lane, rec);
}

// ------------------------------------------------------------- KvOp scan

struct KvArgs {
  GVS_VSCAN_FIELDS
  const uint4* rpos;       // B sorted positions (RtxOp)
  const uint4* meta;       // B x 128 B, by seq: {kind, e0, overflow, 0}
  const uint4* img;        // B x 1 KiB, by seq
  const uint4* snapp;      // B x 1 KiB: row snapshots at their first op's position
  uint4* pbuf;             // B x 1 KiB: final states of the positions that are not a row's last
  uint4* psd;              // B x 128 B side entries {row lo, row hi, valid, slot}
  uint4* psink;            // the other positions' states, by position (plain: PS's B sink lines; AUTH: P)
  uint4* ps;               // plain: W*c x 1 KiB, each row's final state at its slot (the pass
                           // reads P by slot); AUTH: null (P by position, sealed)
  uint4* out;              // ORAM: n x 1 KiB (caller); OMAP: B x kRespSlot
  uint4* outdummy;         // ORAM: B x 1 KiB for padding ops
  uint32_t n, S, omap;
};

struct KvHdr {
  uint32_t seq, flags, slot, kind, e0, ovf, invalid;
  uint64_t prow;
};

// A position's record (8 uint4, read once per kernel through LDS: a line read
// twice hits or misses L2 depending on the traffic in between, whose
// addresses depend on the data): word 0 its RPOS entry, word 1 its op's meta
// word, 2..7 the rest of the meta line (the whole line is read).
__device__ inline uint4 kv_rec_line(const KvArgs& a, uint64_t i) {
  const uint32_t k = (uint32_t)i & 7u;
  const uint4 rp = a.rpos[i >> 3];
  const uint4 m = a.meta[(uint64_t)(rp.x & kSeqMask) * 8 + ((k + 7u) & 7u)];
  return k == 0u ? rp : m;
}

__device__ inline KvHdr kv_hdr_rec(const KvArgs& a, const uint4* r) {
  const uint4 rp = uni4(r[0]), m = uni4(r[1]);
  KvHdr h;
  h.seq = rp.x & kSeqMask;
  h.flags = rp.x;
  h.slot = rp.y;
  h.prow = (rp.x & kPosNull) ? 0ull : (uint64_t)rp.z * a.S + rp.w;
  h.kind = m.x;
  h.e0 = m.y;
  h.ovf = m.z;
  h.invalid = m.w;
  return h;
}

struct KvOp {
  using Args = KvArgs;
  static constexpr bool kSelect = true;
  static constexpr bool kStash = true;  // each position's record read once (kv_rec_line)
  __device__ static uint4 rec_line(const Args& a, uint64_t i) { return kv_rec_line(a, i); }
  __device__ static uint4 f_identity() { return make_uint4(kTId, 0, 0, 0); }
  // a then b: function composition of the transforms
  __device__ static uint4 f_combine(uint4 a, uint4 b) {
    const uint4 one = make_uint4(kTConst, 1u, 0, 0);
    uint4 r = sel4(b.x == kTConst, b, a);
    const uint4 ifa = sel4(a.x == kTId, b, sel4(a.x == kTConst && a.y == 0u, one, a));
    return sel4(b.x == kTIfAbsent, ifa, r);
  }
  __device__ static bool takes_b(uint4 a, uint4 b) {
    return b.x == kTConst || (b.x == kTIfAbsent && (a.x == kTId || (a.x == kTConst && a.y == 0u)));
  }
  __device__ static uint4 v_combine(uint4 fa, uint4 va, uint4 fb, uint4 vb) {
    return sel4(takes_b(fa, fb), vb, va);
  }
  // the op's own transform (an overflowed INSERT / WRITE changes nothing)
  __device__ static uint4 own_f(const KvHdr& h) {
    const bool creates = h.kind == KV_WRITE || h.kind == KV_INSERT;
    uint32_t k = kTId, e = 0;
    k = selu32(h.kind == KV_WRITE || h.kind == KV_REMOVE, kTConst, k);
    e = selu32(h.kind == KV_WRITE, 1u, e);
    k = selu32(h.kind == KV_INSERT, kTIfAbsent, k);
    k = selu32(creates && h.ovf, kTId, k);
    return make_uint4(k, e, 0, 0);
  }
  // element of position p: a row head starts from const(e0, snapshot)
  __device__ static uint4 f_of_hdr(const KvHdr& h) {
    const uint4 o = own_f(h);
    const uint4 hd = f_combine(make_uint4(kTConst, h.e0, 0, 0), o);
    const bool head = h.flags & kPosHead, null = h.flags & kPosNull;
    return sel4(null, make_uint4(kTConst, 0, 0, 0), sel4(head, hd, o));
  }
  // (the stash scan takes f from the record; S is in the args, not the record)
  __device__ static uint4 f_of_rec(const uint4* r) {
    const uint4 rp = uni4(r[0]), m = uni4(r[1]);
    KvHdr h{};
    h.flags = rp.x;
    h.kind = m.x;
    h.e0 = m.y;
    h.ovf = m.z;
    return f_of_hdr(h);
  }
  // value of position p's element: the op's image when its own transform
  // supplies the value (WRITE; INSERT into an absent row), else the snapshot
  // (a head whose own transform keeps the row), zero for REMOVE / null
  __device__ static bool from_img(const KvHdr& h) {
    const uint4 o = own_f(h);
    const bool head = h.flags & kPosHead;
    return (o.x == kTConst && o.y == 1u) || (o.x == kTIfAbsent && !(head && h.e0));
  }
  // k_vscan_a: every op's two rows (its SNAPP line and its image) are read,
  // the defining op's value kept: addresses that do not depend on the ops
  __device__ static uint4 elem_value(const Args& a, uint32_t p, const uint4* r) {
    const KvHdr h = kv_hdr_rec(a, r);
    const bool head = h.flags & kPosHead;
    const uint4 sv = ld_row<false>(&a.snapp[(uint64_t)p * 64 + lane_id()]);
    const uint4 iv = ld_row<false>(&a.img[(uint64_t)h.seq * 64 + lane_id()]);
    const uint4 x = sel4(head && !from_img(h), sv, iv);
    const uint4 o = own_f(h);
    const bool zero = (h.flags & kPosNull) || (o.x == kTConst && o.y == 0u) || (!head && o.x == kTId);
    return sel4(zero, make_uint4(0, 0, 0, 0), x);
  }
  __device__ static uint4 value_fin(uint4, uint4 v) { return v; }
};

// k_kv_c: each wave walks its 16 ops from its carry: the state before the op
// (row head: (e0, snapshot)), the op's status and returned value, the state
// after it into P at the op's position, and its side entry.
__global__ __launch_bounds__(256) void k_kv_c(KvArgs a) {
  if (a.scal->error) return;
  __shared__ uint4 s_v[4][64];
  __shared__ uint4 s_f[4];
  __shared__ uint4 s_rec[4][16 * 8];  // each wave's 16 position records
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t p0 = blockIdx.x * kVBlk + wave * 16;
  uint4* rec = s_rec[wave];
  rec[lane] = kv_rec_line(a, (uint64_t)p0 * 8 + lane);
  rec[64 + lane] = kv_rec_line(a, (uint64_t)p0 * 8 + 64 + lane);
  wave_lds_sync();
  // each op's own SNAPP line (heads: the row's snapshot) and its image, read once
  uint4 svs[16], ivs[16];
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const KvHdr h = kv_hdr_rec(a, rec + j * 8);
    svs[j] = ld_row<false>(&a.snapp[(uint64_t)(p0 + j) * 64 + lane]);
    ivs[j] = ld_row<false>(&a.img[(uint64_t)h.seq * 64 + lane]);
  }
  uint4 cf, cv;
  {  // the wave's aggregate from registers, then the carry
    uint4 f = KvOp::f_identity(), v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const KvHdr h = kv_hdr_rec(a, rec + j * 8);
      const uint4 e = KvOp::f_of_hdr(h);
      const bool head = h.flags & kPosHead;
      const uint4 o = KvOp::own_f(h);
      const bool zero = (h.flags & kPosNull) || (o.x == kTConst && o.y == 0u) || (!head && o.x == kTId);
      const uint4 x = sel4(head && !KvOp::from_img(h), svs[j], ivs[j]);
      v = sel4(KvOp::takes_b(f, e), sel4(zero, make_uint4(0, 0, 0, 0), x), v);
      f = KvOp::f_combine(f, e);
    }
    vscan_carry_tail<KvOp>(a, s_v, s_f, f, v, cf, cv);
  }
  uint4 sd = make_uint4(0, 0, 0, 0);
  const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t p = p0 + j;
    const KvHdr h = kv_hdr_rec(a, rec + j * 8);
    const bool head = h.flags & kPosHead, null = h.flags & kPosNull, last = h.flags & kPosLast;
    const uint4 sv = svs[j], iv = ivs[j];
    // the state before the op
    const bool e = head ? h.e0 != 0u : (cf.x == kTConst && cf.y != 0u);
    const uint4 v = sel4(head, sv, cv);
    const bool creates = h.kind == KV_WRITE || h.kind == KV_INSERT;
    uint32_t status = e ? kOmapFound : kOmapNotFound;
    status = selu32((creates && h.ovf) || (null && creates && a.omap), kOmapOverflow, status);
    status = selu32(null && !creates, kOmapNotFound, status);
    status = selu32(null && h.invalid, kOmapInvalidKey, status);
    const bool ovf = status == kOmapOverflow;
    // the value handed back: the row's value (READ, WRITE, REMOVE, INSERT of
    // a present key); the default an INSERT put in; zero when absent
    uint4 resp = sel4(e && !null, v, z);
    resp = sel4(h.kind == KV_INSERT && !e && !ovf && !null, iv, resp);
    // the state after it
    bool e2 = e;
    uint4 v2 = v;
    const bool wr = h.kind == KV_WRITE && !ovf, ins = h.kind == KV_INSERT && !ovf && !e;
    v2 = sel4(wr || ins, iv, v2);
    e2 = (wr || ins) ? true : e2;
    v2 = sel4(h.kind == KV_REMOVE, z, v2);
    e2 = h.kind == KV_REMOVE ? false : e2;
    v2 = sel4(null, z, v2);
    e2 = null ? false : e2;
    cv = v2;
    cf = make_uint4(kTConst, e2 ? 1u : 0u, 0, 0);
    if (a.omap) {
      const uint64_t r0 = (uint64_t)h.seq * (kRespSlot / 16);
      st_drop(a.out, r0 + lane, resp);
      if (lane < 8) st_drop(a.out, r0 + 64 + lane, make_uint4(lane == 0 ? status : 0u, 0, 0, 0));
    } else {
      st_drop(null ? a.outdummy : a.out, (uint64_t)h.seq * 64 + lane, v);
    }
    // a row's final state to its slot (the next pass reads P by slot), the
    // other positions' states to their own sink line of PS after the slots:
    // one write per position, B lines into PS whatever the batch (AUTH: all
    // by position into P, sealed next; the unseal moves them to PS)
    const bool to_slot = a.ps && last;
    st_drop(to_slot ? a.ps : a.psink, (to_slot ? (uint64_t)h.slot : p) * 64 + lane, v2);
    sd = sel4(lane == j, make_uint4((uint32_t)h.prow, (uint32_t)(h.prow >> 32), last ? 1u : 0u, h.slot), sd);
  }
  if (lane < 16) st_drop(a.psd, (uint64_t)(p0 + lane) * 8, sd);
}

}  // namespace gvs
