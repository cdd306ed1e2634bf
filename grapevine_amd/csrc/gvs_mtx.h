// gvs_mtx.h — fixed-slot transactions of the mailbox passes.
//
// The mailbox passes used to discover each partition's recipient groups from
// its sorted ops and to visit every op inside the partition's workgroup, so a
// hot recipient made one workgroup long (a timing leak).  Here:
//
//   k_gtx_{a,b,c}  over the S1-sorted ops (recipient hash, class, seq): each
//                  recipient group becomes ONE slot of its mailbox partition
//                  (cm slots; more groups is a batch overflow); the group's
//                  last op writes the 128-B group descriptor (counts per
//                  class, first create), every other op a dummy line.
//   k_m1x          mailbox read pass, one workgroup per partition: matches
//                  rows to its cm slots, admits new recipients, and writes
//                  every slot's snapshot (the row's 62 ids, with the group's
//                  verdict in lanes 0..1): cm slots whatever they hold.
//   k_m1r_*        op-parallel copy-forward of the snapshot along the group:
//                  next-message ops take id d, creates their mailbox verdict,
//                  by-id deletes the position of their id.
//   k_m2r_*        op-parallel after the message pass: per group the ids of
//                  its successful creates (lane 2 + rank) and the removal mask
//                  of its successful by-id deletes -> the group's result slot.
//   k_m2x          mailbox write pass: every row rewritten, every result slot
//                  read once.
#pragma once
#include "gvs_txn.h"

namespace gvs {

// ---------------------------------------------------------------- k_gtx

// per S1-sorted position: x = seq | head << 20 | last << 21 | null << 22 |
// class << 23 | sub << 25, y = slot q*cm + k (kNone: no mailbox), z = q,
// w = rank among the group's creates
constexpr uint32_t kMPosHead = 1u << 20, kMPosLast = 1u << 21, kMPosNull = 1u << 22;
__host__ __device__ inline uint32_t mpos_cls(uint32_t x) { return (x >> 23) & 3u; }
__host__ __device__ inline uint32_t mpos_sub(uint32_t x) { return (x >> 25) & 1u; }

struct GtxV {
  uint32_t preset, gcnt;                            // partition segments: group heads
  uint32_t greset, n_next, n_del, n_create, n_x;    // group segments: counts per class
  uint32_t fcs, g0, c1;                             // first create's seq, group start, first create
};

struct GtxArgs {
  const Key128* keys;  // sorted
  const OpState* ops;
  uint4* mpos;         // B
  uint4* gtx;          // 128-B records: Q*cm group slots, then B dummies
  GtxV* agg;
  GtxV* carry;
  Scal* scal;
  uint32_t B, Q, logQ, cm, nblk, stamp;
  uint4* mpid;         // B: each position's message id (OpState words 10..13), for k_m1r_c
};

struct GtxOp {
  using V = GtxV;
  using Args = GtxArgs;
  __device__ static bool stop(const Args&) { return false; }  // phase A
  __device__ static V identity() { return V{0, 0, 0, 0, 0, 0, 0, kNone, 0, kNone}; }
  __device__ static V combine(const V& a, const V& b) {
    V r;
    r.preset = selu32(b.preset != 0u, 1u, a.preset);
    r.gcnt = selu32(b.preset != 0u, b.gcnt, a.gcnt + b.gcnt);
    const bool g = b.greset != 0u;
    r.greset = selu32(g, 1u, a.greset);
    r.n_next = selu32(g, b.n_next, a.n_next + b.n_next);
    r.n_del = selu32(g, b.n_del, a.n_del + b.n_del);
    r.n_create = selu32(g, b.n_create, a.n_create + b.n_create);
    r.n_x = selu32(g, b.n_x, a.n_x + b.n_x);
    r.fcs = selu32(g, b.fcs, selu32(a.fcs != kNone, a.fcs, b.fcs));
    r.g0 = selu32(g, b.g0, a.g0);
    r.c1 = selu32(g, b.c1, selu32(a.c1 != kNone, a.c1, b.c1));
    return r;
  }
  __device__ static uint32_t part(const Args& a, const Key128& k) {
    const bool null = s1_class(k.lo) == 3u;
    return null ? a.Q : (a.logQ ? (uint32_t)(k.hi >> (64 - a.logQ)) : 0u);
  }
  __device__ static bool same_group(const Key128& x, const Key128& y) {
    return x.hi == y.hi && s1_group(x.lo) == s1_group(y.lo);
  }
  __device__ static V local(const Args& a, uint32_t p, uint4*) {
    const Key128 k = a.keys[p];
    Key128 pk = {~0ull, ~0ull};
    if (p) pk = a.keys[p - 1];
    const uint32_t cls = s1_class(k.lo), seq = s1_seq(k.lo);
    const bool null = cls == 3u;
    const bool gh = !null && (p == 0 || !same_group(k, pk));
    const bool ph = p == 0 || part(a, k) != part(a, pk);
    V v;
    v.preset = ph ? 1u : 0u;
    v.gcnt = gh ? 1u : 0u;
    v.greset = (gh || null) ? 1u : 0u;
    v.n_next = (!null && cls == 0u) ? 1u : 0u;
    v.n_del = (!null && cls == 0u && s1_sub(k.lo)) ? 1u : 0u;
    v.n_create = (!null && cls == 1u) ? 1u : 0u;
    v.n_x = (!null && cls == 2u) ? 1u : 0u;
    v.fcs = (!null && cls == 1u) ? seq : kNone;
    v.g0 = p;
    v.c1 = (!null && cls == 1u) ? p : kNone;
    return v;
  }
  __device__ static void emit(const Args& a, uint32_t p, const V& ex, const V& loc, uint4* stage) {
    const Key128 k = a.keys[p];
    Key128 nk = {~0ull, ~0ull};
    if (p + 1 < a.B) nk = a.keys[p + 1];
    const V in = combine(ex, loc);
    const uint32_t cls = s1_class(k.lo), seq = s1_seq(k.lo), sub = (uint32_t)s1_sub(k.lo);
    const bool null = cls == 3u;
    const bool head = loc.gcnt != 0u;
    const bool last = !null && (p + 1 == a.B || !same_group(k, nk));
    const uint32_t before = loc.preset ? 0u : ex.gcnt;
    const uint32_t kslot = head ? before : before - 1u;
    if (head && kslot >= a.cm) atomicOr(&a.scal->error, 1u);
    const uint32_t kk = min(kslot, a.cm - 1u);
    const uint32_t q = part(a, k);
    const uint32_t rank = (!null && cls == 1u && in.c1 != kNone) ? p - in.c1 : 0u;
    a.mpos[p] = make_uint4(seq | (head ? kMPosHead : 0u) | (last ? kMPosLast : 0u) |
                               (null ? kMPosNull : 0u) | (cls << 23) | (sub << 25),
                           null ? kNone : q * a.cm + kk, q, rank);
    uint4 ol[8];  // OpState: x (the mailbox key) is 32-bit words 14..21
    wave_load128(stage, reinterpret_cast<const uint4*>(a.ops + seq), ol);
    const uint32_t* ow = reinterpret_cast<const uint32_t*>(ol);
    const uint64_t glo = s1_group(k.lo);
    a.mpid[p] = make_uint4(ow[10], ow[11], ow[12], ow[13]);
    uint4 rec[8];
    rec[0] = make_uint4(a.stamp, in.n_next, in.n_del, in.n_create);
    rec[1] = make_uint4(in.n_x, in.fcs, in.g0, in.c1);
    rec[2] = make_uint4((uint32_t)k.hi, (uint32_t)(k.hi >> 32), (uint32_t)glo, (uint32_t)(glo >> 32));
    rec[3] = make_uint4(ow[14], ow[15], ow[16], ow[17]);
    rec[4] = make_uint4(ow[18], ow[19], ow[20], ow[21]);
    rec[5] = rec[6] = rec[7] = make_uint4(0, 0, 0, 0);
    const uint64_t idx = last ? (uint64_t)q * a.cm + kk : (uint64_t)a.Q * a.cm + p;
    wave_store128(stage, a.gtx, idx, rec);
  }
};

// ------------------------------------------------------ LDS group table

struct GroupM {  // 64 B
  uint64_t hi, glo;
  uint32_t n_del, n_create, fcs, len;
  int32_t slot;
  uint32_t flags, fl, n_succ, mlo, mhi;
  uint32_t head;  // sorted position of the group's first op (its snapshot line in MSNAPP)
  uint32_t pad;
};

// A group slot's fields, read whatever the batch holds: a short-circuit
// `k < ng && G.slot >= 0 && ...` compiled to branches that skipped the reads
// of unused slots, so the admission ranks (cm x cm reads) ran 10 us faster
// under batches without mailbox groups at the routed shape's cm
// (profiles/r05l-r05p_timing_c3_routed.txt, k_m1x)
struct GroupFields {
  uint32_t slot, len, n_del, n_create, fcs;
};
__device__ inline GroupFields group_fields(const GroupM& G) {
  GroupFields f{(uint32_t)G.slot, G.len, G.n_del, G.n_create, G.fcs};
  asm volatile("" : "+v"(f.slot), "+v"(f.len), "+v"(f.n_del), "+v"(f.n_create), "+v"(f.fcs));
  return f;
}
// the group's length after its pops (0: no row, or not a group of this batch)
__device__ inline uint32_t len_after_pops(const GroupFields& f, bool real) {
  return selu32(real & ((int32_t)f.slot >= 0), f.len - min(f.n_del, f.len), 0u);
}
// admission (grapevine.proto:74): rows that empty after the pops are free
// again (s_empt), new recipients are admitted by the seq of their first create
__device__ inline void count_empty(const GroupM* g, uint32_t ng, uint32_t cm, uint32_t* s_empt) {
  for (uint32_t k = threadIdx.x; k < cm; k += 256) {
    const GroupFields f = group_fields(g[k]);
    const bool real = k < ng;
    atomicAdd(s_empt, (real & ((int32_t)f.slot >= 0) & (f.len == min(f.n_del, f.len))) ? 1u : 0u);
  }
}
__device__ inline void admit_groups(GroupM* g, uint32_t ng, uint32_t cm, uint32_t freeq) {
  for (uint32_t k = threadIdx.x; k < cm; k += 256) {
    GroupM& G = g[k];
    const GroupFields f = group_fields(G);
    const bool real = k < ng;
    const uint32_t len1 = len_after_pops(f, real);
    const bool exists1 = len1 > 0;
    const bool isnew = real & !exists1 & (f.n_create > 0);
    uint32_t rank = 0;
    for (uint32_t k2 = 0; k2 < cm; ++k2) {  // every slot, every field: fixed work
      const GroupFields h = group_fields(g[k2]);
      const bool r2 = k2 < ng;
      const uint32_t hl = len_after_pops(h, r2);
      rank += (r2 & (hl == 0) & (h.n_create > 0) & (h.fcs < f.fcs)) ? 1u : 0u;
    }
    G.fl = len1;
    G.flags = (exists1 ? 1u : 0u) | ((isnew & (rank < freeq)) ? 2u : 0u);
  }
}

// group of (hi, glo) among g[0, ng) (sorted), or -1: a fixed-step search
// (g holds cm + 1 entries: the slots and the sink g[cm])
__device__ inline int find_group_m(const GroupM* g, uint32_t ng, uint32_t cm, uint64_t hi, uint64_t glo) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t step = kGroupMax; step > 0; step >>= 1) {
    const uint32_t c = pos + step;
    const GroupM& G = g[min(c - 1, cm)];
    uint64_t ghi = G.hi, gglo = G.glo;  // both read at every step (no short-circuit branch)
    asm volatile("" : "+v"(ghi), "+v"(gglo));
    const bool less = (ghi < hi) | ((ghi == hi) & (gglo < glo));
    pos = ((c <= ng) & less) ? c : pos;
  }
  const GroupM& G = g[min(pos, cm)];
  uint64_t ghi = G.hi, gglo = G.glo;
  asm volatile("" : "+v"(ghi), "+v"(gglo));
  return ((pos < ng) & (ghi == hi) & (gglo == glo)) ? (int)pos : -1;
}

// occupied rows of the partition -> groups, every side entry read; s_keep
// (LDS, or null) keeps the entries as read, so that a later use does not read
// them again (sealed stores: ma_prepass, gvs_mauth.h)
// (s_src, LDS: the partition's side entries as an earlier stage left them,
// read instead of HBM; k_m21x)
__device__ inline void side_prepass_m(const MArgs& a, uint32_t q, GroupM* g, uint32_t ng,
                                      int16_t* s_sg, uint8_t* s_occb, uint32_t* s_occ,
                                      uint4* s_keep = nullptr, const uint4* s_src = nullptr) {
  for (uint32_t j = threadIdx.x; j < a.Sr; j += 256) {
    const uint64_t row = (uint64_t)q * a.Sr + j;
    uint4 sd = s_src ? s_src[j] : a.side[row];
    if (s_keep) s_keep[j] = sd;
    const uint64_t hi = u4lo(sd), w1 = u4hi(sd);
    const bool occ = (w1 & 1u) != 0;
    const int kf = find_group_m(g, ng, a.cm, hi, w1 >> 23);  // every row: no code skipped
    const int k = occ ? kf : -1;
    atomicAdd(s_occ, occ ? 1u : 0u);
    // rows without a group write the sink entry g[cm]: the same code runs
    // whatever the batch holds (instruction fetch shows in FETCH_SIZE)
    const uint32_t kk = k >= 0 ? (uint32_t)k : a.cm;
    g[kk].slot = (int32_t)j;
    g[kk].len = (uint32_t)(w1 >> 1) & 63u;
    s_sg[j] = (int16_t)k;
    s_occb[j] = occ ? 1 : 0;
  }
}

// this partition's group slots: real ones (stamped by this batch) are dense
// at the front; every descriptor line is read
__device__ inline uint32_t load_groups(const MArgs& a, uint32_t q, GroupM* g, uint32_t* s_ng,
                                       bool with_results) {
  if (threadIdx.x == 0) *s_ng = 0;
  __syncthreads();
  // a record by 8 lanes, one whole line per load instruction (words 1..2 go
  // to the record's first lane by shuffles): a line read in 16-B pieces by
  // several instructions is fetched whole or in halves depending on timing
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  for (uint32_t k0 = wave * 8; k0 < a.cm; k0 += 32) {  // cm only
    const uint32_t k = k0 + (lane >> 3);
    const uint64_t gi = (uint64_t)q * a.cm + min(k, a.cm - 1u);
    const uint4 x = a.gtx[gi * 8 + (lane & 7u)];
    const uint4 hx = with_results ? a.m2tx[gi * kVLineU4 + (lane & 7u)] : make_uint4(0, 0, 0, 0);
    const int l0 = (int)(lane & ~7u);
    const uint4 r0 = x, r1 = shfl4(x, l0 + 1), r2 = shfl4(x, l0 + 2), h = hx;
    if ((lane & 7u) == 0u && k < a.cm) {
      GroupM G;
      G.hi = u4lo(r2);
      G.glo = u4hi(r2);
      G.n_del = r0.z;
      G.n_create = r0.w;
      G.fcs = r1.y;
      G.len = 0;
      G.slot = -1;
      G.flags = 0;
      G.fl = 0;
      G.n_succ = h.y;
      G.mlo = h.z;
      G.mhi = h.w;
      G.head = r1.z;
      G.pad = 0;
      g[k] = G;
      atomicAdd(s_ng, r0.x == a.stamp ? 1u : 0u);  // unconditional: no code path skipped
    }
  }
  __syncthreads();
  return *s_ng;
}

// The row passes run one iteration of their per-group code for every row the
// batch touches (in the row stream, by the wave that streams the row) and one
// for every group slot no row takes.  Touched rows fall to the waves by the
// data, so the slot iterations are dealt out by what each wave already has:
// wave w takes T - t_w of them (T = ceil(cm / 4), t_w its touched rows) and
// spreads them evenly over its chunks, so that every wave runs T iterations
// in the stream, whatever the batch touched (fewer touched rows made k_m1x /
// k_m2x 11-15 us faster at C3: profiles/r04g_timing_c3_store.txt).  A wave
// with more than T touched rows (2^-20-rare under the keyed recipient hash)
// runs them all.  Past the list of slots, iterations use the dry lines.
constexpr uint32_t kRowWaves = 4;
__device__ inline void slot_share(const uint32_t* s_tw, uint32_t cm, uint32_t wave, uint32_t* start,
                                  uint32_t* cnt) {
  const uint32_t T = (cm + kRowWaves - 1) / kRowWaves;
  uint32_t s = 0, c = 0;
#pragma unroll
  for (uint32_t v = 0; v < kRowWaves; ++v) {
    const uint32_t cv = T > s_tw[v] ? T - s_tw[v] : 0u;
    s += v < wave ? cv : 0u;
    c = v == wave ? cv : c;
  }
  *start = s;
  *cnt = c;
}

// chunk i of n: its share of the wave's d slot iterations (even spread)
__device__ inline uint32_t spread_lo(uint32_t i, uint32_t n, uint32_t d) { return n ? (i * d) / n : 0u; }

// --------------------------------------------------------------- k_m1x

// mailbox read pass: snapshot of every group's row, with the verdict header
// lane 0 = {len, fl (length after the pops), flags (1 exists after the
// pops, 2 admitted as a new mailbox), row}; lanes 2.. = the 62 ids
template <bool AUTH>
__global__ __launch_bounds__(256) void k_m1x(MArgs a) {
  static_assert(!AUTH, "sealed stores run k_m1a (gvs_mauth.h)");
  // the group slots and the sink, cm + 1 entries in dynamic LDS sized at
  // launch (9 KiB at C3 instead of 33): more workgroups per CU
  extern __shared__ uint4 s_dyn[];
  GroupM* g = reinterpret_cast<GroupM*>(s_dyn);
  __shared__ int16_t s_sg[kSrMax];
  __shared__ uint8_t s_occb[kSrMax];
  __shared__ uint32_t s_ng, s_occ, s_empt, s_w[4], s_tw[kRowWaves];
  __shared__ uint8_t s_tf[kGroupMax];     // tail: slots without a row
  __shared__ uint16_t s_tp[kGroupMax + 1];
  __shared__ int16_t s_tl[kGroupMax];
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = blockIdx.x;
  if (a.scal->error) return;
  const uint4* part = a.mbox + (uint64_t)q * a.Sr * 64;
  uint4 va[kMU], vb[kMU];
  load_rows(va, part, wave * kMU, a.Sr);
  const uint32_t ng = load_groups(a, q, g, &s_ng, false);
  if (tid == 0) {
    s_occ = 0;
    s_empt = 0;
  }
  __syncthreads();
  side_prepass_m(a, q, g, ng, s_sg, s_occb, &s_occ);
  __syncthreads();
  count_empty(g, ng, a.cm, &s_empt);
  __syncthreads();
  admit_groups(g, ng, a.cm, (a.Sr - s_occ) + s_empt);
  __syncthreads();
  // group snapshots go to MSNAPP at the head's sorted position, so that every
  // op of k_m1r_c reads line p (an address stream that does not depend on the
  // batch); slots without a row write a header-only line there, unused slots
  // their own line of the MSNAP sink: every slot written once
  uint4* dry = a.mdry + (uint64_t)q * kMDryU4;  // slot iterations past the list: 1 KiB line 1
  // each wave's touched rows, and the slots without a row, listed
  if (tid < kRowWaves) s_tw[tid] = 0;
  __syncthreads();
  for (uint32_t j = tid; j < a.Sr; j += 256) atomicAdd(&s_tw[(j / kMU) % kRowWaves], s_sg[j] >= 0 ? 1u : 0u);
  for (uint32_t k = tid; k < a.cm; k += 256) s_tf[k] = ((k < ng) & ((int32_t)group_fields(g[k]).slot >= 0)) ? 0 : 1;
  __syncthreads();
  block_flag_scan(s_tf, a.cm, s_tp, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)
    if (s_tf[k]) s_tl[s_tp[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t nfree = s_tp[a.cm];
  uint32_t d0, dn;
  slot_share(s_tw, a.cm, wave, &d0, &dn);
  const uint32_t nch = a.Sr > wave * kMU ? (a.Sr - wave * kMU + 4 * kMU - 1) / (4 * kMU) : 0u;
  // one iteration: a touched row's snapshot (bit set) or a slot without a row
  // (bit 0: header only), the same code and one 1-KiB line written either way
  auto step = [&](const uint4 (&v)[kMU], uint32_t bit, uint32_t j0, uint32_t di) {
    const bool slot_it = bit == 0u;
    uint4 cur = v[0];
#pragma unroll
    for (int uu = 1; uu < kMU; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
    const uint32_t u0 = (uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u;
    const bool listed = slot_it && di < nfree;
    const int k = slot_it ? (listed ? (int)s_tl[di] : 0) : s_sg[j0 + u0];
    const GroupM& G = g[k >= 0 ? (uint32_t)k : 0u];
    const bool real = !slot_it || (listed && (uint32_t)k < ng);
    const uint4 hdr = sel4(real, make_uint4(slot_it ? 0u : G.len, G.fl, G.flags, (uint32_t)G.slot),
                           make_uint4(0, 0, 0, 0));
    cur = sel4(lane == 0, hdr, sel4(lane == 1 || slot_it, make_uint4(0, 0, 0, 0), cur));
    // an unused slot's sink line is scattered over MSNAP like the heads'
    // lines over MSNAPP: the partition's 1-KiB sink lines written in a row
    // made a batch without groups 7-9 us faster (DRAM page locality)
    const uint32_t sl = ((q * a.cm + (uint32_t)k) * a.sink_mul) % (a.Q * a.cm);
    uint4* dst = !listed && slot_it ? dry + 64 : real ? a.msnapp + (uint64_t)G.head * 64 : a.msnap + (uint64_t)sl * 64;
    st_drop(dst, lane, cur);
  };
  uint32_t ci = 0;  // the wave's chunk index
  for (uint32_t j0 = wave * kMU; j0 < a.Sr; j0 += 4 * kMU, ++ci) {
    if (j0 + 4 * kMU < a.Sr) load_rows(vb, part, j0 + 4 * kMU, a.Sr);
    uint4 v[kMU];
    uint32_t mm = 0;
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      v[u] = va[u];
      keep4(v[u]);  // every row is read, used or not
      mm |= (j0 + u < a.Sr && s_sg[j0 + u] >= 0) ? (1u << u) : 0u;
    }
    mm = __builtin_amdgcn_readfirstlane(mm);
    // the chunk's touched rows, then its share of the slot iterations
    const uint32_t nt = (uint32_t)__popc(mm), dlo = spread_lo(ci, nch, dn);
    const uint32_t nr = nt + spread_lo(ci + 1, nch, dn) - dlo;
    uint32_t mq = mm;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint32_t low = mq & (0u - mq);
      mq &= mq - 1u;
      step(v, low, j0, d0 + dlo + (r - nt));
    }
#pragma unroll
    for (int u = 0; u < kMU; ++u) va[u] = vb[u];
  }
  if (nch == 0) {  // a wave with no rows (partitions under 4 chunks): its slot iterations here
    uint4 v[kMU];
#pragma unroll
    for (int u = 0; u < kMU; ++u) v[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t r = 0; r < dn; ++r) step(v, 0u, 0u, d0 + r);
  }
}

// -------------------------------------------------------------- k_m1r
// copy-forward of the group snapshot; F = {reset, next-deletes, creates, 0}

struct M1rArgs {
  GVS_VSCAN_FIELDS
  const uint4* mpos;
  const OpState* ops;
  const uint4* msnapp;  // B x 1 KiB: group snapshots at their heads' positions
  const uint4* mpid;    // B x 16 B: each position's message id (k_gtx)
  M1Out* m1out;
  uint64_t N;
  KeyCtx kc;
};

struct M1rOp {
  using Args = M1rArgs;
  static constexpr bool kSelect = true;
  // the block's 64 MPOS records read once, one whole line per load instruction
  // (8 lanes each; a 16-B record loaded by itself fetched its line whole or in
  // halves depending on timing: FETCH_SIZE moved with the mix)
  static constexpr bool kStash = true;
  __device__ static uint4 rec_line(const Args& a, uint64_t i) {
    return (i & 7u) == 0u ? a.mpos[i >> 3] : make_uint4(0, 0, 0, 0);
  }
  __device__ static uint4 f_of_rec(const uint4* r) { return f_of_pos(uni4(r[0]).x); }
  __device__ static uint4 f_identity() { return make_uint4(0, 0, 0, 0); }
  __device__ static uint4 f_combine(uint4 a, uint4 b) {
    return sel4(b.x != 0u, b, make_uint4(a.x, a.y + b.y, a.z + b.z, 0u));
  }
  __device__ static bool takes_b(uint4, uint4 b) { return b.x != 0u; }
  __device__ static uint4 v_combine(uint4, uint4 va, uint4 fb, uint4 vb) { return sel4(fb.x != 0u, vb, va); }
  __device__ static uint4 f_of_pos(uint32_t x) {
    const bool null = x & kMPosNull, head = x & kMPosHead;
    const uint32_t cls = mpos_cls(x);
    return make_uint4((head || null) ? 1u : 0u, (!null && cls == 0u && mpos_sub(x)) ? 1u : 0u,
                      (!null && cls == 1u) ? 1u : 0u, 0u);
  }
  __device__ static uint4 f_of(const Args& a, uint32_t p) { return f_of_pos(uni4(a.mpos[p]).x); }
  // every op reads its own position's line (heads find their group's
  // snapshot there; the others' lines are read and ignored)
  __device__ static const uint4* src_of(const Args& a, uint32_t p, uint4) {
    return a.msnapp + (uint64_t)p * 64;
  }
  // k_vscan_a: every op's line is read, the defining op's kept
  __device__ static uint4 elem_value(const Args& a, uint32_t p, const uint4*) {
    return ld_row<false>(&src_of(a, p, make_uint4(0, 0, 0, 0))[lane_id()]);
  }
  __device__ static uint4 value_fin(uint4, uint4 v) { return v; }
};

__global__ __launch_bounds__(256) void k_m1r_c(M1rArgs a) {
  __shared__ uint4 s_v[4][64];
  __shared__ uint4 s_f[4];
  if (a.scal->error) return;
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t p0 = blockIdx.x * kVBlk + wave * 16;
  // the wave's 16 MPOS records in one load (two whole lines), op j's to every
  // lane by a shuffle; each op's own MSNAPP line, read once
  const uint4 mp_l = a.mpos[p0 + (lane & 15u)];
  // the 16 ops' ids by position (k_gtx copied them there from the OpStates it
  // reads anyway): read by seq here, the OpState lines came in the sort's
  // order, and runs of ascending seqs under the hot and all-miss mixes made
  // the kernel 3 us faster (profiles/r04z_timing_c3_store.txt)
  const uint4 id_l = a.mpid[p0 + (lane & 15u)];
  uint4 As[16];
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint4 mp = uni4(shfl4(mp_l, (int)j));
    As[j] = ld_row<false>(&M1rOp::src_of(a, p0 + j, mp)[lane]);
  }
  uint4 cf, cv;
  {  // the wave's aggregate from registers, then the carry
    uint4 f = M1rOp::f_identity(), v = As[0];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const uint4 e = M1rOp::f_of_pos(uni4(shfl4(mp_l, (int)j)).x);
      v = sel4(M1rOp::takes_b(f, e), As[j], v);
      f = M1rOp::f_combine(f, e);
    }
    vscan_carry_tail<M1rOp>(a, s_v, s_f, f, v, cf, cv);
  }
  // Pass 1, op by op (the carry is sequential): everything but the id decode.
  // Lane j keeps op j's result words and the id it must decode.
  uint4 my_idv = make_uint4(0, 0, 0, 0), my_w = make_uint4(0, 0, 0, 0), my_oid = my_idv;
  uint32_t my_need = 0;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint4 mp = uni4(shfl4(mp_l, (int)j));
    const uint32_t seq = mp.x & kSeqMask, cls = mpos_cls(mp.x);
    const bool head = mp.x & kMPosHead, null = mp.x & kMPosNull;
    const uint4 A = As[j];
    const uint4 myid = uni4(shfl4(id_l, (int)j));
    const uint4 pf = sel4(head, make_uint4(1u, 0u, 0u, 0u), cf);
    const uint4 pv = sel4(head, A, cv);
    const uint4 hdr = uni4(shfl4(pv, 0));
    const uint32_t len = hdr.x, fl = hdr.y, gflags = hdr.z;
    // next-message op: the one with d delete-nexts before it reads id d
    const uint32_t d = pf.y;
    const uint4 idv = shfl4(pv, 2 + (int)min(d, 61u));
    const bool found = !null && d < len;
    // create: rank r among the group's creates (grapevine.proto:73-75)
    const uint32_t r = pf.z;
    const bool exists1 = gflags & 1u, admitted = gflags & 2u;
    const bool cok = exists1 ? (fl + r < GVS_MAILBOX_SLOTS) : (admitted && r < GVS_MAILBOX_SLOTS);
    // by-id delete: the position of its id in the mailbox (for the write pass)
    const uint64_t hit = __ballot(lane >= 2 && lane < 2 + len && eq4(pv, myid));
    const uint32_t pos = hit ? (uint32_t)__builtin_ctzll(hit) - 2u : 63u;
    // selects, no branch over the op class (null ops sort last: a wave of
    // them would skip the code, and instruction fetch shows in FETCH_SIZE)
    const bool c0 = !null && cls == 0u, c1 = !null && cls == 1u, c2 = !null && cls > 1u;
    const uint32_t st1 = selu32(cok, kPending, selu32(exists1 || admitted, 5u, 6u));
    const uint32_t status = selu32(c0, selu32(found, kPending, 2u), selu32(c1, st1, kPending));
    const uint32_t flags = selu32(c0 && found && mpos_sub(mp.x), CF_POP, selu32(c1 && cok, CF_MBOX_OK, 0u));
    const uint32_t opos = selu32(c2, pos, 63u);
    const bool mine = lane == j;
    my_idv = sel4(mine, idv, my_idv);
    my_oid = sel4(mine, sel4(c0 && found, idv, make_uint4(0, 0, 0, 0)), my_oid);
    my_w = sel4(mine, make_uint4(status, seq, flags, opos), my_w);
    my_need = selu32(mine, (c0 && found) ? 1u : 0u, my_need);
    const uint4 e = M1rOp::f_of_pos(mp.x);
    cv = M1rOp::v_combine(cf, cv, e, A);
    cf = M1rOp::f_combine(cf, e);
  }
  // Pass 2: the 16 id decodes at once, one per lane (every lane decodes:
  // fixed work), then the records in op order.
  const uint32_t my_dec = id_decode(a.kc, u4lo(my_idv), u4hi(my_idv), a.N);
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint4 w = uni4(shfl4(my_w, (int)j));
    const uint4 oid = shfl4(my_oid, (int)j);
    const uint32_t dec = __shfl(my_dec, (int)j), need = __shfl(my_need, (int)j);
    const uint32_t slot = selu32(need != 0u, dec, kNone);
    if (lane < 8)
      st_drop(a.m1out, (uint64_t)w.y * 8 + lane,
              sel4(lane == 0, make_uint4(w.x, slot, w.z, w.w), sel4(lane == 1, oid, make_uint4(0, 0, 0, 0))));
  }
}

// -------------------------------------------------------------- k_m2r
// per group: the new ids of its successful creates at lane 2 + rank and the
// mailbox positions its successful by-id deletes remove.  F = {reset, mask lo,
// mask hi, creates}; values merge lane-wise (ids are never zero).

struct M2rArgs {
  GVS_VSCAN_FIELDS
  const uint4* mpos;
  const OpState* ops;
  const ROp* rop;
  const RRes* rres;
  const M1Out* m1out;
  uint4* m2tx;  // (Q*cm + B) x 1152 B
  uint32_t Q, cm, stamp;
  uint4* m2g;   // B x 128 B by position (k_m2g): F, appended id, recipient key
};

struct M2rOp {
  using Args = M2rArgs;
  static constexpr bool kSelect = false;
  // phase A reads each position's M2G line once, whole (k_m2g puts MPOS.w,
  // the create rank, in word 4)
  static constexpr bool kStash = true;
  __device__ static uint4 rec_line(const Args& a, uint64_t i) { return a.m2g[i]; }
  __device__ static uint4 f_of_rec(const uint4* r) { return uni4(r[0]); }
  __device__ static uint4 value_of_rec(const uint4* r, uint4 e) {
    const uint32_t rank = uni4(r[4]).x;
    return sel4(e.w != 0u && lane_id() == 2u + rank && rank < GVS_MAILBOX_SLOTS, r[1], make_uint4(0, 0, 0, 0));
  }
  __device__ static uint4 f_identity() { return make_uint4(0, 0, 0, 0); }
  __device__ static uint4 f_combine(uint4 a, uint4 b) {
    return sel4(b.x != 0u, b, make_uint4(a.x, a.y | b.y, a.z | b.z, a.w + b.w));
  }
  __device__ static bool takes_b(uint4, uint4 b) { return b.x != 0u; }
  __device__ static uint4 v_combine(uint4, uint4 va, uint4 fb, uint4 vb) {
    return sel4(fb.x != 0u || nz4(vb), vb, va);
  }
  // the element flags from the op's gathered lines (k_m2g)
  __device__ static uint4 f_from(uint32_t mpx, uint32_t status, uint32_t pos) {
    const uint32_t cls = mpos_cls(mpx);
    const bool null = mpx & kMPosNull, head = mpx & kMPosHead;
    const bool succ = status == 1u;
    const bool del = !null && cls == 2u && succ && pos < GVS_MAILBOX_SLOTS;
    return make_uint4((head || null) ? 1u : 0u, (del && pos < 32u) ? 1u << pos : 0u,
                      (del && pos >= 32u) ? 1u << (pos - 32u) : 0u, (!null && cls == 1u && succ) ? 1u : 0u);
  }
  __device__ static uint4 f_of(const Args& a, uint32_t p) { return uni4(a.m2g[(uint64_t)p * 8]); }
  __device__ static uint4 value_of(const Args& a, uint32_t p, uint4 e) {
    const uint4 mp = uni4(a.mpos[p]);
    const uint4 id = a.m2g[(uint64_t)p * 8 + 1];
    return sel4(e.w != 0u && lane_id() == 2u + mp.w && mp.w < GVS_MAILBOX_SLOTS, id, make_uint4(0, 0, 0, 0));
  }
};

// Gather, once per batch, each sorted position's lines (RRes, M1Out, ROp,
// OpState) into a position-indexed 128-B record: {F, appended id, recipient
// key x[0..3], x[4..7]}.  The scans and k_m2r_c read only these records
// (addresses that do not depend on the data).
__global__ __launch_bounds__(256) void k_m2g(M2rArgs a) {
  __shared__ uint4 stage[4 * 64 * 8];
  if (a.scal->error) return;
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  uint4* st = stage + (threadIdx.x >> 6) * 64 * 8;
  const uint4 mp4 = a.mpos[p];
  const uint32_t mpx = mp4.x, seq = mpx & kSeqMask;
  uint4 l[8], rec[8];
  wave_load128(st, reinterpret_cast<const uint4*>(a.rres + seq), l);
  const uint32_t status = l[0].x;
  wave_load128(st, reinterpret_cast<const uint4*>(a.m1out + seq), l);
  const uint32_t pos = l[0].w;
  wave_load128(st, reinterpret_cast<const uint4*>(a.rop + seq), l);
  rec[0] = M2rOp::f_from(mpx, status, pos);
  rec[1] = l[1];  // ROp id
  wave_load128(st, reinterpret_cast<const uint4*>(a.ops + seq), l);
  const uint32_t* ow = reinterpret_cast<const uint32_t*>(l);  // OpState: x is words 14..21
  rec[2] = make_uint4(ow[14], ow[15], ow[16], ow[17]);
  rec[3] = make_uint4(ow[18], ow[19], ow[20], ow[21]);
  rec[4] = make_uint4(mp4.w, 0, 0, 0);  // the op's rank among its group's creates
#pragma unroll
  for (int i = 5; i < 8; ++i) rec[i] = make_uint4(0, 0, 0, 0);
  wave_store128(st, a.m2g, p, rec);
}

__global__ __launch_bounds__(256) void k_m2r_c(M2rArgs a) {
  __shared__ uint4 s_v[4][64];
  __shared__ uint4 s_f[4];
  if (a.scal->error) return;
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t p0 = blockIdx.x * kVBlk + wave * 16;
  // the wave's 16 MPOS records and 16 M2G lines, each line read whole by one
  // load instruction (records handed to every lane by shuffles), read once:
  // the wave's aggregate comes from them too
  const uint4 mp_l = a.mpos[p0 + (lane & 15u)];
  const uint4 g_lo = a.m2g[(uint64_t)p0 * 8 + lane], g_hi = a.m2g[(uint64_t)p0 * 8 + 64 + lane];
  uint4 cf, cv;
  {
    uint4 f = M2rOp::f_identity(), v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const uint4 gl = j < 8 ? g_lo : g_hi;
      const int gb = (int)(j & 7u) * 8;
      const uint4 e = uni4(shfl4(gl, gb));
      const uint32_t rank = uni4(shfl4(mp_l, (int)j)).w;
      const uint4 id = shfl4(gl, gb + 1);
      v = M2rOp::v_combine(f, v, e, sel4(e.w != 0u && lane == 2u + rank && rank < GVS_MAILBOX_SLOTS, id,
                                         make_uint4(0, 0, 0, 0)));
      f = M2rOp::f_combine(f, e);
    }
    vscan_carry_tail<M2rOp>(a, s_v, s_f, f, v, cf, cv);
  }
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t p = p0 + j;
    const uint4 mp = uni4(shfl4(mp_l, (int)j));
    const bool last = (mp.x & kMPosLast) && !(mp.x & kMPosNull);
    const uint4 gl = j < 8 ? g_lo : g_hi;
    const int gb = (int)(j & 7u) * 8;
    const uint4 e = uni4(shfl4(gl, gb));
    const uint4 id = shfl4(gl, gb + 1);
    const uint4 val = sel4(e.w != 0u && lane == 2u + mp.w && mp.w < GVS_MAILBOX_SLOTS, id, make_uint4(0, 0, 0, 0));
    cv = M2rOp::v_combine(cf, cv, e, val);
    cf = M2rOp::f_combine(cf, e);
    // the group's last op writes its result slot, every other op a dummy
    const uint4 x0 = shfl4(gl, gb + 2), x1 = shfl4(gl, gb + 3);
    const uint64_t o = (last ? (uint64_t)mp.y : (uint64_t)a.Q * a.cm + p) * kVLineU4;
    // value: lanes 0..1 the recipient key (a new mailbox's first 32 B), lanes
    // 2.. the appended ids; header: stamp, creates, removal mask
    st_drop(a.m2tx, o + 8 + lane, sel4(lane == 0, x0, sel4(lane == 1, x1, cv)));
    if (lane < 8) st_drop(a.m2tx, o + lane, sel4(lane == 0, make_uint4(a.stamp, cf.w, cf.y, cf.z), make_uint4(0, 0, 0, 0)));
  }
}

// --------------------------------------------------------------- k_m2x

// new state of a mailbox row: matched rows drop their first dp ids and the
// ids at the positions of `mask`, then take the appended ids; a row placed
// for a new recipient takes the recipient key and the appended ids
__device__ inline uint4 m2_row(uint4 v, bool matched, uint32_t len, uint32_t dp, uint64_t mask,
                               uint32_t n_succ, uint4 app, uint4* wst, uint32_t* fl_out) {
  const uint32_t lane = lane_id();
  const uint32_t i = lane - 2u;
  const bool keep = matched && lane >= 2 && i < len && i >= dp && !((mask >> i) & 1ull);
  const uint64_t km = __ballot(keep);
  const uint32_t nk = (uint32_t)__popcll(km);
  // compaction through the wave's LDS stage: survivors at [0, nk), every
  // other lane after them (all lanes store: the same code runs whatever the
  // row holds, and instruction fetch shows in FETCH_SIZE)
  wst[keep ? mbcnt64(km) : nk + mbcnt64(~km)] = v;
  wave_lds_sync();
  const uint32_t r = lane - 2u;
  const uint4 w = wst[min(r, 63u)];
  uint4 out = sel4(lane >= 2 && r < nk, w, make_uint4(0, 0, 0, 0));
  const uint32_t ra = lane - 2u - nk;  // appended ids follow the survivors
  const uint4 a = shfl4(app, (int)(2u + min(ra, 61u)));
  out = sel4(lane >= 2 + nk && ra < n_succ && lane < 64, a, out);
  wave_lds_sync();
  const uint32_t fl = nk + min(n_succ, GVS_MAILBOX_SLOTS - nk);
  out = sel4(lane < 2, sel4(matched, v, app), out);  // recipient key
  *fl_out = fl;
  return sel4(fl != 0u, out, make_uint4(0, 0, 0, 0));
}

template <bool AUTH>
__global__ __launch_bounds__(256) void k_m2x(MArgs a) {
  static_assert(!AUTH, "sealed stores run k_m2a (gvs_mauth.h)");
  // dynamic LDS sized at launch: (plain) the partition's Sr side entries as
  // the prepass read them, then the group slots and the sink, cm + 1 entries
  // (9 KiB at C3 instead of 33): more workgroups per CU.  The side entries are
  // read from HBM once: read again in the row stream, their lines were
  // fetched twice or once depending on what the stream had evicted meanwhile,
  // i.e. on the batch's timing (FETCH_SIZE -16 KiB under hot and all-miss
  // mixes, profiles/r04x_m2x_read_counters.txt)
  extern __shared__ uint4 s_dyn[];
  uint4* s_side = s_dyn;
  GroupM* g = reinterpret_cast<GroupM*>(s_dyn + a.Sr);
  __shared__ int16_t s_sg[kSrMax];
  __shared__ uint8_t s_occb[kSrMax];
  __shared__ uint4 s_wst[4][64];
  __shared__ int16_t s_place[kSrMax];
  __shared__ uint8_t s_flag[kSrMax];
  __shared__ uint16_t s_pfx[kSrMax + 1];
  __shared__ uint16_t s_gpfx[kGroupMax + 1];
  __shared__ uint8_t s_gflag[kGroupMax + 1];
  __shared__ int16_t s_pend[kGroupMax + 1];
  __shared__ uint8_t s_ld[kGroupMax + 1];
  __shared__ uint32_t s_w[4], s_ng, s_occ, s_delta, s_tw[kRowWaves];
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = blockIdx.x;
  if (a.scal->error) return;
  uint4* part = a.mbox + (uint64_t)q * a.Sr * 64;
  uint4* side = a.side + (uint64_t)q * a.Sr;
  uint4 va[kMU], vb[kMU];
  load_rows(va, part, wave * kMU, a.Sr);
  const uint32_t ng = load_groups(a, q, g, &s_ng, true);
  if (tid == 0) {
    s_occ = 0;
    s_delta = 0;
  }
  __syncthreads();
  side_prepass_m(a, q, g, ng, s_sg, s_occb, &s_occ, s_side);
  __syncthreads();
  // final lengths; pending = groups with no row that end non-empty
  for (uint32_t k = tid; k < a.cm; k += 256) {
    GroupM& G = g[k];
    const bool real = k < ng;
    const GroupFields f = group_fields(G);
    const uint32_t len = selu32(real & ((int32_t)f.slot >= 0), f.len, 0u);
    const uint32_t dp = min(G.n_del, len);
    const uint64_t lenmask = len >= 64 ? ~0ull : ((1ull << len) - 1ull);
    const uint64_t mask = (((uint64_t)G.mhi << 32) | G.mlo) & lenmask & ~((1ull << dp) - 1ull);
    const uint32_t nk = len - dp - (uint32_t)__popcll(mask);
    G.fl = selu32(real, nk + min(G.n_succ, GVS_MAILBOX_SLOTS - nk), 0u);
    s_gflag[k] = (real & ((int32_t)f.slot < 0) & (G.fl > 0)) ? 1 : 0;
    s_ld[k] = 0;
  }
  __syncthreads();
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int k = s_sg[j];
    const bool occ = s_occb[j] != 0;
    s_flag[j] = (!occ || (k >= 0 && g[k].fl == 0)) ? 1 : 0;
  }
  __syncthreads();
  block_flag_scan(s_flag, a.Sr, s_pfx, s_w);
  block_flag_scan(s_gflag, a.cm, s_gpfx, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)  // groups not pending write the sink entry
    s_pend[s_gflag[k] ? s_gpfx[k] : (uint32_t)kGroupMax] = (int16_t)k;
  __syncthreads();
  const uint32_t npend = s_gpfx[a.cm];
  if (tid == 0 && npend > s_pfx[a.Sr]) atomicOr(&a.scal->error, 2u);
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int16_t cand = s_pend[min((uint32_t)s_pfx[j], (uint32_t)kGroupMax)];
    s_place[j] = (s_flag[j] && s_pfx[j] < npend) ? cand : (int16_t)-1;
    const int k = s_sg[j];
    atomicSub(&s_delta, (k >= 0 && g[k >= 0 ? k : 0].fl == 0) ? 1u : 0u);
  }
  if (tid == 0) atomicAdd(&s_delta, npend);
  if (tid < kRowWaves) s_tw[tid] = 0;
  __syncthreads();
  // the slot each touched row takes (a new recipient placed in it, else the
  // row's own group), and each wave's touched rows (chunk j / kMU of the
  // partition is streamed by wave (j / kMU) % 4)
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int k = s_sg[j], pl = s_place[j];
    const int ge = pl >= 0 ? pl : k;
    s_ld[ge >= 0 ? (uint32_t)ge : (uint32_t)kGroupMax] = 1;
    atomicAdd(&s_tw[(j / kMU) % kRowWaves], ge >= 0 ? 1u : 0u);
  }
  __syncthreads();
  // the slots no row takes, listed: each is read once, by a slot iteration
  for (uint32_t k = tid; k < a.cm; k += 256) s_gflag[k] = s_ld[k] ? 0 : 1;
  __syncthreads();
  block_flag_scan(s_gflag, a.cm, s_gpfx, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)
    if (s_gflag[k]) s_pend[s_gpfx[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t nfree = s_gpfx[a.cm];
  uint32_t d0, dn;
  slot_share(s_tw, a.cm, wave, &d0, &dn);
  const uint32_t nch = a.Sr > wave * kMU ? (a.Sr - wave * kMU + 4 * kMU - 1) / (4 * kMU) : 0u;
  const uint4* res = a.m2tx + (uint64_t)q * a.cm * kVLineU4;
  // the workgroup's dry block: k_m1x writes its first 4 KiB; slot iterations
  // past the list read 1 KiB lines 4..7 (no line is read twice in a kernel)
  const uint4* dry = a.mdry + (uint64_t)q * kMDryU4 + 256;
  uint4* wst = s_wst[wave];
  // one iteration: a touched row (bit set: its row in v is replaced) or a
  // slot no row takes (bit 0: the same work, nothing kept)
  // mine: lane u < kMU holds row u's side entry
  auto step = [&](uint4 (&v)[kMU], uint4& mine, uint32_t bit, uint32_t j0, uint32_t di) {
    const bool slot_it = bit == 0u;
    uint4 cur = v[0];
#pragma unroll
    for (int uu = 1; uu < kMU; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
    const uint32_t j = j0 + ((uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u);
    const bool listed = slot_it && di < nfree;
    const int k = slot_it ? -1 : s_sg[j], pl = slot_it ? -1 : s_place[j];
    const int ge = slot_it ? (listed ? (int)s_pend[di] : 0) : (pl >= 0 ? pl : k);
    const GroupM& G = g[ge >= 0 ? (uint32_t)ge : 0u];
    const uint4* rs = (slot_it && !listed) ? dry + 64u * min(di - nfree, 3u)
                                           : res + (uint64_t)(ge >= 0 ? ge : 0) * kVLineU4 + 8;
    const uint4 app = ld_row<true>(&rs[lane]);
    const bool matched = pl < 0;
    const uint32_t len = matched ? G.len : 0u;
    const uint32_t dp = min(G.n_del, len);
    const uint64_t mask = ((uint64_t)G.mhi << 32) | G.mlo;
    uint32_t fl;
    const uint4 nv = m2_row(cur, matched, len, dp, mask, G.n_succ, app, wst, &fl);
    const uint64_t w1 = (G.glo << 23) | ((uint64_t)fl << 1) | 1ull;
    const uint4 nsd = sel4(fl > 0, make_uint4((uint32_t)G.hi, (uint32_t)(G.hi >> 32), (uint32_t)w1,
                                              (uint32_t)(w1 >> 32)),
                           make_uint4(0, 0, 0, 0));
#pragma unroll
    for (int uu = 0; uu < kMU; ++uu) v[uu] = sel4((bit >> uu) & 1u, nv, v[uu]);  // a slot iteration has bit 0
    mine = sel4(bit != 0u && lane == ((uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u), nsd, mine);
  };
  uint32_t ci = 0;  // the wave's chunk index
  for (uint32_t j0 = wave * kMU; j0 < a.Sr; j0 += 4 * kMU, ++ci) {
    if (j0 + 4 * kMU < a.Sr) load_rows(vb, part, j0 + 4 * kMU, a.Sr);
    uint4 v[kMU];
    uint32_t mm = 0;
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      const bool in = j0 + u < a.Sr;  // wave-uniform
      v[u] = va[u];
      mm |= (in && (s_sg[j0 + u] >= 0 || s_place[j0 + u] >= 0)) ? (1u << u) : 0u;
    }
    // the chunk's side entries, one per lane u < kMU, as the prepass read them
    uint4 mine = (lane < (uint32_t)kMU && j0 + lane < a.Sr) ? s_side[j0 + lane] : make_uint4(0, 0, 0, 0);
    mm = __builtin_amdgcn_readfirstlane(mm);
    // the chunk's touched rows, then its share of the slot iterations
    const uint32_t nt = (uint32_t)__popc(mm), dlo = spread_lo(ci, nch, dn);
    const uint32_t nr = nt + spread_lo(ci + 1, nch, dn) - dlo;
    uint32_t mq = mm;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint32_t low = mq & (0u - mq);
      mq &= mq - 1u;
      step(v, mine, low, j0, d0 + dlo + (r - nt));
    }
    // the chunk's side entries: one store, kMU lanes (one whole line at kMU = 8;
    // eight 16-B stores of one line from one lane left partial lines behind)
    if (lane < (uint32_t)kMU && j0 + lane < a.Sr) side[j0 + lane] = mine;
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      if (j0 + u < a.Sr) st_stream(part, (uint64_t)(j0 + u) * 64 + lane, v[u]);
      va[u] = vb[u];
    }
  }
  if (nch == 0) {  // a wave with no rows (partitions under 4 chunks): its slot iterations here
    uint4 v[kMU], mine = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kMU; ++u) v[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t r = 0; r < dn; ++r) step(v, mine, 0u, 0u, d0 + r);
  }
  // every workgroup adds, zero included: a fixed set of atomics
  if (tid == 0)
    atomicAdd((unsigned long long*)&a.scal->n_mailboxes, (unsigned long long)(int64_t)(int32_t)s_delta);
}

// ------------------------------------------------------------- k_m21x
//
// The write pass of batch t and the read pass of batch t + 1 in one stream
// over the mailbox table (DESIGN.md §3 "Fused mailbox passes"): every row is
// read once, rewritten with batch t's results, stored, and then snapshotted
// for batch t + 1's groups, which saves k_m1x's 1-GiB read per batch.  The
// work per partition is exactly k_m2x's followed by k_m1x's, on the same
// fixed schedule (every row read and written once, T slot iterations per
// wave for each pass, one 1-KiB line per iteration).  Batch t + 1's read
// prologue needs the side entries after batch t: they follow from batch t's
// prologue (a touched row takes its group's key and final length, a row whose
// group ends empty is cleared), computed for every row into the side array in
// LDS before the stream; the stream stores the same values.
//
// w: batch t's write-pass arguments (its group descriptors and results),
// r: batch t + 1's read-pass arguments.  gerr: batch t + 1's group-slot
// overflow flag (its k_gtx scan runs before this kernel and must not stop
// batch t's write pass, whose status was already decided); the read pass of
// a failed batch t + 1 is skipped (its snapshots are never used).
#ifndef GVS_DIAG_M21
#define GVS_DIAG_M21 0  // diagnostic builds only: 1 = no slot iterations, 2 = prologues only
#endif

struct M21Args {
  MArgs w, r;
  const uint32_t* gerr;
};

__global__ __launch_bounds__(256) void k_m21x(M21Args A) {
  const MArgs& a = A.w;
  const MArgs& b = A.r;
  extern __shared__ uint4 s_dyn[];
  uint4* s_side = s_dyn;                                           // Sr
  GroupM* g = reinterpret_cast<GroupM*>(s_dyn + a.Sr);             // cm + 1: batch t
  GroupM* g1 = g + a.cm + 1;                                       // cm + 1: batch t + 1
  __shared__ int16_t s_sg[kSrMax];
  __shared__ uint8_t s_occb[kSrMax];
  __shared__ uint4 s_wst[4][64];
  __shared__ int16_t s_place[kSrMax];
  __shared__ uint8_t s_flag[kSrMax];
  __shared__ uint16_t s_pfx[kSrMax + 1];
  __shared__ uint16_t s_gpfx[kGroupMax + 1];
  __shared__ uint8_t s_gflag[kGroupMax + 1];
  __shared__ int16_t s_pend[kGroupMax + 1];
  __shared__ uint8_t s_ld[kGroupMax + 1];
  __shared__ uint32_t s_w[4], s_ng, s_occ, s_delta, s_tw[kRowWaves];
  // batch t + 1's read pass
  __shared__ int16_t s_sg1[kSrMax];
  __shared__ uint8_t s_occb1[kSrMax];
  __shared__ uint32_t s_ng1, s_occ1, s_empt1, s_tw1[kRowWaves];
  __shared__ uint8_t s_tf1[kGroupMax];
  __shared__ uint16_t s_tp1[kGroupMax + 1];
  __shared__ int16_t s_tl1[kGroupMax];
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = blockIdx.x;
  if (a.scal->error) return;  // batch t failed (multi-batch calls): neither pass runs
  const bool rd = *A.gerr == 0u;  // uniform: batch t + 1's read pass runs
  uint4* part = a.mbox + (uint64_t)q * a.Sr * 64;
  uint4* side = a.side + (uint64_t)q * a.Sr;
  uint4 va[kMU], vb[kMU];
  load_rows(va, part, wave * kMU, a.Sr);
  // ---- batch t's write prologue (k_m2x)
  const uint32_t ng = load_groups(a, q, g, &s_ng, true);
  if (tid == 0) {
    s_occ = 0;
    s_delta = 0;
  }
  __syncthreads();
  side_prepass_m(a, q, g, ng, s_sg, s_occb, &s_occ, s_side);
  __syncthreads();
  for (uint32_t k = tid; k < a.cm; k += 256) {
    GroupM& G = g[k];
    const bool real = k < ng;
    const GroupFields f = group_fields(G);
    const uint32_t len = selu32(real & ((int32_t)f.slot >= 0), f.len, 0u);
    const uint32_t dp = min(G.n_del, len);
    const uint64_t lenmask = len >= 64 ? ~0ull : ((1ull << len) - 1ull);
    const uint64_t mask = (((uint64_t)G.mhi << 32) | G.mlo) & lenmask & ~((1ull << dp) - 1ull);
    const uint32_t nk = len - dp - (uint32_t)__popcll(mask);
    G.fl = selu32(real, nk + min(G.n_succ, GVS_MAILBOX_SLOTS - nk), 0u);
    s_gflag[k] = (real & ((int32_t)f.slot < 0) & (G.fl > 0)) ? 1 : 0;
    s_ld[k] = 0;
  }
  __syncthreads();
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int k = s_sg[j];
    const bool occ = s_occb[j] != 0;
    s_flag[j] = (!occ || (k >= 0 && g[k].fl == 0)) ? 1 : 0;
  }
  __syncthreads();
  block_flag_scan(s_flag, a.Sr, s_pfx, s_w);
  block_flag_scan(s_gflag, a.cm, s_gpfx, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)
    s_pend[s_gflag[k] ? s_gpfx[k] : (uint32_t)kGroupMax] = (int16_t)k;
  __syncthreads();
  const uint32_t npend = s_gpfx[a.cm];
  if (tid == 0 && npend > s_pfx[a.Sr]) atomicOr(&a.scal->error, 2u);
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int16_t cand = s_pend[min((uint32_t)s_pfx[j], (uint32_t)kGroupMax)];
    s_place[j] = (s_flag[j] && s_pfx[j] < npend) ? cand : (int16_t)-1;
    const int k = s_sg[j];
    atomicSub(&s_delta, (k >= 0 && g[k >= 0 ? k : 0].fl == 0) ? 1u : 0u);
  }
  if (tid == 0) atomicAdd(&s_delta, npend);
  if (tid < kRowWaves) s_tw[tid] = 0;
  __syncthreads();
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int k = s_sg[j], pl = s_place[j];
    const int ge = pl >= 0 ? pl : k;
    s_ld[ge >= 0 ? (uint32_t)ge : (uint32_t)kGroupMax] = 1;
    atomicAdd(&s_tw[(j / kMU) % kRowWaves], ge >= 0 ? 1u : 0u);
  }
  __syncthreads();
  for (uint32_t k = tid; k < a.cm; k += 256) s_gflag[k] = s_ld[k] ? 0 : 1;
  __syncthreads();
  block_flag_scan(s_gflag, a.cm, s_gpfx, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)
    if (s_gflag[k]) s_pend[s_gpfx[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t nfree = s_gpfx[a.cm];
  // ---- the side entries after batch t, every row (what the stream stores):
  // a touched row its group's key and final length (cleared if it ends
  // empty), every other row as it was
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const int k = s_sg[j], pl = s_place[j];
    const int ge = pl >= 0 ? pl : k;
    const GroupM& G = g[ge >= 0 ? (uint32_t)ge : 0u];
    const uint32_t fl = G.fl;
    const uint64_t w1 = (G.glo << 23) | ((uint64_t)fl << 1) | 1ull;
    const uint4 nsd = sel4(fl > 0, make_uint4((uint32_t)G.hi, (uint32_t)(G.hi >> 32), (uint32_t)w1,
                                              (uint32_t)(w1 >> 32)),
                           make_uint4(0, 0, 0, 0));
    s_side[j] = sel4(ge >= 0, nsd, s_side[j]);
  }
  __syncthreads();
  // ---- batch t + 1's read prologue (k_m1x) on those side entries
  const uint32_t ng1 = load_groups(b, q, g1, &s_ng1, false);
  if (tid == 0) {
    s_occ1 = 0;
    s_empt1 = 0;
  }
  __syncthreads();
  side_prepass_m(b, q, g1, ng1, s_sg1, s_occb1, &s_occ1, nullptr, s_side);
  __syncthreads();
  count_empty(g1, ng1, b.cm, &s_empt1);
  __syncthreads();
  admit_groups(g1, ng1, b.cm, (b.Sr - s_occ1) + s_empt1);
  __syncthreads();
  if (tid < kRowWaves) s_tw1[tid] = 0;
  __syncthreads();
  for (uint32_t j = tid; j < b.Sr; j += 256) atomicAdd(&s_tw1[(j / kMU) % kRowWaves], s_sg1[j] >= 0 ? 1u : 0u);
  for (uint32_t k = tid; k < b.cm; k += 256)
    s_tf1[k] = ((k < ng1) & ((int32_t)group_fields(g1[k]).slot >= 0)) ? 0 : 1;
  __syncthreads();
  block_flag_scan(s_tf1, b.cm, s_tp1, s_w);
  for (uint32_t k = tid; k < b.cm; k += 256)
    if (s_tf1[k]) s_tl1[s_tp1[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t nfree1 = s_tp1[b.cm];
#if GVS_DIAG_M21 == 2
  return;  // diagnostic builds only: the prologues alone
#endif
  uint32_t d0, dn, e0, en;
  slot_share(s_tw, a.cm, wave, &d0, &dn);
  slot_share(s_tw1, b.cm, wave, &e0, &en);
  const uint32_t nch = a.Sr > wave * kMU ? (a.Sr - wave * kMU + 4 * kMU - 1) / (4 * kMU) : 0u;
  const uint4* res = a.m2tx + (uint64_t)q * a.cm * kVLineU4;
  // the dry block: the write pass reads 1 KiB lines 4..7 (k_m2x), the read
  // pass writes line 1 (k_m1x): no line read and written in one kernel
  uint4* dry = a.mdry + (uint64_t)q * kMDryU4;
  uint4* wst = s_wst[wave];
  // batch t's iteration (k_m2x's step)
  // the 1-KiB line an iteration appends from: its group's result line, or a
  // dry line past the list of slots no row takes
  auto app_src = [&](uint32_t bit, uint32_t j0, uint32_t di) -> const uint4* {
    const bool slot_it = bit == 0u;
    const uint32_t j = j0 + ((uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u);
    const bool listed = slot_it && di < nfree;
    const int k = slot_it ? -1 : s_sg[j], pl = slot_it ? -1 : s_place[j];
    const int ge = slot_it ? (listed ? (int)s_pend[di] : 0) : (pl >= 0 ? pl : k);
    return (slot_it && !listed) ? dry + 256 + 64u * min(di - nfree, 3u)
                                : res + (uint64_t)(ge >= 0 ? ge : 0) * kVLineU4 + 8;
  };
  auto step2 = [&](uint4 (&v)[kMU], uint4& mine, uint32_t bit, uint32_t j0, uint32_t di, uint4 app) {
    const bool slot_it = bit == 0u;
    uint4 cur = v[0];
#pragma unroll
    for (int uu = 1; uu < kMU; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
    const uint32_t j = j0 + ((uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u);
    const bool listed = slot_it && di < nfree;
    const int k = slot_it ? -1 : s_sg[j], pl = slot_it ? -1 : s_place[j];
    const int ge = slot_it ? (listed ? (int)s_pend[di] : 0) : (pl >= 0 ? pl : k);
    const GroupM& G = g[ge >= 0 ? (uint32_t)ge : 0u];
    const bool matched = pl < 0;
    const uint32_t len = matched ? G.len : 0u;
    const uint32_t dp = min(G.n_del, len);
    const uint64_t mask = ((uint64_t)G.mhi << 32) | G.mlo;
    uint32_t fl;
    const uint4 nv = m2_row(cur, matched, len, dp, mask, G.n_succ, app, wst, &fl);
    const uint64_t w1 = (G.glo << 23) | ((uint64_t)fl << 1) | 1ull;
    const uint4 nsd = sel4(fl > 0, make_uint4((uint32_t)G.hi, (uint32_t)(G.hi >> 32), (uint32_t)w1,
                                              (uint32_t)(w1 >> 32)),
                           make_uint4(0, 0, 0, 0));
#pragma unroll
    for (int uu = 0; uu < kMU; ++uu) v[uu] = sel4((bit >> uu) & 1u, nv, v[uu]);
    mine = sel4(bit != 0u && lane == ((uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u), nsd, mine);
  };
  // batch t + 1's iteration (k_m1x's step)
  auto step1 = [&](const uint4 (&v)[kMU], uint32_t bit, uint32_t j0, uint32_t di) {
    const bool slot_it = bit == 0u;
    uint4 cur = v[0];
#pragma unroll
    for (int uu = 1; uu < kMU; ++uu) cur = sel4((bit >> uu) & 1u, v[uu], cur);
    const uint32_t u0 = (uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u;
    const bool listed = slot_it && di < nfree1;
    const int k = slot_it ? (listed ? (int)s_tl1[di] : 0) : s_sg1[j0 + u0];
    const GroupM& G = g1[k >= 0 ? (uint32_t)k : 0u];
    const bool real = !slot_it || (listed && (uint32_t)k < ng1);
    const uint4 hdr = sel4(real, make_uint4(slot_it ? 0u : G.len, G.fl, G.flags, (uint32_t)G.slot),
                           make_uint4(0, 0, 0, 0));
    cur = sel4(lane == 0, hdr, sel4(lane == 1 || slot_it, make_uint4(0, 0, 0, 0), cur));
    const uint32_t sl = ((q * b.cm + (uint32_t)k) * b.sink_mul) % (b.Q * b.cm);
    uint4* dst = !listed && slot_it ? dry + 64 : real ? b.msnapp + (uint64_t)G.head * 64 : b.msnap + (uint64_t)sl * 64;
    st_drop(dst, lane, cur);
  };
  uint32_t ci = 0;
  for (uint32_t j0 = wave * kMU; j0 < a.Sr; j0 += 4 * kMU, ++ci) {
    if (j0 + 4 * kMU < a.Sr) load_rows(vb, part, j0 + 4 * kMU, a.Sr);
    uint4 v[kMU];
    uint32_t mm = 0, m1 = 0;
#pragma unroll
    for (int u = 0; u < kMU; ++u) {
      const bool in = j0 + u < a.Sr;  // wave-uniform
      v[u] = va[u];
      mm |= (in && (s_sg[j0 + u] >= 0 || s_place[j0 + u] >= 0)) ? (1u << u) : 0u;
    }
    uint4 mine = (lane < (uint32_t)kMU && j0 + lane < a.Sr) ? s_side[j0 + lane] : make_uint4(0, 0, 0, 0);
    mm = __builtin_amdgcn_readfirstlane(mm);
    const uint32_t nt = (uint32_t)__popc(mm), dlo = spread_lo(ci, nch, dn);
    const uint32_t nr = nt + spread_lo(ci + 1, nch, dn) - dlo;
    uint32_t mq = mm;
    for (uint32_t r = 0; r < (GVS_DIAG_M21 == 1 ? 0u : nr); ++r) {
      const uint32_t low = mq & (0u - mq);
      mq &= mq - 1u;
      const uint32_t di = d0 + dlo + (r - nt);
      step2(v, mine, low, j0, di, ld_row<true>(&app_src(low, j0, di)[lane]));
    }
    if (lane < (uint32_t)kMU && j0 + lane < a.Sr) side[j0 + lane] = mine;
#pragma unroll
    for (int u = 0; u < kMU; ++u)
      if (j0 + u < a.Sr) st_stream(part, (uint64_t)(j0 + u) * 64 + lane, v[u]);
    if (rd && GVS_DIAG_M21 != 1) {  // batch t + 1 on the rows as just written
#pragma unroll
      for (int u = 0; u < kMU; ++u) m1 |= (j0 + u < b.Sr && s_sg1[j0 + u] >= 0) ? (1u << u) : 0u;
      m1 = __builtin_amdgcn_readfirstlane(m1);
      const uint32_t nt1 = (uint32_t)__popc(m1), elo = spread_lo(ci, nch, en);
      const uint32_t nr1 = nt1 + spread_lo(ci + 1, nch, en) - elo;
      uint32_t mq1 = m1;
      for (uint32_t r = 0; r < nr1; ++r) {
        const uint32_t low = mq1 & (0u - mq1);
        mq1 &= mq1 - 1u;
        step1(v, low, j0, e0 + elo + (r - nt1));
      }
    }
#pragma unroll
    for (int u = 0; u < kMU; ++u) va[u] = vb[u];
  }
  if (nch == 0) {  // a wave with no rows: its slot iterations of both passes here
    uint4 v[kMU], mine = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kMU; ++u) v[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t r = 0; r < dn; ++r) step2(v, mine, 0u, 0u, d0 + r, ld_row<true>(&app_src(0u, 0u, d0 + r)[lane]));
    if (rd)
      for (uint32_t r = 0; r < en; ++r) step1(v, 0u, 0u, e0 + r);
  }
  if (tid == 0)
    atomicAdd((unsigned long long*)&a.scal->n_mailboxes, (unsigned long long)(int64_t)(int32_t)s_delta);
}

// after k_m21x: batch t + 1's group-slot overflow joins its error word, and
// the flag is cleared for the next batch
__global__ void k_err_fold(Scal* scal, uint32_t* gerr) {
  if (threadIdx.x == 0) {
    atomicOr(&scal->error, *gerr);
    *gerr = 0u;
  }
}

}  // namespace gvs
