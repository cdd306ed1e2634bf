// gvs_txn.h — fixed-slot transactions of the message-table pass.
//
// The message pass used to apply every op to its row inside the workgroup
// that owns the row's partition, so a workgroup's time grew with the ops
// routed to it (a hot message or recipient made one workgroup long: a timing
// leak, api/proto/grapevine.proto:120-122).  Here every piece of work has a
// fixed size:
//
//   k_rtx_{a,b,c}  over the R-sorted ops (row, class, seq): each row an op
//                  touches becomes ONE transaction slot of its partition (the
//                  segmented rank of the row's first op); a partition has c
//                  slots, more distinct rows is a batch overflow.  128-B slot
//                  descriptors T (this batch) are stamped with the run id.
//   k_rpass2       table pass, one workgroup per partition: streams all S rows,
//                  applies the PREVIOUS batch's final row states P (c slots)
//                  and snapshots this batch's rows (c slots of SNAP), reads
//                  and writes every slot of both whether used or not.
//   k_rr1_{a,b,c}  op-parallel: copy-forward of the row's identity along its
//                  segment (the row's pre-batch identity from the snapshot,
//                  the pop of a next-message DELETE, the record of a CREATE);
//                  statuses of next ops and creates, match of by-id ops.
//   k_rr2_{a,b,c}  op-parallel, one wave per op: copy-forward of the 1 KiB
//                  record along the segment (a DELETE freezes it empty, an
//                  UPDATE replaces it), every response, and the row's final
//                  state into P by the segment's last op.
//
// P is applied by the next batch's pass (deferred write-back): the table pass
// is the only kernel that touches table rows, every row exactly once.  Every
// op reads and writes the same bytes whatever its kind or outcome, and every
// per-position record is written by whole-line stores (DESIGN.md §3 rules).
#pragma once
#include "gvs_kernels.h"

namespace gvs {

constexpr uint32_t kScanT = 256;  // positions per block of the op scans (one thread each)
constexpr uint32_t kRErr = 16u;   // error bit: a partition's distinct rows exceed c

// -------------------------------------------------------------- utilities

// Store a 128-B record per lane (rec[0..7]) to base[idx] through the wave's
// LDS stage (64 x 128 B): every store instruction then writes 8 whole records,
// so no record line is ever left partially written (DESIGN.md §3 rule 2).
__device__ inline void wave_store128(uint4* stage, uint4* base, uint64_t idx, const uint4 (&rec)[8]) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int c = 0; c < 8; ++c) stage[lane * 8 + c] = rec[c];
  wave_lds_sync();
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const uint32_t r = (uint32_t)it * 8 + (lane >> 3), ch = lane & 7u;
    const uint64_t ix = shfl_u64(idx, (int)r);
    st_drop(base, ix * 8 + ch, stage[r * 8 + ch]);
  }
  wave_lds_sync();
}

// Gathers of per-op records (addresses that depend on the data) read whole
// 128-B lines, 8 lanes per line in one instruction.  A partial read of a line
// is fetched as 32- or 64-B sectors, how many depending on the other requests
// to that line in flight, which made FETCH_SIZE depend on the data.

// thread level: lane l gets the 128-B line at its own `src` in rec
__device__ inline void wave_load128(uint4* stage, const uint4* src, uint4 (&rec)[8]) {
  const uint32_t lane = lane_id();
  const uint64_t a = (uint64_t)src;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const uint32_t r = (uint32_t)it * 8 + (lane >> 3), ch = lane & 7u;
    const uint4* s = reinterpret_cast<const uint4*>(shfl_u64(a, (int)r));
    stage[r * 8 + ch] = s[ch];
  }
  wave_lds_sync();
#pragma unroll
  for (int c = 0; c < 8; ++c) rec[c] = stage[lane * 8 + c];
  wave_lds_sync();
}

// wave level: the line at a wave-uniform address, lane l holding its 16-B
// word l mod 8; line_u32 hands 32-bit word k (a constant) to every lane
__device__ inline uint4 line_load(const void* line) {
  return reinterpret_cast<const uint4*>(line)[lane_id() & 7u];
}
__device__ inline uint32_t line_u32(uint4 x, uint32_t k) {
  const uint32_t c = (k & 3u) == 0u ? x.x : (k & 3u) == 1u ? x.y : (k & 3u) == 2u ? x.z : x.w;
  return (uint32_t)__shfl((int)c, (int)(k >> 2));
}

// ---------------------------------------------------- generic op scans
//
// Three kernels over B positions, one thread per position: (a) block
// aggregates, (b) one workgroup scans the aggregates, (c) each position gets
// its exclusive prefix and emits.  Op supplies V, identity(), combine(a, b)
// (a precedes b; associative), local(args, p) and emit(args, p, excl, loc).
// Each phase reads every position's inputs once, whatever they hold.

template <class V>
__device__ inline void v_copy(V& d, const V& s) { d = s; }

// A block's values in LDS word-major: word k of element i at s[k * (kScanT +
// 1) + i], so that the 64 lanes of a wave touch 64 consecutive words (element-
// major, a value of 48 words put the lanes of one load on one bank group:
// Rr1V's scans ran 20-35 us).  kScanT + 1 elements: s[kScanT] is the identity,
// so that every step combines unconditionally (a branch around a struct
// assignment puts the struct in scratch).
template <class V>
constexpr uint32_t scan_words() {
  static_assert(sizeof(V) % 4 == 0, "scan values are whole words");
  return sizeof(V) / 4;
}
template <class V>
__device__ inline void lds_put(uint32_t* s, uint32_t i, const V& v) {
  uint32_t w[scan_words<V>()];
  __builtin_memcpy(w, &v, sizeof(V));
#pragma unroll
  for (uint32_t k = 0; k < scan_words<V>(); ++k) s[k * (kScanT + 1) + i] = w[k];
}
template <class V>
__device__ inline V lds_get(const uint32_t* s, uint32_t i) {
  uint32_t w[scan_words<V>()];
#pragma unroll
  for (uint32_t k = 0; k < scan_words<V>(); ++k) w[k] = s[k * (kScanT + 1) + i];
  V v;
  __builtin_memcpy(&v, w, sizeof(V));
  return v;
}
#define GVS_SCAN_LDS(V, name) __shared__ uint32_t name[(kScanT + 1) * scan_words<V>()]

// exclusive block scan; *total gets the block's total
template <class Op>
__device__ inline typename Op::V block_excl(const typename Op::V& x, uint32_t* s, typename Op::V* total = nullptr) {
  using V = typename Op::V;
  const uint32_t t = threadIdx.x;
  lds_put<V>(s, t, x);
  if (t == 0) lds_put<V>(s, kScanT, Op::identity());
  __syncthreads();
  for (uint32_t d = 1; d < kScanT; d <<= 1) {
    const V y = Op::combine(lds_get<V>(s, t >= d ? t - d : kScanT), lds_get<V>(s, t));
    __syncthreads();
    lds_put<V>(s, t, y);
    __syncthreads();
  }
  const V ex = lds_get<V>(s, t ? t - 1 : kScanT);
  if (total) *total = lds_get<V>(s, kScanT - 1);
  __syncthreads();
  return ex;
}

// Phase-B scans stop when the batch already failed (Op::stop): an abandoned
// batch must not overwrite the pending final states of the previous one.
template <class Op>
__global__ __launch_bounds__(kScanT) void k_scan_a(typename Op::Args a) {
  GVS_SCAN_LDS(typename Op::V, s);
  if (Op::stop(a)) return;
  __shared__ uint4 stage[4 * 64 * 8];  // per-wave record stage (wave_load128)
  const uint32_t p = blockIdx.x * kScanT + threadIdx.x;
  typename Op::V tot;
  block_excl<Op>(Op::local(a, p, stage + (threadIdx.x >> 6) * 64 * 8), s, &tot);
  if (threadIdx.x == 0) a.agg[blockIdx.x] = tot;
}

template <class Op>
__global__ __launch_bounds__(kScanT) void k_scan_b(typename Op::Args a) {
  using V = typename Op::V;
  GVS_SCAN_LDS(V, s);
  if (Op::stop(a)) return;
  const uint32_t t = threadIdx.x, nb = a.nblk;
  const uint32_t per = (nb + kScanT - 1) / kScanT, lo = min(nb, t * per), hi = min(nb, lo + per);
  V r = Op::identity();
  for (uint32_t i = lo; i < hi; ++i) r = Op::combine(r, a.agg[i]);
  V ex = block_excl<Op>(r, s);
  for (uint32_t i = lo; i < hi; ++i) {
    a.carry[i] = ex;
    ex = Op::combine(ex, a.agg[i]);
  }
}

template <class Op>
__global__ __launch_bounds__(kScanT) void k_scan_c(typename Op::Args a) {
  GVS_SCAN_LDS(typename Op::V, s);
  __shared__ uint4 stage[4 * 64 * 8];  // per-wave record stage (wave_store128)
  if (Op::stop(a)) return;
  const uint32_t p = blockIdx.x * kScanT + threadIdx.x;
  const typename Op::V loc = Op::local(a, p, stage + (threadIdx.x >> 6) * 64 * 8);
  typename Op::V ex = block_excl<Op>(loc, s);
  ex = Op::combine(a.carry[blockIdx.x], ex);
  Op::emit(a, p, ex, loc, stage + (threadIdx.x >> 6) * 64 * 8);
}

// ------------------------------------------------------------ k_rtx

// per sorted position: x = seq | head << 20 | last << 21 | null << 22,
// y = global slot w*c + k of the op's row (kNone for null ops), z = w, w = row
// offset in the partition
constexpr uint32_t kPosHead = 1u << 20, kPosLast = 1u << 21, kPosNull = 1u << 22;

struct RtxV {
  uint32_t reset;  // position starts a partition
  uint32_t cnt;    // row heads since the last partition start
  uint32_t hp;     // position of the latest row head (kNone: none yet)
  uint32_t pad;
};

struct RtxArgs {
  const uint64_t* rkeys;  // sorted
  uint4* rpos;            // B
  uint4* tbuf;            // 128-B records: this batch's slots (W*c), then B dummies
  RtxV* agg;
  RtxV* carry;
  Scal* scal;
  uint32_t B, W, S, c, nblk, stamp;
};

struct RtxOp {
  using V = RtxV;
  using Args = RtxArgs;
  // a batch that already failed (e.g. a slot overflow before its row keys
  // were written) stops here
  __device__ static bool stop(const Args& a) { return a.scal->error != 0u; }
  __device__ static V identity() { return V{0u, 0u, kNone, 0u}; }
  __device__ static V combine(const V& a, const V& b) {
    const uint32_t hp = b.hp != kNone ? b.hp : a.hp;
    return b.reset ? V{b.reset, b.cnt, hp, 0u} : V{a.reset, a.cnt + b.cnt, hp, 0u};
  }
  // 32-bit arithmetic and selects only: a 64-bit division expands to a branch
  // on the dividend's high word, and a branch around it for null rows would
  // skip code by the data (instruction fetch shows in FETCH_SIZE)
  __device__ static void row_of_key(const Args& a, uint64_t k, uint64_t& row, uint32_t& w) {
    const uint64_t n = (uint64_t)a.W * a.S;
    const bool valid = (k >> 22) < n;  // never index past the table
    const uint32_t r32 = valid ? (uint32_t)(k >> 22) : 0u;
    row = valid ? (uint64_t)r32 : kRNullRow;
    w = valid ? r32 / a.S : a.W;
  }
  // Every key this kernel needs is read from HBM once, in local() (before
  // any record is written): each lane its own, lane 0 the one before the
  // wave's and lane 63 the one after, the neighbours' by shuffles.  emit()
  // takes them from the wave's stage.  Read again in emit, after the slot
  // records (data-dependent destinations) had started to land, the key lines
  // hit or missed L2 by the batch (FETCH_SIZE +3-8 KiB under the hot mixes,
  // profiles/r04zd_oblivious_FETCH_SIZE_plain.txt).
  __device__ static V local(const Args& a, uint32_t p, uint4* st) {
    const uint32_t lane = lane_id();
    const uint64_t k = a.rkeys[p];
    uint64_t pk = shfl_u64(k, (int)(lane ? lane - 1u : 0u));
    uint64_t nk = shfl_u64(k, (int)min(lane + 1u, 63u));
    if (lane == 0u) pk = p ? a.rkeys[p - 1] : 0ull;
    if (lane == 63u) nk = p + 1 < a.B ? a.rkeys[p + 1] : 0ull;
    st[lane] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)nk, (uint32_t)(nk >> 32));
    uint64_t row, prow = ~0ull;
    uint32_t w, pw = ~0u;
    row_of_key(a, k, row, w);
    if (p) row_of_key(a, pk, prow, pw);
    const bool head = row != kRNullRow && (p == 0 || row != prow);
    return V{(uint32_t)(p == 0 || w != pw), head ? 1u : 0u, head ? p : kNone, 0u};
  }
  __device__ static void emit(const Args& a, uint32_t p, const V& ex, const V& loc, uint4* stage) {
    const uint4 kk4 = stage[lane_id()];
    const uint64_t key = ((uint64_t)kk4.y << 32) | kk4.x, nkey = ((uint64_t)kk4.w << 32) | kk4.z;
    uint64_t row, nrow = ~0ull;
    uint32_t w, nw;
    row_of_key(a, key, row, w);
    if (p + 1 < a.B) row_of_key(a, nkey, nrow, nw);
    const bool null = row == kRNullRow;
    const bool head = loc.cnt != 0u;
    const bool last = !null && (p + 1 == a.B || nrow != row);
    // heads before this position in its partition (the row's own head included
    // for non-heads)
    const uint32_t before = loc.reset ? 0u : ex.cnt;
    const uint32_t k = head ? before : before - 1u;
    if (head && k >= a.c) atomicOr(&a.scal->error, kRErr);
    const uint32_t kk = min(k, a.c - 1u);
    const uint32_t o = null ? 0u : (uint32_t)(row - (uint64_t)w * a.S);
    const uint32_t seq = (uint32_t)key & kSeqMask;
    a.rpos[p] = make_uint4(seq | (head ? kPosHead : 0u) | (last ? kPosLast : 0u) | (null ? kPosNull : 0u),
                           null ? kNone : w * a.c + kk, w, o);
    // the row's LAST op writes the slot descriptor: the row, the stamp, the
    // position whose final state (k_rr2_c) the next pass applies, and the
    // row's first op (the pass writes the row's snapshot at that position)
    const uint32_t hp = combine(ex, loc).hp;
    uint4 rec[8];
    rec[0] = make_uint4(o, a.stamp, p, hp);
#pragma unroll
    for (int i = 1; i < 8; ++i) rec[i] = make_uint4(0, 0, 0, 0);
    const uint64_t idx = last ? (uint64_t)w * a.c + kk : (uint64_t)a.W * a.c + p;
    wave_store128(stage, a.tbuf, idx, rec);
  }
};

// wave-uniform copy (lane 0's value in scalar registers)
__device__ inline uint4 uni4(uint4 x) {
  return make_uint4(__builtin_amdgcn_readfirstlane(x.x), __builtin_amdgcn_readfirstlane(x.y),
                    __builtin_amdgcn_readfirstlane(x.z), __builtin_amdgcn_readfirstlane(x.w));
}

// --------------------------------------------------------- k_rpass2

struct R2Args {
  uint4* table;        // N rows x 64 uint4, partition-major
  const uint4* tcur;   // this batch's slot descriptors (W*c records of 128 B)
  const uint4* tprev;  // the previous applied batch's
  uint32_t stamp_cur, stamp_prev;
  const uint4* ps;     // W*c x 1 KiB: the previous batch's final row states, by slot
                       // (every slot's line is read, used or not)
  const uint4* psds;   // AUTH: W*c x 128 B, their side entries {row lo, row hi, valid, slot}
  uint4* snap;         // W*c x 1 KiB: sink of the slots this batch does not use
  uint4* snapid;       // W*c x 128 B: the same for the identity lines
  uint4* snapp;        // B x 1 KiB: each touched row's snapshot at its first op's position
  uint4* snapidp;      // B x 128 B: its first line (identity), for k_rr1
  uint4* dry;          // W x 4 KiB: each workgroup's dry-run lines, one 1 KiB per use
                       // (merge read, snapshot write, identity write, side read): a line
                       // touched twice in one kernel hits or misses L2 by the timing
  Scal* scal;
  uint32_t W, S, c;
  // authenticated storage (AUTH instantiations)
  SealCtx sc;
  const uint32_t* te;
  uint4* mtag;
  // expiry sweep: on the rows as they stand before this batch
  uint32_t xon, xk, xrot, xep, xexcl;
  uint64_t cutoff;
  uint4* xbuf;         // records written by this pass
  const uint4* xprev;  // records being deleted by this batch (exclusion)
};

// Expiry detection on a chunk (v1 x_detect plus the exclusion of rows whose
// delete this batch already carries, lane 0 compares the row's id).
template <int U>
__device__ inline uint32_t x_detect2(const R2Args& a, const uint4 (&v)[U], uint4* buf, uint32_t xc,
                                     const uint4* s_xx, uint32_t nx) {
  const uint32_t lane = lane_id();
  const uint32_t part = lane == 0 ? 0u : lane - 2u;
  const bool writer = lane == 0 || lane == 3 || lane == 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t ts = ((uint64_t)v[u].y << 32) | v[u].x;
    bool ex = false;
    for (uint32_t k = 0; k < nx; ++k) ex |= eq4(v[u], s_xx[k]);
    const uint64_t m_old = __ballot(lane == 5 && ts < a.cutoff);
    const uint64_t m_msg = __ballot(lane == 0 && nz4(v[u]) && !ex);
    const uint32_t hit = (uint32_t)((m_old >> 5) & m_msg & 1ull);
    const uint32_t slot = min(xc, a.xep);
    if (writer) buf[slot * 3 + part] = v[u];
    xc += hit;
  }
  return xc;
}

template <int NW>
__device__ inline uint32_t x_merge2(uint32_t xep, const uint4* s_xw, const uint32_t* s_xc,
                                    uint4* s_xp, uint32_t tot) {
  const uint32_t tid = threadIdx.x, cap = xep;
  uint32_t add = 0;
  if (tid < 3 * cap) {
    const uint32_t k = tid / 3, c = tid % 3;
    uint32_t off = k - tot, src = kNone;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t cw = min(s_xc[w], cap);
      const bool take = k >= tot && src == kNone && off < cw;
      src = selu32(take, ((uint32_t)w * (kXepMax + 1) + off) * 3 + c, src);
      off -= cw;
    }
    if (src != kNone) s_xp[k * 3 + c] = s_xw[src];
  }
#pragma unroll
  for (int w = 0; w < NW; ++w) add += min(s_xc[w], cap);
  return min(tot + add, cap);
}

template <bool NTL>
__device__ inline uint4 ld_line(const uint4* p) { return ld_row<NTL>(p); }

constexpr uint32_t kSlotMax = 1024;      // transaction slots per partition (c) at most

// One chunk of U rows (partition row rj) of the plain message pass's
// fallback (more slots than k_rpass2s stages): apply the previous batch's
// final states, snapshot the rows this batch touches, expiry selection.
// Returns the expiry count.
//
// The first chunk of wave 0 (`first`) runs each loop once "dry" on the
// workgroup's own dry line, so every workgroup executes the same code whatever
// its slots hold (instruction fetch shows in FETCH_SIZE, DESIGN.md §3 rule 6).
// The dry iteration is an extra mask bit (1 << U), taken last by the same loop
// code: a loop whose first iteration were special could be peeled by the
// compiler, and then not every workgroup would fetch the loop's code.
template <int U>
__device__ inline uint32_t rpass_chunk_merge(const R2Args& a, uint4 (&v)[U], uint32_t rj, bool first,
                                             const int16_t* s_pk, const int16_t* s_sk, const uint32_t* s_sh,
                                             uint64_t sbase, uint4* dry, uint32_t xc, uint4* s_xw_w,
                                             const uint4* s_xx, uint32_t nx) {
  const uint32_t lane = lane_id();
  uint32_t mp = 0, ms = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    mp |= s_pk[rj + u] >= 0 ? (1u << u) : 0u;
    ms |= s_sk[rj + u] >= 0 ? (1u << u) : 0u;
  }
  mp = __builtin_amdgcn_readfirstlane(mp);
  ms = __builtin_amdgcn_readfirstlane(ms);
  uint32_t mq = mp | (first ? (1u << U) : 0u);
  while (mq) {  // rows the previous batch changed: its final state
    const uint32_t low = mq & (0u - mq);
    mq &= mq - 1u;
    const bool dry_p = low == (1u << U);
    const uint32_t bit = dry_p ? 0u : low;
    const uint32_t u0 = (uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u;
    const int16_t k = dry_p ? (int16_t)0 : s_pk[rj + u0];
    const uint4* src = dry_p ? dry : a.ps + (sbase + (uint64_t)k) * 64;
    const uint4 x = ld_row<true>(&src[lane]);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = sel4((bit >> u) & 1u, x, v[u]);
  }
  uint32_t sq = ms | (first ? (1u << U) : 0u);
  while (sq) {  // rows this batch touches: their snapshot
    const uint32_t low = sq & (0u - sq);
    sq &= sq - 1u;
    const bool dry_s = low == (1u << U);
    const uint32_t bit = dry_s ? 0u : low;
    const uint32_t u0 = (uint32_t)__builtin_ctz(bit | (1u << 31));
    const int16_t k = dry_s ? (int16_t)0 : s_sk[rj + (u0 & 31u)];
    uint4 cur = v[0];
#pragma unroll
    for (int u = 1; u < U; ++u) cur = sel4((bit >> u) & 1u, v[u], cur);
    // the snapshot goes to the position of the row's first op, so that
    // every op of the phase-C scans reads its own position's line
    const uint32_t hp = s_sh[(uint32_t)k & (kSlotMax - 1u)];
    uint4* dst = dry_s ? dry + 64 : a.snapp + (uint64_t)hp * 64;
    st_drop(dst, lane, cur);
    if (lane < 8) st_drop(dry_s ? dry + 2 * 64 : a.snapidp + (uint64_t)hp * 8, lane, cur);
  }
  if (a.xon) xc = x_detect2<U>(a, v, s_xw_w, xc, s_xx, nx);
  return xc;
}
constexpr uint32_t kPendTable = 0x100u;  // header table field of a row whose final state is pending

// Authenticated storage: a row the batch touches is sealed with the pending
// flag in its header, so the next pass must find its final state in P (a
// hidden P slot fails that row's tag); P rows are sealed as table 2, bound to
// their position and, through their side entry, to the row they replace.
// The sealed pass is k_spass (gvs_spass.h).

// The plain pass's fallback (c > kStageSlots or S not a multiple of the
// staged pass's rounds): NW waves per workgroup, 64 rows per wave per tile
// (tiles of 64 * NW rows; S must be a multiple), U rows per chunk, the slot
// lines read and written in the stream.
template <int U, bool NTL, bool NTS, int MINW, int NW = 4>
__global__ __launch_bounds__(64 * NW, MINW) void k_rpass2(R2Args a) {
  constexpr uint32_t kT = 64u * NW;  // rows per tile
  __shared__ int16_t s_pk[kRowsMax], s_sk[kRowsMax];
  __shared__ uint32_t s_sh[kSlotMax];  // this batch's slot -> position of the row's first op
  __shared__ uint32_t s_np, s_ns;
  __shared__ uint4 s_xw[NW * (kXepMax + 1) * 3];
  __shared__ uint4 s_xp[kXepMax * 3];
  __shared__ uint4 s_xx[kXepMax];
  __shared__ uint32_t s_xc[NW], s_xt;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t w = blockIdx.x;
  if (a.scal->error) return;
  for (uint32_t o = tid; o < a.S; o += kT) {
    s_pk[o] = -1;
    s_sk[o] = -1;
  }
  if (tid == 0) {
    s_np = 0;
    s_ns = 0;
    s_xt = 0;
  }
  __syncthreads();
  // every slot descriptor of this partition, both batches (fixed reads): a
  // record by 8 lanes, one whole line per load instruction (c is a multiple
  // of 8).  A 16-B load per record fetched each line as a partial request,
  // and how often the memory side merged those into whole-line reads
  // (TCC_BUBBLE, counted twice in FETCH_SIZE) followed the timing.
  const uint64_t sbase = (uint64_t)w * a.c;
  for (uint32_t k0 = wave * 8; k0 < a.c; k0 += NW * 8) {
    const uint32_t k = k0 + (lane >> 3);
    const uint4 xp = a.tprev[(sbase + k) * 8 + (lane & 7u)];
    const uint4 xc = a.tcur[(sbase + k) * 8 + (lane & 7u)];
    const uint4 dp = shfl4(xp, (int)(lane & ~7u)), ds = shfl4(xc, (int)(lane & ~7u));
    if ((lane & 7u) == 0u) {
      if (dp.y == a.stamp_prev && dp.x < a.S) {
        s_pk[dp.x] = (int16_t)k;
        atomicAdd(&s_np, 1u);
      }
      s_sh[k] = ds.w;
      if (ds.y == a.stamp_cur && ds.x < a.S) {
        s_sk[ds.x] = (int16_t)k;
        atomicAdd(&s_ns, 1u);
      }
    }
  }
  // the expiry deletes this batch already carries for this partition
  uint32_t nx = 0;
  if (a.xon && a.xexcl) {
    if (wave == 0) {  // the records as whole lines (8 lanes each), words 0 and 3 by shuffles
      const uint32_t kr = lane >> 3;
      const uint4 x = kr < a.xep ? a.xprev[((uint64_t)w * a.xep + kr) * 8 + (lane & 7u)] : make_uint4(0, 0, 0, 0);
      const uint4 r = shfl4(x, (int)(lane & ~7u)), vld = shfl4(x, (int)((lane & ~7u) + 3u));
      if ((lane & 7u) == 0u && kr < a.xep) s_xx[kr] = sel4(vld.x != 0u, r, make_uint4(0, 0, 0, 0));
    }
    nx = a.xep;
  }
  __syncthreads();
  const uint32_t np = s_np, ns = s_ns;
  const uint64_t rowbase = (uint64_t)w * a.S;
  uint4* part = a.table + rowbase * 64;
  uint4* sslot = a.snap + sbase * 64;
  uint4* dry = a.dry + (uint64_t)w * 256;
  const uint32_t tiles = a.S / kT;
  for (uint32_t t = 0; t < tiles; ++t) {
    uint32_t xc = 0;
    const uint32_t rb = t * kT + wave * 64;
    for (uint32_t j = 0; j < 64; j += U) {
      uint4 v[U];
      const uint32_t rj = rb + j;
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld_row<NTL>(&part[(uint64_t)(rj + u) * 64 + lane]);
      const bool first = t == 0 && j == 0 && wave == 0;
      xc = rpass_chunk_merge<U>(a, v, rj, first, s_pk, s_sk, s_sh, sbase, dry, xc,
                                s_xw + wave * (kXepMax + 1) * 3, s_xx, nx);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (NTS) st_stream(part, (uint64_t)(rj + u) * 64 + lane, v[u]);
        else st_row<NTS>(&part[(uint64_t)(rj + u) * 64 + lane], v[u]);
      }
    }
    // The waves meet after every tile, expiry or not: without the barrier they
    // drift apart and the plain pass runs 4-5% slower.  A barrier after every
    // chunk as well gains another 2%, but moves the pass's WRITE_SIZE with the
    // request mix by 90-135 KiB (profiles/r03n_pass_ab.txt): not taken.
    if (lane == 0) s_xc[wave] = xc;
    __syncthreads();
    if (a.xon) {
      const uint32_t tot = x_merge2<NW>(a.xep, s_xw, s_xc, s_xp, s_xt);
      __syncthreads();
      if (tid == 0) s_xt = tot;
    }
  }
  // unused slots (slots are dense from 0: [np, c) were not used by the
  // previous batch): every slot's final-state line is read once per pass
  for (uint32_t k = np + wave; k < a.c; k += NW) {
    uint4 x = ld_row<true>(&a.ps[(sbase + k) * 64 + lane]);
    keep4(x);
  }
  for (uint32_t k = ns + wave; k < a.c; k += NW) {
    st_drop(sslot, (uint64_t)k * 64 + lane, make_uint4(0, 0, 0, 0));
    if (lane < 8) st_drop(a.snapid, (sbase + k) * 8 + lane, make_uint4(0, 0, 0, 0));
  }
  if (a.xon && w % a.xk == a.xrot) {
    __syncthreads();
    if (wave == 0 && lane < 8 * a.xep) {
      const uint32_t k = lane >> 3, part8 = lane & 7;
      const bool valid = k < s_xt;
      uint4 val = make_uint4(part8 == 3 && valid ? 1u : 0u, 0, 0, 0);
      if (part8 < 3) val = sel4(valid, s_xp[k * 3 + part8], make_uint4(0, 0, 0, 0));
      a.xbuf[((uint64_t)(w / a.xk) * a.xep + k) * 8 + part8] = val;
    }
  }
}

// --------------------------------------------------------- k_rpass2s
//
// The plain table pass with a fixed memory schedule.  k_rpass2 reads a used
// slot's final state and writes a touched row's snapshot in the row stream,
// at the position of the row, so where those 1-KiB accesses fall among the
// row loads and stores followed the batch.  The memory side's request timing
// followed it too: FETCH_SIZE counts 128-B reads that arrived with a gap
// (TCC_BUBBLE) twice, and their number moved with the request mix by 3-6 K per
// launch (2^20 rows, profiles/r04_*).  Here a workgroup
//   (1) reads every slot's final state (c lines, used or not) into LDS,
//   (2) streams its rows: merges and snapshots go through LDS only,
//   (3) writes every slot's snapshot (c lines; unused slots to their sink),
// so the order and number of its HBM accesses depend on (S, c) only.  Up to
// kStageSlots slots (2 x 65 KiB of LDS: one workgroup of NW waves per CU).
constexpr uint32_t kStageSlots = 64;

// Every row of every chunk does the same LDS work, used or not (DESIGN.md §3
// rule 10): it reads a final state (its slot's, or the dry slot's, kept only
// for a row the previous batch changed) and writes its snapshot (to its
// slot, or to the dry slot).  Round 4 merged and snapshot only the touched
// rows, one LDS loop iteration each, and the pass's duration followed how
// many rows the batch touched (hot and all-miss mixes up to 19 us faster,
// profiles/r04zf_timing_c3_store.txt).
template <int U>
__device__ inline uint32_t stage_chunk(const R2Args& a, uint4 (&v)[U], uint32_t rj,
                                       const int16_t* s_pk, const int16_t* s_sk, const uint4* s_fin,
                                       uint4* s_snp, uint32_t xc, uint4* s_xw_w, const uint4* s_xx,
                                       uint32_t nx) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int u = 0; u < U; ++u) {  // rows the previous batch changed: their final state
    const int16_t k = s_pk[rj + u];
    const uint32_t b = selu32(k >= 0, (uint32_t)k, kStageSlots);
    v[u] = sel4(k >= 0, s_fin[b * 64 + lane], v[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {  // rows this batch touches: their snapshot
    const int16_t k = s_sk[rj + u];
    s_snp[selu32(k >= 0, (uint32_t)k, kStageSlots) * 64 + lane] = v[u];
  }
  if (a.xon) xc = x_detect2<U>(a, v, s_xw_w, xc, s_xx, nx);
  return xc;
}

// NW waves, chunks of U rows dealt round-robin (round r: wave w streams rows
// (r NW + w) U ..): S must be a multiple of U NW, c at most kStageSlots.
template <int U, int NW, bool NTL = true>
__global__ __launch_bounds__(64 * NW, 1) void k_rpass2s(R2Args a) {
  constexpr uint32_t kR = (uint32_t)U * NW;           // rows per round
  constexpr uint32_t kPer = kStageSlots / NW;          // slot lines per wave
  __shared__ int16_t s_pk[kRowsMax], s_sk[kRowsMax];
  __shared__ uint32_t s_sh[kStageSlots];
  __shared__ uint32_t s_np, s_ns, s_xt;
  __shared__ uint4 s_fin[(kStageSlots + 1) * 64];      // final states by slot (+ the dry slot)
  __shared__ uint4 s_snp[(kStageSlots + 1) * 64];      // snapshots by slot (+ the dry slot)
  __shared__ uint4 s_xw[NW * (kXepMax + 1) * 3];
  __shared__ uint4 s_xp[kXepMax * 3];
  __shared__ uint4 s_xx[kXepMax];
  __shared__ uint32_t s_xc[NW];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t w = blockIdx.x;
  if (a.scal->error) return;
  const uint64_t sbase = (uint64_t)w * a.c;
  // (1) every slot's final-state line, the wave's kPer loads in flight together
  uint4 fin[kPer];
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t k = wave + NW * i;
    fin[i] = k < a.c ? ld_row<true>(&a.ps[(sbase + k) * 64 + lane]) : make_uint4(0, 0, 0, 0);
  }
  for (uint32_t o = tid; o < a.S; o += 64 * NW) {
    s_pk[o] = -1;
    s_sk[o] = -1;
  }
  if (tid == 0) {
    s_np = 0;
    s_ns = 0;
    s_xt = 0;
  }
  __syncthreads();
  // slot descriptors of both batches, whole lines (k_rpass2)
  for (uint32_t k0 = wave * 8; k0 < a.c; k0 += NW * 8) {
    const uint32_t k = k0 + (lane >> 3);
    const uint4 xp = a.tprev[(sbase + k) * 8 + (lane & 7u)];
    const uint4 xc = a.tcur[(sbase + k) * 8 + (lane & 7u)];
    const uint4 dp = shfl4(xp, (int)(lane & ~7u)), ds = shfl4(xc, (int)(lane & ~7u));
    if ((lane & 7u) == 0u) {
      if (dp.y == a.stamp_prev && dp.x < a.S) {
        s_pk[dp.x] = (int16_t)k;
        atomicAdd(&s_np, 1u);
      }
      s_sh[k] = ds.w;
      if (ds.y == a.stamp_cur && ds.x < a.S) {
        s_sk[ds.x] = (int16_t)k;
        atomicAdd(&s_ns, 1u);
      }
    }
  }
  uint32_t nx = 0;
  if (a.xon && a.xexcl) {
    if (wave == 0) {
      const uint32_t kr = lane >> 3;
      const uint4 x = kr < a.xep ? a.xprev[((uint64_t)w * a.xep + kr) * 8 + (lane & 7u)] : make_uint4(0, 0, 0, 0);
      const uint4 r = shfl4(x, (int)(lane & ~7u)), vld = shfl4(x, (int)((lane & ~7u) + 3u));
      if ((lane & 7u) == 0u && kr < a.xep) s_xx[kr] = sel4(vld.x != 0u, r, make_uint4(0, 0, 0, 0));
    }
    nx = a.xep;
  }
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t k = wave + NW * i;
    if (k < a.c) s_fin[k * 64 + lane] = fin[i];
  }
  __syncthreads();
  const uint32_t ns = s_ns;
  // (2) the rows
  uint4* part = a.table + (uint64_t)w * a.S * 64;
  const uint32_t rounds = a.S / kR;
  for (uint32_t t = 0; t < rounds; ++t) {
    const uint32_t rj = t * kR + wave * U;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld_row<NTL>(&part[(uint64_t)(rj + u) * 64 + lane]);
    const uint32_t xc = stage_chunk<U>(a, v, rj, s_pk, s_sk, s_fin, s_snp, 0u,
                                       s_xw + wave * (kXepMax + 1) * 3, s_xx, nx);
#pragma unroll
    for (int u = 0; u < U; ++u) st_stream(part, (uint64_t)(rj + u) * 64 + lane, v[u]);
    if (lane == 0) s_xc[wave] = xc;
    __syncthreads();
    if (a.xon) {
      const uint32_t tot = x_merge2<NW>(a.xep, s_xw, s_xc, s_xp, s_xt);
      __syncthreads();
      if (tid == 0) s_xt = tot;
    }
  }
  __syncthreads();
  // (3) every slot's snapshot: the touched rows' to their first ops'
  // positions, the unused slots' (zero) to their sink lines
  uint4* sslot = a.snap + sbase * 64;
  for (uint32_t k = wave; k < a.c; k += NW) {
    const bool used = k < ns;
    const uint32_t hp = s_sh[k];
    const uint4 x = sel4(used, s_snp[k * 64 + lane], make_uint4(0, 0, 0, 0));
    st_drop(used ? a.snapp + (uint64_t)hp * 64 : sslot + (uint64_t)k * 64, lane, x);
    if (lane < 8) st_drop(used ? a.snapidp + (uint64_t)hp * 8 : a.snapid + (sbase + k) * 8, lane, x);
  }
  if (a.xon && w % a.xk == a.xrot) {
    __syncthreads();
    if (wave == 0 && lane < 8 * a.xep) {
      const uint32_t k = lane >> 3, part8 = lane & 7;
      const bool valid = k < s_xt;
      uint4 val = make_uint4(part8 == 3 && valid ? 1u : 0u, 0, 0, 0);
      if (part8 < 3) val = sel4(valid, s_xp[k * 3 + part8], make_uint4(0, 0, 0, 0));
      a.xbuf[((uint64_t)(w / a.xk) * a.xep + k) * 8 + part8] = val;
    }
  }
}

// ------------------------------------------------- P sealing (AUTH)
//
// P rows (final states by sorted position, B of them) are sealed as table 2
// at the epoch the pass writes (epoch + 1), their side entry (target row,
// valid) authenticated with them; the next batch unseals all B in place
// before its pass.  One wave per 16 positions; every position every batch.

struct PsealArgs {
  uint4* pbuf;   // B x 1 KiB
  uint4* psd;    // B side entries {row lo, row hi, valid (row's last op), slot}
  uint4* ptag;   // B tags
  SealCtx sc;
  const uint32_t* te;
  Scal* scal;
  uint32_t ep;   // epoch of the P rows (seal: written; unseal: read)
  uint4* ps;     // unseal: (W*c + B) x 1 KiB final states by slot (the pass reads every slot), then sinks
  uint4* psds;   // unseal: (W*c + B) x 128 B their side entries
  uint32_t nslots;  // W*c
};

template <bool SEAL>
__global__ __launch_bounds__(256) void k_pseal(PsealArgs a) {
  constexpr int U = 16;
  GVS_TE_LDS s_te[kTeWords];
  __shared__ uint4 s_st[4 * stage_u4(U)];
  if (a.scal->error) return;
  load_te(s_te, a.te);
  __syncthreads();
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  uint4* st = s_st + wave * stage_u4(U);
  const uint64_t p0 = ((uint64_t)blockIdx.x * 4 + wave) * U;
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld_row<true>(&a.pbuf[(p0 + u) * 64 + lane]);
  const uint4 ks = ctr_keystream(a.sc.rk, lds_te(s_te), 2u, p0 + (lane & 15u), a.ep, 64u);
  const uint4 sd = a.psd[(p0 + (lane & 15u)) * 8];
  const uint4 sct = SEAL ? xor4(sd, ks) : sd;  // side ciphertext
  if (lane < (uint32_t)U) st[U * 4 * kSegU4 + lane] = sct;
  wave_lds_sync();
  const uint32_t ur = (lane >> 2) % (uint32_t)U;
  const uint4 x = st[U * 4 * kSegU4 + ur];
  const uint64_t sdv[2] = {u4lo(x), u4hi(x)};
  uint64_t hdr[2];
  head_aes(a.sc.rkh, lds_te(s_te), p0 + ur, a.ep, 2u, sdv, hdr);  // table 2: its side ciphertext bound in
  bool ok = true;
  if (SEAL) {
    wave_seal<U, 8>(a.sc, s_te, 2u, p0, a.ep, v, a.ptag, true, st, hdr);
  } else {
    ok = wave_unseal<U, 8>(a.sc, s_te, 2u, p0, v, a.ptag, true, st, hdr);  // wave-uniform
    if (!ok && lane == 0) atomicOr(&a.scal->error, 8u);
  }
  if (SEAL) {
#pragma unroll
    for (int u = 0; u < U; ++u) st_drop(a.pbuf, (p0 + u) * 64 + lane, v[u]);
    if (lane < (uint32_t)U) st_drop(a.psd, (p0 + lane) * 8, sct);
  } else {
    // a row's last op's state goes to its slot's line of PS (the pass reads
    // PS by slot), every other position's to its own sink line of PS, after
    // the slots: one 1-KiB line and one side line of PS per position, so the
    // lines each array takes do not depend on the batch
    const uint4 pt = xor4(sd, ks);  // lane u < U: position p0 + u's side entry
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 e = uni4(shfl4(pt, u));
      // only an authenticated side entry names a slot (a forged or replayed
      // one fails the batch and goes to its sink)
      const bool last = ok && e.z != 0u && e.w < a.nslots;
      const uint64_t d = last ? (uint64_t)e.w : (uint64_t)a.nslots + p0 + u;
      st_drop(a.ps, d * 64 + lane, v[u]);
      if (lane < 8) st_drop(a.psds, d * 8 + lane, lane == 0 ? e : make_uint4(0, 0, 0, 0));
    }
  }
}

// ------------------------------------------------------------- k_rr1

// set kinds of the record copy-forward (k_rr2)
constexpr uint32_t kSetNone = 0, kSetRec = 1, kSetZero = 2, kFreeze = 3;
// RS flags (word 1 of the 128-B per-position record)
constexpr uint32_t kRsHead = 1u, kRsLast = 2u, kRsNull = 4u, kRsClass2 = 8u, kRsCand = 16u,
                   kRsRcptOk = 32u, kRsExpiry = 64u;
__device__ inline uint32_t rs_setkind(uint32_t f) { return (f >> 8) & 3u; }

struct Rr1V {
  uint32_t reset, nd_valid, cr_valid, pad;
  uint4 r0[5];  // the row's identity before the batch: id, sender, recipient
  uint4 nd;     // id popped by a next-message DELETE
  uint4 cr[5];  // identity of the record a CREATE put in the row
};

struct Rr1Args {
  const uint4* rpos;
  const ROp* rop;
  uint4* rs;               // B x 128 B
  Rr1V* agg;
  Rr1V* carry;
  const Scal* scal;
  uint32_t B, nblk, xbase, S;
  uint4* g;                // B x 256 B: what pass 0 gathered, by position
  uint32_t pass;           // 0: k_scan_a gathers; 1: k_scan_c reads g
  const uint4* idn;        // B x 128 B: request identity lines (k_meta)
  const uint4* snapidp;    // B x 128 B: snapshot identity lines at the rows' first
                           // positions (k_rpass2); every op reads its own
};

struct Rr1Op {
  using V = Rr1V;
  using Args = Rr1Args;
  __device__ static bool stop(const Args& a) { return a.scal->error != 0u; }
  __device__ static V identity() {
    V v;
    v.reset = v.nd_valid = v.cr_valid = v.pad = 0;
    for (int i = 0; i < 5; ++i) v.r0[i] = v.cr[i] = make_uint4(0, 0, 0, 0);
    v.nd = make_uint4(0, 0, 0, 0);
    return v;
  }
  // selects only (a branch over a struct would put it in scratch)
  __device__ static V combine(const V& a, const V& b) {
    V r;
    const bool br = b.reset != 0u, bn = br || b.nd_valid, bc = br || b.cr_valid;
    r.reset = selu32(br, 1u, a.reset);
    r.nd_valid = selu32(bn, b.nd_valid, a.nd_valid);
    r.cr_valid = selu32(bc, b.cr_valid, a.cr_valid);
    r.pad = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      r.r0[i] = sel4(br, b.r0[i], a.r0[i]);
      r.cr[i] = sel4(bc, b.cr[i], a.cr[i]);
    }
    r.nd = sel4(bn, b.nd, a.nd);
    return r;
  }
  // Pass 0 gathers the op's lines (ROp, request identity, snapshot identity:
  // copies kept for this pass, so k_rr2 reads the image and snapshot rows for
  // the first time) once and stores what both passes need by position: g[p] = {kind,
  // status}, id, image words 0..4, snapshot words 0..4.  Pass 1 and emit read
  // g (addresses that do not depend on the data), so no data-dependent line
  // is read twice in the batch.
  __device__ static void gathered(const Args& a, uint32_t p, uint4* stage, uint4 (&g)[16]) {
    if (a.pass == 0) {
      const uint4 rp = a.rpos[p];
      const uint32_t seq = rp.x & kSeqMask;
      uint4 rr[8], im[8], sn[8];  // ROp: {status, slot, kind, flags}, id, ...
      wave_load128(stage, reinterpret_cast<const uint4*>(a.rop + seq), rr);
      wave_load128(stage, a.idn + (uint64_t)seq * 8, im);
      wave_load128(stage, a.snapidp + (uint64_t)p * 8, sn);  // heads: the row's identity
      g[0] = make_uint4(rr[0].z, rr[0].x, 0u, 0u);
      g[1] = rr[1];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        g[2 + i] = im[i];
        g[7 + i] = sn[i];
      }
#pragma unroll
      for (int i = 12; i < 16; ++i) g[i] = make_uint4(0, 0, 0, 0);
      uint4 h0[8], h1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        h0[i] = g[i];
        h1[i] = g[8 + i];
      }
      wave_store128(stage, a.g, 2ull * p, h0);
      wave_store128(stage, a.g, 2ull * p + 1, h1);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) g[i] = a.g[(uint64_t)p * 16 + i];
    }
  }
  __device__ static V local(const Args& a, uint32_t p, uint4* stage) {
    const uint4 rp = a.rpos[p];
    const bool head = rp.x & kPosHead, null = rp.x & kPosNull;
    uint4 g[16];
    gathered(a, p, stage, g);
    const uint32_t kind = g[0].x, st = g[0].y;
    V v = identity();
    v.reset = (head || null) ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 5; ++i) v.r0[i] = sel4(head, g[7 + i], make_uint4(0, 0, 0, 0));
    const uint4 id = g[1];
    const uint4 q1 = g[3], q2 = g[4], q3 = g[5], q4 = g[6];
    v.nd_valid = (!null && kind == KIND_NEXT_DEL && st == kPending) ? 1u : 0u;
    v.nd = id;
    v.cr_valid = (!null && kind == KIND_CREATE && st == kPending) ? 1u : 0u;
    v.cr[0] = id;
    v.cr[1] = q1;
    v.cr[2] = q2;
    v.cr[3] = q3;
    v.cr[4] = q4;
    return v;
  }
  __device__ static void emit(const Args& a, uint32_t p, const V& ex, const V& loc, uint4* stage) {
    const uint4 rp = a.rpos[p];
    const uint32_t seq = rp.x & kSeqMask;
    const bool head = rp.x & kPosHead, last = rp.x & kPosLast, null = rp.x & kPosNull;
    uint4 g[16];
    gathered(a, p, stage, g);  // pass 1: the position-indexed copy
    const uint32_t kind = g[0].x, rstatus = g[0].y;
    const uint4 qid = g[2], q1 = g[3], q2 = g[4], q3 = g[5], q4 = g[6];
    const V in = combine(ex, loc);  // this op's own head / pop / create included
    const bool r0_exists = nz4(in.r0[0]);
    const uint4 rid = g[1];
    // the pop of a next-message DELETE succeeds on a row that holds its id
    const bool nd_ok = (in.nd_valid != 0u) & r0_exists & eq4(in.nd, in.r0[0]);
    const bool is_next = kind == KIND_NEXT_READ || kind == KIND_NEXT_DEL;
    const bool is_create = kind == KIND_CREATE;
    // Every case is computed and the op's own one selected (no branch over op
    // kinds: a wave of padding ops would skip the code, and instruction fetch
    // shows in FETCH_SIZE; routed shard pipelines end in a data-dependent
    // number of padding ops).
    const bool c_next = !null && is_next, c_cr = !null && !is_next && is_create;
    const bool c_byid = !null && !is_next && !is_create;
    // next: M1 resolved it to this row, which must hold that id
    const uint32_t st_next = (r0_exists & eq4(in.r0[0], rid)) ? 1u : 8u;
    const uint32_t sk_next = (kind == KIND_NEXT_DEL && st_next == 1u) ? kSetZero : kSetNone;
    // create: the allocator hands out free rows, empty after the pops
    const uint32_t st_cr = (r0_exists & !nd_ok) ? 8u : 1u;
    const uint32_t sk_cr = st_cr == 1u ? kSetRec : kSetNone;
    // by-id READ / UPDATE / DELETE: the row as the creates and pops of this
    // batch left it (class order: pops, creates, then these)
    const bool cr_ok = (in.cr_valid != 0u) & !(r0_exists & !nd_ok);
    uint4 idb[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) idb[i] = sel4(cr_ok, in.cr[i], sel4(nd_ok, make_uint4(0, 0, 0, 0), in.r0[i]));
    const bool exists1 = nz4(idb[0]);
    const bool cand = exists1 & eq4(qid, idb[0]) &
                      ((eq4(q1, idb[1]) & eq4(q2, idb[2])) | (eq4(q1, idb[3]) & eq4(q2, idb[4])));
    const bool rcpt_ok = eq4(q3, idb[3]) & eq4(q4, idb[4]);
    const bool expiry = seq >= a.xbase;
    const bool apply = cand & rcpt_ok & !expiry;
    const uint32_t sk_b = selu32(apply && kind == KIND_UPDATE, kSetRec,
                                 selu32(apply && kind == KIND_DELETE, kFreeze, kSetNone));
    const uint32_t fl_b = kRsClass2 | (cand ? kRsCand : 0u) | (rcpt_ok ? kRsRcptOk : 0u) | (expiry ? kRsExpiry : 0u);
    const uint32_t status = selu32(c_next, st_next, selu32(c_cr, st_cr, rstatus));
    const uint32_t setk = selu32(c_next, sk_next, selu32(c_cr, sk_cr, selu32(c_byid, sk_b, kSetNone)));
    uint32_t flags = selu32(c_byid, fl_b, 0u);
    uint4 ident[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) ident[i] = sel4(c_cr, in.cr[i], sel4(c_byid, idb[i], in.r0[i]));
    flags |= (head ? kRsHead : 0u) | (last ? kRsLast : 0u) | (null ? kRsNull : 0u) | (setk << 8);
    uint4 rec[8];
    rec[0] = make_uint4(seq, flags, status, kind);
    // the physical row (P side entry: the row a final state replaces)
    const uint64_t prow = null ? 0ull : (uint64_t)rp.z * a.S + rp.w;
    rec[1] = make_uint4(rp.y, (uint32_t)prow, (uint32_t)(prow >> 32), 0u);
#pragma unroll
    for (int i = 0; i < 5; ++i) rec[2 + i] = ident[i];
    rec[7] = make_uint4(0, 0, 0, 0);
    wave_store128(stage, a.rs, p, rec);
  }
};

// ------------------------------------------------- 1 KiB copy-forward scans
//
// Scans whose carried value is a 1 KiB row (lane l of a wave holds 16 B) and
// whose element flags F (4 words, wave-uniform) say how the value moves:
// Op::takes_b(a, b) is true when b's value replaces the running one, and
// Op::f_combine is associative.  The value itself is never combined, only
// selected, so a block aggregate carries the value of one op.
//   vscan_a   one wave per block of 64 ops: flag scan, then the defining
//             op's value (one 1 KiB read per block) -> agg
//   vscan_b1  one workgroup per 64 blocks: sequential in registers, 16 blocks
//             per wave -> per-64-block aggregates
//   vscan_b2  one wave: exclusive carries of the 64-block aggregates
//   vscan_b3  as b1, re-walked from its carry: exclusive carry of every block
// Every aggregate is read the same number of times whatever it holds, and each
// value is copied, never re-read by many readers (shared reads would hit in L2
// and make FETCH_SIZE depend on the data).  The op-specific phase C walks 16
// ops per wave from its carry (vscan_carry_in).

constexpr uint32_t kVBlk = 64;        // ops per block aggregate
constexpr uint32_t kVLineU4 = 72;     // aggregate record: flag line + 1 KiB value

template <class Op>
__device__ inline void f_walk(const typename Op::Args& a, uint32_t p0, uint32_t n, uint4& f,
                              uint32_t& idx) {
  f = Op::f_identity();
  idx = 0;
#pragma unroll 16
  for (uint32_t j = 0; j < n; ++j) {
    const uint4 e = Op::f_of(a, p0 + j);
    idx = Op::takes_b(f, e) ? j : idx;
    f = Op::f_combine(f, e);
  }
}

__device__ inline void vrec_store(uint4* rec, uint4 f, uint4 v) {
  const uint32_t lane = lane_id();
  rec[8 + lane] = v;
  if (lane < 8) rec[lane] = lane == 0 ? f : make_uint4(0, 0, 0, 0);
}

// Select scans (Op::kSelect): the block value is the value of one op, the
// block's defining op d (the last whose element replaces the running value).
// Every op's rows are read and op d's kept, so the address stream does not
// depend on which op defines the block (one row read at a data-dependent
// position per block showed in FETCH_SIZE; DESIGN.md §3 rule 3).  Merge scans
// (values synthesized from small per-op data, combined lane-wise by
// Op::v_combine): the block walks all of its ops.
template <class Op>
__global__ __launch_bounds__(256) void k_vscan_a(typename Op::Args a) {
  if (a.scal->error) return;
  if constexpr (Op::kSelect) {
    // one block per wave: its 64 position records read once into LDS (8
    // whole-line loads), the block's transform and defining op d from them,
    // then every op's rows are read and op d's kept.  (One block per
    // workgroup, each wave reading 16 ops' rows, ran 2-3x faster and made the
    // kernel's duration follow how many of the rows the previous kernel had
    // just written, i.e. the number of groups: tests/test_timing.py,
    // profiles/r03u_timing_c3.txt.)
    static_assert(Op::kStash, "select scans read their records once (stash)");
    __shared__ uint4 s_rec[4][kVBlk * 8];
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
    if (b >= a.nvb) return;
    uint4* rec = s_rec[threadIdx.x >> 6];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) rec[i * 64 + lane] = Op::rec_line(a, (uint64_t)b * kVBlk * 8 + i * 64 + lane);
    wave_lds_sync();
    uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
    uint32_t d = 0;
    for (uint32_t j = 0; j < kVBlk; ++j) {
      const uint4 e = Op::f_of_rec(rec + j * 8);
      d = Op::takes_b(f, e) ? j : d;
      f = Op::f_combine(f, e);
    }
    for (uint32_t j0 = 0; j0 < kVBlk; j0 += 8) {
      uint4 x[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) x[u] = Op::elem_value(a, b * kVBlk + j0 + u, rec + (j0 + u) * 8);
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) v = sel4(j0 + u == d, x[u], v);
    }
    vrec_store(a.vagg + (uint64_t)b * kVLineU4, f, Op::value_fin(f, v));
  } else if constexpr (Op::kStash) {
    // merge scans with stashed records: a block per wave, its 64 records
    // read once (8 whole-line loads in flight together), walked from LDS
    __shared__ uint4 s_rec[4][kVBlk * 8];
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
    if (b >= a.nvb) return;  // the grid's last workgroup only
    uint4* rec = s_rec[threadIdx.x >> 6];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) rec[i * 64 + lane] = Op::rec_line(a, (uint64_t)b * kVBlk * 8 + i * 64 + lane);
    wave_lds_sync();
    uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
    for (uint32_t j = 0; j < kVBlk; ++j) {
      const uint4 e = Op::f_of_rec(rec + j * 8);
      v = Op::v_combine(f, v, e, Op::value_of_rec(rec + j * 8, e));
      f = Op::f_combine(f, e);
    }
    vrec_store(a.vagg + (uint64_t)b * kVLineU4, f, v);
  } else {
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= a.nvb) return;
    uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
    for (uint32_t j = 0; j < kVBlk; ++j) {
      const uint4 e = Op::f_of(a, b * kVBlk + j);
      v = Op::v_combine(f, v, e, Op::value_of(a, b * kVBlk + j, e));
      f = Op::f_combine(f, e);
    }
    vrec_store(a.vagg + (uint64_t)b * kVLineU4, f, v);
  }
}

// sequential combine of records rec[i], i in [lo, hi), into (f, v); with
// `out`, also the exclusive carries out[i]
template <class Op>
__device__ inline void vwalk_records(const uint4* rec, uint32_t lo, uint32_t hi, uint4& f, uint4& v,
                                     uint4* out) {
  const uint32_t lane = lane_id();
  for (uint32_t i0 = lo; i0 < hi; i0 += 8) {
    uint4 rf[8], rv[8];
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {  // loads of 8 records in flight together
      const uint32_t i = min(i0 + u, hi - 1);
      rf[u] = rec[(uint64_t)i * kVLineU4];
      rv[u] = rec[(uint64_t)i * kVLineU4 + 8 + lane];
    }
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      if (i0 + u < hi) {
        if (out) vrec_store(out + (uint64_t)(i0 + u) * kVLineU4, f, v);
        const uint4 e = uni4(rf[u]);
        v = Op::v_combine(f, v, e, rv[u]);
        f = Op::f_combine(f, e);
      }
    }
  }
}

template <class Op>
__global__ __launch_bounds__(256) void k_vscan_b1(typename Op::Args a) {
  if (a.scal->error) return;
  __shared__ uint4 s_v[4][64];
  __shared__ uint4 s_f[4];
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t lo = min(a.nvb, blockIdx.x * 64 + wave * 16), hi = min(a.nvb, lo + 16);
  uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
  vwalk_records<Op>(a.vagg, lo, hi, f, v, nullptr);
  s_v[wave][lane] = v;
  if (lane == 0) s_f[wave] = f;
  __syncthreads();
  if (wave == 0) {
    uint4 g = Op::f_identity(), gv = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < 4; ++k) {
      const uint4 e = s_f[k];
      gv = Op::v_combine(g, gv, e, s_v[k][lane]);
      g = Op::f_combine(g, e);
    }
    vrec_store(a.vagg2 + (uint64_t)blockIdx.x * kVLineU4, g, gv);
  }
}

template <class Op>
__global__ __launch_bounds__(64) void k_vscan_b2(typename Op::Args a) {
  if (a.scal->error) return;
  uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
  vwalk_records<Op>(a.vagg2, 0, a.nvb2, f, v, a.vcarry2);
}

template <class Op>
__global__ __launch_bounds__(256) void k_vscan_b3(typename Op::Args a) {
  if (a.scal->error) return;
  __shared__ uint4 s_v[4][64];
  __shared__ uint4 s_f[4];
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t lo = min(a.nvb, blockIdx.x * 64 + wave * 16), hi = min(a.nvb, lo + 16);
  uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
  vwalk_records<Op>(a.vagg, lo, hi, f, v, nullptr);
  s_v[wave][lane] = v;
  if (lane == 0) s_f[wave] = f;
  __syncthreads();
  const uint4* c = a.vcarry2 + (uint64_t)blockIdx.x * kVLineU4;
  uint4 cf = uni4(c[0]), cv = c[8 + lane];
  for (uint32_t k = 0; k < wave; ++k) {
    const uint4 e = s_f[k];
    cv = Op::v_combine(cf, cv, e, s_v[k][lane]);
    cf = Op::f_combine(cf, e);
  }
  vwalk_records<Op>(a.vagg, lo, hi, cf, cv, a.vcarry);
}

// Phase C prologue, second half: given the aggregate (f, v) of this wave's
// 16 ops, the carry into its first op (block carry, then the aggregates of
// the block's earlier waves through LDS).
// The block's carry record into LDS, read by wave 0 only and as whole lines
// (the flag line by 8 lanes, the value by 64): four waves reading the same
// lines hit or miss depending on timing, and a 16-B read fetches its line
// whole or in halves.  The caller's barrier publishes it.
__device__ inline void vcarry_stage(const uint4* c, uint4* s_c) {
  const uint32_t lane = lane_id();
  if ((threadIdx.x >> 6) == 0) {
    s_c[8 + lane] = c[8 + lane];
    if (lane < 8) s_c[lane] = c[lane];
  }
}

template <class Op>
__device__ inline void vscan_carry_tail(const typename Op::Args& a, uint4 (*s_v)[64], uint4* s_f,
                                        uint4 f, uint4 v, uint4& cf, uint4& cv) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x;
  __shared__ uint4 s_c[kVLineU4];
  vcarry_stage(a.vcarry + (uint64_t)b * kVLineU4, s_c);
  s_v[wave][lane] = v;
  if (lane == 0) s_f[wave] = f;
  __syncthreads();
  cf = s_c[0];
  cv = s_c[8 + lane];
  for (uint32_t k = 0; k < wave; ++k) {
    const uint4 e = s_f[k];
    cv = Op::v_combine(cf, cv, e, s_v[k][lane]);
    cf = Op::f_combine(cf, e);
  }
}

// Phase C prologue: the carry into the first of this wave's 16 ops.  Merge
// scans (values from position-indexed records) only; select scans read their
// ops' lines once into registers and use vscan_carry_tail (a data-dependent
// line read twice in one kernel hits or misses L2 depending on what else the
// XCD read, which made FETCH_SIZE depend on the data).
template <class Op>
__device__ inline void vscan_carry_in(const typename Op::Args& a, uint4 (*s_v)[64], uint4* s_f,
                                      uint4& cf, uint4& cv) {
  static_assert(!Op::kSelect, "select scans: read the lines once, then vscan_carry_tail");
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x, p0 = b * kVBlk + wave * 16;
  uint4 f = Op::f_identity(), v = make_uint4(0, 0, 0, 0);
  for (uint32_t j = 0; j < 16; ++j) {
    const uint4 e = Op::f_of(a, p0 + j);
    v = Op::v_combine(f, v, e, Op::value_of(a, p0 + j, e));
    f = Op::f_combine(f, e);
  }
  __shared__ uint4 s_c[kVLineU4];
  vcarry_stage(a.vcarry + (uint64_t)b * kVLineU4, s_c);
  s_v[wave][lane] = v;
  if (lane == 0) s_f[wave] = f;
  __syncthreads();
  cf = s_c[0];
  cv = s_c[8 + lane];
  for (uint32_t k = 0; k < wave; ++k) {
    const uint4 e = s_f[k];
    cv = Op::v_combine(cf, cv, e, s_v[k][lane]);
    cf = Op::f_combine(cf, e);
  }
}

// common vscan buffers (each Op's Args embeds these names)
#define GVS_VSCAN_FIELDS                                                    \
  uint4* vagg;    /* nvb block aggregates */                                \
  uint4* vagg2;   /* nvb2 = ceil(nvb / 64) aggregates of 64 blocks */      \
  uint4* vcarry2; /* their exclusive carries */                             \
  uint4* vcarry;  /* nvb exclusive block carries */                         \
  const Scal* scal;                                                         \
  uint32_t nvb, nvb2;

// ------------------------------------------------------------- k_rr2
//
// The record copy-forward of the message rows.  The element of an op: reset
// (row head: the snapshot), then its own effect: a set (CREATE, UPDATE: the
// request image with the row identity in lanes 0..4), a set to empty (a
// popping next DELETE), or a freeze (a DELETE: empty, and nothing after it in
// the row applies).  F = {reset, frozen, has, 0}.

struct Rr2Args {
  GVS_VSCAN_FIELDS
  const uint4* rs;        // B x 128 B
  const uint4* img;
  const uint4* snapp;     // B x 1 KiB: row snapshots at their first op's position
  uint4* pbuf;            // B final states, by sorted position (AUTH: all of them,
                          // sealed next; plain: the positions that are not a row's last)
  uint4* psd;             // B x 128 B: {physical row lo, hi, valid (the row's last op), slot}
  uint4* psink;           // the other positions' states, by position (plain: PS's B sink lines; AUTH: P)
  uint4* ps;              // plain: W*c x 1 KiB, each row's final state at its slot
  uint4* resp;            // B internal response slots (kRespSlot)
  RRes* rres;
  uint32_t B;
  uint64_t cutoff;
};

// the per-position record words every lane needs (RS lines 0 and 1)
struct RsHdr {
  uint32_t seq, flags, status, kind, slot, prow_lo, prow_hi;
};

__device__ inline RsHdr rs_hdr(const uint4* rs, uint32_t p) {
  const uint4 w0 = uni4(rs[(uint64_t)p * 8]), w1 = uni4(rs[(uint64_t)p * 8 + 1]);
  return RsHdr{w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z};
}

struct Rr2Op {
  using Args = Rr2Args;
  __device__ static uint4 f_identity() { return make_uint4(0, 0, 0, 0); }
  __device__ static uint4 f_combine(uint4 a, uint4 b) {
    uint4 r = sel4(b.z != 0u, make_uint4(a.x, 0u, 1u, 0u), a);
    r = sel4(b.y != 0u, make_uint4(a.x, 1u, 1u, 0u), r);
    r = sel4(a.y != 0u, a, r);
    return sel4(b.x != 0u, b, r);
  }
  static constexpr bool kSelect = true;
  __device__ static bool takes_b(uint4 a, uint4 b) { return b.x || (!a.y && (b.y || b.z)); }
  __device__ static uint4 v_combine(uint4 fa, uint4 va, uint4 fb, uint4 vb) {
    return sel4(takes_b(fa, fb), vb, va);
  }
  __device__ static uint4 f_of_hdr(const RsHdr& h) {
    const uint32_t sk = rs_setkind(h.flags);
    uint4 e = make_uint4((h.flags & (kRsHead | kRsNull)) ? 1u : 0u, 0u, 0u, 0u);
    e.z = e.x;
    if (sk == kSetRec || sk == kSetZero) e.z = 1u;
    if (sk == kFreeze) e.y = e.z = 1u;
    return e;
  }
  __device__ static uint4 f_of(const Args& a, uint32_t p) { return f_of_hdr(rs_hdr(a.rs, p)); }
  // value of op p's own element, lane-wise, from its sources: the snapshot for
  // a head without a set, the request image with the row identity (RS lines
  // 2..6 -> lanes 0..4) for a set, empty for a pop / freeze / null op
  __device__ static uint4 own_value(const RsHdr& h, uint4 snapv, uint4 imgv, uint4 identv) {
    const uint32_t lane = lane_id(), sk = rs_setkind(h.flags);
    const uint4 z = make_uint4(0, 0, 0, 0);
    uint4 v = sel4((h.flags & kRsHead) != 0u, snapv, z);
    v = sel4(sk == kSetRec, sel4(lane < 5, identv, imgv), v);
    v = sel4(sk == kSetZero || sk == kFreeze || (h.flags & kRsNull), z, v);
    return v;
  }
  __device__ static uint4 ident_of(const Args& a, uint32_t p) {
    return a.rs[(uint64_t)p * 8 + 2 + min(lane_id(), 4u)];
  }
  // k_vscan_a reads the 64 position records of a block once (kStash) and
  // every op's element value (its snapshot line and request image)
  static constexpr bool kStash = true;
  __device__ static uint4 rec_line(const Args& a, uint64_t i) { return a.rs[i]; }
  __device__ static RsHdr hdr_of_rec(const uint4* r) {
    const uint4 w0 = uni4(r[0]), w1 = uni4(r[1]);
    return RsHdr{w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z};
  }
  __device__ static uint4 f_of_rec(const uint4* r) { return f_of_hdr(hdr_of_rec(r)); }
  __device__ static uint4 elem_value(const Args& a, uint32_t p, const uint4* r) {
    const uint32_t lane = lane_id();
    const RsHdr h = hdr_of_rec(r);
    const uint4 sv = ld_row<false>(&a.snapp[(uint64_t)p * 64 + lane]);
    const uint4 iv = ld_row<false>(&a.img[(uint64_t)h.seq * 64 + lane]);
    const bool from_snap = (h.flags & kRsHead) && rs_setkind(h.flags) != kSetRec;
    const uint4 x = sel4(from_snap, sv, iv);
    return own_value(h, x, x, r[2 + min(lane, 4u)]);
  }
  __device__ static uint4 value_fin(uint4 f, uint4 v) { return sel4(f.y || !f.z, make_uint4(0, 0, 0, 0), v); }
};

// failure record: all zero but the request's server time (lane 5 low 8 B)
__device__ inline uint4 fail_rec(uint4 imgv, uint32_t status) {
  const uint32_t lane = lane_id();
  const uint4 ts = shfl4(imgv, 5);
  const bool keep = lane == 5 && status != 0u;  // selects: no code skipped for hard errors
  return make_uint4(selu32(keep, ts.x, 0u), selu32(keep, ts.y, 0u), 0u, 0u);
}

// k_rr2_c: each wave walks its 16 ops in order from its carry: statuses of
// by-id ops, every response, and the state of the row after every op into P
// at the op's position (the next pass applies the row's last one, named by
// the slot descriptor; the side entry says which row it replaces)
__global__ __launch_bounds__(256) void k_rr2_c(Rr2Args a) {
  if (a.scal->error) return;
  __shared__ uint4 s_v[4][64];
  __shared__ uint4 s_f[4];
  __shared__ uint4 s_rs[4][16 * 8];  // each wave's 16 RS records
  __shared__ uint4 s_blk[kVLineU4];  // the block's carry record
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x, p0 = b * kVBlk + wave * 16;
  // Every global line this kernel needs is read once: a line read twice in a
  // kernel hits or misses L2 depending on the traffic in between, whose
  // addresses depend on the data (FETCH_SIZE would).  RS records and the
  // block's records go through LDS.
  s_rs[wave][lane] = a.rs[(uint64_t)p0 * 8 + lane];
  s_rs[wave][64 + lane] = a.rs[(uint64_t)p0 * 8 + 64 + lane];
  if (wave == 0) {
    const uint4* c = a.vcarry + (uint64_t)b * kVLineU4;
    s_blk[8 + lane] = c[8 + lane];
    if (lane < 8) s_blk[lane] = c[lane];
  }
  __syncthreads();
  auto hdr = [&](uint32_t j) {
    const uint4 w0 = uni4(s_rs[wave][j * 8]), w1 = uni4(s_rs[wave][j * 8 + 1]);
    return RsHdr{w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z};
  };
  auto ident = [&](uint32_t j) { return s_rs[wave][j * 8 + 2 + min(lane, 4u)]; };
  // the rows: every op's own SNAPP line (heads find their row's snapshot
  // there) and its request image
  uint4 svs[16], ivs[16];
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const RsHdr h = hdr(j);
    svs[j] = ld_row<false>(&a.snapp[(uint64_t)(p0 + j) * 64 + lane]);
    ivs[j] = ld_row<false>(&a.img[(uint64_t)h.seq * 64 + lane]);
  }
  uint4 cf, cv;
  {  // the wave's aggregate from registers, then the carry
    uint4 f = Rr2Op::f_identity(), xs = svs[0], xi = ivs[0], id = ident(0);
    uint32_t d = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const uint4 e = Rr2Op::f_of_hdr(hdr(j));
      const bool t = Rr2Op::takes_b(f, e);
      d = t ? j : d;
      xs = sel4(t, svs[j], xs);
      xi = sel4(t, ivs[j], xi);
      id = sel4(t, ident(j), id);
      f = Rr2Op::f_combine(f, e);
    }
    const RsHdr hd = hdr(d);
    const bool from_snap = (hd.flags & kRsHead) && rs_setkind(hd.flags) != kSetRec;
    const uint4 x = sel4(from_snap, xs, xi);
    const uint4 v = sel4(f.y || !f.z, make_uint4(0, 0, 0, 0), Rr2Op::own_value(hd, x, x, id));
    s_v[wave][lane] = v;
    if (lane == 0) s_f[wave] = f;
    __syncthreads();
    cf = uni4(s_blk[0]);
    cv = s_blk[8 + lane];
    for (uint32_t k = 0; k < wave; ++k) {
      const uint4 e = s_f[k];
      cv = Rr2Op::v_combine(cf, cv, e, s_v[k][lane]);
      cf = Rr2Op::f_combine(cf, e);
    }
  }
  uint4 sd = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    const uint32_t p = p0 + j;
    const RsHdr h = hdr(j);
    const bool head = h.flags & kRsHead;
    const uint4 sv = svs[j], iv = ivs[j];
    const uint4 idv = ident(j);
    // the row state before this op
    const uint4 pf = sel4(head, make_uint4(1u, 0u, 1u, 0u), cf);
    const uint4 pv = sel4(head, sv, cv);
    // by-id op: the row must still hold the record it named (no DELETE before
    // it in this batch); an expiry delete also needs the record's current
    // time below the cutoff.  Computed for every op and selected (padding ops
    // sort last: a branch would leave their waves' code unfetched).
    const uint64_t ts = ((uint64_t)__shfl(pv.y, 5) << 32) | __shfl(pv.x, 5);
    const bool fresh = (h.flags & kRsExpiry) && !(ts < a.cutoff);
    const bool found = (h.flags & kRsCand) && !pf.y && !fresh;
    const uint32_t st2 = selu32(!found, 2u, selu32(h.kind != KIND_READ && !(h.flags & kRsRcptOk), 4u, 1u));
    const uint32_t status = selu32((h.flags & kRsClass2) != 0u, st2, h.status);
    const bool ok = status == 1u;
    const uint4 own = Rr2Op::own_value(h, sv, iv, idv);
    const uint4 resp = sel4(!ok, fail_rec(iv, status), sel4(rs_setkind(h.flags) == kSetRec, own, pv));
    const uint4 e = Rr2Op::f_of_hdr(h);
    cv = sel4(Rr2Op::takes_b(cf, e), own, cv);
    cf = Rr2Op::f_combine(cf, e);
    // an expiry delete is the last op of its row: it only decides the final state
    const uint4 fin = sel4((h.flags & kRsExpiry) && ok, make_uint4(0, 0, 0, 0), cv);
    const uint64_t r0 = (uint64_t)h.seq * (kRespSlot / 16);
    st_drop(a.resp, r0 + lane, resp);
    if (lane < 8) {
      const uint4 t = make_uint4(lane == 0 ? status : 0u, 0, 0, 0);
      st_drop(a.resp, r0 + 64 + lane, t);
      st_drop(a.rres, (uint64_t)h.seq * 8 + lane, t);
    }
    // the row's final state: plain stores put it at the row's slot (the next
    // pass reads P by slot), every other position's state in its own sink
    // line after the slots (so PS takes B lines whatever the batch); AUTH
    // keeps all of them by position (sealed next, k_pseal)
    const bool to_slot = a.ps && (h.flags & kRsLast);
    st_drop(to_slot ? a.ps : a.psink, (to_slot ? (uint64_t)h.slot : p) * 64 + lane, fin);
    sd = sel4(lane == j, make_uint4(h.prow_lo, h.prow_hi, (h.flags & kRsLast) ? 1u : 0u, h.slot), sd);
  }
  if (lane < 16) st_drop(a.psd, (uint64_t)(p0 + lane) * 8, sd);
}

}  // namespace gvs
