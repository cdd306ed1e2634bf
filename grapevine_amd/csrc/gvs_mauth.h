// gvs_mauth.h — the mailbox passes of a sealed store (authenticated storage,
// DESIGN.md §8): k_m1a / k_m2a, the AUTH forms of k_m1x / k_m2x (gvs_mtx.h).
//
// Round 4's sealed mailbox passes staged every 8-row chunk in a per-wave LDS
// area (35 KiB per workgroup beside the 64-KiB AES window) to transpose it for
// the 256-B leaf hashes, and computed each row's header PRF in the same
// instructions as the leaves (half the lanes' second compression wasted): one
// workgroup of four waves per CU, one wave per SIMD, 2.8 ms (read pass) and
// 5.5 ms (write pass) at C5 for 1 GiB of mailboxes, twice the message pass's
// time per row.  Here, as in the sealed message pass (gvs_spass.h):
//   * a sealed mailbox table is stored in 16-row tiles (mtile_unit): the 16
//     coalesced 1-KiB loads of a chunk leave leaf L & 3 (256 B) of row L >> 2
//     in lane L's registers, so the row hash (NH over the leaf, the sums added
//     over the row's four lanes; BLAKE2b leaf PRFs until round 6) and the CTR keystream
//     (blocks 16 (L & 3) .. + 15 of the lane's row) work on registers;
//   * the header PRFs are computed one row per thread for the partition at
//     once: the read headers in the prepass (with the side entries' keystream
//     at both epochs), the write headers after the stream; the per-row values
//     live in the AES window's 128-B holes, as does each wave's 1-KiB row
//     buffer (the touched rows move between the tile and the row-major wave
//     layout the mailbox logic uses through it);
//   * 78 KiB of LDS per workgroup: two workgroups, eight waves, per CU.
// The mailbox logic (groups, admission, placement, the fixed number of slot
// iterations per wave) is k_m1x's / k_m2x's, on 16-row chunks.  Mailbox
// partitions of a sealed store hold at most kSrAuth rows, a multiple of 16.
#pragma once
#include "gvs_mtx.h"

namespace gvs {

constexpr int kMA = 16;              // rows per chunk
constexpr uint32_t kSrAuth = 256;    // mailbox rows per partition, sealed stores

// 16-B slot i of the AES window's holes (bytes [128, 256) of each 256-B entry
// row, gvs_seal_dev.h): 2048 slots
__device__ inline uint4* hole(uint32_t* s_te, uint32_t i) {
  return reinterpret_cast<uint4*>(reinterpret_cast<char*>(s_te) + ((i >> 3) << 8) + 128u + ((i & 7u) << 4));
}
// hole slots: [0, 256) the waves' row buffers (64 each); then per row of the
// partition: read header, side plaintext, side keystream at the write epoch
// (the write pass turns it into the new side ciphertext), write row hash G
constexpr uint32_t kHoWst = 0, kHoHr = 256, kHoSide = kHoHr + kSrAuth, kHoKsw = kHoSide + kSrAuth,
                   kHoLsum = kHoKsw + kSrAuth;
static_assert(kHoLsum + kSrAuth <= 2048, "the holes hold 2048 slots");

// The row hash's NH key (gvs_crypto.h) in LDS as four leaf windows: leaf l
// needs key words 64 l .. 64 l + 75 (its 64 words and three 4-word shifts),
// kept at s_nk + 76 l.  A stride of 76 words puts the four windows' 16-B reads
// of one instruction in different banks (64 words would put them all in one).
constexpr uint32_t kMNkWin = 76;
// the key windows, then the L3 keys and pads (kept in LDS rather than in
// scalar registers: the passes' round keys already fill those)
struct MNk {
  uint32_t w[4 * kMNkWin];
  uint64_t l3k[16];
  uint32_t l3p[4];
  AesRk rkh;  // the header PRF's round keys (read by the per-row header loops)
};
__device__ inline void load_nk(MNk* s, const SealCtx& c) {
  for (uint32_t i = threadIdx.x; i < 4u * kMNkWin; i += blockDim.x)
    s->w[i] = c.nhk[64u * (i / kMNkWin) + i % kMNkWin];
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s->l3k[i] = c.l3k[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) s->l3p[i] = c.l3p[i];
#pragma unroll
    for (int i = 0; i < 44; ++i) s->rkh.w[i] = c.rkh.w[i];
  }
}

// G of the lane's row (the row hash, gvs_crypto.h) in every lane of the row:
// NH of the lane's 256-B leaf (lane L: leaf L & 3 of row L >> 2, v[i] its
// words 4i .. 4i + 3) against the leaf's key window, the four sums added over
// the row's four lanes, then L3.  Word pairs (4i, 4i + 1) and (4i + 2, 4i + 3)
// meet key words 4(i + t) .. 4(i + t) + 3 of the window in iteration t: a
// sliding window of four 16-B key reads.
__device__ inline void mrow_hash(const MNk* s_nk, const uint4 (&v)[kMA], uint64_t r[2]) {
  const uint4* kp = reinterpret_cast<const uint4*>(s_nk->w + kMNkWin * (lane_id() & 3u));
  uint64_t s[4] = {0, 0, 0, 0};
  uint4 k0 = kp[0], k1 = kp[1], k2 = kp[2];
#pragma unroll
  for (int i = 0; i < kMA; ++i) {
    const uint4 k3 = kp[i + 3];
    const uint4 kk[4] = {k0, k1, k2, k3};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t a0 = v[i].x + kk[t].x, b0 = v[i].y + kk[t].y;
      const uint32_t a1 = v[i].z + kk[t].z, b1 = v[i].w + kk[t].w;
      s[t] += (uint64_t)a0 * (uint64_t)b0;  // v_mad_u64_u32
      s[t] += (uint64_t)a1 * (uint64_t)b1;
    }
    k0 = k1;
    k1 = k2;
    k2 = k3;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    s[t] += shfl_u64(s[t], (int)(lane_id() ^ 1u));
    s[t] += shfl_u64(s[t], (int)(lane_id() ^ 2u));
  }
  row_hash_fin(s, s_nk->l3k, s_nk->l3p, r);
}

// XOR the keystream of (mailbox table, row, epoch) blocks 16 (L & 3) .. + 15
// into the lane's registers
__device__ inline void ma_ctr(const SealCtx& c, const LdsTe& te, uint64_t row, uint32_t epoch, uint4 (&v)[kMA]) {
  constexpr int NB = 2;
  const CtrRound1J c1 = ctr_round1_row(c.rk, te, 1u, row, epoch, (lane_id() & 3u) * 16u);
  const CtrRound2J c2 = ctr_round2_row1(c.rk, te, c1);  // round 2 cached too
#pragma unroll
  for (uint32_t i = 0; i < kMA; i += NB) {
    uint4 ks[NB];
    ctr_keystream_jn3_1<NB, true>(c.rk, te, c2, i, ks);  // rounds rolled: code size (gvs_seal_dev.h)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      v[i + b] = xor4(v[i + b], ks[b]);
      // the XOR done here: left to the compiler, it was sunk into the step
      // loop that follows, with the keystream and the ciphertext both held
      // (more registers than two waves per SIMD have)
      keep4(v[i + b]);
    }
  }
}

// row u of the chunk in the row-major wave layout (lane b = 16-B block b),
// through the wave's row buffer
__device__ inline uint4 ma_row_out(uint32_t* s_te, uint32_t wave, const uint4 (&v)[kMA], uint32_t u) {
  const uint32_t lane = lane_id();
  const bool mine = (lane >> 2) == u;
#pragma unroll
  for (uint32_t i = 0; i < kMA; ++i)
    if (mine) *hole(s_te, kHoWst + wave * 64u + 16u * (lane & 3u) + i) = v[i];
  wave_lds_sync();
  const uint4 r = *hole(s_te, kHoWst + wave * 64u + lane);
  wave_lds_sync();
  return r;
}

// and back: row u of the chunk replaced by x (row-major, lane b = block b)
__device__ inline void ma_row_in(uint32_t* s_te, uint32_t wave, uint4 (&v)[kMA], uint32_t u, uint4 x) {
  const uint32_t lane = lane_id();
  const bool mine = (lane >> 2) == u;
  *hole(s_te, kHoWst + wave * 64u + lane) = x;
  wave_lds_sync();
#pragma unroll
  for (uint32_t i = 0; i < kMA; ++i) v[i] = sel4(mine, *hole(s_te, kHoWst + wave * 64u + 16u * (lane & 3u) + i), v[i]);
  wave_lds_sync();
}

// m2_row (gvs_mtx.h) with its compaction stage in the holes (64 slots from
// `base`)
__device__ inline uint4 m2_row_h(uint4 v, bool matched, uint32_t len, uint32_t dp, uint64_t mask, uint32_t n_succ,
                                 uint4 app, uint32_t* s_te, uint32_t base, uint32_t* fl_out) {
  const uint32_t lane = lane_id();
  const uint32_t i = lane - 2u;
  const bool keep = matched && lane >= 2 && i < len && i >= dp && !((mask >> i) & 1ull);
  const uint64_t km = __ballot(keep);
  const uint32_t nk = (uint32_t)__popcll(km);
  *hole(s_te, base + (keep ? mbcnt64(km) : nk + mbcnt64(~km))) = v;
  wave_lds_sync();
  const uint32_t r = lane - 2u;
  const uint4 w = *hole(s_te, base + min(r, 63u));
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

// the chunk's 16 rows (tile t of the table), one whole KiB per load
__device__ inline void ma_load(uint4 (&v)[kMA], const uint4* mbox, uint64_t t) {
  const uint4* p = mbox + t * (kMA * 64);
#pragma unroll
  for (int i = 0; i < kMA; ++i) v[i] = ld_row<true>(&p[i * 64 + lane_id()]);
}

// Prepass: every row's side entry (decrypted at the read epoch) matched to
// the groups as side_prepass_m does; per row the read header H (side
// ciphertext bound in), and for the write pass the side plaintext and the
// side keystream at the write epoch.  One row per thread.
template <bool WR>
__device__ inline void ma_prepass(const MArgs& a, uint32_t q, GroupM* g, uint32_t ng, int16_t* s_sg,
                                  uint8_t* s_occb, uint32_t* s_occ, uint32_t* s_te, const MNk* s_nk) {
  const LdsTe te = lds_te(s_te);
  for (uint32_t j = threadIdx.x; j < a.Sr; j += 256) {
    const uint64_t row = (uint64_t)q * a.Sr + j;
    const uint4 sct = a.side[row];
    // the side entry's keystream at the read epoch (and, writing, at epoch + 1:
    // through one copy of the AES code, which keeps k_m2a's code well inside
    // the instruction cache)
    uint4 ksr = make_uint4(0, 0, 0, 0), ksw = ksr;
    if constexpr (WR) {
#pragma unroll 1
      for (uint32_t w = 0; w < 2u; ++w) {
        const uint4 k = ctr_keystream(a.sc.rk, te, 1u, row, a.sc.epoch + w, 64u);
        ksr = sel4(w == 0u, k, ksr);
        ksw = k;
      }
    } else {
      ksr = ctr_keystream(a.sc.rk, te, 1u, row, a.sc.epoch, 64u);
    }
    const uint4 sd = xor4(sct, ksr);
    const uint64_t hi = u4lo(sd), w1 = u4hi(sd);
    const bool occ = (w1 & 1u) != 0;
    const int kf = find_group_m(g, ng, a.cm, hi, w1 >> 23);
    const int k = occ ? kf : -1;
    atomicAdd(s_occ, occ ? 1u : 0u);
    const uint32_t kk = k >= 0 ? (uint32_t)k : a.cm;  // rows without a group: the sink entry
    g[kk].slot = (int32_t)j;
    g[kk].len = (uint32_t)(w1 >> 1) & 63u;
    s_sg[j] = (int16_t)k;
    s_occb[j] = occ ? 1 : 0;
    uint64_t h[2];
    head_aes_w(s_nk->rkh, te, row, a.sc.epoch, 1u, true, u4lo(sct), u4hi(sct), h);
    *hole(s_te, kHoHr + j) = make_uint4((uint32_t)h[0], (uint32_t)(h[0] >> 32), (uint32_t)h[1], (uint32_t)(h[1] >> 32));
    if (WR) {
      *hole(s_te, kHoSide + j) = sd;
      *hole(s_te, kHoKsw + j) = ksw;
    }
  }
}

// Verify and decrypt the chunk at the read epoch (rows j0 .. j0 + 15 of
// partition q): a tag mismatch fails the batch and the handle for good.
__device__ inline void ma_unseal(const MArgs& a, uint32_t* s_te, const MNk* s_nk, uint32_t q, uint32_t j0,
                                 uint4 (&v)[kMA]) {
  const uint32_t lane = lane_id(), u = lane >> 2;
  const uint64_t row = (uint64_t)q * a.Sr + j0 + u;
  uint64_t ls[2];
  mrow_hash(s_nk, v, ls);
  const uint4 hr = *hole(s_te, kHoHr + j0 + u);
  const uint4 want = a.btag[row];  // 16 rows' tags: two whole lines
  const bool bad = (u4lo(want) != (ls[0] ^ u4lo(hr))) | (u4hi(want) != (ls[1] ^ u4hi(hr)));
  if (__ballot(bad) && lane == 0) atomicOr(&a.scal->error, 8u);
  ma_ctr(a.sc, lds_te(s_te), row, a.sc.epoch, v);
}

// --------------------------------------------------------------- k_m1a
// the sealed read pass (k_m1x's snapshot of every group's row, the verdict
// header in lane 0)
__global__ __launch_bounds__(256, 2) void k_m1a(MArgs a) {
  extern __shared__ uint4 s_dyn[];
  GroupM* g = reinterpret_cast<GroupM*>(s_dyn);
  GVS_TE_LDS s_te[kTeWords];
  __shared__ int16_t s_sg[kSrAuth];
  __shared__ uint8_t s_occb[kSrAuth];
  __shared__ uint32_t s_ng, s_occ, s_empt, s_w[4], s_tw[kRowWaves];
  __shared__ uint8_t s_tf[kGroupMax];
  __shared__ uint16_t s_tp[kGroupMax + 1];
  __shared__ int16_t s_tl[kGroupMax];
  __shared__ __attribute__((aligned(16))) MNk s_nk;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = blockIdx.x;
  if (a.scal->error) return;
  load_te(s_te, a.te);
  load_nk(&s_nk, a.sc);
  const uint32_t ng = load_groups(a, q, g, &s_ng, false);
  if (tid == 0) {
    s_occ = 0;
    s_empt = 0;
  }
  __syncthreads();
  ma_prepass<false>(a, q, g, ng, s_sg, s_occb, &s_occ, s_te, &s_nk);
  __syncthreads();
  // admission (grapevine.proto:74), as k_m1x
  count_empty(g, ng, a.cm, &s_empt);
  __syncthreads();
  admit_groups(g, ng, a.cm, (a.Sr - s_occ) + s_empt);
  __syncthreads();
  uint4* dry = a.mdry + (uint64_t)q * kMDryU4;
  if (tid < kRowWaves) s_tw[tid] = 0;
  __syncthreads();
  for (uint32_t j = tid; j < a.Sr; j += 256) atomicAdd(&s_tw[(j / kMA) % kRowWaves], s_sg[j] >= 0 ? 1u : 0u);
  for (uint32_t k = tid; k < a.cm; k += 256) s_tf[k] = ((k < ng) & ((int32_t)group_fields(g[k]).slot >= 0)) ? 0 : 1;
  __syncthreads();
  block_flag_scan(s_tf, a.cm, s_tp, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)
    if (s_tf[k]) s_tl[s_tp[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t nfree = s_tp[a.cm];
  uint32_t d0, dn;
  slot_share(s_tw, a.cm, wave, &d0, &dn);
  const uint32_t nch = __builtin_amdgcn_readfirstlane(
      a.Sr > wave * kMA ? (a.Sr - wave * kMA + kRowWaves * kMA - 1) / (kRowWaves * kMA) : 0u);
  // one iteration: a touched row's snapshot or a slot without a row (k_m1x)
  auto step = [&](const uint4 (&v)[kMA], uint32_t bit, uint32_t j0, uint32_t di) {
    const bool slot_it = bit == 0u;
    const uint32_t u0 = (uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u;
    uint4 cur = ma_row_out(s_te, wave, v, u0 & (kMA - 1u));
    const bool listed = slot_it && di < nfree;
    const int k = slot_it ? (listed ? (int)s_tl[di] : 0) : s_sg[j0 + (u0 & (kMA - 1u))];
    const GroupM& G = g[k >= 0 ? (uint32_t)k : 0u];
    const bool real = !slot_it || (listed && (uint32_t)k < ng);
    const uint4 hdr = sel4(real, make_uint4(slot_it ? 0u : G.len, G.fl, G.flags, (uint32_t)G.slot),
                           make_uint4(0, 0, 0, 0));
    cur = sel4(lane == 0, hdr, sel4(lane == 1 || slot_it, make_uint4(0, 0, 0, 0), cur));
    const uint32_t sl = (uint32_t)(((uint64_t)(q * a.cm + (uint32_t)k) * a.sink_mul) % ((uint64_t)a.Q * a.cm));
    uint4* dst = !listed && slot_it ? dry + 64 : real ? a.msnapp + (uint64_t)G.head * 64 : a.msnap + (uint64_t)sl * 64;
    st_drop(dst, lane, cur);
  };
  uint32_t ci = 0;
  for (uint32_t j0 = wave * kMA; j0 < a.Sr; j0 += kRowWaves * kMA, ++ci) {
    uint4 v[kMA];
    ma_load(v, a.mbox, ((uint64_t)q * a.Sr + j0) / kMA);
    ma_unseal(a, s_te, &s_nk, q, j0, v);
    uint32_t mm = 0;
#pragma unroll
    for (int u = 0; u < kMA; ++u) mm |= (s_sg[j0 + u] >= 0) ? (1u << u) : 0u;
    mm = __builtin_amdgcn_readfirstlane(mm);
    const uint32_t nt = (uint32_t)__popc(mm), dlo = spread_lo(ci, nch, dn);
    const uint32_t nr = nt + spread_lo(ci + 1, nch, dn) - dlo;
    uint32_t mq = mm;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint32_t low = mq & (0u - mq);
      mq &= mq - 1u;
      step(v, low, j0, d0 + dlo + (r - nt));
    }
  }
  if (nch == 0) {
    uint4 v[kMA];
#pragma unroll
    for (int u = 0; u < kMA; ++u) v[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t r = 0; r < dn; ++r) step(v, 0u, 0u, d0 + r);
  }
}

// --------------------------------------------------------------- k_m2a
// the sealed write pass (k_m2x): every row rewritten, every result slot read
// once; rows re-encrypted and their side entries re-sealed at epoch + 1, the
// tags after the stream
#ifndef GVS_M2A_WGS
#define GVS_M2A_WGS 2  // workgroups per CU the register budget is sized for
#endif
__global__ __launch_bounds__(256, GVS_M2A_WGS) void k_m2a(MArgs a) {
  extern __shared__ uint4 s_dyn[];
  GroupM* g = reinterpret_cast<GroupM*>(s_dyn);
  GVS_TE_LDS s_te[kTeWords];
  __shared__ int16_t s_sg[kSrAuth];
  __shared__ uint8_t s_occb[kSrAuth];
  __shared__ int16_t s_place[kSrAuth];
  __shared__ uint8_t s_flag[kSrAuth];
  __shared__ uint16_t s_pfx[kSrAuth + 1];
  __shared__ uint16_t s_gpfx[kGroupMax + 1];
  __shared__ uint8_t s_gflag[kGroupMax + 1];
  __shared__ int16_t s_pend[kGroupMax + 1];
  __shared__ uint8_t s_ld[kGroupMax + 1];
  __shared__ uint32_t s_w[4], s_ng, s_occ, s_delta, s_tw[kRowWaves];
  __shared__ __attribute__((aligned(16))) MNk s_nk;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t q = blockIdx.x;
  if (a.scal->error) return;
  load_te(s_te, a.te);
  load_nk(&s_nk, a.sc);
  uint4* side = a.side + (uint64_t)q * a.Sr;
  const uint32_t ng = load_groups(a, q, g, &s_ng, true);
  if (tid == 0) {
    s_occ = 0;
    s_delta = 0;
  }
  __syncthreads();
  ma_prepass<true>(a, q, g, ng, s_sg, s_occb, &s_occ, s_te, &s_nk);
  __syncthreads();
  // final lengths, placement of new recipients, the slot each touched row
  // takes: as k_m2x
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
    atomicAdd(&s_tw[(j / kMA) % kRowWaves], ge >= 0 ? 1u : 0u);
  }
  __syncthreads();
  for (uint32_t k = tid; k < a.cm; k += 256) s_gflag[k] = s_ld[k] ? 0 : 1;
  __syncthreads();
  block_flag_scan(s_gflag, a.cm, s_gpfx, s_w);
  for (uint32_t k = tid; k < a.cm; k += 256)
    if (s_gflag[k]) s_pend[s_gpfx[k]] = (int16_t)k;
  __syncthreads();
  const uint32_t nfree = s_gpfx[a.cm];
  uint32_t d0, dn;
  slot_share(s_tw, a.cm, wave, &d0, &dn);
  const uint32_t nch = __builtin_amdgcn_readfirstlane(
      a.Sr > wave * kMA ? (a.Sr - wave * kMA + kRowWaves * kMA - 1) / (kRowWaves * kMA) : 0u);
  const uint4* res = a.m2tx + (uint64_t)q * a.cm * kVLineU4;
  const uint4* dry = a.mdry + (uint64_t)q * kMDryU4 + 256;
  // the wave's compaction stage (m2_row): its row buffer's slots in the holes
  // are not contiguous, so m2_row gets a 64-slot view through hole()
  auto step = [&](uint4 (&v)[kMA], uint4& mine, uint32_t bit, uint32_t j0, uint32_t di) {
    const bool slot_it = bit == 0u;
    const uint32_t u0 = (uint32_t)__builtin_ctz(bit | (1u << 31)) & 31u, uu = u0 & (kMA - 1u);
    const uint4 cur = ma_row_out(s_te, wave, v, uu);
    const uint32_t j = j0 + uu;
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
    const uint4 nv = m2_row_h(cur, matched, len, dp, mask, G.n_succ, app, s_te, kHoWst + wave * 64u, &fl);
    const uint64_t w1 = (G.glo << 23) | ((uint64_t)fl << 1) | 1ull;
    const uint4 nsd = sel4(fl > 0, make_uint4((uint32_t)G.hi, (uint32_t)(G.hi >> 32), (uint32_t)w1,
                                              (uint32_t)(w1 >> 32)),
                           make_uint4(0, 0, 0, 0));
    // a slot iteration (bit 0) writes row uu back unchanged
    ma_row_in(s_te, wave, v, uu, slot_it ? cur : nv);
    mine = sel4(!slot_it && lane == uu, nsd, mine);
  };
  const uint32_t ep = a.sc.epoch + 1u;
  uint32_t ci = 0;
  for (uint32_t j0 = wave * kMA; j0 < a.Sr; j0 += kRowWaves * kMA, ++ci) {
    uint4 v[kMA];
    const uint64_t t = ((uint64_t)q * a.Sr + j0) / kMA;
    // the per-lane row recomputed per chunk: hoisted, its 64-bit base stayed
    // live across the loop and was spilled to scratch (k_m2a, 24 B per lane)
    uint32_t ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t u = ln >> 2;
    const uint64_t row = (uint64_t)q * a.Sr + j0 + u;
    // four jobs, one copy of each crypto step: 0 verify, 1 decrypt and the
    // mailbox steps, 2 re-encrypt, 3 the new row hashes and the stores.  The
    // unrolled sequence (220 KB of code; k_m1a's 112 KB) made the read pass's
    // FETCH_SIZE follow the request mix by 17-30 KiB under the all-miss and
    // hot mixes (profiles/r05e_*, r05h_*), where the rolled form is flat
    // within 1 KiB (r05g): the steps between the crypto stretches differ by
    // chunk with the mix, and so did what instruction lines the unrolled code
    // had to fetch again.
#pragma unroll 1
    for (uint32_t job = 0; job < 4; ++job) {
      if (job == 0u) ma_load(v, a.mbox, t);
      if (job == 0u || job == 3u) {
        uint64_t ls[2];
        mrow_hash(&s_nk, v, ls);
        if (job == 0u) {  // the read tag: H at the read epoch (prepass) over the old side ciphertext
          const uint4 hr = *hole(s_te, kHoHr + j0 + u);
          const uint4 want = a.btag[row];  // 16 rows' tags: two whole lines
          const bool bad = (u4lo(want) != (ls[0] ^ u4lo(hr))) | (u4hi(want) != (ls[1] ^ u4hi(hr)));
          if (__ballot(bad) && lane == 0) atomicOr(&a.scal->error, 8u);
        } else {  // the write tags are finished after the stream (H over the new side ciphertext)
          if ((lane & 3u) == 0u)
            *hole(s_te, kHoLsum + j0 + u) = make_uint4((uint32_t)ls[0], (uint32_t)(ls[0] >> 32), (uint32_t)ls[1],
                                                       (uint32_t)(ls[1] >> 32));
          uint4* p = a.mbox + t * (kMA * 64);
#pragma unroll
          for (int i = 0; i < kMA; ++i) st_stream(p, (uint64_t)i * 64 + lane, v[i]);
        }
      } else {
        ma_ctr(a.sc, lds_te(s_te), row, job == 1u ? a.sc.epoch : ep, v);
        if (job == 1u) {
          // the chunk's side entries, lane u < 16 row u's plaintext
          uint4 mine = *hole(s_te, kHoSide + j0 + (lane & (kMA - 1u)));
          uint32_t mm = 0;
#pragma unroll
          for (int uu = 0; uu < kMA; ++uu) mm |= (s_sg[j0 + uu] >= 0 || s_place[j0 + uu] >= 0) ? (1u << uu) : 0u;
          mm = __builtin_amdgcn_readfirstlane(mm);
          const uint32_t nt = (uint32_t)__popc(mm), dlo = spread_lo(ci, nch, dn);
          const uint32_t nr = nt + spread_lo(ci + 1, nch, dn) - dlo;
          uint32_t mq = mm;
          for (uint32_t r = 0; r < nr; ++r) {
            const uint32_t low = mq & (0u - mq);
            mq &= mq - 1u;
            step(v, mine, low, j0, d0 + dlo + (r - nt));
          }
          // the new side entries sealed (ciphertext kept for the write headers)
          const uint4 sct = xor4(mine, *hole(s_te, kHoKsw + j0 + (lane & (kMA - 1u))));
          if (lane < (uint32_t)kMA) {
            side[j0 + lane] = sct;
            *hole(s_te, kHoKsw + j0 + lane) = sct;
          }
        }
      }
    }
  }
  if (nch == 0) {
    uint4 v[kMA], mine = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kMA; ++u) v[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t r = 0; r < dn; ++r) step(v, mine, 0u, 0u, d0 + r);
  }
  __syncthreads();
  // the write tags: H at epoch + 1 over the new side ciphertext, one row per
  // thread (the rows' tags are consecutive: whole lines)
  for (uint32_t j = tid; j < a.Sr; j += 256) {
    const uint64_t row = (uint64_t)q * a.Sr + j;
    const uint4 sct = *hole(s_te, kHoKsw + j), ls = *hole(s_te, kHoLsum + j);
    uint64_t h[2];
    head_aes_w(s_nk.rkh, lds_te(s_te), row, ep, 1u, true, u4lo(sct), u4hi(sct), h);
    const uint64_t t0 = h[0] ^ u4lo(ls), t1 = h[1] ^ u4hi(ls);
    a.btag[row] = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32));
  }
  if (tid == 0)
    atomicAdd((unsigned long long*)&a.scal->n_mailboxes, (unsigned long long)(int64_t)(int32_t)s_delta);
}

}  // namespace gvs
