// gvs_spass.h — the sealed message-table pass (authenticated storage,
// DESIGN.md §8) on a fixed memory schedule (DESIGN.md §3 rule 8).
//
// The table pass of a sealed store does what k_rpass2s does for a plain one:
// stream every row of its partition, apply the previous batch's final states
// (PS, by transaction slot), snapshot the rows this batch touches, select
// expired rows; and between load and store each row is verified, decrypted,
// re-encrypted at epoch + 1 and re-tagged (AES-128-CTR + BLAKE2b, gvs_crypto.h).
//
// Round 4's sealed pass read a used slot's final state and wrote a touched
// row's snapshot inside the row stream, at the row, and the unused slots'
// lines after it: so where those 1-KiB accesses fell among the row traffic
// followed the batch, and FETCH_SIZE moved with the request mix by up to
// -304 KiB of 1.25 GB (profiles/r04zi_oblivious_FETCH_SIZE_auth.txt).  The
// plain pass had been fixed by staging every slot line in LDS; the sealed pass
// had no room, its LDS holding 64 AES table replicas and a per-wave stage for
// the leaf hashes.  Here:
//   * sealed rows are stored in the tile layout (gvs_seal_dev.h tile_unit):
//     a coalesced load leaves each lane one whole 128-B leaf, so the leaf
//     hashes read registers and the per-wave stage is gone;
//   * the AES tables keep 32 replicas each (conflict-free for ds_read_b32,
//     gvs_seal_dev.h): T0 and T1 fill the 64-KiB window (GVS_SP_DUAL, one
//     rotation per column instead of three: 5.4 % faster, r05m); with T0
//     alone the window's other half (256 holes of 128 B) stages 32 slot lines;
//   * kSpBufs 1-KiB staging buffers hold the previous batch's final states
//     (buffer k = previous slot k, read before the stream, all c of them) and
//     this batch's snapshots (buffer kSpBufs - 1 - k = slot k, written after
//     the stream, all c of them).  The two batches' used slots of a partition
//     share the buffers: k_sjoint fails a batch (GVS_ERR_BATCH_OVERFLOW)
//     before anything changes when they would overlap, i.e. when the
//     partition's distinct rows over the two batches exceed kSpBufs (86 at
//     C3/C5 against a mean of 32: beyond 9 standard deviations);
//   * in the stream every chunk of 8 rows does the same LDS work: each row
//     reads a final state (its own buffer or a dry one) and writes a
//     snapshot (its own buffer or the dry one), selected per lane.
// So the order and number of a workgroup's HBM accesses depend on (S, c) only.
//
// Rows are dealt to waves in groups of 32 (4 chunks): group g of the
// partition goes to wave g mod NW.  A group's 64 header PRFs (32 rows at the
// read and the write epoch) are one compression per lane.  The waves meet
// after every round of NW groups (the expiry selection merges there, in row
// order).
//
// The fallback (LB = false: more slots than the LDS holds; test-sized tables
// with large batches) keeps the slot lines in HBM and merges / snapshots the
// touched rows in the stream, as round 4 did.
#pragma once
#include "gvs_txn.h"

namespace gvs {

#ifndef GVS_SP_DUAL
#define GVS_SP_DUAL 1  // T0 and T1 in the AES window (load_te2), every staging buffer after it
#endif
constexpr uint32_t kSpBufs = GVS_SP_DUAL ? 86 : 96;  // LDS staging buffers (1 KiB each)
constexpr uint32_t kSpSlots = 64;             // transaction slots per partition (c) with LDS staging
constexpr uint32_t kSpDry = kSpBufs;          // the dry buffer
constexpr uint32_t kSpHoles = GVS_SP_DUAL ? 0 : 32;  // buffers living in the AES window's holes
constexpr uint32_t kSpWords = kRowsMax / 32;  // bitmap words per partition
constexpr uint32_t kJErr = 128u;  // error bit: k_sjoint, two batches' rows of a partition exceed kSpBufs

// byte address (from the 64-KiB-aligned window at LDS 0) of 16-B block i of
// 128-B piece q of staging buffer b.  Blocks are rotated by the piece inside
// it, so the 8 lanes of a row (pieces 0..7, block i each) hit distinct banks.
__device__ inline uint32_t sp_addr(uint32_t b, uint32_t q, uint32_t i) {
  const uint32_t rot = ((i + q) & 7u) * 16u;
  const uint32_t hole = (8u * b + q) * 256u + 128u + rot;
  const uint32_t buf = 65536u + (b - kSpHoles) * 1024u + q * 128u + rot;
  return kSpHoles ? selu32(b < kSpHoles, hole, buf) : buf;
}

template <bool LB>
__device__ inline uint4 sp_ld(const uint32_t* s_lds, uint32_t a) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(s_lds) + a);
}
__device__ inline void sp_st(uint32_t* s_lds, uint32_t a, uint4 x) {
  *reinterpret_cast<uint4*>(reinterpret_cast<char*>(s_lds) + a) = x;
}

// Expiry selection on a chunk in the leaf-major layout: lane 8u holds blocks
// 0..7 of row u (id = block 0, recipient = blocks 3, 4, timestamp = block 5).
// Rows in order u = 0..7; the record of a row goes to slot min(xc, xep) of the
// wave's list and the count advances on a hit (x_detect2, row layout).
__device__ inline uint32_t x_detect_lm(const R2Args& a, const uint4 (&v)[8], uint4* buf, uint32_t xc,
                                       const uint4* s_xx, uint32_t nx) {
  const uint32_t lane = lane_id();
  const uint64_t ts = ((uint64_t)v[5].y << 32) | v[5].x;
  bool ex = false;
  for (uint32_t k = 0; k < nx; ++k) ex |= eq4(v[0], s_xx[k]);
  const uint64_t hits = __ballot((lane & 7u) == 0u && ts < a.cutoff && nz4(v[0]) && !ex);
#pragma unroll
  for (uint32_t u = 0; u < 8; ++u) {
    const uint32_t slot = min(xc, a.xep);
    if (lane == 8u * u) {
      buf[slot * 3 + 0] = v[0];
      buf[slot * 3 + 1] = v[3];
      buf[slot * 3 + 2] = v[4];
    }
    xc += (uint32_t)(hits >> (8u * u)) & 1u;
  }
  return xc;
}

// A 128-B leaf in one lane's registers (v[q] = its 16-B block q) as the 16
// little-endian words BLAKE2b reads
__device__ inline void leaf_words(const uint4 (&v)[8], uint64_t (&m)[16]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    m[2 * q] = u4lo(v[q]);
    m[2 * q + 1] = u4hi(v[q]);
  }
}

// Tag of the lane's row (leaf-major: lane L holds leaf L & 7 of row L >> 3):
// the row hash (gvs_crypto.h): NH of the lane's 32 words against its leaf's
// window of the key (s_nh in LDS: words 32 (L & 7) .. + 43), the four sums
// added over the row's 8 lanes, L3, then the header H.
__device__ inline void lm_tag(const uint32_t* s_nh, const SealCtx& c, const uint4 (&v)[8], const uint64_t hdr[2],
                              uint64_t out[2]) {
  const uint32_t leaf = lane_id() & 7u;
  uint32_t w[32], k[44];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    w[4 * q] = v[q].x;
    w[4 * q + 1] = v[q].y;
    w[4 * q + 2] = v[q].z;
    w[4 * q + 3] = v[q].w;
  }
  const uint4* kp = reinterpret_cast<const uint4*>(s_nh + 32u * leaf);
#pragma unroll
  for (int q = 0; q < 11; ++q) {
    const uint4 x = kp[q];
    k[4 * q] = x.x;
    k[4 * q + 1] = x.y;
    k[4 * q + 2] = x.z;
    k[4 * q + 3] = x.w;
  }
  uint64_t sm[4] = {0, 0, 0, 0};
  nh_words(k, 0u, w, sm);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    sm[t] += shfl_u64(sm[t], (int)(lane_id() ^ 1u));
    sm[t] += shfl_u64(sm[t], (int)(lane_id() ^ 2u));
    sm[t] += shfl_u64(sm[t], (int)(lane_id() ^ 4u));
  }
  uint64_t g[2];
  row_hash_fin(sm, c.l3k, c.l3p, g);
  out[0] = g[0] ^ hdr[0];
  out[1] = g[1] ^ hdr[1];
}

// A value the compiler must treat as unknown where this is called: the loop
// bodies below recompute what depends on it instead of hoisting invariant
// pieces (round-1 AES lookups of the fixed counter words, the header PRF's
// first G functions over its zero words) out of the loop into registers, which
// cost the sealed pass more registers than waves per SIMD allow.
__device__ inline uint32_t opaque(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ inline B2State opaque(const B2State& k) {
  B2State r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t lo = (uint32_t)k.h[i], hi = (uint32_t)(k.h[i] >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi));
    r.h[i] = (uint64_t)lo | ((uint64_t)hi << 32);
  }
  return r;
}

// XOR the keystream of (message table, row, epoch) blocks 8 (L & 7) .. + 7
// into the lane's registers (the row is the lane's own, L >> 3 of the chunk),
// NB blocks in flight at a time
#ifndef GVS_SP_NB
#define GVS_SP_NB 2
#endif
#ifndef GVS_SP_R2
#define GVS_SP_R2 1  // round 2 cached per row (ctr_round2_row); 0 in A/B builds only
#endif
__device__ inline void lm_ctr(const SealCtx& c, const LdsTe& te, uint64_t row, uint32_t epoch, uint4 (&v)[8]) {
  constexpr int NB = GVS_SP_NB;
  // the row's high word and the lane's block offset are the same for every
  // chunk: left visible, the compiler hoisted the round-1 lookup addresses
  // that depend only on them out of the stream, and at 16 waves spilled them
  // (a scratch reload in front of every keystream)
  const uint64_t r = ((uint64_t)opaque((uint32_t)(row >> 32)) << 32) | opaque((uint32_t)row);
  const CtrRound1J c1 = ctr_round1_row(c.rk, te, 0u, r, epoch, opaque((lane_id() & 7u) * 8u));
  CtrRound2J c2{};
  if (GVS_SP_DUAL && GVS_SP_R2) c2 = ctr_round2_row(c.rk, te, c1);
#pragma unroll
  for (uint32_t i = 0; i < 8; i += NB) {
    uint4 ks[NB];
    if (GVS_SP_DUAL && GVS_SP_R2)
      ctr_keystream_jn3<NB>(c.rk, te, c2, i, ks);
    else if (GVS_SP_DUAL)
      ctr_keystream_jn2<NB>(c.rk, te, c1, i, ks);
    else
      ctr_keystream_jn<NB>(c.rk, te, c1, i, ks);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      v[i + b] = xor4(v[i + b], ks[b]);
      keep4(v[i + b]);  // XORed here, not sunk to the re-encryption with both keystreams held
    }
  }
}

// NW waves; every slot line of the partition staged in LDS (LB) or read and
// written in the stream (LB = false).
template <int NW, bool LB>
__global__ __launch_bounds__(64 * NW, 1) void k_spass(R2Args a) {
  constexpr uint32_t kLdsBytes = LB ? 65536u + (kSpBufs + 1u - kSpHoles) * 1024u : 65536u;
  constexpr uint32_t kShMax = LB ? kSpSlots : kSlotMax;
  GVS_TE_LDS s_lds[kLdsBytes / 4];              // AES window (table + holes), then buffers 32..kSpBufs
  __shared__ uint32_t s_pbm[kSpWords], s_cbm[kSpWords];  // rows the previous / this batch touches
  __shared__ uint32_t s_ppre[kSpWords], s_cpre[kSpWords];  // their counts before each word
  __shared__ uint32_t s_sh[kShMax];             // this batch's slot -> position of the row's first op
  __shared__ uint32_t s_np, s_ns, s_xt;
  __shared__ uint4 s_xw[NW * (kXepMax + 1) * 3];
  __shared__ uint4 s_xp[kXepMax * 3];
  __shared__ uint4 s_xx[kXepMax];
  __shared__ uint32_t s_xc[NW];
  __shared__ __attribute__((aligned(16))) uint32_t s_nh[kNhWords];  // the row hash's NH key
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t w = blockIdx.x;
  if (a.scal->error) return;
  if (GVS_SP_DUAL)
    load_te2(s_lds, a.te);
  else
    load_te(s_lds, a.te);
  for (uint32_t o = tid; o < kNhWords; o += 64 * NW) s_nh[o] = a.sc.nhk[o];
  const uint32_t nwd = a.S / 32u;
  for (uint32_t o = tid; o < nwd; o += 64 * NW) {
    s_pbm[o] = 0u;
    s_cbm[o] = 0u;
  }
  if (tid == 0) {
    s_np = 0;
    s_ns = 0;
    s_xt = 0;
  }
  __syncthreads();
  const uint64_t sbase = (uint64_t)w * a.c, rowbase = (uint64_t)w * a.S;
  // every slot descriptor of this partition, both batches, as whole lines (8
  // lanes each); each used previous slot's side entry must name its row
  uint32_t bad = 0u;
  for (uint32_t k0 = wave * 8; k0 < a.c; k0 += NW * 8) {
    const uint32_t k = k0 + (lane >> 3);
    const uint4 xp = a.tprev[(sbase + k) * 8 + (lane & 7u)];
    const uint4 xc = a.tcur[(sbase + k) * 8 + (lane & 7u)];
    const uint4 xs = a.psds[(sbase + k) * 8 + (lane & 7u)];
    const uint4 dp = shfl4(xp, (int)(lane & ~7u)), ds = shfl4(xc, (int)(lane & ~7u));
    const uint4 sd = shfl4(xs, (int)(lane & ~7u));
    if ((lane & 7u) == 0u) {
      const bool pu = dp.y == a.stamp_prev && dp.x < a.S;
      if (pu) {
        atomicOr(&s_pbm[dp.x >> 5], 1u << (dp.x & 31u));
        atomicAdd(&s_np, 1u);
      }
      bad |= (uint32_t)(pu & ((sd.z == 0u) | (u4lo(sd) != rowbase + dp.x)));
      s_sh[k] = ds.w;
      if (ds.y == a.stamp_cur && ds.x < a.S) {
        atomicOr(&s_cbm[ds.x >> 5], 1u << (ds.x & 31u));
        atomicAdd(&s_ns, 1u);
      }
    }
  }
  if (__ballot(bad != 0u) && lane == 0) atomicOr(&a.scal->error, 8u);  // a forged final-state target
  // the expiry deletes this batch already carries for this partition
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
  if (LB) {  // (1) every previous slot's final state into buffer k, used or not
    for (uint32_t k = wave; k < a.c; k += NW) {
      const uint4 x = ld_row<true>(&a.ps[(sbase + k) * 64 + lane]);
      sp_st(s_lds, sp_addr(k, lane >> 3, lane & 7u), x);
    }
  }
  __syncthreads();
  // prefix counts of the bitmaps (slot k = the k-th touched row in row order)
  for (uint32_t o = tid; o < nwd; o += 64 * NW) {
    uint32_t pp = 0, cp = 0;
    for (uint32_t j = 0; j < o; ++j) {
      pp += __popc(s_pbm[j]);
      cp += __popc(s_cbm[j]);
    }
    s_ppre[o] = pp;
    s_cpre[o] = cp;
  }
  __syncthreads();
  const uint32_t np = s_np, ns = s_ns;
  uint4* part = a.table + rowbase * 64;
  const LdsTe te = lds_te(s_lds);
  const uint32_t ngroups = a.S / 32u, rounds = (ngroups + NW - 1) / NW;
  const uint32_t u = lane >> 3, f = lane & 7u;
  for (uint32_t t = 0; t < rounds; ++t) {
    uint32_t xc = 0;
    const uint32_t g = t * NW + wave;
    if (g < ngroups) {
      // the group's header PRFs: lane l < 32 row g*32 + l at the read epoch,
      // lane 32 + l the same row at the write epoch; the pending flag of a
      // row comes from the slots of each batch
      const uint32_t pbits = s_pbm[g], cbits = s_cbm[g];
      uint64_t hh[2];
      {
        const uint32_t r = lane & 31u;
        const bool wr = lane >= 32u;
        const uint32_t bits = wr ? cbits : pbits;
        const uint32_t tab = ((bits >> r) & 1u) ? kPendTable : 0u;
        // H = AES-128_kh(le64(row) | le32(epoch) | le32(table)) (gvs_crypto.h
        // head_aes), one block per lane on the two LDS tables
        const uint64_t row = rowbase + g * 32u + r;
        const uint32_t ep = opaque(a.sc.epoch + (wr ? 1u : 0u));
        uint32_t hs[1][4] = {{bswap32((uint32_t)row) ^ a.sc.rkh.w[0], bswap32((uint32_t)(row >> 32)) ^ a.sc.rkh.w[1],
                              bswap32(ep) ^ a.sc.rkh.w[2], bswap32(tab) ^ a.sc.rkh.w[3]}};
        if (GVS_SP_DUAL)
          aes128_rounds_n2<1, 1>(a.sc.rkh, te, hs);
        else
          aes128_rounds_n<1, 1>(a.sc.rkh, te, hs);
        hh[0] = (uint64_t)bswap32(hs[0][0]) | ((uint64_t)bswap32(hs[0][1]) << 32);
        hh[1] = (uint64_t)bswap32(hs[0][2]) | ((uint64_t)bswap32(hs[0][3]) << 32);
      }
#pragma unroll 1
      for (uint32_t jj = 0; jj < 4; ++jj) {
        const uint32_t rj = g * 32u + jj * 8u;  // the chunk's first row in the partition
        const uint32_t rr = jj * 8u + u;        // the lane's row in the group
        uint4 v[8];
        uint4* tile = part + (uint64_t)rj * 64;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ld_row<true>(&tile[i * 64 + lane]);
        const uint4 tl = line_load(a.mtag + rowbase + rj);
        const uint64_t row = rowbase + rj + u;
        // (2) verify and decrypt at the read epoch
        {
          const uint64_t hr[2] = {shfl_u64(hh[0], (int)rr), shfl_u64(hh[1], (int)rr)};
          uint64_t tg[2];
          lm_tag(s_nh, a.sc, v, hr, tg);
          const uint4 want = shfl4(tl, (int)u);
          if (__ballot((u4lo(want) != tg[0]) | (u4hi(want) != tg[1])) && lane == 0)
            atomicOr(&a.scal->error, 8u);  // integrity failure: the batch and the handle are dead
          lm_ctr(a.sc, te, row, opaque(a.sc.epoch), v);
        }
        // (3) the previous batch's final state, this batch's snapshot
        const bool app = (pbits >> rr) & 1u, tch = (cbits >> rr) & 1u;
        const uint32_t pslot = s_ppre[g] + __popc(pbits & ((1u << rr) - 1u));
        const uint32_t cslot = s_cpre[g] + __popc(cbits & ((1u << rr) - 1u));
        if (LB) {
          const uint32_t bp = selu32(app, pslot, kSpDry), bs = selu32(tch, kSpBufs - 1u - cslot, kSpDry);
#pragma unroll
          for (uint32_t i = 0; i < 8; ++i) v[i] = sel4(app, sp_ld<LB>(s_lds, sp_addr(bp, f, i)), v[i]);
#pragma unroll
          for (uint32_t i = 0; i < 8; ++i) sp_st(s_lds, sp_addr(bs, f, i), v[i]);
        } else {
          if (app) {
            const uint4* src = a.ps + (sbase + pslot) * 64 + f * 8;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) v[i] = ld_row<true>(&src[i]);
          }
          if (tch) {
            const uint32_t hp = s_sh[min(cslot, kShMax - 1u)];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) st_drop(a.snapp, (uint64_t)hp * 64 + f * 8 + i, v[i]);
            if (f == 0u) {
#pragma unroll
              for (uint32_t i = 0; i < 8; ++i) st_drop(a.snapidp, (uint64_t)hp * 8 + i, v[i]);
            }
          }
        }
        if (a.xon) xc = x_detect_lm(a, v, s_xw + wave * (kXepMax + 1) * 3, xc, s_xx, nx);
        // (4) encrypt and tag at the write epoch, store
        {
          lm_ctr(a.sc, te, row, opaque(a.sc.epoch + 1u), v);
          const uint64_t hw[2] = {shfl_u64(hh[0], (int)(32u + rr)), shfl_u64(hh[1], (int)(32u + rr))};
          uint64_t tg[2];
          lm_tag(s_nh, a.sc, v, hw, tg);
          // lane r < 8 writes row r's tag: the 8 rows' tags are one whole line
          const uint64_t t0 = shfl_u64(tg[0], (int)(8u * (lane & 7u))), t1 = shfl_u64(tg[1], (int)(8u * (lane & 7u)));
          if (lane < 8u)
            a.mtag[rowbase + rj + lane] = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1,
                                                     (uint32_t)(t1 >> 32));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) st_row<true>(&tile[i * 64 + lane], v[i]);
      }
    }
    // the waves meet after every round: the expiry lists merge in row order
    if (lane == 0) s_xc[wave] = xc;
    __syncthreads();
    if (a.xon) {
      const uint32_t tot = x_merge2<NW>(a.xep, s_xw, s_xc, s_xp, s_xt);
      __syncthreads();
      if (tid == 0) s_xt = tot;
    }
  }
  __syncthreads();
  uint4* sslot = a.snap + sbase * 64;
  if (LB) {
    // (5) every slot's snapshot: the touched rows' to their first ops'
    // positions, the unused slots' (zero) to their sink lines
    for (uint32_t k = wave; k < a.c; k += NW) {
      const bool used = k < ns;
      const uint32_t hp = s_sh[k];
      const uint4 x = sel4(used, sp_ld<LB>(s_lds, sp_addr(kSpBufs - 1u - k, lane >> 3, lane & 7u)),
                           make_uint4(0, 0, 0, 0));
      st_drop(used ? a.snapp + (uint64_t)hp * 64 : sslot + (uint64_t)k * 64, lane, x);
      if (lane < 8) st_drop(used ? a.snapidp + (uint64_t)hp * 8 : a.snapid + (sbase + k) * 8, lane, x);
    }
  } else {
    // unused slots: every final-state line is read once per pass, every
    // unused slot's snapshot sink written once
    for (uint32_t k = np + wave; k < a.c; k += NW) {
      uint4 x = ld_row<true>(&a.ps[(sbase + k) * 64 + lane]);
      keep4(x);
    }
    for (uint32_t k = ns + wave; k < a.c; k += NW) {
      st_drop(sslot, (uint64_t)k * 64 + lane, make_uint4(0, 0, 0, 0));
      if (lane < 8) st_drop(a.snapid, (sbase + k) * 8 + lane, make_uint4(0, 0, 0, 0));
    }
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

// Before any state changes: a partition whose used slots over the previous
// and this batch exceed the staging buffers fails the batch (batch overflow,
// like a partition with more distinct rows than c).  One wave per partition,
// every descriptor line of both batches read whole.
__global__ __launch_bounds__(256) void k_sjoint(const uint4* tprev, const uint4* tcur, uint32_t stamp_prev,
                                                uint32_t stamp_cur, uint32_t W, uint32_t S, uint32_t c,
                                                uint32_t cap, Scal* scal) {
  if (scal->error) return;
  const uint32_t lane = lane_id(), w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= W) return;
  const uint64_t sbase = (uint64_t)w * c;
  uint32_t n = 0;
  for (uint32_t k0 = 0; k0 < c; k0 += 8) {
    const uint32_t k = k0 + (lane >> 3);
    const uint4 xp = tprev[(sbase + k) * 8 + (lane & 7u)];
    const uint4 xc = tcur[(sbase + k) * 8 + (lane & 7u)];
    const uint4 dp = shfl4(xp, (int)(lane & ~7u)), ds = shfl4(xc, (int)(lane & ~7u));
    const bool first = (lane & 7u) == 0u;
    n += (uint32_t)(first & (dp.y == stamp_prev) & (dp.x < S));
    n += (uint32_t)(first & (ds.y == stamp_cur) & (ds.x < S));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) n += (uint32_t)__shfl_xor((int)n, o);
  if (lane == 0 && n > cap) atomicOr(&scal->error, kJErr);
}

}  // namespace gvs
