// gvs_route.h — gfx950 kernels of the multi-shard request router.
//
// A sharded store keeps every message on the shard that owns its recipient's
// mailbox, so each request touches exactly one shard:
//   CREATE                      -> shard of the recipient
//   READ / DELETE with zero id  -> shard of auth_identity (its mailbox)
//   by-id READ / UPDATE / DELETE -> shard encoded in the id (tag bits)
//   malformed, zero recipient, undecodable id -> i mod S (answer is the same
//                                                on every shard)
// Each source rank packs its requests into S buckets of exactly C slots
// (stable: submission order is kept inside a bucket), pads the rest with
// zero requests (type 0, answered as hard errors) and exchanges the buckets
// all-to-all.  Slots are 1152 B (9 whole 128-B lines) so that no line is ever
// shared between two requests; every slot is written by one wave.  Sizes seen
// outside the device are S, C and B only.
//
// Hot keys [D] (DESIGN.md §6 "Hot keys"): a source routes at most kRouteKeyCap
// requests per routing key (the mailbox a create or a next-message op
// addresses, the id of a by-id op) in one window.  The later ones are shed:
// they travel as hard errors to the shard i mod S (spread like malformed
// requests, so they never load the hot key's shard) and the source answers
// them INTERNAL_ERROR (8) with the request's time.  One recipient can then put
// at most kRouteKeyCap requests of one kind into a bucket, so a hot key fails
// its own excess instead of the whole window.  The cap is shared by every
// client of the key: the requests past the first kRouteKeyCap to one mailbox
// or id in a window are shed whoever sent them (a client that floods a
// recipient also sheds other senders' creates to it in that window).  Keys
// are keyed hashes (SipHash with the store's recipient key), so a client
// cannot aim its requests at another mailbox's or id's key without naming it.
#pragma once
#include "gvs_device.h"

namespace gvs {

constexpr uint32_t kSlotU4 = kRespSlot / 16;  // 72 x 16 B per routed slot
constexpr uint32_t kAbiU4 = 65;               // gvs_request / gvs_response: 1040 B
constexpr uint32_t kShardsMax = 64;
constexpr uint32_t kRouteKeyCap = 64;  // requests routed per routing key, per source window
constexpr uint32_t kKeyNone = 0u;      // routing-key class of unkeyed requests (never shed)

struct RouteArgs {
  const uint4* in;   // caller requests (kAbiU4 stride)
  uint32_t n, B, S, C;
  uint32_t* dest;    // B
  uint64_t* rkey;    // B: routing key << 32 | index, sorted by the router (k_route_mark reads them)
  uint32_t* shed;    // B: 1 = shed (the key's cap was reached)
  uint32_t* bcnt;    // nblk * S: per-block per-shard counts
  uint32_t* pos;     // B: slot in `send`, or kNone
  uint32_t* tot;     // S: per-shard totals of this source
  uint4* send;       // S*C slots
  uint32_t* err;     // the local shard's error word (bit 2: route overflow)
  uint64_t N;
  KeyCtx kc;
};

// request i -> owning shard (S = padding, i >= n) and its 32-bit routing key
// (low 2 bits: 1 create, 2 next-message op, 3 by-id op, 0 unkeyed).  Host and
// device: the test library's gvs_route_plan runs this same function on the
// CPU; oracle/gvs_oracle.c gvo_route_key restates the key.
__host__ __device__ inline uint32_t route_dest_key(const RouteArgs& a, uint32_t i, uint32_t& key) {
  key = kKeyNone;
  if (i >= a.n) return a.S;
  const uint4* r = a.in + (uint64_t)i * kAbiU4;
  const uint4 c0 = r[0], c1 = r[1], c2 = r[2], c3 = r[3], c4 = r[4];
  const uint32_t type = r[64].x;
  const bool id_zero = !nz4(c0);
  const bool auth_zero = !nz4(c1) && !nz4(c2);
  const bool rcpt_zero = !nz4(c3) && !nz4(c4);
  const bool hard = type < 1u || type > 4u || auth_zero || (type == 3u && id_zero);
  const bool next = (type == 2u || type == 4u) && id_zero;
  const uint4 xa = next ? c1 : c3, xb = next ? c2 : c4;
  // every hash runs for every request (fixed work)
  const uint64_t x[4] = {u4lo(xa), u4hi(xa), u4lo(xb), u4hi(xb)};
  const uint64_t lo = siphash24_blocks(a.kc.hk0, a.kc.hk1, x, 4, 2, 33);
  const uint32_t by_key = shard_of_hash(lo, a.S);
  const uint32_t by_id = id_shard(a.kc, u4lo(c0), u4hi(c0), a.N);
  const uint32_t spread = i % a.S;
  const uint64_t idw[2] = {u4lo(c0), u4hi(c0)};
  const uint64_t hid = siphash24_blocks(a.kc.hk0, a.kc.hk1, idw, 2, 3, 17);  // id || 0x03
  const uint32_t kh = (uint32_t)(lo >> 32) & ~3u, ki = (uint32_t)(hid >> 32) & ~3u;
  // one selection for every kind (a branch per kind let the compiler sink the
  // id decode and the id hash into the by-id path, whose code a batch without
  // by-id ops then never fetched: FETCH_SIZE followed the mix)
  const bool create = type == 1u;
  const uint32_t d_cr = rcpt_zero ? spread : by_key;
  const uint32_t d_id = by_id != kNone ? by_id : spread;
  const uint32_t k_cr = rcpt_zero ? kKeyNone : (kh | 1u);
  uint32_t d = d_id, k = ki | 3u;
  d = next ? by_key : d;
  k = next ? (kh | 2u) : k;
  d = create ? d_cr : d;
  k = create ? k_cr : k;
  d = hard ? spread : d;
  k = hard ? kKeyNone : k;
  key = k;
  return d;
}

__host__ __device__ inline uint32_t route_dest(const RouteArgs& a, uint32_t i) {
  uint32_t key;
  return route_dest_key(a, i, key);
}

// dest and routing key of every request (padding: unkeyed)
__global__ __launch_bounds__(1024) void k_route_dest(RouteArgs a) {
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  uint32_t key;
  uint32_t d = route_dest_key(a, i, key);
  asm volatile("" : "+v"(d), "+v"(key));  // every request's selection computed in full
  a.dest[i] = d;
  a.rkey[i] = ((uint64_t)key << 32) | i;
}

// Over the keys sorted by (key, index): a request is shed when the request
// kRouteKeyCap places before it has the same key (it is at least the
// (kRouteKeyCap + 1)-th of its key in this window); a shed request goes to
// shard i mod S.  The flag is found at the sorted position and taken back to
// request order by a second sort (by index), not by a scatter:
//   * round 3 scattered 4-B writes by request index from many workgroups:
//     FETCH_SIZE followed the key order (DESIGN.md §3 rule 4);
//   * round 4 set bits of an LDS bitmap by request index in one workgroup:
//     a hot key's sorted run has dense request indices, so the wave's LDS
//     atomics met on few words and serialised, and the kernel ran 10-20 us
//     longer under the hot mixes (profiles/r05k_timing_c3_routed.txt).
// k_route_mark: sorted position j -> (index << 32 | shed), coalesced
__global__ __launch_bounds__(1024) void k_route_mark(RouteArgs a, uint64_t* marks) {
  const uint32_t j = blockIdx.x * 1024 + threadIdx.x;
  const uint64_t k = a.rkey[j];
  const uint64_t kp = a.rkey[j >= kRouteKeyCap ? j - kRouteKeyCap : j];
  const uint32_t key = (uint32_t)(k >> 32), i = (uint32_t)k;
  const bool shed = j >= kRouteKeyCap && (key & 3u) != kKeyNone && (uint32_t)(kp >> 32) == key;
  marks[j] = ((uint64_t)i << 32) | (shed ? 1u : 0u);
}

// after the marks are sorted (by index): shed flags and destinations in
// request order
__global__ __launch_bounds__(1024) void k_route_apply(RouteArgs a, const uint64_t* marks) {
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const bool shed = (marks[i] & 1u) != 0u;
  const uint32_t d = a.dest[i];
  a.shed[i] = shed ? 1u : 0u;
  a.dest[i] = shed ? i % a.S : d;
}

// per-block per-shard histogram of the final destinations (all S bins stored)
__global__ __launch_bounds__(1024) void k_route_hist(RouteArgs a) {
  __shared__ uint32_t s_h[kShardsMax];
  const uint32_t tid = threadIdx.x, i = blockIdx.x * 1024 + tid;
  if (tid < a.S) s_h[tid] = 0;
  __syncthreads();
  const uint32_t d = a.dest[i];
  if (d < a.S) atomicAdd(&s_h[d], 1u);
  __syncthreads();
  if (tid < a.S) a.bcnt[blockIdx.x * a.S + tid] = s_h[tid];
}

// stable slot of every request: bucket d, rank = earlier requests for d
__global__ __launch_bounds__(1024) void k_route_pos(RouteArgs a) {
  __shared__ uint32_t s_off[kShardsMax];
  __shared__ uint32_t s_wc[kShardsMax][16];
  __shared__ uint32_t s_over;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const uint32_t nblk = gridDim.x;
  if (tid < a.S) {
    uint32_t o = 0;
    for (uint32_t b = 0; b < blockIdx.x; ++b) o += a.bcnt[b * a.S + tid];
    s_off[tid] = o;
    if (blockIdx.x == nblk - 1) a.tot[tid] = o + a.bcnt[blockIdx.x * a.S + tid];
  }
  if (tid == 0) s_over = 0;
  const uint32_t i = blockIdx.x * 1024 + tid;
  const uint32_t d = a.dest[i];
  uint32_t in_wave = 0;
  for (uint32_t k = 0; k < a.S; ++k) {
    const uint64_t m = __ballot(d == k);
    if (d == k) in_wave = mbcnt64(m);
    if (lane == 0) s_wc[k][wave] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  uint32_t p = kNone;
  if (d < a.S) {
    uint32_t r = s_off[d] + in_wave;
    for (uint32_t w = 0; w < wave; ++w) r += s_wc[d][w];
    if (r < a.C) p = d * a.C + r;
    else atomicOr(&s_over, 1u);
  }
  a.pos[i] = p;
  __syncthreads();
  if (tid == 0) atomicOr(a.err, s_over ? 4u : 0u);  // one atomic per block, always
}

// one wave per request: its 1040 B into its slot (1152 B, whole lines)
__global__ __launch_bounds__(256) void k_route_copy(RouteArgs a) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (i >= a.n) return;
  const uint32_t p = a.pos[i];
  if (p == kNone) return;
  const uint4* src = a.in + (uint64_t)i * kAbiU4;
  uint4* dst = a.send + (uint64_t)p * kSlotU4;
  dst[lane] = src[lane];
  // a shed request travels as a hard error (type 0): the shard changes nothing
  const uint4 t = src[64];
  const uint32_t sh = a.shed[i];
  if (lane < 8) dst[64 + lane] = lane == 0 ? make_uint4(sh ? 0u : t.x, t.y, t.z, t.w) : make_uint4(0, 0, 0, 0);
}

// one wave per slot: zero-fill the slots no request took
__global__ __launch_bounds__(256) void k_route_fill(RouteArgs a) {
  const uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (j >= a.S * a.C) return;
  const uint32_t d = j / a.C, r = j % a.C;
  if (r < min(a.tot[d], a.C)) return;
  uint4* dst = a.send + (uint64_t)j * kSlotU4;
  const uint4 z = make_uint4(0, 0, 0, 0);
  dst[lane] = z;
  if (lane < 8) dst[64 + lane] = z;
}

// the responses (slot layout) back to the caller layout, kGatherPerWave
// requests per wave: 8 rows of 1040 B are 65 whole lines, so every output line
// is written by one wave, and by one store instruction (wave_put_rec8).  A shed request's response is INTERNAL_ERROR with the request's
// time: its shard's hard-error response and its request's time word are read
// for every request and selected, so every request reads the same lines.
constexpr uint32_t kGatherPerWave = 8;
__global__ __launch_bounds__(256) void k_route_gather(const uint32_t* __restrict__ pos,
                                                      const uint32_t* __restrict__ shed,
                                                      const uint4* __restrict__ in,
                                                      const uint4* __restrict__ back, uint32_t n,
                                                      uint4* __restrict__ out) {
  constexpr uint32_t R = kGatherPerWave;
  static_assert(R == 8, "wave_put_rec8");
  __shared__ uint4 s_rec[4][R * kAbiU4];
  __shared__ uint32_t s_pos[4 * R], s_shed[4 * R];
  const uint32_t i0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R, lane = lane_id();
  // the block's 32 positions and shed flags: their two 128-B lines read whole
  // by one instruction of wave 0 (the four waves' 32-B pieces, read by each
  // wave itself, were fetched in 32- or 64-B requests as their timing fell:
  // FETCH_SIZE +3.7 KiB under the all-miss and hot mixes, r05m)
  if (threadIdx.x < 64) {
    const uint32_t b = min(blockIdx.x * 4 * R + (lane & 31u), n - 1u);
    const uint32_t x = lane < 32 ? pos[b] : shed[b];
    if (lane < 32)
      s_pos[lane] = x;
    else
      s_shed[lane - 32] = x;
  }
  __syncthreads();
  if (i0 >= n) return;
  uint4 v[R], t = make_uint4(0, 0, 0, 0);  // t: lane r holds request r's status word
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {  // wave-uniform conditions
    const uint32_t i = min(i0 + r, n - 1u), il = i - blockIdx.x * 4 * R;
    const uint32_t p = s_pos[il];
    // an overflowed batch (p == kNone) fails as a whole; out is then undefined
    // the status word's and the time word's 128-B lines are each read whole,
    // by 8 lanes in one instruction, and the word taken by a shuffle: a 16-B
    // read of a line was fetched as 32 or 64 B depending on the requests in
    // flight, which follow the batch's routing (FETCH_SIZE -6..-28 KiB under
    // the hot mixes, profiles/r04ze_oblivious_FETCH_SIZE_routed.txt)
    v[r] = p != kNone ? back[(uint64_t)p * kSlotU4 + lane] : make_uint4(0, 0, 0, 0);
    const uint4 tl = p != kNone ? back[(uint64_t)p * kSlotU4 + 64 + (lane & 7u)] : make_uint4(0, 0, 0, 0);
    uint4 tw = shfl4(tl, 0);
    const uint64_t tsa = (uint64_t)i * kAbiU4 + 5;  // the request's server time (record word 5)
    const uint4 tsl = in[(tsa & ~7ull) + (lane & 7u)];
    uint4 ts = shfl4(tsl, (int)(tsa & 7u));
    // pinned: only shed requests use ts and only the others the slot, and the
    // compiler would otherwise load each under its condition (the time word's
    // line was then read once per shed request: FETCH_SIZE followed the mix)
    keep4(ts);
    keep4(v[r]);
    keep4(tw);
    const bool s = s_shed[il] != 0u;
    v[r] = sel4(s, sel4(lane == 5, make_uint4(ts.x, ts.y, 0u, 0u), make_uint4(0, 0, 0, 0)), v[r]);
    tw = sel4(s, make_uint4(8u, 0, 0, 0), tw);
    // a mask select: `lane == r ? tw[r] : t` over an array was compiled to a
    // select of addresses, which put the array in scratch (160 B per lane);
    // scratch lines written back or not with the timing moved FETCH_SIZE by
    // +-25 KiB (profiles/r05l_oblivious_FETCH_SIZE_routed.txt)
    t = sel4(lane == r, tw, t);
  }
  wave_put_rec8(out + (uint64_t)i0 * kAbiU4, s_rec[threadIdx.x >> 6], v, t, n - i0);
}

// single-process shards: OR of every shard's error word into each of them
struct ErrSet {
  uint32_t* e[kShardsMax];
  uint32_t n;
};
__global__ void k_err_or(ErrSet s) {
  if (threadIdx.x != 0) return;
  uint32_t v = 0;
  for (uint32_t k = 0; k < s.n; ++k) v |= *s.e[k];
  for (uint32_t k = 0; k < s.n; ++k) *s.e[k] = v;
}

}  // namespace gvs
