// gvs_wire.h — gfx950 kernels of the batched wire codec (SURVEY.md §8(f)
// rank 1): protobuf QueryRequest bytes -> gvs_request slabs in front of the
// store, gvs_response slabs -> protobuf QueryResponse bytes behind it.
//
// Messages: api/proto/grapevine.proto:123-176, the prost structs of
// types/src/lib.rs:27-120 (QueryRequest {1: fixed32 request_type, 2: bytes
// auth_identity, 3: bytes auth_signature, 4: RequestRecord {1: msg_id,
// 2: recipient, 3: payload}}; QueryResponse {1: Record {1: msg_id, 2: sender,
// 3: recipient, 4: fixed64 timestamp, 5: payload}, 2: fixed32 status_code}).
// A fully populated request is 1099 B and a response with nonzero timestamp
// and status 1042 B (api/tests/grapevine_types.rs:22-31,46-55).
//
// Decoding follows prost's rules, so any encoding prost accepts decodes the
// same way, not only the canonical 1099-B layout:
//   * keys and lengths are varints of at most 10 bytes (the 10th <= 1); a key
//     above 2^32 - 1, field number 0 or wire type 6/7 is an error;
//   * a known field with another wire type is an error; unknown fields are
//     skipped (varint, fixed64, length-delimited, fixed32);
//   * scalars and bytes: the last occurrence wins; the embedded RequestRecord
//     is MERGED over all its occurrences (field by field, last wins);
//   * a length or fixed field running past its message (or past the
//     embedded record's end) is an error.
//   [D] Groups (wire types 3/4) are rejected; prost would skip an unknown
//   group.  No grapevine client emits them.  [D] So is a message that needs
//   more than kWireSteps field steps (fixed-work decoding, below).
// A message that fails to decode, or whose fields do not have the sizes the
// handler requires (auth_identity 32, auth_signature 64, msg_id 16,
// recipient 32, payload 936), becomes a request of type 0: the store answers
// it as a hard error, which the handler turns into a gRPC error
// (grapevine.proto:57-64).  Encoding writes the proto3 bytes prost would
// write; a hard-error response (status 0) has length 0.
//
// Decode: one wave per kWireMsgs messages, staged whole in LDS, one lane's
// field walk per message; encode: one wave per message.  Every message's
// whole input slot (stride bytes) is read and its whole output slab written,
// so the HBM traffic depends on n and the strides only.
#pragma once
#include "gvs_device.h"
#include "gvs_route.h"

namespace gvs {

constexpr uint32_t kWireReq = 1099;       // canonical QueryRequest
constexpr uint32_t kWireResp = 1042;      // canonical QueryResponse
constexpr uint32_t kWireSlotMax = 2048;   // largest slot stride (LDS stage per wave)
constexpr uint32_t kWirePayload = 936;    // README.md:148

// per-message decode status (gvs_wire_decode_device)
constexpr uint32_t kWireOk = 0, kWireDecodeError = 1, kWireBadField = 2;

struct WireDecArgs {
  const uint8_t* in;       // n slots of `stride` bytes
  uint32_t stride, n;
  const uint32_t* lens;    // message k has lens[k] <= stride bytes
  const uint64_t* times;   // server time per request
  uint4* out;              // gvs_request[n]
  uint4* sigs;             // n x 64 B (may be null)
  uint32_t* status;        // n (may be null)
};

// A field walk over the wave's LDS copy.  All lanes run it on the same bytes,
// so every value below is wave-uniform.  The walk takes exactly kWireSteps
// steps whatever the message holds (a step parses one field, leaves an
// embedded record, or idles once the message is done), and each step reads a
// fixed number of bytes with selects, so a batch's decode time does not depend
// on its messages.  [D] A message that needs more steps (fields + embedded
// records + 1) is a decode error; prost has no such bound (a canonical
// request needs 9).
constexpr int kWireSteps = 32;

struct Varint {
  uint64_t v;
  uint32_t next;  // position after the varint
  bool ok;        // prost decode_varint accepts it (at most 10 bytes, the 10th <= 1, inside lim)
  uint32_t w0;    // the 4 bytes at the varint's start (a fixed32 read at the same place)
};

// Encode stage: one slot plus slack for the 5-dword window reads.
constexpr uint32_t kWireStage = kWireSlotMax + 32;

// 16 bytes at byte offset p of a dword-aligned LDS stage: five aligned dword
// reads and byte funnel shifts (no byte loads, no divergence).
__device__ inline uint4 lds_bytes16(const uint8_t* m, uint32_t p) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(m) + (p >> 2);
  const uint32_t sh = p & 3u, d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
  return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                    __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
}

// The 7-bit groups of 8 varint bytes, packed (56 bits).
__device__ inline uint64_t varint_pack8(uint64_t w) {
  uint64_t y = w & 0x7f7f7f7f7f7f7f7full;
  y = (y & 0x007f007f007f007full) | ((y >> 1) & 0x3f803f803f803f80ull);
  y = (y & 0x00003fff00003fffull) | ((y >> 2) & 0x0fffc0000fffc000ull);
  y = (y & 0x000000000fffffffull) | ((y >> 4) & 0x00fffffff0000000ull);
  return y;
}

// The varint at message offset p (bytes at or past lim do not count) of the
// message at byte `base` of the stage, from one 16-byte window: the
// terminator is the first byte below 0x80, found with a mask over 8 bytes at
// once; bytes 9 and 10 are handled apart.  Same results as a byte-by-byte
// decode, in a fixed instruction count.
__device__ inline Varint varint_at(const uint8_t* m, uint32_t base, uint32_t p, uint32_t lim) {
  const uint4 win = lds_bytes16(m, base + p);
  const uint64_t w = (uint64_t)win.y << 32 | win.x;
  const uint32_t b8 = win.z & 0xFFu, b9 = (win.z >> 8) & 0xFFu;
  const uint32_t n = lim > p ? lim - p : 0u;  // bytes inside the limit
  const uint64_t inlim = n >= 8u ? ~0ull : ((1ull << (8u * n)) - 1ull);
  const uint64_t term = ~w & 0x8080808080808080ull & inlim;
  const uint32_t i = term ? (uint32_t)__builtin_ctzll(term) >> 3 : 8u;  // first terminator (8: none)
  const uint64_t keep = i >= 7u ? ~0ull : ((1ull << (8u * (i + 1u))) - 1ull);
  const uint64_t lo = varint_pack8(w & keep);
  const bool t8 = i == 8u && n >= 9u && b8 < 0x80u;
  const bool t9 = i == 8u && !t8 && n >= 10u && b8 >= 0x80u && b9 < 0x80u;
  Varint r;
  r.v = lo | (i == 8u ? (uint64_t)(b8 & 0x7Fu) << 56 : 0ull) | (t9 ? (uint64_t)(b9 & 1u) << 63 : 0ull);
  r.ok = i < 8u || t8 || (t9 && b9 <= 1u);
  r.next = i < 8u ? p + i + 1u : (t8 ? p + 9u : (t9 ? p + 10u : p));
  r.w0 = win.x;
  return r;
}

// Messages per decode workgroup (one wave): the wave stages its messages'
// slots in LDS as one contiguous copy, each lane walks one message, then the
// whole wave assembles each message's gvs_request in turn.
constexpr uint32_t kWireMsgs = 32;

// LDS bytes of one decode workgroup at slot stride `stride`.
inline uint32_t wire_decode_lds(uint32_t stride) { return (kWireMsgs * stride + 32u + 15u) & ~15u; }

__global__ void __launch_bounds__(64) k_wire_decode(WireDecArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t m[];
  const uint32_t lane = threadIdx.x;
  const uint32_t k0 = blockIdx.x * kWireMsgs;
  const uint32_t nm = min(kWireMsgs, a.n - k0);  // messages of this wave
  {
    // the wave's slots are contiguous in HBM and in the stage: 16 B per lane
    // when the slots are 16-B aligned (the usual strides), else 4 B, else
    // bytes (a kernel-wide choice)
    const uint8_t* src = a.in + (uint64_t)k0 * a.stride;
    const uint32_t total = nm * a.stride;
    const uintptr_t al = reinterpret_cast<uintptr_t>(a.in) | a.stride;
    if ((al & 15u) == 0) {
      for (uint32_t b = lane * 16u; b < total; b += 1024u)
        *reinterpret_cast<uint4*>(m + b) = *reinterpret_cast<const uint4*>(src + b);
    } else if ((al & 3u) == 0) {
      for (uint32_t b = lane * 4u; b < total; b += 256u)
        *reinterpret_cast<uint32_t*>(m + b) = *reinterpret_cast<const uint32_t*>(src + b);
    } else {
      for (uint32_t b = lane; b < total; b += 64u) m[b] = src[b];
    }
  }
  __syncthreads();

  // lane i < nm walks message k0 + i; the other lanes walk an empty message
  const bool mine = lane < nm;
  const uint32_t k = k0 + (mine ? lane : 0u);
  const uint32_t base = mine ? lane * a.stride : 0u;
  uint32_t len = mine ? a.lens[k] : 0u;
  bool err = len > a.stride;
  len = err ? 0u : len;
  // last offset and length of each field (length kNone: absent)
  uint32_t rt = 0;
  uint32_t o_auth = 0, l_auth = kNone, o_sig = 0, l_sig = kNone;
  uint32_t o_id = 0, l_id = kNone, o_rc = 0, l_rc = kNone, o_pl = 0, l_pl = kNone;
  uint32_t p = 0, depth = 0, nend = 0;
  bool done = false;
  for (int step = 0; step < kWireSteps; ++step) {
    const bool idle = done || err;
    const uint32_t lim = depth ? nend : len;
    const bool at_end = p == lim;
    const bool pop = !idle && at_end && depth;
    done = done || (!idle && at_end && !depth);
    const bool field = !idle && !at_end;
    // the key, then the varint / fixed / length that follows it (all read)
    const Varint kv = varint_at(m, base, p, lim);
    const uint32_t wt = (uint32_t)(kv.v & 7u);
    const uint64_t tag = kv.v >> 3;
    const Varint vv = varint_at(m, base, kv.next, lim);
    const uint32_t fx = vv.w0;  // a fixed32 at kv.next
    const bool known = depth ? (tag >= 1 && tag <= 3) : (tag >= 1 && tag <= 4);
    const uint32_t want = (!depth && tag == 1) ? 5u : 2u;
    const uint32_t sz = wt == 1 ? 8u : 4u;
    bool bad = !kv.ok || kv.v > 0xFFFFFFFFull || tag == 0 || wt == 3 || wt == 4 || wt > 5 ||
               (known && wt != want);
    bad = bad || (wt == 0 && !vv.ok) || ((wt == 1 || wt == 5) && lim - kv.next < sz) ||
          (wt == 2 && (!vv.ok || vv.v > lim - vv.next));
    err = err || (field && bad);
    const bool apply = field && !bad;
    const uint32_t L = (uint32_t)vv.v, body = vv.next;
    const bool rec = apply && known && !depth && tag == 4;  // RequestRecord: merge its fields
    const bool ldk = apply && known && wt == 2 && !rec;
    rt = (apply && known && wt == 5) ? fx : rt;
    o_auth = (ldk && !depth && tag == 2) ? body : o_auth;
    l_auth = (ldk && !depth && tag == 2) ? L : l_auth;
    o_sig = (ldk && !depth && tag == 3) ? body : o_sig;
    l_sig = (ldk && !depth && tag == 3) ? L : l_sig;
    o_id = (ldk && depth && tag == 1) ? body : o_id;
    l_id = (ldk && depth && tag == 1) ? L : l_id;
    o_rc = (ldk && depth && tag == 2) ? body : o_rc;
    l_rc = (ldk && depth && tag == 2) ? L : l_rc;
    o_pl = (ldk && depth && tag == 3) ? body : o_pl;
    l_pl = (ldk && depth && tag == 3) ? L : l_pl;
    const uint32_t np = wt == 0 ? vv.next : (wt == 2 ? body + L : kv.next + sz);
    p = apply ? (rec ? body : np) : p;
    nend = rec ? body + L : nend;
    depth = rec ? 1u : (pop ? 0u : depth);
  }
  err = err || !done;
  const bool sizes = l_auth == 32u && l_sig == 64u && l_id == 16u && l_rc == 32u &&
                     l_pl == kWirePayload;
  const uint32_t st = err ? kWireDecodeError : (sizes ? kWireOk : kWireBadField);
  // stage positions of the fields (a failed message reads its own slot start;
  // the reads stay inside the stage, the values are not used)
  const bool ok = st == kWireOk;
  o_id = base + (ok ? o_id : 0u);
  o_auth = base + (ok ? o_auth : 0u);
  o_rc = base + (ok ? o_rc : 0u);
  o_pl = base + (ok ? o_pl : 0u);
  o_sig = base + (ok ? o_sig : 0u);
  const uint64_t ts = mine ? a.times[k] : 0ull;

  // gvs_request: msg_id | auth_identity | recipient | timestamp | payload |
  // request_type | reserved.  For each message in turn, lane u writes 16-B
  // unit u (lane 0 also unit 64): unit 0 is msg_id, 1-2 auth_identity, 3-4
  // recipient, 5 the timestamp and payload bytes 0-7, 6-63 payload bytes
  // 16u-88 on; 64 request_type.
  const uint32_t u = lane;
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (uint32_t i = 0; i < nm; ++i) {
    const uint32_t st_i = __builtin_amdgcn_readlane(st, i);
    const bool ok_i = st_i == kWireOk;
    const uint32_t id_i = __builtin_amdgcn_readlane(o_id, i);
    const uint32_t au_i = __builtin_amdgcn_readlane(o_auth, i);
    const uint32_t rc_i = __builtin_amdgcn_readlane(o_rc, i);
    const uint32_t pl_i = __builtin_amdgcn_readlane(o_pl, i);
    const uint32_t sg_i = __builtin_amdgcn_readlane(o_sig, i);
    const uint32_t rt_i = __builtin_amdgcn_readlane(rt, i);
    const uint32_t tlo = __builtin_amdgcn_readlane((uint32_t)ts, i);
    const uint32_t thi = __builtin_amdgcn_readlane((uint32_t)(ts >> 32), i);
    const uint32_t at = u == 0 ? id_i
                      : u <= 2 ? au_i + 16u * (u - 1u)
                      : u <= 4 ? rc_i + 16u * (u - 3u)
                      : u == 5 ? pl_i : pl_i + 16u * u - 88u;
    uint4 v = lds_bytes16(m, at);
    // mask selects: a `c ? x : y` over uint4 values was compiled to a select
    // of their addresses, with the values in scratch (64 B per lane)
    v = sel4(u == 5, make_uint4(tlo, thi, v.x, v.y), v);
    uint4* dst = a.out + (uint64_t)(k0 + i) * kAbiU4;
    dst[lane] = sel4(ok_i, v, z);
    if (lane == 0) dst[64] = sel4(ok_i, make_uint4(rt_i, 0, 0, 0), z);
    if (a.sigs && lane < 4) {
      const uint4 sg = lds_bytes16(m, sg_i + 16u * lane);
      a.sigs[(uint64_t)(k0 + i) * 4u + lane] = sel4(ok_i, sg, z);
    }
  }
  if (a.status && mine) a.status[k] = st;
}

struct WireEncArgs {
  const uint4* in;   // gvs_response[n]
  uint32_t n, stride;
  uint8_t* out;      // n slabs of `stride` bytes
  uint32_t* lens;    // n: encoded length (0: hard error)
};

// QueryResponse as prost writes it: record {1: msg_id, 2: sender,
// 3: recipient, 4: timestamp (omitted when 0), 5: payload}, then status_code
// (2).  Status 0 (a hard error) has no response message: length 0, zero bytes.
__global__ void __launch_bounds__(256) k_wire_encode(WireEncArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4][kAbiU4 * 16 + 16];
  __shared__ __attribute__((aligned(16))) uint8_t image[4][kWireStage];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t k = blockIdx.x * 4u + wv;
  const bool live = k < a.n;
  uint8_t* r = stage[wv];
  uint8_t* im = image[wv];
  const uint32_t* r32 = reinterpret_cast<const uint32_t*>(r);
  const uint4* src = a.in + (uint64_t)k * kAbiU4;
  if (live) {
    reinterpret_cast<uint4*>(r)[lane] = src[lane];
    if (lane == 0) reinterpret_cast<uint4*>(r)[64] = src[64];
  }
  __syncthreads();
  uint32_t total = 0;
  if (live) {
    // the response slab as prost writes it, built in LDS a dword per lane
    const uint32_t status = r32[256];
    const uint64_t ts = (uint64_t)r32[21] << 32 | r32[20];
    const uint32_t t = ts ? 9u : 0u;
    const uint32_t reclen = 1025u + t;            // 1034 with a timestamp
    const uint32_t base = 89u + t;                // payload field header
    const uint32_t e = base + 939u;               // status_code field
    const uint32_t delta = base + 3u - 88u;       // payload: out[j] = r[j - delta]
    total = status ? base + 944u : 0u;
    auto hdr_byte = [&](uint32_t j) -> uint32_t {  // bytes 0-127: fields before the payload body
      if (j == 0) return 0x0A;
      if (j == 1) return (reclen & 0x7Fu) | 0x80u;
      if (j == 2) return reclen >> 7;
      if (j == 3) return 0x0A;
      if (j == 4) return 0x10;
      if (j < 21) return r[j - 5];                // msg_id
      if (j == 21) return 0x12;
      if (j == 22) return 0x20;
      if (j < 55) return r[16 + j - 23];          // sender
      if (j == 55) return 0x1A;
      if (j == 56) return 0x20;
      if (j < 89) return r[48 + j - 57];          // recipient
      if (t && j == 89) return 0x21;
      if (t && j < 98) return r[80 + j - 90];     // timestamp
      if (j == base) return 0x2A;
      if (j == base + 1) return 0xA8;
      if (j == base + 2) return 0x07;
      return r[j - delta];                        // payload
    };
    const uint32_t nd = (a.stride + 3u) >> 2;
    for (uint32_t i = lane; i < nd; i += 64u) {
      const uint32_t j = 4u * i;
      uint32_t w = 0;
      if (j < 128u) {
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c) w |= (j + c < total ? hdr_byte(j + c) : 0u) << (8 * c);
      } else {
        // payload bytes, then the status_code field (0x15 + fixed32), then zeros
        const uint32_t o = min(j - delta, 1024u);
        const uint32_t pay = __builtin_amdgcn_alignbyte(r32[(o >> 2) + 1], r32[o >> 2], o & 3u);
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c) {
          const uint32_t jj = j + c, x = jj - e;
          const uint32_t tb = x == 0 ? 0x15u : (status >> (8u * (x - 1u))) & 0xFFu;
          const uint32_t b = jj < e ? (pay >> (8 * c)) & 0xFFu : tb;
          w |= (jj < total ? b : 0u) << (8 * c);
        }
      }
      reinterpret_cast<uint32_t*>(im)[i] = w;
    }
  }
  __syncthreads();
  if (!live) return;
  // slab -> output slot: head bytes to a 4-B boundary, dwords, tail bytes
  uint8_t* dst = a.out + (uint64_t)k * a.stride;
  const uint32_t h = (4u - (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u;
  const uint32_t nb = (a.stride - h) >> 2, t0 = h + 4u * nb;
  const uint32_t* im32 = reinterpret_cast<const uint32_t*>(im);
  if (lane < h) dst[lane] = im[lane];
  for (uint32_t i = lane; i < nb; i += 64u) {
    const uint32_t o = h + 4u * i;
    *reinterpret_cast<uint32_t*>(dst + o) = __builtin_amdgcn_alignbyte(im32[(o >> 2) + 1], im32[o >> 2], o & 3u);
  }
  if (t0 + lane < a.stride) dst[t0 + lane] = im[t0 + lane];
  if (lane == 0) a.lens[k] = total;
}

}  // namespace gvs
