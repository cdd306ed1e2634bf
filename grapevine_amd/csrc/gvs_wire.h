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
// One wave per message.  Every wave reads its whole input slot (stride
// bytes) and writes its whole output slab, so the HBM traffic depends on n
// and the strides only; the field walk itself runs on the wave's LDS copy.
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
};

__device__ inline Varint varint_at(const uint8_t* m, uint32_t p, uint32_t lim) {
  Varint r{0, p, false};
  bool done = false;
#pragma unroll
  for (uint32_t c = 0; c < 10; ++c) {
    const uint32_t b = m[min(p + c, kWireSlotMax - 1u)];
    const bool take = !done && p + c < lim;
    r.v |= take ? (uint64_t)(b & 0x7Fu) << (7 * c) : 0ull;
    const bool last = take && b < 0x80u;
    r.ok = last ? !(c == 9 && b > 1u) : r.ok;
    r.next = last ? p + c + 1 : r.next;
    done = done || last || !take;
  }
  return r;
}

__global__ void __launch_bounds__(256) k_wire_decode(WireDecArgs a) {
  __shared__ uint8_t stage[4][kWireSlotMax];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t k = blockIdx.x * 4u + wv;
  const bool live = k < a.n;
  uint8_t* m = stage[wv];
  const uint8_t* src = a.in + (uint64_t)k * a.stride;
  if (live)
    for (uint32_t b = lane; b < a.stride; b += 64) m[b] = src[b];
  __syncthreads();
  if (!live) return;

  uint32_t len = a.lens[k];
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
    const Varint kv = varint_at(m, p, lim);
    const uint32_t wt = (uint32_t)(kv.v & 7u);
    const uint64_t tag = kv.v >> 3;
    const Varint vv = varint_at(m, kv.next, lim);
    const uint32_t q = min(kv.next, kWireSlotMax - 4u);
    const uint32_t fx = (uint32_t)m[q] | (uint32_t)m[q + 1] << 8 | (uint32_t)m[q + 2] << 16 |
                        (uint32_t)m[q + 3] << 24;
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
  const bool ok = st == kWireOk;
  if (!ok) o_id = o_auth = o_rc = o_pl = o_sig = 0;  // keep the reads inside the stage
  const uint64_t ts = a.times[k];

  // gvs_request: msg_id | auth_identity | recipient | timestamp | payload |
  // request_type | reserved.  Lane u writes 16-B unit u (lane 0 also unit 64).
  auto unit = [&](uint32_t u) -> uint4 {
    uint32_t wds[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t v = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t j = u * 16u + (uint32_t)q * 4u + (uint32_t)c;
        uint32_t byte;
        if (j < 16u) byte = m[o_id + j];
        else if (j < 48u) byte = m[o_auth + j - 16u];
        else if (j < 80u) byte = m[o_rc + j - 48u];
        else if (j < 88u) byte = (uint32_t)(ts >> (8u * (j - 80u))) & 0xFFu;
        else if (j < 1024u) byte = m[o_pl + j - 88u];
        else if (j < 1028u) byte = (rt >> (8u * (j - 1024u))) & 0xFFu;
        else byte = 0;
        v |= byte << (8 * c);
      }
      wds[q] = ok ? v : 0u;
    }
    return make_uint4(wds[0], wds[1], wds[2], wds[3]);
  };
  uint4* dst = a.out + (uint64_t)k * kAbiU4;
  dst[lane] = unit(lane);
  if (lane == 0) dst[64] = unit(64);
  if (a.sigs && lane < 4) {
    uint32_t wds[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t v = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) v |= (uint32_t)m[o_sig + lane * 16u + q * 4u + c] << (8 * c);
      wds[q] = ok ? v : 0u;
    }
    a.sigs[(uint64_t)k * 4u + lane] = make_uint4(wds[0], wds[1], wds[2], wds[3]);
  }
  if (a.status && lane == 0) a.status[k] = st;
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
  __shared__ uint8_t stage[4][kAbiU4 * 16];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t k = blockIdx.x * 4u + wv;
  const bool live = k < a.n;
  uint8_t* r = stage[wv];
  const uint4* src = a.in + (uint64_t)k * kAbiU4;
  if (live) {
    reinterpret_cast<uint4*>(r)[lane] = src[lane];
    if (lane == 0) reinterpret_cast<uint4*>(r)[64] = src[64];
  }
  __syncthreads();
  if (!live) return;
  const uint32_t status = *reinterpret_cast<const uint32_t*>(r + 1024);
  uint64_t ts = 0;
  for (int c = 0; c < 8; ++c) ts |= (uint64_t)r[80 + c] << (8 * c);
  const uint32_t t = ts ? 9u : 0u;
  const uint32_t reclen = 1025u + t;            // 1034 with a timestamp
  const uint32_t base = 89u + t;                // payload field header
  const uint32_t total = status ? base + 944u : 0u;
  uint8_t* dst = a.out + (uint64_t)k * a.stride;
  for (uint32_t j = lane; j < a.stride; j += 64) {
    uint32_t b;
    if (j == 0) b = 0x0A;
    else if (j == 1) b = (reclen & 0x7Fu) | 0x80u;
    else if (j == 2) b = reclen >> 7;
    else if (j == 3) b = 0x0A;
    else if (j == 4) b = 0x10;
    else if (j < 21) b = r[j - 5];               // msg_id
    else if (j == 21) b = 0x12;
    else if (j == 22) b = 0x20;
    else if (j < 55) b = r[16 + j - 23];         // sender
    else if (j == 55) b = 0x1A;
    else if (j == 56) b = 0x20;
    else if (j < 89) b = r[48 + j - 57];         // recipient
    else if (t && j == 89) b = 0x21;
    else if (t && j < 98) b = r[80 + j - 90];    // timestamp
    else if (j == base) b = 0x2A;
    else if (j == base + 1) b = 0xA8;
    else if (j == base + 2) b = 0x07;
    else if (j < base + 939) b = r[88 + j - base - 3];  // payload
    else if (j == base + 939) b = 0x15;
    else if (j < base + 944) b = r[1024 + j - base - 940];  // status_code
    else b = 0;
    dst[j] = (uint8_t)(j < total ? b : 0u);
  }
  if (lane == 0) a.lens[k] = total;
}

}  // namespace gvs
