// sr_host.cpp — the field, curve and scalar arithmetic of the device
// signature check (grapevine_amd/csrc/gvs_sr25519.h, host-callable), built
// for the CPU so that tests/test_sr_host.py can check it against the oracle
// (oracle/sr25519.py) without a GPU.  Test infrastructure only.
#include "../grapevine_amd/csrc/gvs_sr25519.h"

#include <cstring>

using namespace gvs::sr;

static Fe fe_from(const uint8_t* b) {
  Fe r;
  for (int i = 0; i < 8; ++i)
    r.v[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 |
             (uint32_t)b[4 * i + 3] << 24;
  return r;
}

static void fe_to(const Fe& f, uint8_t* b) {
  for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(f.v[i / 4] >> (8 * (i % 4)));
}

extern "C" {

// out = encode(s*B - k*A) with A = decode(pk); returns decode's verdict (1 ok)
int sr_host_combine(const uint8_t* s, const uint8_t* k, const uint8_t* pk, uint8_t* out) {
  uint32_t ok = 0;
  const Pt A = ristretto_decode(fe_from(pk), &ok);
  fe_to(ristretto_encode(double_scalar_mul_host(fe_from(s), fe_from(k), A)), out);
  return ok ? 1 : 0;
}

// decode then re-encode; returns the verdict
int sr_host_roundtrip(const uint8_t* in, uint8_t* out) {
  uint32_t ok = 0;
  const Pt p = ristretto_decode(fe_from(in), &ok);
  fe_to(ristretto_encode(p), out);
  return ok ? 1 : 0;
}

// 64-byte little-endian integer mod l
void sr_host_reduce_wide(const uint8_t* in, uint8_t* out) {
  uint32_t w[16];
  for (int i = 0; i < 16; ++i) {
    w[i] = 0;
    for (int c = 0; c < 4; ++c) w[i] |= (uint32_t)in[4 * i + c] << (8 * c);
  }
  fe_to(sc_reduce_wide(w, 1), out);
}

// a*b and a^2 mod p, canonical
void sr_host_mul(const uint8_t* a, const uint8_t* b, uint8_t* prod, uint8_t* sq) {
  fe_to(fe_canon(fe_mul(fe_from(a), fe_from(b))), prod);
  fe_to(fe_canon(fe_sq(fe_from(a))), sq);
}
}
