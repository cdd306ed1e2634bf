// gvs_sr25519.h — gfx950 kernel of grapevine's challenge check (SURVEY.md
// §8(f) rank 3): schnorrkel signatures over ristretto255, verified in batch
// before the store sees the requests.
//
// Reference: README.md:187-200 (each request carries a signature over a
// 32-byte challenge under the signing context "grapevine-challenge",
// types/src/lib.rs:13; mc-crypto-keys' sign_schnorrkel / verify).  The crates
// (schnorrkel, merlin, curve25519-dalek) are absent from the reference; the
// algorithm below is restated in oracle/sr25519.py (test infrastructure,
// pinned to SHAKE128, merlin's published vector, RFC 9496 and openssl
// Ed25519) and checked against it bit for bit by tests/test_gpu_sr25519.py.
//
// Verify(pk, msg, sig = R || s):
//   s's top bit (schnorrkel's marker) set, s < l, pk a canonical ristretto
//   encoding; t = merlin Transcript("SigningContext") + (b"", context) +
//   ("sign-bytes", msg) + ("proto-name", "Schnorr-sig") + ("sign:pk", pk) +
//   ("sign:R", R); k = challenge_bytes("sign:c", 64) mod l;
//   accept iff encode(s*B - k*A) == R.
//
// One thread per signature.  Field elements are 8 x 32-bit limbs kept below
// 2^256 (lazy: reduced to [0, p) only for comparisons and encodings), products
// schoolbook with 64-bit multiply-adds and a 2^256 = 38 fold.  The scalar
// multiplication runs fixed signed radix-8 windows over both scalars
// (Straus: 252 doublings, 170 additions) with masked table selects; the
// transcript's STROBE state, then the per-signature table, live in LDS (one
// column per thread).  No branch depends on the signature,
// key or message: every thread runs the same instruction stream.
#pragma once
#include "gvs_device.h"

namespace gvs {
namespace sr {

#define GVS_SR_FN __host__ __device__ __forceinline__
// the larger steps (each called once per signature): inlined too.  Out of
// line, their reference arguments, out-parameters and point returns lived in
// scratch (80 B per lane, tests/test_code_object.py); inlined, the kernel has
// none, at the same registers and occupancy
#define GVS_SR_FN_NI __host__ __device__ __forceinline__

struct Fe {
  uint32_t v[8];
};

GVS_SR_FN Fe fe_k(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4,
                                   uint32_t a5, uint32_t a6, uint32_t a7) {
  Fe r;
  r.v[0] = a0, r.v[1] = a1, r.v[2] = a2, r.v[3] = a3;
  r.v[4] = a4, r.v[5] = a5, r.v[6] = a6, r.v[7] = a7;
  return r;
}

GVS_SR_FN Fe fe_zero() { return fe_k(0, 0, 0, 0, 0, 0, 0, 0); }
GVS_SR_FN Fe fe_one() { return fe_k(1, 0, 0, 0, 0, 0, 0, 0); }
GVS_SR_FN Fe fe_p() {
  return fe_k(0xFFFFFFEDu, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, 0x7FFFFFFFu);
}
// edwards25519 / ristretto255 constants (oracle/sr25519.py)
GVS_SR_FN Fe fe_d2() {
  return fe_k(0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au, 0xeef3d130u, 0x198e80f2u,
              0x56dffce7u, 0x2406d9dcu);
}
GVS_SR_FN Fe fe_d() {
  return fe_k(0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u,
              0x2b6ffe73u, 0x52036ceeu);
}
GVS_SR_FN Fe fe_sqrt_m1() {
  return fe_k(0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u,
              0x4fc1df0bu, 0x2b832480u);
}
GVS_SR_FN Fe fe_invsqrt_a_minus_d() {
  return fe_k(0x805d40eau, 0x99c8fdaau, 0x5a4172beu, 0x9d2f1617u, 0xfe01d840u, 0x16c27b91u,
              0xcfaffca2u, 0x786c8905u);
}

// r += 38 * c (c small), carried through; returns the carry out
GVS_SR_FN uint32_t fe_add_small(Fe& r, uint32_t c) {
  uint64_t x = (uint64_t)r.v[0] + c;
  r.v[0] = (uint32_t)x;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    x = (uint64_t)r.v[i] + (x >> 32);
    r.v[i] = (uint32_t)x;
  }
  return (uint32_t)(x >> 32);
}

// r -= c (c small), borrowed through; returns the borrow out
GVS_SR_FN uint32_t fe_sub_small(Fe& r, uint32_t c) {
  uint64_t x = (uint64_t)r.v[0] - c;
  r.v[0] = (uint32_t)x;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    x = (uint64_t)r.v[i] - ((x >> 32) & 1u);
    r.v[i] = (uint32_t)x;
  }
  return (uint32_t)(x >> 32) & 1u;
}

GVS_SR_FN Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x = (uint64_t)a.v[i] + b.v[i] + (x >> 32);
    r.v[i] = (uint32_t)x;
  }
  uint32_t c = fe_add_small(r, (uint32_t)(x >> 32) * 38u);  // 2^256 = 38 (mod p)
  (void)fe_add_small(r, c * 38u);
  return r;
}

GVS_SR_FN Fe fe_sub(const Fe& a, const Fe& b) {
  Fe r;
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x = (uint64_t)a.v[i] - b.v[i] - ((x >> 32) & 1u);
    r.v[i] = (uint32_t)x;
  }
  uint32_t bw = fe_sub_small(r, ((uint32_t)(x >> 32) & 1u) * 38u);
  (void)fe_sub_small(r, bw * 38u);
  return r;
}

GVS_SR_FN Fe fe_neg(const Fe& a) { return fe_sub(fe_zero(), a); }

GVS_SR_FN Fe fe_mul(const Fe& a, const Fe& b) {
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t x = (uint64_t)a.v[i] * b.v[j] + t[i + j] + c;
      t[i + j] = (uint32_t)x;
      c = x >> 32;
    }
    t[i + 8] = (uint32_t)c;
  }
  Fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t x = (uint64_t)t[8 + i] * 38u + t[i] + c;
    r.v[i] = (uint32_t)x;
    c = x >> 32;
  }
  const uint32_t c2 = fe_add_small(r, (uint32_t)c * 38u);
  (void)fe_add_small(r, c2 * 38u);
  return r;
}

// a^2: the 28 cross products once, doubled, plus the 8 squares (36 multiply-
// adds against fe_mul's 64)
GVS_SR_FN Fe fe_sq(const Fe& a) {
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; ++j) {
      const uint64_t x = (uint64_t)a.v[i] * a.v[j] + t[i + j] + c;
      t[i + j] = (uint32_t)x;
      c = x >> 32;
    }
    t[i + 8] = (uint32_t)c;
  }
  uint32_t top = 0;  // cross terms < 2^511: doubling fits
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t nt = t[k] >> 31;
    t[k] = (t[k] << 1) | top;
    top = nt;
  }
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t x = (uint64_t)a.v[i] * a.v[i] + t[2 * i] + c;
    t[2 * i] = (uint32_t)x;
    const uint64_t y = (uint64_t)t[2 * i + 1] + (x >> 32);
    t[2 * i + 1] = (uint32_t)y;
    c = y >> 32;
  }
  Fe r;
  c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t x = (uint64_t)t[8 + i] * 38u + t[i] + c;
    r.v[i] = (uint32_t)x;
    c = x >> 32;
  }
  const uint32_t c2 = fe_add_small(r, (uint32_t)c * 38u);
  (void)fe_add_small(r, c2 * 38u);
  return r;
}

GVS_SR_FN Fe fe_sqn(Fe a, int n) {
  for (int i = 0; i < n; ++i) a = fe_sq(a);
  return a;
}

GVS_SR_FN Fe fe_select(uint32_t m, const Fe& a, const Fe& b) {  // m ? a : b
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = (a.v[i] & m) | (b.v[i] & ~m);
  return r;
}

// the representative in [0, p): x < 2^256 = 2p + 38, so p goes at most twice
GVS_SR_FN Fe fe_canon(Fe x) {
  const Fe p = fe_p();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    Fe y;
    uint64_t t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      t = (uint64_t)x.v[i] - p.v[i] - ((t >> 32) & 1u);
      y.v[i] = (uint32_t)t;
    }
    const uint32_t keep = 0u - ((uint32_t)(t >> 32) & 1u);  // borrow: x < p
    x = fe_select(keep, x, y);
  }
  return x;
}

GVS_SR_FN uint32_t fe_mask_eq(const Fe& a, const Fe& b) {  // all ones if a == b (mod p)
  const Fe x = fe_canon(a), y = fe_canon(b);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) d |= x.v[i] ^ y.v[i];
  return 0u - (uint32_t)(d == 0);
}

GVS_SR_FN uint32_t fe_mask_neg(const Fe& a) {  // IS_NEGATIVE: canonical value odd
  return 0u - (fe_canon(a).v[0] & 1u);
}

GVS_SR_FN Fe fe_abs(const Fe& a) { return fe_select(fe_mask_neg(a), fe_neg(a), a); }

// z^((p-5)/8) = z^(2^252 - 3)
GVS_SR_FN_NI Fe fe_pow22523(const Fe& z) {
  Fe t0 = fe_sq(z);                       // 2
  Fe t1 = fe_sqn(t0, 2);                  // 8
  t1 = fe_mul(z, t1);                     // 9
  t0 = fe_mul(t0, t1);                    // 11
  t0 = fe_sq(t0);                         // 22
  t0 = fe_mul(t1, t0);                    // 2^5 - 1
  t1 = fe_sqn(t0, 5);
  t0 = fe_mul(t1, t0);                    // 2^10 - 1
  t1 = fe_sqn(t0, 10);
  t1 = fe_mul(t1, t0);                    // 2^20 - 1
  Fe t2 = fe_sqn(t1, 20);
  t1 = fe_mul(t2, t1);                    // 2^40 - 1
  t1 = fe_sqn(t1, 10);
  t0 = fe_mul(t1, t0);                    // 2^50 - 1
  t1 = fe_sqn(t0, 50);
  t1 = fe_mul(t1, t0);                    // 2^100 - 1
  t2 = fe_sqn(t1, 100);
  t1 = fe_mul(t2, t1);                    // 2^200 - 1
  t1 = fe_sqn(t1, 50);
  t0 = fe_mul(t1, t0);                    // 2^250 - 1
  t0 = fe_sqn(t0, 2);                     // 2^252 - 4
  return fe_mul(t0, z);                   // 2^252 - 3
}

// RFC 9496 §4.2 SQRT_RATIO_M1(u, v) -> r; *was_square all ones or zero
GVS_SR_FN_NI Fe fe_sqrt_ratio_m1(const Fe& u, const Fe& v, uint32_t* was_square) {
  const Fe v3 = fe_mul(fe_sq(v), v);
  const Fe v7 = fe_mul(fe_sq(v3), v);
  Fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  const Fe check = fe_mul(v, fe_sq(r));
  const Fe nu = fe_neg(u);
  const uint32_t correct = fe_mask_eq(check, u);
  const uint32_t flipped = fe_mask_eq(check, nu);
  const uint32_t flipped_i = fe_mask_eq(check, fe_mul(nu, fe_sqrt_m1()));
  r = fe_select(flipped | flipped_i, fe_mul(fe_sqrt_m1(), r), r);
  *was_square = correct | flipped;
  return fe_abs(r);
}

struct Pt {
  Fe X, Y, Z, T;
};

GVS_SR_FN Pt pt_identity() { return Pt{fe_zero(), fe_one(), fe_one(), fe_zero()}; }

GVS_SR_FN Pt pt_base() {
  return Pt{fe_k(0x8f25d51au, 0xc9562d60u, 0x9525a7b2u, 0x692cc760u, 0xfdd6dc5cu, 0xc0a4e231u,
                 0xcd6e53feu, 0x216936d3u),
            fe_k(0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u,
                 0x66666666u, 0x66666666u),
            fe_one(),
            fe_k(0xa5b7dda3u, 0x6dde8ab3u, 0x775152f5u, 0x20f09f80u, 0x64abe37du, 0x66ea4e8eu,
                 0xd78b7665u, 0x67875f0fu)};
}

// extended coordinates, a = -1: add-2008-hwcd-3 (complete on edwards25519)
GVS_SR_FN Pt pt_add(const Pt& p, const Pt& q) {
  const Fe a = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  const Fe b = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  const Fe c = fe_mul(fe_mul(p.T, fe_d2()), q.T);
  const Fe zz = fe_mul(p.Z, q.Z);
  const Fe d = fe_add(zz, zz);
  const Fe e = fe_sub(b, a), f = fe_sub(d, c), g = fe_add(d, c), h = fe_add(b, a);
  return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
}

// An addend in cached form (Y - X, Y + X, 2Z, 2dT): adding it costs 8
// multiplies instead of 9 and no sums of its coordinates.
struct PtC {
  Fe ymx, ypx, z2, t2d;
};

GVS_SR_FN PtC pt_cache(const Pt& q) {
  return PtC{fe_sub(q.Y, q.X), fe_add(q.Y, q.X), fe_add(q.Z, q.Z), fe_mul(q.T, fe_d2())};
}

// p + q, the same formula as pt_add with q's sums and products precomputed
GVS_SR_FN Pt pt_add_c(const Pt& p, const PtC& q) {
  const Fe a = fe_mul(fe_sub(p.Y, p.X), q.ymx);
  const Fe b = fe_mul(fe_add(p.Y, p.X), q.ypx);
  const Fe c = fe_mul(p.T, q.t2d);
  const Fe d = fe_mul(p.Z, q.z2);
  const Fe e = fe_sub(b, a), f = fe_sub(d, c), g = fe_add(d, c), h = fe_add(b, a);
  return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
}

GVS_SR_FN PtC ptc_select(uint32_t m, const PtC& a, const PtC& b) {
  return PtC{fe_select(m, a.ymx, b.ymx), fe_select(m, a.ypx, b.ypx), fe_select(m, a.z2, b.z2),
             fe_select(m, a.t2d, b.t2d)};
}

// dbl-2008-hwcd, a = -1
GVS_SR_FN Pt pt_dbl(const Pt& p) {
  const Fe a = fe_sq(p.X), b = fe_sq(p.Y);
  const Fe zz = fe_sq(p.Z);
  const Fe c = fe_add(zz, zz);
  const Fe d = fe_neg(a);
  const Fe e = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), a), b);
  const Fe g = fe_add(d, b), f = fe_sub(g, c), h = fe_sub(d, b);
  return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
}

// the same doubling without T, for a result that is only doubled again
// (dbl-2008-hwcd reads X, Y, Z)
GVS_SR_FN Pt pt_dbl_noT(const Pt& p) {
  const Fe a = fe_sq(p.X), b = fe_sq(p.Y);
  const Fe zz = fe_sq(p.Z);
  const Fe c = fe_add(zz, zz);
  const Fe d = fe_neg(a);
  const Fe e = fe_sub(fe_sub(fe_sq(fe_add(p.X, p.Y)), a), b);
  const Fe g = fe_add(d, b), f = fe_sub(g, c), h = fe_sub(d, b);
  return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_zero()};
}

GVS_SR_FN Pt pt_neg(const Pt& p) { return Pt{fe_neg(p.X), p.Y, p.Z, fe_neg(p.T)}; }

GVS_SR_FN Pt pt_select(uint32_t m, const Pt& a, const Pt& b) {
  return Pt{fe_select(m, a.X, b.X), fe_select(m, a.Y, b.Y), fe_select(m, a.Z, b.Z),
            fe_select(m, a.T, b.T)};
}

// RFC 9496 §4.3.1; *ok all ones when s is a canonical encoding of a point
GVS_SR_FN_NI Pt ristretto_decode(const Fe& s, uint32_t* ok) {
  const Fe p = fe_p();
  uint64_t t = 0;  // s < p
#pragma unroll
  for (int i = 0; i < 8; ++i) t = (uint64_t)s.v[i] - p.v[i] - ((t >> 32) & 1u);
  const uint32_t canonical = 0u - ((uint32_t)(t >> 32) & 1u);
  const uint32_t nonneg = 0u - (uint32_t)((s.v[0] & 1u) == 0);
  const Fe ss = fe_sq(s);
  const Fe u1 = fe_sub(fe_one(), ss), u2 = fe_add(fe_one(), ss);
  const Fe u2_sqr = fe_sq(u2);
  const Fe v = fe_sub(fe_neg(fe_mul(fe_d(), fe_sq(u1))), u2_sqr);
  uint32_t was_square;
  const Fe invsqrt = fe_sqrt_ratio_m1(fe_one(), fe_mul(v, u2_sqr), &was_square);
  const Fe den_x = fe_mul(invsqrt, u2);
  const Fe den_y = fe_mul(fe_mul(invsqrt, den_x), v);
  const Fe sx = fe_add(s, s);
  const Fe x = fe_abs(fe_mul(sx, den_x));
  const Fe y = fe_mul(u1, den_y);
  const Fe tt = fe_mul(x, y);
  const uint32_t y_nonzero = ~fe_mask_eq(y, fe_zero());
  *ok = canonical & nonneg & was_square & ~fe_mask_neg(tt) & y_nonzero;
  return Pt{x, y, fe_one(), tt};
}

// RFC 9496 §4.3.2 -> canonical s
GVS_SR_FN_NI Fe ristretto_encode(const Pt& q) {
  const Fe u1 = fe_mul(fe_add(q.Z, q.Y), fe_sub(q.Z, q.Y));
  const Fe u2 = fe_mul(q.X, q.Y);
  uint32_t ws;
  const Fe invsqrt = fe_sqrt_ratio_m1(fe_one(), fe_mul(u1, fe_sq(u2)), &ws);
  const Fe den1 = fe_mul(invsqrt, u1), den2 = fe_mul(invsqrt, u2);
  const Fe z_inv = fe_mul(fe_mul(den1, den2), q.T);
  const Fe ix0 = fe_mul(q.X, fe_sqrt_m1()), iy0 = fe_mul(q.Y, fe_sqrt_m1());
  const Fe enchanted = fe_mul(den1, fe_invsqrt_a_minus_d());
  const uint32_t rotate = fe_mask_neg(fe_mul(q.T, z_inv));
  const Fe x = fe_select(rotate, iy0, q.X);
  Fe y = fe_select(rotate, ix0, q.Y);
  const Fe den_inv = fe_select(rotate, enchanted, den2);
  y = fe_select(fe_mask_neg(fe_mul(x, z_inv)), fe_neg(y), y);
  return fe_canon(fe_abs(fe_mul(den_inv, fe_sub(q.Z, y))));
}

// ---------------------------------------------------------------- scalars

GVS_SR_FN Fe sc_l() {
  return fe_k(0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0, 0, 0, 0x10000000u);
}

// all ones if s < l
GVS_SR_FN uint32_t sc_mask_lt_l(const Fe& s) {
  const Fe l = sc_l();
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t = (uint64_t)s.v[i] - l.v[i] - ((t >> 32) & 1u);
  return 0u - ((uint32_t)(t >> 32) & 1u);
}

// a 512-bit little-endian integer mod l, one bit at a time (fixed 512 steps);
// word i at w[i * stride] (a thread's LDS column: a private array passed by
// pointer to this out-of-line function lived in scratch)
GVS_SR_FN_NI Fe sc_reduce_wide(const uint32_t* w, uint32_t stride) {
  const Fe l = sc_l();
  Fe r = fe_zero();
#pragma unroll
  for (int wi = 15; wi >= 0; --wi) {
    const uint32_t word = w[wi * stride];
    for (int b = 31; b >= 0; --b) {
      uint32_t c = (word >> b) & 1u;
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // r = 2r + bit  (< 2l < 2^254)
        const uint32_t nx = r.v[i] >> 31;
        r.v[i] = (r.v[i] << 1) | c;
        c = nx;
      }
      Fe y;
      uint64_t t = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        t = (uint64_t)r.v[i] - l.v[i] - ((t >> 32) & 1u);
        y.v[i] = (uint32_t)t;
      }
      r = fe_select(0u - ((uint32_t)(t >> 32) & 1u), r, y);
    }
  }
  return r;
}

GVS_SR_FN void shl1(Fe& x) {
#pragma unroll
  for (int i = 7; i > 0; --i) x.v[i] = (x.v[i] << 1) | (x.v[i - 1] >> 31);
  x.v[0] <<= 1;
}

GVS_SR_FN void ptc_store(uint32_t* t, uint32_t ts, const PtC& q) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    t[(0 + i) * ts] = q.ymx.v[i];
    t[(8 + i) * ts] = q.ypx.v[i];
    t[(16 + i) * ts] = q.z2.v[i];
    t[(24 + i) * ts] = q.t2d.v[i];
  }
}

// {P, 2P, 3P, 4P} in cached form at t (entry j at word 32j, stride ts)
GVS_SR_FN void ptc_table4(uint32_t* t, uint32_t ts, const Pt& P) {
  const Pt P2 = pt_dbl(P);
  const Pt P3 = pt_add(P2, P);
  ptc_store(t, ts, pt_cache(P));
  ptc_store(t + 32 * ts, ts, pt_cache(P2));
  ptc_store(t + 64 * ts, ts, pt_cache(P3));
  ptc_store(t + 96 * ts, ts, pt_cache(pt_dbl(P2)));
}

// Signed radix-8 digits of a scalar below 2^253: 85 digits in [-4, 4],
// digit i in 4-bit field i of dig (magnitude bits 0-2, sign bit 3).
GVS_SR_FN void sc_digits8(const Fe& x, uint32_t dig[11]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 11; ++w) dig[w] = 0;
#pragma unroll
  for (int i = 0; i < 85; ++i) {
    const int bit = 3 * i, wd = bit >> 5, sh = bit & 31;
    uint32_t v = x.v[wd] >> sh;
    if (sh > 29 && wd < 7) v |= x.v[wd + 1] << (32 - sh);
    v = (v & 7u) + carry;
    carry = v > 4u ? 1u : 0u;
    const uint32_t neg = carry, mag = neg ? 8u - v : v;  // v - 8 when carrying
    dig[i >> 3] |= (mag | (neg << 3)) << (4 * (i & 7));
  }
}

// The cached addend for digit d of table t: |d| selects among the identity
// and the 4 entries (all read), the sign swaps Y - X / Y + X and negates 2dT.
GVS_SR_FN PtC ptc_digit(const uint32_t* t, uint32_t ts, uint32_t d) {
  const uint32_t mag = d & 7u, neg = 0u - ((d >> 3) & 1u);
  uint32_t w[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    uint32_t v = (j == 0 || j == 8) ? 1u : (j == 16 ? 2u : 0u);  // cached identity (1, 1, 2, 0)
#pragma unroll
    for (uint32_t e = 0; e < 4; ++e) {
      const uint32_t m = 0u - (uint32_t)(mag == e + 1u);
      v = (t[(32 * e + j) * ts] & m) | (v & ~m);
    }
    w[j] = v;
  }
  PtC q;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    q.ymx.v[i] = (w[8 + i] & neg) | (w[i] & ~neg);
    q.ypx.v[i] = (w[i] & neg) | (w[8 + i] & ~neg);
    q.z2.v[i] = w[16 + i];
    q.t2d.v[i] = w[24 + i];
  }
  q.t2d = fe_select(neg, fe_neg(q.t2d), q.t2d);
  return q;
}

// s*B - k*A for scalars below 2^253: fixed signed radix-8 windows over both
// scalars (Straus), 85 digits each, 252 doublings and 170 additions of cached
// addends; btab holds {B, 2B, 3B, 4B} (shared by every thread), atab gets
// {-A, -2A, -3A, -4A} (this thread's, 128 words at stride ts).  Every digit
// reads all table entries and selects, so the instruction and LDS-access
// sequence does not depend on the scalars.
GVS_SR_FN_NI Pt double_scalar_mul(const Fe& s, const Fe& k, const Pt& A, uint32_t* atab, uint32_t ts,
                                  const uint32_t* btab) {
  ptc_table4(atab, ts, pt_neg(A));
  uint32_t ds[11], dk[11];
  sc_digits8(s, ds);
  sc_digits8(k, dk);
  Pt acc = pt_identity();
  for (int i = 84; i >= 0; --i) {
    // the table reads stay inside the loop: hoisted, they would hold 256
    // registers for its whole length
    __asm__ volatile("" ::: "memory");
    if (i < 84) {
      acc = pt_dbl_noT(acc);
      acc = pt_dbl_noT(acc);
      acc = pt_dbl(acc);
    }
    acc = pt_add_c(acc, ptc_digit(atab, ts, (dk[i >> 3] >> (4 * (i & 7))) & 15u));
    acc = pt_add_c(acc, ptc_digit(btab, 1, (ds[i >> 3] >> (4 * (i & 7))) & 15u));
  }
  return acc;
}

// Host form (tests/sr_host.cpp): the tables in local arrays.
inline Pt double_scalar_mul_host(const Fe& s, const Fe& k, const Pt& A) {
  uint32_t atab[128], btab[128];
  ptc_table4(btab, 1, pt_base());
  return double_scalar_mul(s, k, A, atab, 1, btab);
}

// ------------------------------------------------------------ STROBE / merlin

constexpr int kStrobeR = 166;

__constant__ uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
constexpr int kSrThreads = 64;

// The sponge of one thread: 50 little-endian words, word w at st[w * 64].
struct Strobe {
  uint32_t* st;
  uint32_t pos, pos_begin, cur_flags;

  __device__ void xor_byte(uint32_t i, uint32_t b) {
    st[(i >> 2) * kSrThreads] ^= (b & 0xFFu) << (8 * (i & 3));
  }
  __device__ uint32_t get_byte(uint32_t i) const {
    return (st[(i >> 2) * kSrThreads] >> (8 * (i & 3))) & 0xFFu;
  }

  __device__ void keccak() {
    uint64_t a[25];
#pragma unroll
    for (int i = 0; i < 25; ++i)
      a[i] = (uint64_t)st[(2 * i) * kSrThreads] | (uint64_t)st[(2 * i + 1) * kSrThreads] << 32;
    constexpr int rotc[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14,
                              27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
    constexpr int piln[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4,
                              15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
    for (int round = 0; round < 24; ++round) {
      uint64_t bc[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) bc[i] = a[i] ^ a[i + 5] ^ a[i + 10] ^ a[i + 15] ^ a[i + 20];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const uint64_t t = bc[(i + 4) % 5] ^ ((bc[(i + 1) % 5] << 1) | (bc[(i + 1) % 5] >> 63));
#pragma unroll
        for (int j = 0; j < 25; j += 5) a[j + i] ^= t;
      }
      uint64_t t = a[1];
#pragma unroll
      for (int i = 0; i < 24; ++i) {
        const int j = piln[i];
        const uint64_t b0 = a[j];
        a[j] = (t << rotc[i]) | (t >> (64 - rotc[i]));
        t = b0;
      }
#pragma unroll
      for (int j = 0; j < 25; j += 5) {
        uint64_t b[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) b[i] = a[j + i];
#pragma unroll
        for (int i = 0; i < 5; ++i) a[j + i] ^= (~b[(i + 1) % 5]) & b[(i + 2) % 5];
      }
      a[0] ^= kKeccakRC[round];
    }
#pragma unroll
    for (int i = 0; i < 25; ++i) {
      st[(2 * i) * kSrThreads] = (uint32_t)a[i];
      st[(2 * i + 1) * kSrThreads] = (uint32_t)(a[i] >> 32);
    }
  }

  __device__ void run_f() {
    xor_byte(pos, pos_begin);
    xor_byte(pos + 1, 0x04);
    xor_byte(kStrobeR + 1, 0x80);
    keccak();
    pos = 0;
    pos_begin = 0;
  }
  __device__ void absorb(uint32_t b) {
    xor_byte(pos, b);
    if (++pos == (uint32_t)kStrobeR) run_f();
  }
  __device__ uint32_t squeeze() {
    const uint32_t b = get_byte(pos);
    xor_byte(pos, b);  // the state byte becomes 0
    if (++pos == (uint32_t)kStrobeR) run_f();
    return b;
  }
  __device__ void begin_op(uint32_t flags) {  // a new (non-"more") operation
    const uint32_t old_begin = pos_begin;
    pos_begin = pos + 1;
    cur_flags = flags;
    absorb(old_begin);
    absorb(flags);
    if ((flags & (4u | 32u)) && pos != 0) run_f();  // C or K forces a permutation
  }
  // merlin append_message(label, msg): meta_ad(label) ; meta_ad(le32 len, more) ; ad(msg)
  template <int N>
  __device__ void label(const char (&s)[N]) {
    begin_op(16u | 2u);  // M | A
    for (int i = 0; i + 1 < N; ++i) absorb((uint8_t)s[i]);
  }
  __device__ void meta_len(uint32_t n) {
    for (int i = 0; i < 4; ++i) absorb((n >> (8 * i)) & 0xFFu);
  }
};

struct SrArgs {
  const uint8_t* pk;        // n public keys, pk_stride bytes apart
  uint32_t pk_stride;
  const uint8_t* msg;       // n messages of msg_len bytes, msg_stride apart
  uint32_t msg_stride, msg_len;
  const uint8_t* sig;       // n 64-B signatures, sig_stride apart
  uint32_t sig_stride, n;
  uint8_t ctx[64];          // signing context ("grapevine-challenge")
  uint32_t ctx_len;
  uint32_t* ok;             // n: 1 valid, 0 invalid (may be null)
  uint4* reqs;              // optional gvs_request slab: an invalid signature sets type 0
  uint32_t* status;         // optional per-request wire status: 0 -> 3 on a bad signature
};

constexpr uint32_t kWireBadSignature = 3;

GVS_SR_FN uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

__global__ void __launch_bounds__(kSrThreads) k_sr_verify(SrArgs a) {
  // per thread: the Keccak state (50 words) while hashing, then this
  // signature's -A table (128 words); plus the B table, shared
  __shared__ uint32_t sponge[128 * kSrThreads];
  __shared__ uint32_t btab[128];
  if (threadIdx.x == 0) ptc_table4(btab, 1, pt_base());
  const uint32_t tid = threadIdx.x;
  const uint32_t k = blockIdx.x * kSrThreads + tid;
  const uint32_t kk = k < a.n ? k : a.n - 1;  // tail threads redo the last signature
  const uint8_t* pk = a.pk + (uint64_t)kk * a.pk_stride;
  const uint8_t* msg = a.msg + (uint64_t)kk * a.msg_stride;
  const uint8_t* sig = a.sig + (uint64_t)kk * a.sig_stride;

  // Strobe128::new(b"Merlin v1.0"); Transcript::new(b"SigningContext");
  // append_message(b"", context)
  Strobe s{sponge + tid, 0, 0, 0};
  for (int w = 0; w < 50; ++w) s.st[w * kSrThreads] = 0;
  {
    const char* init = "\x01\xa8\x01\x00\x01\x60STROBEv1.0.2";  // the literal, not a local copy
    for (int i = 0; i < 18; ++i) s.xor_byte(i, (uint8_t)init[i]);
    s.keccak();
  }
  s.label("Merlin v1.0");
  s.label("dom-sep");
  s.meta_len(14);
  s.begin_op(2u);
  const char* sctx = "SigningContext";
  for (int i = 0; i < 14; ++i) s.absorb((uint8_t)sctx[i]);
  s.label("");
  s.meta_len(a.ctx_len);
  s.begin_op(2u);
  for (uint32_t i = 0; i < a.ctx_len; ++i) s.absorb(a.ctx[i]);
  // append_message(b"sign-bytes", msg)
  s.label("sign-bytes");
  s.meta_len(a.msg_len);
  s.begin_op(2u);  // A
  for (uint32_t i = 0; i < a.msg_len; ++i) s.absorb(msg[i]);
  // proto_name(b"Schnorr-sig")
  s.label("proto-name");
  s.meta_len(11);
  s.begin_op(2u);
  const char* proto = "Schnorr-sig";
  for (int i = 0; i < 11; ++i) s.absorb((uint8_t)proto[i]);
  // commit_point(b"sign:pk", pk), commit_point(b"sign:R", R)
  s.label("sign:pk");
  s.meta_len(32);
  s.begin_op(2u);
  for (int i = 0; i < 32; ++i) s.absorb(pk[i]);
  s.label("sign:R");
  s.meta_len(32);
  s.begin_op(2u);
  for (int i = 0; i < 32; ++i) s.absorb(sig[i]);
  // challenge_scalar(b"sign:c"): 64 bytes, wide reduction mod l
  s.label("sign:c");
  s.meta_len(64);
  s.begin_op(1u | 2u | 4u);  // I | A | C
  // the 16 words go to sponge words 50-65 of this thread (past the state)
  for (int i = 0; i < 16; ++i) {
    uint32_t w = 0;
    for (int c = 0; c < 4; ++c) w |= s.squeeze() << (8 * c);
    s.st[(50 + i) * kSrThreads] = w;
  }
  const Fe kc = sc_reduce_wide(s.st + 50 * kSrThreads, kSrThreads);

  Fe sc, A_s, R_s;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc.v[i] = ld_le32(sig + 32 + 4 * i);
    A_s.v[i] = ld_le32(pk + 4 * i);
    R_s.v[i] = ld_le32(sig + 4 * i);
  }
  const uint32_t marked = 0u - (sc.v[7] >> 31);
  sc.v[7] &= 0x7FFFFFFFu;
  uint32_t ok = marked & sc_mask_lt_l(sc);
  uint32_t pk_ok;
  const Pt A = ristretto_decode(A_s, &pk_ok);
  ok &= pk_ok;

  __syncthreads();  // btab written
  const Pt acc = double_scalar_mul(sc, kc, A, sponge + tid, kSrThreads, btab);
  const Fe enc = ristretto_encode(acc);
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) diff |= enc.v[i] ^ R_s.v[i];
  ok &= 0u - (uint32_t)(diff == 0);

  if (k >= a.n) return;
  const uint32_t valid = ok & 1u;
  if (a.ok) a.ok[k] = valid;
  if (a.reqs) {  // the request's type word: unchanged if valid, 0 (a hard error) if not
    uint4* r = a.reqs + (uint64_t)k * 65u + 64u;
    uint4 v = *r;
    v.x = valid ? v.x : 0u;
    *r = v;
  }
  if (a.status) {
    const uint32_t st = a.status[k];
    a.status[k] = (st == 0 && !valid) ? kWireBadSignature : st;
  }
}

}  // namespace sr
}  // namespace gvs
