// p384_field.h -- NIST P-384 arithmetic for identities whose certificates carry P-384 keys
// (host + device, one definition).  The reference verifies them like any ECDSA key
// (fabric-lib-go bccsp/sw/ecdsa.go:41-57 -> Go crypto/ecdsa.Verify over crypto/internal/nistec
// P384), with the P-384 half order of bccsp/utils/ecdsa.go:26-31 for the low-S rule.
//
// Radix 2^32, 12 little-endian limbs, Montgomery form (R = 2^384) for both the field (mod p) and
// the scalars (mod n).  Every operation returns a fully reduced value, so equal points compare
// equal limb by limb.  Points are Jacobian (X, Y, Z), Z == 0 the point at infinity; the addition
// formulas are exact (a doubling or the infinity when the x coordinates meet), so no input needs a
// second, slower path.  P-384 items are rare (a handful of identities): the kernels are written
// for exactness and a short chain per item, not for throughput.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p384 {

#define P384_HD __host__ __device__ inline
constexpr int NL = 12;

// p = 2^384 - 2^128 - 2^96 + 2^32 - 1; n the group order; constants checked in tests/test_p384.py
struct Consts {
  uint32_t p[NL], n[NL], rr_p[NL], one_p[NL], rr_n[NL], b_m[NL], gx_m[NL], gy_m[NL], half_n[NL], p_minus_n[NL];
  uint32_t n0_p, n0_n;  // -m^-1 mod 2^32
};
#define P384_CONSTS { \
      {0xffffffffu, 0x00000000u, 0x00000000u, 0xffffffffu, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, \
       0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}, \
      {0xccc52973u, 0xecec196au, 0x48b0a77au, 0x581a0db2u, 0xf4372ddfu, 0xc7634d81u, 0xffffffffu, 0xffffffffu, \
       0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}, \
      {0x00000001u, 0xfffffffeu, 0x00000000u, 0x00000002u, 0x00000000u, 0xfffffffeu, 0x00000000u, 0x00000002u, \
       0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u}, \
      {0x00000001u, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u, \
       0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}, \
      {0x19b409a9u, 0x2d319b24u, 0xdf1aa419u, 0xff3d81e5u, 0xfcb82947u, 0xbc3e483au, 0x4aab1cc5u, 0xd40d4917u, \
       0x28266895u, 0x3fb05b7au, 0x2b39bf21u, 0x0c84ee01u}, \
      {0x9d412dccu, 0x08118871u, 0x7a4c32ecu, 0xf729add8u, 0x1920022eu, 0x77f2209bu, 0x94938ae2u, 0xe3374beeu, \
       0x1f022094u, 0xb62b21f4u, 0x604fbff9u, 0xcd08114bu}, \
      {0x49c0b528u, 0x3dd07566u, 0xa0d6ce38u, 0x20e378e2u, 0x541b4d6eu, 0x879c3afcu, 0x59a30effu, 0x64548684u, \
       0x614ede2bu, 0x812ff723u, 0x299e1513u, 0x4d3aadc2u}, \
      {0x4b03a4feu, 0x23043dadu, 0x7bb4a9acu, 0xa1bfa8bfu, 0x2e83b050u, 0x8bade756u, 0x68f4ffd9u, 0xc6c35219u, \
       0x3969a840u, 0xdd800226u, 0x5a15c5e9u, 0x2b78abc2u}, \
      {0x666294b9u, 0x76760cb5u, 0x245853bdu, 0xac0d06d9u, 0xfa1b96efu, 0xe3b1a6c0u, 0xffffffffu, 0xffffffffu, \
       0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu}, \
      {0x333ad68cu, 0x1313e696u, 0xb74f5885u, 0xa7e5f24cu, 0x0bc8d21fu, 0x389cb27eu, 0x00000000u, 0x00000000u, \
       0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}, \
      0x00000001u, \
      0xe88fdc45u}
static __constant__ const Consts kP384Dev = P384_CONSTS;
static const Consts kP384Host = P384_CONSTS;
P384_HD const Consts &C() {
#if defined(__HIP_DEVICE_COMPILE__)
  return kP384Dev;
#else
  return kP384Host;
#endif
}

P384_HD void cpy(uint32_t r[NL], const uint32_t a[NL]) {
  for (int i = 0; i < NL; i++) r[i] = a[i];
}
P384_HD bool is_zero(const uint32_t a[NL]) {
  uint32_t x = 0;
  for (int i = 0; i < NL; i++) x |= a[i];
  return x == 0;
}
P384_HD bool eq(const uint32_t a[NL], const uint32_t b[NL]) {
  uint32_t x = 0;
  for (int i = 0; i < NL; i++) x |= a[i] ^ b[i];
  return x == 0;
}
P384_HD bool geq(const uint32_t a[NL], const uint32_t b[NL]) {  // a >= b
  for (int i = NL - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return true;
}
P384_HD uint32_t sub_raw(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL]) {  // -> borrow
  uint64_t br = 0;
  for (int i = 0; i < NL; i++) {
    const uint64_t d = (uint64_t)a[i] - b[i] - br;
    r[i] = (uint32_t)d;
    br = (d >> 63) & 1u;
  }
  return (uint32_t)br;
}
P384_HD uint32_t add_raw(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL]) {  // -> carry
  uint64_t c = 0;
  for (int i = 0; i < NL; i++) {
    c += (uint64_t)a[i] + b[i];
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}
// a, b < m
P384_HD void add_mod(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL], const uint32_t m[NL]) {
  uint32_t t[NL], u[NL];
  const uint32_t c = add_raw(t, a, b);
  const uint32_t br = sub_raw(u, t, m);
  if (c || !br) cpy(r, u);
  else cpy(r, t);
}
P384_HD void sub_mod(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL], const uint32_t m[NL]) {
  uint32_t t[NL];
  if (sub_raw(t, a, b)) add_raw(t, t, m);
  cpy(r, t);
}
// Montgomery product a b R^-1 mod m (CIOS), a, b < m
P384_HD void mont_mul(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL], const uint32_t m[NL], uint32_t n0) {
  uint32_t t[NL + 2];
  for (int i = 0; i < NL + 2; i++) t[i] = 0;
  for (int i = 0; i < NL; i++) {
    uint64_t c = 0;
    for (int j = 0; j < NL; j++) {
      const uint64_t x = (uint64_t)a[j] * b[i] + t[j] + c;
      t[j] = (uint32_t)x;
      c = x >> 32;
    }
    uint64_t x = (uint64_t)t[NL] + c;
    t[NL] = (uint32_t)x;
    t[NL + 1] = (uint32_t)(x >> 32);
    const uint32_t q = t[0] * n0;
    x = (uint64_t)q * m[0] + t[0];
    c = x >> 32;
    for (int j = 1; j < NL; j++) {
      x = (uint64_t)q * m[j] + t[j] + c;
      t[j - 1] = (uint32_t)x;
      c = x >> 32;
    }
    x = (uint64_t)t[NL] + c;
    t[NL - 1] = (uint32_t)x;
    t[NL] = t[NL + 1] + (uint32_t)(x >> 32);
  }
  uint32_t u[NL];
  const uint32_t br = sub_raw(u, t, m);
  if (t[NL] || !br) cpy(r, u);
  else cpy(r, t);
}

// ---- the field mod p (Montgomery)
P384_HD void fmul(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL]) { mont_mul(r, a, b, C().p, C().n0_p); }
P384_HD void fsqr(uint32_t r[NL], const uint32_t a[NL]) { mont_mul(r, a, a, C().p, C().n0_p); }
P384_HD void fadd(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL]) { add_mod(r, a, b, C().p); }
P384_HD void fsub(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL]) { sub_mod(r, a, b, C().p); }
P384_HD void to_mont_p(uint32_t r[NL], const uint32_t a[NL]) { fmul(r, a, C().rr_p); }
P384_HD void from_mont_p(uint32_t r[NL], const uint32_t a[NL]) {
  uint32_t one[NL] = {1};
  fmul(r, a, one);
}
// a^(p-2) (Fermat), 4-bit fixed windows; a != 0 (Montgomery in, Montgomery out)
P384_HD void finv(uint32_t r[NL], const uint32_t a[NL]) {
  uint32_t tab[16][NL];
  cpy(tab[0], C().one_p);
  cpy(tab[1], a);
  for (int i = 2; i < 16; i++) fmul(tab[i], tab[i - 1], a);
  uint32_t e[NL], two[NL] = {2};
  sub_raw(e, C().p, two);
  uint32_t acc[NL];
  cpy(acc, C().one_p);
  for (int nib = NL * 8 - 1; nib >= 0; nib--) {
    for (int k = 0; k < 4; k++) fsqr(acc, acc);
    const uint32_t d = (e[nib >> 3] >> (4 * (nib & 7))) & 15u;
    if (d) fmul(acc, acc, tab[d]);
  }
  cpy(r, acc);
}

// ---- points
struct J {
  uint32_t X[NL], Y[NL], Z[NL];
};
P384_HD void set_inf(J &r) {
  for (int i = 0; i < NL; i++) r.X[i] = r.Y[i] = r.Z[i] = 0;
}
// dbl-2001-b (a = -3); the infinity (Z = 0) maps to itself
P384_HD void dbl(J &r, const J &p) {
  uint32_t delta[NL], gamma[NL], beta[NL], alpha[NL], t1[NL], t2[NL], t3[NL];
  fsqr(delta, p.Z);
  fsqr(gamma, p.Y);
  fmul(beta, p.X, gamma);
  fsub(t1, p.X, delta);
  fadd(t2, p.X, delta);
  fmul(t3, t1, t2);
  fadd(alpha, t3, t3);
  fadd(alpha, alpha, t3);  // 3 (X - delta)(X + delta)
  uint32_t X3[NL], Y3[NL], Z3[NL], b4[NL], b8[NL];
  fadd(b4, beta, beta);
  fadd(b4, b4, b4);        // 4 beta
  fadd(b8, b4, b4);        // 8 beta
  fsqr(X3, alpha);
  fsub(X3, X3, b8);
  fadd(t1, p.Y, p.Z);
  fsqr(Z3, t1);
  fsub(Z3, Z3, gamma);
  fsub(Z3, Z3, delta);
  fsub(t1, b4, X3);
  fmul(Y3, alpha, t1);
  fsqr(t2, gamma);         // gamma^2
  fadd(t2, t2, t2);
  fadd(t2, t2, t2);
  fadd(t2, t2, t2);        // 8 gamma^2
  fsub(Y3, Y3, t2);
  cpy(r.X, X3);
  cpy(r.Y, Y3);
  cpy(r.Z, Z3);
}
// p + (x2, y2) with the affine point given in Montgomery form (never the infinity), exact
P384_HD void madd(J &r, const J &p, const uint32_t x2[NL], const uint32_t y2[NL]) {
  if (is_zero(p.Z)) {
    cpy(r.X, x2);
    cpy(r.Y, y2);
    cpy(r.Z, C().one_p);
    return;
  }
  uint32_t z1z1[NL], u2[NL], s2[NL], h[NL], rr[NL], t[NL];
  fsqr(z1z1, p.Z);
  fmul(u2, x2, z1z1);
  fmul(t, p.Z, z1z1);
  fmul(s2, y2, t);
  fsub(h, u2, p.X);
  fsub(rr, s2, p.Y);
  if (is_zero(h)) {
    if (is_zero(rr)) dbl(r, p);
    else set_inf(r);
    return;
  }
  uint32_t hh[NL], hhh[NL], v[NL], X3[NL], Y3[NL], Z3[NL];
  fsqr(hh, h);
  fmul(hhh, h, hh);
  fmul(v, p.X, hh);
  fsqr(X3, rr);
  fsub(X3, X3, hhh);
  fsub(X3, X3, v);
  fsub(X3, X3, v);
  fsub(t, v, X3);
  fmul(Y3, rr, t);
  fmul(t, p.Y, hhh);
  fsub(Y3, Y3, t);
  fmul(Z3, p.Z, h);
  cpy(r.X, X3);
  cpy(r.Y, Y3);
  cpy(r.Z, Z3);
}
// p + q, both Jacobian, exact
P384_HD void add(J &r, const J &p, const J &q) {
  if (is_zero(p.Z)) {
    r = q;
    return;
  }
  if (is_zero(q.Z)) {
    r = p;
    return;
  }
  uint32_t z1z1[NL], z2z2[NL], u1[NL], u2[NL], s1[NL], s2[NL], h[NL], rr[NL], t[NL];
  fsqr(z1z1, p.Z);
  fsqr(z2z2, q.Z);
  fmul(u1, p.X, z2z2);
  fmul(u2, q.X, z1z1);
  fmul(t, q.Z, z2z2);
  fmul(s1, p.Y, t);
  fmul(t, p.Z, z1z1);
  fmul(s2, q.Y, t);
  fsub(h, u2, u1);
  fsub(rr, s2, s1);
  if (is_zero(h)) {
    if (is_zero(rr)) dbl(r, p);
    else set_inf(r);
    return;
  }
  uint32_t hh[NL], hhh[NL], v[NL], X3[NL], Y3[NL], Z3[NL];
  fsqr(hh, h);
  fmul(hhh, h, hh);
  fmul(v, u1, hh);
  fsqr(X3, rr);
  fsub(X3, X3, hhh);
  fsub(X3, X3, v);
  fsub(X3, X3, v);
  fsub(t, v, X3);
  fmul(Y3, rr, t);
  fmul(t, s1, hhh);
  fsub(Y3, Y3, t);
  fmul(t, p.Z, q.Z);
  fmul(Z3, t, h);
  cpy(r.X, X3);
  cpy(r.Y, Y3);
  cpy(r.Z, Z3);
}
// y^2 == x^3 - 3x + b, both < p (plain form)
P384_HD bool on_curve(const uint32_t x[NL], const uint32_t y[NL]) {
  if (geq(x, C().p) || geq(y, C().p)) return false;
  uint32_t xm[NL], ym[NL], t[NL], u[NL];
  to_mont_p(xm, x);
  to_mont_p(ym, y);
  fsqr(t, xm);
  fmul(t, t, xm);  // x^3
  fadd(u, xm, xm);
  fadd(u, u, xm);  // 3x
  fsub(t, t, u);
  fadd(t, t, C().b_m);
  fsqr(u, ym);
  return eq(t, u);
}

// ---- scalars mod n
// a^-1 mod n (plain form), 0 < a < n: the binary extended Euclid (data-dependent time is fine:
// verification handles public values only)
P384_HD void inv_mod_n(uint32_t r[NL], const uint32_t a[NL]) {
  const uint32_t *N = C().n;
  uint32_t u[NL], v[NL], x1[NL], x2[NL];
  cpy(u, a);
  cpy(v, N);
  for (int i = 0; i < NL; i++) x1[i] = x2[i] = 0;
  x1[0] = 1;
  auto is_one = [](const uint32_t w[NL]) {
    uint32_t x = w[0] ^ 1u;
    for (int i = 1; i < NL; i++) x |= w[i];
    return x == 0;
  };
  auto half = [&](uint32_t w[NL], uint32_t x[NL]) {  // w /= 2, x = x / 2 mod n
    for (int i = 0; i < NL - 1; i++) w[i] = (w[i] >> 1) | (w[i + 1] << 31);
    w[NL - 1] >>= 1;
    uint32_t top = 0;
    if (x[0] & 1u) top = add_raw(x, x, N);
    for (int i = 0; i < NL - 1; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
    x[NL - 1] = (x[NL - 1] >> 1) | (top << 31);
  };
  while (!is_one(u) && !is_one(v)) {
    while (!(u[0] & 1u)) half(u, x1);
    while (!(v[0] & 1u)) half(v, x2);
    if (geq(u, v)) {
      sub_raw(u, u, v);
      sub_mod(x1, x1, x2, N);
    } else {
      sub_raw(v, v, u);
      sub_mod(x2, x2, x1, N);
    }
  }
  if (is_one(u)) cpy(r, x1);
  else cpy(r, x2);
}
// a b mod n (plain in, plain out), a, b < n
P384_HD void mul_mod_n(uint32_t r[NL], const uint32_t a[NL], const uint32_t b[NL]) {
  uint32_t t[NL];
  mont_mul(t, a, b, C().n, C().n0_n);
  mont_mul(r, t, C().rr_n, C().n, C().n0_n);
}

}  // namespace p384
