// p256_field.h -- P-256 arithmetic for gfx950 (CDNA4), one field element per lane.
//
// Representation: 8 x 32-bit little-endian limbs held in VGPRs.
//   * Field F_p (p = 2^256 - 2^224 + 2^192 + 2^96 - 1): Montgomery form, R = 2^256.
//     Because p == -1 mod 2^32, the Montgomery factor is m = t[i] and m*p only touches
//     limbs i, i+3, i+6, i+7, i+8 -- the reduction is 9 VALU adds per limb, no multiplies.
//   * Scalar field Z_n (group order): generic CIOS Montgomery, used only in the per-item
//     scalar preparation (u1 = e*w, u2 = r*w; the inversion itself is p256_modinv.h).
// All integer VALU work (v_mad_u64_u32 + add-with-carry chains); no MFMA, no FP.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FGV_DEV __device__ __forceinline__

struct fe {
  uint32_t v[8];
};

// ---- constants ---------------------------------------------------------------
// p, little-endian limbs
#define P_0 0xFFFFFFFFu
#define P_1 0xFFFFFFFFu
#define P_2 0xFFFFFFFFu
#define P_3 0x00000000u
#define P_4 0x00000000u
#define P_5 0x00000000u
#define P_6 0x00000001u
#define P_7 0xFFFFFFFFu
// n, little-endian limbs
__constant__ static const uint32_t N_LIMBS[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                                                 0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};
#define N_0INV 0xEE00BC4Fu  // -n^-1 mod 2^32

FGV_DEV uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t *cout) {
  return __builtin_addc(a, b, cin, cout);
}
FGV_DEV uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t *bout) {
  return __builtin_subc(a, b, bin, bout);
}

FGV_DEV void fe_set_one(fe &r) {  // R mod p = 2^256 - p
  r.v[0] = 1u; r.v[1] = 0u; r.v[2] = 0u; r.v[3] = 0xFFFFFFFFu;
  r.v[4] = 0xFFFFFFFFu; r.v[5] = 0xFFFFFFFFu; r.v[6] = 0xFFFFFFFEu; r.v[7] = 0u;
}
FGV_DEV void fe_set_zero(fe &r) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0u;
}
FGV_DEV bool fe_is_zero(const fe &a) {
  uint32_t x = a.v[0] | a.v[1] | a.v[2] | a.v[3] | a.v[4] | a.v[5] | a.v[6] | a.v[7];
  return x == 0u;
}
FGV_DEV bool fe_eq(const fe &a, const fe &b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.v[i] ^ b.v[i];
  return x == 0u;
}

// r = (t - p) if (hi || t >= p) else t      (t < 2p)
FGV_DEV void fe_final_sub(fe &r, const uint32_t t[8], uint32_t hi) {
  uint32_t d[8], b;
  d[0] = subb(t[0], P_0, 0u, &b);
  d[1] = subb(t[1], P_1, b, &b);
  d[2] = subb(t[2], P_2, b, &b);
  d[3] = subb(t[3], P_3, b, &b);
  d[4] = subb(t[4], P_4, b, &b);
  d[5] = subb(t[5], P_5, b, &b);
  d[6] = subb(t[6], P_6, b, &b);
  d[7] = subb(t[7], P_7, b, &b);
  bool take = (hi != 0u) | (b == 0u);
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = take ? d[i] : t[i];
}

FGV_DEV void fe_add(fe &r, const fe &a, const fe &b) {
  uint32_t t[8], c;
  t[0] = addc(a.v[0], b.v[0], 0u, &c);
#pragma unroll
  for (int i = 1; i < 8; i++) t[i] = addc(a.v[i], b.v[i], c, &c);
  fe_final_sub(r, t, c);
}

FGV_DEV void fe_sub(fe &r, const fe &a, const fe &b) {
  uint32_t t[8], bo;
  t[0] = subb(a.v[0], b.v[0], 0u, &bo);
#pragma unroll
  for (int i = 1; i < 8; i++) t[i] = subb(a.v[i], b.v[i], bo, &bo);
  // if borrow: add p back (mask the constant limbs)
  uint32_t m = 0u - bo, c;
  t[0] = addc(t[0], P_0 & m, 0u, &c);
  t[1] = addc(t[1], P_1 & m, c, &c);
  t[2] = addc(t[2], P_2 & m, c, &c);
  t[3] = addc(t[3], 0u, c, &c);
  t[4] = addc(t[4], 0u, c, &c);
  t[5] = addc(t[5], 0u, c, &c);
  t[6] = addc(t[6], P_6 & m, c, &c);
  t[7] = addc(t[7], P_7 & m, c, &c);
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
}

FGV_DEV void fe_neg(fe &r, const fe &a) {  // p - a (a != 0), 0 -> 0
  fe z;
  fe_set_zero(z);
  fe_sub(r, z, a);
}

// 8x8 -> 16 limb product, operand scanning (each step fits a 64-bit accumulator)
FGV_DEV void mul_256(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c = (uint64_t)a[j] * b[i] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
}

// Squaring: off-diagonal products once, doubled, plus the diagonal.
FGV_DEV void sqr_256(uint32_t t[16], const uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = 0u;
#pragma unroll
  for (int i = 0; i < 7; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; j++) {
      c = (uint64_t)a[j] * a[i] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  // double
  uint32_t top = t[15] >> 31;
#pragma unroll
  for (int i = 15; i > 0; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 31);
  t[0] <<= 1;
  (void)top;  // 2*sum(off-diag) < 2^511, no overflow past limb 15
  // add diagonal
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t d = (uint64_t)a[i] * a[i];
    t[2 * i] = addc(t[2 * i], (uint32_t)d, c, &c);
    t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(d >> 32), c, &c);
  }
}

// Montgomery reduction mod p of a 512-bit t: returns t * 2^-256 mod p.
// Round i: m = t[i]; t += m*p at limb i, where m*p = m*2^256 + m*2^192 + m*2^96 - m*2^224 - m
// = m at limbs i+3, i+6 and m*(2^32-1) at limb i+7 (lo) / i+8 (hi); limb i cancels.
// The carry out of limb i+8 is deferred to round i+1 (added at its limb i+9).
FGV_DEV void mont_reduce_p(fe &r, uint32_t t[16]) {
  uint32_t pend = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t m = t[i];
    uint32_t bw;
    uint32_t lo = subb(0u, m, 0u, &bw);  // 2^32 - m (mod 2^32); bw = (m != 0)
    uint32_t hi = m - bw;                // m - 1 if m != 0 else 0
    uint32_t hp = hi + pend;             // <= 2^32 - 1
    uint32_t c;
    t[i + 3] = addc(t[i + 3], m, 0u, &c);
    t[i + 4] = addc(t[i + 4], 0u, c, &c);
    t[i + 5] = addc(t[i + 5], 0u, c, &c);
    t[i + 6] = addc(t[i + 6], m, c, &c);
    t[i + 7] = addc(t[i + 7], lo, c, &c);
    t[i + 8] = addc(t[i + 8], hp, c, &c);
    pend = c;
  }
  fe_final_sub(r, t + 8, pend);
}

FGV_DEV void fe_mul(fe &r, const fe &a, const fe &b) {
  uint32_t t[16];
  mul_256(t, a.v, b.v);
  mont_reduce_p(r, t);
}
FGV_DEV void fe_sqr(fe &r, const fe &a) {
  uint32_t t[16];
  sqr_256(t, a.v);
  mont_reduce_p(r, t);
}

// a^(p-2) by a fixed square-and-multiply chain (key-table build only).
// p - 2 = FFFFFFFF 00000001 00000000 00000000 00000000 FFFFFFFF FFFFFFFF FFFFFFFD
__device__ __noinline__ void fe_inv(fe &r, const fe &a) {
  const uint32_t e[8] = {0xFFFFFFFDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u, 1u, 0xFFFFFFFFu};
  fe acc;
  fe_set_one(acc);
  for (int i = 255; i >= 0; i--) {
    fe_sqr(acc, acc);
    if ((e[i >> 5] >> (i & 31)) & 1u) fe_mul(acc, acc, a);
  }
  r = acc;
}

// ---- scalar field (mod n), generic Montgomery ------------------------------------
FGV_DEV void sn_final_sub(uint32_t r[8], const uint32_t t[8], uint32_t hi) {
  uint32_t d[8], b = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = subb(t[i], N_LIMBS[i], b, &b);
  bool take = (hi != 0u) | (b == 0u);
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = take ? d[i] : t[i];
}

FGV_DEV void sn_mul(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c = (uint64_t)a[j] * b[i] + t[j] + (c >> 32);
      t[j] = (uint32_t)c;
    }
    uint64_t s = (uint64_t)t[8] + (c >> 32);
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    uint32_t m = t[0] * N_0INV;
    c = (uint64_t)m * N_LIMBS[0] + t[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * N_LIMBS[j] + t[j] + (c >> 32);
      t[j - 1] = (uint32_t)c;
    }
    s = (uint64_t)t[8] + (c >> 32);
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  sn_final_sub(r, t, t[8]);
}

// Montgomery reduction mod n of a 512-bit t (generic REDC, 8 rounds)
FGV_DEV void sn_redc(uint32_t r[8], uint32_t t[16]) {
  uint32_t pend = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t m = t[i] * N_0INV;
    uint64_t c = (uint64_t)m * N_LIMBS[0] + t[i];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c = (uint64_t)m * N_LIMBS[j] + t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    uint64_t s = (uint64_t)t[i + 8] + (c >> 32) + pend;
    t[i + 8] = (uint32_t)s;
    pend = (uint32_t)(s >> 32);
  }
  sn_final_sub(r, t + 8, pend);
}
// Montgomery squaring mod n (off-diagonal products once)
FGV_DEV void sn_sqr(uint32_t r[8], const uint32_t a[8]) {
  uint32_t t[16];
  sqr_256(t, a);
  sn_redc(r, t);
}

// compare 256-bit little-endian: a < b
FGV_DEV bool lt_256(const uint32_t a[8], const uint32_t b[8]) {
  uint32_t bo = 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)subb(a[i], b[i], bo, &bo);
  return bo != 0u;
}

// ---- points ----------------------------------------------------------------------
struct jpoint {  // Jacobian, Montgomery form; Z == 0 <=> point at infinity
  fe x, y, z;
};
struct apoint {  // affine, Montgomery form
  fe x, y;
};

// dbl-2001-b, a = -3: 3M + 5S
FGV_DEV void pt_dbl(jpoint &r, const jpoint &p) {
  if (fe_is_zero(p.z) || fe_is_zero(p.y)) {
    fe_set_zero(r.x); fe_set_zero(r.y); fe_set_zero(r.z);
    return;
  }
  fe delta, gamma, beta, alpha, t1, t2;
  fe_sqr(delta, p.z);
  fe_sqr(gamma, p.y);
  fe_mul(beta, p.x, gamma);
  fe_sub(t1, p.x, delta);
  fe_add(t2, p.x, delta);
  fe_mul(alpha, t1, t2);
  fe_add(t1, alpha, alpha);
  fe_add(alpha, t1, alpha);  // 3(X-d)(X+d)
  fe_add(t1, p.y, p.z);
  fe_sqr(t1, t1);
  fe_sub(t1, t1, gamma);
  fe_sub(r.z, t1, delta);  // Z3 (p.z no longer needed)
  fe_add(beta, beta, beta);
  fe_add(beta, beta, beta);  // 4 beta
  fe_sqr(t1, alpha);
  fe_add(t2, beta, beta);
  fe_sub(r.x, t1, t2);  // X3 = alpha^2 - 8 beta
  fe_sub(t1, beta, r.x);
  fe_mul(t1, alpha, t1);
  fe_sqr(t2, gamma);
  fe_add(t2, t2, t2);
  fe_add(t2, t2, t2);
  fe_add(t2, t2, t2);  // 8 gamma^2
  fe_sub(r.y, t1, t2);
}

// Complete mixed addition r = p + q (q affine, never infinity), madd-2004-hmv (8M + 3S)
// with the exceptional cases routed: p = inf -> q; p = q -> dbl; p = -q -> inf.
// Inlined: callers keep exactly one call site in their loop (no scratch traffic).
FGV_DEV void pt_madd(jpoint &r, const jpoint &p, const apoint &q) {
  if (fe_is_zero(p.z)) {
    r.x = q.x; r.y = q.y; fe_set_one(r.z);
    return;
  }
  fe z1z1, u2, s2, h, rr, t;
  fe_sqr(z1z1, p.z);
  fe_mul(u2, q.x, z1z1);
  fe_mul(t, p.z, z1z1);
  fe_mul(s2, q.y, t);
  fe_sub(h, u2, p.x);
  fe_sub(rr, s2, p.y);
  if (fe_is_zero(h)) {
    if (fe_is_zero(rr)) {
      jpoint pp = p;
      pt_dbl(r, pp);
    } else {
      fe_set_zero(r.x); fe_set_zero(r.y); fe_set_zero(r.z);
    }
    return;
  }
  fe hh, hhh, v;
  fe_sqr(hh, h);
  fe_mul(hhh, h, hh);
  fe_mul(v, p.x, hh);
  fe x3, y3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, hhh);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, p.y, hhh);
  fe_sub(y3, y3, t);
  fe_mul(r.z, p.z, h);
  r.x = x3;
  r.y = y3;
}

// Complete Jacobian addition (inlined form: one call site per loop)
FGV_DEV void pt_add_inl(jpoint &r, const jpoint &p, const jpoint &q) {
  if (fe_is_zero(p.z)) { r = q; return; }
  if (fe_is_zero(q.z)) { r = p; return; }
  fe z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
  fe_sqr(z1z1, p.z);
  fe_sqr(z2z2, q.z);
  fe_mul(u1, p.x, z2z2);
  fe_mul(u2, q.x, z1z1);
  fe_mul(t, q.z, z2z2);
  fe_mul(s1, p.y, t);
  fe_mul(t, p.z, z1z1);
  fe_mul(s2, q.y, t);
  fe_sub(h, u2, u1);
  fe_sub(rr, s2, s1);
  if (fe_is_zero(h)) {
    if (fe_is_zero(rr)) {
      jpoint pp = p;
      pt_dbl(r, pp);
    } else {
      fe_set_zero(r.x); fe_set_zero(r.y); fe_set_zero(r.z);
    }
    return;
  }
  fe hh, hhh, v, x3, y3, z3;
  fe_sqr(hh, h);
  fe_mul(hhh, h, hh);
  fe_mul(v, u1, hh);
  fe_sqr(x3, rr);
  fe_sub(x3, x3, hhh);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, s1, hhh);
  fe_sub(y3, y3, t);
  fe_mul(z3, p.z, q.z);
  fe_mul(z3, z3, h);
  r.x = x3; r.y = y3; r.z = z3;
}

// out-of-line form (key-table build)
__device__ __noinline__ void pt_add(jpoint &r, const jpoint &p, const jpoint &q) { pt_add_inl(r, p, q); }
