/*
 * fgv_oracle.c -- CPU restatement of the crypto leg of Fabric's committer path.
 *
 * TEST INFRASTRUCTURE ONLY (see fgv_oracle.h).  Written for clarity, not speed:
 * 4x64-bit limbs, generic Montgomery multiplication for both p and n, Jacobian
 * points with explicit exceptional-case handling, plain double-and-add.
 *
 * Parity pins (tests/test_oracle_golden.py):
 *   - SHA-256 against Python hashlib on the same inputs;
 *   - ECDSA against the CA signatures held in the reference's own MSP fixtures
 *     (msp/testdata, sampleconfig/msp), including the high-S signcert asserted by
 *     msp/msp_test.go:1492-1535, and against OpenSSL 3.0.2 on generated vectors.
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include "fgv_oracle.h"

#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <string.h>

/* ------------------------------------------------------------------ SHA-256 */

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t *p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
           ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = k + S1 + ch + K256[i] + w[i];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

void oracle_sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t full = len / 64;
  for (size_t i = 0; i < full; i++) sha256_block(h, msg + 64 * i);
  uint8_t tail[128];
  size_t rem = len - 64 * full;
  memset(tail, 0, sizeof tail);
  if (rem) memcpy(tail, msg + 64 * full, rem);
  tail[rem] = 0x80;
  size_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha256_block(h, tail);
  if (tl == 128) sha256_block(h, tail + 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

/* ------------------------------------------------------------ 256-bit ints */

typedef struct { uint64_t v[4]; } u256;
typedef unsigned __int128 u128;

static void u256_from_be(u256 *a, const uint8_t b[32]) {
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int j = 0; j < 8; j++) w = (w << 8) | b[(3 - i) * 8 + j];
    a->v[i] = w;
  }
}
static void u256_to_be(uint8_t b[32], const u256 *a) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256 *a, const u256 *b) {
  for (int i = 3; i >= 0; i--) {
    if (a->v[i] > b->v[i]) return 1;
    if (a->v[i] < b->v[i]) return -1;
  }
  return 0;
}
static int u256_is_zero(const u256 *a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3]); }
static uint64_t u256_add(u256 *r, const u256 *a, const u256 *b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a->v[i] + b->v[i];
    r->v[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static uint64_t u256_sub(u256 *r, const u256 *a, const u256 *b) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a->v[i] - b->v[i] - borrow;
    r->v[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) & 1;
  }
  return borrow;
}

/* Montgomery context for an odd modulus m < 2^256, R = 2^256. */
typedef struct {
  u256 m;
  uint64_t m0inv; /* -m^-1 mod 2^64 */
  u256 rr;        /* R^2 mod m */
  u256 one;       /* R mod m */
} mctx;

static void mod_add(u256 *r, const u256 *a, const u256 *b, const mctx *c) {
  u256 t;
  uint64_t carry = u256_add(&t, a, b);
  u256 t2;
  uint64_t borrow = u256_sub(&t2, &t, &c->m);
  *r = (carry || !borrow) ? t2 : t;
}
static void mod_sub(u256 *r, const u256 *a, const u256 *b, const mctx *c) {
  u256 t;
  uint64_t borrow = u256_sub(&t, a, b);
  if (borrow) u256_add(&t, &t, &c->m);
  *r = t;
}

static void mont_mul(u256 *r, const u256 *a, const u256 *b, const mctx *c) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 x;
    uint64_t carry = 0;
    for (int j = 0; j < 4; j++) {
      x = (u128)a->v[j] * b->v[i] + t[j] + carry;
      t[j] = (uint64_t)x;
      carry = (uint64_t)(x >> 64);
    }
    x = (u128)t[4] + carry;
    t[4] = (uint64_t)x;
    t[5] = (uint64_t)(x >> 64);
    uint64_t m = t[0] * c->m0inv;
    x = (u128)m * c->m.v[0] + t[0];
    carry = (uint64_t)(x >> 64);
    for (int j = 1; j < 4; j++) {
      x = (u128)m * c->m.v[j] + t[j] + carry;
      t[j - 1] = (uint64_t)x;
      carry = (uint64_t)(x >> 64);
    }
    x = (u128)t[4] + carry;
    t[3] = (uint64_t)x;
    t[4] = t[5] + (uint64_t)(x >> 64);
  }
  u256 res = {{t[0], t[1], t[2], t[3]}};
  u256 sub;
  uint64_t borrow = u256_sub(&sub, &res, &c->m);
  *r = (t[4] || !borrow) ? sub : res;
}

static void mctx_init(mctx *c, const u256 *m) {
  c->m = *m;
  /* Newton iteration for m^-1 mod 2^64 */
  uint64_t inv = 1;
  for (int i = 0; i < 7; i++) inv *= 2 - m->v[0] * inv;
  c->m0inv = (uint64_t)0 - inv;
  /* R mod m = 2^256 - m (m > 2^255 for both P-256 moduli) */
  u256 zero = {{0, 0, 0, 0}};
  u256_sub(&c->one, &zero, m);
  /* R^2 mod m by 256 modular doublings of R */
  u256 x = c->one;
  for (int i = 0; i < 256; i++) mod_add(&x, &x, &x, c);
  c->rr = x;
}
static void to_mont(u256 *r, const u256 *a, const mctx *c) { mont_mul(r, a, &c->rr, c); }
static void from_mont(u256 *r, const u256 *a, const mctx *c) {
  u256 one = {{1, 0, 0, 0}};
  mont_mul(r, a, &one, c);
}
/* a^e (a in Montgomery form), plain left-to-right square and multiply */
static void mont_pow(u256 *r, const u256 *a, const u256 *e, const mctx *c) {
  u256 acc = c->one;
  for (int i = 255; i >= 0; i--) {
    mont_mul(&acc, &acc, &acc, c);
    if ((e->v[i / 64] >> (i % 64)) & 1) mont_mul(&acc, &acc, a, c);
  }
  *r = acc;
}
/* Fermat inverse; a in Montgomery form, a != 0 */
static void mont_inv(u256 *r, const u256 *a, const mctx *c) {
  u256 e, two = {{2, 0, 0, 0}};
  u256_sub(&e, &c->m, &two);
  mont_pow(r, a, &e, c);
}

/* ---------------------------------------------------------------- P-256 */

static const uint8_t P256_P[32] = {
    0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
static const uint8_t P256_N[32] = {
    0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x00, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xbc, 0xe6, 0xfa, 0xad, 0xa7, 0x17, 0x9e, 0x84, 0xf3, 0xb9, 0xca, 0xc2, 0xfc, 0x63, 0x25, 0x51};
static const uint8_t P256_B[32] = {
    0x5a, 0xc6, 0x35, 0xd8, 0xaa, 0x3a, 0x93, 0xe7, 0xb3, 0xeb, 0xbd, 0x55, 0x76, 0x98, 0x86, 0xbc,
    0x65, 0x1d, 0x06, 0xb0, 0xcc, 0x53, 0xb0, 0xf6, 0x3b, 0xce, 0x3c, 0x3e, 0x27, 0xd2, 0x60, 0x4b};
static const uint8_t P256_GX[32] = {
    0x6b, 0x17, 0xd1, 0xf2, 0xe1, 0x2c, 0x42, 0x47, 0xf8, 0xbc, 0xe6, 0xe5, 0x63, 0xa4, 0x40, 0xf2,
    0x77, 0x03, 0x7d, 0x81, 0x2d, 0xeb, 0x33, 0xa0, 0xf4, 0xa1, 0x39, 0x45, 0xd8, 0x98, 0xc2, 0x96};
static const uint8_t P256_GY[32] = {
    0x4f, 0xe3, 0x42, 0xe2, 0xfe, 0x1a, 0x7f, 0x9b, 0x8e, 0xe7, 0xeb, 0x4a, 0x7c, 0x0f, 0x9e, 0x16,
    0x2b, 0xce, 0x33, 0x57, 0x6b, 0x31, 0x5e, 0xce, 0xcb, 0xb6, 0x40, 0x68, 0x37, 0xbf, 0x51, 0xf5};
/* n >> 1, bccsp/utils/ecdsa.go:26-31 (curveHalfOrders) */
static const uint8_t P256_HALF_N[32] = {
    0x7f, 0xff, 0xff, 0xff, 0x80, 0x00, 0x00, 0x00, 0x7f, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xde, 0x73, 0x7d, 0x56, 0xd3, 0x8b, 0xcf, 0x42, 0x79, 0xdc, 0xe5, 0x61, 0x7e, 0x31, 0x92, 0xa8};

typedef struct {
  mctx fp, fn;
  u256 b_m, gx_m, gy_m, three_m; /* Montgomery form over p */
  u256 p, n, half_n;
} curve_t;

static curve_t CURVE;
static pthread_once_t CURVE_ONCE = PTHREAD_ONCE_INIT;

static void curve_init(void) {
  u256_from_be(&CURVE.p, P256_P);
  u256_from_be(&CURVE.n, P256_N);
  u256_from_be(&CURVE.half_n, P256_HALF_N);
  mctx_init(&CURVE.fp, &CURVE.p);
  mctx_init(&CURVE.fn, &CURVE.n);
  u256 t;
  u256_from_be(&t, P256_B);
  to_mont(&CURVE.b_m, &t, &CURVE.fp);
  u256_from_be(&t, P256_GX);
  to_mont(&CURVE.gx_m, &t, &CURVE.fp);
  u256_from_be(&t, P256_GY);
  to_mont(&CURVE.gy_m, &t, &CURVE.fp);
  u256 three = {{3, 0, 0, 0}};
  to_mont(&CURVE.three_m, &three, &CURVE.fp);
}
static const curve_t *curve(void) {
  pthread_once(&CURVE_ONCE, curve_init);
  return &CURVE;
}

typedef struct { u256 x, y, z; } jpoint; /* Jacobian, Montgomery form; z == 0 <=> infinity */

#define FP (&C->fp)
static void fmul(u256 *r, const u256 *a, const u256 *b, const curve_t *C) { mont_mul(r, a, b, FP); }
static void fadd(u256 *r, const u256 *a, const u256 *b, const curve_t *C) { mod_add(r, a, b, FP); }
static void fsub(u256 *r, const u256 *a, const u256 *b, const curve_t *C) { mod_sub(r, a, b, FP); }

/* dbl-2001-b (a = -3) */
static void jdouble(jpoint *r, const jpoint *p, const curve_t *C) {
  if (u256_is_zero(&p->z) || u256_is_zero(&p->y)) {
    memset(r, 0, sizeof *r);
    return;
  }
  u256 delta, gamma, beta, alpha, t1, t2, x3, y3, z3;
  fmul(&delta, &p->z, &p->z, C);
  fmul(&gamma, &p->y, &p->y, C);
  fmul(&beta, &p->x, &gamma, C);
  fsub(&t1, &p->x, &delta, C);
  fadd(&t2, &p->x, &delta, C);
  fmul(&alpha, &t1, &t2, C);
  fmul(&alpha, &alpha, &C->three_m, C);
  fmul(&x3, &alpha, &alpha, C);
  u256 beta8;
  fadd(&beta8, &beta, &beta, C);
  fadd(&beta8, &beta8, &beta8, C);
  fadd(&beta8, &beta8, &beta8, C);
  fsub(&x3, &x3, &beta8, C);
  fadd(&t1, &p->y, &p->z, C);
  fmul(&z3, &t1, &t1, C);
  fsub(&z3, &z3, &gamma, C);
  fsub(&z3, &z3, &delta, C);
  u256 beta4;
  fadd(&beta4, &beta, &beta, C);
  fadd(&beta4, &beta4, &beta4, C);
  fsub(&t1, &beta4, &x3, C);
  fmul(&y3, &alpha, &t1, C);
  fmul(&t2, &gamma, &gamma, C);
  fadd(&t2, &t2, &t2, C);
  fadd(&t2, &t2, &t2, C);
  fadd(&t2, &t2, &t2, C);
  fsub(&y3, &y3, &t2, C);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}

/* general Jacobian addition with every exceptional case handled (group law is complete) */
static void jadd(jpoint *r, const jpoint *p, const jpoint *q, const curve_t *C) {
  if (u256_is_zero(&p->z)) { *r = *q; return; }
  if (u256_is_zero(&q->z)) { *r = *p; return; }
  u256 z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
  fmul(&z1z1, &p->z, &p->z, C);
  fmul(&z2z2, &q->z, &q->z, C);
  fmul(&u1, &p->x, &z2z2, C);
  fmul(&u2, &q->x, &z1z1, C);
  fmul(&t, &q->z, &z2z2, C);
  fmul(&s1, &p->y, &t, C);
  fmul(&t, &p->z, &z1z1, C);
  fmul(&s2, &q->y, &t, C);
  fsub(&h, &u2, &u1, C);
  fsub(&rr, &s2, &s1, C);
  if (u256_is_zero(&h)) {
    if (u256_is_zero(&rr)) { jdouble(r, p, C); return; }
    memset(r, 0, sizeof *r);
    return;
  }
  u256 h2, h3, u1h2, x3, y3, z3;
  fmul(&h2, &h, &h, C);
  fmul(&h3, &h2, &h, C);
  fmul(&u1h2, &u1, &h2, C);
  fmul(&x3, &rr, &rr, C);
  fsub(&x3, &x3, &h3, C);
  fsub(&x3, &x3, &u1h2, C);
  fsub(&x3, &x3, &u1h2, C);
  fsub(&t, &u1h2, &x3, C);
  fmul(&y3, &rr, &t, C);
  fmul(&t, &s1, &h3, C);
  fsub(&y3, &y3, &t, C);
  fmul(&z3, &p->z, &q->z, C);
  fmul(&z3, &z3, &h, C);
  r->x = x3;
  r->y = y3;
  r->z = z3;
}

static void jmul(jpoint *r, const jpoint *p, const u256 *k, const curve_t *C) {
  jpoint acc;
  memset(&acc, 0, sizeof acc);
  for (int i = 255; i >= 0; i--) {
    jdouble(&acc, &acc, C);
    if ((k->v[i / 64] >> (i % 64)) & 1) jadd(&acc, &acc, p, C);
  }
  *r = acc;
}

/* y^2 == x^3 - 3x + b with x,y < p  (Go nistec pointFromAffine) */
static int on_curve(const u256 *x, const u256 *y, jpoint *out, const curve_t *C) {
  if (u256_cmp(x, &C->p) >= 0 || u256_cmp(y, &C->p) >= 0) return 0;
  u256 xm, ym, lhs, rhs, t;
  to_mont(&xm, x, FP);
  to_mont(&ym, y, FP);
  fmul(&lhs, &ym, &ym, C);
  fmul(&rhs, &xm, &xm, C);
  fmul(&rhs, &rhs, &xm, C);
  fmul(&t, &xm, &C->three_m, C);
  fsub(&rhs, &rhs, &t, C);
  fadd(&rhs, &rhs, &C->b_m, C);
  if (u256_cmp(&lhs, &rhs) != 0) return 0;
  out->x = xm;
  out->y = ym;
  out->z = C->fp.one;
  return 1;
}

static int verify_core(const u256 *qx, const u256 *qy, const u256 *r, const u256 *s,
                       const uint8_t *digest, size_t digest_len) {
  const curve_t *C = curve();
  jpoint Q, G;
  if (!on_curve(qx, qy, &Q, C)) return 5;
  if (u256_is_zero(r) || u256_is_zero(s)) return 4;
  if (u256_cmp(r, &C->n) >= 0 || u256_cmp(s, &C->n) >= 0) return 4;
  /* hashToNat: leftmost bitlen(n)=256 bits of the digest, then mod n */
  uint8_t eb[32];
  memset(eb, 0, 32);
  if (digest_len >= 32) memcpy(eb, digest, 32);
  else memcpy(eb + (32 - digest_len), digest, digest_len);
  u256 e;
  u256_from_be(&e, eb);
  if (u256_cmp(&e, &C->n) >= 0) u256_sub(&e, &e, &C->n);
  const mctx *N = &C->fn;
  u256 sm, w, em, rm, u1m, u2m, u1, u2;
  to_mont(&sm, s, N);
  mont_inv(&w, &sm, N);
  to_mont(&em, &e, N);
  to_mont(&rm, r, N);
  mont_mul(&u1m, &em, &w, N);
  mont_mul(&u2m, &rm, &w, N);
  from_mont(&u1, &u1m, N);
  from_mont(&u2, &u2m, N);
  G.x = C->gx_m;
  G.y = C->gy_m;
  G.z = C->fp.one;
  jpoint p1, p2, R;
  jmul(&p1, &G, &u1, C);
  jmul(&p2, &Q, &u2, C);
  jadd(&R, &p1, &p2, C);
  if (u256_is_zero(&R.z)) return 1;
  u256 zi, zi2, xm, x;
  mont_inv(&zi, &R.z, FP);
  fmul(&zi2, &zi, &zi, C);
  fmul(&xm, &R.x, &zi2, C);
  from_mont(&x, &xm, FP);
  if (u256_cmp(&x, &C->n) >= 0) u256_sub(&x, &x, &C->n);
  return u256_cmp(&x, r) == 0 ? 0 : 1;
}

int oracle_p256_base_mult(const uint8_t kb[32], uint8_t out_x[32], uint8_t out_y[32]) {
  const curve_t *C = curve();
  u256 k;
  u256_from_be(&k, kb);
  jpoint G = {C->gx_m, C->gy_m, C->fp.one}, R;
  jmul(&R, &G, &k, C);
  if (u256_is_zero(&R.z)) return 1;
  u256 zi, zi2, zi3, x, y;
  mont_inv(&zi, &R.z, FP);
  fmul(&zi2, &zi, &zi, C);
  fmul(&zi3, &zi2, &zi, C);
  fmul(&x, &R.x, &zi2, C);
  fmul(&y, &R.y, &zi3, C);
  from_mont(&x, &x, FP);
  from_mont(&y, &y, FP);
  u256_to_be(out_x, &x);
  u256_to_be(out_y, &y);
  return 0;
}

/* --------------------------------------------------- Go encoding/asn1 rules */

/* parseTagAndLength (Go 1.21.9 encoding/asn1/asn1.go).  Returns 0 on success. */
static int der_tag_len(const uint8_t *b, size_t n, size_t *off, int *cls, int *compound,
                       int *tag, size_t *length) {
  size_t o = *off;
  if (o >= n) return -1;
  uint8_t t = b[o++];
  *cls = t >> 6;
  *compound = (t & 0x20) != 0;
  *tag = t & 0x1f;
  if (*tag == 0x1f) {
    /* high-tag-number form: base-128, minimal, >= 0x1f, < 2^31 */
    uint64_t v = 0;
    int shifted = 0;
    for (;;) {
      if (o >= n) return -1;
      if (shifted == 5) return -1;
      uint8_t c = b[o++];
      if (shifted == 0 && c == 0x80) return -1;
      v = (v << 7) | (c & 0x7f);
      shifted++;
      if (!(c & 0x80)) break;
    }
    if (v > 0x7fffffff) return -1;
    if (v < 0x1f) return -1;
    *tag = (int)v;
  }
  if (o >= n) return -1;
  uint8_t l = b[o++];
  if (!(l & 0x80)) {
    *length = l & 0x7f;
  } else {
    int nb = l & 0x7f;
    if (nb == 0) return -1; /* indefinite length */
    size_t len = 0;
    for (int i = 0; i < nb; i++) {
      if (o >= n) return -1;
      if (len >= (1u << 23)) return -1;
      len = (len << 8) | b[o++];
      if (len == 0) return -1; /* superfluous leading zeros */
    }
    if (len < 0x80) return -1; /* non-minimal */
    *length = len;
  }
  *off = o;
  return 0;
}

/* one INTEGER into a big.Int: returns 0 ok; *neg = 1 if negative; value bytes span */
static int der_integer(const uint8_t *b, size_t n, size_t *off, const uint8_t **val,
                       size_t *vlen, int *neg) {
  if (*off == n) return -1; /* sequence truncated */
  int cls, compound, tag;
  size_t len;
  if (der_tag_len(b, n, off, &cls, &compound, &tag, &len)) return -1;
  if (cls != 0 || tag != 2 || compound) return -1;
  if (*off + len < *off || *off + len > n) return -1;
  const uint8_t *v = b + *off;
  *off += len;
  if (len == 0) return -1; /* empty integer */
  if (len > 1 && ((v[0] == 0 && !(v[1] & 0x80)) || (v[0] == 0xff && (v[1] & 0x80))))
    return -1; /* not minimally encoded */
  *neg = (v[0] & 0x80) != 0;
  *val = v;
  *vlen = len;
  return 0;
}

static int bytes_to_u256(const uint8_t *v, size_t len, uint8_t out[32]) {
  /* strip leading zeros; returns 1 if value >= 2^256 */
  while (len > 0 && v[0] == 0) { v++; len--; }
  memset(out, 0, 32);
  if (len > 32) return 1;
  memcpy(out + 32 - len, v, len);
  return 0;
}

int oracle_der_decode(const uint8_t *sig, size_t n, uint8_t r[32], uint8_t s[32], int *r_big,
                      int *s_big) {
  size_t off = 0;
  int cls, compound, tag;
  size_t len;
  if (n == 0) return 2;
  if (der_tag_len(sig, n, &off, &cls, &compound, &tag, &len)) return 2;
  if (cls != 0 || tag != 16 || !compound) return 2;
  if (off + len < off || off + len > n) return 2;
  const uint8_t *inner = sig + off;
  size_t in_n = len, io = 0;
  /* bytes after the outer SEQUENCE are ignored (utils/ecdsa.go:44 drops `rest`) */
  const uint8_t *rv, *sv;
  size_t rl, sl;
  int rneg, sneg;
  if (der_integer(inner, in_n, &io, &rv, &rl, &rneg)) return 2;
  if (der_integer(inner, in_n, &io, &sv, &sl, &sneg)) return 2;
  /* extra elements/bytes inside the SEQUENCE are ignored (Go struct parsing) */
  /* R.Sign() != 1 / S.Sign() != 1 -> error (utils/ecdsa.go:56-62) */
  int rz = 1, sz = 1;
  for (size_t i = 0; i < rl; i++) if (rv[i]) rz = 0;
  for (size_t i = 0; i < sl; i++) if (sv[i]) sz = 0;
  if (rneg || rz || sneg || sz) return 2;
  *r_big = bytes_to_u256(rv, rl, r);
  *s_big = bytes_to_u256(sv, sl, s);
  return 0;
}

int oracle_p256_verify_rs(const uint8_t qx[32], const uint8_t qy[32], const uint8_t rb[32],
                          const uint8_t sb[32], const uint8_t digest[32]) {
  u256 x, y, r, s;
  u256_from_be(&x, qx);
  u256_from_be(&y, qy);
  u256_from_be(&r, rb);
  u256_from_be(&s, sb);
  return verify_core(&x, &y, &r, &s, digest, 32);
}

/* front half shared by both arithmetic back-ends: sw/impl.go:247-270 + sw/ecdsa.go:41-57 */
static int verify_front(const uint8_t *sig, size_t sig_len, size_t digest_len, uint8_t r[32],
                        uint8_t s[32], int *big) {
  if (sig_len == 0 || digest_len == 0) return 6;
  int r_big = 0, s_big = 0;
  if (oracle_der_decode(sig, sig_len, r, s, &r_big, &s_big)) return 2;
  const curve_t *C = curve();
  u256 sv;
  u256_from_be(&sv, s);
  if (s_big || u256_cmp(&sv, &C->half_n) > 0) return 3;
  *big = r_big;
  return 0;
}

int oracle_p256_verify_der(const uint8_t qx[32], const uint8_t qy[32], const uint8_t *sig,
                           size_t sig_len, const uint8_t *digest, size_t digest_len) {
  uint8_t r[32], s[32];
  int big = 0;
  int st = verify_front(sig, sig_len, digest_len, r, s, &big);
  if (st) return st;
  u256 x, y, rv, sv;
  u256_from_be(&x, qx);
  u256_from_be(&y, qy);
  const curve_t *C = curve();
  jpoint Q;
  if (!on_curve(&x, &y, &Q, C)) return 5;
  if (big) return 4;
  u256_from_be(&rv, r);
  u256_from_be(&sv, s);
  return verify_core(&x, &y, &rv, &sv, digest, digest_len);
}

/* ------------------------------------------------------- OpenSSL back-end */

int oracle_p256_verify_der_ossl(const uint8_t qx[32], const uint8_t qy[32], const uint8_t *sig,
                                size_t sig_len, const uint8_t *digest, size_t digest_len) {
  uint8_t r[32], s[32];
  int big = 0;
  int st = verify_front(sig, sig_len, digest_len, r, s, &big);
  if (st) return st;
  int ret = 1;
  EC_KEY *key = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
  BIGNUM *bx = BN_bin2bn(qx, 32, NULL), *by = BN_bin2bn(qy, 32, NULL);
  if (!key || !bx || !by) { ret = -1; goto out; }
  if (EC_KEY_set_public_key_affine_coordinates(key, bx, by) != 1) { ret = 5; goto out; }
  if (big) { ret = 4; goto out; }
  {
    const curve_t *C = curve();
    u256 rv;
    u256_from_be(&rv, r);
    if (u256_cmp(&rv, &C->n) >= 0) { ret = 4; goto out; }
  }
  {
    ECDSA_SIG *es = ECDSA_SIG_new();
    BIGNUM *br = BN_bin2bn(r, 32, NULL), *bs = BN_bin2bn(s, 32, NULL);
    ECDSA_SIG_set0(es, br, bs);
    int v = ECDSA_do_verify(digest, (int)digest_len, es, key);
    ECDSA_SIG_free(es);
    ret = (v == 1) ? 0 : 1;
  }
out:
  BN_free(bx);
  BN_free(by);
  EC_KEY_free(key);
  return ret;
}

/* the same with the key parsed once (EC_KEY made by oracle_p256_key_new, shared read-only by
 * threads): what a long-running peer does with its deserialized identities */
void *oracle_p256_key_new(const uint8_t qx[32], const uint8_t qy[32]) {
  EC_KEY *key = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
  BIGNUM *bx = BN_bin2bn(qx, 32, NULL), *by = BN_bin2bn(qy, 32, NULL);
  if (!key || !bx || !by || EC_KEY_set_public_key_affine_coordinates(key, bx, by) != 1) {
    EC_KEY_free(key);
    key = NULL;
  }
  BN_free(bx);
  BN_free(by);
  return key;
}
void oracle_p256_key_free(void *key) { EC_KEY_free((EC_KEY *)key); }
int oracle_p256_verify_der_key(void *key, const uint8_t *sig, size_t sig_len, const uint8_t *digest,
                               size_t digest_len) {
  uint8_t r[32], s[32];
  int big = 0;
  int st = verify_front(sig, sig_len, digest_len, r, s, &big);
  if (st) return st;
  if (!key) return 5;
  if (big) return 4;
  const curve_t *C = curve();
  u256 rv;
  u256_from_be(&rv, r);
  if (u256_cmp(&rv, &C->n) >= 0) return 4;
  ECDSA_SIG *es = ECDSA_SIG_new();
  BIGNUM *br = BN_bin2bn(r, 32, NULL), *bs = BN_bin2bn(s, 32, NULL);
  ECDSA_SIG_set0(es, br, bs);
  const int v = ECDSA_do_verify(digest, (int)digest_len, es, (EC_KEY *)key);
  ECDSA_SIG_free(es);
  return v == 1 ? 0 : 1;
}

/* ------------------------------------------------------- threaded batches */

typedef struct {
  const uint8_t *keys, *msg_buf, *sig_buf;
  const uint64_t *msg_off, *sig_off;
  const uint32_t *msg_len, *sig_len;
  uint8_t *status;
  size_t lo, hi;
  int use_ossl;
} job_t;

static void *verify_worker(void *arg) {
  job_t *j = (job_t *)arg;
  for (size_t i = j->lo; i < j->hi; i++) {
    uint8_t d[32];
    oracle_sha256(j->msg_buf + j->msg_off[i], j->msg_len[i], d);
    const uint8_t *k = j->keys + 64 * i;
    const uint8_t *sg = j->sig_buf + j->sig_off[i];
    j->status[i] = (uint8_t)(j->use_ossl ? oracle_p256_verify_der_ossl(k, k + 32, sg, j->sig_len[i], d, 32)
                                         : oracle_p256_verify_der(k, k + 32, sg, j->sig_len[i], d, 32));
  }
  return NULL;
}

void oracle_verify_msgs_batch(const uint8_t *keys, const uint8_t *msg_buf, const uint64_t *msg_off,
                              const uint32_t *msg_len, const uint8_t *sig_buf,
                              const uint64_t *sig_off, const uint32_t *sig_len, size_t n,
                              uint8_t *status, int threads, int use_ossl) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  curve();
  pthread_t tid[256];
  job_t jobs[256];
  size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){keys, msg_buf, sig_buf, msg_off, sig_off, msg_len, sig_len, status,
                      t * per < n ? t * per : n, (t + 1) * per < n ? (t + 1) * per : n, use_ossl};
    pthread_create(&tid[t], NULL, verify_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

/* ------------------------------------------------------- P-384 (OpenSSL back-end)
 * bccsp sw verifyECDSA for a P-384 key (fabric-lib-go bccsp/sw/ecdsa.go:41-57): the same Go-rule
 * DER decode (48-byte integers), the low-S rule with the P-384 half order (bccsp/utils/
 * ecdsa.go:26-31), then Go ecdsa.Verify's rules with OpenSSL's group arithmetic (r, s in [1, n),
 * the 32-byte digest as e -- no truncation against a 384-bit order --, R != inf, x_R mod n == r).
 * Status bytes as for P-256. */
int oracle_p384_verify_der(const uint8_t qx[48], const uint8_t qy[48], const uint8_t *sig, size_t sig_len,
                           const uint8_t *digest, size_t digest_len) {
  if (sig_len == 0 || digest_len == 0) return 6;
  size_t off = 0, len;
  int cls, compound, tag;
  if (der_tag_len(sig, sig_len, &off, &cls, &compound, &tag, &len)) return 2;
  if (cls != 0 || tag != 16 || !compound) return 2;
  if (off + len < off || off + len > sig_len) return 2;
  const uint8_t *inner = sig + off, *rv, *sv;
  size_t io = 0, rl, sl;
  int rneg, sneg;
  if (der_integer(inner, len, &io, &rv, &rl, &rneg)) return 2;
  if (der_integer(inner, len, &io, &sv, &sl, &sneg)) return 2;
  int rz = 1, sz = 1;
  for (size_t i = 0; i < rl; i++) if (rv[i]) rz = 0;
  for (size_t i = 0; i < sl; i++) if (sv[i]) sz = 0;
  if (rneg || rz || sneg || sz) return 2;
  int ret = 1;
  EC_KEY *key = EC_KEY_new_by_curve_name(NID_secp384r1);
  const EC_GROUP *grp = EC_KEY_get0_group(key);
  BIGNUM *br = BN_bin2bn(rv, (int)rl, NULL), *bs = BN_bin2bn(sv, (int)sl, NULL);
  BIGNUM *half = BN_dup(EC_GROUP_get0_order(grp));
  BIGNUM *bx = BN_bin2bn(qx, 48, NULL), *by = BN_bin2bn(qy, 48, NULL);
  BN_rshift1(half, half);
  if (BN_cmp(bs, half) > 0) { ret = 3; goto out; }
  if (EC_KEY_set_public_key_affine_coordinates(key, bx, by) != 1) { ret = 5; goto out; }
  if (BN_cmp(br, EC_GROUP_get0_order(grp)) >= 0) { ret = 4; goto out; }
  {
    ECDSA_SIG *es = ECDSA_SIG_new();
    ECDSA_SIG_set0(es, br, bs);
    br = bs = NULL;
    const int v = ECDSA_do_verify(digest, (int)digest_len, es, key);
    ECDSA_SIG_free(es);
    ret = v == 1 ? 0 : 1;
  }
out:
  BN_free(br);
  BN_free(bs);
  BN_free(half);
  BN_free(bx);
  BN_free(by);
  EC_KEY_free(key);
  return ret;
}
