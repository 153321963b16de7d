// p256_fe28.h -- P-256 field arithmetic in radix 2^28 for the k_point fast path (gfx950).
//
// Why a second representation: with 8 x 32-bit limbs every partial product needs a carry
// chain (v_mad_u64_u32 + 64-bit add + register-pair moves, ~4.5 VALU per product, see
// DESIGN.md s4).  With 10 limbs of 28 bits a column of the schoolbook product is a plain
// 64-bit accumulation -- ONE v_mad_u64_u32 per partial product, no carries -- and the
// Montgomery reduction needs no multiplier: p == -1 mod 2^28, so m = t_i mod 2^28 and
// m*p only lands on limbs i+3, i+6, i+8, i+9 (four v_mad_u64_u32 by small constants).
//
// Representation: f28 = 10 limbs, value = sum v[i] * 2^(28 i), Montgomery form with
// R = 2^280 (x -> x * 2^280 mod p).  Limbs are NOT kept canonical (lazy reduction):
//   normalized  limbs 0..8 < 2^28, limb 9 small   (f28_mul / f28_sqr / f28_norm outputs)
//   loose       limbs < 2^30                      (f28_sub outputs; valid mul/sqr inputs)
// Value bounds (multiples of p) are tracked at the call sites (p256_kernels.hip); a product
// of inputs below 2^12 p stays < 2p after reduction (R = 2^280 > 2^24 p).  Overflow bound of
// a column: 10 * (2^30)^2 + reduction terms < 2^64.
//
// Zero tests work on normalized values < 2p, whose representation is unique: x == 0 mod p
// <=> limbs == 0 or limbs == p.
#pragma once
#include "p256_field.h"

#define F28_MASK 0x0FFFFFFFu

struct f28 {
  uint32_t v[10];
};

// p in radix 2^28
__constant__ static const uint32_t P28[10] = {0xFFFFFFFu, 0xFFFFFFFu, 0xFFFFFFFu, 0xFFFu, 0u,
                                              0u,         0x1000000u, 0u,         0xFFFFFFFu, 0xFu};
// k*p with every limb 0..8 in [2^29 - 2, 3 * 2^28): subtrahend constants of f28_sub (a limb of a
// normalized subtrahend is < 2^28, its top limb must stay <= the constant's top limb)
__constant__ static const uint32_t C4P28[10] = {0x2ffffffcu, 0x2ffffffdu, 0x2ffffffdu, 0x20003ffdu, 0x1ffffffeu,
                                                0x1ffffffeu, 0x23fffffeu, 0x1ffffffeu, 0x2ffffffau, 0x3du};
__constant__ static const uint32_t C8P28[10] = {0x2ffffff8u, 0x2ffffffdu, 0x2ffffffdu, 0x20007ffdu, 0x1ffffffeu,
                                                0x1ffffffeu, 0x27fffffeu, 0x1ffffffeu, 0x2ffffff6u, 0x7du};
__constant__ static const uint32_t C16P28[10] = {0x2ffffff0u, 0x2ffffffdu, 0x2ffffffdu, 0x2000fffdu, 0x1ffffffeu,
                                                 0x1ffffffeu, 0x1ffffffeu, 0x1fffffffu, 0x2fffffeeu, 0xfdu};
// R^2 mod p (to Montgomery-280) and R mod p (Montgomery one), radix 2^28
__constant__ static const uint32_t R2P28[10] = {0x50000u,    0x300000u,  0u,         0u,         0xffffffau,
                                                0xfffffbfu,  0xffffeffu, 0xfffafffu, 0x2ffffu,   0u};
__constant__ static const uint32_t ONE28[10] = {0x1000000u, 0u,         0u,         0u,         0xfffff00u,
                                                0xfffffffu, 0xfffffffu, 0xfefffffu, 0xffffffu,  0u};
// 2^232 (< p) as 8 x 32-bit limbs: fe_mul(x * 2^280, C232) = x * 2^256 (the exact kernel's view of a
// Montgomery-280 key-comb entry)
__constant__ static const uint32_t C232_32[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0x100u};
// 2^280 mod p as 8 x 32-bit limbs: fe_mul(x * 2^256, C280) = x * 2^280 (table conversion)
__constant__ static const uint32_t C280_32[8] = {0x1000000u, 0u,         0u,         0xff000000u,
                                                 0xffffffffu, 0xffffffffu, 0xfeffffffu, 0xffffffu};

FGV_DEV void f28_load_c(f28 &r, const uint32_t *c) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c[i];
}

// 8 x 32-bit little-endian limbs (a value < 2^256) -> radix 2^28
FGV_DEV void f28_from32(f28 &r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 28 * i, wi = bit >> 5, sh = bit & 31;
    const uint32_t hi = wi + 1 < 8 ? w[wi + 1] : 0u;
    r.v[i] = __builtin_amdgcn_alignbit(hi, w[wi], (uint32_t)sh) & F28_MASK;
  }
  r.v[9] = w[7] >> 28;
}

// A multiplier the compiler cannot see: keeps `t += m * K` one v_mad_u64_u32 (m * 2^12 would
// otherwise become a 64-bit shift + a 64-bit add, and m * (2^28 - 1) a mul_lo/mul_hi pair).
template <uint32_t K>
FGV_DEV uint32_t f28_opaque() {
  uint32_t k;
  asm("s_mov_b32 %0, %1" : "=s"(k) : "i"(K));
  return k;
}

// Montgomery reduction of the 19-column product t[0..18] (t[19] == 0): r = t / 2^280 mod p,
// normalized, value < t / 2^280 + p.
FGV_DEV void f28_redc(f28 &r, uint64_t t[20]) {
  const uint32_t k12 = f28_opaque<0x1000u>(), k24 = f28_opaque<0x1000000u>(), km = f28_opaque<0xFFFFFFFu>(),
                 k15 = f28_opaque<0xFu>();
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t m = (uint32_t)t[i] & F28_MASK;
    t[i + 1] += t[i] >> 28;                 // (t_i - m) / 2^28
    t[i + 3] += (uint64_t)m * k12;          // m * 2^96
    t[i + 6] += (uint64_t)m * k24;          // m * 2^192
    t[i + 8] += (uint64_t)m * km;           // -m * 2^224 + m * 2^252 ...
    t[i + 9] += (uint64_t)m * k15;          // ... + 15 m * 2^252  (= m * 2^256 - m * 2^224)
  }
#pragma unroll
  for (int i = 10; i < 19; i++) {
    r.v[i - 10] = (uint32_t)t[i] & F28_MASK;
    t[i + 1] += t[i] >> 28;
  }
  r.v[9] = (uint32_t)t[19];
}

// inputs loose (limbs < 2^30); output normalized, < 2p when a*b < 2^280 p
FGV_DEV void f28_mul(f28 &r, const f28 &a, const f28 &b) {
  uint64_t t[20];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = k - i;
      if (j >= 0 && j < 10) acc += (uint64_t)a.v[i] * b.v[j];
    }
    t[k] = acc;
  }
  t[19] = 0;
  f28_redc(r, t);
}

// r = (a*b + c*d) / 2^280 mod p: the two products summed column by column, ONE reduction.
// a, b, c loose (limbs < 2^30), d normalized: a column stays below 10 * 2^60 + 10 * 2^58 <
// 2^63.7, the reduction's terms fit in the rest; output normalized, < 2p when a*b + c*d < 2^280 p
FGV_DEV void f28_mul2(f28 &r, const f28 &a, const f28 &b, const f28 &c, const f28 &d) {
  uint64_t t[20];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = k - i;
      if (j >= 0 && j < 10) acc += (uint64_t)a.v[i] * b.v[j] + (uint64_t)c.v[i] * d.v[j];
    }
    t[k] = acc;
  }
  t[19] = 0;
  f28_redc(r, t);
}

FGV_DEV void f28_sqr(f28 &r, const f28 &a) {
  uint32_t d[10];
#pragma unroll
  for (int i = 0; i < 10; i++) d[i] = a.v[i] << 1;
  uint64_t t[20];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int j = k - i;
      if (j > i && j < 10) acc += (uint64_t)d[i] * a.v[j];
    }
    if ((k & 1) == 0) acc += (uint64_t)a.v[k >> 1] * a.v[k >> 1];
    t[k] = acc;
  }
  t[19] = 0;
  f28_redc(r, t);
}

// r = a + b, limb-wise (no carries)
FGV_DEV void f28_add(f28 &r, const f28 &a, const f28 &b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + b.v[i];
}
// r = a + C - b with C one of the C*P28 constants: a normalized, b normalized with top limb
// <= C's -> loose, value < a + k p
FGV_DEV void f28_sub(f28 &r, const f28 &a, const f28 &b, const uint32_t *C) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + C[i] - b.v[i];
}
// carry pass: limbs < 2^32 -> normalized (same value)
FGV_DEV void f28_norm(f28 &a) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    a.v[i + 1] += a.v[i] >> 28;
    a.v[i] &= F28_MASK;
  }
}
// normalized value < 2p: == 0 mod p
FGV_DEV bool f28_is_zero(const f28 &a) {
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    z |= a.v[i];
    q |= a.v[i] ^ P28[i];
  }
  return z == 0u || q == 0u;
}
