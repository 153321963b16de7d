// p256_modinv.h -- x^-1 mod n (P-256 group order) by Bernstein-Yang divsteps ("safegcd",
// Bernstein & Yang, "Fast constant-time gcd computation and modular inversion", TCHES 2019),
// in the signed 30-bit-limb form: 20 rounds of 30 divsteps (600 >= 590 needed for 256-bit
// inputs), each round a 2x2 transition matrix applied to (f, g) and to (d, e) mod n.
//
// Why: the Fermat chain a^(n-2) is ~300 dependent Montgomery multiplications (~95k VALU
// instructions on one lane's critical path); this is ~15k simple 32-bit ops with short
// dependency chains, so the per-lane latency that bounds k_inv drops ~6x.  Control flow is
// input-independent (fixed trip counts, masks instead of branches): lanes never diverge.
//
// Attribution: the branch-free 30-divstep inner loop (divsteps_30: the c1/c2 masks of a
// "zeta < 0 and g odd" swap-and-negate, then the conditional add and halving) and the signed
// 30-bit limb layout follow libsecp256k1's modinv32 implementation (src/modinv32_impl.h,
// secp256k1_modinv32_divsteps_30; MIT licence, (c) Pieter Wuille, Peter Dettman),
// which restates the paper's algorithm; the rest (P-256 group order constants, the
// matrix-application and normalisation code, the device batching) is ours.
//
// __host__ __device__ so the same code is checked on the host (tools/modinv_check.cpp)
// against an independent big-integer inverse.
//
// libsecp256k1's licence, for the adapted inner loop:
//
//   Copyright (c) 2013 Pieter Wuille
//
//   Permission is hereby granted, free of charge, to any person obtaining a copy
//   of this software and associated documentation files (the "Software"), to deal
//   in the Software without restriction, including without limitation the rights
//   to use, copy, modify, merge, publish, distribute, sublicense, and/or sell
//   copies of the Software, and to permit persons to whom the Software is
//   furnished to do so, subject to the following conditions:
//
//   The above copyright notice and this permission notice shall be included in
//   all copies or substantial portions of the Software.
//
//   THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND, EXPRESS OR
//   IMPLIED, INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY,
//   FITNESS FOR A PARTICULAR PURPOSE AND NONINFRINGEMENT. IN NO EVENT SHALL THE
//   AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR ANY CLAIM, DAMAGES OR OTHER
//   LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR OTHERWISE, ARISING FROM,
//   OUT OF OR IN CONNECTION WITH THE SOFTWARE OR THE USE OR OTHER DEALINGS IN
//   THE SOFTWARE.
#pragma once
#include <stdint.h>

#ifndef FGV_HD
#define FGV_HD __host__ __device__ __forceinline__
#endif

namespace fgv_modinv {

struct s30 {
  int32_t v[9];
};

// n in signed-30 limbs, and n^-1 mod 2^30
#define MI_N0 0x3c632551
#define MI_N1 0x0ee72b0b
#define MI_N2 0x3179e84f
#define MI_N3 0x39beab69
#define MI_N4 0x3fffffbc
#define MI_N5 0x3fffffff
#define MI_N6 0x00000fff
#define MI_N7 0x3fffc000
#define MI_N8 0x0000ffff
#define MI_NINV30 0x11ff43b1u

FGV_HD int32_t mi_nlimb(int i) {
  return i == 0 ? MI_N0 : i == 1 ? MI_N1 : i == 2 ? MI_N2 : i == 3 ? MI_N3 : i == 4 ? MI_N4
       : i == 5 ? MI_N5 : i == 6 ? MI_N6 : i == 7 ? MI_N7 : MI_N8;
}

// 30 divsteps on the low bits of f, g: transition matrix (u v; q r) scaled by 2^30.
FGV_HD int32_t divsteps_30(int32_t zeta, uint32_t f, uint32_t g, int32_t &tu, int32_t &tv, int32_t &tq,
                           int32_t &tr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    uint32_t m1 = (uint32_t)(zeta >> 31);  // zeta < 0
    const uint32_t m2 = 0u - (g & 1u);     // g odd
    const uint32_t x = (f ^ m1) - m1, y = (u ^ m1) - m1, z = (v ^ m1) - m1;
    g += x & m2;
    q += y & m2;
    r += z & m2;
    m1 &= m2;
    zeta = (int32_t)(((uint32_t)zeta ^ m1) - 1u);
    f += g & m1;
    u += q & m1;
    v += r & m1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  tu = (int32_t)u;
  tv = (int32_t)v;
  tq = (int32_t)q;
  tr = (int32_t)r;
  return zeta;
}

// (d, e) <- t * (d, e) / 2^30 mod n (adding multiples of n to clear the low 30 bits)
FGV_HD void update_de_30(s30 &d, s30 &e, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t M30 = (int32_t)(UINT32_MAX >> 2);
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int32_t di = d.v[0], ei = e.v[0];
  int64_t cd = (int64_t)u * di + (int64_t)v * ei;
  int64_t ce = (int64_t)q * di + (int64_t)r * ei;
  md -= (int32_t)((MI_NINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((MI_NINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)MI_N0 * md;
  ce += (int64_t)MI_N0 * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    di = d.v[i];
    ei = e.v[i];
    const int64_t ni = mi_nlimb(i);
    cd += (int64_t)u * di + (int64_t)v * ei + ni * md;
    ce += (int64_t)q * di + (int64_t)r * ei + ni * me;
    d.v[i - 1] = (int32_t)cd & M30;
    cd >>= 30;
    e.v[i - 1] = (int32_t)ce & M30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// (f, g) <- t * (f, g) / 2^30 (exact)
FGV_HD void update_fg_30(s30 &f, s30 &g, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t M30 = (int32_t)(UINT32_MAX >> 2);
  int32_t fi = f.v[0], gi = g.v[0];
  int64_t cf = (int64_t)u * fi + (int64_t)v * gi;
  int64_t cg = (int64_t)q * fi + (int64_t)r * gi;
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    fi = f.v[i];
    gi = g.v[i];
    cf += (int64_t)u * fi + (int64_t)v * gi;
    cg += (int64_t)q * fi + (int64_t)r * gi;
    f.v[i - 1] = (int32_t)cf & M30;
    cf >>= 30;
    g.v[i - 1] = (int32_t)cg & M30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// r in (-2n, n) -> [0, n), negated first when sign < 0
FGV_HD void normalize_30(s30 &r, int32_t sign) {
  const int32_t M30 = (int32_t)(UINT32_MAX >> 2);
  int32_t c = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] += mi_nlimb(i) & c;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = (r.v[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= M30;
  }
  c = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] += mi_nlimb(i) & c;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= M30;
  }
}

// 8 x 32-bit little-endian limbs <-> 9 x 30-bit
FGV_HD void to_s30(s30 &o, const uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 30 * i, li = bit >> 5, sh = bit & 31;
    uint32_t w = a[li] >> sh;
    if (sh > 2 && li < 7) w |= a[li + 1] << (32 - sh);
    o.v[i] = (int32_t)(w & 0x3FFFFFFFu);
  }
}
FGV_HD void from_s30(uint32_t a[8], const s30 &x) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int bit = 32 * i, li = bit / 30, sh = bit % 30;
    uint64_t w = (uint64_t)(uint32_t)x.v[li] >> sh;
    if (li + 1 < 9) w |= (uint64_t)(uint32_t)x.v[li + 1] << (30 - sh);
    if (li + 2 < 9 && 60 - sh < 32) w |= (uint64_t)(uint32_t)x.v[li + 2] << (60 - sh);
    a[i] = (uint32_t)w;
  }
}

// out = x^-1 mod n for 0 < x < n (plain, not Montgomery); x = 0 gives 0
FGV_HD void modinv_n(uint32_t out[8], const uint32_t x[8]) {
  s30 d, e, f, g;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    d.v[i] = 0;
    e.v[i] = 0;
    f.v[i] = mi_nlimb(i);
  }
  e.v[0] = 1;
  to_s30(g, x);
  int32_t zeta = -1;
#pragma unroll 1
  for (int it = 0; it < 20; it++) {
    int32_t u, v, q, r;
    zeta = divsteps_30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], u, v, q, r);
    update_de_30(d, e, u, v, q, r);
    update_fg_30(f, g, u, v, q, r);
  }
  normalize_30(d, f.v[8]);
  from_s30(out, d);
}

}  // namespace fgv_modinv
