// p256_kernels.hip -- ECDSA-P256 batch verification for gfx950.
//
// Per batch, on the context's streams (fgv_host.cpp launch_inv / launch_prep_point):
//   k_keytab  (per NEW comb key, cached across batches) -- fixed-base comb table
//             T_Q[w][k-1] = k * 2^(13w) * Q, 20 windows of 13 bits, k = 1..4096 (signed digits),
//             affine Montgomery-280 (5.2 MB per key, fgv_kernels.h).  The generator comb T_G
//             (12 windows of 22 bits, 1.61 GB) is built once per context by k_gtab.
//   k_keyprep (per NEW key id) -- on-curve check, coordinates for the variable-base kernel.
//   k_inv     (PREP_B items per lane) -- range checks, w = s^-1 mod n with a per-lane
//             batched (Montgomery-trick) inversion; independent of the digests, so it runs
//             concurrently with the SHA-256 jobs of a block batch (second stream).
//   k_prep    (per item) -- u1 = e*w, u2 = r*w; signed recoding into 12 generator digits
//             (22-bit) and 20 key digits (13-bit).
//   k_point28 (L lanes per item, L chosen per batch) -- R = sum_w T_G[w][d1_w] + T_Q[w][d2_w]: 32
//             mixed additions and NO doublings (radix 2^28, incomplete formulas), split over the
//             lanes of a group, then a log2(L)-level butterfly across the group; x_R mod n == r
//             checked projectively.  k_point (exact radix-2^32 arithmetic, complete formulas)
//             finishes the items whose sum hit an exceptional addition.
//   keys without a comb (kmap[id] == KEY_NONE; k_inv lists their items):
//   k_vb_mul  (8 lanes per listed item, beside the hashes: u2 = r * s^-1 needs no digest) --
//             u2 * Q as the sum over 32-bit slices of u2 against the key's slice bases 2^(32 s) Q
//             (k_keyprep): per lane a 1Q..15Q table, 28 doublings and <= 8 additions, then a
//             butterfly across the lanes; exact formulas;
//   k_vb_fin  (after k_prep) -- + u1 * G from the generator comb (12 terms), x_R check.
//
// Semantics restated: Go 1.21.9 crypto/ecdsa verifyNISTEC (SEC 1 v2 s4.1.4) behind
// fabric-lib-go bccsp/sw/ecdsa.go:41-57.  Exceptional additions (P == Q, P == -Q, inf)
// are handled exactly, so results are bit-exact for adversarial inputs as well.
#include "p256_field.h"
#include "p256_fe28.h"
#include "fgv_kernels.h"
#include "p256_modinv.h"

// R^2 mod p (to Montgomery), little-endian limbs
__constant__ static const uint32_t R2P[8] = {0x00000003u, 0x00000000u, 0xFFFFFFFFu, 0xFFFFFFFBu,
                                              0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFDu, 0x00000004u};
// R^2 mod n
__constant__ static const uint32_t R2N[8] = {0xBE79EEA2u, 0x83244C95u, 0x49BD6FA6u, 0x4699799Cu,
                                              0x2B6BEC59u, 0x2845B239u, 0xF3D95620u, 0x66E12D94u};
// R mod n = 2^256 - n
__constant__ static const uint32_t ONEN[8] = {0x039CDAAFu, 0x0C46353Du, 0x58E8617Bu, 0x43190552u,
                                              0x00000000u, 0x00000000u, 0xFFFFFFFFu, 0x00000000u};
// b (curve coefficient), plain little-endian
__constant__ static const uint32_t B_PLAIN[8] = {0x27D2604Bu, 0x3BCE3C3Eu, 0xCC53B0F6u, 0x651D06B0u,
                                                 0x769886BCu, 0xB3EBBD55u, 0xAA3A93E7u, 0x5AC635D8u};

FGV_DEV void fe_load_c(fe &r, const uint32_t *c) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
}
FGV_DEV void fe_to_mont(fe &r, const fe &a) {
  fe r2;
  fe_load_c(r2, R2P);
  fe_mul(r, a, r2);
}
FGV_DEV bool lt_p(const uint32_t a[8]) {
  const uint32_t p[8] = {P_0, P_1, P_2, P_3, P_4, P_5, P_6, P_7};
  return lt_256(a, p);
}
FGV_DEV bool lt_n(const uint32_t a[8]) {
  uint32_t n[8];
#pragma unroll
  for (int i = 0; i < 8; i++) n[i] = N_LIMBS[i];
  return lt_256(a, n);
}
FGV_DEV bool is_zero8(const uint32_t a[8]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a[i];
  return x == 0u;
}

// y^2 == x^3 - 3x + b, coordinates < p (Go nistec pointFromAffine)
FGV_DEV bool on_curve(const fe &x, const fe &y, fe &xm, fe &ym) {
  if (!lt_p(x.v) || !lt_p(y.v)) return false;
  fe_to_mont(xm, x);
  fe_to_mont(ym, y);
  fe lhs, rhs, t, b;
  fe_sqr(lhs, ym);
  fe_sqr(rhs, xm);
  fe_mul(rhs, rhs, xm);
  fe_add(t, xm, xm);
  fe_add(t, t, xm);
  fe_sub(rhs, rhs, t);
  fe_load_c(t, B_PLAIN);
  fe_to_mont(b, t);
  fe_add(rhs, rhs, b);
  return fe_eq(lhs, rhs);
}

FGV_DEV void store_fe(uint32_t *dst, const fe &a) {
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
FGV_DEV void load_fe(fe &a, const uint32_t *src) {
  const uint4 *s = reinterpret_cast<const uint4 *>(src);
  uint4 p = s[0], q = s[1];
  a.v[0] = p.x; a.v[1] = p.y; a.v[2] = p.z; a.v[3] = p.w;
  a.v[4] = q.x; a.v[5] = q.y; a.v[6] = q.z; a.v[7] = q.w;
}

// ---------------------------------------------------------------- k_keytab
// T_Q[w][k-1] = k * 2^(17w) * Q, w < NWIN, k = 1..TAB_K.  KT_THREADS_PER_KEY threads per key, thread
// (w, chunk) builds entries k0..k0+31 of window w: B = 2^(17w) Q by doublings, P = k0 * B by
// double-and-add, then P += B, one Montgomery-trick inversion per chunk (complete formulas:
// pt_add routes P == B to a doubling).  Montgomery-280 form (k_point28; k_point converts an entry
// when it reads it).  key_ok (nullable): the key's on-curve bit at its slot.
// qxy: [nkeys][16] plain little-endian limbs (x then y); scratch: [nkeys][KT_ENTRIES] jpoint_raw.
// k_keybase: the window bases B_w = 2^(17w) Q of each key (one thread per (key, w): 17 w doublings),
// so that k_keytab's 32,768 threads per key start from their base instead of each redoing up to
// 255 doublings (half of a 17-bit table's build).  Off-curve keys: nothing (k_keytab skips them).
__global__ __launch_bounds__(64) void k_keybase(const uint32_t *__restrict__ qxy, uint32_t nkeys,
                                                jpoint_raw *__restrict__ bases) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t kid = t / NWIN, w = t % NWIN;
  if (kid >= nkeys) return;
  fe x, y, xm, ym;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = qxy[kid * 16 + i];
    y.v[i] = qxy[kid * 16 + 8 + i];
  }
  if (!on_curve(x, y, xm, ym)) return;
  jpoint b;
  b.x = xm;
  b.y = ym;
  fe_set_one(b.z);
  for (uint32_t i = 0; i < WBITS * w; i++) pt_dbl(b, b);
  jpoint_raw &o = bases[(size_t)kid * NWIN + w];
  store_fe(o.x, b.x);
  store_fe(o.y, b.y);
  store_fe(o.z, b.z);
}

__global__ __launch_bounds__(64) void k_keytab(const uint32_t *__restrict__ qxy,
                                               const uint32_t *__restrict__ slots,
                                               apoint_raw *__restrict__ tables,
                                               apoint_raw *__restrict__ tables28,
                                               jpoint_raw *__restrict__ scratch,
                                               uint8_t *__restrict__ key_ok, uint32_t nkeys,
                                               const jpoint_raw *__restrict__ bases) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t kid = t / KT_THREADS_PER_KEY, r = t % KT_THREADS_PER_KEY;
  if (kid >= nkeys) return;
  constexpr uint32_t CPW = TAB_K / KT_CHUNK;  // chunks per window
  const uint32_t w = r / CPW, ch = r % CPW;
  const uint32_t k0 = ch * KT_CHUNK + 1;
  fe x, y, xm, ym;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = qxy[kid * 16 + i];
    y.v[i] = qxy[kid * 16 + 8 + i];
  }
  const bool ok = on_curve(x, y, xm, ym);
  const uint32_t slot = slots[kid];
  if (r == 0 && key_ok) key_ok[slot] = ok ? 1 : 0;
  if (!ok) return;
  jpoint b;
  if (bases) {  // (k_keybase)
    const jpoint_raw &o = bases[(size_t)kid * NWIN + w];
    load_fe(b.x, o.x);
    load_fe(b.y, o.y);
    load_fe(b.z, o.z);
  } else {
    b.x = xm;
    b.y = ym;
    fe_set_one(b.z);
    for (uint32_t i = 0; i < WBITS * w; i++) pt_dbl(b, b);
  }
  jpoint pk = b;
  for (int bit = 30 - __builtin_clz(k0 | 1u); bit >= 0; bit--) {
    jpoint t2 = pk;
    pt_dbl(pk, t2);
    if ((k0 >> bit) & 1u) {
      t2 = pk;
      pt_add(pk, t2, b);
    }
  }
  jpoint_raw *scr = scratch + (size_t)kid * KT_ENTRIES + (size_t)w * TAB_K + (k0 - 1);
  const size_t e0 = (size_t)slot * KT_ENTRIES + (size_t)w * TAB_K + (k0 - 1);
  fe pref;
  fe_set_one(pref);
  for (uint32_t j = 0; j < KT_CHUNK; j++) {
    if (j > 0) {
      jpoint t2 = pk;
      pt_add(pk, t2, b);
    }
    fe_mul(pref, pref, pk.z);
    store_fe(scr[j].x, pk.x);
    store_fe(scr[j].y, pk.y);
    store_fe(scr[j].z, pk.z);
    store_fe(scr[j].pref, pref);
  }
  fe inv;
  fe_inv(inv, pref);
  fe c280;
  fe_load_c(c280, C280_32);
  for (int j = KT_CHUNK - 1; j >= 0; j--) {
    fe X, Y, Z, prev, zinv, z2, z3, ax, ay;
    load_fe(X, scr[j].x);
    load_fe(Y, scr[j].y);
    load_fe(Z, scr[j].z);
    if (j > 0) load_fe(prev, scr[j - 1].pref);
    else fe_set_one(prev);
    fe_mul(zinv, inv, prev);  // Z_j^-1 = (Z_0..Z_j)^-1 * (Z_0..Z_{j-1})
    fe_mul(inv, inv, Z);      // (Z_0..Z_{j-1})^-1
    fe_sqr(z2, zinv);
    fe_mul(z3, z2, zinv);
    fe_mul(ax, X, z2);
    fe_mul(ay, Y, z3);
    if (tables) {  // (the exact Montgomery-256 copy: the generator table only)
      store_fe(tables[e0 + j].x, ax);
      store_fe(tables[e0 + j].y, ay);
    }
    // the same point in Montgomery-280 form (k_point28): x * 2^256 -> x * 2^280
    fe_mul(ax, ax, c280);
    fe_mul(ay, ay, c280);
    store_fe(tables28[e0 + j].x, ax);
    store_fe(tables28[e0 + j].y, ay);
  }
}

// ---------------------------------------------------------------- k_gtab
// Generator comb table T_G[w][k-1] = k * 2^(22w) * G, w < NGWIN, k = 1..GT_K (signed digits).
// Thread t builds GT_CHUNK consecutive entries k0..k0+31 of one window: B = 2^(22w) G by
// doublings, P = k0 * B by double-and-add, then P += B, and one Montgomery-trick inversion for
// the chunk's Z's (complete formulas throughout: pt_add routes P == B to a doubling).
// Montgomery-280 form (k_point converts an entry when it reads it).
__constant__ static const uint32_t G_PLAIN[16] = {
    0xD898C296u, 0xF4A13945u, 0x2DEB33A0u, 0x77037D81u, 0x63A440F2u, 0xF8BCE6E5u, 0xE12C4247u, 0x6B17D1F2u,
    0x37BF51F5u, 0xCBB64068u, 0x6B315ECEu, 0x2BCE3357u, 0x7C0F9E16u, 0x8EE7EB4Au, 0xFE1A7F9Bu, 0x4FE342E2u};

__global__ __launch_bounds__(64) void k_gtab(apoint_raw *__restrict__ tables28, jpoint_raw *__restrict__ scratch,
                                             uint32_t w) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // chunk of window w
  if (t >= GT_THREADS_PER_WIN) return;
  const uint32_t k0 = t * GT_CHUNK + 1;
  fe gx, gy;
  fe_load_c(gx, G_PLAIN);
  fe_load_c(gy, G_PLAIN + 8);
  jpoint b;
  fe_to_mont(b.x, gx);
  fe_to_mont(b.y, gy);
  fe_set_one(b.z);
  for (uint32_t i = 0; i < GWBITS * w; i++) pt_dbl(b, b);
  // P = k0 * B, left to right
  jpoint pk = b;
  for (int bit = 30 - __builtin_clz(k0 | 1u); bit >= 0; bit--) {
    jpoint t2 = pk;
    pt_dbl(pk, t2);
    if ((k0 >> bit) & 1u) {
      t2 = pk;
      pt_add(pk, t2, b);
    }
  }
  jpoint_raw *scr = scratch + (size_t)t * GT_CHUNK;
  const size_t e0 = (size_t)w * GT_K + (k0 - 1);
  fe pref;
  fe_set_one(pref);
  for (uint32_t j = 0; j < GT_CHUNK; j++) {
    if (j > 0) {
      jpoint t2 = pk;
      pt_add(pk, t2, b);
    }
    fe_mul(pref, pref, pk.z);
    store_fe(scr[j].x, pk.x);
    store_fe(scr[j].y, pk.y);
    store_fe(scr[j].z, pk.z);
    store_fe(scr[j].pref, pref);
  }
  fe inv;
  fe_inv(inv, pref);
  fe c280;
  fe_load_c(c280, C280_32);
  for (int j = GT_CHUNK - 1; j >= 0; j--) {
    fe X, Y, Z, prev, zinv, z2, z3, ax, ay;
    load_fe(X, scr[j].x);
    load_fe(Y, scr[j].y);
    load_fe(Z, scr[j].z);
    if (j > 0) load_fe(prev, scr[j - 1].pref);
    else fe_set_one(prev);
    fe_mul(zinv, inv, prev);
    fe_mul(inv, inv, Z);
    fe_sqr(z2, zinv);
    fe_mul(z3, z2, zinv);
    fe_mul(ax, X, z2);
    fe_mul(ay, Y, z3);
    fe_mul(ax, ax, c280);  // Montgomery-256 -> Montgomery-280 (k_point28's form)
    fe_mul(ay, ay, c280);
    store_fe(tables28[e0 + j].x, ax);
    store_fe(tables28[e0 + j].y, ay);
  }
}

// ---------------------------------------------------------------- k_inv / k_prep
// Scalar preparation is split so the long part (s^-1, which needs only s) can run
// concurrently with the SHA-256 jobs that produce the digests:
//   k_inv   items in PREP_B strided rounds per lane (item = lane + b * nlanes): range checks
//           (status 4/5), s -> Montgomery, prefix products, ONE inversion per lane by
//           Bernstein-Yang divsteps (p256_modinv.h; ~6x shorter critical path than the Fermat
//           chain), walk back -> w = s^-1 (Montgomery form) [8][n].
//   k_prep  one item per lane: e = digest mod n, u1 = e*w, u2 = r*w, signed recoding into
//           the comb digits [n][DIG_STRIDE] (u2 itself for a key without a comb).
// R^3 mod n: maps the plain inverse of a Montgomery representative back to Montgomery form
// (sn_mul(X^-1, R^3) = (A*R)^-1 * R^2 = A^-1 * R)
__constant__ static const uint32_t R3N[8] = {0x0b65a624u, 0xac8ebec9u, 0x0c0555c9u, 0x111f28aeu,
                                              0x6ba5e93fu, 0x2543b924u, 0x6407be65u, 0x503a54e7u};

__global__ __launch_bounds__(INV_THREADS) void k_inv(uint32_t n, const uint32_t *__restrict__ dn,
                                                     uint8_t *__restrict__ status,
                                                     const uint32_t *__restrict__ key_slot,
                                                     const uint8_t *__restrict__ key_ok,
                                                     const uint32_t *__restrict__ r_limbs,
                                                     const uint32_t *__restrict__ s_limbs,
                                                     uint32_t *__restrict__ w_out,
                                                     uint32_t *__restrict__ w_scratch,
                                                     const uint32_t *__restrict__ kmap,
                                                     uint32_t *__restrict__ vb_list, uint32_t *__restrict__ vb_cnt) {
  // latency-critical: it runs beside the SHA-256 jobs (second stream); win VALU arbitration
  __builtin_amdgcn_s_setprio(3);
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  // lanes in use: the grid, or -- for a device-side count -- just enough lanes for PREP_B items
  // each (the grid is sized for the capacity; the rest exit), so the batch inversion amortises
  const uint32_t cnt = dn ? min(n, *dn) : n;
  const uint32_t nl = dn ? ((cnt + PREP_B - 1) / PREP_B + INV_THREADS - 1) / INV_THREADS * INV_THREADS
                         : gridDim.x * blockDim.x;
  if (lane >= nl) return;
  uint32_t one[8], r2n[8], acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    one[i] = ONEN[i];
    r2n[i] = R2N[i];
    acc[i] = one[i];
  }
  // pass 1: validate, s -> Montgomery, prefix products (kept in w_scratch [b][8][nl])
  uint32_t live = 0;
#pragma unroll 1
  for (int b = 0; b < PREP_B; b++) {
    const uint32_t i = lane + (uint32_t)b * nl;
    uint32_t sm[8];
    bool use = false;
    if (i < cnt && status[i] == ST_PENDING) {
      uint32_t r[8], s[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        r[k] = r_limbs[(size_t)k * n + i];
        s[k] = s_limbs[(size_t)k * n + i];
      }
      if (!key_ok[key_slot[i]]) {
        status[i] = 5;
      } else if (is_zero8(r) || is_zero8(s) || !lt_n(r) || !lt_n(s)) {
        status[i] = 4;
      } else {
        sn_mul(sm, s, r2n);
        use = true;
      }
    }
    if (use) {
      live |= 1u << b;
      sn_mul(acc, acc, sm);
    }
    if (kmap) {  // items of keys without a comb: the variable-base list (one atomic per wave)
      const bool vb = use && kmap[key_slot[i]] == KEY_NONE;
      const uint64_t m = __ballot(vb);
      if (m) {
        const uint32_t ln = __lane_id(), lead = (uint32_t)__builtin_ctzll(m);
        uint32_t b0 = 0;
        if (ln == lead) b0 = atomicAdd(vb_cnt, (uint32_t)__popcll(m));
        b0 = (uint32_t)__shfl((int)b0, (int)lead);
        if (vb) {
          vb_list[b0 + (uint32_t)__popcll(m & ((1ull << ln) - 1ull))] = i;
          status[i] = ST_VB;  // (the path is decided here, once: kmap may change under a batch)
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) w_scratch[((size_t)b * 8 + k) * nl + lane] = acc[k];
  }
  if (live == 0) return;
  uint32_t inv[8], r3n[8];
  fgv_modinv::modinv_n(inv, acc);  // plain inverse of the Montgomery representative
#pragma unroll
  for (int i = 0; i < 8; i++) r3n[i] = R3N[i];
  sn_mul(inv, inv, r3n);  // (prod s_m)^-1 in Montgomery form
  // pass 2: walk back, w_b = inv * prefix_{b-1}; inv *= s_m[b]
#pragma unroll 1
  for (int b = PREP_B - 1; b >= 0; b--) {
    if (!((live >> b) & 1u)) continue;
    const uint32_t i = lane + (uint32_t)b * nl;
    uint32_t prev[8], w[8], s[8], sm[8];
    if (b > 0) {
#pragma unroll
      for (int k = 0; k < 8; k++) prev[k] = w_scratch[((size_t)(b - 1) * 8 + k) * nl + lane];
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) prev[k] = one[k];
    }
    sn_mul(w, inv, prev);  // s^-1 * R (Montgomery)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      s[k] = s_limbs[(size_t)k * n + i];
      w_out[(size_t)k * n + i] = w[k];
    }
    sn_mul(sm, s, r2n);
    sn_mul(inv, inv, sm);
  }
}

// in:  status, r limbs, w = s^-1 (Montgomery) from k_inv, digests [*][32] big-endian, item i
//      using digest dig_idx[i] (or i when dig_idx is null).
// out: digits [n][DIG_STRIDE]: u1 digits (int32 x NGWIN) at 0, u2 digits (int16 x NWIN) at DIG_Q_OFF
//      (items of keys without a comb use the generator digits only: k_vb_fin).
__global__ __launch_bounds__(256) void k_prep(uint32_t n, const uint32_t *__restrict__ dn,
                                              const uint8_t *__restrict__ status,
                                              const uint32_t *__restrict__ r_limbs,
                                              const uint32_t *__restrict__ w_in,
                                              const uint8_t *__restrict__ digests,
                                              const uint32_t *__restrict__ dig_idx,
                                              int8_t *__restrict__ digits, uint32_t *__restrict__ redo) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && redo) {  // k_point28's hand-over count (read by k_point) + both kernels' work counters
    redo[0] = 0u;
    redo[1] = 0u;
    redo[2] = 0u;
  }
  if (i >= (dn ? min(n, *dn) : n) || (status[i] != ST_PENDING && status[i] != ST_VB)) return;
  uint32_t w[8], r[8], e[8], u1[8], u2[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    w[k] = w_in[(size_t)k * n + i];
    r[k] = r_limbs[(size_t)k * n + i];
  }
  // e = leftmost 256 bits of the digest, mod n (digest is exactly 32 bytes)
  const uint32_t di = dig_idx ? dig_idx[i] : i;
  const uint32_t *dg = reinterpret_cast<const uint32_t *>(digests + (size_t)di * 32);
#pragma unroll
  for (int k = 0; k < 8; k++) e[k] = __builtin_bswap32(dg[7 - k]);
  if (!lt_n(e)) {
    uint32_t bo = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) e[k] = subb(e[k], N_LIMBS[k], bo, &bo);
  }
  sn_mul(u1, e, w);  // e * s^-1 (plain)
  sn_mul(u2, r, w);  // r * s^-1 (plain)
  // signed recoding, digits in [-2^(W-1), 2^(W-1) - 1]: u1 in base 2^22 (12 int32 digits,
  // generator comb), u2 in base 2^17 (16 int32 digits); the top window of a scalar < 2^256
  // (bits 242.. / 255..) is far below half its range, so the final carry never leaves it
  int8_t *dp = digits + (size_t)i * DIG_STRIDE;
  {
    constexpr int GMASK = (1 << GWBITS) - 1, GHALF = 1 << (GWBITS - 1);
    int32_t *g = reinterpret_cast<int32_t *>(dp);
    int c1 = 0;
#pragma unroll
    for (int win = 0; win < NGWIN; win++) {
      const int bit = GWBITS * win, li = bit >> 5, sh = bit & 31;
      uint32_t v1 = li < 8 ? u1[li] >> sh : 0u;
      if (sh > 32 - GWBITS && li < 7) v1 |= u1[li + 1] << (32 - sh);
      int a1 = (int)(v1 & GMASK) + c1;
      c1 = a1 >= GHALF;
      a1 -= c1 << GWBITS;
      g[win] = a1;
    }
  }
  constexpr int WMASK = (1 << WBITS) - 1, WHALF = 1 << (WBITS - 1);
  int c2 = 0;
  int32_t *q = reinterpret_cast<int32_t *>(dp + DIG_Q_OFF);
#pragma unroll
  for (int win = 0; win < NWIN; win++) {
    const int bit = WBITS * win, li = bit >> 5, sh = bit & 31;
    uint32_t v2 = li < 8 ? u2[li] >> sh : 0u;
    if (sh > 32 - WBITS && li < 7) v2 |= u2[li + 1] << (32 - sh);
    int a2 = (int)(v2 & WMASK) + c2;
    c2 = a2 >= WHALF;
    a2 -= c2 << WBITS;
    q[win] = a2;
  }
}

// ---------------------------------------------------------------- k_point
// The exact fallback of k_point28: the same comb terms with complete formulas in radix-2^32
// Montgomery arithmetic; T_G and T_Q entries gathered from HBM (64 B per term).

FGV_DEV void shfl_fe(fe &r, const fe &a, int src_lane) {
#pragma unroll
  for (int k = 0; k < 8; k++) r.v[k] = (uint32_t)__shfl((int)a.v[k], src_lane);
}

// L lanes per item (1..8, any value): a wave holds floor(64/L) groups (the remaining lanes
// idle); lane `sub` of a group sums windows sub, sub+L, ...; then a binary tree over the
// group's lanes (level m: lane sub takes lane sub^m's sum when that lane exists), leaving the
// total in lane 0.  Persistent grid: one workgroup per CU, groups stride over the items.
// Work distribution (k_point and k_point28): a wave takes chunks of gpw items (one per lane
// group) from a device counter until they run out, so waves that start late -- a workgroup
// placed only once another kernel's waves left the CU -- or run beside other kernels' waves
// simply take fewer chunks.  counter == nullptr: static grid stride (no work-counter word).
FGV_DEV bool next_chunk(uint32_t *counter, uint32_t &chunk, uint32_t waves, uint32_t gpw, uint32_t n) {
  if (counter) {
    uint32_t c = 0;
    if ((threadIdx.x & 63u) == 0u) c = atomicAdd(counter, 1u);
    chunk = __builtin_amdgcn_readfirstlane(c);
  } else {
    chunk += waves;
  }
  return (uint64_t)chunk * gpw < n;
}

__global__ __launch_bounds__(POINT_THREADS, 2) void k_point(
    uint32_t n, const uint32_t *__restrict__ dn, uint32_t L, uint8_t *__restrict__ status, const uint32_t *__restrict__ key_slot,
    const apoint_raw *__restrict__ gtab, const apoint_raw *__restrict__ ktab,
    const int8_t *__restrict__ digits, const uint32_t *__restrict__ r_limbs, uint32_t *__restrict__ redo,
    const uint32_t *__restrict__ kmap) {
  // after k_point28: only the items it left pending (exceptional additions) remain
  if (redo && *redo == 0u) return;
  __builtin_amdgcn_s_setprio(3);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t gpw = 64u / L;  // groups per wave
  const uint32_t g = lane / L, sub = lane % L;
  if (g >= gpw) return;  // idle tail lanes of the wave (no barrier follows; lane 0 stays)
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  const uint32_t base = lane - sub;  // lane of sub 0 in this group
  uint32_t *ctr = redo ? redo + 2 : nullptr;
  uint32_t chunk = blockIdx.x * (blockDim.x >> 6) + wave - waves;
  // every lane of a group runs the same iterations (item-uniform control flow), so the
  // cross-lane reads below always find their partners active
  const uint32_t cnt = dn ? min(n, *dn) : n;  // items (n: the column stride of r_limbs)
  while (next_chunk(ctr, chunk, waves, gpw, cnt)) {
    const uint32_t i = chunk * gpw + g;
    if (i >= cnt || status[i] != ST_PENDING) continue;
    const uint32_t cs = kmap[key_slot[i]];  // the key id's comb slot
    if (cs == KEY_NONE) continue;  // (k_point_vb's item)
    const apoint_raw *qt = ktab + (size_t)cs * KT_ENTRIES;
    const int8_t *dg = digits + (size_t)i * DIG_STRIDE;
    jpoint acc;
    fe_set_zero(acc.x);
    fe_set_zero(acc.y);
    fe_set_zero(acc.z);
    // comb terms tt = sub + t*L: tt < NGWIN generator window tt, else key window tt - NGWIN
    // (one madd call site)
    const int nterms = (NTERMS - (int)sub + (int)L - 1) / (int)L;
#pragma unroll 1
    for (int t = 0; t < nterms; t++) {
      const int tt = (int)sub + t * (int)L;
      const bool isq = tt >= NGWIN;
      const int d = isq ? reinterpret_cast<const int32_t *>(dg + DIG_Q_OFF)[tt - NGWIN]
                        : reinterpret_cast<const int32_t *>(dg)[tt];
      if (d == 0) continue;
      const int k = (d < 0 ? -d : d) - 1;
      apoint p;
      const apoint_raw *e = isq ? qt + (size_t)(tt - NGWIN) * TAB_K + k : gtab + (size_t)tt * GT_K + k;
      load_fe(p.x, e->x);
      load_fe(p.y, e->y);
      {  // the combs are held in Montgomery-280 form: x 2^280 * 2^232 / 2^256 = x 2^256
        fe c232;
        fe_load_c(c232, C232_32);
        fe_mul(p.x, p.x, c232);
        fe_mul(p.y, p.y, c232);
      }
      if (d < 0) fe_neg(p.y, p.y);
      pt_madd(acc, acc, p);
    }
    // tree: at level m lane sub adds lane (sub ^ m)'s partial sum when that lane exists;
    // lane 0 ends with the sum over all L lanes
#pragma unroll 1
    for (uint32_t m = 1; m < L; m <<= 1) {
      const uint32_t peer = sub ^ m;
      const int src = (int)(base + (peer < L ? peer : sub));
      jpoint o;
      shfl_fe(o.x, acc.x, src);
      shfl_fe(o.y, acc.y, src);
      shfl_fe(o.z, acc.z, src);
      if (peer < L) pt_add_inl(acc, acc, o);
    }
    if (sub != 0) continue;
    uint8_t st = 1;
    if (!fe_is_zero(acc.z)) {
      fe r, rm, z2, lhs;
#pragma unroll
      for (int k = 0; k < 8; k++) r.v[k] = r_limbs[(size_t)k * n + i];
      fe_sqr(z2, acc.z);
      fe_to_mont(rm, r);
      fe_mul(lhs, rm, z2);
      if (fe_eq(lhs, acc.x)) {
        st = 0;
      } else {
        // x_R in [n, p): x_R mod n == r  <=>  x_R == r + n  (only if r + n < p)
        uint32_t c = 0;
        fe rn;
#pragma unroll
        for (int k = 0; k < 8; k++) rn.v[k] = addc(r.v[k], N_LIMBS[k], c, &c);
        if (c == 0u && lt_p(rn.v)) {
          fe_to_mont(rm, rn);
          fe_mul(lhs, rm, z2);
          if (fe_eq(lhs, acc.x)) st = 0;
        }
      }
    }
    status[i] = st;
  }
}

// ---------------------------------------------------------------- k_point28 (fast path)
// Same comb and lane split as k_point, in radix-2^28 Montgomery-280 arithmetic
// (p256_fe28.h) with INCOMPLETE addition formulas: no per-addition exceptional-case tests.
// An exceptional addition (H == 0 mod p: P == +-Q, including a partial sum passing through
// infinity) makes that addition's Z3 = Z1*H == 0, and every later Z stays 0 (Z3 = Z1*H,
// Z3 = Z1*Z2*H).  So a final Z != 0 proves no exceptional case occurred and the result is
// exact; a final Z == 0 leaves the item ST_PENDING and counts it in *redo, and k_point (the
// complete formulas) finishes exactly those items.  Honest inputs never hit it; adversarial
// ones (Q = +-G, u1 = +-u2 ...) do, and stay bit-exact through the exact kernel.
//
// Value bounds (multiples of p) of the lazy representation, per coordinate of the running
// sum: X < 10p, Y < 2p, Z < 2p, all normalized; the constants of each f28_sub are chosen so
// the subtrahend's top limb stays below the constant's (p256_fe28.h).
struct jp28 {
  f28 x, y, z;
};

// acc += (x2, y2): madd-2004-hmv, 8M + 3S
FGV_DEV void madd28(jp28 &a, const f28 &x2, const f28 &y2) {
  f28 z1z1, u2, t, s2, h, r, hh, hhh, v, x3, y3;
  f28_sqr(z1z1, a.z);
  f28_mul(u2, x2, z1z1);
  f28_mul(t, a.z, z1z1);
  f28_mul(s2, y2, t);
  f28_sub(h, u2, a.x, C16P28);  // < 18p
  f28_sub(r, s2, a.y, C8P28);   // < 10p
  f28_sqr(hh, h);
  f28_mul(hhh, h, hh);
  f28_mul(v, a.x, hh);
  f28_add(t, hhh, v);
  f28_add(t, t, v);
  f28_norm(t);                  // < 6p
  f28_sqr(x3, r);
  f28_sub(x3, x3, t, C8P28);
  f28_norm(x3);                 // < 10p
  f28_sub(t, v, x3, C16P28);    // < 18p
  // y3 = r (v - x3) + (8p - y1) hhh: both products in one column sum, one reduction
  f28 ny;
#pragma unroll
  for (int j = 0; j < 10; j++) ny.v[j] = C8P28[j] - a.y.v[j];  // < 8p, loose
  f28_mul2(y3, r, t, ny, hhh);  // < 2p
  f28_mul(a.z, a.z, h);
  a.x = x3;
  a.y = y3;
}

// a += b (both running sums, not infinity), add-2007-bl shape without the exceptional tests
FGV_DEV void add28(jp28 &a, const jp28 &b) {
  f28 z1z1, z2z2, u1, u2, s1, s2, t, h, r, hh, hhh, v, x3, y3;
  f28_sqr(z1z1, a.z);
  f28_sqr(z2z2, b.z);
  f28_mul(u1, a.x, z2z2);
  f28_mul(u2, b.x, z1z1);
  f28_mul(t, b.z, z2z2);
  f28_mul(s1, a.y, t);
  f28_mul(t, a.z, z1z1);
  f28_mul(s2, b.y, t);
  f28_sub(h, u2, u1, C4P28);
  f28_sub(r, s2, s1, C4P28);
  f28_sqr(hh, h);
  f28_mul(hhh, h, hh);
  f28_mul(v, u1, hh);
  f28_add(t, hhh, v);
  f28_add(t, t, v);
  f28_norm(t);
  f28_sqr(x3, r);
  f28_sub(x3, x3, t, C8P28);
  f28_norm(x3);
  f28_sub(t, v, x3, C16P28);
  f28 ns1;
#pragma unroll
  for (int j = 0; j < 10; j++) ns1.v[j] = C4P28[j] - s1.v[j];  // s1 < 2p: 4p - s1, loose
  f28_mul2(y3, r, t, ns1, hhh);
  f28_mul(t, a.z, b.z);
  f28_mul(a.z, t, h);
  a.x = x3;
  a.y = y3;
}

FGV_DEV void shfl_f28(f28 &r, const f28 &a, int src_lane) {
#pragma unroll
  for (int k = 0; k < 10; k++) r.v[k] = (uint32_t)__shfl((int)a.v[k], src_lane);
}
// plain 8 x 32-bit value < p -> Montgomery-280, normalized (< 2p)
FGV_DEV void f28_to_mont(f28 &r, const uint32_t w[8]) {
  f28 a, r2;
  f28_from32(a, w);
  f28_load_c(r2, R2P28);
  f28_mul(r, a, r2);
}

__global__ __launch_bounds__(POINT_THREADS, 2) void k_point28(
    uint32_t n, const uint32_t *__restrict__ dn, uint32_t L, uint8_t *__restrict__ status, const uint32_t *__restrict__ key_slot,
    const apoint_raw *__restrict__ gtab28, const apoint_raw *__restrict__ ktab28,
    const int8_t *__restrict__ digits, const uint32_t *__restrict__ r_limbs, uint32_t *__restrict__ redo,
    const uint32_t *__restrict__ kmap) {
  __builtin_amdgcn_s_setprio(3);  // the verify chain; a next batch's front half may run beside it
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gpw = 64u / L;
  const uint32_t g = lane / L, sub = lane % L;
  if (g >= gpw) return;
  const uint32_t waves = gridDim.x * (blockDim.x >> 6);
  const uint32_t base = lane - sub;
  uint32_t chunk = 0;
  const uint32_t cnt = dn ? min(n, *dn) : n;  // items (n: the column stride of r_limbs)
  while (next_chunk(redo + 1, chunk, waves, gpw, cnt)) {
    const uint32_t i = chunk * gpw + g;
    if (i >= cnt || status[i] != ST_PENDING) continue;
    const uint32_t cs = kmap[key_slot[i]];  // the key id's comb slot
    if (cs == KEY_NONE) continue;  // (k_point_vb's item)
    const apoint_raw *qt = ktab28 + (size_t)cs * KT_ENTRIES;
    const int8_t *dg = digits + (size_t)i * DIG_STRIDE;
    jp28 acc;
    bool inf = true;
    const int nterms = (NTERMS - (int)sub + (int)L - 1) / (int)L;
    // the table entry of term t+1 is loaded while term t is added (one gather in flight);
    // comb term tt = sub + t*L: generator window tt (tt < NGWIN), else key window tt - NGWIN
    auto entry = [&](int t, int &d) -> const uint4 * {
      const int tt = (int)sub + t * (int)L;
      const bool isq = tt >= NGWIN;
      d = isq ? reinterpret_cast<const int32_t *>(dg + DIG_Q_OFF)[tt - NGWIN] : reinterpret_cast<const int32_t *>(dg)[tt];
      const int k = d == 0 ? 0 : (d < 0 ? -d : d) - 1;
      return reinterpret_cast<const uint4 *>(isq ? qt + (size_t)(tt - NGWIN) * TAB_K + k : gtab28 + (size_t)tt * GT_K + k);
    };
    int dn;
    const uint4 *pn = entry(0, dn);
    uint4 n0 = pn[0], n1 = pn[1], n2 = pn[2], n3 = pn[3];
#pragma unroll 1
    for (int t = 0; t < nterms; t++) {
      const int d = dn;
      const uint32_t wx[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
      const uint32_t wy[8] = {n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
      if (t + 1 < nterms) {
        pn = entry(t + 1, dn);
        n0 = pn[0];
        n1 = pn[1];
        n2 = pn[2];
        n3 = pn[3];
      }
      if (d == 0) continue;
      f28 px, py;
      f28_from32(px, wx);
      f28_from32(py, wy);
      if (d < 0) {
        f28 z;
#pragma unroll
        for (int j = 0; j < 10; j++) z.v[j] = 0u;
        f28_sub(py, z, py, C4P28);
        f28_norm(py);
      }
      if (inf) {
        acc.x = px;
        acc.y = py;
        f28_load_c(acc.z, ONE28);
        inf = false;
      } else {
        madd28(acc, px, py);
      }
    }
#pragma unroll 1
    for (uint32_t m = 1; m < L; m <<= 1) {
      const uint32_t peer = sub ^ m;
      const int src = (int)(base + (peer < L ? peer : sub));
      jp28 o;
      shfl_f28(o.x, acc.x, src);
      shfl_f28(o.y, acc.y, src);
      shfl_f28(o.z, acc.z, src);
      const bool oinf = __shfl((int)inf, src) != 0;
      if (peer < L && !oinf) {
        if (inf) {
          acc = o;
          inf = false;
        } else {
          add28(acc, o);
        }
      }
    }
    if (sub != 0) continue;
    uint8_t st = 1;
    if (inf) {
      st = 1;  // R = infinity (only u1 = u2 = 0 -> unreachable: r != 0), invalid
    } else if (f28_is_zero(acc.z)) {
      // an exceptional addition (or a true infinity): the complete kernel decides
      atomicAdd(redo, 1u);
      continue;
    } else {
      uint32_t r[8];
#pragma unroll
      for (int k = 0; k < 8; k++) r[k] = r_limbs[(size_t)k * n + i];
      f28 z2, rm, lhs, d, one;
      f28_sqr(z2, acc.z);
      f28_load_c(one, ONE28);
      f28_to_mont(rm, r);
      f28_mul(lhs, rm, z2);
      f28_sub(d, acc.x, lhs, C4P28);
      f28_mul(d, d, one);
      if (f28_is_zero(d)) {
        st = 0;
      } else {
        // x_R in [n, p): x_R mod n == r  <=>  x_R == r + n  (only if r + n < p)
        uint32_t c = 0, rn[8];
#pragma unroll
        for (int k = 0; k < 8; k++) rn[k] = addc(r[k], N_LIMBS[k], c, &c);
        if (c == 0u && lt_p(rn)) {
          f28_to_mont(rm, rn);
          f28_mul(lhs, rm, z2);
          f28_sub(d, acc.x, lhs, C4P28);
          f28_mul(d, d, one);
          if (f28_is_zero(d)) st = 0;
        }
      }
    }
    status[i] = st;
  }
}

// ---------------------------------------------------------------- keys without a comb
// k_keyprep: new key ids -> on-curve bit (k_inv reports 5 for a key off the curve, before the
// range checks, as ecdsa.Verify does) and the variable-base kernel's per-key table
// vbt[id][w][d-1] = d * W_w, W_w = 2^(4 w) * Q, w < VB_WINS, d = 1..VB_TAB (affine, Montgomery-280
// form as the comb tables, 60 KB per key: one base per 4-bit window of the scalar, so the verify's
// u2 * Q is a sum of table entries).  One thread per (key, window): 4 w doublings to W_w, 14
// complete additions, one inversion for the window's 15 Z's (prefix products).  qxy: [nkeys][16]
// plain little-endian limbs (x then y).
__global__ __launch_bounds__(64) void k_keyprep(const uint32_t *__restrict__ qxy, const uint32_t *__restrict__ ids,
                                                uint32_t nkeys, uint32_t *__restrict__ vbt,
                                                uint8_t *__restrict__ key_ok) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k = t / VB_WINS, sl = t % VB_WINS;
  if (k >= nkeys) return;
  fe x, y, xm, ym;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = qxy[k * 16 + i];
    y.v[i] = qxy[k * 16 + 8 + i];
  }
  const bool ok = on_curve(x, y, xm, ym);
  const uint32_t id = ids[k];
  if (sl == 0) key_ok[id] = ok ? 1 : 0;
  uint32_t *o = vbt + (size_t)id * VBT_WORDS + sl * (VB_TAB * 16);
  if (!ok) {  // (never read: k_inv fails the key's items first)
    fe z;
    fe_set_zero(z);
    for (int d = 0; d < VB_TAB; d++) store_fe(o + 16 * d, z), store_fe(o + 16 * d + 8, z);
    return;
  }
  jpoint q;  // W_w (never infinity: 2^(4 w) < n)
  q.x = xm;
  q.y = ym;
  fe_set_one(q.z);
#pragma unroll 1
  for (uint32_t d = 0; d < 4 * sl; d++) {
    jpoint t2 = q;
    pt_dbl(q, t2);
  }
  jpoint T[VB_TAB];  // d * W_w (d * 2^(4 w) < n: never infinity)
  fe pref[VB_TAB];
  T[0] = q;
  pref[0] = q.z;
  for (int d = 1; d < VB_TAB; d++) {
    pt_add_inl(T[d], T[d - 1], q);  // (d = 1: T[0] == q, routed to the doubling)
    fe_mul(pref[d], pref[d - 1], T[d].z);
  }
  fe inv;
  fe_inv(inv, pref[VB_TAB - 1]);
  for (int d = VB_TAB - 1; d >= 0; d--) {
    fe zinv, z2, z3, ax, ay;
    if (d > 0) {
      fe_mul(zinv, inv, pref[d - 1]);  // Z_d^-1
      fe_mul(inv, inv, T[d].z);
    } else {
      zinv = inv;
    }
    fe_sqr(z2, zinv);
    fe_mul(z3, z2, zinv);
    fe_mul(ax, T[d].x, z2);
    fe_mul(ay, T[d].y, z3);
    fe c280;  // (stored in the Montgomery-280 form k_vb_mul28 reads, like the comb tables)
    fe_load_c(c280, C280_32);
    fe_mul(ax, ax, c280);
    fe_mul(ay, ay, c280);
    store_fe(o + 16 * d, ax);
    store_fe(o + 16 * d + 8, ay);
  }
}
// ids whose comb tables k_keytab has just built (stream order) now take the comb path
__global__ __launch_bounds__(64) void k_kmap_set(const uint32_t *__restrict__ ids, const uint32_t *__restrict__ slots,
                                                 uint32_t n, uint32_t *__restrict__ kmap) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) kmap[ids[k]] = slots[k];
}

// `per` items per wave, taken per atomic from `take`; every lane of the wave runs the same
// number of rounds (the count is read once).  j = the wave's first item of the round.
FGV_DEV bool vb_next(uint32_t *take, uint32_t cnt, uint32_t per, uint32_t &j) {
  uint32_t b = 0;
  if (__lane_id() == 0) b = atomicAdd(take, per);
  b = __builtin_amdgcn_readfirstlane(b);
  j = b;
  return b < cnt;
}
FGV_DEV void store_jp(uint32_t *d, const jpoint &p) {
  store_fe(d, p.x);
  store_fe(d + 8, p.y);
  store_fe(d + 16, p.z);
}
FGV_DEV void load_jp(jpoint &p, const uint32_t *s) {
  load_fe(p.x, s);
  load_fe(p.y, s + 8);
  load_fe(p.z, s + 16);
}

// k_vb_mul: acc[j] = u2 * Q for list entry j (item i = list[j], key id key_slot[i]), u2 = r * s^-1
// (plain; k_inv's w is s^-1 in Montgomery form) -- needs no digest, so it runs beside the hashes.
// VB_LANES lanes per item: lane s takes the 32 bits u2[s] of the scalar -- windows 8 s .. 8 s + 7
// -- against the key's window tables d * 2^(4 w) Q (k_keyprep, affine), so u2 * Q = sum_w
// digit_w * 2^(4 w) Q:
//   <= 8 mixed additions, no doublings (each next entry loaded during the addition);
//   a 3-level butterfly of complete additions across the 8 lanes (cross-lane shuffles).
// Complete formulas throughout (pt_madd / pt_add_inl): exact for every input.  uses[id] counts the key's variable-base verifies;
// the one that reaches `promote` queues the id (promo[0] count, ids from promo[2]) for a comb build
// by the host; promo[1] = the batch's variable-base items.
// remap (the exact hand-over of k_vb_mul28): ctr[RD_VB_CNT] counts the remap entries, each the
// list index of an item k_vb_mul28 could not finish; no use counting then (uses == nullptr)
FGV_DEV void vb_mul_body(uint32_t n, const uint32_t *__restrict__ key_slot, const uint32_t *__restrict__ vbt,
                         const uint32_t *__restrict__ r_limbs, const uint32_t *__restrict__ w_in,
                         const uint32_t *__restrict__ ctr, uint32_t *__restrict__ take,
                         const uint32_t *__restrict__ list, uint32_t *__restrict__ acc, uint32_t *__restrict__ uses,
                         uint32_t promote, uint32_t *__restrict__ promo, const uint32_t *__restrict__ remap) {
  __builtin_amdgcn_s_setprio(2);
  const uint32_t cnt = ctr[RD_VB_CNT];
  if (!remap && blockIdx.x == 0 && threadIdx.x == 0) atomicExch(&promo[1], cnt);  // (statistics: fgv_key_stats)
  if (cnt == 0) return;
  const uint32_t lane = __lane_id(), sl = lane % VB_LANES, base = lane - sl;
  constexpr uint32_t PER = 64u / VB_LANES;  // items per wave and round
  fe c232;  // (the table is Montgomery-280: x 2^280 * 2^232 / 2^256 = x 2^256)
  fe_load_c(c232, C232_32);
  uint32_t j0;
  while (vb_next(take, cnt, PER, j0)) {
    const uint32_t jr = j0 + lane / VB_LANES;
    if (jr >= cnt) continue;  // (uniform within the lane group: its partners skip too)
    const uint32_t j = remap ? remap[jr] : jr;
    const uint32_t i = list[j];
    const uint32_t id = key_slot[i];
    uint32_t r[8], w[8], u2[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      r[k] = r_limbs[(size_t)k * n + i];
      w[k] = w_in[(size_t)k * n + i];
    }
    sn_mul(u2, r, w);
    uint32_t dg = u2[0];  // this lane's 32 bits: u2[sl] (a select chain: no private array)
#pragma unroll
    for (int k = 1; k < 8; k++) dg = sl == (uint32_t)k ? u2[k] : dg;
    // window w = 8 sl + k of this lane: table rows (8 sl + k), digit (dg >> 4 k) & 15
    const uint32_t *qt = vbt + (size_t)id * VBT_WORDS + (8 * sl) * (VB_TAB * 16);
    jpoint a;
    fe_set_zero(a.x);
    fe_set_zero(a.y);
    fe_set_zero(a.z);
#pragma unroll 1
    for (int k = 0; k < 8; k++) {
      const uint32_t d = (dg >> (4 * k)) & 15u;
      if (!d) continue;
      const uint32_t *row = qt + k * (VB_TAB * 16) + 16 * (d - 1);
      apoint e;
      load_fe(e.x, row);
      load_fe(e.y, row + 8);
      fe_mul(e.x, e.x, c232);
      fe_mul(e.y, e.y, c232);
      jpoint t2 = a;
      pt_madd(a, t2, e);  // (a = infinity: e itself)
    }
    // butterfly: at level m lane s adds lane s ^ m's partial sum; lane 0 of the group ends with all
#pragma unroll 1
    for (uint32_t m = 1; m < VB_LANES; m <<= 1) {
      jpoint o;
      const int src = (int)(base + (sl ^ m));
#pragma unroll
      for (int k = 0; k < 8; k++) {
        o.x.v[k] = (uint32_t)__shfl((int)a.x.v[k], src);
        o.y.v[k] = (uint32_t)__shfl((int)a.y.v[k], src);
        o.z.v[k] = (uint32_t)__shfl((int)a.z.v[k], src);
      }
      jpoint t2 = a;
      pt_add_inl(a, t2, o);
    }
    if (sl != 0) continue;
    store_jp(acc + (size_t)j * VB_ACC_WORDS, a);
    if (!uses) continue;
    const uint32_t u = atomicAdd(&uses[id], 1u);
    if (u + 1u == promote) {
      const uint32_t s = atomicAdd(&promo[0], 1u);
      if (s < VB_PROMO_CAP) atomicExch(&promo[2 + s], id);
    }
  }
}

#define VB_MUL_ARGS                                                                                               \
  uint32_t n, const uint32_t *__restrict__ key_slot, const uint32_t *__restrict__ vbt,                            \
      const uint32_t *__restrict__ r_limbs, const uint32_t *__restrict__ w_in, const uint32_t *__restrict__ ctr, \
      uint32_t *__restrict__ take, const uint32_t *__restrict__ list, uint32_t *__restrict__ acc,                 \
      uint32_t *__restrict__ uses, uint32_t promote, uint32_t *__restrict__ promo, const uint32_t *__restrict__ remap
__global__ __launch_bounds__(VB_THREADS) void k_vb_mul(VB_MUL_ARGS) {
  vb_mul_body(n, key_slot, vbt, r_limbs, w_in, ctr, take, list, acc, uses, promote, promo, remap);
}
// the same held to 128 VGPRs (4 waves per SIMD, a few more spills): FGV_VB_WGS=4 (A/B)
__global__ __launch_bounds__(VB_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_vb_mul_o4(VB_MUL_ARGS) {
  vb_mul_body(n, key_slot, vbt, r_limbs, w_in, ctr, take, list, acc, uses, promote, promo, remap);
}

// ---------------------------------------------------------------- k_vb_mul28 (fast path)
// The variable-base product u2 * Q in radix-2^28 Montgomery-280 arithmetic (p256_fe28.h), the
// structure of vb_mul_body: LANES (8 or 16) lanes per item, lane s sums its 8 (4) windows of 4
// bits of u2 against the key's window tables d * 2^(4 w) Q -- <= 8 (4) mixed additions and no
// doublings (round 6: the 28 (12) doublings per lane of the 15 KB slice tables were ~70 % of the
// kernel's multiplications) -- then a 3- (4-) level butterfly.  16 lanes halve the serial chain of
// a lane (small batches: latency).  Incomplete formulas, as k_point28: an exceptional addition (a partial sum
// equal to +-the added point) leaves Z = 0, which stays 0; such an item goes to the hand-over list
// (redo[RD_VB2_CNT], its list index in `hand`) and the exact k_vb_mul finishes it.  The result is
// converted to the Montgomery-256 Jacobian form k_vb_fin reads.
// 2^256 mod p (radix 2^28): Montgomery-280 -> -256
__constant__ static const uint32_t C256_28[10] = {0x1u, 0x0u, 0x0u, 0xffff000u, 0xfffffffu,
                                                  0xfffffffu, 0xeffffffu, 0xfffffffu, 0x0u, 0x0u};

// normalized value < 2p -> canonical (< p), packed into 8 x 32-bit limbs
FGV_DEV void f28_to32(uint32_t w[8], const f28 &a) {
  f28 r;
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {  // r = a - p (with borrow)
    const int32_t d = (int32_t)a.v[i] - (int32_t)P28[i] + br;
    br = d >> 28;  // (arithmetic: -1 on borrow)
    r.v[i] = (uint32_t)d & F28_MASK;
  }
  const bool ge = br >= 0;  // a >= p: take a - p
  uint32_t v[10];
#pragma unroll
  for (int i = 0; i < 10; i++) v[i] = ge ? r.v[i] : a.v[i];
  // 10 x 28 bits -> 8 x 32 bits
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int bit = 32 * k, li = bit / 28, sh = bit % 28;
    uint32_t x = v[li] >> sh;
    if (li + 1 < 10) x |= v[li + 1] << (28 - sh);
    if (sh > 24 && li + 2 < 10) x |= v[li + 2] << (56 - sh);
    w[k] = x;
  }
}

template <uint32_t LANES>
FGV_DEV void vb_mul28_body(uint32_t n, const uint32_t *__restrict__ key_slot,
                                                          const uint32_t *__restrict__ vbt,
                                                          const uint32_t *__restrict__ r_limbs,
                                                          const uint32_t *__restrict__ w_in,
                                                          uint32_t *__restrict__ ctr, const uint32_t *__restrict__ list,
                                                          uint32_t *__restrict__ acc, uint32_t *__restrict__ uses,
                                                          uint32_t promote, uint32_t *__restrict__ promo,
                                                          uint32_t *__restrict__ hand) {
  __builtin_amdgcn_s_setprio(2);
  const uint32_t cnt = ctr[RD_VB_CNT];
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(&promo[1], cnt);  // (statistics: fgv_key_stats)
  if (cnt == 0) return;
  // LANES lanes per item, lane sl taking BITS bits of u2: windows sl * WINS .. sl * WINS + WINS - 1
  constexpr uint32_t BITS = 256u / LANES, WINS = BITS / 4u;
  const uint32_t lane = __lane_id(), sl = lane % LANES, base = lane - sl;
  constexpr uint32_t PER = 64u / LANES;
  uint32_t j0;
  while (vb_next(ctr + RD_VB_MUL, cnt, PER, j0)) {
    const uint32_t j = j0 + lane / LANES;
    if (j >= cnt) continue;  // (uniform within the lane group)
    const uint32_t i = list[j];
    const uint32_t id = key_slot[i];
    uint32_t r[8], w[8], u2[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      r[k] = r_limbs[(size_t)k * n + i];
      w[k] = w_in[(size_t)k * n + i];
    }
    sn_mul(u2, r, w);
    // this lane's BITS bits of u2, low-aligned (a select chain: no private array)
    const uint32_t li = sl * BITS / 32u;
    uint32_t dg = u2[0];
#pragma unroll
    for (int k = 1; k < 8; k++) dg = li == (uint32_t)k ? u2[k] : dg;
    if (BITS == 16u) dg = (sl & 1u) ? (dg >> 16) : (dg & 0xFFFFu);
    // window sl * WINS + k: digit (dg >> 4 k) & 15, row block k of this lane's tables
    const uint4 *qt = reinterpret_cast<const uint4 *>(vbt + (size_t)id * VBT_WORDS + sl * WINS * (VB_TAB * 16));
    jp28 a;
    bool inf = true;
    // the entry of window k+1 is loaded while window k is added (one gather in flight)
    uint32_t d = dg & 15u;
    uint4 n0, n1, n2, n3;
    if (d) n0 = qt[4 * (d - 1)], n1 = qt[4 * (d - 1) + 1], n2 = qt[4 * (d - 1) + 2], n3 = qt[4 * (d - 1) + 3];
#pragma unroll 1
    for (uint32_t k = 0; k < WINS; k++) {
      const uint32_t wx[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
      const uint32_t wy[8] = {n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
      const uint32_t dn = k + 1 < WINS ? (dg >> (4 * (k + 1))) & 15u : 0u;  // the next window's digit
      if (dn) {
        const uint4 *e = qt + (k + 1) * (VB_TAB * 4) + 4 * (dn - 1);
        n0 = e[0], n1 = e[1], n2 = e[2], n3 = e[3];
      }
      if (d) {
        f28 px, py;
        f28_from32(px, wx);
        f28_from32(py, wy);
        if (inf) {
          a.x = px;
          a.y = py;
          f28_load_c(a.z, ONE28);
          inf = false;
        } else {
          madd28(a, px, py);
        }
      }
      d = dn;
    }
    // butterfly over the item's lanes (infinite partial sums skipped)
#pragma unroll 1
    for (uint32_t m = 1; m < LANES; m <<= 1) {
      const int src = (int)(base + (sl ^ m));
      jp28 o;
      shfl_f28(o.x, a.x, src);
      shfl_f28(o.y, a.y, src);
      shfl_f28(o.z, a.z, src);
      const bool oinf = __shfl((int)inf, src) != 0;
      if (!oinf) {
        if (inf) {
          a = o;
          inf = false;
        } else {
          add28(a, o);
        }
      }
    }
    if (sl != 0) continue;
    const uint32_t u = atomicAdd(&uses[id], 1u);
    if (u + 1u == promote) {
      const uint32_t s = atomicAdd(&promo[0], 1u);
      if (s < VB_PROMO_CAP) atomicExch(&promo[2 + s], id);
    }
    if (inf || f28_is_zero(a.z)) {  // an exceptional addition (u2 * Q is never infinity): exact kernel
      hand[atomicAdd(ctr + RD_VB2_CNT, 1u)] = j;
      continue;
    }
    // Montgomery-280 -> Montgomery-256 Jacobian (k_vb_fin's form), canonical limbs
    f28 c, x, y, z;
    f28_load_c(c, C256_28);
    f28_mul(x, a.x, c);
    f28_mul(y, a.y, c);
    f28_mul(z, a.z, c);
    uint32_t *o = acc + (size_t)j * VB_ACC_WORDS;
    uint32_t t[8];
    f28_to32(t, x);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = t[k];
    f28_to32(t, y);
#pragma unroll
    for (int k = 0; k < 8; k++) o[8 + k] = t[k];
    f28_to32(t, z);
#pragma unroll
    for (int k = 0; k < 8; k++) o[16 + k] = t[k];
  }
}

#define VB_MUL28_ARGS                                                                                              \
  uint32_t n, const uint32_t *__restrict__ key_slot, const uint32_t *__restrict__ vbt,                           \
      const uint32_t *__restrict__ r_limbs, const uint32_t *__restrict__ w_in, uint32_t *__restrict__ ctr,      \
      const uint32_t *__restrict__ list, uint32_t *__restrict__ acc, uint32_t *__restrict__ uses, uint32_t promote, \
      uint32_t *__restrict__ promo, uint32_t *__restrict__ hand
__global__ __launch_bounds__(VB_THREADS) void k_vb_mul28(VB_MUL28_ARGS) {
  vb_mul28_body<8>(n, key_slot, vbt, r_limbs, w_in, ctr, list, acc, uses, promote, promo, hand);
}
__global__ __launch_bounds__(VB_THREADS) void k_vb_mul28_16(VB_MUL28_ARGS) {
  vb_mul28_body<16>(n, key_slot, vbt, r_limbs, w_in, ctr, list, acc, uses, promote, promo, hand);
}

// 2^304 mod p, radix 2^28: f28_mul(x * 2^256, K304) = x * 2^280 (Montgomery-256 -> Montgomery-280)
__constant__ static const uint32_t K304_28[10] = {0xffffu,    0x100000u, 0x0u,      0x1000u,    0xfffffffu,
                                                  0xfffffefu, 0xffffffu, 0xffff000u, 0xffffffeu, 0xfu};

// k_vb_fin: after k_prep -- acc[j] + sum of the 12 generator comb terms of u1 (k_prep's digits),
// then the projective x_R check of k_point -> status[list[j]].  The last workgroup to finish
// zeroes the list counters for the next batch (atomics only: no fence, no extra launch).
// The sum runs in radix 2^28 (k_point28's incomplete mixed addition on the Montgomery-280 comb
// entries as stored); an item whose sum met an exceptional case (Z = 0 at the end) is summed
// again with the complete radix-2^32 addition, as every item was before round 5.
__global__ __launch_bounds__(256) void k_vb_fin(uint32_t n, uint8_t *__restrict__ status,
                                                const apoint_raw *__restrict__ gtab28,
                                                const int8_t *__restrict__ digits,
                                                const uint32_t *__restrict__ r_limbs, uint32_t *__restrict__ ctr,
                                                const uint32_t *__restrict__ list, const uint32_t *__restrict__ acc) {
  __builtin_amdgcn_s_setprio(3);
  const uint32_t cnt = ctr[RD_VB_CNT];
  uint32_t j0;
  while (cnt && vb_next(ctr + RD_VB_FIN, cnt, 64u, j0)) {
    const uint32_t j = j0 + __lane_id();  // one item per lane
    if (j >= cnt) continue;
    const uint32_t i = list[j];
    jpoint a;
    load_jp(a, acc + (size_t)j * VB_ACC_WORDS);
    const int32_t *g = reinterpret_cast<const int32_t *>(digits + (size_t)i * DIG_STRIDE);
    uint32_t r[8];
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = r_limbs[(size_t)k * n + i];
    uint8_t st = 1;
    bool exact = fe_is_zero(a.z);
    if (!exact) {
      jp28 b;
      f28 t, k304;
      f28_load_c(k304, K304_28);
      f28_from32(t, a.x.v);
      f28_mul(b.x, t, k304);
      f28_from32(t, a.y.v);
      f28_mul(b.y, t, k304);
      f28_from32(t, a.z.v);
      f28_mul(b.z, t, k304);
#pragma unroll 1
      for (int win = 0; win < NGWIN; win++) {
        const int dd = g[win];
        if (dd == 0) continue;
        const uint4 *e = reinterpret_cast<const uint4 *>(gtab28 + (size_t)win * GT_K + ((dd < 0 ? -dd : dd) - 1));
        const uint4 n0 = e[0], n1 = e[1], n2 = e[2], n3 = e[3];
        const uint32_t wx[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
        const uint32_t wy[8] = {n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
        f28 px, py;
        f28_from32(px, wx);
        f28_from32(py, wy);
        if (dd < 0) {
          f28 z;
#pragma unroll
          for (int q = 0; q < 10; q++) z.v[q] = 0u;
          f28_sub(py, z, py, C4P28);
          f28_norm(py);
        }
        madd28(b, px, py);
      }
      if (f28_is_zero(b.z)) {
        exact = true;  // an exceptional addition: the complete sum below decides
      } else {
        f28 z2, rm, lhs, d, one;
        f28_sqr(z2, b.z);
        f28_load_c(one, ONE28);
        f28_to_mont(rm, r);
        f28_mul(lhs, rm, z2);
        f28_sub(d, b.x, lhs, C4P28);
        f28_mul(d, d, one);
        if (f28_is_zero(d)) {
          st = 0;
        } else {
          // x_R in [n, p): x_R mod n == r  <=>  x_R == r + n  (only if r + n < p)
          uint32_t c = 0, rn[8];
#pragma unroll
          for (int k = 0; k < 8; k++) rn[k] = addc(r[k], N_LIMBS[k], c, &c);
          if (c == 0u && lt_p(rn)) {
            f28_to_mont(rm, rn);
            f28_mul(lhs, rm, z2);
            f28_sub(d, b.x, lhs, C4P28);
            f28_mul(d, d, one);
            if (f28_is_zero(d)) st = 0;
          }
        }
      }
    }
    if (exact) {
      fe c232;
      fe_load_c(c232, C232_32);
#pragma unroll 1
      for (int win = 0; win < NGWIN; win++) {
        const int dd = g[win];
        if (dd == 0) continue;
        const apoint_raw *e = gtab28 + (size_t)win * GT_K + ((dd < 0 ? -dd : dd) - 1);
        apoint p;
        load_fe(p.x, e->x);
        load_fe(p.y, e->y);
        fe_mul(p.x, p.x, c232);  // Montgomery-280 -> Montgomery-256 (as k_point)
        fe_mul(p.y, p.y, c232);
        if (dd < 0) fe_neg(p.y, p.y);
        jpoint t2 = a;
        pt_madd(a, t2, p);
      }
      st = 1;
      if (!fe_is_zero(a.z)) {
        fe rr, rm, z2, lhs;
#pragma unroll
        for (int k = 0; k < 8; k++) rr.v[k] = r[k];
        fe_sqr(z2, a.z);
        fe_to_mont(rm, rr);
        fe_mul(lhs, rm, z2);
        if (fe_eq(lhs, a.x)) {
          st = 0;
        } else {
          uint32_t c = 0;
          fe rn;
#pragma unroll
          for (int k = 0; k < 8; k++) rn.v[k] = addc(rr.v[k], N_LIMBS[k], c, &c);
          if (c == 0u && lt_p(rn.v)) {
            fe_to_mont(rm, rn);
            fe_mul(lhs, rm, z2);
            if (fe_eq(lhs, a.x)) st = 0;
          }
        }
      }
    }
    status[i] = st;
  }
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(ctr + RD_VB_DONE, 1u) + 1u == gridDim.x) {
    atomicExch(ctr + RD_VB_CNT, 0u);
    atomicExch(ctr + RD_VB_MUL, 0u);
    atomicExch(ctr + RD_VB_FIN, 0u);
    atomicExch(ctr + RD_VB_DONE, 0u);
    atomicExch(ctr + RD_VB2_CNT, 0u);
    atomicExch(ctr + RD_VB2_MUL, 0u);
  }
}
