// p384.hip -- identity.Verify for P-384 keys on the GPU.
//
// The reference verifies a P-384 identity like any ECDSA key: identity.Verify digests the message
// with the MSP's hash family (msp/identities.go:170-199) and bccsp's verifyECDSA
// (fabric-lib-go bccsp/sw/ecdsa.go:41-57) decodes the DER signature (bccsp/utils/ecdsa.go:41-65),
// applies the low-S rule with the P-384 half order (bccsp/utils/ecdsa.go:26-31, 82-89) and calls
// Go's ecdsa.Verify (go1.21.9 crypto/ecdsa verifyNISTEC over nistec.P384Point): r, s in [1, n),
// e = the digest (32 bytes: no truncation against a 384-bit order), w = s^-1, R = (e w) G + (r w) Q,
// R != infinity, x_R mod n == r.
//
// Per item, on the committer's verify list: k_der leaves an item whose key slot carries
// KEY_P384_FLAG as ST_P384, the P-256 stages skip it, and k_p384_verify decides it -- status bytes
// as for P-256 (0 valid, 1 false, 2 DER, 3 high-S, 4 range, 5 key, 6 empty).  So only the P-384
// signatures leave the P-256 kernels; their transactions and blocks stay on the device path.
//
// Both scalar multiplications use fixed-base combs of 8-bit windows (48 windows x 255 affine
// points, 1.2 MB per table): the generator's, built once per context, and one per registered P-384
// key, built at registration (P-384 keys belong to a handful of identities).  A verify is then 96
// exact mixed additions and no doublings, split over P384_LANES lanes (each a quarter of the
// windows) and summed with two exact Jacobian additions.  w = s^-1 is a binary extended Euclid.
#include <hip/hip_runtime.h>

#include <array>
#include <cstring>
#include <map>
#include <vector>

#include "fgv_der.h"
#include "fgv_internal.h"
#include "fgv_kernels.h"
#include "p384_field.h"

using namespace p384;

namespace {

__device__ inline void load_be32(uint32_t out[NL], const uint8_t *d) {  // a 32-byte big-endian digest
  for (int k = 0; k < NL; k++) out[k] = 0;
  for (int k = 0; k < 8; k++) {
    const uint8_t *q = d + 4 * (7 - k);
    out[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}
__device__ inline uint32_t scalar_byte(const uint32_t u[NL], uint32_t w) { return (u[w >> 2] >> (8 * (w & 3))) & 0xFFu; }

// table entry (window w, digit d >= 1) of a comb: x || y Montgomery
__device__ inline void load_entry(const uint32_t *tab, uint32_t w, uint32_t d, uint32_t x[NL], uint32_t y[NL]) {
  const uint32_t *e = tab + ((size_t)w * P384_TK + (d - 1)) * P384_ENTRY_WORDS;
  for (int k = 0; k < NL; k++) {
    x[k] = e[k];
    y[k] = e[NL + k];
  }
}

}  // namespace

// Comb build, step 1: one thread per (key, window w): B_w = 2^(8w) P (affine), then d B_w for
// d = 1..255 as Jacobian points into scratch[(k P384_WIN + w) P384_TK + d - 1].  pts: plain affine
// x || y, 12 little-endian limbs each, on the curve.
__global__ __launch_bounds__(64) void k_p384_tab(const uint32_t *__restrict__ pts, uint32_t nk, J *__restrict__ scratch) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nk * P384_WIN) return;
  const uint32_t k = t / P384_WIN, w = t % P384_WIN;
  uint32_t x[NL], y[NL];
  for (int i = 0; i < NL; i++) {
    x[i] = pts[(size_t)k * 2 * NL + i];
    y[i] = pts[(size_t)k * 2 * NL + NL + i];
  }
  J B;
  to_mont_p(B.X, x);
  to_mont_p(B.Y, y);
  cpy(B.Z, C().one_p);
  for (uint32_t i = 0; i < 8 * w; i++) dbl(B, B);
  uint32_t zi[NL], zi2[NL], bx[NL], by[NL];
  finv(zi, B.Z);
  fsqr(zi2, zi);
  fmul(bx, B.X, zi2);
  fmul(zi2, zi2, zi);
  fmul(by, B.Y, zi2);
  J cur;
  cpy(cur.X, bx);
  cpy(cur.Y, by);
  cpy(cur.Z, C().one_p);
  J *out = scratch + ((size_t)k * P384_WIN + w) * P384_TK;
  out[0] = cur;
  for (uint32_t d = 2; d <= P384_TK; d++) {
    madd(cur, cur, bx, by);
    out[d - 1] = cur;
  }
}

// Comb build, step 2: every entry to affine (one inversion per thread).  d 2^(8w) < n for every
// entry, so none is the infinity.
__global__ __launch_bounds__(64) void k_p384_norm(const J *__restrict__ scratch, uint32_t count, uint32_t *__restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const J P = scratch[i];
  uint32_t zi[NL], zi2[NL], x[NL], y[NL];
  finv(zi, P.Z);
  fsqr(zi2, zi);
  fmul(x, P.X, zi2);
  fmul(zi2, zi2, zi);
  fmul(y, P.Y, zi2);
  uint32_t *e = out + (size_t)i * P384_ENTRY_WORDS;
  for (int k = 0; k < NL; k++) {
    e[k] = x[k];
    e[NL + k] = y[k];
  }
}

// One verify per P384_LANES lanes (items with status ST_PENDING-P384 only; the others return at
// once, whole groups together).  sigp / sigl / slot / dig_idx: the committer's verify columns (or
// those of fgv_p384_verify_msgs); digests: 32 bytes each at dig_idx[i] (i when null).
__global__ __launch_bounds__(256) void k_p384_verify(uint32_t n, const uint32_t *__restrict__ dn,
                                                     uint8_t *__restrict__ status, const uint64_t *__restrict__ sigp,
                                                     const uint32_t *__restrict__ sigl,
                                                     const uint32_t *__restrict__ slot,
                                                     const uint32_t *__restrict__ dig_idx,
                                                     const uint8_t *__restrict__ digests,
                                                     const uint32_t *__restrict__ gtab,
                                                     const uint32_t *__restrict__ ktab,
                                                     const uint8_t *__restrict__ key_ok, uint32_t nkeys) {
  const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = gt / P384_LANES, l = gt % P384_LANES;
  const uint32_t cnt = dn ? min(n, *dn) : n;
  if (i >= cnt || status[i] != ST_P384) return;
  // every lane of the group decodes and inverts (the same values; no hand-over needed)
  const uint32_t L = sigl[i];
  const uint8_t *sig = reinterpret_cast<const uint8_t *>((uintptr_t)sigp[i]);
  uint32_t r[NL], s[NL];
  bool rb = false, sb = false;
  uint8_t code = ST_P384;
  const uint32_t kidx = slot[i] & ~KEY_P384_FLAG;
  if (L == 0) {
    code = 6;
  } else if (fgv::der_decode_sig<NL>(sig, L, r, s, rb, sb)) {
    code = 2;
  } else if (sb || (geq(s, C().half_n) && !eq(s, C().half_n))) {
    code = 3;  // s > n >> 1 (IsLowS with the P-384 half order)
  } else if (kidx >= nkeys || !key_ok[kidx]) {
    code = 5;
  } else if (rb || geq(r, C().n)) {
    code = 4;  // (r, s > 0: the DER decode; s < n: low S)
  }
  if (code != ST_P384) {
    if (l == 0) status[i] = code;
    return;
  }
  uint32_t e[NL], w[NL], u1[NL], u2[NL];
  load_be32(e, digests + 32 * (size_t)(dig_idx ? dig_idx[i] : i));
  inv_mod_n(w, s);
  mul_mod_n(u1, e, w);  // (e < 2^256 < n)
  mul_mod_n(u2, r, w);
  // this lane's windows: w = l, l + P384_LANES, ...
  const uint32_t *kt = ktab + (size_t)kidx * P384_ENTRIES * P384_ENTRY_WORDS;
  J acc;
  set_inf(acc);
  uint32_t x[NL], y[NL];
  for (uint32_t win = l; win < P384_WIN; win += P384_LANES) {
    const uint32_t d1 = scalar_byte(u1, win), d2 = scalar_byte(u2, win);
    if (d1) {
      load_entry(gtab, win, d1, x, y);
      madd(acc, acc, x, y);
    }
    if (d2) {
      load_entry(kt, win, d2, x, y);
      madd(acc, acc, x, y);
    }
  }
  // the lanes' partial sums, exact Jacobian additions (butterfly: every lane ends with the total)
  for (uint32_t m = 1; m < P384_LANES; m <<= 1) {
    J o;
    for (int k = 0; k < NL; k++) {
      o.X[k] = (uint32_t)__shfl_xor((int)acc.X[k], (int)m, P384_LANES);
      o.Y[k] = (uint32_t)__shfl_xor((int)acc.Y[k], (int)m, P384_LANES);
      o.Z[k] = (uint32_t)__shfl_xor((int)acc.Z[k], (int)m, P384_LANES);
    }
    add(acc, acc, o);
  }
  if (l != 0) return;
  if (is_zero(acc.Z)) {  // R at infinity
    status[i] = 1;
    return;
  }
  // x_R mod n == r  <=>  X == r Z^2, or (r + n < p) X == (r + n) Z^2 (x_R < p < 2n)
  uint32_t z2[NL], rm[NL], t[NL];
  fsqr(z2, acc.Z);
  to_mont_p(rm, r);
  fmul(t, rm, z2);
  bool ok = eq(t, acc.X);
  if (!ok && !geq(r, C().p_minus_n)) {
    uint32_t rn[NL];
    add_raw(rn, r, C().n);
    to_mont_p(rm, rn);
    fmul(t, rm, z2);
    ok = eq(t, acc.X);
  }
  status[i] = ok ? 0 : 1;
}

// ------------------------------------------------------------------------------- host side
struct fgv_p384_state {
  std::map<std::array<uint8_t, 96>, uint32_t> ids;  // key (X || Y big-endian) -> index
  std::vector<uint8_t> ok;                          // on the curve (its comb exists)
  DevBuf gtab, ktab, key_ok, scratch, pts;
  uint32_t cap = 0;                                 // keys ktab holds room for
  bool g_built = false;
};

static void be48_to_limbs(const uint8_t *b, uint32_t out[NL]) {
  for (int k = 0; k < NL; k++) {
    const uint8_t *q = b + 4 * (NL - 1 - k);
    out[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
}

// one comb table (pts: plain affine limbs) into dst, synchronously on c->stream
static int build_comb(fgv_ctx *c, fgv_p384_state &P, const uint32_t pts[2 * NL], uint32_t *dst) {
  if (!P.scratch.ensure(P384_ENTRIES * sizeof(J)) || !P.pts.ensure(2 * NL * 4)) return FGV_ENOMEM;
  HIP_TRY(hipMemcpyAsync(P.pts.p, pts, 2 * NL * 4, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(k_p384_tab, dim3(1), dim3(64), 0, c->stream, P.pts.as<uint32_t>(), 1u, P.scratch.as<J>());
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_p384_norm, dim3((uint32_t)((P384_ENTRIES + 63) / 64)), dim3(64), 0, c->stream,
                     P.scratch.as<const J>(), (uint32_t)P384_ENTRIES, dst);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  return FGV_OK;
}

// The key's index in the context's P-384 table (registered once; c->mu held).  An off-curve key
// gets an index whose verifies all fail with status 5, as Go's would not deserialize it.
int fgv_p384_key_locked(fgv_ctx *c, const uint8_t pub[96], uint32_t *idx) {
  if (!c->p384) c->p384 = new fgv_p384_state();
  fgv_p384_state &P = *c->p384;
  std::array<uint8_t, 96> k;
  memcpy(k.data(), pub, 96);
  auto it = P.ids.find(k);
  if (it != P.ids.end()) {
    *idx = it->second;
    return FGV_OK;
  }
  if (hipSetDevice(c->device) != hipSuccess) return FGV_EDEVICE;
  const uint32_t id = (uint32_t)P.ok.size();
  uint32_t pts[2 * NL];
  be48_to_limbs(pub, pts);
  be48_to_limbs(pub + 48, pts + NL);
  const bool on = on_curve(pts, pts + NL);
  if (!P.g_built) {
    const size_t tb = P384_ENTRIES * P384_ENTRY_WORDS * 4;
    if (!P.gtab.ensure(tb)) return FGV_ENOMEM;
    uint32_t g[2 * NL];
    from_mont_p(g, C().gx_m);
    from_mont_p(g + NL, C().gy_m);
    const int rc = build_comb(c, P, g, P.gtab.as<uint32_t>());
    if (rc) return rc;
    P.g_built = true;
  }
  if (id >= P.cap) {  // room for more keys: double, keep the built tables
    const uint32_t ncap = std::max<uint32_t>(4, 2 * P.cap);
    const size_t tb = P384_ENTRIES * P384_ENTRY_WORDS * 4;
    DevBuf nt;
    if (!nt.ensure(tb * ncap)) return FGV_ENOMEM;
    if (P.cap) HIP_TRY(hipMemcpy(nt.p, P.ktab.p, tb * P.cap, hipMemcpyDeviceToDevice));
    P.ktab.release();
    P.ktab = nt;
    P.cap = ncap;
    if (!P.key_ok.ensure(ncap)) return FGV_ENOMEM;
  }
  if (on) {
    const int rc = build_comb(c, P, pts, P.ktab.as<uint32_t>() + (size_t)id * P384_ENTRIES * P384_ENTRY_WORDS);
    if (rc) return rc;
  }
  P.ok.push_back(on ? 1 : 0);
  HIP_TRY(hipMemcpy(P.key_ok.p, P.ok.data(), P.ok.size(), hipMemcpyHostToDevice));
  P.ids.emplace(k, id);
  *idx = id;
  return FGV_OK;
}

uint32_t fgv_p384_nkeys(const fgv_ctx *c) { return c->p384 ? (uint32_t)c->p384->ok.size() : 0u; }

// k_p384_verify over a verify list (n = capacity, dn = the count in device memory or null) on
// stream st; nothing when the context has no P-384 key
int fgv_p384_launch(fgv_ctx *c, hipStream_t st, uint32_t n, const uint32_t *dn, uint8_t *status, const uint64_t *sigp,
                    const uint32_t *sigl, const uint32_t *slot, const uint32_t *dig_idx, const uint8_t *digests) {
  const uint32_t nk = fgv_p384_nkeys(c);
  if (nk == 0 || n == 0) return FGV_OK;
  const fgv_p384_state &P = *c->p384;
  const uint64_t threads = (uint64_t)n * P384_LANES;
  hipLaunchKernelGGL(k_p384_verify, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st, n, dn, status, sigp,
                     sigl, slot, dig_idx, digests, P.gtab.as<uint32_t>(), P.ktab.as<uint32_t>(),
                     P.key_ok.as<uint8_t>(), nk);
  HIP_TRY(hipGetLastError());
  return FGV_OK;
}

void fgv_p384_free(fgv_ctx *c) {
  if (!c->p384) return;
  fgv_p384_state &P = *c->p384;
  P.gtab.release();
  P.ktab.release();
  P.key_ok.release();
  P.scratch.release();
  P.pts.release();
  delete c->p384;
  c->p384 = nullptr;
}
