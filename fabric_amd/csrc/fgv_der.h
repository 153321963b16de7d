// fgv_der.h -- Go encoding/asn1 decoding of an ECDSA signature, exactly as
// fabric-lib-go bccsp/utils/ecdsa.go:41-65 (asn1.Unmarshal into struct{R,S *big.Int}),
// Go 1.21.9 encoding/asn1 rules:
//   * outer element: universal, constructed SEQUENCE; bytes after it are ignored
//     (UnmarshalECDSASignature discards `rest`);
//   * inside: two universal primitive INTEGERs; anything after S is ignored
//     (Go's struct decoding tolerates trailing elements);
//   * lengths definite and minimal; INTEGER contents non-empty and minimal;
//   * R.Sign() != 1 or S.Sign() != 1 (zero or negative) is an error.
// Compiled for host (buffers handed over by the BCCSP-shaped calls) and for the device
// (k_der, for batches already resident in HBM); one definition, so both agree.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace fgv {

struct DerTL {
  int cls, tag;
  bool constructed;
  size_t len;
};

// parseTagAndLength; returns false on any error
__host__ __device__ inline bool der_read_tl(const uint8_t *b, size_t n, size_t &o, DerTL &t) {
  if (o >= n) return false;
  const uint8_t first = b[o++];
  t.cls = first >> 6;
  t.constructed = (first & 0x20) != 0;
  t.tag = first & 0x1f;
  if (t.tag == 0x1f) {  // high-tag-number form (base 128, minimal, >= 31, < 2^31)
    uint64_t v = 0;
    for (int shifted = 0;; shifted++) {
      if (o >= n || shifted == 5) return false;
      const uint8_t c = b[o++];
      if (shifted == 0 && c == 0x80) return false;
      v = (v << 7) | (c & 0x7f);
      if (!(c & 0x80)) break;
    }
    if (v > 0x7fffffffu || v < 0x1f) return false;
    t.tag = (int)v;
  }
  if (o >= n) return false;
  const uint8_t l = b[o++];
  if (!(l & 0x80)) {
    t.len = l;
  } else {
    const int nb = l & 0x7f;
    if (nb == 0) return false;  // indefinite
    size_t len = 0;
    for (int i = 0; i < nb; i++) {
      if (o >= n) return false;
      if (len >= (1u << 23)) return false;
      len = (len << 8) | b[o++];
      if (len == 0) return false;  // leading zero length byte
    }
    if (len < 0x80) return false;  // long form for a short length
    t.len = len;
  }
  return true;
}

// One INTEGER.  Writes the magnitude as NLIMB little-endian u32 limbs (8: P-256, 12: P-384);
// big=true if >= 2^(32 NLIMB).
template <int NLIMB = 8>
__host__ __device__ inline bool der_read_int(const uint8_t *b, size_t n, size_t &o, uint32_t limbs[NLIMB], bool &big,
                         bool &positive) {
  if (o == n) return false;  // "sequence truncated"
  DerTL t;
  if (!der_read_tl(b, n, o, t)) return false;
  if (t.cls != 0 || t.tag != 2 || t.constructed) return false;
  if (o + t.len < o || o + t.len > n) return false;
  const uint8_t *v = b + o;
  size_t len = t.len;
  o += len;
  if (len == 0) return false;
  if (len > 1 && ((v[0] == 0x00 && !(v[1] & 0x80)) || (v[0] == 0xff && (v[1] & 0x80)))) return false;
  const bool neg = (v[0] & 0x80) != 0;
  while (len > 0 && v[0] == 0) {
    v++;
    len--;
  }
  positive = !neg && len > 0;
  big = len > 4u * NLIMB;
  for (int k = 0; k < NLIMB; k++) limbs[k] = 0;
  if (!big) {
    for (size_t i = 0; i < len; i++) {
      const size_t bytepos = len - 1 - i;  // little-endian byte index
      limbs[bytepos >> 2] |= (uint32_t)v[i] << (8 * (bytepos & 3));
    }
  }
  return true;
}

// Returns 0 on success (r, s written), 2 (FGV_SIG_DER) on any error.
template <int NLIMB = 8>
__host__ __device__ inline int der_decode_sig(const uint8_t *sig, size_t n, uint32_t r[NLIMB], uint32_t s[NLIMB],
                                              bool &r_big, bool &s_big) {
  size_t o = 0;
  DerTL t;
  if (n == 0 || !der_read_tl(sig, n, o, t)) return 2;
  if (t.cls != 0 || t.tag != 16 || !t.constructed) return 2;
  if (o + t.len < o || o + t.len > n) return 2;
  const uint8_t *in = sig + o;
  const size_t in_n = t.len;
  size_t io = 0;
  bool rp, sp;
  if (!der_read_int<NLIMB>(in, in_n, io, r, r_big, rp)) return 2;
  if (!der_read_int<NLIMB>(in, in_n, io, s, s_big, sp)) return 2;
  if (!rp || !sp) return 2;
  return 0;
}

// s <= n >> 1 (bccsp/utils/ecdsa.go:82-89); limbs little-endian
__host__ __device__ inline bool is_low_s(const uint32_t s[8]) {
  const uint32_t HALF_N[8] = {0x7E3192A8u, 0x79DCE561u, 0xD38BCF42u, 0xDE737D56u,
                                     0xFFFFFFFFu, 0x7FFFFFFFu, 0x80000000u, 0x7FFFFFFFu};
  for (int i = 7; i >= 0; i--) {
    if (s[i] < HALF_N[i]) return true;
    if (s[i] > HALF_N[i]) return false;
  }
  return true;
}

}  // namespace fgv
