// fgv_x509.cpp -- X.509 subset of the MSP cache-miss path (see fgv_x509.h).
// Go 1.21 crypto/x509 ParseCertificate / encoding/asn1 / encoding/pem, restricted to the shapes
// Fabric CAs issue; the oracle's restatement of the same rules is oracle/x509.py.
#include "fgv_x509.h"

#include <string.h>
#include <time.h>

#include <algorithm>

#include "p384_field.h"
#include "pbwire.h"

namespace fgvx {
namespace {

struct XErr {
  int code;
};
[[noreturn]] void perr() { throw XErr{X_PARSE}; }
[[noreturn]] void unsup() { throw XErr{X_UNSUP}; }

struct T {  // one DER element
  uint8_t tag;
  size_t hs, cs, ce;  // header start, content start, content end
};

// strict definite-length DER header at b[i..end)
T tlv(const uint8_t *b, size_t i, size_t end) {
  if (i + 2 > end) perr();
  const uint8_t tag = b[i];
  if ((tag & 0x1F) == 0x1F) perr();
  size_t ln = b[i + 1], o = i + 2;
  if (ln & 0x80) {
    const size_t nb = ln & 0x7F;
    if (nb == 0 || nb > 4 || o + nb > end) perr();
    if (b[o] == 0) perr();
    ln = 0;
    for (size_t k = 0; k < nb; k++) ln = (ln << 8) | b[o + k];
    if (ln < 128) perr();
    o += nb;
  }
  if (ln > end - o) perr();
  return T{tag, i, o, o + ln};
}

std::vector<T> children(const uint8_t *b, size_t s, size_t e) {
  std::vector<T> out;
  while (s < e) {
    out.push_back(tlv(b, s, e));
    s = out.back().ce;
  }
  return out;
}

bool eq(const uint8_t *b, const T &t, const char *hex_bytes, size_t n) {
  return t.ce - t.cs == n && memcmp(b + t.cs, hex_bytes, n) == 0;
}

#define OIDV(name, ...) const char name[] = {__VA_ARGS__}
OIDV(OID_EC_KEY, '\x2a', '\x86', '\x48', '\xce', '\x3d', '\x02', '\x01');
OIDV(OID_P256, '\x2a', '\x86', '\x48', '\xce', '\x3d', '\x03', '\x01', '\x07');
OIDV(OID_P384, '\x2b', '\x81', '\x04', '\x00', '\x22');  // secp384r1
OIDV(OID_ED25519, '\x2b', '\x65', '\x70');
OIDV(OID_RSA, '\x2a', '\x86', '\x48', '\x86', '\xf7', '\x0d', '\x01', '\x01', '\x01');
OIDV(OID_OU, '\x55', '\x04', '\x0b');
#undef OIDV
// AlgorithmIdentifier{ecdsa-with-SHA256} with no parameters
const uint8_t ALG_ECDSA_SHA256[12] = {0x30, 0x0a, 0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x04, 0x03, 0x02};

// id-ce-* extension (2.5.29.x) number, or -1
int ce_ext(const uint8_t *b, const T &t) {
  if (t.ce - t.cs == 3 && b[t.cs] == 0x55 && b[t.cs + 1] == 0x1d) return b[t.cs + 2];
  return -1;
}
const uint8_t OID_AIA[8] = {0x2b, 0x06, 0x01, 0x05, 0x05, 0x07, 0x01, 0x01};

// cryptobyte ReadASN1ObjectIdentifier: non-empty, every subidentifier minimal (no leading 0x80),
// at most 5 bytes and below 2^31, none truncated
bool valid_oid(const uint8_t *b, size_t n) {
  if (n == 0) return false;
  size_t i = 0;
  while (i < n) {
    uint32_t ret = 0;
    for (int k = 0;; k++) {
      if (k == 5 || i >= n || ret >= (1u << 24)) return false;
      const uint8_t c = b[i++];
      if (k == 0 && c == 0x80) return false;
      ret = (ret << 7) | (c & 0x7F);
      if (!(c & 0x80)) break;
    }
  }
  return true;
}
bool valid_oid(const uint8_t *b, const T &t) { return t.tag == 0x06 && valid_oid(b + t.cs, t.ce - t.cs); }

// minimal two's-complement INTEGER content: false if empty / non-minimal
bool int_minimal(const uint8_t *b, size_t s, size_t e) {
  if (e == s) return false;
  if (e - s > 1 && ((b[s] == 0 && b[s + 1] < 0x80) || (b[s] == 0xFF && b[s + 1] >= 0x80))) return false;
  return true;
}

int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}

int64_t parse_time(const uint8_t *b, const T &t) {
  const size_t n = t.ce - t.cs;
  const uint8_t *v = b + t.cs;
  auto digits = [&](size_t k) {
    for (size_t i = 0; i < k; i++)
      if (v[i] < '0' || v[i] > '9') return false;
    return true;
  };
  auto two = [](const uint8_t *p) { return (p[0] - '0') * 10 + (p[1] - '0'); };
  int64_t y;
  const uint8_t *rest;
  if (t.tag == 0x17 && n == 13 && v[12] == 'Z' && digits(12)) {
    const int yy = two(v);
    y = yy >= 50 ? 1900 + yy : 2000 + yy;
    rest = v + 2;
  } else if (t.tag == 0x18 && n == 15 && v[14] == 'Z' && digits(14)) {
    y = two(v) * 100 + two(v + 2);
    rest = v + 4;
  } else {
    unsup();
  }
  const int mo = two(rest), d = two(rest + 2), hh = two(rest + 4), mm = two(rest + 6), ss = two(rest + 8);
  static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  if (!(mo >= 1 && mo <= 12)) perr();
  const int dim = mdays[mo - 1] + (mo == 2 && leap ? 1 : 0);
  if (!(d >= 1 && d <= dim && hh < 24 && mm < 60 && ss < 60)) perr();  // (time.Parse: day out of range)
  return days_from_civil(y, (unsigned)mo, 1) * 86400 + (int64_t)(d - 1) * 86400 + hh * 3600 + mm * 60 + ss;
}

std::string name_string(const uint8_t *b, const T &t) {
  const uint8_t *p = b + t.cs;
  const size_t n = t.ce - t.cs;
  if (t.tag == 0x0C) {
    if (!pbw::utf8_valid(p, n)) perr();
  } else if (t.tag == 0x13) {
    for (size_t i = 0; i < n; i++) {
      const uint8_t c = p[i];
      const bool ok = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
                      (c && strchr(" '()+,-./:=?*&", c));
      if (!ok) perr();
    }
  } else if (t.tag == 0x16) {
    for (size_t i = 0; i < n; i++)
      if (p[i] >= 0x80) perr();
  } else if (t.tag == 0x12 || t.tag == 0x14 || t.tag == 0x1E) {  // Numeric, T61, BMP: not restated
    unsup();
  } else {
    perr();  // parseASN1String: unsupported string type
  }
  return std::string((const char *)p, n);
}

// cryptobyte.String over b[s..e): each read mirrors the Go call named beside it.  A read Go
// makes that fails is a parse error (X_PARSE, Go's ParseCertificate returns an error); bytes Go
// leaves unread where this restatement would need to know what Go does with them are X_UNSUP.
struct Rd {
  const uint8_t *b;
  size_t s, e;
  bool empty() const { return s >= e; }
  bool peek(uint8_t tag) const { return s < e && b[s] == tag; }  // PeekASN1Tag
  T any() {  // ReadAnyASN1Element
    const T t = tlv(b, s, e);
    s = t.ce;
    return t;
  }
  T elem(uint8_t tag) {  // ReadASN1Element / ReadASN1 with a tag
    const T t = any();
    if (t.tag != tag) perr();
    return t;
  }
  Rd in(const T &t) const { return Rd{b, t.cs, t.ce}; }
  void rest_unread() const {  // Go ignores what is left here: outside the model
    if (!empty()) unsup();
  }
};

// ReadASN1BitString's validity rules (padding count <= 7, none without data, padding bits zero)
void bitstring_ok(const uint8_t *b, const T &t) {
  if (t.ce == t.cs || b[t.cs] > 7 || (t.ce - t.cs == 1 && b[t.cs]) || (b[t.ce - 1] & ((1u << b[t.cs]) - 1))) perr();
}

// parseName: RDNSequence of SETs of AttributeTypeAndValue {OID, any string}; what an attribute
// holds after its value is never read by Go (nor here)
void name_ous(const uint8_t *b, const T &name, std::vector<std::string> *out) {
  Rd raw{b, name.cs, name.ce};
  while (!raw.empty()) {
    Rd set = raw.in(raw.elem(0x31));
    while (!set.empty()) {
      Rd atv = set.in(set.elem(0x30));
      const T t1 = atv.elem(0x06);
      if (!valid_oid(b, t1)) perr();
      const T t2 = atv.any();
      std::string s = name_string(b, t2);  // parseASN1String: every attribute value parses
      if (out && eq(b, t1, OID_OU, sizeof OID_OU)) out->push_back(std::move(s));
    }
  }
}

bool der_bool(const uint8_t *b, const T &t) {  // ReadASN1Boolean
  if (t.ce - t.cs != 1 || (b[t.cs] != 0x00 && b[t.cs] != 0xFF)) perr();
  return b[t.cs] == 0xFF;
}

// ReadASN1Integer into a Go int (64-bit): minimal, at most 8 bytes
int64_t int64_of(const uint8_t *b, const T &t) {
  if (t.tag != 0x02 || !int_minimal(b, t.cs, t.ce) || t.ce - t.cs > 8) perr();
  int64_t x = (b[t.cs] & 0x80) ? -1 : 0;
  for (size_t q = t.cs; q < t.ce; q++) x = (int64_t)(((uint64_t)x << 8) | b[q]);
  return x;
}

// parseAI: OID, then at most one parameters element; anything after it is never read by Go
void parse_ai(const uint8_t *b, const T &ai, T *oid, T *params, bool *has_params) {
  Rd r{b, ai.cs, ai.ce};
  *oid = r.elem(0x06);
  if (!valid_oid(b, *oid)) perr();
  *has_params = !r.empty();
  if (*has_params) *params = r.any();
  r.rest_unread();
}

// x509.ParseCertificate (Go 1.21 crypto/x509/parser.go parseCertificate), in Go's read order
void parse(Cert &c) {
  const uint8_t *b = c.der.data();
  const size_t n = c.der.size();
  Rd all{b, 0, n};
  const T top = all.elem(0x30);  // "x509: malformed certificate"
  if (top.ce != n) perr();       // "x509: trailing data"
  Rd input = all.in(top);
  const T tbs = input.elem(0x30);  // "x509: malformed tbs certificate"
  c.tbs_off = tbs.hs;
  c.tbs_len = tbs.ce - tbs.hs;
  Rd t = input.in(tbs);
  int64_t version = 0;
  if (t.peek(0xA0)) {  // ReadOptionalASN1Integer([0] EXPLICIT, default 0)
    Rd vr = t.in(t.elem(0xA0));
    version = int64_of(b, vr.elem(0x02));
    if (!vr.empty()) perr();
  }
  if (version < 0 || version > 2) perr();  // "x509: malformed version" / "invalid version"
  if (version != 2) unsup();               // v1 / v2 certificates: not restated
  c.version = 3;
  const T serial = t.elem(0x02);  // ReadASN1Integer(*big.Int)
  if (!int_minimal(b, serial.cs, serial.ce)) perr();
  c.serial_off = serial.cs;
  c.serial_len = serial.ce - serial.cs;
  const T alg = t.elem(0x30);
  const T oalg = input.elem(0x30);
  if (alg.ce - alg.cs != oalg.ce - oalg.cs || memcmp(b + alg.cs, b + oalg.cs, alg.ce - alg.cs)) perr();
  T aoid, apar;
  bool ahas;
  parse_ai(b, alg, &aoid, &apar, &ahas);
  if (oalg.ce - oalg.hs != sizeof ALG_ECDSA_SHA256 || memcmp(b + oalg.hs, ALG_ECDSA_SHA256, sizeof ALG_ECDSA_SHA256))
    unsup();
  const T issuer = t.elem(0x30);
  name_ous(b, issuer, nullptr);
  Rd validity = t.in(t.elem(0x30));
  const bool time_tag = validity.peek(0x17) || validity.peek(0x18);  // parseTime
  if (!time_tag) perr();  // "x509: unsupported time format"
  c.not_before = parse_time(b, validity.any());
  if (!(validity.peek(0x17) || validity.peek(0x18))) perr();
  c.not_after = parse_time(b, validity.any());
  validity.rest_unread();
  const T subject = t.elem(0x30);
  name_ous(b, subject, &c.ous);
  c.issuer_off = issuer.hs;
  c.issuer_len = issuer.ce - issuer.hs;
  c.subject_off = subject.hs;
  c.subject_len = subject.ce - subject.hs;
  // public key
  Rd spki = t.in(t.elem(0x30));
  const T pkai = spki.elem(0x30);
  T koid, kpar;
  bool khas;
  parse_ai(b, pkai, &koid, &kpar, &khas);
  const T spk = spki.elem(0x03);
  bitstring_ok(b, spk);
  spki.rest_unread();
  c.key = XK_OTHER;
  if (eq(b, koid, OID_EC_KEY, sizeof OID_EC_KEY)) {
    if (khas && kpar.tag == 0x06 && eq(b, kpar, OID_P256, sizeof OID_P256)) {
      const uint8_t *bits = b + spk.cs;
      const size_t bl = spk.ce - spk.cs;
      if (bl != 66 || bits[0] != 0 || bits[1] != 4) unsup();
      if (!p256_on_curve(bits + 2, bits + 34)) perr();  // elliptic.Unmarshal fails
      memcpy(c.pub, bits + 2, 64);
      c.key = XK_P256;
    } else if (khas && kpar.tag == 0x06 && eq(b, kpar, OID_P384, sizeof OID_P384)) {
      // P-384 leaves (round 6): elliptic.Unmarshal of the uncompressed point, verified per item
      // on the GPU (p384.hip) like the registered P-384 identities
      const uint8_t *bits = b + spk.cs;
      const size_t bl = spk.ce - spk.cs;
      if (bl != 98 || bits[0] != 0 || bits[1] != 4) unsup();
      if (!p384_on_curve(bits + 2, bits + 50)) perr();
      memcpy(c.pub384, bits + 2, 96);
      c.key = XK_P384;
    } else {  // (other curves: not restated; no GPU verify either)
      unsup();
    }
  } else if (eq(b, koid, OID_ED25519, sizeof OID_ED25519)) {
    c.key = XK_UNDESERIALIZABLE;  // (a parse error or a KeyImport error: undeserializable either way)
  } else if (eq(b, koid, OID_RSA, sizeof OID_RSA)) {
    // RSA never passes identity.Verify (msp/identities.go:190 passes nil opts, rejected by
    // bccsp/sw/rsa.go:48-61): key accepted or not by Go's PKCS#1 checks, every path
    // treats the identity alike (creator: BAD_CREATOR_SIGNATURE; endorsement, orderer signature:
    // skipped) -- FGV_KEY_OTHER, whose Verify always fails
    c.key = XK_OTHER;
  } else {
    unsup();
  }
  // issuerUniqueID / subjectUniqueID: not restated
  if (t.peek(0x81) || t.peek(0x82)) unsup();
  struct Ext {
    int id;
    T val;
    bool crit;
  };
  std::vector<Ext> exts;
  if (t.peek(0xA3)) {
    Rd xr = t.in(t.elem(0xA3));
    Rd er = xr.in(xr.elem(0x30));  // "x509: malformed extensions"
    xr.rest_unread();
    std::vector<std::vector<uint8_t>> seen;
    while (!er.empty()) {
      Rd e = er.in(er.elem(0x30));  // parseExtension
      const T eo = e.elem(0x06);
      if (!valid_oid(b, eo)) perr();
      bool crit = false;
      if (e.peek(0x01)) crit = der_bool(b, e.elem(0x01));
      const T val = e.elem(0x04);
      e.rest_unread();
      std::vector<uint8_t> oid(b + eo.cs, b + eo.ce);
      if (std::find(seen.begin(), seen.end(), oid) != seen.end()) perr();  // duplicate extensions
      seen.push_back(oid);
      const int id = ce_ext(b, eo);
      // extensions Go parses that this restatement does not: name constraints (30), CRL
      // distribution points (31), certificate policies (32), AIA, freshest CRL (46); a critical
      // SKI / AKI (rejected by some Go versions' parsers)
      if (id == 30 || id == 31 || id == 32 || id == 46 ||
          (oid.size() == sizeof OID_AIA && memcmp(oid.data(), OID_AIA, sizeof OID_AIA) == 0) ||
          ((id == 14 || id == 35) && crit))
        unsup();
      if (id == 14 || id == 15 || id == 17 || id == 19 || id == 35 || id == 37) {
        exts.push_back(Ext{id, val, crit});
      } else if (crit) {
        c.unhandled_critical = true;
      }
    }
  }
  t.rest_unread();  // what follows the extensions in the TBS is never read by Go
  for (const Ext &x : exts) {  // processExtensions
    Rd v{b, x.val.cs, x.val.ce};
    if (x.id == 19) {  // parseBasicConstraintsExtension
      Rd k = v.in(v.elem(0x30));
      v.rest_unread();
      if (k.peek(0x01)) c.is_ca = der_bool(b, k.elem(0x01));
      if (k.peek(0x02)) c.path_len = int64_of(b, k.elem(0x02));
      k.rest_unread();
      c.bc_valid = true;
    } else if (x.id == 14) {  // subjectKeyIdentifier
      const T k = v.elem(0x04);
      v.rest_unread();
      c.has_ski = true;
      c.ski_off = k.cs;
      c.ski_len = k.ce - k.cs;
    } else if (x.id == 15) {  // parseKeyUsageExtension: ReadASN1BitString, its first 9 bits
      const T bs = v.elem(0x03);
      bitstring_ok(b, bs);
      v.rest_unread();
      uint32_t ku = 0;
      for (size_t q = bs.cs + 1, kk = 0; q < bs.ce; q++, kk++)
        for (int bit = 0; bit < 8; bit++)
          if (b[q] & (0x80 >> bit) && 8 * kk + bit < 9) ku |= 1u << (8 * kk + bit);
      c.key_usage = ku;
    } else if (x.id == 35) {  // authorityKeyIdentifier: SEQUENCE, an optional [0] keyIdentifier
      Rd k = v.in(v.elem(0x30));
      v.rest_unread();
      if (k.peek(0x80)) k.elem(0x80);  // (the rest of the SEQUENCE is never read by Go)
    } else {  // extKeyUsage (37), subjectAltName (17): SEQUENCE, every element read
      Rd k = v.in(v.elem(0x30));
      v.rest_unread();
      int names = 0;
      while (!k.empty()) {
        const T e = k.any();
        if (x.id == 37 && !valid_oid(b, e)) perr();  // "x509: invalid extended key usages"
        if (x.id == 17) {                            // parseSANExtension (by tag ^ 0x80)
          if (e.tag == 0x81 || e.tag == 0x82)
            for (size_t q = e.cs; q < e.ce; q++)
              if (b[q] >= 0x80) perr();  // rfc822Name / dNSName malformed
          if (e.tag == 0x86) unsup();    // URI (url.Parse not restated)
          if (e.tag == 0x87 && e.ce - e.cs != 4 && e.ce - e.cs != 16) perr();
          names += e.tag == 0x81 || e.tag == 0x82 || e.tag == 0x87;
        }
      }
      if (x.id == 17 && !names && x.crit) c.unhandled_critical = true;  // (nothing parsed)
    }
  }
  const T sigb = input.elem(0x03);  // "x509: malformed signature"
  bitstring_ok(b, sigb);
  if (b[sigb.cs] != 0) unsup();  // (RightAlign of a padded signature: not restated)
  c.sig_off = sigb.cs + 1;
  c.sig_len = sigb.ce - sigb.cs - 1;
  input.rest_unread();  // elements after the signature: Go ignores them (cert.Raw keeps them)
}

// ---- P-256 field arithmetic for the on-curve check (4 x 64-bit limbs, little-endian) ----
typedef unsigned __int128 u128;
struct U256 {
  uint64_t w[4];
};
const U256 P = {{0xFFFFFFFFFFFFFFFFull, 0x00000000FFFFFFFFull, 0x0000000000000000ull, 0xFFFFFFFF00000001ull}};
const U256 Bc = {{0x3BCE3C3E27D2604Bull, 0x651D06B0CC53B0F6ull, 0xB3EBBD55769886BCull, 0x5AC635D8AA3A93E7ull}};
const U256 N = {{0xF3B9CAC2FC632551ull, 0xBCE6FAADA7179E84ull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFF00000000ull}};
const U256 NH = {{0x79DCE5617E3192A8ull, 0xDE737D56D38BCF42ull, 0x7FFFFFFFFFFFFFFFull, 0x7FFFFFFF80000000ull}};

U256 from_be(const uint8_t *p) {
  U256 r;
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | p[(3 - i) * 8 + k];
    r.w[i] = v;
  }
  return r;
}
void to_be(const U256 &a, uint8_t *p) {
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) p[(3 - i) * 8 + k] = (uint8_t)(a.w[i] >> (56 - 8 * k));
}
int cmp(const U256 &a, const U256 &b) {
  for (int i = 3; i >= 0; i--)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
uint64_t sub(U256 &r, const U256 &a, const U256 &b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 d = (u128)a.w[i] - b.w[i] - br;
    r.w[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
uint64_t add(U256 &r, const U256 &a, const U256 &b) {
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 s = (u128)a.w[i] + b.w[i] + c;
    r.w[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  return c;
}
U256 addm(const U256 &a, const U256 &b) {
  U256 r;
  const uint64_t c = add(r, a, b);
  if (c || cmp(r, P) >= 0) sub(r, r, P);
  return r;
}
U256 subm(const U256 &a, const U256 &b) {
  U256 r;
  if (sub(r, a, b)) add(r, r, P);
  return r;
}
// a*b mod p by double-and-add over b's bits (host check, a few microseconds)
U256 mulm(const U256 &a, const U256 &b) {
  U256 r = {{0, 0, 0, 0}};
  for (int i = 255; i >= 0; i--) {
    r = addm(r, r);
    if ((b.w[i / 64] >> (i % 64)) & 1) r = addm(r, a);
  }
  return r;
}

}  // namespace

// encoding/pem Decode, first block, for the one shape the engine models (X_OK):
//   "-----BEGIN <type>-----" at offset 0, lines of base64 alphabet only, "-----END <type>-----"
//   at a line start, then nothing, "\n" or "\r\n" (what follows that line is never read);
//   line ends "\n" or "\r\n"; canonical padding.
// X_PARSE only where Go's Decode certainly returns nil: no "-----BEGIN " anywhere in the input.
// Every other shape is X_UNSUP: Go's Decode may still find a block there (a BEGIN after a '\n',
// a later block after a malformed one, headers, spaces and tabs it strips, ...).
int pem_decode(const uint8_t *p, size_t n, std::vector<uint8_t> &der) {
  static const char BEGIN[] = "-----BEGIN ", END[] = "-----END ", DASH[] = "-----";
  if (!memmem(p, n, BEGIN, 11)) return X_PARSE;
  if (n < 11 || memcmp(p, BEGIN, 11)) return X_UNSUP;
  size_t i = 11;
  const size_t ts = i;
  while (i < n && p[i] != '-' && p[i] >= 0x20 && p[i] < 0x7F) i++;
  const size_t te = i;
  auto eol = [&](size_t &k) {
    if (k < n && p[k] == '\n') return k++, true;
    if (k + 1 < n && p[k] == '\r' && p[k + 1] == '\n') return k += 2, true;
    return false;
  };
  auto b64c = [](uint8_t ch) {
    return (ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9') || ch == '+' ||
           ch == '/' || ch == '=';
  };
  if (n - i < 5 || memcmp(p + i, DASH, 5)) return X_UNSUP;
  i += 5;
  if (!eol(i)) return X_UNSUP;
  std::string b64;
  for (;;) {
    if (i >= n) return X_UNSUP;  // no END line
    if (n - i >= 9 && !memcmp(p + i, END, 9)) break;
    const size_t a = i;
    while (i < n && b64c(p[i])) i++;
    b64.append((const char *)p + a, i - a);
    if (!eol(i)) return X_UNSUP;
  }
  i += 9;
  const size_t tl = te - ts;
  if (n - i < tl + 5 || memcmp(p + i, p + ts, tl) || memcmp(p + i + tl, DASH, 5)) return X_UNSUP;
  i += tl + 5;
  if (i != n && !eol(i)) return X_UNSUP;
  // base64.StdEncoding: whole quanta, '=' only as the last one or two characters
  if (b64.size() % 4) return X_UNSUP;
  der.clear();
  der.reserve(b64.size() / 4 * 3);
  auto val = [](char ch) -> int {
    if (ch >= 'A' && ch <= 'Z') return ch - 'A';
    if (ch >= 'a' && ch <= 'z') return ch - 'a' + 26;
    if (ch >= '0' && ch <= '9') return ch - '0' + 52;
    if (ch == '+') return 62;
    if (ch == '/') return 63;
    return -1;
  };
  for (size_t q = 0; q < b64.size(); q += 4) {
    int v[4], pad = 0;
    for (int t = 0; t < 4; t++) {
      const char ch = b64[q + t];
      if (ch == '=') {
        if (q + 4 != b64.size() || t < 2) return X_UNSUP;
        v[t] = 0;
        pad++;
      } else {
        if (pad) return X_UNSUP;
        v[t] = val(ch);
      }
    }
    const uint32_t w = (uint32_t)v[0] << 18 | (uint32_t)v[1] << 12 | (uint32_t)v[2] << 6 | (uint32_t)v[3];
    der.push_back((uint8_t)(w >> 16));
    if (pad < 2) der.push_back((uint8_t)(w >> 8));
    if (pad < 1) der.push_back((uint8_t)w);
  }
  return X_OK;
}

namespace {
const uint8_t OID_AKI[3] = {0x55, 0x1d, 0x23};
const uint8_t OID_ECDSA_SHA256_B[8] = {0x2a, 0x86, 0x48, 0xce, 0x3d, 0x04, 0x03, 0x02};

// AlgorithmIdentifier {OID, [NULL]} -> the OID element
T crl_alg(const uint8_t *b, size_t s, size_t e) {
  const std::vector<T> k = children(b, s, e);
  if (k.empty() || !valid_oid(b, k[0])) unsup();
  if (k.size() > 2 || (k.size() == 2 && (k[1].tag != 0x05 || k[1].ce != k[1].cs))) unsup();
  return k[0];
}
void crl_time(const uint8_t *b, const T &t) {
  if (t.tag != 0x17 && t.tag != 0x18) unsup();
  parse_time(b, t);
}
// Extensions: (OID element, value element) of each {OID, [BOOLEAN], OCTET STRING}
std::vector<std::pair<T, T>> crl_exts(const uint8_t *b, size_t s, size_t e) {
  std::vector<std::pair<T, T>> out;
  for (const T &x : children(b, s, e)) {
    if (x.tag != 0x30) unsup();
    std::vector<T> k = children(b, x.cs, x.ce);
    if (k.size() == 3 && k[1].tag == 0x01) {
      if (k[1].ce - k[1].cs != 1 || (b[k[1].cs] != 0x00 && b[k[1].cs] != 0xFF)) perr();  // asn1 parseBool
      k.erase(k.begin() + 1);
    }
    if (k.size() != 2 || !valid_oid(b, k[0]) || k[1].tag != 0x04) unsup();
    out.push_back({k[0], k[1]});
  }
  return out;
}
void parse_crl_der(Crl &c) {
  const uint8_t *b = c.der.data();
  const size_t n = c.der.size();
  const T top = tlv(b, 0, n);
  if (top.tag != 0x30 || top.ce != n) perr();  // "x509: trailing data after CRL"
  const std::vector<T> t3 = children(b, top.cs, top.ce);
  if (t3.size() != 3 || t3[0].tag != 0x30 || t3[1].tag != 0x30 || t3[2].tag != 0x03) unsup();
  c.tbs_off = t3[0].hs;
  c.tbs_len = t3[0].ce - t3[0].hs;
  const std::vector<T> k = children(b, t3[0].cs, t3[0].ce);
  size_t i = 0;
  if (i < k.size() && k[i].tag == 0x02) {  // version (optional, default 0): 0 or 1
    if (!int_minimal(b, k[i].cs, k[i].ce)) perr();
    if (k[i].ce - k[i].cs != 1 || b[k[i].cs] > 1) unsup();
    i++;
  }
  if (i >= k.size() || k[i].tag != 0x30) unsup();
  crl_alg(b, k[i].cs, k[i].ce);
  i++;
  if (i >= k.size() || k[i].tag != 0x30) unsup();
  for (const T &rdn : children(b, k[i].cs, k[i].ce)) {  // issuer RDNSequence
    if (rdn.tag != 0x31) unsup();
    for (const T &atv : children(b, rdn.cs, rdn.ce)) {
      if (atv.tag != 0x30) unsup();
      const std::vector<T> a = children(b, atv.cs, atv.ce);
      if (a.size() != 2 || !valid_oid(b, a[0])) unsup();
      if (a[1].tag != 0x13 && a[1].tag != 0x0C && a[1].tag != 0x16) unsup();
      name_string(b, a[1]);
    }
  }
  i++;
  if (i >= k.size()) unsup();
  crl_time(b, k[i++]);  // thisUpdate
  if (i < k.size() && (k[i].tag == 0x17 || k[i].tag == 0x18)) crl_time(b, k[i++]);  // nextUpdate
  if (i < k.size() && k[i].tag == 0x30) {  // revokedCertificates
    for (const T &rc : children(b, k[i].cs, k[i].ce)) {
      if (rc.tag != 0x30) unsup();
      const std::vector<T> r = children(b, rc.cs, rc.ce);
      if ((r.size() != 2 && r.size() != 3) || r[0].tag != 0x02) unsup();
      if (!int_minimal(b, r[0].cs, r[0].ce)) perr();
      c.serials.emplace_back(b + r[0].cs, b + r[0].ce);
      crl_time(b, r[1]);
      if (r.size() == 3) {
        if (r[2].tag != 0x30) unsup();
        crl_exts(b, r[2].cs, r[2].ce);
      }
    }
    i++;
  }
  std::vector<std::pair<T, T>> exts;
  if (i < k.size() && k[i].tag == 0xA0) {  // crlExtensions [0] EXPLICIT
    const std::vector<T> in = children(b, k[i].cs, k[i].ce);
    if (in.size() != 1 || in[0].tag != 0x30) unsup();
    exts = crl_exts(b, in[0].cs, in[0].ce);
    i++;
  }
  if (i != k.size()) unsup();
  // exactly one AuthorityKeyIdentifier, holding only a [0] keyIdentifier
  int naki = 0;
  for (const auto &x : exts) {
    if (x.first.ce - x.first.cs != 3 || memcmp(b + x.first.cs, OID_AKI, 3) != 0) continue;
    naki++;
    const T a = tlv(b, x.second.cs, x.second.ce);
    if (a.tag != 0x30 || a.ce != x.second.ce) unsup();
    const std::vector<T> ak = children(b, a.cs, a.ce);
    if (ak.size() != 1 || ak[0].tag != 0x80) unsup();
    c.aki.assign(b + ak[0].cs, b + ak[0].ce);
  }
  if (naki != 1) unsup();
  const T alg = crl_alg(b, t3[1].cs, t3[1].ce);
  if (alg.ce - alg.cs != 8 || memcmp(b + alg.cs, OID_ECDSA_SHA256_B, 8) != 0) unsup();
  // signatureValue BIT STRING, no padding bits; utils.UnmarshalECDSASignature reads the first two
  // INTEGERs of the SEQUENCE (R, S > 0, else setup fails)
  if (t3[2].ce == t3[2].cs || b[t3[2].cs] != 0) unsup();
  const size_t ss = t3[2].cs + 1, se = t3[2].ce;
  T sq;
  try {
    sq = tlv(b, ss, se);
  } catch (const XErr &) {
    perr();
  }
  if (sq.tag != 0x30) perr();
  const std::vector<T> rs = children(b, sq.cs, sq.ce);
  if (rs.size() < 2 || rs[0].tag != 0x02 || rs[1].tag != 0x02) unsup();
  bool ok = true;
  uint8_t *out[2] = {c.r, c.s};
  for (int q = 0; q < 2; q++) {
    size_t a = rs[q].cs;
    const size_t e = rs[q].ce;
    if (!int_minimal(b, a, e)) perr();
    if (b[a] & 0x80) perr();  // negative: "R/S must be larger than zero"
    if (e - a == 1 && b[a] == 0) perr();  // zero
    if (b[a] == 0) a++;
    if (e - a > 32) {
      ok = false;  // >= 2^256 > n: CheckCRLSignature fails
      continue;
    }
    memset(out[q], 0, 32);
    memcpy(out[q] + 32 - (e - a), b + a, e - a);
  }
  c.rs_ok = ok && lt_n(c.r) && lt_n(c.s);
}
}  // namespace

int parse_crl(const uint8_t *p, size_t n, Crl &out) {
  out = Crl();
  static const char PFX[] = "-----BEGIN X509 CRL";
  static const char FULL[] = "-----BEGIN X509 CRL-----";
  if (n >= sizeof PFX - 1 && memcmp(p, PFX, sizeof PFX - 1) == 0) {
    if (n < sizeof FULL - 1 || memcmp(p, FULL, sizeof FULL - 1) != 0) return X_UNSUP;
    const int rc = pem_decode(p, n, out.der);
    if (rc != X_OK) return rc == X_PARSE ? X_UNSUP : rc;
  } else {
    out.der.assign(p, p + n);
  }
  try {
    parse_crl_der(out);
  } catch (const XErr &e) {
    return e.code;
  }
  return X_OK;
}

int parse_certificate(std::vector<uint8_t> der, Cert &c) {
  c = Cert();
  c.der = std::move(der);
  try {
    parse(c);
  } catch (const XErr &e) {
    return e.code;
  }
  return X_OK;
}

bool strict_sig(const uint8_t *sig, size_t n, uint8_t r[32], uint8_t s[32]) {
  try {
    const T t = tlv(sig, 0, n);
    if (t.tag != 0x30 || t.ce != n) return false;
    const std::vector<T> k = children(sig, t.cs, t.ce);
    if (k.size() != 2 || k[0].tag != 0x02 || k[1].tag != 0x02) return false;
    uint8_t *out[2] = {r, s};
    for (int q = 0; q < 2; q++) {
      size_t a = k[q].cs, e = k[q].ce;
      if (!int_minimal(sig, a, e)) return false;
      if (sig[a] & 0x80) return false;  // negative: outside (0, n)
      if (sig[a] == 0) a++;
      if (e - a > 32) return false;
      memset(out[q], 0, 32);
      memcpy(out[q] + 32 - (e - a), sig + a, e - a);
    }
    return true;
  } catch (const XErr &) {
    return false;
  }
}

static void put_len(std::vector<uint8_t> &o, size_t n) {
  if (n < 128) {
    o.push_back((uint8_t)n);
  } else if (n < 256) {
    o.push_back(0x81);
    o.push_back((uint8_t)n);
  } else if (n < 65536) {
    o.push_back(0x82);
    o.push_back((uint8_t)(n >> 8));
    o.push_back((uint8_t)n);
  } else {
    o.push_back(0x83);
    o.push_back((uint8_t)(n >> 16));
    o.push_back((uint8_t)(n >> 8));
    o.push_back((uint8_t)n);
  }
}

static void put_int(std::vector<uint8_t> &o, const uint8_t v[32]) {
  size_t a = 0;
  while (a < 31 && v[a] == 0) a++;
  const bool pad = v[a] & 0x80;
  o.push_back(0x02);
  put_len(o, 32 - a + pad);
  if (pad) o.push_back(0);
  o.insert(o.end(), v + a, v + 32);
}

std::vector<uint8_t> der_sig(const uint8_t r[32], const uint8_t s[32]) {
  std::vector<uint8_t> body;
  put_int(body, r);
  put_int(body, s);
  std::vector<uint8_t> o{0x30};
  put_len(o, body.size());
  o.insert(o.end(), body.begin(), body.end());
  return o;
}

bool lt_n(const uint8_t v[32]) { return cmp(from_be(v), N) < 0; }

bool is_zero(const uint8_t v[32]) {
  for (int i = 0; i < 32; i++)
    if (v[i]) return false;
  return true;
}

bool to_low_s(uint8_t s[32]) {
  const U256 v = from_be(s);
  if (cmp(v, NH) <= 0) return false;
  U256 r;
  sub(r, N, v);
  to_be(r, s);
  return true;
}

int sanitized_raw(const Cert &c, std::vector<uint8_t> &out) {
  uint8_t r[32], s[32];
  std::vector<uint8_t> sig;
  // (a strict parse with r or s wider than 256 bits or negative: outside the model)
  if (!strict_sig(c.sig(), c.sig_len, r, s) || is_zero(r) || is_zero(s) || !lt_n(r) || !lt_n(s)) return X_UNSUP;
  if (to_low_s(s)) {
    sig = der_sig(r, s);
  } else {
    sig.assign(c.sig(), c.sig() + c.sig_len);
  }
  std::vector<uint8_t> body(c.tbs(), c.tbs() + c.tbs_len);
  body.insert(body.end(), ALG_ECDSA_SHA256, ALG_ECDSA_SHA256 + sizeof ALG_ECDSA_SHA256);
  body.push_back(0x03);
  put_len(body, sig.size() + 1);
  body.push_back(0);
  body.insert(body.end(), sig.begin(), sig.end());
  out.assign(1, 0x30);
  put_len(out, body.size());
  out.insert(out.end(), body.begin(), body.end());
  return X_OK;
}

bool p384_on_curve(const uint8_t xb[48], const uint8_t yb[48]) {  // both < p, y^2 = x^3 - 3x + b
  uint32_t x[p384::NL], y[p384::NL];
  for (int k = 0; k < p384::NL; k++) {
    const uint8_t *q = xb + 4 * (p384::NL - 1 - k), *r = yb + 4 * (p384::NL - 1 - k);
    x[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    y[k] = ((uint32_t)r[0] << 24) | ((uint32_t)r[1] << 16) | ((uint32_t)r[2] << 8) | (uint32_t)r[3];
  }
  return p384::on_curve(x, y);
}

bool p256_on_curve(const uint8_t xb[32], const uint8_t yb[32]) {
  const U256 x = from_be(xb), y = from_be(yb);
  if (cmp(x, P) >= 0 || cmp(y, P) >= 0) return false;
  const U256 y2 = mulm(y, y);
  const U256 x3 = mulm(mulm(x, x), x);
  const U256 t3 = addm(addm(x, x), x);
  const U256 rhs = addm(subm(x3, t3), Bc);
  return cmp(y2, rhs) == 0;
}

}  // namespace fgvx

// ---- CPU probe for the parity tests (tests/test_x509_parity.py) and the sanitizer harness: a
// PEM certificate through pem_decode -> parse_certificate -> sanitized_raw, the fields the MSP
// path reads as one JSON object (no GPU call)
#include <stdio.h>

#include "sha256_host.h"

static std::string hex(const uint8_t *p, size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) s[2 * i] = d[p[i] >> 4], s[2 * i + 1] = d[p[i] & 15];
  return s;
}

extern "C" int fgv_x509_probe(const uint8_t *pem, size_t n, char *out, size_t cap) {
  using namespace fgvx;
  std::vector<uint8_t> der;
  std::string j;
  int st = pem_decode(pem, n, der);
  if (st != X_OK) {
    j = "{\"stage\":\"pem\",\"status\":" + std::to_string(st) + "}";
  } else {
    Cert c;
    st = parse_certificate(der, c);
    if (st != X_OK) {
      j = "{\"stage\":\"parse\",\"status\":" + std::to_string(st) + "}";
    } else {
      uint8_t h[32];
      std::vector<uint8_t> raw2;
      const int rs = sanitized_raw(c, raw2);
      j = "{\"stage\":\"ok\",\"status\":0,\"key\":" + std::to_string(c.key) + ",\"version\":" +
          std::to_string(c.version) + ",\"is_ca\":" + std::to_string(c.is_ca) + ",\"bc_valid\":" +
          std::to_string(c.bc_valid) + ",\"path_len\":" + std::to_string(c.path_len) + ",\"has_ski\":" + std::to_string(c.has_ski) + ",\"key_usage\":" +
          std::to_string(c.key_usage) + ",\"unhandled_critical\":" + std::to_string(c.unhandled_critical) +
          ",\"not_before\":" + std::to_string(c.not_before) + ",\"not_after\":" + std::to_string(c.not_after) +
          ",\"pub\":\"" + (c.key == XK_P256 ? hex(c.pub, 64) : c.key == XK_P384 ? hex(c.pub384, 96) : std::string()) + "\"";
      fgvsha::sha256(c.tbs(), c.tbs_len, h);
      j += ",\"tbs\":\"" + hex(h, 32) + "\"";
      fgvsha::sha256(c.der.data() + c.issuer_off, c.issuer_len, h);
      j += ",\"issuer\":\"" + hex(h, 32) + "\"";
      fgvsha::sha256(c.der.data() + c.subject_off, c.subject_len, h);
      j += ",\"subject\":\"" + hex(h, 32) + "\"";
      j += ",\"sig\":\"" + hex(c.sig(), c.sig_len) + "\"";
      j += ",\"raw2_status\":" + std::to_string(rs);
      if (rs == X_OK) {
        fgvsha::sha256(raw2.data(), raw2.size(), h);
        j += ",\"raw2\":\"" + hex(h, 32) + "\"";
      }
      j += ",\"ous\":[";
      for (size_t i = 0; i < c.ous.size(); i++) j += (i ? ",\"" : "\"") + hex((const uint8_t *)c.ous[i].data(), c.ous[i].size()) + "\"";
      j += "]}";
    }
  }
  if (j.size() + 1 > cap) return -1;
  memcpy(out, j.c_str(), j.size() + 1);
  return (int)j.size();
}
