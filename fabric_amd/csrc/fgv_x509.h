// fgv_x509.h -- the X.509 subset of the MSP identity path on a cache miss (host code of
// libfgv.so): PEM, certificate DER parse, signature re-marshalling (sanitizeCert), P-256 point
// check.  Restates Go 1.21 crypto/x509 + encoding/asn1 for the shapes Fabric CAs and cryptogen
// issue (v3, ECDSA P-256 keys, ecdsa-with-SHA256, the usual extensions); any other shape is
// reported as outside the model (the caller returns FGV_EUNSUPPORTED -- the reference decides).
// The same rules as oracle/x509.py, which the tests compare it with.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

namespace fgvx {

enum : int { X_OK = 0, X_PARSE = 1, X_UNSUP = 2 };  // parse error = Go's ParseCertificate fails
enum : int { XK_P256 = 1, XK_P384 = 2, XK_OTHER = 3, XK_UNDESERIALIZABLE = 4 };  // = FGV_KEY_*

struct Cert {
  std::vector<uint8_t> der;                 // the certificate bytes (PEM decoded)
  size_t tbs_off = 0, tbs_len = 0;          // RawTBSCertificate within der
  size_t sig_off = 0, sig_len = 0;          // signature value (BIT STRING content after 0x00)
  size_t issuer_off = 0, issuer_len = 0;    // RawIssuer (the whole Name TLV)
  size_t subject_off = 0, subject_len = 0;  // RawSubject
  int64_t not_before = 0, not_after = 0;    // seconds since the epoch (UTC)
  std::vector<std::string> ous;             // subject OrganizationalUnit values, in order
  int key = XK_OTHER;                       // subject public key class
  uint8_t pub[64] = {};                     // P-256 X || Y
  uint8_t pub384[96] = {};                  // P-384 X || Y (XK_P384, round 6)
  bool is_ca = false, bc_valid = false, has_ski = false, unhandled_critical = false;
  int64_t path_len = -1;                    // basicConstraints MaxPathLen (-1: none)
  uint32_t key_usage = 0;                   // Go KeyUsage bits
  int version = 0;                          // 1..3
  size_t serial_off = 0, serial_len = 0;    // serialNumber INTEGER content (minimal)
  size_t ski_off = 0, ski_len = 0;          // subjectKeyIdentifier OCTET STRING content (has_ski)
  const uint8_t *tbs() const { return der.data() + tbs_off; }
  const uint8_t *sig() const { return der.data() + sig_off; }
  bool same_issuer_as_subject_of(const Cert &ca) const {
    return issuer_len == ca.subject_len &&
           std::equal(der.begin() + issuer_off, der.begin() + issuer_off + issuer_len, ca.der.begin() + ca.subject_off);
  }
};

// encoding/pem Decode of the first block: X_OK (der filled), X_PARSE (no block / bad base64),
// X_UNSUP (PEM headers)
int pem_decode(const uint8_t *p, size_t n, std::vector<uint8_t> &der);
// x509.ParseCertificate subset: X_OK, X_PARSE, X_UNSUP
int parse_certificate(std::vector<uint8_t> der, Cert &c);
// crypto/ecdsa VerifyASN1's strict SEQUENCE{INTEGER r, INTEGER s}: r, s as 32-byte big-endian
// (false: malformed, negative or wider than 256 bits -- the verify fails)
bool strict_sig(const uint8_t *sig, size_t n, uint8_t r[32], uint8_t s[32]);
// DER of ECDSA-Sig-Value{r, s} (minimal INTEGERs)
std::vector<uint8_t> der_sig(const uint8_t r[32], const uint8_t s[32]);
// s -> n - s when s > n/2 (returns true when it changed s); s must be < n
bool to_low_s(uint8_t s[32]);
bool lt_n(const uint8_t v[32]);
bool is_zero(const uint8_t v[32]);
// sanitizeECDSASignedCert: the certificate re-marshalled with a low-S signature (X_UNSUP when the
// signature is not strict DER: Go's re-marshal would differ from what this restates)
int sanitized_raw(const Cert &c, std::vector<uint8_t> &out);
// A certificate revocation list of an MSP (setupCRLs, mspimplsetup.go:215-245; the modelled
// shape of oracle/crl.py): the TBSCertList bytes, its AuthorityKeyIdentifier keyIdentifier, the
// revoked serial numbers (minimal INTEGER contents), the re-marshalled ECDSA (r, s)
struct Crl {
  std::vector<uint8_t> der;
  size_t tbs_off = 0, tbs_len = 0;
  std::vector<uint8_t> aki;
  std::vector<std::vector<uint8_t>> serials;
  uint8_t r[32] = {}, s[32] = {};
  bool rs_ok = false;  // 0 < r, s < n (else CheckCRLSignature fails)
  bool revokes(const Cert &c) const {
    for (const auto &v : serials)
      if (v.size() == c.serial_len && std::equal(v.begin(), v.end(), c.der.begin() + c.serial_off)) return true;
    return false;
  }
};
// x509.ParseCRL (+ setupCRLs' signature re-marshal): X_OK, X_PARSE (Go fails: the MSP does not
// set up), X_UNSUP (outside the modelled shape)
int parse_crl(const uint8_t *p, size_t n, Crl &out);
// P-256 affine point on the curve (x, y < p and y^2 = x^3 - 3x + b)
bool p256_on_curve(const uint8_t x[32], const uint8_t y[32]);
bool p384_on_curve(const uint8_t x[48], const uint8_t y[48]);

}  // namespace fgvx
