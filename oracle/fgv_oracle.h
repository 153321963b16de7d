/*
 * fgv_oracle.h -- CPU restatement (TEST INFRASTRUCTURE ONLY) of the crypto leg of
 * Fabric's committer hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path (fabric_amd/libfgv.so)
 * never links or calls it.
 *
 * What it restates (reference file:line under /root/reference):
 *   - SHA-256 digest of a message          bccsp/sw/hash.go:29-33, msp/identities.go:179
 *   - Go encoding/asn1 DER decode of an ECDSA signature (Go 1.21.9 rules)
 *                                          fabric-lib-go bccsp/utils/ecdsa.go:41-65
 *   - low-S rule  s <= n>>1                bccsp/utils/ecdsa.go:82-89, bccsp/sw/ecdsa.go:41-57
 *   - crypto/ecdsa.Verify (Go 1.21.9 verifyNISTEC, external stdlib; algorithm restated
 *     from SEC 1 v2 s4.1.4): r,s in [1,n-1], e = H mod n, w = s^-1,
 *     R = (e*w)G + (r*w)Q, R != inf, x_R mod n == r
 *   - bccsp CSP.Verify empty-argument checks  bccsp/sw/impl.go:247-270
 *
 * Status bytes (shared with include/fgv.h):
 *   0 valid, 1 equation false / R at infinity, 2 DER decode error (incl. r<=0, s<=0),
 *   3 high-S, 4 r or s out of range (>= n), 5 public key not a P-256 point,
 *   6 empty signature or digest.
 * Only 0 means "valid"; the reference maps every other outcome to an error.
 */
#ifndef FGV_ORACLE_H
#define FGV_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

void oracle_sha256(const uint8_t *msg, size_t len, uint8_t out[32]);

/* Go-rule DER decode.  On success returns 0 and writes r,s as 32-byte big-endian
 * values (r_big/s_big set to 1 if the integer does not fit in 256 bits).
 * Returns 2 on any decode error, including r<=0 or s<=0. */
int oracle_der_decode(const uint8_t *sig, size_t len, uint8_t r[32], uint8_t s[32],
                      int *r_big, int *s_big);

/* Full bccsp Verify(pk, sig, digest) with Go semantics, own bignum arithmetic. */
int oracle_p256_verify_der(const uint8_t qx[32], const uint8_t qy[32], const uint8_t *sig,
                           size_t sig_len, const uint8_t *digest, size_t digest_len);

/* Equation-only check on already-decoded (r,s) (no low-S rule). */
int oracle_p256_verify_rs(const uint8_t qx[32], const uint8_t qy[32], const uint8_t r[32],
                          const uint8_t s[32], const uint8_t digest[32]);

/* Same contract as oracle_p256_verify_der, but the group arithmetic is OpenSSL's
 * (independent cross-check and the fast CPU baseline). */
int oracle_p256_verify_der_ossl(const uint8_t qx[32], const uint8_t qy[32], const uint8_t *sig,
                                size_t sig_len, const uint8_t *digest, size_t digest_len);

/* identity.Verify(msg, sig) = SHA-256(msg) then the above, over a batch, on `threads`
 * host threads (CPU baseline).  use_ossl selects the arithmetic. */
void oracle_verify_msgs_batch(const uint8_t *keys /* n*64: qx||qy */, const uint8_t *msg_buf,
                              const uint64_t *msg_off, const uint32_t *msg_len,
                              const uint8_t *sig_buf, const uint64_t *sig_off,
                              const uint32_t *sig_len, size_t n, uint8_t *status, int threads,
                              int use_ossl);

/* Scalar mult helper for tests: out = k*G affine (32B BE x||y); returns 0 or 1 if inf. */
int oracle_p256_base_mult(const uint8_t k[32], uint8_t out_x[32], uint8_t out_y[32]);

/* key parsed once (oracle_p256_key_new), verified against many times (cpu_validator.c) */
/* bccsp Verify for a P-384 key: Go-rule DER (48-byte integers), the P-384 half order, then
 * Go ecdsa.Verify's rules over OpenSSL's secp384r1 arithmetic; the same status bytes. */
int oracle_p384_verify_der(const uint8_t qx[48], const uint8_t qy[48], const uint8_t *sig, size_t sig_len,
                           const uint8_t *digest, size_t digest_len);
void *oracle_p256_key_new(const uint8_t qx[32], const uint8_t qy[32]);
void oracle_p256_key_free(void *key);
int oracle_p256_verify_der_key(void *key, const uint8_t *sig, size_t sig_len, const uint8_t *digest,
                               size_t digest_len);

#ifdef __cplusplus
}
#endif
#endif
