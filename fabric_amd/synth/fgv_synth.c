/*
 * fgv_synth.c -- synthetic-workload helper (NOT the product path, NOT the oracle).
 * OpenSSL 3 supplies keys, X.509 certificates and ECDSA signatures for the synthetic
 * blocks used by tests and bench.py, so every signature the GPU engine checks was
 * produced by an implementation independent of both the engine and the oracle.
 * Fabric signers always emit low-S signatures (bccsp/sw/ecdsa.go signECDSA -> ToLowS);
 * mode 1 deliberately produces the high-S twin (n - s) for fault injection.
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/pem.h>
#include <openssl/sha.h>
#include <openssl/x509.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

static EC_GROUP *G_GROUP;
static pthread_once_t G_ONCE = PTHREAD_ONCE_INIT;
static void group_init(void) { G_GROUP = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1); }
static EC_GROUP *group(void) {
  pthread_once(&G_ONCE, group_init);
  return G_GROUP;
}
#define GRP group()

static EC_KEY *key_from_priv(const uint8_t priv[32]) {
  EC_KEY *k = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
  BIGNUM *d = BN_bin2bn(priv, 32, NULL);
  EC_POINT *pub = EC_POINT_new(GRP);
  EC_POINT_mul(GRP, pub, d, NULL, NULL, NULL);
  EC_KEY_set_private_key(k, d);
  EC_KEY_set_public_key(k, pub);
  EC_POINT_free(pub);
  BN_free(d);
  return k;
}

/* priv = SHA-256("fgv-synth" || seed || idx || ctr) reduced into [1, n-1] */
int synth_keygen(uint64_t seed, uint32_t idx, uint8_t priv[32], uint8_t qx[32], uint8_t qy[32]) {
  const BIGNUM *n = EC_GROUP_get0_order(GRP);
  for (uint32_t ctr = 0;; ctr++) {
    uint8_t buf[9 + 8 + 4 + 4];
    memcpy(buf, "fgv-synth", 9);
    memcpy(buf + 9, &seed, 8);
    memcpy(buf + 17, &idx, 4);
    memcpy(buf + 21, &ctr, 4);
    SHA256(buf, sizeof buf, priv);
    BIGNUM *d = BN_bin2bn(priv, 32, NULL);
    int ok = !BN_is_zero(d) && BN_cmp(d, n) < 0;
    BN_free(d);
    if (ok) break;
  }
  EC_KEY *k = key_from_priv(priv);
  BIGNUM *x = BN_new(), *y = BN_new();
  EC_POINT_get_affine_coordinates(GRP, EC_KEY_get0_public_key(k), x, y, NULL);
  BN_bn2binpad(x, qx, 32);
  BN_bn2binpad(y, qy, 32);
  BN_free(x);
  BN_free(y);
  EC_KEY_free(k);
  return 0;
}

/* minimal DER INTEGER for a non-negative big-endian 32-byte value */
static size_t der_int(uint8_t *out, const uint8_t v[32]) {
  size_t i = 0;
  while (i < 31 && v[i] == 0) i++;
  size_t len = 32 - i;
  int pad = (v[i] & 0x80) != 0;
  out[0] = 0x02;
  out[1] = (uint8_t)(len + pad);
  size_t o = 2;
  if (pad) out[o++] = 0;
  memcpy(out + o, v + i, len);
  return o + len;
}

size_t synth_der_encode(const uint8_t r[32], const uint8_t s[32], uint8_t *out) {
  uint8_t tmp[80];
  size_t a = der_int(tmp, r);
  size_t b = der_int(tmp + a, s);
  out[0] = 0x30;
  out[1] = (uint8_t)(a + b);
  memcpy(out + 2, tmp, a + b);
  return 2 + a + b;
}

/* raw (r,s) signature; mode 0 = low-S (Fabric), 1 = high-S twin */
int synth_sign_rs(const uint8_t priv[32], const uint8_t digest[32], int mode, uint8_t r[32],
                  uint8_t s[32]) {
  EC_KEY *k = key_from_priv(priv);
  ECDSA_SIG *sig = ECDSA_do_sign(digest, 32, k);
  const BIGNUM *br, *bs;
  ECDSA_SIG_get0(sig, &br, &bs);
  const BIGNUM *n = EC_GROUP_get0_order(GRP);
  BIGNUM *half = BN_dup(n);
  BN_rshift1(half, half);
  BIGNUM *ss = BN_dup(bs);
  int high = BN_cmp(ss, half) > 0;
  if ((mode == 0 && high) || (mode == 1 && !high)) BN_sub(ss, n, ss);
  BN_bn2binpad(br, r, 32);
  BN_bn2binpad(ss, s, 32);
  BN_free(ss);
  BN_free(half);
  ECDSA_SIG_free(sig);
  EC_KEY_free(k);
  return 0;
}

typedef struct {
  const uint8_t *privs, *digests;
  uint8_t *der;
  uint32_t *der_len;
  size_t lo, hi, stride;
  int mode;
} sjob;

static void *sign_worker(void *a) {
  sjob *j = (sjob *)a;
  for (size_t i = j->lo; i < j->hi; i++) {
    uint8_t r[32], s[32];
    synth_sign_rs(j->privs + 32 * i, j->digests + 32 * i, j->mode, r, s);
    j->der_len[i] = (uint32_t)synth_der_encode(r, s, j->der + j->stride * i);
  }
  return NULL;
}

/* batch sign: der_out has `stride` (>= 72) bytes per item */
int synth_sign_batch(const uint8_t *privs, const uint8_t *digests, size_t n, uint8_t *der_out,
                     uint32_t *der_len, size_t stride, int mode, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t tid[64];
  sjob jobs[64];
  size_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    size_t lo = t * per < n ? t * per : n, hi = (t + 1) * per < n ? (t + 1) * per : n;
    jobs[t] = (sjob){privs, digests, der_out, der_len, lo, hi, stride, mode};
    pthread_create(&tid[t], NULL, sign_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  return 0;
}

/* X.509 v3 certificate for subject key, signed by issuer key (ecdsa-with-SHA256), PEM out.
 * Returns PEM length or -1. */
int synth_make_cert(const uint8_t subj_priv[32], const uint8_t issuer_priv[32], const char *cn,
                    const char *org, const char *issuer_cn, int is_ca, long serial, char *pem_out,
                    size_t cap) {
  EC_KEY *sk = key_from_priv(subj_priv), *ik = key_from_priv(issuer_priv);
  EVP_PKEY *spk = EVP_PKEY_new(), *ipk = EVP_PKEY_new();
  EVP_PKEY_assign_EC_KEY(spk, sk);
  EVP_PKEY_assign_EC_KEY(ipk, ik);
  X509 *x = X509_new();
  X509_set_version(x, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(x), serial);
  ASN1_TIME_set_string(X509_getm_notBefore(x), "20240101000000Z");
  ASN1_TIME_set_string(X509_getm_notAfter(x), "20340101000000Z");
  X509_NAME *sn = X509_NAME_new(), *in = X509_NAME_new();
  X509_NAME_add_entry_by_txt(sn, "O", MBSTRING_ASC, (const unsigned char *)org, -1, -1, 0);
  X509_NAME_add_entry_by_txt(sn, "CN", MBSTRING_ASC, (const unsigned char *)cn, -1, -1, 0);
  X509_NAME_add_entry_by_txt(in, "O", MBSTRING_ASC, (const unsigned char *)org, -1, -1, 0);
  X509_NAME_add_entry_by_txt(in, "CN", MBSTRING_ASC, (const unsigned char *)issuer_cn, -1, -1, 0);
  X509_set_subject_name(x, sn);
  X509_set_issuer_name(x, in);
  X509_set_pubkey(x, spk);
  if (is_ca) {
    X509V3_CTX ctx;
    X509V3_set_ctx_nodb(&ctx);
    X509V3_set_ctx(&ctx, x, x, NULL, NULL, 0);
    X509_EXTENSION *e = X509V3_EXT_conf_nid(NULL, &ctx, NID_basic_constraints, "critical,CA:TRUE");
    X509_add_ext(x, e, -1);
    X509_EXTENSION_free(e);
  }
  X509_sign(x, ipk, EVP_sha256());
  BIO *b = BIO_new(BIO_s_mem());
  PEM_write_bio_X509(b, x);
  char *data;
  long len = BIO_get_mem_data(b, &data);
  int ret = -1;
  if (len >= 0 && (size_t)len < cap) {
    memcpy(pem_out, data, len);
    pem_out[len] = 0;
    ret = (int)len;
  }
  BIO_free(b);
  X509_NAME_free(sn);
  X509_NAME_free(in);
  X509_free(x);
  EVP_PKEY_free(spk);
  EVP_PKEY_free(ipk);
  return ret;
}

/* ---------------------------------------------------------------- Ed25519 (config C5)
 * Fabric v3-style Ed25519 identities.  The reference snapshot's BCCSP x509 key importer
 * accepts only ECDSA/RSA keys, so these identities fail DeserializeIdentity;
 * the generator still produces real RFC 8032 signatures so the blocks are well formed. */
static EVP_PKEY *ed_from_priv(const uint8_t priv[32]) {
  return EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, priv, 32);
}

/* priv = SHA-256("fgv-ed25519" || seed || idx); pub = the RFC 8032 public key */
int synth_ed25519_keygen(uint64_t seed, uint32_t idx, uint8_t priv[32], uint8_t pub[32]) {
  uint8_t buf[11 + 8 + 4];
  memcpy(buf, "fgv-ed25519", 11);
  memcpy(buf + 11, &seed, 8);
  memcpy(buf + 19, &idx, 4);
  SHA256(buf, sizeof buf, priv);
  EVP_PKEY *k = ed_from_priv(priv);
  if (!k) return -1;
  size_t n = 32;
  int ok = EVP_PKEY_get_raw_public_key(k, pub, &n) == 1 && n == 32;
  EVP_PKEY_free(k);
  return ok ? 0 : -1;
}

/* n messages (concatenated, offsets/lengths) signed with privs[i] (32 B each); 64-byte
 * signatures into sig_out[i*64] */
int synth_ed25519_sign_batch(const uint8_t *privs, const uint8_t *msgs, const uint64_t *off,
                             const uint32_t *len, size_t n, uint8_t *sig_out) {
  for (size_t i = 0; i < n; i++) {
    EVP_PKEY *k = ed_from_priv(privs + 32 * i);
    EVP_MD_CTX *c = EVP_MD_CTX_new();
    size_t sl = 64;
    int ok = k && c && EVP_DigestSignInit(c, NULL, NULL, NULL, k) == 1 &&
             EVP_DigestSign(c, sig_out + 64 * i, &sl, msgs + off[i], len[i]) == 1 && sl == 64;
    EVP_MD_CTX_free(c);
    EVP_PKEY_free(k);
    if (!ok) return -1;
  }
  return 0;
}

/* X.509 certificate for an Ed25519 subject key, issued (ecdsa-with-SHA256) by a P-256 CA */
int synth_make_cert_ed25519(const uint8_t subj_ed_priv[32], const uint8_t issuer_priv[32], const char *cn,
                            const char *org, const char *issuer_cn, long serial, char *pem_out, size_t cap) {
  EVP_PKEY *spk = ed_from_priv(subj_ed_priv), *ipk = EVP_PKEY_new();
  EVP_PKEY_assign_EC_KEY(ipk, key_from_priv(issuer_priv));
  X509 *x = X509_new();
  X509_set_version(x, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(x), serial);
  ASN1_TIME_set_string(X509_getm_notBefore(x), "20240101000000Z");
  ASN1_TIME_set_string(X509_getm_notAfter(x), "20340101000000Z");
  X509_NAME *sn = X509_NAME_new(), *in = X509_NAME_new();
  X509_NAME_add_entry_by_txt(sn, "O", MBSTRING_ASC, (const unsigned char *)org, -1, -1, 0);
  X509_NAME_add_entry_by_txt(sn, "CN", MBSTRING_ASC, (const unsigned char *)cn, -1, -1, 0);
  X509_NAME_add_entry_by_txt(in, "O", MBSTRING_ASC, (const unsigned char *)org, -1, -1, 0);
  X509_NAME_add_entry_by_txt(in, "CN", MBSTRING_ASC, (const unsigned char *)issuer_cn, -1, -1, 0);
  X509_set_subject_name(x, sn);
  X509_set_issuer_name(x, in);
  X509_set_pubkey(x, spk);
  X509_sign(x, ipk, EVP_sha256());
  BIO *b = BIO_new(BIO_s_mem());
  PEM_write_bio_X509(b, x);
  char *data;
  long len = BIO_get_mem_data(b, &data);
  int ret = -1;
  if (len >= 0 && (size_t)len < cap) {
    memcpy(pem_out, data, len);
    pem_out[len] = 0;
    ret = (int)len;
  }
  BIO_free(b);
  X509_NAME_free(sn);
  X509_NAME_free(in);
  X509_free(x);
  EVP_PKEY_free(spk);
  EVP_PKEY_free(ipk);
  return ret;
}

/* ---------------------------------------------------------------- P-384 identities
 * Keys, signatures (over a 32-byte SHA-256 / SHA3-256 digest, as identity.Verify hashes with the
 * MSP's family; Fabric signers emit low-S) and certificates issued by a P-256 CA. */
static EC_GROUP *G384;
static pthread_once_t G384_ONCE = PTHREAD_ONCE_INIT;
static void g384_init(void) { G384 = EC_GROUP_new_by_curve_name(NID_secp384r1); }
static EC_GROUP *g384(void) {
  pthread_once(&G384_ONCE, g384_init);
  return G384;
}
static EC_KEY *key384_from_priv(const uint8_t priv[48]) {
  EC_KEY *k = EC_KEY_new_by_curve_name(NID_secp384r1);
  BIGNUM *d = BN_bin2bn(priv, 48, NULL);
  EC_POINT *pub = EC_POINT_new(g384());
  EC_POINT_mul(g384(), pub, d, NULL, NULL, NULL);
  EC_KEY_set_private_key(k, d);
  EC_KEY_set_public_key(k, pub);
  EC_POINT_free(pub);
  BN_free(d);
  return k;
}
/* priv = SHA-384("fgv-p384" || seed || idx || ctr) in [1, n-1] */
int synth_p384_keygen(uint64_t seed, uint32_t idx, uint8_t priv[48], uint8_t qx[48], uint8_t qy[48]) {
  const BIGNUM *n = EC_GROUP_get0_order(g384());
  for (uint32_t ctr = 0;; ctr++) {
    uint8_t buf[8 + 8 + 4 + 4];
    memcpy(buf, "fgv-p384", 8);
    memcpy(buf + 8, &seed, 8);
    memcpy(buf + 16, &idx, 4);
    memcpy(buf + 20, &ctr, 4);
    SHA384(buf, sizeof buf, priv);
    BIGNUM *d = BN_bin2bn(priv, 48, NULL);
    int ok = !BN_is_zero(d) && BN_cmp(d, n) < 0;
    BN_free(d);
    if (ok) break;
  }
  EC_KEY *k = key384_from_priv(priv);
  BIGNUM *x = BN_new(), *y = BN_new();
  EC_POINT_get_affine_coordinates(g384(), EC_KEY_get0_public_key(k), x, y, NULL);
  BN_bn2binpad(x, qx, 48);
  BN_bn2binpad(y, qy, 48);
  BN_free(x);
  BN_free(y);
  EC_KEY_free(k);
  return 0;
}
/* raw (r, s), 48 bytes each; mode 0 low-S, 1 the high-S twin */
int synth_p384_sign_rs(const uint8_t priv[48], const uint8_t *digest, size_t dlen, int mode, uint8_t r[48], uint8_t s[48]) {
  EC_KEY *k = key384_from_priv(priv);
  ECDSA_SIG *sig = ECDSA_do_sign(digest, (int)dlen, k);
  const BIGNUM *br, *bs;
  ECDSA_SIG_get0(sig, &br, &bs);
  const BIGNUM *n = EC_GROUP_get0_order(g384());
  BIGNUM *half = BN_dup(n);
  BN_rshift1(half, half);
  BIGNUM *ss = BN_dup(bs);
  int high = BN_cmp(ss, half) > 0;
  if ((mode == 0 && high) || (mode == 1 && !high)) BN_sub(ss, n, ss);
  BN_bn2binpad(br, r, 48);
  BN_bn2binpad(ss, s, 48);
  BN_free(ss);
  BN_free(half);
  ECDSA_SIG_free(sig);
  EC_KEY_free(k);
  return 0;
}
/* X.509 v3 certificate for a P-384 subject key, signed by a P-256 issuer key (ecdsa-with-SHA256) */
int synth_make_cert_p384(const uint8_t subj_priv[48], const uint8_t issuer_priv[32], const char *cn, const char *org,
                         const char *ou, const char *issuer_cn, long serial, char *pem_out, size_t cap) {
  EC_KEY *sk = key384_from_priv(subj_priv), *ik = key_from_priv(issuer_priv);
  EVP_PKEY *spk = EVP_PKEY_new(), *ipk = EVP_PKEY_new();
  EVP_PKEY_assign_EC_KEY(spk, sk);
  EVP_PKEY_assign_EC_KEY(ipk, ik);
  X509 *x = X509_new();
  X509_set_version(x, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(x), serial);
  ASN1_TIME_set_string(X509_getm_notBefore(x), "20240101000000Z");
  ASN1_TIME_set_string(X509_getm_notAfter(x), "20340101000000Z");
  X509_NAME *sn = X509_NAME_new(), *in = X509_NAME_new();
  X509_NAME_add_entry_by_txt(sn, "O", MBSTRING_ASC, (const unsigned char *)org, -1, -1, 0);
  if (ou && *ou) X509_NAME_add_entry_by_txt(sn, "OU", MBSTRING_ASC, (const unsigned char *)ou, -1, -1, 0);
  X509_NAME_add_entry_by_txt(sn, "CN", MBSTRING_ASC, (const unsigned char *)cn, -1, -1, 0);
  X509_NAME_add_entry_by_txt(in, "O", MBSTRING_ASC, (const unsigned char *)org, -1, -1, 0);
  X509_NAME_add_entry_by_txt(in, "CN", MBSTRING_ASC, (const unsigned char *)issuer_cn, -1, -1, 0);
  X509_set_subject_name(x, sn);
  X509_set_issuer_name(x, in);
  X509_set_pubkey(x, spk);
  X509_sign(x, ipk, EVP_sha256());
  BIO *b = BIO_new(BIO_s_mem());
  PEM_write_bio_X509(b, x);
  char *data;
  long len = BIO_get_mem_data(b, &data);
  int ret = -1;
  if (len >= 0 && (size_t)len < cap) {
    memcpy(pem_out, data, len);
    pem_out[len] = 0;
    ret = (int)len;
  }
  BIO_free(b);
  X509_NAME_free(sn);
  X509_NAME_free(in);
  X509_free(x);
  EVP_PKEY_free(spk);
  EVP_PKEY_free(ipk);
  return ret;
}
