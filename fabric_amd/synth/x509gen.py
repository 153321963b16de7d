"""X.509 certificates in the shapes a Fabric CA / cryptogen issues -- and deliberate deviations
from them -- for the MSP cache-miss tests (input generation, not the product path).  DER is
assembled here field by field so a test can set each one (OUs, SKI, key usage, validity,
critical extensions, SAN, high-S CA signatures); the ECDSA signatures come from OpenSSL
(fgv_synth.c synth_sign_rs)."""
import base64
import hashlib

from . import Key, der_encode, sign_rs

OID_EC, OID_P256 = "2a8648ce3d0201", "2a8648ce3d030107"
OID_CN, OID_O, OID_OU = "550403", "55040a", "55040b"
ALG = bytes.fromhex("300a06082a8648ce3d040302")


def der_len(n):
    if n < 128:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag, body):
    return bytes([tag]) + der_len(len(body)) + body


def seq(*xs):
    return tlv(0x30, b"".join(xs))


def oid(h):
    return tlv(0x06, bytes.fromhex(h))


def integer(v):
    return tlv(0x02, v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big"))


def name(cn, org="Org1", ous=(), string_tag=0x0C):
    rdns = [tlv(0x31, seq(oid(OID_O), tlv(string_tag, org.encode())))]
    rdns += [tlv(0x31, seq(oid(OID_OU), tlv(string_tag, o.encode()))) for o in ous]
    rdns.append(tlv(0x31, seq(oid(OID_CN), tlv(string_tag, cn.encode()))))
    return seq(*rdns)


def ext(oid_hex, value, critical=False):
    return seq(oid(oid_hex), *([tlv(0x01, b"\xff")] if critical else []), tlv(0x04, value))


def ski(key):
    return ext("551d0e", tlv(0x04, hashlib.sha256(key.pub).digest()[:20]))


def basic_constraints(ca, critical=True, path_len=None):
    body = (tlv(0x01, b"\xff") if ca else b"") + (integer(path_len) if path_len is not None else b"")
    return ext("551d13", seq(body) if body else seq(), critical)


def key_usage(bits, critical=True):
    """bits: KeyUsage bit numbers (0 digitalSignature ... 5 keyCertSign)"""
    v = 0
    for b in bits:
        v |= 0x80 >> b if b < 8 else 0
    return ext("551d0f", tlv(0x03, b"\x00" + bytes([v])), critical)


def san_dns(*names):
    return ext("551d11", seq(*[tlv(0x82, n.encode()) for n in names]))


def cert(subject_key: Key, issuer_key: Key, subject, issuer, serial=1, not_before="240101000000Z",
         not_after="340101000000Z", extensions=(), high_s=False, spki=None):
    """-> PEM bytes; subject / issuer: name(...) DER; extensions: ext(...) DER list"""
    if spki is None:
        spki = seq(seq(oid(OID_EC), oid(OID_P256)), tlv(0x03, b"\x00\x04" + subject_key.qx + subject_key.qy))
    body = tlv(0xA0, integer(2)) + integer(serial) + ALG + issuer + \
        seq(tlv(0x17, not_before.encode()), tlv(0x17, not_after.encode())) + subject + spki
    if extensions:
        body += tlv(0xA3, seq(*extensions))
    tbs = tlv(0x30, body)
    r, s = sign_rs(issuer_key, hashlib.sha256(tbs).digest(), high_s)
    der = seq(tbs, ALG, tlv(0x03, b"\x00" + der_encode(r, s)))
    b64 = base64.encodebytes(der)
    return b"-----BEGIN CERTIFICATE-----\n" + b64 + b"-----END CERTIFICATE-----\n"


def ca_cert(key: Key, cn="ca.org1", org="Org1", with_ski=True, usage=(0, 5, 6), serial=1, issuer_key=None,
            issuer_cn=None, path_len=None):
    """a root CA (self-signed), or an intermediate when issuer_key / issuer_cn are given"""
    nm = name(cn, org)
    exts = [key_usage(usage), basic_constraints(True, path_len=path_len)] + ([ski(key)] if with_ski else [])
    return cert(key, issuer_key or key, nm, name(issuer_cn, org) if issuer_cn else nm, serial=serial, extensions=exts)


def crl(signer_key: Key, issuer_cn, aki_key: Key, serials, org="Org1", high_s=False, this_update="240601000000Z"):
    """-> PEM "X509 CRL": v2 CertificateList revoking `serials`, signed (ecdsa-with-SHA256) by
    signer_key, its AuthorityKeyIdentifier the SKI x509gen gives aki_key's certificate"""
    revoked = seq(*[seq(integer(v), tlv(0x17, this_update.encode())) for v in serials]) if serials else b""
    aki = ext("551d23", seq(tlv(0x80, hashlib.sha256(aki_key.pub).digest()[:20])))
    tbs = seq(integer(1), ALG, name(issuer_cn, org), tlv(0x17, this_update.encode()),
              tlv(0x17, b"340101000000Z"), revoked, tlv(0xA0, seq(aki)))
    r, s = sign_rs(signer_key, hashlib.sha256(tbs).digest(), high_s)
    der = seq(tbs, ALG, tlv(0x03, b"\x00" + der_encode(r, s)))
    return b"-----BEGIN X509 CRL-----\n" + base64.encodebytes(der) + b"-----END X509 CRL-----\n"
