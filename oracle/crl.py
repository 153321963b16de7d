"""Restated certificate revocation lists of an MSP (TEST INFRASTRUCTURE ONLY -- the oracle).

The reference (MSP version 1.4.3, Go 1.21):
  mspimplsetup.go:215-245  setupCRLs: x509.ParseCRL of every RevocationList entry (an error fails
                           the MSP's setup); an ECDSA-signed CRL's signature value is re-marshalled
                           from utils.UnmarshalECDSASignature's (R, S) (R, S > 0, else setup fails)
  mspimplvalidate.go:94-140 validateCertAgainstChain: SKI of the certificate's issuing CA
                           (validationChain[1]); for every CRL whose AuthorityKeyIdentifier equals
                           it, a revoked serial equal to the certificate's -- when that CA's
                           CheckCRLSignature accepts the CRL -- makes the certificate revoked
                           (an identity: invalid; an intermediate CA: finalizeSetupCAs fails)
  crypto/x509 ParseCRL -> ParseDERCRL -> encoding/asn1 Unmarshal into pkix.CertificateList
  (TBSCertList{Version optional, Signature, Issuer RDNSequence, ThisUpdate, NextUpdate optional,
  RevokedCertificates optional, Extensions [0] optional}); CheckCRLSignature ->
  CheckSignature(algorithm, TBSCertList.Raw, SignatureValue.RightAlign()) -> ecdsa.VerifyASN1
  (high-S accepted).

Modelled CRL shape (anything else raises v20.Unsupported -- the reference decides): PEM "X509 CRL"
or DER; minimal DER throughout; version absent or a small INTEGER; AlgorithmIdentifiers of an OID
with no or NULL parameters, the outer one ecdsa-with-SHA256; issuer attribute values
PrintableString / UTF8String / IA5String; UTCTime / GeneralizedTime in their "Z" seconds forms;
revoked entries {serial, time[, extensions]}; extensions {OID, [BOOLEAN], OCTET STRING} with exactly
one AuthorityKeyIdentifier holding only a [0] keyIdentifier; a signature BIT STRING without
padding bits whose value is SEQUENCE{INTEGER r, INTEGER s, ...}.
"""
import hashlib

from .v20 import Unsupported
from . import x509 as X

PEM_CRL_PREFIX = b"-----BEGIN X509 CRL"
OID_AKI = bytes.fromhex("551d23")
ALG_ECDSA = {bytes.fromhex(h) for h in ("2a8648ce3d0401", "2a8648ce3d040302", "2a8648ce3d040303", "2a8648ce3d040304")}
ALG_ECDSA_SHA256 = bytes.fromhex("2a8648ce3d040302")


def _alg(b, s, e):
    """AlgorithmIdentifier -> OID bytes (parameters: none or NULL)"""
    k = X.children(b, s, e)
    if not k or k[0][0] != 0x06 or not X.valid_oid(b[k[0][1]:k[0][2]]):
        raise Unsupported("CRL algorithm identifier")
    if len(k) > 2 or (len(k) == 2 and (k[1][0] != 0x05 or k[1][2] != k[1][1])):
        raise Unsupported("CRL algorithm parameters")
    return b[k[0][1]:k[0][2]]


def _name(b, s, e):
    """RDNSequence with attribute values of the modelled string types"""
    for t, cs, ce, _ in X.children(b, s, e):
        if t != 0x31:
            raise Unsupported("CRL issuer RDN")
        for t2, cs2, ce2, _ in X.children(b, cs, ce):
            if t2 != 0x30:
                raise Unsupported("CRL issuer attribute")
            a = X.children(b, cs2, ce2)
            if len(a) != 2 or a[0][0] != 0x06 or not X.valid_oid(b[a[0][1]:a[0][2]]):
                raise Unsupported("CRL issuer attribute")
            if a[1][0] not in (0x13, 0x0C, 0x16):
                raise Unsupported("CRL issuer attribute string type")
            X._string(b, a[1][0], a[1][1], a[1][2])  # (ParseError: asn1.Unmarshal fails)


def _time(b, t, s, e):
    if t not in (0x17, 0x18):
        raise Unsupported("CRL time")
    X._time(b, t, s, e)


def _extensions(b, s, e):
    """[(oid, value bytes)]"""
    out = []
    for t, cs, ce, _ in X.children(b, s, e):
        if t != 0x30:
            raise Unsupported("CRL extension")
        k = X.children(b, cs, ce)
        if len(k) == 3 and k[1][0] == 0x01:
            if k[1][2] - k[1][1] != 1:
                raise X.ParseError("bad boolean")
            if b[k[1][1]] not in (0x00, 0xFF):
                raise X.ParseError("bad boolean")  # (asn1 parseBool)
            k = [k[0], k[2]]
        if len(k) != 2 or k[0][0] != 0x06 or k[1][0] != 0x04 or not X.valid_oid(b[k[0][1]:k[0][2]]):
            raise Unsupported("CRL extension shape")
        out.append((b[k[0][1]:k[0][2]], b[k[1][1]:k[1][2]]))
    return out


def parse_crl(data):
    """x509.ParseCRL + setupCRLs' signature re-marshal -> dict(tbs, aki, serials, alg, r, s);
    ParseError where Go fails (the MSP does not set up), Unsupported outside the model"""
    der = data
    if data.startswith(PEM_CRL_PREFIX):
        d = X.pem_decode(data)
        if d is None or not data.startswith(b"-----BEGIN X509 CRL-----"):
            raise Unsupported("CRL PEM type")
        der = d
    t, s, e = X.tlv(der, 0)
    if t != 0x30 or e != len(der):
        raise X.ParseError("CRL: not one SEQUENCE")
    top = X.children(der, s, e)
    if len(top) != 3 or top[0][0] != 0x30 or top[1][0] != 0x30 or top[2][0] != 0x03:
        raise Unsupported("CRL structure")
    tbs = der[top[0][3]:top[0][2]]
    k = X.children(der, top[0][1], top[0][2])
    i = 0
    if i < len(k) and k[i][0] == 0x02:  # version (optional, default 0)
        v = X.der_int(der, k[i][1], k[i][2])
        if not 0 <= v <= 1:
            raise Unsupported("CRL version")
        i += 1
    if i >= len(k) or k[i][0] != 0x30:
        raise Unsupported("CRL signature algorithm")
    _alg(der, k[i][1], k[i][2])
    i += 1
    if i >= len(k) or k[i][0] != 0x30:
        raise Unsupported("CRL issuer")
    _name(der, k[i][1], k[i][2])
    i += 1
    if i >= len(k):
        raise Unsupported("CRL thisUpdate")
    _time(der, k[i][0], k[i][1], k[i][2])
    i += 1
    if i < len(k) and k[i][0] in (0x17, 0x18):  # nextUpdate
        _time(der, k[i][0], k[i][1], k[i][2])
        i += 1
    serials = set()
    if i < len(k) and k[i][0] == 0x30:  # revokedCertificates
        for t2, cs, ce, _ in X.children(der, k[i][1], k[i][2]):
            if t2 != 0x30:
                raise Unsupported("CRL revoked entry")
            r = X.children(der, cs, ce)
            if len(r) not in (2, 3) or r[0][0] != 0x02:
                raise Unsupported("CRL revoked entry")
            serials.add(X.der_int(der, r[0][1], r[0][2]))
            _time(der, r[1][0], r[1][1], r[1][2])
            if len(r) == 3:
                if r[2][0] != 0x30:
                    raise Unsupported("CRL entry extensions")
                _extensions(der, r[2][1], r[2][2])
        i += 1
    exts = []
    if i < len(k) and k[i][0] == 0xA0:  # crlExtensions [0] EXPLICIT
        inner = X.children(der, k[i][1], k[i][2])
        if len(inner) != 1 or inner[0][0] != 0x30:
            raise Unsupported("CRL extensions")
        exts = _extensions(der, inner[0][1], inner[0][2])
        i += 1
    if i != len(k):
        raise Unsupported("CRL: unread TBS fields")
    akis = [v for o, v in exts if o == OID_AKI]
    if len(akis) != 1:
        raise Unsupported("CRL without exactly one AuthorityKeyIdentifier")
    a = akis[0]
    t3, cs3, ce3 = X.tlv(a, 0)
    if t3 != 0x30 or ce3 != len(a):
        raise Unsupported("CRL AKI shape")
    ak = X.children(a, cs3, ce3)
    if len(ak) != 1 or ak[0][0] != 0x80:
        raise Unsupported("CRL AKI fields")
    aki = a[ak[0][1]:ak[0][2]]
    alg = _alg(der, top[1][1], top[1][2])
    if alg != ALG_ECDSA_SHA256:
        raise Unsupported("CRL signature algorithm other than ecdsa-with-SHA256")
    bits = der[top[2][1]:top[2][2]]
    if not bits or bits[0] != 0:
        raise Unsupported("CRL signature padding bits")
    sig = bits[1:]
    # utils.UnmarshalECDSASignature: asn1.Unmarshal into {R, S *big.Int} (bytes after the SEQUENCE,
    # and elements after S inside it, are not read); R, S > 0 else setup fails
    try:
        t4, cs4, ce4 = X.tlv(sig, 0)
    except X.ParseError:
        raise X.ParseError("CRL signature value")
    if t4 != 0x30:
        raise X.ParseError("CRL signature value")
    rs = X.children(sig, cs4, ce4)
    if len(rs) < 2 or rs[0][0] != 0x02 or rs[1][0] != 0x02:
        raise Unsupported("CRL signature value shape")
    r, s_ = X.der_int(sig, rs[0][1], rs[0][2]), X.der_int(sig, rs[1][1], rs[1][2])
    if r <= 0 or s_ <= 0:
        raise X.ParseError("CRL signature R, S must be positive")
    return dict(tbs=tbs, aki=aki, serials=serials, alg=alg, r=r, s=s_)


def crl_signed_by(crl, ca, verify_der):
    """CheckCRLSignature by the CA: ECDSA over SHA-256 of TBSCertList.Raw with the re-marshalled
    (r, s); high-S accepted (Go's ecdsa), r, s >= n rejected"""
    if ca["key"] != "p256":
        raise Unsupported("CA key other than P-256")
    r, s = crl["r"], crl["s"]
    if not (0 < r < X.P256_N and 0 < s < X.P256_N):
        return False
    if s > X.P256_N >> 1:
        s = X.P256_N - s
    body = X._der_intb(r) + X._der_intb(s)
    low = b"\x30" + X._der_len(len(body)) + body
    return verify_der(ca["pub"][:32], ca["pub"][32:], low, hashlib.sha256(crl["tbs"]).digest()) == 0


def revoked(cert, chain, crls, verify_der):
    """validateCertAgainstChain's CRL loop: cert's serial revoked by a CRL of its issuing CA
    (chain[1]) that the CA signed"""
    ski = chain[1]["ski"]
    for crl in crls:
        if crl["aki"] == ski and cert["serial"] in crl["serials"] and crl_signed_by(crl, chain[1], verify_der):
            return True
    return False
