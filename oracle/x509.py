"""Restated X.509 subset the MSP identity path needs (TEST INFRASTRUCTURE ONLY -- the oracle).

What the reference does with a certificate it meets for the first time (msp/mspimpl.go:398-422
deserializeIdentityInternal -> msp/identities.go:48-84 newIdentity -> mspimpl.go:892-938
sanitizeCert, mspimplvalidate.go validateIdentity) rests on Go's crypto/x509 (Go 1.21,
ParseCertificate, Certificate.Verify, CheckSignatureFrom) and encoding/asn1.  Go's x509 is not
in /root/reference (the toolchain's standard library), so its rules are restated here for the
certificate shapes a Fabric CA / cryptogen issues -- v3, ECDSA P-256 keys, ecdsa-with-SHA256
signatures, the usual extensions -- and every shape outside them raises Unsupported (the engine
returns FGV_EUNSUPPORTED for it; the reference decides).  Parity is pinned by the reference's
own MSP fixture certificates (msp/testdata, sampleconfig/msp) and their test assertions.
"""
import base64
import calendar
import hashlib

from .v20 import Unsupported


class ParseError(Exception):
    """x509.ParseCertificate (or pem.Decode) fails: DeserializeIdentity returns an error"""


OID_EC_KEY = bytes.fromhex("2a8648ce3d0201")
OID_P256 = bytes.fromhex("2a8648ce3d030107")
OID_P384 = bytes.fromhex("2b81040022")
OID_ED25519 = bytes.fromhex("2b6570")
OID_RSA = bytes.fromhex("2a864886f70d010101")
OID_ECDSA_SHA256 = bytes.fromhex("2a8648ce3d040302")
OID_OU = bytes.fromhex("55040b")
EXT_SKI, EXT_KU, EXT_SAN, EXT_BC, EXT_AKI, EXT_EKU = (bytes.fromhex(h) for h in
                                                       ("551d0e", "551d0f", "551d11", "551d13", "551d23", "551d25"))
# extensions Go parses (errors possible) that this restatement does not: present -> Unsupported
EXT_GO_PARSED = {bytes.fromhex(h) for h in ("551d1e", "551d1f", "551d20", "2b06010505070101", "551d2e")}
P256_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
P256_P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
P256_B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B


def tlv(b, i, end=None):
    """one DER element at b[i:] -> (tag, content start, content end); strict definite lengths"""
    end = len(b) if end is None else end
    if i + 2 > end:
        raise ParseError("truncated")
    tag = b[i]
    if tag & 0x1F == 0x1F:
        raise ParseError("high tag number")
    ln = b[i + 1]
    o = i + 2
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or nb > 4 or o + nb > end:
            raise ParseError("bad length")
        if b[o] == 0:
            raise ParseError("non-minimal length")
        ln = int.from_bytes(b[o:o + nb], "big")
        if ln < 128:
            raise ParseError("non-minimal length")
        o += nb
    if o + ln > end:
        raise ParseError("length past end")
    return tag, o, o + ln


def children(b, s, e):
    out = []
    while s < e:
        t, cs, ce = tlv(b, s, e)
        out.append((t, cs, ce, s))
        s = ce
    return out


def der_int(b, s, e):
    if e == s:
        raise ParseError("empty integer")
    if e - s > 1 and ((b[s] == 0 and b[s + 1] < 0x80) or (b[s] == 0xFF and b[s + 1] >= 0x80)):
        raise ParseError("non-minimal integer")
    return int.from_bytes(b[s:e], "big", signed=True)


def valid_oid(b):
    """cryptobyte ReadASN1ObjectIdentifier: non-empty, every subidentifier minimal (no leading
    0x80), at most 5 bytes and below 2^31, none truncated"""
    if not b:
        return False
    i = 0
    while i < len(b):
        ret = 0
        for k in range(6):
            if k == 5 or i >= len(b) or ret >= 1 << 24:
                return False
            c = b[i]
            i += 1
            if k == 0 and c == 0x80:
                return False
            ret = (ret << 7) | (c & 0x7F)
            if not c & 0x80:
                break
    return True


def pem_decode(data):
    """encoding/pem Decode of the first block (any type; trailing text ignored) -> DER or None"""
    i = data.find(b"-----BEGIN ")
    if i < 0:
        return None
    j = data.find(b"-----", i + 11)
    if j < 0:
        return None
    end_tag = b"-----END " + data[i + 11:j] + b"-----"
    k = data.find(end_tag, j)
    if k < 0:
        return None
    body = data[j + 5:k]
    lines = [ln.strip() for ln in body.split(b"\n") if ln.strip()]
    if any(b":" in ln for ln in lines):
        raise Unsupported("PEM headers")
    try:
        return base64.b64decode(b"".join(lines), validate=True)
    except Exception:
        return None


def _time(b, t, s, e):
    v = b[s:e].decode("ascii", "replace")
    if t == 0x17 and len(v) == 13 and v.endswith("Z") and v[:12].isdigit():
        yy = int(v[0:2])
        y = 1900 + yy if yy >= 50 else 2000 + yy
        rest = v[2:12]
    elif t == 0x18 and len(v) == 15 and v.endswith("Z") and v[:14].isdigit():
        y = int(v[0:4])
        rest = v[4:14]
    else:
        raise Unsupported("time encoding")
    mo, d, hh, mm, ss = (int(rest[k:k + 2]) for k in range(0, 10, 2))
    if not (1 <= mo <= 12 and 1 <= d <= calendar.monthrange(y, mo)[1] and hh < 24 and mm < 60 and ss < 60):
        raise ParseError("bad time")  # (time.Parse: day out of range)
    return calendar.timegm((y, mo, d, hh, mm, ss, 0, 0, 0))


def _string(b, t, s, e):
    raw = b[s:e]
    if t == 0x0C:  # UTF8String
        try:
            return raw.decode("utf-8")
        except UnicodeDecodeError:
            raise ParseError("invalid UTF8String")
    if t == 0x13:  # PrintableString
        ok = all((c < 0x80 and chr(c).isalnum()) or chr(c) in " '()+,-./:=?*&" for c in raw)
        if not ok:
            raise ParseError("invalid PrintableString")
        return raw.decode()
    if t == 0x16:  # IA5String
        if any(c >= 0x80 for c in raw):
            raise ParseError("invalid IA5String")
        return raw.decode()
    if t in (0x12, 0x14, 0x1E):  # NumericString, T61String, BMPString: not restated
        raise Unsupported("name attribute string type %#x" % t)
    raise ParseError("unsupported string type %#x" % t)  # (parseASN1String)


def _ous(b, s, e):
    out = []
    for st, ss, se, _ in children(b, s, e):
        if st != 0x31:
            raise ParseError("RDN is not a SET")
        for at, as_, ae, _ in children(b, ss, se):
            if at != 0x30:
                raise ParseError("attribute is not a SEQUENCE")
            # (parseName reads the type and the value; anything after them is not read)
            t1 = tlv(b, as_, ae)
            if t1[0] != 0x06 or not valid_oid(b[t1[1]:t1[2]]):
                raise ParseError("bad attribute type")
            t2 = tlv(b, t1[2], ae)
            v = _string(b, t2[0], t2[1], t2[2])  # every attribute value parses (parseASN1String)
            if b[t1[1]:t1[2]] == OID_OU:
                out.append(v)
    return out


def parse_certificate(der):
    """-> dict of the fields the MSP path reads; ParseError / Unsupported"""
    t, cs, ce = tlv(der, 0)
    if t != 0x30 or ce != len(der):
        raise ParseError("not a single SEQUENCE (trailing data)")
    top = children(der, cs, ce)
    if len(top) != 3 or top[0][0] != 0x30 or top[1][0] != 0x30 or top[2][0] != 0x03:
        raise ParseError("bad certificate structure")
    tbs_raw = der[top[0][3]:top[0][2]]
    outer_alg = der[top[1][3]:top[1][2]]
    sig_bits = der[top[2][1]:top[2][2]]
    if not sig_bits or sig_bits[0] != 0:
        raise Unsupported("signature BIT STRING with unused bits")
    f = children(der, top[0][1], top[0][2])
    i = 0
    version = 0
    if f and f[0][0] == 0xA0:
        vk = children(der, f[0][1], f[0][2])
        if len(vk) != 1 or vk[0][0] != 0x02:
            raise ParseError("bad version")
        version = der_int(der, vk[0][1], vk[0][2])
        i = 1
    if version != 2:
        raise Unsupported("certificate version %d" % (version + 1))
    if len(f) < i + 6:
        raise ParseError("short TBSCertificate")
    serial_t, alg, issuer, validity, subject, spki = f[i:i + 6]
    if serial_t[0] != 0x02:
        raise ParseError("bad serial")
    serial = der_int(der, serial_t[1], serial_t[2])
    if der[alg[3]:alg[2]] != outer_alg:
        raise ParseError("signature algorithm identifier mismatch")
    if outer_alg != bytes.fromhex("300a06082a8648ce3d040302"):
        raise Unsupported("signature algorithm other than ecdsa-with-SHA256 (no parameters)")
    vk = children(der, validity[1], validity[2])
    if len(vk) != 2:
        raise ParseError("bad validity")
    not_before = _time(der, vk[0][0], vk[0][1], vk[0][2])
    not_after = _time(der, vk[1][0], vk[1][1], vk[1][2])
    if issuer[0] != 0x30 or subject[0] != 0x30:
        raise ParseError("bad name")
    ous = _ous(der, subject[1], subject[2])
    _ous(der, issuer[1], issuer[2])  # (issuer names parse too)
    # public key
    sk = children(der, spki[1], spki[2])
    if len(sk) != 2 or sk[0][0] != 0x30 or sk[1][0] != 0x03:
        raise ParseError("bad SubjectPublicKeyInfo")
    ak = children(der, sk[0][1], sk[0][2])
    if not ak or ak[0][0] != 0x06 or not valid_oid(der[ak[0][1]:ak[0][2]]):
        raise ParseError("malformed public key algorithm identifier")
    koid = der[ak[0][1]:ak[0][2]]
    bits = der[sk[1][1]:sk[1][2]]
    key, pub = "other", None
    if koid == OID_EC_KEY:
        curve = der[ak[1][1]:ak[1][2]] if len(ak) == 2 and ak[1][0] == 0x06 else b""
        if curve == OID_P256:
            pt = bits[1:] if bits[:1] == b"\x00" else b""
            if len(pt) != 65 or pt[0] != 4:
                raise Unsupported("P-256 point encoding")
            x, y = int.from_bytes(pt[1:33], "big"), int.from_bytes(pt[33:], "big")
            if x >= P256_P or y >= P256_P or (y * y - (x * x * x - 3 * x + P256_B)) % P256_P:
                raise ParseError("point not on curve")
            key, pub = "p256", pt[1:]
        else:  # (P-384: Go checks the point on the curve -- not restated; the engine cannot verify it either)
            raise Unsupported("EC curve")
    elif koid == OID_ED25519:
        key = "undeserializable"  # bccsp KeyImport rejects it
    else:  # (RSA: Go's PKCS#1 key checks are not restated)
        raise Unsupported("public key algorithm")
    # extensions
    rest = f[i + 6:]
    exts = {}
    unhandled_critical = False
    for r in rest:
        if r[0] in (0x81, 0x82):
            raise Unsupported("issuer/subject unique id")
        if r[0] != 0xA3:
            raise ParseError("unexpected TBSCertificate field")
        ek = children(der, r[1], r[2])
        if len(ek) != 1 or ek[0][0] != 0x30:
            raise ParseError("bad extensions")
        for et, es, ee, _ in children(der, ek[0][1], ek[0][2]):
            ef = children(der, es, ee)
            if et != 0x30 or not ef or ef[0][0] != 0x06:
                raise ParseError("bad extension")
            oid = der[ef[0][1]:ef[0][2]]
            if not valid_oid(oid):
                raise ParseError("malformed extension OID")
            crit = False
            j = 1
            if len(ef) > j and ef[j][0] == 0x01:
                if der[ef[j][1]:ef[j][2]] not in (b"\x00", b"\xff"):
                    raise ParseError("bad BOOLEAN")
                crit = der[ef[j][1]] == 0xFF
                j += 1
            if len(ef) != j + 1 or ef[j][0] != 0x04:
                raise ParseError("bad extension value")
            if oid in exts:
                raise ParseError("duplicate extension")
            val = der[ef[j][1]:ef[j][2]]
            exts[oid] = (crit, val)
            if oid in EXT_GO_PARSED:
                raise Unsupported("extension %s" % oid.hex())
            if oid not in (EXT_SKI, EXT_KU, EXT_BC, EXT_AKI, EXT_EKU, EXT_SAN) and crit:
                unhandled_critical = True
    is_ca, bc_valid, path_len = False, False, -1
    if EXT_BC in exts:
        v = exts[EXT_BC][1]
        t, s, e = tlv(v, 0)
        if t != 0x30 or e != len(v):
            raise ParseError("bad basicConstraints")
        k = children(v, s, e)
        if k and k[0][0] == 0x01:
            if v[k[0][1]:k[0][2]] not in (b"\x00", b"\xff"):
                raise ParseError("bad BOOLEAN")
            is_ca = v[k[0][1]] == 0xFF
            k = k[1:]
        if k and (k[0][0] != 0x02 or len(k) > 1):
            raise ParseError("bad pathLen")
        if k:  # MaxPathLen (ReadASN1Integer into an int: must fit in 64 bits)
            path_len = der_int(v, k[0][1], k[0][2])
            if not -(1 << 63) <= path_len < (1 << 63):
                raise ParseError("pathLen out of range")
        bc_valid = True
    ski = None
    if EXT_SKI in exts:
        v = exts[EXT_SKI][1]
        t, s, e = tlv(v, 0)
        if t != 0x04 or e != len(v):
            raise ParseError("bad SKI")
        ski = v[s:e]
    key_usage = 0
    if EXT_KU in exts:
        v = exts[EXT_KU][1]
        t, s, e = tlv(v, 0)
        # cryptobyte ReadASN1BitString: unused-bit count <= 7, none with no data, unused bits zero
        if t != 0x03 or e != len(v) or e == s or v[s] > 7 or (e - s == 1 and v[s]) or \
                (v[e - 1] & ((1 << v[s]) - 1)):
            raise ParseError("bad keyUsage")
        # parseKeyUsageExtension reads the first 9 bits
        for k, byte in enumerate(v[s + 1:e]):
            for bit in range(8):
                if byte & (0x80 >> bit) and 8 * k + bit < 9:
                    key_usage |= 1 << (8 * k + bit)
    for oid in (EXT_AKI, EXT_EKU, EXT_SAN):
        if oid in exts:
            v = exts[oid][1]
            t, s, e = tlv(v, 0)
            if t != 0x30 or e != len(v):
                raise ParseError("bad extension content")
            names = 0
            for kt, ks, ke, _ in children(v, s, e):
                if oid == EXT_EKU and (kt != 0x06 or not valid_oid(v[ks:ke])):
                    raise ParseError("invalid extended key usages")
                if oid == EXT_SAN:  # parseSANExtension (by tag ^ 0x80)
                    if kt in (0x81, 0x82) and any(c >= 0x80 for c in v[ks:ke]):
                        raise ParseError("SAN rfc822Name / dNSName is malformed")
                    if kt == 0x86:
                        raise Unsupported("SAN URI (url.Parse not restated)")
                    if kt == 0x87 and ke - ks not in (4, 16):
                        raise ParseError("SAN iPAddress of wrong length")
                    names += kt in (0x81, 0x82, 0x87)
            if oid == EXT_SAN and not names and exts[oid][0]:
                unhandled_critical = True  # (nothing parsed: Go's critical check applies)
    return dict(der=der, tbs=tbs_raw, sig=sig_bits[1:], serial=serial, issuer=der[issuer[3]:issuer[2]],
                subject=der[subject[3]:subject[2]], not_before=not_before, not_after=not_after, ous=ous,
                key=key, pub=pub, is_ca=is_ca, bc_valid=bc_valid, path_len=path_len, ski=ski, key_usage=key_usage,
                unhandled_critical=unhandled_critical, version=version + 1)


def strict_sig(sig):
    """crypto/ecdsa VerifyASN1's cryptobyte parse: SEQUENCE{INTEGER r, INTEGER s}, nothing else
    -> (r, s) or None (verification fails)"""
    try:
        t, s, e = tlv(sig, 0)
        if t != 0x30 or e != len(sig):
            return None
        k = children(sig, s, e)
        if len(k) != 2 or k[0][0] != 0x02 or k[1][0] != 0x02:
            return None
        return der_int(sig, k[0][1], k[0][2]), der_int(sig, k[1][1], k[1][2])
    except ParseError:
        return None


def _der_len(n):
    if n < 128:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _der_intb(v):
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
    return b"\x02" + _der_len(len(b)) + b


def sanitized_raw(c):
    """sanitizeECDSASignedCert (msp/cert.go): the certificate re-marshalled with a low-S
    signature (utils.SignatureToLowS keeps the signature bytes when already low-S)."""
    sig = c["sig"]
    rs = strict_sig(sig)
    if rs is None or not (0 < rs[0] < P256_N and 0 < rs[1] < P256_N):
        # (a leaf's chain check rejects these first; a root CA's would fail MSP setup)
        raise Unsupported("certificate signature not strict DER with 0 < r, s < n")
    r, s = rs
    if s > P256_N >> 1:
        body = _der_intb(r) + _der_intb(P256_N - s)
        sig = b"\x30" + _der_len(len(body)) + body
    bits = b"\x00" + sig
    alg = bytes.fromhex("300a06082a8648ce3d040302")
    body = c["tbs"] + alg + b"\x03" + _der_len(len(bits)) + bits
    return b"\x30" + _der_len(len(body)) + body


def ca_verifies(ca, c, verify_der):
    """parent.CheckSignature(ECDSAWithSHA256, c.RawTBSCertificate, c.Signature): ECDSA over
    SHA-256 of the TBS, high-S accepted (Go's ecdsa, not Fabric's low-S rule)."""
    if ca["key"] != "p256":
        raise Unsupported("CA key other than P-256")
    rs = strict_sig(c["sig"])
    if rs is None:
        return False
    r, s = rs
    if not (0 < r < P256_N and 0 < s < P256_N):
        return False
    if s > P256_N >> 1:
        s = P256_N - s
    body = _der_intb(r) + _der_intb(s)
    low = b"\x30" + _der_len(len(body)) + body
    return verify_der(ca["pub"][:32], ca["pub"][32:], low, hashlib.sha256(c["tbs"]).digest()) == 0
