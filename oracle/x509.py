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
P384_P = 2 ** 384 - 2 ** 128 - 2 ** 96 + 2 ** 32 - 1
P384_B = 0xB3312FA7E23EE7E4988E056BE3F82D19181D9C6EFE8141120314088F5013875AC656398D8A2ED19D2A85C8EDD3EC2AEF


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
    """encoding/pem Decode of the first block (Go 1.21 encoding/pem/pem.go Decode), for the one
    shape the engine models: "-----BEGIN <type>-----" at offset 0, lines of base64 alphabet only,
    "-----END <type>-----" at a line start followed by nothing, "\n" or "\r\n"; line ends "\n" or
    "\r\n"; canonical padding.  -> DER.  None only where Go's Decode certainly returns nil (no
    "-----BEGIN " anywhere).  Any other shape raises Unsupported: Go may still find a block there
    (a BEGIN after a newline, a later block after a malformed one, headers, stripped blanks...)."""
    if b"-----BEGIN " not in data:
        return None
    if not data.startswith(b"-----BEGIN "):
        raise Unsupported("PEM: BEGIN not at offset 0")
    i = 11
    ts = i
    while i < len(data) and data[i] != 0x2D and 0x20 <= data[i] < 0x7F:
        i += 1
    typ = data[ts:i]

    def eol(k):
        if data[k:k + 1] == b"\n":
            return k + 1
        if data[k:k + 2] == b"\r\n":
            return k + 2
        return None

    if data[i:i + 5] != b"-----":
        raise Unsupported("PEM: type line")
    i = eol(i + 5)
    if i is None:
        raise Unsupported("PEM: type line")
    alpha = set(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/=")
    b64 = bytearray()
    while True:
        if i >= len(data):
            raise Unsupported("PEM: no END line")
        if data.startswith(b"-----END ", i):
            break
        a = i
        while i < len(data) and data[i] in alpha:
            i += 1
        b64 += data[a:i]
        i = eol(i)
        if i is None:
            raise Unsupported("PEM: body line")
    i += 9
    if data[i:i + len(typ) + 5] != typ + b"-----":
        raise Unsupported("PEM: END line")
    i += len(typ) + 5
    if i != len(data) and eol(i) is None:
        raise Unsupported("PEM: END line")
    if len(b64) % 4:
        raise Unsupported("PEM: base64 length")
    core = b64.rstrip(b"=")
    if b"=" in core or len(b64) - len(core) > 2:
        raise Unsupported("PEM: base64 padding")
    return base64.b64decode(bytes(b64))  # (non-zero trailing bits accepted, as Go's StdEncoding)


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


class _Rd:
    """cryptobyte.String over b[s:e]; each read mirrors the Go call named beside it.  A failing
    read Go makes is a ParseError; bytes Go leaves unread where the restatement would need to know
    what Go does with them raise Unsupported."""

    def __init__(self, b, s, e):
        self.b, self.s, self.e = b, s, e

    def empty(self):
        return self.s >= self.e

    def peek(self, tag):  # PeekASN1Tag
        return self.s < self.e and self.b[self.s] == tag

    def any(self):  # ReadAnyASN1Element -> (tag, cs, ce, hs)
        t, cs, ce = tlv(self.b, self.s, self.e)
        hs, self.s = self.s, ce
        return t, cs, ce, hs

    def elem(self, tag):  # ReadASN1Element / ReadASN1 with a tag
        x = self.any()
        if x[0] != tag:
            raise ParseError("tag %#x where %#x expected" % (x[0], tag))
        return x

    def into(self, x):
        return _Rd(self.b, x[1], x[2])

    def rest_unread(self):
        if not self.empty():
            raise Unsupported("bytes Go leaves unread")


def _ous(b, s, e):
    """parseName: RDNSequence of SETs of AttributeTypeAndValue {OID, any string}; what an
    attribute holds after its value is never read by Go (nor here)"""
    out = []
    raw = _Rd(b, s, e)
    while not raw.empty():
        st = raw.into(raw.elem(0x31))
        while not st.empty():
            atv = st.into(st.elem(0x30))
            t1 = atv.elem(0x06)
            if not valid_oid(b[t1[1]:t1[2]]):
                raise ParseError("bad attribute type")
            t2 = atv.any()
            v = _string(b, t2[0], t2[1], t2[2])  # every attribute value parses (parseASN1String)
            if b[t1[1]:t1[2]] == OID_OU:
                out.append(v)
    return out


def _bool(b, x):  # ReadASN1Boolean
    if b[x[1]:x[2]] not in (b"\x00", b"\xff"):
        raise ParseError("bad BOOLEAN")
    return b[x[1]] == 0xFF


def _int64(b, x):  # ReadASN1Integer into a Go int (64-bit)
    if x[0] != 0x02 or x[2] - x[1] > 8:
        raise ParseError("bad integer")
    return der_int(b, x[1], x[2])


def _bitstring_ok(b, x):  # ReadASN1BitString's validity rules
    s, e = x[1], x[2]
    if e == s or b[s] > 7 or (e - s == 1 and b[s]) or (b[e - 1] & ((1 << b[s]) - 1)):
        raise ParseError("bad BIT STRING")


def _ai(b, x):
    """parseAI: OID, then at most one parameters element (anything after it: Unsupported)"""
    r = _Rd(b, x[1], x[2])
    o = r.elem(0x06)
    if not valid_oid(b[o[1]:o[2]]):
        raise ParseError("malformed OID")
    par = None if r.empty() else r.any()
    r.rest_unread()
    return b[o[1]:o[2]], par


ALG_ECDSA_SHA256 = bytes.fromhex("300a06082a8648ce3d040302")


def parse_certificate(der):
    """x509.ParseCertificate (Go 1.21 crypto/x509/parser.go parseCertificate), in Go's read
    order -> dict of the fields the MSP path reads; ParseError / Unsupported"""
    top = _Rd(der, 0, len(der)).elem(0x30)  # "x509: malformed certificate"
    if top[2] != len(der):
        raise ParseError("x509: trailing data")
    inp = _Rd(der, top[1], top[2])
    tbs = inp.elem(0x30)
    tbs_raw = der[tbs[3]:tbs[2]]
    t = inp.into(tbs)
    version = 0
    if t.peek(0xA0):  # ReadOptionalASN1Integer([0] EXPLICIT, default 0)
        vr = t.into(t.elem(0xA0))
        version = _int64(der, vr.elem(0x02))
        if not vr.empty():
            raise ParseError("bad version")
    if not 0 <= version <= 2:
        raise ParseError("x509: malformed / invalid version")
    if version != 2:
        raise Unsupported("certificate version %d" % (version + 1))
    serial_t = t.elem(0x02)
    serial = der_int(der, serial_t[1], serial_t[2])
    alg = t.elem(0x30)
    oalg = inp.elem(0x30)
    if der[alg[1]:alg[2]] != der[oalg[1]:oalg[2]]:
        raise ParseError("signature algorithm identifier mismatch")
    _ai(der, alg)
    if der[oalg[3]:oalg[2]] != ALG_ECDSA_SHA256:
        raise Unsupported("signature algorithm other than ecdsa-with-SHA256 (no parameters)")
    issuer = t.elem(0x30)
    _ous(der, issuer[1], issuer[2])  # (issuer names parse too)
    vr = t.into(t.elem(0x30))
    times = []
    for _ in range(2):  # parseTime
        if not (vr.peek(0x17) or vr.peek(0x18)):
            raise ParseError("x509: unsupported time format")
        x = vr.any()
        times.append(_time(der, x[0], x[1], x[2]))
    vr.rest_unread()
    not_before, not_after = times
    subject = t.elem(0x30)
    ous = _ous(der, subject[1], subject[2])
    # public key
    sp = t.into(t.elem(0x30))
    koid, kpar = _ai(der, sp.elem(0x30))
    spk = sp.elem(0x03)
    _bitstring_ok(der, spk)
    sp.rest_unread()
    bits = der[spk[1]:spk[2]]
    key, pub = "other", None
    if koid == OID_EC_KEY:
        if kpar is not None and kpar[0] == 0x06 and der[kpar[1]:kpar[2]] == OID_P256:
            pt = bits[1:] if bits[:1] == b"\x00" else b""
            if len(pt) != 65 or pt[0] != 4:
                raise Unsupported("P-256 point encoding")
            x, y = int.from_bytes(pt[1:33], "big"), int.from_bytes(pt[33:], "big")
            if x >= P256_P or y >= P256_P or (y * y - (x * x * x - 3 * x + P256_B)) % P256_P:
                raise ParseError("point not on curve")
            key, pub = "p256", pt[1:]
        elif kpar is not None and kpar[0] == 0x06 and der[kpar[1]:kpar[2]] == OID_P384:
            # P-384 leaves (round 6): crypto/elliptic Unmarshal of the uncompressed point
            pt = bits[1:] if bits[:1] == b"\x00" else b""
            if len(pt) != 97 or pt[0] != 4:
                raise Unsupported("P-384 point encoding")
            x, y = int.from_bytes(pt[1:49], "big"), int.from_bytes(pt[49:], "big")
            if x >= P384_P or y >= P384_P or (y * y - (x * x * x - 3 * x + P384_B)) % P384_P:
                raise ParseError("point not on curve")
            key, pub = "p384", pt[1:]
        else:  # (other curves: not restated; the engine cannot verify them either)
            raise Unsupported("EC curve")
    elif koid == OID_ED25519:
        key = "undeserializable"  # (a parse or a KeyImport error: undeserializable either way)
    elif koid == OID_RSA:
        # RSA can never pass identity.Verify: msp/identities.go:190 passes nil opts and the RSA
        # verifiers reject them (fabric-lib-go bccsp/sw/rsa.go:48-61).  Whether Go's
        # PKCS#1 key checks accept the key (a deserialized identity that never verifies) or not
        # (DeserializeIdentity fails) the outcome is the same on every path that uses it --
        # creator: BAD_CREATOR_SIGNATURE; endorsement / orderer signature: skipped, before any
        # de-duplication (common/policies/policy.go:363-395) -- so those checks are not restated.
        key = "other"
    else:
        raise Unsupported("public key algorithm")
    if t.peek(0x81) or t.peek(0x82):
        raise Unsupported("issuer/subject unique id")
    exts = {}
    unhandled_critical = False
    if t.peek(0xA3):
        xr = t.into(t.elem(0xA3))
        er = xr.into(xr.elem(0x30))
        xr.rest_unread()
        while not er.empty():
            e = er.into(er.elem(0x30))  # parseExtension
            o = e.elem(0x06)
            oid = der[o[1]:o[2]]
            if not valid_oid(oid):
                raise ParseError("malformed extension OID")
            crit = _bool(der, e.elem(0x01)) if e.peek(0x01) else False
            val = e.elem(0x04)
            e.rest_unread()
            if oid in exts:
                raise ParseError("duplicate extension")
            exts[oid] = (crit, val)
            if oid in EXT_GO_PARSED or (oid in (EXT_SKI, EXT_AKI) and crit):
                raise Unsupported("extension %s" % oid.hex())
            if oid not in (EXT_SKI, EXT_KU, EXT_BC, EXT_AKI, EXT_EKU, EXT_SAN) and crit:
                unhandled_critical = True
    t.rest_unread()  # what follows the extensions in the TBS is never read by Go
    is_ca, bc_valid, path_len = False, False, -1
    ski = None
    key_usage = 0
    for oid, (crit, val) in exts.items():  # processExtensions
        v = _Rd(der, val[1], val[2])
        if oid == EXT_BC:
            k = v.into(v.elem(0x30))
            v.rest_unread()
            if k.peek(0x01):
                is_ca = _bool(der, k.elem(0x01))
            if k.peek(0x02):
                path_len = _int64(der, k.elem(0x02))
            k.rest_unread()
            bc_valid = True
        elif oid == EXT_SKI:
            x = v.elem(0x04)
            v.rest_unread()
            ski = der[x[1]:x[2]]
        elif oid == EXT_KU:
            x = v.elem(0x03)
            _bitstring_ok(der, x)
            v.rest_unread()
            for k, byte in enumerate(der[x[1] + 1:x[2]]):  # parseKeyUsageExtension: the first 9 bits
                for bit in range(8):
                    if byte & (0x80 >> bit) and 8 * k + bit < 9:
                        key_usage |= 1 << (8 * k + bit)
        elif oid == EXT_AKI:
            k = v.into(v.elem(0x30))
            v.rest_unread()
            if k.peek(0x80):
                k.elem(0x80)  # (the rest of the SEQUENCE is never read by Go)
        elif oid in (EXT_EKU, EXT_SAN):
            k = v.into(v.elem(0x30))
            v.rest_unread()
            names = 0
            while not k.empty():
                kt, ks, ke, _ = k.any()
                if oid == EXT_EKU and (kt != 0x06 or not valid_oid(der[ks:ke])):
                    raise ParseError("invalid extended key usages")
                if oid == EXT_SAN:  # parseSANExtension (by tag ^ 0x80)
                    if kt in (0x81, 0x82) and any(c >= 0x80 for c in der[ks:ke]):
                        raise ParseError("SAN rfc822Name / dNSName is malformed")
                    if kt == 0x86:
                        raise Unsupported("SAN URI (url.Parse not restated)")
                    if kt == 0x87 and ke - ks not in (4, 16):
                        raise ParseError("SAN iPAddress of wrong length")
                    names += kt in (0x81, 0x82, 0x87)
            if oid == EXT_SAN and not names and crit:
                unhandled_critical = True  # (nothing parsed: Go's critical check applies)
    sig_t = inp.elem(0x03)  # "x509: malformed signature"
    _bitstring_ok(der, sig_t)
    sig_bits = der[sig_t[1]:sig_t[2]]
    if sig_bits[0] != 0:
        raise Unsupported("signature BIT STRING with unused bits")
    inp.rest_unread()  # elements after the signature: Go ignores them (cert.Raw keeps them)
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
