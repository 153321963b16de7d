"""Minimal X.509 DER reader for test harnesses (subject OUs, EC public key): what the peer's
MSP layer extracts before it registers an identity with the engine.  Test infrastructure."""
import base64

OID_OU = bytes.fromhex("55040b")
OID_EC = bytes.fromhex("2a8648ce3d0201")
OID_P256 = bytes.fromhex("2a8648ce3d030107")
OID_P384 = bytes.fromhex("2b81040022")


def _tlv(b, o):
    tag = b[o]
    ln = b[o + 1]
    o += 2
    if ln & 0x80:
        nb = ln & 0x7F
        ln = int.from_bytes(b[o:o + nb], "big")
        o += nb
    return tag, o, ln


def _kids(b, o, ln):
    out, end = [], o + ln
    while o < end:
        t, co, cl = _tlv(b, o)
        out.append((t, co, cl))
        o = co + cl
    return out


def pem_to_der(pem):
    body = pem.split(b"-----BEGIN CERTIFICATE-----")[1].split(b"-----END CERTIFICATE-----")[0]
    return base64.b64decode(b"".join(body.split()))


def cert_info(der):
    """-> dict(ous=[...], key="p256"|"p384"|"other", pub=X||Y (P-256/P-384) or None)"""
    _, co, cl = _tlv(der, 0)
    tbs = _kids(der, co, cl)[0]
    f = _kids(der, tbs[1], tbs[2])
    i = 1 if f[0][0] == 0xA0 else 0
    subj, spki = f[i + 4], f[i + 5]
    ous = []
    for rdn in _kids(der, subj[1], subj[2]):
        for atv in _kids(der, rdn[1], rdn[2]):
            k = _kids(der, atv[1], atv[2])
            if der[k[0][1]:k[0][1] + k[0][2]] == OID_OU:
                ous.append(der[k[1][1]:k[1][1] + k[1][2]].decode())
    sp = _kids(der, spki[1], spki[2])
    alg = _kids(der, sp[0][1], sp[0][2])
    kalg = der[alg[0][1]:alg[0][1] + alg[0][2]]
    curve = der[alg[1][1]:alg[1][1] + alg[1][2]] if len(alg) > 1 else b""
    point = der[sp[1][1] + 1:sp[1][1] + sp[1][2]]  # BIT STRING, skip unused-bits byte
    key, pub = "other", None
    if kalg == OID_EC and curve == OID_P256 and point[:1] == b"\x04":
        key, pub = "p256", point[1:]
    elif kalg == OID_EC and curve == OID_P384:
        key, pub = "p384", point[1:]
    return dict(ous=ous, key=key, pub=pub)
