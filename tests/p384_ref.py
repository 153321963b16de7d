"""A pure-Python restatement of ECDSA P-384 verification with the reference's rules (TEST
INFRASTRUCTURE): bccsp sw verifyECDSA (fabric-lib-go bccsp/sw/ecdsa.go:41-57; low S against the
P-384 half order, bccsp/utils/ecdsa.go:26-31) over Go's ecdsa.Verify (go1.21.9: r, s in [1, n), e
= the digest, R = (e/s) G + (r/s) Q, R != inf, x_R mod n == r).  Independent of the OpenSSL-backed
oracle (oracle.verify_der_p384) and of the GPU kernel; the DER decode is oracle.der_decode's rules
generalised to any integer width."""
P = 2 ** 384 - 2 ** 128 - 2 ** 96 + 2 ** 32 - 1
N = int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973", 16)
B = int("b3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef", 16)
GX = int("aa87ca22be8b05378eb1c71ef320ad746e1d3b628ba79b9859f741e082542a385502f25dbf55296c3a545e3872760ab7", 16)
GY = int("3617de4a96262c6f5d9e98bf9292dc29f8f41dbd289a147ce9da3113b5f0b8c00a60b1ce1d7e819d7a431d7c90ea0e5f", 16)


def on_curve(x, y):
    return 0 <= x < P and 0 <= y < P and (y * y - (x ** 3 - 3 * x + B)) % P == 0


def add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    (x1, y1), (x2, y2) = p, q
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 - 3) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def mul(k, p):
    r = None
    while k:
        if k & 1:
            r = add(r, p)
        p = add(p, p)
        k >>= 1
    return r


def _tl(b, o):
    if o >= len(b):
        return None
    t = b[o]
    o += 1
    if t & 0x1F == 0x1F:
        return None  # (no high tag numbers in these vectors' valid shapes)
    if o >= len(b):
        return None
    ln = b[o]
    o += 1
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or o + nb > len(b):
            return None
        v = int.from_bytes(b[o:o + nb], "big")
        if b[o] == 0 or v < 0x80:
            return None
        o += nb
        ln = v
    return t, ln, o


def der_decode(sig):
    """-> (r, s) or None (Go encoding/asn1 rules for ECDSASignature{R, S})"""
    h = _tl(sig, 0)
    if h is None or h[0] != 0x30 or h[2] + h[1] > len(sig):
        return None
    inner = sig[h[2]:h[2] + h[1]]
    out, o = [], 0
    for _ in range(2):
        e = _tl(inner, o)
        if e is None or e[0] != 0x02 or e[2] + e[1] > len(inner) or e[1] == 0:
            return None
        v = inner[e[2]:e[2] + e[1]]
        if len(v) > 1 and ((v[0] == 0 and not v[1] & 0x80) or (v[0] == 0xFF and v[1] & 0x80)):
            return None
        x = int.from_bytes(v, "big", signed=True)
        if x <= 0:
            return None
        out.append(x)
        o = e[2] + e[1]
    return tuple(out)


def verify(pub96, sig, digest):
    """status byte (oracle / fgv.h): 0 valid, 1 false, 2 DER, 3 high S, 4 range, 5 key, 6 empty"""
    if not sig or not digest:
        return 6
    rs = der_decode(sig)
    if rs is None:
        return 2
    r, s = rs
    if s > N >> 1:
        return 3
    qx, qy = int.from_bytes(pub96[:48], "big"), int.from_bytes(pub96[48:96], "big")
    if not on_curve(qx, qy):
        return 5
    if r >= N:
        return 4
    e = int.from_bytes(digest, "big")
    w = pow(s, -1, N)
    R = add(mul(e * w % N, (GX, GY)), mul(r * w % N, (qx, qy)))
    if R is None:
        return 1
    return 0 if R[0] % N == r else 1
