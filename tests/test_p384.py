"""CPU: the P-384 path's constants and its two checkers.  p384_field.h's constants against values
derived here; the OpenSSL-backed oracle (oracle.verify_der_p384) against the pure-Python
restatement (tests/p384_ref.py) on signatures made by an independent signer (OpenSSL through
fabric_amd/synth) -- valid, tampered, high S, out of range, malformed DER, off-curve keys, Q = +-G."""
import hashlib
import os
import re

import pytest

import oracle
from fabric_amd import synth
from tests import p384_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))


def _header_consts():
    src = open(os.path.join(HERE, "..", "fabric_amd", "csrc", "p384_field.h")).read()
    body = src[src.index("#define P384_CONSTS"):src.index("static __constant__")]
    words = [int(w, 16) for w in re.findall(r"0x([0-9a-fA-F]{8})u", body)]
    arrs = [words[12 * i:12 * i + 12] for i in range(10)]
    val = [sum(w << (32 * k) for k, w in enumerate(a)) for a in arrs]
    return val, words[120], words[121]


def test_field_constants():
    (p, n, rr_p, one_p, rr_n, b_m, gx_m, gy_m, half_n, p_minus_n), n0p, n0n = _header_consts()
    Rm = 1 << 384
    assert p == R.P and n == R.N
    assert rr_p == Rm * Rm % R.P and one_p == Rm % R.P and rr_n == Rm * Rm % R.N
    assert b_m == R.B * Rm % R.P and gx_m == R.GX * Rm % R.P and gy_m == R.GY * Rm % R.P
    assert half_n == R.N >> 1 and p_minus_n == R.P - R.N
    assert n0p == (-pow(R.P, -1, 1 << 32)) % (1 << 32) and n0n == (-pow(R.N, -1, 1 << 32)) % (1 << 32)
    assert R.on_curve(R.GX, R.GY) and R.mul(R.N, (R.GX, R.GY)) is None


def vectors():
    """[(pub96, sig, digest, label, msg)]: digest = SHA-256(msg) (what identity.Verify hashes)"""
    out = []
    keys = [synth.Key384(61, i) for i in range(3)]
    for i in range(24):
        k = keys[i % 3]
        m = b"p384-%d" % i
        d = hashlib.sha256(m).digest()
        r, s = synth.sign384_rs(k, d)
        out.append((k.pub, synth.der_encode_int(r, s), d, "valid", m))
        out.append((k.pub, synth.der_encode_int(r, s), hashlib.sha256(b"x%d" % i).digest(), "tampered", b"x%d" % i))
        if i % 4 == 0:
            out.append((k.pub, synth.der_encode_int(r, R.N - s), d, "high_s", m))
            out.append((k.pub, synth.der_encode_int(r + R.N, s), d, "r_ge_n", m))
            out.append((k.pub, synth.der_encode_int(r, s)[:-1], d, "truncated", m))
            out.append((k.pub, synth.der_encode_int(r, s) + b"\x00\x01", d, "trailing_bytes", m))
            out.append((k.pub, b"", d, "empty", m))
            out.append((k.pub, synth.der_encode_int(1, 1), d, "r_s_one", m))
            out.append((k.pub, b"\x30\x06\x02\x01\x00\x02\x01\x01", d, "r_zero", m))
            out.append((bytes(96), synth.der_encode_int(r, s), d, "zero_key", m))
            out.append((k.qx + bytes(47) + b"\x01", synth.der_encode_int(r, s), d, "off_curve", m))
    # Q = G and Q = -G (private keys 1 and n - 1): the comb's exceptional additions
    for priv, tag in ((1, "q_is_g"), (R.N - 1, "q_is_minus_g")):
        k = synth.Key384.__new__(synth.Key384)
        k.priv = priv.to_bytes(48, "big")
        Q = R.mul(priv, (R.GX, R.GY))
        k.qx, k.qy = Q[0].to_bytes(48, "big"), Q[1].to_bytes(48, "big")
        for j in range(4):
            m = b"%s-%d" % (tag.encode(), j)
            d = hashlib.sha256(m).digest()
            out.append((k.pub, synth.sign384(k, d), d, tag, m))
    return out


def test_oracle_matches_restatement():
    for pub, sig, d, label, _ in vectors():
        want = R.verify(pub, sig, d)
        assert oracle.verify_der_p384(pub, sig, d) == want, label
        if label in ("valid", "q_is_g", "q_is_minus_g"):
            assert want == 0, label
        elif label == "tampered":
            assert want == 1
