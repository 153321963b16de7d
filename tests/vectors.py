"""Shared deterministic test vectors (signatures produced by OpenSSL via fabric_amd.synth)."""
import hashlib
import json
import os
import random

from fabric_amd import synth

N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
P = 2**256 - 2**224 + 2**192 + 2**96 - 1
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def der_int(x: int) -> bytes:
    b = x.to_bytes((x.bit_length() + 7) // 8 or 1, "big")
    if b[0] & 0x80:
        b = b"\x00" + b
    return b"\x02" + bytes([len(b)]) + b


def der_seq(body: bytes) -> bytes:
    if len(body) < 128:
        return b"\x30" + bytes([len(body)]) + body
    return b"\x30\x81" + bytes([len(body)]) + body


def edge_vectors(seed=5, nkeys=4):
    """(qx, qy, sig, digest, label) covering every acceptance rule of Appendix A."""
    rng = random.Random(seed)
    keys = [synth.Key(seed, i) for i in range(nkeys)]
    out = []
    for i in range(24):
        k = keys[i % nkeys]
        d = hashlib.sha256(b"m%d" % i).digest()
        r, s = synth.sign_rs(k, d)
        body = der_int(r) + der_int(s)
        good = der_seq(body)
        V = lambda sig, lab, dg=d, kq=(k.qx, k.qy): out.append((kq[0], kq[1], sig, dg, lab))
        V(good, "valid")
        V(good + b"\x00\xff\x13", "trailing bytes after SEQUENCE (Go accepts)")
        V(der_seq(body + der_int(7)), "extra element inside SEQUENCE (Go accepts)")
        V(der_seq(body + b"\xff\xff"), "garbage after S inside SEQUENCE (Go accepts)")
        V(der_seq(der_int(r) + der_int(N - s)), "high-S twin")
        V(good[:-1], "truncated")
        V(b"\x31" + good[1:], "SET instead of SEQUENCE")
        V(b"\x30\x80" + body + b"\x00\x00", "indefinite length")
        V(b"\x30\x81" + bytes([len(body)]) + body, "non-minimal long-form length")
        V(der_seq(b"\x02" + bytes([len(der_int(r)) - 1]) + b"\x00" + der_int(r)[2:] + der_int(s))
          if der_int(r)[2] != 0 else der_seq(b"\x02" + bytes([len(der_int(r)) - 1]) + b"\x00\x00" + der_int(r)[3:] + der_int(s)),
          "non-minimal INTEGER")
        V(der_seq(der_int(r) + b"\x02\x01\x00"), "s = 0")
        V(der_seq(b"\x02\x01\x00" + der_int(s)), "r = 0")
        V(der_seq(b"\x02\x01\xff" + der_int(s)), "r negative")
        V(der_seq(der_int(r + N) + der_int(s)) if r + N < 2**256 else der_seq(der_int(r + 2**256) + der_int(s)),
          "r >= n")
        V(der_seq(der_int(r + 2**256) + der_int(s)), "r >= 2^256")
        V(der_seq(der_int(r) + b"\x02\x00"), "empty INTEGER")
        V(der_seq(der_int(r)), "missing S")
        V(b"", "empty signature")
        V(good, "digest flipped", dg=bytes([d[0] ^ 0x80]) + d[1:])
        V(good, "wrong key", kq=(keys[(i + 1) % nkeys].qx, keys[(i + 1) % nkeys].qy))
        V(good, "key not on curve", kq=(k.qx, bytes(31) + b"\x01"))
        V(good, "key x >= p", kq=((P + 1).to_bytes(32, "big"), k.qy))
        V(b"\x30\x1f" + b"\x02\x00" * 15 + b"\x00", "junk")
        V(b"\x3f\x10" + good[1:], "high-tag-number form")
    return out


def golden_cert_vectors():
    d = json.load(open(os.path.join(GOLDEN, "msp_cert_sigs.json")))
    return [(bytes.fromhex(v["qx"]), bytes.fromhex(v["qy"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["digest"]),
             v["expected"], v["source"] + " / " + v["kind"]) for v in d["vectors"]]
