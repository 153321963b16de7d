"""Synthetic Fabric workloads (keys, certificates, signed blocks) for tests and bench.

Signing uses OpenSSL through fgv_synth.c -- an implementation independent of both the
GPU engine and the oracle.  This package is input generation, not the product path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libfgv_synth.so")
        if not os.path.exists(path):
            raise RuntimeError("fabric_amd/synth/libfgv_synth.so not built (run `make`)")
        L = ctypes.CDLL(path)
        L.synth_keygen.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.c_char_p]
        L.synth_sign_rs.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                    ctypes.c_char_p]
        L.synth_der_encode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.synth_der_encode.restype = ctypes.c_size_t
        L.synth_sign_batch.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.synth_make_cert.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                      ctypes.c_char_p, ctypes.c_int, ctypes.c_long, ctypes.c_char_p,
                                      ctypes.c_size_t]
        L.synth_ed25519_keygen.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p]
        L.synth_ed25519_sign_batch.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_void_p]
        L.synth_make_cert_ed25519.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                              ctypes.c_char_p, ctypes.c_long, ctypes.c_char_p, ctypes.c_size_t]
        L.synth_p384_keygen.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p,
                                        ctypes.c_char_p]
        L.synth_p384_sign_rs.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_char_p, ctypes.c_char_p]
        L.synth_make_cert_p384.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.c_char_p, ctypes.c_char_p, ctypes.c_long, ctypes.c_char_p,
                                           ctypes.c_size_t]
        _LIB = L
    return _LIB


class Key:
    """A P-256 key pair derived deterministically from (seed, idx)."""

    def __init__(self, seed: int, idx: int):
        priv = ctypes.create_string_buffer(32)
        qx = ctypes.create_string_buffer(32)
        qy = ctypes.create_string_buffer(32)
        lib().synth_keygen(seed, idx, priv, qx, qy)
        self.priv, self.qx, self.qy = priv.raw, qx.raw, qy.raw

    @property
    def pub(self) -> bytes:
        return self.qx + self.qy


def der_encode(r: int, s: int) -> bytes:
    out = ctypes.create_string_buffer(80)
    n = lib().synth_der_encode(r.to_bytes(32, "big"), s.to_bytes(32, "big"), out)
    return out.raw[:n]


def sign_rs(key: Key, digest: bytes, high_s: bool = False):
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    lib().synth_sign_rs(key.priv, digest, 1 if high_s else 0, r, s)
    return int.from_bytes(r.raw, "big"), int.from_bytes(s.raw, "big")


def sign(key: Key, digest: bytes, high_s: bool = False) -> bytes:
    r, s = sign_rs(key, digest, high_s)
    return der_encode(r, s)


def sign_batch(privs: bytes, digests: bytes, n: int, threads: int = 8, high_s: bool = False):
    """Sign n digests; privs/digests are n*32 concatenated bytes.  Returns list of DER sigs."""
    stride = 80
    buf = ctypes.create_string_buffer(stride * n)
    lens = (ctypes.c_uint32 * n)()
    lib().synth_sign_batch(privs, digests, n, buf, lens, stride, 1 if high_s else 0, threads)
    raw = buf.raw
    return [raw[stride * i: stride * i + lens[i]] for i in range(n)]


def make_cert(subject: Key, issuer: Key, cn: str, org: str, issuer_cn: str, is_ca: bool,
              serial: int) -> bytes:
    out = ctypes.create_string_buffer(4096)
    n = lib().synth_make_cert(subject.priv, issuer.priv, cn.encode(), org.encode(), issuer_cn.encode(),
                              1 if is_ca else 0, serial, out, 4096)
    if n < 0:
        raise RuntimeError("certificate generation failed")
    return out.raw[:n]


class EdKey:
    """An Ed25519 key pair derived deterministically from (seed, idx) (config C5)."""

    kind = "ed25519"

    def __init__(self, seed: int, idx: int):
        priv = ctypes.create_string_buffer(32)
        pub = ctypes.create_string_buffer(32)
        if lib().synth_ed25519_keygen(seed, idx, priv, pub) != 0:
            raise RuntimeError("ed25519 keygen failed")
        self.priv, self.pub = priv.raw, pub.raw


def ed25519_sign_batch(privs: bytes, msgs):
    """RFC 8032 signatures (64 B) of msgs[i] under privs[32*i:32*i+32]."""
    import numpy as np
    n = len(msgs)
    if n == 0:
        return []
    off = np.zeros(n, np.uint64)
    ln = np.array([len(m) for m in msgs], np.uint32)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = b"".join(msgs)
    out = ctypes.create_string_buffer(64 * n)
    if lib().synth_ed25519_sign_batch(privs, buf, off.ctypes.data, ln.ctypes.data, n, out) != 0:
        raise RuntimeError("ed25519 signing failed")
    raw = out.raw
    return [raw[64 * i: 64 * i + 64] for i in range(n)]


def make_cert_ed25519(subject: EdKey, issuer: Key, cn: str, org: str, issuer_cn: str, serial: int) -> bytes:
    out = ctypes.create_string_buffer(4096)
    n = lib().synth_make_cert_ed25519(subject.priv, issuer.priv, cn.encode(), org.encode(), issuer_cn.encode(),
                                      serial, out, 4096)
    if n < 0:
        raise RuntimeError("certificate generation failed")
    return out.raw[:n]


# ---------------------------------------------------------------- P-384 identities
N384 = int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973", 16)


class Key384:
    """A P-384 key pair derived deterministically from (seed, idx); pub = X || Y (96 bytes)."""

    kind = "p384"

    def __init__(self, seed: int, idx: int):
        priv = ctypes.create_string_buffer(48)
        qx = ctypes.create_string_buffer(48)
        qy = ctypes.create_string_buffer(48)
        lib().synth_p384_keygen(seed, idx, priv, qx, qy)
        self.priv, self.qx, self.qy = priv.raw, qx.raw, qy.raw

    @property
    def pub(self) -> bytes:
        return self.qx + self.qy


def der_encode_int(r: int, s: int) -> bytes:
    """DER ECDSASignature of arbitrary-size non-negative r, s (minimal INTEGERs)"""
    def i(v):
        b = v.to_bytes(v.bit_length() // 8 + 1, "big")
        return b"\x02" + bytes([len(b)]) + b
    body = i(r) + i(s)
    return b"\x30" + bytes([len(body)]) + body


def sign384_rs(key: Key384, digest: bytes, high_s: bool = False):
    r = ctypes.create_string_buffer(48)
    s = ctypes.create_string_buffer(48)
    lib().synth_p384_sign_rs(key.priv, digest, len(digest), 1 if high_s else 0, r, s)
    return int.from_bytes(r.raw, "big"), int.from_bytes(s.raw, "big")


def sign384(key: Key384, digest: bytes, high_s: bool = False) -> bytes:
    return der_encode_int(*sign384_rs(key, digest, high_s))


def make_cert_p384(subject: Key384, issuer: Key, cn: str, org: str, issuer_cn: str, serial: int, ou: str = "") -> bytes:
    """X.509 certificate of a P-384 key issued by a P-256 CA (ecdsa-with-SHA256)"""
    out = ctypes.create_string_buffer(4096)
    n = lib().synth_make_cert_p384(subject.priv, issuer.priv, cn.encode(), org.encode(), ou.encode(),
                                   issuer_cn.encode(), serial, out, 4096)
    if n < 0:
        raise RuntimeError("certificate generation failed")
    return out.raw[:n]
