"""CPU oracle for the Fabric committer hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package.  The product (fabric_amd, libfgv.so) never imports, links or calls it.

  liboracle.so   C restatement of SHA-256, Go-rule DER, low-S, ECDSA-P256 verify
                 (fgv_oracle.c; reference citations in fgv_oracle.h)
  protowire.py   Go protobuf-wire decoding rules for the Fabric messages on the path
  v20.py         restated committer validation (txvalidator/v20 + msgvalidation +
                 plugindispatcher + builtin v20 + cauthdsl + SignatureSetToValidIdentities)
  mvcc.py        restated sequential MVCC (kvledger/txmgmt/validation)
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so not built (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        c_u8p = ctypes.c_char_p
        L.oracle_sha256.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_der_decode.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p,
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_p256_verify_der.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t]
        L.oracle_p256_verify_der_ossl.argtypes = L.oracle_p256_verify_der.argtypes
        L.oracle_p256_verify_rs.argtypes = [c_u8p] * 5
        L.oracle_p256_base_mult.argtypes = [c_u8p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_verify_msgs_batch.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_size_t, ctypes.c_void_p,
                                                                       ctypes.c_int, ctypes.c_int]
        L.oracle_verify_msgs_batch.restype = None
        L.oracle_p384_verify_der.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t]
        _LIB = L
    return _LIB


def sha256(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_sha256(msg, len(msg), out)
    return out.raw


def der_decode(sig: bytes):
    """Go encoding/asn1 decode of ECDSASignature{R,S} (bccsp/utils/ecdsa.go:41-65).
    Returns (r, s) ints or None on error (incl. r<=0 / s<=0)."""
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    rb, sb = ctypes.c_int(0), ctypes.c_int(0)
    if lib().oracle_der_decode(sig, len(sig), r, s, ctypes.byref(rb), ctypes.byref(sb)):
        return None
    return (int.from_bytes(r.raw, "big") if not rb.value else 1 << 256,
            int.from_bytes(s.raw, "big") if not sb.value else 1 << 256)


def verify_der(qx: bytes, qy: bytes, sig: bytes, digest: bytes, ossl: bool = False) -> int:
    """bccsp Verify(pk, sig, digest) status byte (0 = valid)."""
    f = lib().oracle_p256_verify_der_ossl if ossl else lib().oracle_p256_verify_der
    return f(qx, qy, sig, len(sig), digest, len(digest))


def verify_der_p384(pub96: bytes, sig: bytes, digest: bytes) -> int:
    """bccsp Verify for a P-384 key (X || Y, 96 bytes): Go-rule DER, the P-384 half order, then
    the equation (OpenSSL arithmetic) -- status byte, 0 = valid."""
    return lib().oracle_p384_verify_der(pub96[:48], pub96[48:96], sig, len(sig), digest, len(digest))


def identity_verify(qx: bytes, qy: bytes, msg: bytes, sig: bytes, ossl: bool = False) -> int:
    """msp identity.Verify(msg, sig): SHA-256 then bccsp Verify (msp/identities.go:170-199)."""
    return verify_der(qx, qy, sig, sha256(msg), ossl)


def base_mult(k: int):
    x = ctypes.create_string_buffer(32)
    y = ctypes.create_string_buffer(32)
    if lib().oracle_p256_base_mult(k.to_bytes(32, "big"), x, y):
        return None
    return x.raw, y.raw
