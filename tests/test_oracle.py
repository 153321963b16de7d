"""CPU tests: the oracle against golden vectors, hashlib and OpenSSL (pins the oracle)."""
import hashlib
import random

import numpy as np
import pytest

import oracle
from fabric_amd import synth
from tests.vectors import N, edge_vectors, golden_cert_vectors


def test_sha256_fips_kats():
    # FIPS 180-2 Appendix B known answers
    assert oracle.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert oracle.sha256(b"").hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
    assert oracle.sha256(b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq").hex() == \
        "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"


def test_sha256_vs_hashlib_all_padding_lengths():
    rng = random.Random(1)
    for n in list(range(0, 200)) + [1000, 4096, 7500]:
        m = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.sha256(m) == hashlib.sha256(m).digest(), n


def test_golden_reference_cert_signatures():
    """CA signatures held in the reference's own MSP fixtures (incl. the high-S one)."""
    vecs = golden_cert_vectors()
    assert len(vecs) >= 100
    for qx, qy, sig, dg, exp, label in vecs:
        assert oracle.verify_der(qx, qy, sig, dg) == exp, label
        assert oracle.verify_der(qx, qy, sig, dg, ossl=True) == exp, label


def test_reference_high_s_fixture():
    # msp/msp_test.go:1524-1535: peer0-cert.pem in testdata/mspid is high-S
    vecs = [v for v in golden_cert_vectors() if "mspid/" in v[5] and "reference-cert" in v[5]]
    assert vecs and all(v[4] == 3 for v in vecs)


@pytest.mark.parametrize("seed", [5, 6])
def test_edge_vectors_oracle_vs_openssl(seed):
    """Both arithmetic back-ends agree on every Go acceptance rule."""
    for qx, qy, sig, dg, label in edge_vectors(seed):
        a = oracle.verify_der(qx, qy, sig, dg)
        b = oracle.verify_der(qx, qy, sig, dg, ossl=True)
        assert a == b, label


def test_edge_vectors_expected_classes():
    got = {}
    for qx, qy, sig, dg, label in edge_vectors(5):
        got.setdefault(label, set()).add(oracle.verify_der(qx, qy, sig, dg))
    assert got["valid"] == {0}
    assert got["trailing bytes after SEQUENCE (Go accepts)"] == {0}
    assert got["extra element inside SEQUENCE (Go accepts)"] == {0}
    assert got["garbage after S inside SEQUENCE (Go accepts)"] == {0}
    assert got["high-S twin"] == {3}
    for lab in ["truncated", "SET instead of SEQUENCE", "indefinite length", "non-minimal long-form length",
                "non-minimal INTEGER", "s = 0", "r = 0", "r negative", "empty INTEGER", "missing S", "junk",
                "high-tag-number form"]:
        assert got[lab] == {2}, lab
    assert got["r >= n"] == {4} and got["r >= 2^256"] == {4}
    assert got["empty signature"] == {6}
    assert got["digest flipped"] == {1} and got["wrong key"] == {1}
    assert got["key not on curve"] == {5} and got["key x >= p"] == {5}


def test_random_signatures_oracle_vs_openssl():
    rng = random.Random(3)
    keys = [synth.Key(9, i) for i in range(4)]
    for i in range(60):
        k = keys[i % 4]
        d = bytes(rng.getrandbits(8) for _ in range(32))
        sig = synth.sign(k, d)
        assert oracle.verify_der(k.qx, k.qy, sig, d) == 0
        d2 = bytes([d[0] ^ 1]) + d[1:]
        assert oracle.verify_der(k.qx, k.qy, sig, d2) == oracle.verify_der(k.qx, k.qy, sig, d2, ossl=True) == 1


def test_base_mult_known_answer():
    # 1*G and (n-1)*G = -G
    gx = "6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296"
    x, y = oracle.base_mult(1)
    assert x.hex() == gx
    x2, y2 = oracle.base_mult(N - 1)
    assert x2 == x and int.from_bytes(y2, "big") == (2**256 - 2**224 + 2**192 + 2**96 - 1) - int.from_bytes(y, "big")
    assert oracle.base_mult(N) is None


def test_threaded_batch_matches_single():
    keys = [synth.Key(4, i) for i in range(3)]
    msgs = [b"x" * (i * 7) for i in range(40)]
    sigs = [synth.sign(keys[i % 3], hashlib.sha256(m).digest(), high_s=(i % 9 == 0)) for i, m in enumerate(msgs)]
    import ctypes
    from fabric_amd._lib import pack
    K = np.frombuffer(b"".join(keys[i % 3].pub for i in range(40)), np.uint8)
    ma, mo, ml = pack(msgs)
    sa, so, sl = pack(sigs)
    for ossl in (0, 1):
        st = np.zeros(40, np.uint8)
        oracle.lib().oracle_verify_msgs_batch(K.ctypes.data, ma.ctypes.data, mo.ctypes.data, ml.ctypes.data,
                                              sa.ctypes.data, so.ctypes.data, sl.ctypes.data, 40, st.ctypes.data,
                                              4, ossl)
        exp = [oracle.identity_verify(keys[i % 3].qx, keys[i % 3].qy, msgs[i], sigs[i]) for i in range(40)]
        assert list(st) == exp
