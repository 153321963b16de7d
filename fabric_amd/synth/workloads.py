"""Synthetic workloads with the shapes of BASELINE.json configs.

sig_pool(): the C1/C4 generator -- endorsement-shaped messages (~1.85 KB uniform random
bytes), 16 P-256 signing keys, low-S DER signatures from OpenSSL, and the injected mix
1 % message bit flip, 0.5 % high-S twin, 0.5 % malformed DER, 0.1 % trailing bytes after
the DER SEQUENCE (valid under Go's rules).  Each item carries its label; `expect_valid`
is what the label implies for the reference (a generation-time fact, not an oracle call).
"""
import hashlib

import numpy as np

from . import Key, sign_batch

N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
LABELS = ("clean", "msg_flip", "high_s", "bad_der", "trailing")


def _der_int(x):
    b = x.to_bytes((x.bit_length() + 7) // 8 or 1, "big")
    if b[0] & 0x80:
        b = b"\x00" + b
    return b"\x02" + bytes([len(b)]) + b


def _der_rs(sig):
    rl = sig[3]
    r = int.from_bytes(sig[4:4 + rl], "big")
    sl = sig[5 + rl]
    s = int.from_bytes(sig[6 + rl:6 + rl + sl], "big")
    return r, s


def sig_pool(n, seed=1, msg_len=1850, nkeys=16, threads=8):
    keys = [Key(seed, i) for i in range(nkeys)]
    rng = np.random.default_rng(seed + 1)
    msgs = rng.integers(0, 256, size=(n, msg_len), dtype=np.uint8)
    digests = b"".join(hashlib.sha256(msgs[i].tobytes()).digest() for i in range(n))
    privs = b"".join(keys[i % nkeys].priv for i in range(n))
    sigs = sign_batch(privs, digests, n, threads=threads)
    u = rng.random(n)
    label = np.zeros(n, dtype=np.uint8)
    label[u < 0.010] = 1
    label[(u >= 0.010) & (u < 0.015)] = 2
    label[(u >= 0.015) & (u < 0.020)] = 3
    label[(u >= 0.020) & (u < 0.021)] = 4
    for i in np.nonzero(label)[0]:
        if label[i] == 1:
            msgs[i, int(rng.integers(msg_len))] ^= 1 << int(rng.integers(8))
        elif label[i] == 2:
            r, s = _der_rs(sigs[i])
            body = _der_int(r) + _der_int(N - s)
            sigs[i] = b"\x30" + bytes([len(body)]) + body
        elif label[i] == 3:
            sigs[i] = sigs[i][:-1] if i % 2 else b"\x30\x81" + sigs[i][1:]
        elif label[i] == 4:
            sigs[i] = sigs[i] + b"\x05\x00"
    keymat = np.frombuffer(b"".join(keys[i % nkeys].pub for i in range(n)), np.uint8).reshape(n, 64)
    expect_valid = (label == 0) | (label == 4)
    return dict(keys=keys, keymat=keymat, msgs=msgs, sigs=sigs, label=label, expect_valid=expect_valid,
                key_index=np.arange(n) % nkeys)
