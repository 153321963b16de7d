"""GPU unit test of the device txid decoder hex64_words (fin_dev.h): the 64-character
TxId of a channel header -> 32 bytes, false on anything but lowercase hex (the index keys of
k_fin_rows / k_fin_index_dev / k_bd_fold).  Every alignment (offset mod 4), a bad character
(uppercase, non-hex, NUL, high byte) at the first / middle / last position, and a txid ending at
the last byte before the buffer's 64-byte tail padding, against bytes.fromhex."""
import ctypes
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
LIB = os.path.join(os.path.dirname(__file__), "gpu_helpers", "libhexcheck.so")


def test_hex64_words_alignments_and_bad_characters():
    L = ctypes.CDLL(LIB)
    rng = random.Random(7)
    buf = bytearray()
    cases = []  # (offset, text)
    for k in range(400):
        pad = rng.randrange(0, 7)
        buf += bytes(rng.randrange(256) for _ in range(pad))
        txt = bytearray(rng.randbytes(32).hex().encode())
        if k % 3 == 0:
            pos = [0, 31, 32, 63][k % 4]
            txt[pos] = rng.choice(b"ABCDEFGZ:/@`g\x00\xff ")
        cases.append((len(buf), bytes(txt)))
        buf += txt
    # the last one ends at the buffer's last byte (the contract: >= 64 bytes of tail padding)
    last = rng.randbytes(32).hex().encode()
    cases.append((len(buf), last))
    buf += last
    offs = np.array([o for o, _ in cases], np.uint32)
    assert len({int(o) % 4 for o in offs}) == 4
    ok = np.zeros(len(cases), np.uint8)
    out = np.zeros((len(cases), 8), np.uint32)
    b = np.frombuffer(bytes(buf), np.uint8)
    rc = L.hexcheck_run(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(len(b)), offs.ctypes.data_as(ctypes.c_void_p),
                        ctypes.c_size_t(len(cases)), ok.ctypes.data_as(ctypes.c_void_p),
                        out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    for i, (o, txt) in enumerate(cases):
        good = all(c in b"0123456789abcdef" for c in txt)
        assert bool(ok[i]) == good, (i, txt)
        if good:
            assert out[i].astype("<u4").tobytes() == bytes.fromhex(txt.decode()), i
