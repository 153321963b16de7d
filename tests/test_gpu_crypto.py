"""GPU parity: libfgv (HIP on MI355X) vs the oracle, bit-exact status bytes."""
import hashlib
import random

import numpy as np
import pytest

import oracle
from fabric_amd import synth
from fabric_amd._lib import SIG_VALID, Engine
from tests.vectors import N, edge_vectors, golden_cert_vectors

pytestmark = pytest.mark.gpu


def _run(engine, vecs):
    K = np.frombuffer(b"".join(v[0] + v[1] for v in vecs), np.uint8).reshape(-1, 64)
    D = np.frombuffer(b"".join(v[3] for v in vecs), np.uint8).reshape(-1, 32)
    return engine.verify_batch(K, [v[2] for v in vecs], D)


def test_golden_reference_certs(engine):
    vecs = golden_cert_vectors()
    st = _run(engine, vecs)
    for i, v in enumerate(vecs):
        assert st[i] == v[4], v[5]


@pytest.mark.parametrize("seed", [5, 6, 7])
def test_edge_vectors_match_oracle(engine, seed):
    vecs = edge_vectors(seed)
    st = _run(engine, vecs)
    exp = [oracle.verify_der(*v[:4]) for v in vecs]
    mism = [(vecs[i][4], int(st[i]), exp[i]) for i in range(len(vecs)) if st[i] != exp[i]]
    assert not mism, mism[:10]


def test_sha256_all_padding_lengths_and_alignments(engine):
    rng = random.Random(2)
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in list(range(0, 260)) + [1000, 1851, 4700, 7500, 65537]]
    # misalign every message start by packing odd-length blobs back to back
    dg = engine.sha256_batch(msgs)
    for i, m in enumerate(msgs):
        assert bytes(dg[i]) == hashlib.sha256(m).digest(), len(m)


def test_fused_verify_msgs_matches_oracle(engine):
    rng = random.Random(4)
    keys = [synth.Key(21, i) for i in range(5)]
    K, M, S, exp = [], [], [], []
    for i in range(300):
        k = keys[i % 5]
        m = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 2500)))
        sig = synth.sign(k, hashlib.sha256(m).digest(), high_s=(i % 13 == 0))
        if i % 7 == 0:
            m = m + b"!"
        K.append(k.pub); M.append(m); S.append(sig)
        exp.append(oracle.identity_verify(k.qx, k.qy, m, sig))
    st = engine.verify_msgs(np.frombuffer(b"".join(K), np.uint8).reshape(-1, 64), M, S)
    assert list(st) == exp


def test_scalar_edge_cases(engine):
    """u1 or u2 hitting window boundaries; r close to n; e >= n (digest all ones)."""
    k = synth.Key(33, 0)
    vecs = []
    for dg in [b"\xff" * 32, b"\x00" * 32, N.to_bytes(32, "big"), (N - 1).to_bytes(32, "big"), b"\x80" + b"\x00" * 31]:
        sig = synth.sign(k, dg)
        vecs.append((k.qx, k.qy, sig, dg))
        vecs.append((k.qx, k.qy, sig, bytes([dg[0] ^ 1]) + dg[1:]))
    st = _run(engine, vecs)
    assert list(st) == [oracle.verify_der(*v) for v in vecs]


def test_adversarial_exceptional_additions(engine):
    """Q = G and Q = -G style keys make partial sums collide: exercises the complete
    mixed-addition branches (doubling / infinity)."""
    gx = bytes.fromhex("6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296")
    x, y = oracle.base_mult(1)
    x2, y2 = oracle.base_mult(N - 1)
    x3, y3 = oracle.base_mult(2)
    rng = random.Random(8)
    vecs = []
    for qx, qy in [(x, y), (x2, y2), (x3, y3)]:
        for _ in range(40):
            # r, s chosen so that u1 = -u2 (R = inf) or u1 = u2 (doubling) for Q = +-G
            s = rng.randrange(1, N // 2)
            r = rng.randrange(1, N)
            e_same = r          # u1 = e/s, u2 = r/s: e == r -> u1 == u2
            e_neg = (N - r) % N  # e == -r -> u1 == -u2
            for e in (e_same, e_neg, rng.randrange(N)):
                from tests.vectors import der_int, der_seq
                vecs.append((qx, qy, der_seq(der_int(r) + der_int(s)), e.to_bytes(32, "big")))
    st = _run(engine, vecs)
    exp = [oracle.verify_der(*v) for v in vecs]
    assert list(st) == exp
    # sanity: the constructed cases do reach the infinity path (status 1) and doubling path,
    # and the fast kernel handed exactly those items to the complete-formula kernel
    assert 1 in exp
    assert engine.point_handovers() > 0


def test_honest_batch_needs_no_handover(engine):
    """Random honest signatures never hit an exceptional addition in the fast kernel."""
    rng = random.Random(21)
    k = synth.Key(44, 0)
    vecs = []
    for i in range(512):
        dg = rng.randbytes(32)
        vecs.append((k.qx, k.qy, synth.sign(k, dg), dg if i % 7 else bytes([dg[0] ^ 4]) + dg[1:]))
    st = _run(engine, vecs)
    assert list(st) == [oracle.verify_der(*v) for v in vecs]
    assert engine.point_handovers() == 0


def test_large_batch_properties(engine):
    """At scale: all-valid batch -> all 0; flipping digests -> all 1 (size-independent check)."""
    n = 65536
    keys = [synth.Key(77, i) for i in range(16)]
    base = []
    for i in range(512):
        d = hashlib.sha256(b"b%d" % i).digest()
        base.append((keys[i % 16], d, synth.sign(keys[i % 16], d)))
    K = np.frombuffer(b"".join(base[i % 512][0].pub for i in range(n)), np.uint8).reshape(-1, 64)
    D = np.frombuffer(b"".join(base[i % 512][1] for i in range(n)), np.uint8).reshape(-1, 32).copy()
    S = [base[i % 512][2] for i in range(n)]
    assert (engine.verify_batch(K, S, D) == SIG_VALID).all()
    D[::3, 5] ^= 0x10
    st = engine.verify_batch(K, S, D)
    assert (st[::3] == 1).all()
    mask = np.ones(n, bool); mask[::3] = False
    assert (st[mask] == 0).all()


def test_key_cache_eviction():
    """A tiny comb cache: hot keys beyond it run on the variable-base kernels; results never change."""
    eng = Engine(0, key_slots=3)
    try:
        keys = [synth.Key(55, i) for i in range(3)]
        for rnd in range(3):
            vecs = []
            for i in range(30):
                k = keys[(i + rnd) % 3] if rnd < 2 else synth.Key(56 + rnd, i % 3)
                d = hashlib.sha256(b"%d-%d" % (rnd, i)).digest()
                vecs.append((k.qx, k.qy, synth.sign(k, d), d))
            assert list(_run(eng, vecs)) == [0] * 30
        # more distinct hot keys than comb slots in one batch: the keys past the cache verify on
        # the variable-base kernels -- no FGV_ENOMEM since round 4
        vecs = []
        for i in range(40 * 5):
            k = synth.Key(90, i % 5)
            d = hashlib.sha256(b"%d" % i).digest()
            vecs.append((k.qx, k.qy, synth.sign(k, d), d if i % 3 else d[::-1]))
        assert list(_run(eng, vecs)) == [oracle.verify_der(*v) for v in vecs]
    finally:
        eng.close()


def test_c4_per_gpu_shard_full_size():
    """BASELINE configs[3] per-GPU share: 131,072 identity.Verify items (1.85 KB messages, the C4
    fault mix: tampered, high-S, bad DER, trailing bytes) through the HBM-resident path the bench
    times; every status agrees with the generator's verdict and a 2,048-item sample with the
    oracle's exact status byte."""
    import torch
    from fabric_amd._lib import pack
    from fabric_amd.synth.workloads import sig_pool
    n, uniq = 131072, 16384
    pool = sig_pool(uniq, seed=1000)
    eng = Engine(0)
    try:
        slots_u = eng.keys_register(np.frombuffer(b"".join(k.pub for k in pool["keys"]), np.uint8).reshape(-1, 64))
        idx = np.arange(n) % uniq
        msgs = np.ascontiguousarray(pool["msgs"][idx])
        dev = torch.device("cuda", 0)
        d_msg = torch.zeros(msgs.size + 64, dtype=torch.uint8, device=dev)
        d_msg[: msgs.size].copy_(torch.from_numpy(msgs.reshape(-1)))
        d_moff = torch.from_numpy((np.arange(n, dtype=np.uint64) * np.uint64(msgs.shape[1])).view(np.int64)).to(dev)
        d_mlen = torch.from_numpy(np.full(n, msgs.shape[1], np.uint32).view(np.int32)).to(dev)
        sa, so, sl = pack([pool["sigs"][i] for i in idx])
        d_sig = torch.zeros(sa.size + 64, dtype=torch.uint8, device=dev)
        d_sig[: sa.size].copy_(torch.from_numpy(sa.copy()))
        d_soff = torch.from_numpy(so.view(np.int64).copy()).to(dev)
        d_slen = torch.from_numpy(sl.view(np.int32).copy()).to(dev)
        d_slot = torch.from_numpy(slots_u[pool["key_index"][idx]].astype(np.uint32).view(np.int32)).to(dev)
        d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
        eng.verify_msgs_dev(d_msg.data_ptr(), d_moff.data_ptr(), d_mlen.data_ptr(), d_sig.data_ptr(), d_soff.data_ptr(),
                            d_slen.data_ptr(), d_slot.data_ptr(), n, d_st.data_ptr())
        st = d_st.cpu().numpy()
        assert ((st == 0) == pool["expect_valid"][idx]).all()
        for i in range(0, uniq, 8):
            k = pool["keys"][pool["key_index"][i]]
            assert st[i] == oracle.identity_verify(k.pub[:32], k.pub[32:], pool["msgs"][i].tobytes(), pool["sigs"][i]), i
    finally:
        eng.close()
