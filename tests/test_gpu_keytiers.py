"""GPU parity of the key tiers: keys with a comb table (k_point28) and keys
without one (the variable-base kernels k_vb_mul / k_vb_fin) give the oracle's status bytes and
flags; a full comb cache changes speed, never results or return codes.

Reference: the verify itself is bccsp/sw/ecdsa.go:41-57 (any key, no per-key precomputation);
the MSP cache holds few identities and deserializes the rest on demand (msp/cache/cache.go:17-19),
so a peer meets cold keys all the time."""
import contextlib
import hashlib
import os
import random

import numpy as np
import pytest

import oracle
from fabric_amd import _lib, synth, txvalidator
from fabric_amd.synth import blocks
from oracle import v20
from tests.vectors import N, der_int, der_seq, edge_vectors, golden_cert_vectors

pytestmark = pytest.mark.gpu

CLIENT, PEER = 1 << 2, 1 << 3


@contextlib.contextmanager
def _env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def vb_engine():
    """every ad-hoc key on the variable-base kernels (no ad-hoc comb builds)"""
    with _env(FGV_ADHOC_COMB=10**9, FGV_PROMOTE_USES=10**9):
        eng = _lib.Engine(0)
    yield eng
    eng.close()


def _run(engine, vecs):
    K = np.frombuffer(b"".join(v[0] + v[1] for v in vecs), np.uint8).reshape(-1, 64)
    D = np.frombuffer(b"".join(v[3] for v in vecs), np.uint8).reshape(-1, 32)
    return engine.verify_batch(K, [v[2] for v in vecs], D)


def _vb_items(engine):
    return engine.key_stats()["vb_verifies_last"]


def test_vb_golden_reference_certs(vb_engine):
    vecs = golden_cert_vectors()
    st = _run(vb_engine, vecs)
    for i, v in enumerate(vecs):
        assert st[i] == v[4], v[5]
    assert _vb_items(vb_engine) > 0


@pytest.mark.parametrize("seed", [5, 6, 7])
def test_vb_edge_vectors(vb_engine, seed):
    vecs = edge_vectors(seed)
    st = _run(vb_engine, vecs)
    exp = [oracle.verify_der(*v[:4]) for v in vecs]
    mism = [(vecs[i][4], int(st[i]), exp[i]) for i in range(len(vecs)) if st[i] != exp[i]]
    assert not mism, mism[:10]


def test_vb_scalar_edges_and_exceptional_additions(vb_engine):
    """u2 * Q with Q = +-G, 2G and u1 = +-u2: the variable-base sum passes through doublings and
    infinity (complete formulas); digests at window boundaries and >= n."""
    vecs = []
    k = synth.Key(33, 0)
    for dg in [b"\xff" * 32, b"\x00" * 32, N.to_bytes(32, "big"), (N - 1).to_bytes(32, "big"), b"\x80" + b"\x00" * 31]:
        sig = synth.sign(k, dg)
        vecs.append((k.qx, k.qy, sig, dg))
        vecs.append((k.qx, k.qy, sig, bytes([dg[0] ^ 1]) + dg[1:]))
    rng = random.Random(8)
    for m in (1, N - 1, 2, 3):
        qx, qy = oracle.base_mult(m)
        for _ in range(12):
            s = rng.randrange(1, N // 2)
            r = rng.randrange(1, N)
            for e in (r, (N - r) % N, (m * r) % N, (N - m * r % N) % N, rng.randrange(N)):
                vecs.append((qx, qy, der_seq(der_int(r) + der_int(s)), e.to_bytes(32, "big")))
    st = _run(vb_engine, vecs)
    exp = [oracle.verify_der(*v) for v in vecs]
    assert list(st) == exp
    assert 1 in exp and 0 in exp


def test_vb_fused_msgs_and_bad_key(vb_engine):
    rng = random.Random(4)
    K, M, S, exp = [], [], [], []
    for i in range(200):
        k = synth.Key(121, i)  # every key distinct: all on the variable-base kernels
        m = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 2500)))
        sig = synth.sign(k, hashlib.sha256(m).digest(), high_s=(i % 13 == 0))
        if i % 7 == 0:
            m = m + b"!"
        qx, qy = k.qx, k.qy
        if i % 29 == 0:  # a point off the curve -> status 5 before any range check
            qy = bytes([qy[0] ^ 1]) + qy[1:]
        K.append(qx + qy)
        M.append(m)
        S.append(sig)
        exp.append(oracle.identity_verify(qx, qy, m, sig))
    st = vb_engine.verify_msgs(np.frombuffer(b"".join(K), np.uint8).reshape(-1, 64), M, S)
    assert list(st) == exp
    assert 5 in exp


def test_mixed_tiers_one_batch():
    """hot keys (>= FGV_ADHOC_COMB uses in the call) on the comb, one-off keys on the variable-base
    kernels, interleaved in one batch, with tampered digests on both"""
    with _env(FGV_ADHOC_COMB=16):
        eng = _lib.Engine(0)
    try:
        rng = random.Random(9)
        hot = [synth.Key(70, i) for i in range(4)]
        vecs = []
        for i in range(3000):
            k = hot[i % 4] if i % 3 else synth.Key(71, i)
            d = rng.randbytes(32)
            sig = synth.sign(k, d)
            if i % 11 == 0:
                d = bytes([d[0] ^ 2]) + d[1:]
            vecs.append((k.qx, k.qy, sig, d))
        st = _run(eng, vecs)
        exp = [oracle.verify_der(*v) for v in vecs]
        assert list(st) == exp
        ks = eng.key_stats()
        assert ks["comb"] == 4 and ks["vb"] == 1000, ks
        assert ks["vb_verifies_last"] == 1000
    finally:
        eng.close()


def test_register_past_comb_capacity():
    """more registered keys than comb slots -- no FGV_ENOMEM; the keys past the cache
    verify on the variable-base kernels, bit-exact (HBM-resident batch through the key ids)."""
    import torch
    eng = _lib.Engine(0, key_slots=4)
    try:
        keys = [synth.Key(90, i) for i in range(40)]
        ids = eng.keys_register(np.frombuffer(b"".join(k.pub for k in keys), np.uint8).reshape(-1, 64))
        assert len(set(ids.tolist())) == 40
        ks = eng.key_stats()
        assert ks["comb"] == 4 and ks["vb"] == 36, ks
        rng = random.Random(3)
        msgs, sigs, slot, exp = [], [], [], []
        for i in range(400):
            k = keys[i % 40]
            m = rng.randbytes(rng.randint(1, 900))
            s = synth.sign(k, hashlib.sha256(m).digest())
            if i % 9 == 0:
                m = m + b"x"
            msgs.append(m)
            sigs.append(s)
            slot.append(ids[i % 40])
            exp.append(oracle.identity_verify(k.qx, k.qy, m, s))
        ma, mo, ml = _lib.pack(msgs)
        sa, so, sl = _lib.pack(sigs)
        dev = torch.device("cuda", 0)

        def t(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).to(dev)
        d_m = torch.zeros(ma.size + 64, dtype=torch.uint8, device=dev)
        d_m[:ma.size] = torch.from_numpy(ma.copy()).to(dev)
        d_s = torch.zeros(sa.size + 64, dtype=torch.uint8, device=dev)
        d_s[:sa.size] = torch.from_numpy(sa.copy()).to(dev)
        d_st = torch.zeros(len(msgs), dtype=torch.uint8, device=dev)
        args = [t(mo, np.int64), t(ml, np.int32), t(so, np.int64), t(sl, np.int32), t(np.array(slot, np.uint32), np.int32)]
        torch.cuda.synchronize()
        eng.verify_msgs_dev(d_m.data_ptr(), args[0].data_ptr(), args[1].data_ptr(), d_s.data_ptr(), args[2].data_ptr(),
                            args[3].data_ptr(), args[4].data_ptr(), len(msgs), d_st.data_ptr())
        assert d_st.cpu().numpy().tolist() == exp
        # ad-hoc keys on top of a full comb cache: no ENOMEM either
        vecs = []
        for i in range(100):
            k = synth.Key(91, i)
            d = rng.randbytes(32)
            vecs.append((k.qx, k.qy, synth.sign(k, d), d))
        assert list(_run(eng, vecs)) == [0] * 100
    finally:
        eng.close()


def test_promotion_by_use():
    """variable-base keys whose verifies reach FGV_PROMOTE_USES get a comb table from the next call
    on (k_vb_mul queues them; built asynchronously); results are the same before, during and after"""
    with _env(FGV_ADHOC_COMB=10**9, FGV_PROMOTE_USES=8, FGV_PROMOTE_PER_CALL=8):
        eng = _lib.Engine(0, key_slots=16)
    try:
        keys = [synth.Key(95, i) for i in range(6)]
        rng = random.Random(5)
        vecs = []
        for i in range(120):
            k = keys[i % 6]
            d = rng.randbytes(32)
            vecs.append((k.qx, k.qy, synth.sign(k, d), d if i % 5 else rng.randbytes(32)))
        exp = [oracle.verify_der(*v) for v in vecs]
        assert list(_run(eng, vecs)) == exp
        assert eng.key_stats()["vb_verifies_last"] == 120
        # the next call starts the comb builds on a side stream and does not wait for them: its
        # items take either path, with the same results
        assert list(_run(eng, vecs)) == exp
        ks = eng.key_stats()  # (waits for the builds)
        assert ks["promoted"] == 6 and ks["comb"] == 6, ks
        assert list(_run(eng, vecs)) == exp
        assert eng.key_stats()["vb_verifies_last"] == 0
    finally:
        eng.close()


MODES = pytest.mark.parametrize("mode", [0, 1], ids=["devparse", "hostparse"])


@MODES
def test_churn_blocks_all_creators_distinct(mode):
    """C2 blocks whose creators are 3000 client identities (CLIENT role: variable-base kernels);
    the endorsing peers keep their combs.  Flags equal the restated committer's."""
    net = blocks.Network(seed=3, orgs=3, clients=3000)
    eng = _lib.Engine(0)
    try:
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        ks = eng.key_stats()
        assert ks["comb"] == 3 + 1 and ks["vb"] == 3000, ks  # the 3 peers and the forged identity hot, clients cold
        blks = [blocks.make_block(net, 500, number=1 + i, seed=40 + i)[0] for i in range(3)]
        got = eng.validate_blocks(blks)
        m = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
        exp = v20.validate_blocks(m, blks)
        for b, (g, e) in enumerate(zip(got, exp)):
            mism = [(i, int(g[i]), e[i]) for i in range(len(e)) if g[i] != e[i]]
            assert len(g) == len(e) and not mism, (b, mism[:10])
        assert eng.key_stats()["vb_verifies_last"] > 1000
    finally:
        eng.close()


def test_c4_churn_every_item_its_own_key():
    """C4-shaped batch (1.85 KB messages, the injected tamper / high-S / bad-DER / trailing mix) where
    every item has its own key, registered cold (fgv_keys_register_tiered, hot = 0): all on the
    variable-base kernels, HBM-resident, statuses equal the oracle's"""
    import torch
    from fabric_amd.synth.workloads import sig_pool
    n = 6000
    pool = sig_pool(n, seed=77, nkeys=n)
    eng = _lib.Engine(0)
    try:
        slots = eng.keys_register(np.frombuffer(b"".join(k.pub for k in pool["keys"]), np.uint8).reshape(-1, 64),
                                  hot=False)
        ks = eng.key_stats()
        assert ks["comb"] == 0 and ks["vb"] == n, ks
        msgs = pool["msgs"]
        dev = torch.device("cuda", 0)
        d_m = torch.zeros(msgs.size + 64, dtype=torch.uint8, device=dev)
        d_m[:msgs.size] = torch.from_numpy(msgs.reshape(-1).copy()).to(dev)
        sa, so, sl = _lib.pack(pool["sigs"])
        d_s = torch.zeros(sa.size + 64, dtype=torch.uint8, device=dev)
        d_s[:sa.size] = torch.from_numpy(sa.copy()).to(dev)

        def t(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a).view(dt).copy()).to(dev)
        hold = [t(np.arange(n, dtype=np.uint64) * np.uint64(msgs.shape[1]), np.int64),
                t(np.full(n, msgs.shape[1], np.uint32), np.int32), t(so, np.int64), t(sl, np.int32),
                t(slots[pool["key_index"]].astype(np.uint32), np.int32)]
        d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        eng.verify_msgs_dev(d_m.data_ptr(), hold[0].data_ptr(), hold[1].data_ptr(), d_s.data_ptr(),
                            hold[2].data_ptr(), hold[3].data_ptr(), hold[4].data_ptr(), n, d_st.data_ptr())
        st = d_st.cpu().numpy()
        exp = [oracle.identity_verify(pool["keys"][i].qx, pool["keys"][i].qy, msgs[i].tobytes(), pool["sigs"][i],
                                      ossl=True) for i in range(n)]
        assert st.tolist() == exp
        assert ((st == 0) == pool["expect_valid"]).all()
        assert eng.key_stats()["vb_verifies_last"] >= int((st == 0).sum())
        assert eng.timing()["vb_mul_ms"] > 0
    finally:
        eng.close()
