"""GPU: one context called from many host threads at once, and the asynchronous comb promotion
landing at chosen points of a batch's verify chain.

The reference calls the BCCSP seam from up to validatorPoolSize goroutines at once
(core/committer/txvalidator/v20/validator.go:193-208: one goroutine per transaction, each ending
in bccsp/sw/impl.go:247-270 Verify), and a peer's committer calls TxValidator.Validate while its
endorser / gossip paths verify signatures.  The engine serialises a context's calls on its mutex
(fgv_host.cpp); these tests check that concurrent callers of one context each get exactly the
oracle's answer for their own inputs.

Promotion: a key whose variable-base verifies reach FGV_PROMOTE_USES gets a comb
table built on a side stream, and k_kmap_set switches its id to the comb slot while later batches
may be in flight.  FGV_PROMOTE_AT=1/2/3 (a test knob) builds the tables first and enqueues that
k_kmap_set on the main stream after k_inv / before k_point28 / before k_vb_fin of the consuming
batch, so each interleaving runs deterministically once -- also with comb slots that another
key's table occupied before fgv_keys_reset."""
import contextlib
import hashlib
import os
import random
import threading

import numpy as np
import pytest

import oracle
from fabric_amd import _lib, synth, txvalidator
from fabric_amd.synth import blocks
from oracle import v20

pytestmark = pytest.mark.gpu


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


def _vecs(keys, n, seed, cycle=False):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        k = keys[i % len(keys)] if cycle else keys[rng.randrange(len(keys))]
        m = rng.randbytes(40 + rng.randrange(300))
        sig = synth.sign(k, hashlib.sha256(m).digest(), high_s=(i % 29 == 7))
        if i % 11 == 3:
            m = m + b"x"  # tampered message
        if i % 37 == 5:
            sig = sig[:-1]  # malformed DER
        out.append((k, m, sig))
    return out


def _verify(eng, vecs):
    K = np.frombuffer(b"".join(k.pub for k, _, _ in vecs), np.uint8).reshape(-1, 64)
    return list(eng.verify_msgs(K, [m for _, m, _ in vecs], [s for _, _, s in vecs]))


def _expect(vecs):
    return [oracle.identity_verify(k.pub[:32], k.pub[32:], m, s) for k, m, s in vecs]


def test_eight_threads_one_context():
    """8 host threads on ONE context: 4 call fgv_p256_verify_msgs (hot, cold and fresh ad-hoc keys:
    comb, variable-base and promotion paths), 4 call fgv_validate_blocks on their own blocks;
    every result equals the oracle's"""
    net = blocks.Network(seed=3, orgs=3, clients=300)
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        hot = [synth.Key(501, i) for i in range(4)]
        blks = [[blocks.make_block(net, 120, number=1 + 3 * w + j, seed=700 + 3 * w + j)[0] for j in range(2)]
                for w in range(4)]
        m = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
        exp_blk = [v20.validate_blocks(m, b) for b in blks]
        jobs = []
        for w in range(4):
            keys = hot + [synth.Key(600 + w, i) for i in range(40)]  # 40 cold / ad-hoc keys each
            batches = [_vecs(keys, 300, 1000 * w + r) for r in range(3)]
            jobs.append((batches, [_expect(b) for b in batches]))
        errors = []
        start = threading.Barrier(8)

        def sig_worker(w):
            try:
                start.wait()
                for it in range(3):
                    for vecs, exp in zip(*jobs[w]):
                        got = _verify(eng, vecs)
                        if got != exp:
                            errors.append(("sig", w, it, [i for i in range(len(exp)) if got[i] != exp[i]][:8]))
            except Exception as e:  # noqa: BLE001
                errors.append(("sig", w, repr(e)))

        def blk_worker(w):
            try:
                start.wait()
                for it in range(3):
                    got = eng.validate_blocks(blks[w])
                    for b, (g, e) in enumerate(zip(got, exp_blk[w])):
                        if list(g) != list(e):
                            errors.append(("blk", w, it, b, [i for i in range(len(e)) if g[i] != e[i]][:8]))
            except Exception as e:  # noqa: BLE001
                errors.append(("blk", w, repr(e)))

        th = [threading.Thread(target=sig_worker, args=(w,)) for w in range(4)]
        th += [threading.Thread(target=blk_worker, args=(w,)) for w in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in th), "a worker did not finish"
        assert not errors, errors[:5]
    finally:
        eng.close()


@pytest.mark.parametrize("at", [1, 2, 3], ids=["after_inv", "before_point28", "before_vb_fin"])
def test_promotion_lands_mid_batch(at):
    """the promotion's k_kmap_set enqueued at a fixed point of the consuming batch's chain; the
    comb slots first hold other keys' tables (registered ad-hoc comb keys, then fgv_keys_reset),
    so a stale table in a reused slot would show as wrong statuses"""
    with _env(FGV_ADHOC_COMB=64, FGV_PROMOTE_USES=8, FGV_PROMOTE_PER_CALL=8, FGV_PROMOTE_AT=at):
        eng = _lib.Engine(0, key_slots=8)
    try:
        # 1) 8 ad-hoc keys used >= 64 times: they take all 8 comb slots
        first = [synth.Key(810 + at, i) for i in range(8)]
        v1 = _vecs(first, 8 * 70, 11, cycle=True)
        assert _verify(eng, v1) == _expect(v1)
        assert eng.key_stats()["comb"] == 8
        # 2) flush the ad-hoc ids: the slots are free, their old tables stay in HBM
        eng.keys_reset()
        # 3) 6 new keys used 20 times each: variable-base (no comb at 20 < 64 uses), queued for
        # promotion (>= 8 uses)
        fresh = [synth.Key(820 + at, i) for i in range(6)]
        v2 = _vecs(fresh, 120, 12, cycle=True)
        exp2 = _expect(v2)
        assert _verify(eng, v2) == exp2
        ks = eng.key_stats()
        assert ks["vb"] == 6 and ks["vb_verifies_last"] > 0, ks
        # 4) the consuming call: tables built into the reused slots, kmap switched at point `at`
        assert _verify(eng, v2) == exp2
        ks = eng.key_stats()
        assert ks["promoted"] == 6 and ks["comb"] == 6, ks
        # 5) now on the comb path, through the reused slots
        assert _verify(eng, v2) == exp2
        assert eng.key_stats()["vb_verifies_last"] == 0
    finally:
        eng.close()
