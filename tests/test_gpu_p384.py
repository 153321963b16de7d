"""GPU: P-384 identities verified per item (p384.hip).

fgv_p384_verify_msgs (bccsp Verify for P-384 keys) against the oracle on the vectors of
tests/test_p384.py (valid, tampered, high S, r >= n, malformed DER, off-curve keys, Q = +-G); then
C2-shaped blocks whose creators and endorsers include P-384 identities: every block final
(per-block status 0) and the flags equal to the oracle's, in both parse modes, through the group
(block and transaction plans) and the shard protocol."""
import hashlib

import numpy as np
import pytest

import oracle
from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks
from oracle import v20
from tests.test_p384 import vectors

pytestmark = pytest.mark.gpu
MODES = pytest.mark.parametrize("mode", [0, 1], ids=["devparse", "hostparse"])


def test_p384_verify_msgs_vectors():
    from fabric_amd import synth
    vec = vectors()
    keys = [v[0] for v in vec]
    sigs = [v[1] for v in vec]
    msgs = [v[4] for v in vec]
    exp = [oracle.verify_der_p384(v[0], v[1], hashlib.sha256(v[4]).digest()) for v in vec]
    assert exp.count(0) >= 30 and 1 in exp and 2 in exp and 3 in exp and 4 in exp and 5 in exp and 6 in exp
    eng = _lib.Engine(0)
    try:
        st = eng.verify_msgs_p384(np.frombuffer(b"".join(keys), np.uint8).reshape(-1, 96), msgs, sigs)
        bad = [(i, vec[i][3], int(st[i]), exp[i]) for i in range(len(vec)) if st[i] != exp[i]]
        assert not bad, bad[:10]
        # a second call: the keys' combs are cached
        k = synth.Key384(62, 0)
        ms = [b"m%d" % i * (i + 1) for i in range(40)]
        ss = [synth.sign384(k, hashlib.sha256(m).digest()) for m in ms]
        st = eng.verify_msgs_p384(np.frombuffer(k.pub * len(ms), np.uint8).reshape(-1, 96), ms, ss)
        assert list(st) == [0] * len(ms)
    finally:
        eng.close()


def _p384_net(seed=3):
    return blocks.Network(seed=seed, orgs=3, clients=60, p384_clients=8, p384_peers=1)


@MODES
def test_blocks_with_p384_identities(mode):
    """C2 blocks with P-384 creators (8 of 60 clients) and a P-384 endorsing peer: final per-block
    outcomes and the oracle's flags (VERDICT r5 next #6 done criterion)"""
    net = _p384_net()
    blks, labels = [], []
    for i in range(4):
        b, lab, _ = blocks.make_block(net, 150, number=1 + i, seed=80 + i)
        blks.append(b)
        labels.append(lab)
    model = v20.ChannelModel(net.channel, net.identities(), net.chaincodes)
    exp, n_final = v20.validate_blocks_outcomes(model, blks)
    assert n_final == 4 and all(e is not None for e in exp)
    for e, lab in zip(exp, labels):
        assert list(e) == [blocks.EXPECTED[x] for x in lab]
    eng = _lib.Engine(0)
    try:
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        eng.set_block_outcomes(True)
        got = eng.validate_blocks(blks)
        st, nf = eng.last_block_status(len(blks))
        assert nf == 4 and st == [0] * 4, st
        for b in range(4):
            assert list(got[b]) == list(exp[b]), b
        # the whole-batch contract too (no block leaves the engine)
        eng.set_block_outcomes(False)
        assert [list(f) for f in eng.validate_blocks(blks)] == [list(e) for e in exp]
    finally:
        eng.close()


@pytest.mark.parametrize("ndev", [2, 5])
def test_group_blocks_with_p384_identities(ndev):
    net = _p384_net(seed=4)
    blks = [blocks.make_block(net, 100, number=1 + i, seed=90 + i)[0] for i in range(3)]
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks)
    g = _lib.Group([0] * ndev)
    try:
        for e in g.engines:
            txvalidator.setup_channel(e, net.channel, net.identities(), net.chaincodes)
        assert [list(f) for f in g.validate_blocks(blks)] == [list(f) for f in exp]
    finally:
        g.close()


def test_p384_creator_high_s_and_bad_signature():
    """creator faults on P-384 identities: a high-S signature (P-384 half order) and a corrupted
    one are BAD_CREATOR_SIGNATURE (4), as the oracle says"""
    net = _p384_net(seed=5)
    p384 = [c for c in net.clients if c.kind == "p384"]
    force = [None] * 60
    for i in range(0, 60, 3):
        force[i] = ("high_s_creator", "bad_creator_sig", "clean")[(i // 3) % 3]
    txs = []
    b, lab, _ = blocks.make_block(net, 60, number=1, seed=7, force=force, out_txs=txs)
    assert any(t.creator.kind == "p384" and t.label == "high_s_creator" for t in txs) or p384
    exp = v20.validate_block(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), b)
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        for mode in (0, 1):
            eng.set_parse_mode(mode)
            assert list(eng.validate_blocks([b])[0]) == list(exp), mode
    finally:
        eng.close()
