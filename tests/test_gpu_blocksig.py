"""GPU parity of fgv_blocks_verify_signed (VerifyBlock with the orderer-signature policy: the
signatures verified by the engine's P-256 kernels, the policy folded over the channel model)
against the oracle (oracle/blockverify.py) and the written-down reference semantics of
tests/blocksig_cases.py -- and the reference's own orderer signatures: blocks 1..19 of the v2.0
sample ledger."""
import pytest

from fabric_amd import _lib, txvalidator
from oracle import blockverify as BV
from oracle import v20
from tests import blocksig_cases as BC
from tests.test_oracle_blocksig import ledger_setup, tamper

pytestmark = pytest.mark.gpu


def _chain(c):
    if c is None:
        return None
    n, h = c
    st = _lib.ChainState(number=n, valid=1, has_hash=0 if h is None else 1)
    if h is not None:
        st.header_hash[:] = list(h)
    return st


def _engine(identities, config, channel):
    eng = _lib.Engine(0)
    txvalidator.setup_channel(eng, channel, identities, {}, config=config)
    return eng


def _compare(eng, model, blocks, chain, policy=None, bft=False):
    cc, cp = _chain(chain), BC.chain_dict(dict(chain=chain))
    got, unsup = eng.blocks_verify_signed(blocks, cc, policy=policy, bft=bft)
    exp = BV.verify_blocks(blocks, cp, sig=dict(model=model, policy=policy, bft=bft))
    assert [g[0] for g in got] == [e[0] for e in exp]
    for g, e in zip(got, exp):
        if e[2] is not None:
            assert g[3] == e[2] and g[4] == e[3]
    assert unsup == (BV.SIG_UNSUPPORTED in [e[0] for e in exp])
    if cp is not None and not unsup:
        assert cc.number == cp["number"]
        if cp.get("header_hash"):
            assert bytes(cc.header_hash) == cp["header_hash"]
    return [g[0] for g in got]


def test_reference_ledger_orderer_signatures():
    blocks, chain, idents, config = ledger_setup()
    eng = _engine(idents, config, "testchannel")
    model = v20.ChannelModel("testchannel", idents, {}, config=config)
    assert _compare(eng, model, blocks, chain) == [BV.OK] * 19
    bad = list(blocks[:6])
    bad[1] = tamper(bad[1], "sig")
    bad[4] = tamper(bad[4], "value")
    assert _compare(eng, model, bad, chain) == [BV.OK, BV.SIGNATURES] + [BV.NUMBER] * 4
    eng.close()
    # the orderer's certificate unregistered: resolved through OrdererOrgMSP (MSP cache miss)
    idents2 = [(s, i) for s, i in idents if i.mspid != "OrdererOrgMSP"]
    eng = _engine(idents2, config, "testchannel")
    model = v20.ChannelModel("testchannel", idents2, {}, config=config)
    assert _compare(eng, model, blocks[:3], chain) == [BV.OK] * 3
    eng.close()


def test_reference_semantics_cases():
    engines = {}
    try:
        for case in BC.cases():
            key = (case["config"], case["drop"])
            if key not in engines:
                engines[key] = _engine(BC.identities_for(case), BC.config_for(case), BC.world()[0].channel)
            st = _compare(engines[key], BC.oracle_model(case), case["blocks"], case["chain"], case["policy"],
                          case["bft"])
            assert st == case["expect"], case["name"]
    finally:
        for e in engines.values():
            e.close()


def test_many_blocks_one_pass():
    """64 signed blocks, 3 signers each (one bad in every 5th block, all bad in every 7th): one
    GPU verify pass for the call, statuses and chain equal the oracle's"""
    from fabric_amd.synth import orderer as OR
    net, ords, ids, cfg = BC.world()
    raw, hashes = BC.chain_blocks(net, 64, seed=9, ntx=2)
    blocks = []
    for i, b in enumerate(raw):
        bad = (0, 1, 2) if i % 7 == 6 else (1,) if i % 5 == 0 else ()
        blocks.append(OR.sign_block(b, [ords.nodes[0], ords.nodes[2], ords.nodes[3]], bad=bad, nonce_seed=i))
    eng = _engine(ids, cfg["majority"], net.channel)
    model = v20.ChannelModel(net.channel, ids, {}, config=cfg["majority"])
    st = _compare(eng, model, blocks, (0, None))
    assert st[:6] == [BV.OK] * 6 and st[6] == BV.SIGNATURES and st[7] == BV.NUMBER
    eng.close()
