"""GPU parity of the channel model: the default Fabric v2 endorsement policy (ImplicitMeta
MAJORITY over org Endorsement = OR('OrgN.peer'), NodeOU roles), collection endorsement
policies (explicit, defaulting to the chaincode EP, implicit org collections, undefined ->
policy failure), the reference's own v2.0 sample ledger, and the inputs that must come out
FGV_EUNSUPPORTED rather than as a guess (unregistered channel identity, P-384 key, SHA3 MSP,
non-vscc plugin, role principal without role bits).  Device parse and host parse both."""
import copy

import dataclasses

import pytest

from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks, chanconfig
from oracle import v20

pytestmark = pytest.mark.gpu
MODES = [0, 1]


def _engine(net, chaincodes, config=None, identities=None, mode=0):
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, net.channel, identities if identities is not None else net.identities(),
                              chaincodes, config=config)
    return eng


def _oracle(net, chaincodes, config=None, identities=None):
    return v20.ChannelModel(net.channel, identities if identities is not None else net.identities(), chaincodes,
                            config=config)


@pytest.mark.parametrize("mode", MODES)
def test_default_v2_endorsement_policy(mode):
    """C2 shape with /Channel/Application/Endorsement (MAJORITY of org Endorsement policies,
    each OR('OrgN.peer')): flags bit-exact with the oracle and the generator labels, nothing
    unsupported."""
    net = blocks.Network(seed=3, orgs=3, clients=30)
    cfg = chanconfig.make_config(net.mspids)
    ccs = {"mycc": chanconfig.channel_ref("/Channel/Application/Endorsement")}
    eng = _engine(net, ccs, cfg, mode=mode)
    model = _oracle(net, ccs, cfg)
    for b in range(2):
        blk, labels, _ = blocks.make_block(net, 400, number=1 + b, seed=50 + b)
        exp = v20.validate_block(model, blk)
        got = list(eng.validate_blocks([blk])[0])
        assert got == exp, b
        known = [(g, e) for g, e in zip(got, blocks.expected_codes(labels)) if e is not None]
        assert all(g == e for g, e in known)
        assert 10 in got and 0 in got
    eng.close()


@pytest.mark.parametrize("mode", MODES)
def test_implicit_meta_unknown_rule(mode):
    """/Channel/Application/Endorsement with an ImplicitMeta rule outside ANY/ALL/MAJORITY:
    threshold 0, and implicitmeta.go:85-103 counts `remaining` down from 0 -- a tx passes only
    when NO org Endorsement policy is satisfied (properly endorsed txs fail with 10)."""
    net = blocks.Network(seed=3, orgs=3, clients=30)
    cfg = chanconfig.make_config(net.mspids, endorsement_rule=7)
    ccs = {"mycc": chanconfig.channel_ref("/Channel/Application/Endorsement")}
    eng = _engine(net, ccs, cfg, mode=mode)
    blk, labels, _ = blocks.make_block(net, 300, number=1, seed=21)
    exp = v20.validate_block(_oracle(net, ccs, cfg), blk)
    got = list(eng.validate_blocks([blk])[0])
    assert got == exp
    clean = [g for g, lab in zip(got, labels) if lab == "clean"]
    assert clean and all(g == 10 for g in clean)
    eng.close()


@pytest.mark.parametrize("mode", MODES)
def test_peer_role_required(mode):
    """The same policy with endorsers registered as CLIENTs: every endorsement fails its org's
    OR('OrgN.peer') -> ENDORSEMENT_POLICY_FAILURE (oracle agrees)."""
    net = blocks.Network(seed=3, orgs=3, clients=30)
    ids = [(s, txvalidator.Identity(i.mspid, i.pub, i.valid, i.id_digest, key=i.key,
                                    roles=(i.roles & ~(1 << 3)) | (1 << 2) if i.roles else i.roles))
           for s, i in net.identities()]
    cfg = chanconfig.make_config(net.mspids)
    ccs = {"mycc": chanconfig.channel_ref("/Channel/Application/Endorsement")}
    eng = _engine(net, ccs, cfg, ids, mode=mode)
    blk, labels, _ = blocks.make_block(net, 200, number=1, seed=7)
    exp = v20.validate_block(_oracle(net, ccs, cfg, ids), blk)
    got = list(eng.validate_blocks([blk])[0])
    assert got == exp and 0 not in got
    eng.close()


@pytest.mark.parametrize("mode", MODES)
def test_collection_endorsement_policies(mode):
    """Hashed writes into: collA (own EP: OR('Org3MSP.peer')), collB (no EP: the chaincode EP),
    _implicit_org_Org1MSP (/Channel/Application/org1/Endorsement), nosuch (undefined -> 10)."""
    net = blocks.Network(seed=3, orgs=3, clients=30)
    cfg = chanconfig.make_config(net.mspids)
    coll_a = b"\x0a" + bytes([0]) + b""  # placeholder replaced below
    spe_a = chanconfig.signature_policy(1, [("Org3MSP", chanconfig.PEER)])
    coll_a = blocks.f_msg(1, spe_a)  # ApplicationPolicy{signature_policy}
    ccs = {"mycc": {"policy": blocks.out_of_policy(2, net.mspids), "collections": {"collA": coll_a, "collB": None}}}
    eng = _engine(net, ccs, cfg, mode=mode)
    model = _oracle(net, ccs, cfg)
    blk, labels, _ = blocks.make_block(net, 400, number=1, seed=9,
                                       collections=["collA", "collB", "_implicit_org_Org1MSP", "nosuch"])
    exp = v20.validate_block(model, blk)
    got = list(eng.validate_blocks([blk])[0])
    assert got == exp
    assert got.count(0) > 50 and got.count(10) > 50
    eng.close()


def _v20_engine(mode, idents, config):
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, "testchannel", idents, {}, config=config)
    return eng


def _define(eng, defs):
    for ns, d in defs.items():
        colls = d.get("collections")
        eng.chaincode_define(ns, d.get("policy") or b"", plugin=d.get("plugin", "vscc"),
                             flags=_lib.CC_COLLECTIONS_KNOWN if colls is not None else 0)
        for name, ep in (colls or {}).items():
            eng.collection_define(ns, name, ep or b"")


@pytest.mark.parametrize("mode", MODES)
def test_v20_sample_ledger(mode):
    """The reference's own v2.0 network (tests/golden/sample_ledgers.*): 15 endorser blocks --
    admin-signed _lifecycle approvals checked against implicit-collection policies, 3-org commits
    against LifecycleEndorsement (MAJORITY), marbles-private collection writes -- come out with
    the TRANSACTIONS_FILTER the reference stored (all VALID)."""
    from tests.sample_channel import v20_channel
    blocks_, config, idents, defs = v20_channel()
    eng = _v20_engine(mode, idents, config)
    n = 0
    for b in blocks_:
        if b["number"] < 5:
            continue
        _define(eng, defs[b["number"]])
        assert list(eng.validate_blocks([b["block"]])[0]) == b["flags"], b["number"]
        n += 1
    assert n == 15
    eng.close()


def test_v20_derived_negatives_match_oracle():
    """Model perturbations (peers stripped of PEER role, only Org1's peer a PEER, a collection
    removed from marbles-private, the creator of block 13 unregistered -- resolved through its MSP)
    give the oracle's codes on the GPU; unknown collections and a P-384 creator give Unsupported."""
    from tests.sample_channel import tx_identities, v20_channel
    from oracle.protowire import decode
    blocks_, config, idents, defs = v20_channel()
    by = {b["number"]: b for b in blocks_}
    Id = txvalidator.Identity

    def conv(pairs, f):
        return [(s, Id(i.mspid, i.pub, i.valid, i.id_digest, key=i.key, hash_family=i.hash_family, roles=f(i)))
                for s, i in pairs]
    no_peer = conv(idents, lambda i: i.roles & ~(1 << 3))
    one_peer = conv(idents, lambda i: i.roles if i.mspid == "Org1MSP" else i.roles & ~(1 << 3))
    d13 = copy.deepcopy(defs[13])
    del d13["marblesp"]["collections"]["collectionMarbles"]
    creator13 = tx_identities(decode("Block", by[13]["block"])["data"]["data"][0])[0]
    unreg13 = [(s, i) for s, i in idents if s != creator13]  # resolved through its MSP (cache miss)
    cases = [(5, no_peer, None), (8, no_peer, None), (5, one_peer, None), (8, one_peer, None), (13, idents, d13),
             (13, unreg13, None)]
    for num, ids, dd in cases:
        d = dd or defs[num]
        exp = v20.validate_block(v20.ChannelModel("testchannel", ids, d, config=config), by[num]["block"])
        eng = _v20_engine(0, ids, config)
        _define(eng, d)
        assert list(eng.validate_blocks([by[num]["block"]])[0]) == exp, num
        eng.close()
    # outside the model
    d_unknown = copy.deepcopy(defs[13])
    d_unknown["marblesp"]["collections"] = None
    p384 = conv(idents, lambda i: i.roles)
    for s, i in p384:
        i.key = "p384"
    for ids, dd, num in [(idents, d_unknown, 13), (p384, None, 5)]:
        eng = _v20_engine(0, ids, config)
        _define(eng, dd or defs[num])
        with pytest.raises(_lib.Unsupported):
            eng.validate_blocks([by[num]["block"]])
        with pytest.raises(v20.Unsupported):
            v20.validate_block(v20.ChannelModel("testchannel", ids, dd or defs[num], config=config), by[num]["block"])
        eng.close()


@pytest.mark.parametrize("mode", MODES)
def test_unsupported_inputs(mode):
    """Non-vscc plugin, a role principal with identities registered without role bits (round-1
    API), an unregistered certificate of a known MSP: FGV_EUNSUPPORTED.  (SHA3 MSPs are modelled
    since round 5: test_sha3_msp.)"""
    net = blocks.Network(seed=3, orgs=3, clients=30)
    blk, _, _ = blocks.make_block(net, 60, number=1, seed=11)
    ref = chanconfig.channel_ref("/Channel/Application/Endorsement")
    cases = [
        dict(ccs={"mycc": {"policy": blocks.out_of_policy(2, net.mspids), "plugin": "custom"}}),  # plugin
        dict(ccs={"mycc": ref}, config=chanconfig.make_config(net.mspids), ids=net.identities_legacy()),  # roles
        dict(ccs={"mycc": blocks.out_of_policy(2, net.mspids)}, ids=net.identities()[5:]),  # unregistered
    ]
    for c in cases:
        eng = _engine(net, c["ccs"], c.get("config"), c.get("ids"), mode=mode)
        with pytest.raises(_lib.Unsupported):
            eng.validate_blocks([blk])
        with pytest.raises(v20.Unsupported):
            v20.validate_block(_oracle(net, c["ccs"], c.get("config"), c.get("ids")), blk)
        eng.close()


@pytest.mark.parametrize("mode", MODES)
def test_sha3_msp(mode):
    """An MSP whose SignatureHashFamily is SHA3 (msp/identities.go:170-227): its identities'
    creator and endorsement signatures are over SHA3-256 digests (k_bd_sha3 on the device parse,
    SHA3 hash jobs on the host parse).  Flags equal the oracle's and the generator's labels, with
    transactions created and endorsed by that MSP among the valid ones; the same blocks against
    a config that says SHA2 for it fail exactly those signatures, as in the oracle."""
    fam = {"Org2MSP": "SHA3"}
    net = blocks.Network(seed=21, orgs=3, clients=30, hash_families=fam)
    cfg = chanconfig.make_config(net.mspids, hash_families=fam)
    ccs = {"mycc": blocks.out_of_policy(2, net.mspids)}
    blks, labels = [], []
    for i in range(2):
        b, lab, _ = blocks.make_block(net, 120, number=1 + i, seed=300 + i)
        blks.append(b)
        labels.append(lab)
    eng = _engine(net, ccs, cfg, mode=mode)
    got = eng.validate_blocks(blks)
    exp = v20.validate_blocks(_oracle(net, ccs, cfg), blks)
    assert [list(g) for g in got] == [list(e) for e in exp]
    for g, lab in zip(got, labels):
        for code, e in zip(g, blocks.expected_codes(lab)):
            assert e is None or code == e
    valid = sum(int((g == 0).sum()) for g in got)
    assert valid > 200  # (a third of the creators are Org2's: they verify under SHA3)
    eng.close()
    # the same identities registered as SHA2 (a config without the SHA3 family): Org2's
    # signatures no longer verify -- the engine and the oracle agree on every flag
    ids2 = [(ser, dataclasses.replace(i, hash_family="SHA2")) for ser, i in net.identities()]
    cfg2 = chanconfig.make_config(net.mspids)
    eng = _engine(net, ccs, cfg2, identities=ids2, mode=mode)
    got2 = eng.validate_blocks(blks)
    exp2 = v20.validate_blocks(_oracle(net, ccs, cfg2, identities=ids2), blks)
    assert [list(g) for g in got2] == [list(e) for e in exp2]
    assert sum(int((g == 0).sum()) for g in got2) < valid
    eng.close()
