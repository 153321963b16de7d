"""GPU parity of the MSP cache miss (fgv_msp_resolve*, auto-resolve in the validate calls): the
engine's deserialization of never-registered identities -- X.509 parse, chain to a root with the
CA signature verified on the GPU, sanitizeCert, Id, Validate, role bits -- against the oracle
(oracle/msp.py) on the reference's own MSP test data (tests/golden/msp_fixtures.json), on the
synthetic cases of tests/msp_cases.py, and end to end on the reference's v2.0 sample ledger with
no identity registered at all (flags = the ledger's stored TRANSACTIONS_FILTER)."""
import json
import os

import pytest

from fabric_amd import _lib, txvalidator
from fabric_amd.synth.blocks import serialized_identity
from fabric_amd.synth.chanconfig import make_config
from oracle import blockverify as BV
from oracle import v20
from oracle.msp import MSP
from oracle.protowire import decode
from tests import msp_cases as MC

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FX = json.load(open(os.path.join(HERE, "golden", "msp_fixtures.json")))


def _expect(m, ser):
    """the oracle's outcome for one serialized identity: (status, Ident | None)"""
    if m is None or isinstance(m, Exception):
        return MC.UNSUP, None
    idb = decode("SerializedIdentity", ser).get("id_bytes") or b""
    try:
        got = m.resolve(idb)
    except v20.Unsupported:
        return MC.UNSUP, None
    return (MC.FAILED, None) if got is None else (MC.OK, got)


def _check(eng, ser, st, exp_st, ident, label):
    assert st == exp_st, (label, st, exp_st)
    rec = eng.msp_identity(ser)
    if exp_st == MC.UNSUP:
        assert rec is None, label
    elif exp_st == MC.FAILED:
        assert rec is not None and rec["key"] == _lib.KEY_TYPES["undeserializable"], label
    elif exp_st == MC.OK:
        assert rec["key"] == _lib.KEY_TYPES[ident.key] and rec["valid"] == ident.valid and rec["roles"] == ident.roles, label
        assert rec["id_digest"] == ident.id_digest, label
        if ident.key in (v20.KEY_P256, v20.KEY_P384):
            assert rec["pub"] == ident.pub, label


@pytest.mark.parametrize("rel", sorted(FX["msps"]))
def test_reference_msp_fixtures(rel):
    conf = bytes.fromhex(FX["msps"][rel]["config"])
    try:
        m = MSP(decode("FabricMSPConfig", conf))
    except v20.Unsupported as e:
        m = e
    eng = _lib.Engine(0)
    eng.channel_init("ch")
    eng.channel_config(make_config(["SampleOrg"], msp_configs={"SampleOrg": conf}))
    labels = sorted(FX["msps"][rel]["identities"])
    sers = [serialized_identity("SampleOrg", FX["msps"][rel]["identities"][k].encode()) for k in labels]
    sts = eng.msp_resolve(sers)
    seen = set()
    for label, ser, st in zip(labels, sers, sts):
        if ser in seen:
            assert st == MC.REPEAT
            continue
        seen.add(ser)
        exp_st, ident = _expect(m, ser)
        _check(eng, ser, st, exp_st, ident, label)
    # a second call finds them registered (or still outside the model)
    again = eng.msp_resolve(sers)
    assert all(a in (0, MC.UNSUP, MC.REPEAT) for a in again)
    eng.close()


def test_synthetic_cases():
    cfg, cases = MC.synthetic()
    models = v20.ChannelModel("ch", [], {}, config=cfg).msp_models()
    eng = _lib.Engine(0)
    eng.channel_init("ch")
    eng.channel_config(cfg)
    sts = eng.msp_resolve([c[1] for c in cases])
    for (label, ser, want, valid, roles), st in zip(cases, sts):
        if want == MC.REPEAT:
            assert st == MC.REPEAT, label
            continue
        exp_st, ident = _expect(models.get(decode("SerializedIdentity", ser).get("mspid", "")), ser)
        assert exp_st == want, label
        _check(eng, ser, st, exp_st, ident, label)
        if want == MC.OK:
            assert (ident.valid, ident.roles) == (valid, roles), label
    eng.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_v20_sample_ledger_without_registered_identities(mode):
    """Every creator and endorser of the reference's v2.0 network is a cache miss: the engine
    resolves each batch's misses through the channel config's MSPs (auto-resolve) and the flags
    equal the ledger's; the registry then holds the same identities the registration carried."""
    from tests.sample_channel import v20_channel
    from tests.test_gpu_channel import _define
    blocks_, config, idents, defs = v20_channel()
    eng = _lib.Engine(0)
    eng.set_parse_mode(mode)
    txvalidator.setup_channel(eng, "testchannel", [], {}, config=config)
    n = 0
    for b in blocks_:
        if b["number"] < 5:
            continue
        _define(eng, defs[b["number"]])
        assert list(eng.validate_blocks([b["block"]])[0]) == b["flags"], b["number"]
        n += 1
    assert n == 15
    for ser, reg in idents:
        rec = eng.msp_identity(ser)
        if rec is None:  # (an identity no endorser block names: resolve it directly)
            assert eng.msp_resolve([ser]) == [MC.OK]
            rec = eng.msp_identity(ser)
        assert (rec["valid"], rec["roles"], rec["id_digest"], rec["pub"]) == (reg.valid, reg.roles, reg.id_digest,
                                                                          bytes(reg.pub)), reg.mspid
    eng.close()


def test_auto_resolve_off_then_explicit():
    from tests.sample_channel import v20_channel
    from tests.test_gpu_channel import _define
    blocks_, config, idents, defs = v20_channel()
    b = [x for x in blocks_ if x["number"] == 8][0]
    eng = _lib.Engine(0)
    txvalidator.setup_channel(eng, "testchannel", [], {}, config=config)
    _define(eng, defs[8])
    eng.set_auto_resolve(False)
    with pytest.raises(_lib.Unsupported):
        eng.validate_blocks([b["block"]])
    assert eng.msp_resolve_blocks([b["block"]]) >= 2  # creator + endorsers
    assert list(eng.validate_blocks([b["block"]])[0]) == b["flags"]
    eng.close()


def test_orderer_signatures_without_registered_orderer():
    """fgv_blocks_verify_signed resolves the orderer's certificate through OrdererOrgMSP"""
    from tests.test_gpu_blocksig import _chain
    from tests.test_oracle_blocksig import ledger_setup
    blocks, (n0, h0), idents, config = ledger_setup()
    idents2 = [(s, i) for s, i in idents if i.mspid != "OrdererOrgMSP"]
    eng = _lib.Engine(0)
    txvalidator.setup_channel(eng, "testchannel", idents2, {}, config=config)
    got, unsup = eng.blocks_verify_signed(blocks[:5], _chain((n0, h0)))
    model = v20.ChannelModel("testchannel", idents2, {}, config=config)
    exp = BV.verify_blocks(blocks[:5], dict(number=n0, header_hash=h0), sig=dict(model=model))
    assert [g[0] for g in got] == [e[0] for e in exp] == [BV.OK] * 5 and not unsup
    eng.close()


def test_group_resolves_on_every_device():
    from tests.sample_channel import v20_channel
    from tests.test_gpu_channel import _define
    blocks_, config, idents, defs = v20_channel()
    sel = [b for b in blocks_ if 5 <= b["number"] <= 7]
    g = _lib.Group([0, 0])
    for e in g.engines:
        txvalidator.setup_channel(e, "testchannel", [], {}, config=config)
        _define(e, defs[7])
    got = g.validate_blocks([b["block"] for b in sel])
    exp = v20.validate_blocks(v20.ChannelModel("testchannel", [], defs[7], config=config), [b["block"] for b in sel])
    assert [list(f) for f in got] == [list(f) for f in exp]
    g.close()


def test_fork_hazard_reframings_are_unsupported():
    """a real msp/testdata leaf re-framed into shapes Go's parsers accept (extra
    element after the outer signature, junk before the PEM, a malformed block before a valid one,
    ...) is Unsupported in the engine and the oracle, never an undeserializable identity; and a
    block whose creator is such a re-framing is an Unsupported batch on both sides."""
    from tests.blockfix import creator_idbytes_path, replace_field
    from tests.sample_channel import tx_identities, v20_channel
    rel = "msp/testdata/nodeous3"
    conf = bytes.fromhex(FX["msps"][rel]["config"])
    m = MSP(decode("FabricMSPConfig", conf))
    ids = FX["msps"][rel]["identities"]
    pem = ids[[k for k in ids if k.startswith("signcerts/")][0]].encode()
    eng = _lib.Engine(0)
    eng.channel_init("ch")
    eng.channel_config(make_config(["SampleOrg"], msp_configs={"SampleOrg": conf}))
    variants = MC.fork_hazard_variants(pem)
    sers = [serialized_identity("SampleOrg", p) for _, p in variants]
    for (label, p), ser, st in zip(variants, sers, eng.msp_resolve(sers)):
        exp_st, ident = _expect(m, ser)
        assert exp_st == (MC.OK if label == "short_line_wrap" else MC.UNSUP), label
        _check(eng, ser, st, exp_st, ident, label)
    eng.close()
    # end to end: block 13 of the v2.0 sample ledger with its creator unregistered and re-framed
    blocks_, config, idents, defs = v20_channel()
    b13 = [b for b in blocks_ if b["number"] == 13][0]["block"]
    creator = tx_identities(decode("Block", b13)["data"]["data"][0])[0]
    unreg = [(s, i) for s, i in idents if s != creator]
    idb = decode("SerializedIdentity", creator)["id_bytes"]
    for label, p in MC.fork_hazard_variants(idb)[:4]:
        blk = replace_field(b13, creator_idbytes_path(0), p)
        eng = _lib.Engine(0)
        txvalidator.setup_channel(eng, "testchannel", unreg, {}, config=config)
        from tests.test_gpu_channel import _define
        _define(eng, defs[13])
        with pytest.raises(_lib.Unsupported):
            eng.validate_blocks([blk])
        with pytest.raises(v20.Unsupported):
            v20.validate_block(v20.ChannelModel("testchannel", unreg, defs[13], config=config), blk)
        eng.close()


def test_admin_setup_cases():
    """an MSP whose admins fail the post-setup checks (a revoked admin without NodeOUs,
    an admin without the client / admin OU, an admin with no chain) does not set up in the
    reference: the engine leaves it to the reference (Unsupported), as the oracle does"""
    for label, cfg, probe, sets_up in MC.admin_setup_cases():
        eng = _lib.Engine(0)
        try:
            eng.channel_init("ch")
            eng.channel_config(cfg)
            st = eng.msp_resolve([probe])
            assert st == ([MC.OK] if sets_up else [MC.UNSUP]), (label, st)
        finally:
            eng.close()
