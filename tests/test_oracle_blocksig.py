"""CPU: the restated orderer-signature check of VerifyBlock (oracle/blockverify.py
block_signatures_ok / verify_blocks(sig=...)) pinned by the reference's own orderer
signatures -- blocks 1..19 of the v2.0 sample ledger (tests/golden/sample_ledgers.*) carry
metadata[SIGNATURES] written by its orderer (BlockWriter.addBlockSignature), verified against the
ledger's /Channel/Orderer/BlockValidation (ImplicitMeta ANY over OrdererOrgMSP Writers) -- and by
the reference-semantics cases of tests/blocksig_cases.py."""
import pytest

from oracle import blockverify as BV
from oracle import v20
from oracle.protowire import decode
from tests import blocksig_cases as BC


def ledger_setup():
    """(blocks 1..19, chain after block 0, identities incl. the orderer's, config)"""
    from tests.sample_channel import identity_of, msp_nodeous, v20_channel
    blocks, config, idents, _ = v20_channel()
    nodeous = msp_nodeous(config)
    seen = {s for s, _ in idents}
    for b in blocks[1:]:
        md = decode("Metadata", decode("Block", b["block"])["metadata"]["metadata"][0])
        for ms in md.get("signatures", []):
            creator = decode("SignatureHeader", ms["signature_header"])["creator"]
            if creator not in seen:
                seen.add(creator)
                idents.append(identity_of(creator, nodeous))
    h0 = decode("Block", blocks[0]["block"])["header"]
    hh0 = BV.block_header_hash(h0.get("number", 0), h0.get("previous_hash"), h0.get("data_hash"))
    return [b["block"] for b in blocks[1:]], (0, hh0), idents, config


def tamper(block, field_path):
    """flip the last byte of metadata[SIGNATURES]'s first signature (field_path 'sig') or of its
    value ('value')"""
    from fabric_amd.synth import orderer as OR
    from fabric_amd.synth.blocks import f_bytes, f_msg
    md = decode("Metadata", decode("Block", block)["metadata"]["metadata"][0])
    value = md.get("value") or b""
    sigs = md["signatures"]
    if field_path == "value":
        value = value[:-1] + bytes([value[-1] ^ 1])
    else:
        s0 = sigs[0]["signature"]
        sigs[0]["signature"] = s0[:-1] + bytes([s0[-1] ^ 1])
    raw = f_bytes(1, value) + b"".join(f_msg(2, f_bytes(1, s["signature_header"]) + f_bytes(2, s["signature"]))
                                       for s in sigs)
    return OR.with_signatures(block, raw)


def test_reference_ledger_orderer_signatures_verify():
    blocks, (n0, h0), idents, config = ledger_setup()
    model = v20.ChannelModel("testchannel", idents, {}, config=config)
    chain = dict(number=n0, header_hash=h0)
    res = BV.verify_blocks(blocks, chain, sig=dict(model=model))
    assert [r[0] for r in res] == [BV.OK] * 19
    assert chain["number"] == 19 and model.verify_calls == 19


@pytest.mark.parametrize("what", ["sig", "value"])
def test_reference_ledger_tampered_signature_fails(what):
    blocks, (n0, h0), idents, config = ledger_setup()
    model = v20.ChannelModel("testchannel", idents, {}, config=config)
    bad = list(blocks[:5])
    bad[2] = tamper(bad[2], what)
    res = BV.verify_blocks(bad, dict(number=n0, header_hash=h0), sig=dict(model=model))
    # block 3 fails its signature and does not advance the chain: block 4 then fails the number
    assert [r[0] for r in res] == [BV.OK, BV.OK, BV.SIGNATURES, BV.NUMBER, BV.NUMBER]


def test_reference_ledger_without_orderer_identity_resolves_through_the_msp():
    """The orderer's certificate was never registered: the MSP cache miss deserializes it through
    the channel config's OrdererOrgMSP (oracle/msp.py) -- the same identity the registration
    carried (Id, key, Validate, roles) -- and the blocks verify."""
    blocks, (n0, h0), idents, config = ledger_setup()
    dropped = [(s, i) for s, i in idents if i.mspid == "OrdererOrgMSP"]
    idents = [(s, i) for s, i in idents if i.mspid != "OrdererOrgMSP"]
    model = v20.ChannelModel("testchannel", idents, {}, config=config)
    res = BV.verify_blocks(blocks[:3], dict(number=n0, header_hash=h0), sig=dict(model=model))
    assert [r[0] for r in res] == [BV.OK] * 3
    for ser, reg in dropped:
        got = model.deserialize(ser)
        assert got is not None and got.id_digest == reg.id_digest and got.pub == reg.pub
        assert got.valid == reg.valid and got.roles == reg.roles


def test_reference_ledger_orderer_msp_outside_the_model_is_unsupported():
    """A channel MSP outside the modelled shapes (here: no root CAs left) cannot judge the miss."""
    from oracle.protowire import decode
    blocks, (n0, h0), idents, config = ledger_setup()
    idents = [(s, i) for s, i in idents if i.mspid != "OrdererOrgMSP"]
    model = v20.ChannelModel("testchannel", idents, {}, config=config)
    fc = dict(model.config_msps["OrdererOrgMSP"])
    fc["root_certs"] = []
    model.config_msps["OrdererOrgMSP"] = fc
    res = BV.verify_blocks(blocks[:3], dict(number=n0, header_hash=h0), sig=dict(model=model))
    assert [r[0] for r in res] == [BV.SIG_UNSUPPORTED] * 3
    assert decode  # (the config bytes themselves are unchanged)


@pytest.mark.parametrize("case", BC.cases(), ids=lambda c: c["name"])
def test_reference_semantics_cases(case):
    model = BC.oracle_model(case)
    res = BV.verify_blocks(case["blocks"], BC.chain_dict(case),
                           sig=dict(model=model, policy=case["policy"], bft=case["bft"]))
    assert [r[0] for r in res] == case["expect"], case["name"]
