"""CPU: the oracle against the reference's own sample ledgers (tests/golden/sample_ledgers.*,
extracted from core/ledger/kvledger/tests/testdata by tests/golden/make_sample_ledgers.py).

* commit hashes: every stored Metadata[COMMIT_HASH] of the three ledgers (36 blocks) is
  reproduced from the stored TRANSACTIONS_FILTER and the block's update batch
  (kv_ledger.go:806-817, update_batch_bytes.go) -- this pins the update-batch semantics
  (last writer wins, deletes, private-data hashes, sort order, height encoding);
* MVCC: replaying the v1.1 ledgers from an empty state with every transaction VALID at the
  committer reproduces the stored flags, including block 8's MVCC_READ_CONFLICT."""
import json
import os
import struct

import pytest

from oracle import commithash as CH
from oracle import mvcc as OM
from oracle.protowire import decode

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ledgers():
    idx = json.load(open(os.path.join(GOLD, "sample_ledgers.json")))
    blob = open(os.path.join(GOLD, "sample_ledgers.bin"), "rb").read()
    out = {}
    for name, blocks in idx.items():
        out[name] = [dict(b, block=blob[b["offset"]:b["offset"] + b["len"]]) for b in blocks]
        for b in blocks:
            assert struct.unpack("<I", blob[b["offset"] - 4:b["offset"]])[0] == b["len"]
    return out


def tx_type(env):
    pl = decode("Payload", decode("Envelope", env).get("payload"))
    return decode("ChannelHeader", pl["header"].get("channel_header")).get("type", 0)


@pytest.mark.parametrize("name", ["v20_testchannel", "v11_ledger1", "v11_ledger2"])
def test_commit_hash_chain(name):
    prev, n = b"", 0
    for b in ledgers()[name]:
        if b["commit_hash"] is None:
            assert b["number"] == 0  # the genesis block carries none (kv_ledger.go:647-652)
            continue
        h = CH.block_commit_hash(b["block"], b["flags"], b["number"], prev)
        assert h.hex() == b["commit_hash"], b["number"]
        prev, n = h, n + 1
    assert n == len(ledgers()[name]) - 1


@pytest.mark.parametrize("name", ["v11_ledger1", "v11_ledger2"])
def test_mvcc_replay_v11(name):
    db = OM.StateDB()
    for b in ledgers()[name]:
        data = decode("Block", b["block"])["data"].get("data", [])
        if b["number"] == 0:
            assert [tx_type(d) for d in data] == [1]
            continue
        got = OM.validate_block(db, b["block"], [0] * len(data), b["number"], commit=True)
        assert got == b["flags"], b["number"]
    assert db.get_version("cc1", "key1") == (7, 0) and db.get_version("cc1", "key2") is None


def test_mvcc_replay_v20():
    """v2.0 network: config blocks 0-4 (outside the model: Unsupported), then 15 endorser blocks
    (_lifecycle approvals/commits with implicit-collection writes, marbles, marbles-private)."""
    db = OM.StateDB()
    for b in ledgers()["v20_testchannel"]:
        data = decode("Block", b["block"])["data"].get("data", [])
        if all(tx_type(d) == 1 for d in data):
            with pytest.raises(OM.Unsupported):
                OM.validate_block(db, b["block"], [0] * len(data), b["number"], commit=True)
            continue
        assert OM.validate_block(db, b["block"], [0] * len(data), b["number"], commit=True) == b["flags"]


@pytest.mark.parametrize("name", ["v20_testchannel", "v11_ledger1", "v11_ledger2"])
def test_engine_commit_hash_chain(name):
    """libfgv's fgv_commit_hash (host C ABI, no GPU) reproduces the stored chain too."""
    from fabric_amd import _lib
    prev = b""
    for b in ledgers()[name]:
        if b["commit_hash"] is None:
            continue
        h = _lib.commit_hash(b["block"], b["flags"], b["number"], prev)
        assert h.hex() == b["commit_hash"], b["number"]
        prev = h


def test_committer_replay_v20():
    """The restated committer (oracle/v20.py) on the reference's v2.0 network blocks: creator
    signatures of admins / clients, single-org approvals validated against implicit-collection
    policies (/Channel/Application/orgN/Endorsement = OR('OrgN.peer')), 3-org commits against
    /Channel/Application/LifecycleEndorsement (ImplicitMeta MAJORITY), marbles-private
    collection writes -> every stored flag (VALID) reproduced."""
    from oracle import v20
    from tests.sample_channel import v20_channel
    blocks, config, idents, defs = v20_channel()
    n = 0
    for b in blocks:
        if b["number"] < 5:
            continue
        model = v20.ChannelModel("testchannel", idents, defs[b["number"]], config=config)
        assert v20.validate_block(model, b["block"]) == b["flags"], b["number"]
        n += 1
    assert n == 15


def test_committer_v20_derived_negatives():
    """Perturbing the MODEL (not the signed blocks) flips outcomes the way the reference's rules
    say: peers without the PEER role -> approvals and commits fail their org / MAJORITY
    policies (10); a marbles-private definition without collectionMarbles -> 10 ("no such
    collection"); unknown collections / a P-384 creator -> Unsupported (never a guess); an
    unregistered channel identity resolves through its MSP."""
    import copy

    import pytest

    from oracle import v20
    from tests.sample_channel import v20_channel
    blocks, config, idents, defs = v20_channel()
    by_num = {b["number"]: b for b in blocks}

    def run(num, idents_=idents, defs_=None):
        model = v20.ChannelModel("testchannel", idents_, defs_ or defs[num], config=config)
        out = v20.validate_block(model, by_num[num]["block"])
        return out, model.verify_calls

    assert run(8) == ([0], 10)  # creator + 3 endorsements x 3 sub-policies (each re-verifies, policy.go:363-395)
    no_peer = [(s, v20.Ident(i.mspid, i.pub, i.valid, i.id_digest, roles=i.roles & ~(1 << 3))) for s, i in idents]
    assert run(5, no_peer)[0] == [10] and run(8, no_peer)[0] == [10]
    one_peer = [(s, v20.Ident(i.mspid, i.pub, i.valid, i.id_digest,
                              roles=i.roles if i.mspid == "Org1MSP" else i.roles & ~(1 << 3))) for s, i in idents]
    assert run(5, one_peer)[0] == [0]   # Org1's implicit collection: OR('Org1MSP.peer')
    assert run(8, one_peer)[0] == [10]  # LifecycleEndorsement: MAJORITY of 3 orgs
    d = copy.deepcopy(defs[13])
    del d["marblesp"]["collections"]["collectionMarbles"]
    assert run(13, defs_=d)[0] == [10]
    d["marblesp"]["collections"] = None
    with pytest.raises(v20.Unsupported):
        run(13, defs_=d)
    from tests.sample_channel import tx_identities
    creator13 = tx_identities(decode("Block", by_num[13]["block"])["data"]["data"][0])[0]
    # a known MSP's certificate never registered: the MSP cache miss resolves it (oracle/msp.py)
    assert run(13, idents_=[(s, i) for s, i in idents if s != creator13])[0] == run(13)[0]
    p384 = [(s, v20.Ident(i.mspid, i.pub, i.valid, i.id_digest, key=v20.KEY_P384, roles=i.roles)) for s, i in idents]
    with pytest.raises(v20.Unsupported):
        run(5, p384)


def test_committer_v20_without_registered_identities():
    """No identity registered at all: every creator and endorser of the v2.0 sample ledger is an
    MSP cache miss, deserialized and validated through the channel config's MSPs (root CAs,
    NodeOUs, admins -- oracle/msp.py), and the replay still reproduces every block's stored
    TRANSACTIONS_FILTER; the resolved identities equal the registered ones."""
    from oracle import v20
    from tests.sample_channel import v20_channel
    blocks, config, idents, defs = v20_channel()
    n = 0
    for b in blocks:
        if b["number"] < 5:
            continue
        model = v20.ChannelModel("testchannel", [], defs[b["number"]], config=config)
        assert v20.validate_block(model, b["block"]) == b["flags"], b["number"]
        n += 1
    assert n == 15
    model = v20.ChannelModel("testchannel", [], {}, config=config)
    for ser, reg in idents:
        got = model.deserialize(ser)
        assert got is not None, reg.mspid
        assert (got.mspid, got.pub, got.valid, got.id_digest, got.roles) == \
            (reg.mspid, reg.pub, reg.valid, reg.id_digest, reg.roles)
