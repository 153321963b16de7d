"""GPU: per-block outcomes (fgv_set_block_outcomes, include/fgv.h).  A transaction outside the
engine's model sends only its own block to the reference; a block whose keys' key-level
parameters an earlier block of the call may change waits for that block's commit (n_final), and
every other block's flags are final and equal the restated committer's
(oracle.v20.validate_blocks_outcomes: validate_block per block, every earlier block's txids
indexed -- validator.go:460-481 reads TxIDExists, whatever the earlier codes were)."""
import pytest

from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks
from oracle import v20
from tests import sbe_cases

pytestmark = pytest.mark.gpu
MODES = pytest.mark.parametrize("mode", [0, 1], ids=["devparse", "hostparse"])


def _check(eng, model, blks):
    got = eng.validate_blocks(blks)
    st, n_final = eng.last_block_status(len(blks))
    exp, exp_final = v20.validate_blocks_outcomes(model, blks)
    assert n_final == exp_final
    for b in range(len(blks)):
        if b >= exp_final:
            assert st[b] == _lib.BLOCK_LATER, b
        elif exp[b] is None:
            assert st[b] == _lib.FGV_EUNSUPPORTED, b
            assert 0xFD in list(got[b])
        else:
            assert st[b] == 0, b
            mism = [(i, int(got[b][i]), exp[b][i]) for i in range(len(exp[b])) if got[b][i] != exp[b][i]]
            assert len(got[b]) == len(exp[b]) and not mism, (b, mism[:10])
    return st, n_final


@MODES
def test_out_of_model_identity_confined_to_its_blocks(mode):
    """one client registered as a P-384 identity (the engine does not verify P-384): only the blocks
    where it creates or endorses a transaction are unsupported; the batch's other blocks are final"""
    net = blocks.Network(seed=3, orgs=3, clients=3000)
    blks, creators = [], []
    for i in range(6):
        txs = []
        blks.append(blocks.make_block(net, 100, number=1 + i, seed=60 + i, out_txs=txs)[0])
        creators.append({t.creator.serialized for t in txs})
    # a creator that appears in blocks 1 and 4 only (or in one block): the P-384 identity
    pick = None
    for ser in creators[1]:
        where = [b for b in range(6) if ser in creators[b]]
        if where == [1]:
            pick = ser
            break
    assert pick is not None
    ids = []
    for ser, ident in net.identities():
        if ser == pick:
            ident = txvalidator.Identity(ident.mspid, None, True, ident.id_digest, key="p384", roles=ident.roles)
        ids.append((ser, ident))
    eng = _lib.Engine(0)
    try:
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, ids, net.chaincodes)
        with pytest.raises(_lib.Unsupported):  # (the whole-batch contract stays the default)
            eng.validate_blocks(blks)
        with pytest.raises(_lib.Unsupported):  # a failed call decided nothing
            eng.last_block_status(6)
        assert eng.unsupported_stats()["blocks"] == 6
        eng.set_block_outcomes(True)
        st, n_final = _check(eng, v20.ChannelModel(net.channel, ids, net.chaincodes), blks)
        assert n_final == 6 and st == [0, _lib.FGV_EUNSUPPORTED, 0, 0, 0, 0], st
        s = eng.unsupported_stats()
        assert s["batches"] == 1 and s["blocks"] == 7 and s["txs"] >= 1, s
    finally:
        eng.close()


@MODES
def test_keylevel_split_at_block_boundary(mode):
    """block 1 sets / clears key-level parameters that block 2 writes: blocks 0..1 are final, block 2
    waits (n_final = 2); after block 1's MVCC commit, block 2 alone equals the oracle on the
    committed state"""
    from oracle import mvcc as OM
    net = sbe_cases_network()
    ccs = {ns: dict(policy=p, collections={"pvt1": None}) for ns, p in net.chaincodes.items()}
    b0 = blocks.make_block(net, 40, number=1, seed=17)[0]
    (b1, kvmeta0), (b2, _) = [sbe_cases.make_sbe_block(net, 50, 948 + k, number=2 + k) for k in range(2)]
    eng = _lib.Engine(0)
    try:
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, net.identities(), ccs, kvmeta=kvmeta0)
        eng.set_block_outcomes(True)
        model = lambda kv: v20.ChannelModel(net.channel, net.identities(), ccs, kvmeta=dict(kv))  # noqa: E731
        st, n_final = _check(eng, model(kvmeta0), [b0, b1, b2])
        assert n_final == 2 and st == [0, 0, _lib.BLOCK_LATER], st
        eng.statedb_init(1 << 16, 8 << 20)
        db = OM.StateDB({}, kvmeta=dict(kvmeta0))
        for num, b in ((1, b0), (2, b1)):
            f = v20.validate_block(model(db.kvmeta), b)
            assert list(eng.mvcc_validate(b, num, f, commit=True)) == list(OM.validate_block(db, b, f, num, commit=True))
        m2 = model(db.kvmeta)
        for b in (b0, b1):
            for d in (v20.decode("Block", b).get("data") or {}).get("data", []):
                t = v20.index_txid(d)
                if t:
                    m2.committed.add(t)
        eng.ledger_add_txids(sorted(m2.committed))
        st, n_final = _check(eng, m2, [b2])
        assert n_final == 1 and st == [0]
    finally:
        eng.close()


def sbe_cases_network():
    from tests.blockfix import network
    return network()


def _check_group(g, model, blks):
    """_check through fgv_group_validate_blocks / fgv_group_last_block_status"""
    got = g.validate_blocks(blks)
    st, n_final = g.last_block_status(len(blks))
    exp, exp_final = v20.validate_blocks_outcomes(model, blks)
    assert n_final == exp_final
    for b in range(len(blks)):
        if b >= exp_final:
            assert st[b] == _lib.BLOCK_LATER, b
        elif exp[b] is None:
            assert st[b] == _lib.FGV_EUNSUPPORTED, b
            assert 0xFD in list(got[b])
        else:
            assert st[b] == 0, b
            mism = [(i, int(got[b][i]), exp[b][i]) for i in range(len(exp[b])) if got[b][i] != exp[b][i]]
            assert len(got[b]) == len(exp[b]) and not mism, (b, mism[:10])
    return st, n_final


@pytest.mark.parametrize("ndev", [2, 3, 7])
def test_group_out_of_model_identity_confined_to_its_blocks(ndev):
    """the P-384 case through fgv_group (block plan with 2 and 3 devices; 7 devices > 6 blocks:
    the transaction-index plan): only the blocks holding the identity's transactions are
    unsupported, on whichever device validated them; the other blocks' flags are final"""
    net = blocks.Network(seed=3, orgs=3, clients=3000)
    blks, creators = [], []
    for i in range(6):
        txs = []
        blks.append(blocks.make_block(net, 100, number=1 + i, seed=60 + i, out_txs=txs)[0])
        creators.append({t.creator.serialized for t in txs})
    pick = next(ser for ser in creators[4] if [b for b in range(6) if ser in creators[b]] == [4])
    ids = []
    for ser, ident in net.identities():
        if ser == pick:
            ident = txvalidator.Identity(ident.mspid, None, True, ident.id_digest, key="p384", roles=ident.roles)
        ids.append((ser, ident))
    g = _lib.Group([0] * ndev)
    try:
        for e in g.engines:
            txvalidator.setup_channel(e, net.channel, ids, net.chaincodes)
        with pytest.raises(_lib.Unsupported):  # (the whole-batch contract stays the default)
            g.validate_blocks(blks)
        with pytest.raises(_lib.Unsupported):  # a failed call decided nothing
            g.last_block_status(6)
        g.set_block_outcomes(True)
        st, n_final = _check_group(g, v20.ChannelModel(net.channel, ids, net.chaincodes), blks)
        assert n_final == 6 and st == [0, 0, 0, 0, _lib.FGV_EUNSUPPORTED, 0], st
    finally:
        g.close()


@pytest.mark.parametrize("ndev", [1, 2, 3, 4, 7])
def test_group_keylevel_split_across_devices(ndev):
    """block 1 sets / clears key-level parameters that block 2 writes; with 2 or 3 devices the
    two blocks sit on different devices (block plan by bytes): blocks 0..1 final, block 2 LATER.
    4 and 7 devices > 3 blocks: the transaction-index plan splits block 1 between devices, and a
    dependent whose metadata writer another device holds is decided there (shadow writers)"""
    net = sbe_cases_network()
    ccs = {ns: dict(policy=p, collections={"pvt1": None}) for ns, p in net.chaincodes.items()}
    b0 = blocks.make_block(net, 40, number=1, seed=17)[0]
    (b1, kvmeta0), (b2, _) = [sbe_cases.make_sbe_block(net, 50, 948 + k, number=2 + k) for k in range(2)]
    g = _lib.Group([0] * ndev)
    try:
        for e in g.engines:
            txvalidator.setup_channel(e, net.channel, net.identities(), ccs, kvmeta=kvmeta0)
        g.set_block_outcomes(True)
        model = v20.ChannelModel(net.channel, net.identities(), ccs, kvmeta=dict(kvmeta0))
        st, n_final = _check_group(g, model, [b0, b1, b2])
        assert n_final == 2 and st == [0, 0, _lib.BLOCK_LATER], st
    finally:
        g.close()


def _shard_protocol_outcomes(eng, blks, shards, mode):
    """fgv_validate_shard_dev per rank (one engine, ranks in turn) into the rank-major gathered
    buffer, fgv_finalize_flags_dev, then shard.block_outcomes over the ranks' n_final"""
    import numpy as np
    import torch
    from fabric_amd import shard
    ntx = np.array([len((v20.decode("Block", b).get("data") or {}).get("data", [])) for b in blks], dtype=np.int64)
    plan = shard.plan(ntx, shards, mode)
    rows = shard.plan_rows(*plan)
    recv = torch.zeros((shards * rows, shard.REC), dtype=torch.uint8, device="cuda")
    batch = eng.block_batch(blks)
    n_final = len(blks)
    for r in range(shards):
        eng.validate_shard_dev(batch, plan[0][r], plan[1][r], recv[r * rows:].data_ptr(), rows)
        n_final = min(n_final, eng.last_block_status(len(blks))[1])
    flags = eng.finalize_flags_dev(ntx, shards, rows, recv.data_ptr(), plan=None if mode == "tx" else plan)
    st, nf = shard.block_outcomes(flags, ntx, n_final)
    out, o = [], 0
    for n in ntx:
        out.append(flags[o:o + int(n)])
        o += int(n)
    return out, st, nf


def _expect(model, blks, got, st, n_final):
    exp, exp_final = v20.validate_blocks_outcomes(model, blks)
    assert n_final == exp_final
    for b in range(len(blks)):
        if b >= exp_final:
            assert st[b] == _lib.BLOCK_LATER, b
        elif exp[b] is None:
            assert st[b] == _lib.FGV_EUNSUPPORTED, b
            assert 0xFD in list(got[b])
        else:
            assert st[b] == 0, b
            mism = [(i, int(got[b][i]), exp[b][i]) for i in range(len(exp[b])) if got[b][i] != exp[b][i]]
            assert len(got[b]) == len(exp[b]) and not mism, (b, mism[:10])


@pytest.mark.parametrize("shards,mode", [(2, "tx"), (3, "tx"), (2, "block"), (3, "block")])
def test_shard_protocol_out_of_model_identity(shards, mode):
    """the P-384 case through the one-process-per-GPU protocol (fgv_set_block_outcomes on the
    ranks' engines): only the identity's block is unsupported, the others equal the oracle"""
    net = blocks.Network(seed=3, orgs=3, clients=3000)
    blks, creators = [], []
    for i in range(6):
        txs = []
        blks.append(blocks.make_block(net, 100, number=1 + i, seed=60 + i, out_txs=txs)[0])
        creators.append({t.creator.serialized for t in txs})
    pick = next(ser for ser in creators[2] if [b for b in range(6) if ser in creators[b]] == [2])
    ids = []
    for ser, ident in net.identities():
        if ser == pick:
            ident = txvalidator.Identity(ident.mspid, None, True, ident.id_digest, key="p384", roles=ident.roles)
        ids.append((ser, ident))
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, ids, net.chaincodes)
        eng.set_block_outcomes(True)
        got, st, n_final = _shard_protocol_outcomes(eng, blks, shards, mode)
        _expect(v20.ChannelModel(net.channel, ids, net.chaincodes), blks, got, st, n_final)
        assert n_final == 6 and st == [0, 0, _lib.FGV_EUNSUPPORTED, 0, 0, 0], st
    finally:
        eng.close()


@pytest.mark.parametrize("shards,mode", [(2, "tx"), (3, "tx"), (5, "tx"), (2, "block"), (3, "block")])
def test_shard_protocol_keylevel_split(shards, mode):
    """the key-level split through the shard protocol: block 0 final, block 2 LATER, block 1 final
    and equal to the oracle in every plan -- split by transaction index, a dependent whose metadata
    writer another rank holds reads that writer's vscc result from the rank's shadow validation of
    the block's earlier metadata writers (vpmanagerimpl.go:296-355)"""
    net = sbe_cases_network()
    ccs = {ns: dict(policy=p, collections={"pvt1": None}) for ns, p in net.chaincodes.items()}
    b0 = blocks.make_block(net, 40, number=1, seed=17)[0]
    (b1, kvmeta0), (b2, _) = [sbe_cases.make_sbe_block(net, 50, 948 + k, number=2 + k) for k in range(2)]
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, net.identities(), ccs, kvmeta=kvmeta0)
        eng.set_block_outcomes(True)
        got, st, n_final = _shard_protocol_outcomes(eng, [b0, b1, b2], shards, mode)
        _expect(v20.ChannelModel(net.channel, net.identities(), ccs, kvmeta=dict(kvmeta0)), [b0, b1, b2], got, st,
                n_final)
        assert n_final == 2 and st == [0, 0, _lib.BLOCK_LATER], st
    finally:
        eng.close()


@pytest.mark.parametrize("seed", [948, 3, 77])
@MODES
def test_shard_protocol_keylevel_tx_split_seeds(seed, mode):
    """one key-level block split by transaction index at every shard count 2..6: dependents whose
    metadata writers sit on other ranks, chains of writers across ranks; every plan's flags equal
    the oracle's and the block is final (no deferral to the reference)"""
    net = sbe_cases_network()
    ccs = {ns: dict(policy=p, collections={"pvt1": None}) for ns, p in net.chaincodes.items()}
    b1, kvmeta0 = sbe_cases.make_sbe_block(net, 60, seed, number=2)
    model = lambda: v20.ChannelModel(net.channel, net.identities(), ccs, kvmeta=dict(kvmeta0))  # noqa: E731
    exp, _ = v20.validate_blocks_outcomes(model(), [b1])  # (it indexes the block's txids: a fresh model each time)
    eng = _lib.Engine(0)
    try:
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, net.identities(), ccs, kvmeta=kvmeta0)
        eng.set_block_outcomes(True)
        for shards in range(2, 7):
            got, st, n_final = _shard_protocol_outcomes(eng, [b1], shards, "tx")
            _expect(model(), [b1], got, st, n_final)
            if exp[0] is not None:
                assert st == [0], (shards, st)
    finally:
        eng.close()


@MODES
def test_config_block_confined(mode):
    """a CONFIG block in the middle of a call: its block goes to the reference and every later
    block waits (LATER: the configuration it applies governs them); with a bad creator signature
    it never reaches ChannelResources.Apply -- code 4, every block final"""
    net = blocks.Network(seed=3, orgs=3, clients=50)
    bl = [blocks.make_block(net, 60, number=n, seed=n)[0] for n in (1, 3, 4)]
    model = lambda: v20.ChannelModel(net.channel, net.identities(), net.chaincodes)  # noqa: E731
    eng = _lib.Engine(0)
    try:
        eng.set_parse_mode(mode)
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        eng.set_block_outcomes(True)
        st, n_final = _check(eng, model(), [bl[0], blocks.config_block(net, 2), bl[1], bl[2]])
        assert n_final == 2 and st == [0, _lib.FGV_EUNSUPPORTED, _lib.BLOCK_LATER, _lib.BLOCK_LATER], st
        st, n_final = _check(eng, model(), [bl[0], blocks.config_block(net, 2, bad_sig=True), bl[1], bl[2]])
        assert n_final == 4 and st == [0, 0, 0, 0], st
    finally:
        eng.close()


@pytest.mark.parametrize("ndev", [2, 5])
def test_group_config_block_confined(ndev):
    """the same through fgv_group (block plan with 2 devices, transaction plan with 5 > 4 blocks)"""
    net = blocks.Network(seed=3, orgs=3, clients=50)
    bl = [blocks.make_block(net, 60, number=n, seed=n)[0] for n in (1, 3, 4)]
    g = _lib.Group([0] * ndev)
    try:
        for e in g.engines:
            txvalidator.setup_channel(e, net.channel, net.identities(), net.chaincodes)
        g.set_block_outcomes(True)
        st, n_final = _check_group(g, v20.ChannelModel(net.channel, net.identities(), net.chaincodes),
                                   [bl[0], blocks.config_block(net, 2), bl[1], bl[2]])
        assert n_final == 2 and st == [0, _lib.FGV_EUNSUPPORTED, _lib.BLOCK_LATER, _lib.BLOCK_LATER], st
    finally:
        g.close()


@pytest.mark.parametrize("shards,mode", [(2, "tx"), (2, "block"), (3, "block")])
def test_shard_protocol_config_block_confined(shards, mode):
    net = blocks.Network(seed=3, orgs=3, clients=50)
    bl = [blocks.make_block(net, 60, number=n, seed=n)[0] for n in (1, 3, 4)]
    blks = [bl[0], blocks.config_block(net, 2), bl[1], bl[2]]
    eng = _lib.Engine(0)
    try:
        txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes)
        eng.set_block_outcomes(True)
        got, st, n_final = _shard_protocol_outcomes(eng, blks, shards, mode)
        _expect(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks, got, st, n_final)
        assert n_final == 2 and st[:2] == [0, _lib.FGV_EUNSUPPORTED], st
    finally:
        eng.close()
