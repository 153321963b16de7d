"""GPU: fgv_group (several devices driven from one process through the C ABI) against the
single-GPU engine and the oracle.  The box has one MI355X, so the group's devices are the same
GPU several times -- every part of the protocol runs (block plan, per-device contexts and
host workers, the gather by peer copies, the finalize of the whole batch on the first device)
except that the copies stay inside one HBM."""
import pytest

from fabric_amd import _lib, txvalidator
from fabric_amd.synth import blocks
from oracle import v20
from tests.blockfix import network

pytestmark = pytest.mark.gpu


def _setup(eng, net, committed=()):
    txvalidator.setup_channel(eng, net.channel, net.identities(), net.chaincodes, committed)


@pytest.mark.parametrize("ndev", [1, 2, 3])
def test_group_matches_single_gpu_and_oracle(ndev):
    """C2 blocks with duplicate txids across blocks (a txid of block 1 again in blocks 3 and 5,
    which the block plan puts on other devices): the finalize on the first device sees the whole
    batch, so flags equal the single GPU's and the oracle's."""
    net = network()
    txs1 = []
    blks = [blocks.make_block(net, 40, number=1, seed=901, faults=(), out_txs=txs1)[0]]
    for i in range(2, 7):
        reuse = {2: (txs1[i].creator, txs1[i].nonce), 7: (txs1[0].creator, txs1[0].nonce)} if i in (3, 5) else None
        blks.append(blocks.make_block(net, 25 + 7 * i, number=i, seed=900 + i, reuse=reuse)[0])
    g = _lib.Group([0] * ndev)
    assert len(g.engines) == ndev
    for e in g.engines:
        _setup(e, net)
    got = g.validate_blocks(blks)
    one = _lib.Engine(0)
    _setup(one, net)
    single = one.validate_blocks(blks)
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks)
    for b in range(len(blks)):
        assert list(got[b]) == list(single[b]) == list(exp[b]), b
    assert any(9 in list(f) for f in got[2:])  # the cross-device duplicates were caught
    one.close()
    g.close()


def test_group_more_devices_than_blocks_and_ledger_txids():
    """4 devices, 2 blocks (two devices idle); ledger txids registered on every context"""
    net = network()
    b0, _, envs0 = blocks.make_block(net, 30, number=1, seed=777, faults=())
    b1 = blocks.make_block(net, 30, number=2, seed=778)[0]
    committed = [v20.index_txid(e) for e in envs0[:4]]
    g = _lib.Group([0, 0, 0, 0])
    for e in g.engines:
        _setup(e, net, committed)
    got = g.validate_blocks([b0, b1])
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes, committed), [b0, b1])
    assert [list(f) for f in got] == [list(f) for f in exp]
    assert list(got[0][:4]) == [9, 9, 9, 9]
    g.close()


def test_group_unsupported_propagates():
    """a block outside the model on any device makes the whole batch FGV_EUNSUPPORTED"""
    net = network()
    blks = [blocks.make_block(net, 20, number=i, seed=950 + i)[0] for i in range(1, 4)]
    g = _lib.Group([0, 0])
    for e in g.engines:
        txvalidator.setup_channel(e, net.channel, net.identities(), {})  # no chaincode definitions...
        e.msp_declare("Org1MSP")
    # ...and an unregistered identity of a declared MSP in the last block: unsupported
    rogue = blocks.Network(seed=99, orgs=1, clients=2)
    blks[-1] = blocks.make_block(rogue, 5, number=3, seed=3)[0]
    with pytest.raises(_lib.Unsupported):
        g.validate_blocks(blks)
    g.close()


@pytest.mark.parametrize("ndev", [2, 3, 4])
def test_group_single_block_split_by_transaction(ndev):
    """one block (fewer blocks than devices) is split by transaction index across
    the devices; a txid repeated across the device ranges (tx 5 again at tx 170) is still caught
    by markTXIdDuplicates in the finalize -- flags equal the single GPU's and the oracle's"""
    net = network()
    txs = []
    b0 = blocks.make_block(net, 60, number=1, seed=961, faults=(), out_txs=txs)[0]
    blk = blocks.make_block(net, 200, number=2, seed=962, reuse={170: (txs[5].creator, txs[5].nonce)})[0]
    one = _lib.Engine(0)
    _setup(one, net)
    single = list(one.validate_blocks([blk])[0])
    one.close()
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), [blk])[0]
    g = _lib.Group([0] * ndev)
    for e in g.engines:
        _setup(e, net)
    got = list(g.validate_blocks([blk])[0])
    assert got == single == list(exp)
    # the same txid twice inside the split block: its second occurrence is 9
    blk2 = blocks.make_block(net, 120, number=3, seed=963, faults=())[0]
    from oracle.protowire import decode
    envs = decode("Block", blk2)["data"]["data"]
    from tests.blockfix import block_from_envs
    dup = block_from_envs(envs[:100] + [envs[3]] + envs[100:], number=3)
    got2 = list(g.validate_blocks([dup])[0])
    exp2 = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), [dup])[0]
    assert got2 == list(exp2) and got2[100] == 9
    # two blocks over more devices: the ranges cross the block boundary
    got3 = g.validate_blocks([b0, blk])
    exp3 = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), [b0, blk])
    assert [list(f) for f in got3] == [list(f) for f in exp3]
    g.close()


def test_group_verify_msgs_c4_share():
    """fgv_group_p256_verify_msgs -- the C4 per-GPU share (131,072 identity.Verify
    items, the fault mix) split over 2 device contexts through the C ABI equals one context"""
    import numpy as np
    from fabric_amd._lib import pack
    from fabric_amd.synth.workloads import sig_pool
    n, uniq = 131072, 16384
    pool = sig_pool(uniq, seed=1001)
    idx = np.arange(n) % uniq
    keys = np.frombuffer(b"".join(pool["keys"][pool["key_index"][i]].pub for i in range(uniq)), np.uint8).reshape(-1, 64)[idx]
    msgs = np.ascontiguousarray(pool["msgs"][idx])
    mlen = np.full(n, msgs.shape[1], np.uint32)
    moff = np.arange(n, dtype=np.uint64) * np.uint64(msgs.shape[1])
    sa, so, sl = pack([pool["sigs"][i] for i in idx])
    margs = (msgs.reshape(-1), moff, mlen)
    g = _lib.Group([0, 0])
    got = g.verify_msgs(keys, margs, (sa, so, sl))
    g.close()
    one = _lib.Engine(0)
    single = one.verify_msgs(keys, margs, (sa, so, sl))
    one.close()
    assert (got == single).all()
    assert ((got == 0) == pool["expect_valid"][idx]).all()


def test_group_verify_msgs_c4_whole_batch():
    """the whole C4 batch -- 1,048,576 identity.Verify items of 1.85 KB messages
    (a 16,384-item pool with the injected tamper / high-S / bad-DER / trailing-bytes mix, repeated)
    -- through fgv_group_p256_verify_msgs over 8 device contexts on the box's one GPU: every
    status is the generator's expectation (the size-independent property at full size; the
    131,072-item share above equals one context bit for bit)"""
    import numpy as np
    from fabric_amd._lib import pack
    from fabric_amd.synth.workloads import sig_pool
    n, uniq = 1 << 20, 16384
    pool = sig_pool(uniq, seed=1002)
    idx = np.arange(n) % uniq
    keys = np.frombuffer(b"".join(pool["keys"][pool["key_index"][i]].pub for i in range(uniq)), np.uint8).reshape(-1, 64)[idx]
    msgs = np.ascontiguousarray(pool["msgs"][idx])
    mlen = np.full(n, msgs.shape[1], np.uint32)
    moff = np.arange(n, dtype=np.uint64) * np.uint64(msgs.shape[1])
    sa, so, sl = pack([pool["sigs"][i] for i in range(uniq)])
    so = so[idx]
    sl = sl[idx]
    g = _lib.Group([0] * 8, key_slots=64)
    got = g.verify_msgs(keys, (msgs.reshape(-1), moff, mlen), (sa, so, sl))
    g.close()
    exp = pool["expect_valid"][idx]
    assert got.shape == (n,)
    bad = np.nonzero((got == 0) != exp)[0]
    assert len(bad) == 0, (len(bad), bad[:8], got[bad[:8]])


def test_group_rccl_collective_world1():
    """fgv_group_set_collective(RCCL) through the C ABI: an RCCL communicator over
    the group's devices (world 1 on the box's one GPU), ncclAllGather of the records on the
    engine's own stream, the finalize on every device; flags equal the peer-copy path's and the
    oracle's, across duplicate txids of earlier blocks and per-block outcomes.  Repeated devices
    cannot form a communicator: FGV_EINVAL, and the group keeps working on peer copies."""
    net = network()
    txs1 = []
    blks = [blocks.make_block(net, 40, number=1, seed=901, faults=(), out_txs=txs1)[0]]
    for i in range(2, 5):
        reuse = {2: (txs1[i].creator, txs1[i].nonce)} if i == 3 else None
        blks.append(blocks.make_block(net, 30 + 7 * i, number=i, seed=900 + i, reuse=reuse)[0])
    exp = v20.validate_blocks(v20.ChannelModel(net.channel, net.identities(), net.chaincodes), blks)
    g = _lib.Group([0])
    try:
        _setup(g.engines[0], net)
        g.set_collective(_lib.Group.COLL_RCCL)
        for rep in range(2):  # (the second call reuses the communicator and buffers)
            got = g.validate_blocks(blks)
            assert [list(f) for f in got] == [list(f) for f in exp], rep
        g.set_block_outcomes(True)
        got = g.validate_blocks(blks)
        assert [list(f) for f in got] == [list(f) for f in exp]
        assert g.last_block_status(len(blks)) == ([0] * len(blks), len(blks))
        g.set_collective(_lib.Group.COLL_PEER)
        assert [list(f) for f in g.validate_blocks(blks)] == [list(f) for f in exp]
    finally:
        g.close()
    g2 = _lib.Group([0, 0])
    try:
        with pytest.raises(_lib.FgvError):
            g2.set_collective(_lib.Group.COLL_RCCL)
        for e in g2.engines:
            _setup(e, net)
        assert [list(f) for f in g2.validate_blocks(blks)] == [list(f) for f in exp]
    finally:
        g2.close()
